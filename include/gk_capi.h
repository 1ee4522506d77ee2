/*
 * gk_capi.h -- C ABI of the MI355X-native batched GKArray engine.
 *
 * The reference (githomin/sketches-py, gkarray/gkarray.py, "gk:N" = line N) is a
 * pure-Python class with no FFI.  This header is the boundary a ctypes (or cgo /
 * JNI) binding binds; each entry point names the reference method it replaces.
 * A "set" holds S independent GKArray streams that share one epsilon; every
 * stream behaves exactly like one reference ``GKArray`` object fed the same
 * values in the same order (tables and quantiles bit-exact).
 *
 * Conventions
 *  - Every call returns an int status: GK_OK (0) or a negative GK_E_* code;
 *    gk_last_error() returns a thread-local message for the last failure.
 *  - Pointers documented "device" must be device memory on the set's GPU
 *    (e.g. a torch tensor's data_ptr()); "host" pointers are host memory.
 *  - `stream` is a hipStream_t passed as void* (NULL = the default stream).
 *    All calls on one set must be ordered on one stream.  gk_ingest,
 *    gk_ingest_quantiles, gk_flush, gk_quantiles, gk_stats and the exports
 *    only ENQUEUE their work and return (no host synchronisation): a stream
 *    whose table outgrows its capacity class is moved to the next class and
 *    re-run by the device itself.  Part of an ingest (the sequential
 *    _sum/_avg chains of streams longer than 16384 values) runs on a stream
 *    the set owns; `stream` is made to wait for it, so every later call
 *    enqueued on `stream` sees the finished state.  Optionally
 *    (GK_HOST_CHAINS=1 or GK_HOST_CHAIN_MIN in the environment; off by
 *    default) the chains of the few longest streams (>= 2^20 values) are
 *    walked on host cores by a worker thread of the set: the call only
 *    hands them over (it does not block)
 *    and `stream` waits for the worker on the device (a kernel polling a
 *    pinned flag, bounded at 20 s; a failed host walk is redone on the
 *    device, same bits).  The set's next call, gk_sync and gk_destroy first
 *    wait for that worker on the host.  While `stream` is being captured
 *    into a graph, no chain is handed to the host.  The caller keeps input
 *    buffers alive and unchanged until the set's next call or gk_sync: a
 *    stream that needs a class whose arena has no free slot yet is deferred
 *    and re-run from them by the host runtime before the next call proceeds.
 *    gk_merge,
 *    gk_merge_compress, gk_import, gk_save / gk_load and gk_num_promoted
 *    synchronise before returning.
 *  - Limits.  Any finite eps > 0 with int(1/eps)+1 < 2^24 is accepted (the
 *    reference: any eps; eps > 1 gives a flush period of 1, gk:60); tables grow through capacity classes up to 2^27 entries per
 *    stream (the last classes are allocated on first use).  One stream may
 *    hold n values while 2*eps*(n-1) <= 2^30 (5.4e10 values at eps=0.01):
 *    its tuples' g and delta are int32 (GKRec).
 *  - Asynchronous errors: a stream that would pass a limit above (or finds no
 *    memory for its class) is refused: its table, pending values and n keep
 *    their pre-call state (_min/_max/_sum/_avg, computed beside the tables,
 *    include the call's values), and GK_E_OVERFLOW is reported by a later
 *    call on the set, at the latest by gk_sync.
 *  - A set is not thread-safe.  The library owns the set's device state;
 *    callers own their input and output buffers.
 */
#ifndef GK_CAPI_H
#define GK_CAPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GK_OK 0
#define GK_E_ARG (-1)          /* bad argument (size, pointer, NaN quantile ...)   */
#define GK_E_EPS_MISMATCH (-2) /* merge of sets with different eps: gk:118-119     */
#define GK_E_OVERFLOW (-3)     /* a stream passed a limit (table size, count)     */
#define GK_E_HIP (-4)          /* HIP runtime failure                              */
#define GK_E_NOMEM (-5)        /* device allocation failed                          */
#define GK_E_UNSUPPORTED (-6)  /* eps below ~6e-8 (flush period beyond 2^24)       */
#define GK_E_IO (-7)           /* state file cannot be opened / written            */
#define GK_E_FORMAT (-8)       /* state file malformed, wrong version or checksum  */

typedef struct gk_set gk_set;

/* Library / ABI version (major*10000 + minor*100 + patch). */
int gk_version(void);

/* Message for the last failed call on this thread ("" if none). */
const char* gk_last_error(void);

/* GKArray(eps) for `num_streams` streams (gk:21-29): empty tables, n=0,
 * min=+inf, max=-inf, sum=avg=0.  `device` is the HIP device ordinal.
 * `cap_hint` (0 = default, < 2^27) is the per-stream table capacity the set
 * starts with; streams whose table outgrows it are promoted to a larger class
 * automatically. */
int gk_create(int64_t num_streams, double eps, int64_t cap_hint, int device,
              gk_set** out);
int gk_destroy(gk_set* set);

/* Reset every stream to the freshly constructed state (gk:21-29). */
int gk_reset(gk_set* set, void* stream);

/* Batched GKArray.add (gk:49-61): stream s receives, in order,
 * values[offsets[s] .. offsets[s+1]).  `values` (float64, device) and
 * `offsets` (int64[num_streams+1], device, non-decreasing) describe a CSR
 * batch over ALL streams of the set.  Flushes (merge_compress, gk:63-109)
 * happen at exactly the reference's flush points (n % (int(1/eps)+1) == 0). */
int gk_ingest(gk_set* set, const double* values, const int64_t* offsets,
              void* stream);

/* Wait for the set's work on `stream`; return (and clear) an asynchronous
 * error of an earlier call (GK_E_OVERFLOW, see Conventions) or GK_OK. */
int gk_sync(gk_set* set, void* stream);

/* GKArray.merge_compress() with no argument (gk:63-109) on every stream that
 * has pending values -- what size()/quantile()/quantiles() do first
 * (gk:45-46, 166-167, 197-198). */
int gk_flush(gk_set* set, void* stream);

/* Batched GKArray.quantiles(qs) (gk:187-232) for every stream.
 * `qs` (host, nq float64 values, no NaN); `out` (device, float64[S*nq],
 * row-major [stream][q]).  Pending values are flushed first (mutation, as in
 * the reference).  mode GK_Q_LIST = quantiles() semantics (the caller passes
 * qs as given; if they are not sorted the per-q quantile() result is used,
 * exactly as gk:205-206 does); mode GK_Q_SINGLE = quantile(q) semantics for
 * every q (gk:156-185). */
#define GK_Q_LIST 0
#define GK_Q_SINGLE 1
int gk_quantiles(gk_set* set, const double* qs, int nq, double* out, int mode,
                 void* stream);

/* gk_ingest followed by gk_quantiles, fused: every stream adds its values
 * (gk:49-61), then answers quantiles(qs) (gk:187-232) -- the leftover pending
 * values are flushed first, as the reference does -- from the table while it
 * is still on chip.  Same arguments and semantics as the two calls. */
int gk_ingest_quantiles(gk_set* set, const double* values, const int64_t* offsets,
                        const double* qs, int nq, double* out, int mode, void* stream);

/* Per-stream accessors num_values/_min/_max/sum/avg (gk:35-42, 25-29) and the
 * table size len(entries) / pending count len(incoming) WITHOUT flushing.
 * Any pointer may be NULL.  All outputs are device arrays of length S. */
int gk_stats(gk_set* set, int64_t* n, double* mn, double* mx, double* sum,
             double* avg, int32_t* table_size, int32_t* pending, void* stream);

/* GKArray.merge(other) (gk:111-154), stream by stream, as the left fold
 * dst.merge(srcs[0]); dst.merge(srcs[1]); ...  Like the reference it mutates
 * each source (flushes its pending values, gk:126, 137).  A source may be dst
 * itself (dst.merge(dst): dst is flushed, then merged with a snapshot of its
 * flushed state, as gk:137-154 do) and may repeat (flushed again at each of
 * its merges).  Returns GK_E_EPS_MISMATCH if any eps differs (gk:118-119) or
 * GK_E_ARG if the stream counts differ. */
int gk_merge(gk_set* dst, gk_set* const* srcs, int nsrcs, void* stream);

/* GKArray.merge_compress(entries) with an explicit entry list (gk:63-109,
 * gk:71): stream s merges extra records [eoffs[s], eoffs[s+1]) given as
 * (v, g, d) device arrays, each list sorted by v as the reference requires of
 * its Entry lists. */
int gk_merge_compress(gk_set* set, const double* v, const int32_t* g,
                      const int32_t* d, const int64_t* eoffs, void* stream);

/* Table export (the reference's `entries`, gk:23): writes per-stream table
 * sizes to `sizes` (device int32[S]); then gk_export copies stream s's table
 * to v/g/d[offs[s] ..] where offs (device int64[S+1]) is the caller's
 * exclusive scan of those sizes.  Pending values (`incoming`, gk:24) go the
 * same way with gk_export_pending_sizes / gk_export_pending. */
int gk_export_sizes(gk_set* set, int32_t* sizes, void* stream);
int gk_export(gk_set* set, const int64_t* offs, double* v, int32_t* g,
              int32_t* d, void* stream);
int gk_export_pending_sizes(gk_set* set, int32_t* sizes, void* stream);
int gk_export_pending(gk_set* set, const int64_t* poffs, double* pv,
                      void* stream);

/* Import full per-stream state (checkpoint / RCCL payload): tables in CSR
 * (offs, v, g, d), pending values in CSR (poffs, pv) and the header arrays
 * (n, mn, mx, sum, avg), all device arrays of the set's S streams. */
int gk_import(gk_set* set, const int64_t* offs, const double* v,
              const int32_t* g, const int32_t* d, const int64_t* poffs,
              const double* pv, const int64_t* n, const double* mn,
              const double* mx, const double* sum, const double* avg,
              void* stream);

/* Versioned state files (format: sketches-py_amd/csrc/gk_format.h, "GKSTATE"
 * version 1: header with magic, version, eps, S, record totals and a
 * checksum; then sizes, pending counts, n/min/max/sum/avg, the tables and the
 * pending values).  The reference has no serialization: its state is the
 * Python object (gk:21-29 -- entries, incoming, _n, _min, _max, _sum, _avg),
 * and this is that state per stream, saved WITHOUT flushing, so a set loaded
 * from a file continues exactly like the saved one.
 * gk_save writes the set's state to `path`.  gk_peek reads eps and the stream
 * count from a file's header (to create a matching set).  gk_load replaces
 * the state of every stream of `set`, which must have the file's stream count
 * (GK_E_ARG) and eps (GK_E_EPS_MISMATCH).  GK_E_IO / GK_E_FORMAT on
 * unreadable, malformed, wrong-version or corrupt files. */
int gk_save(gk_set* set, const char* path, void* stream);
int gk_peek(const char* path, double* eps, int64_t* num_streams);
int gk_load(gk_set* set, const char* path, void* stream);

/* ---- row-shard exchange ----------------------------------
 * A set's whole state as one contiguous, self-describing "packed state"
 * buffer (layout: sketches-py_amd/csrc/gk_pack.h) that any transport moves as
 * bytes -- rcclAllGather / MPI_Allgather of device buffers, a socket, a file --
 * and the rank-ordered fold of such buffers: for every stream, the
 * reference's left fold sk0.merge(sk1).merge(sk2)... (gk:111-154; each merge
 * flushes `other` first, gk:126/137).  Buffers are device memory on the
 * set's GPU (host memory for the CPU engine).  All three calls synchronise.
 *
 * gk_pack_bytes: size of the set's packed state (read back from the device).
 * gk_pack:       writes it into `buf` (`bytes` >= gk_pack_bytes; trailing
 *                bytes untouched, so equal-sized padded buffers work for an
 *                all-gather).
 * gk_fold_packed: dst := bufs[0], then dst.merge(bufs[r]) for r = 1..n-1.
 *                Every buffer must hold dst's stream count and eps
 *                (GK_E_EPS_MISMATCH otherwise, as gk_merge).  The previous
 *                state of dst is replaced. */
int gk_pack_bytes(gk_set* set, int64_t* bytes, void* stream);
int gk_pack(gk_set* set, void* buf, int64_t bytes, void* stream);
/* Each bufs[r] must hold the whole packed state its header describes (the
 * header's byte count, as gk_pack_bytes returned it for the packing set):
 * headers and offset tables are checked for consistency, but the buffers'
 * own lengths are not known to this call. */
int gk_fold_packed(gk_set* dst, const void* const* bufs, int nbufs, void* stream);

/* Introspection for tests and benchmarks. */
int64_t gk_num_streams(const gk_set* set);
double gk_eps(const gk_set* set);
int gk_flush_period(const gk_set* set);       /* int(1.0/eps) + 1 (gk:60)  */
int gk_capacity(const gk_set* set, int cls);  /* table capacity of a class */
int64_t gk_num_promoted(const gk_set* set);   /* streams in the large class */
/* Streams whose gk:52-59 chains the host walked in the last completed
 * ingest (host-walked chains; 0 when none were picked or
 * the walk failed and the device walked them), -1 for a bad set.  Waits for
 * the set's host worker.  Diagnostics only: results never depend on it. */
int64_t gk_host_chains_taken(gk_set* set);

/* Kernel timing: `on` bit 0 -- gk_ingest records HIP events around the
 * flush kernel it launches on `stream`; bit 1 -- also around the call's
 * stats fork (stats_ms; two more event markers per call).  gk_timing_read
 * returns the summed milliseconds and the number of launches since the last
 * read. */
int gk_timing_enable(gk_set* set, int on);
int gk_timing_read(gk_set* set, double* flush_ms, double* stats_ms,
                   int64_t* launches);

#ifdef __cplusplus
}
#endif

#endif /* GK_CAPI_H */
