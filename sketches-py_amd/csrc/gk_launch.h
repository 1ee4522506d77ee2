// gk_launch.h -- host-side launchers of the HIP kernels (gk_kernels.hip),
// used by the C ABI runtime (gk_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gk_state.h"

// Capacity of the fast LDS class (every stream starts there when P <= 128).
#ifndef GK_SMALL_CAP
#define GK_SMALL_CAP 128
#endif

// optional query fused into an ingest/flush launch (gk:187-232 after the flush)
struct GKQuery {
  const double* qs = nullptr;  // device, nq values (NULL: no query)
  int nq = 0;
  double* out = nullptr;       // device [S * nq]
  int mode = 0;                // 0 quantiles() list semantics, 1 quantile() per q
};

struct MergeArgsHost {
  GKState dst;
  GKState src;
  const double* ev;
  const int32_t* eg;
  const int32_t* ed;
  const int64_t* eoffs;
  int mode;  // 0 = merge(other), 1 = merge_compress(entries)
  int cap;
  const int32_t* list;
  int64_t count;
  int32_t* ovf_count;
  int32_t* ovf_list;
  unsigned char* ws;  // global workspace for capacities beyond LDS (NULL = LDS)
  size_t ws_bytes;    // per block
  int64_t ws_blocks;
};

int gk_num_cu();
// the device has CUs to spare for k_long_prep beside an early k_ingest_wg grid
int gk_wg_early_ok();
size_t gk_ingest_ws_bytes(int cap, int vpl);
// k_ingest_big (any capacity, any flush period): bytes of one block's workspace
size_t gk_big_ws_bytes(int cap, int P);
#define GK_WORK_BYTES 2048  // 8 hand-out counters + 8 stats-role batch counters, one 128-byte line each
// `work`: device counters of the launch's dynamic stream hand-out, ZEROED BY THE CALLER
// (GK_WORK_BYTES for the small-class launch, 8 bytes for the others; gk_capi.cpp
// zeroes every counter of a call with one memset, GK_CALL_* below).
// cap GK_SMALL_CAP / 2048: LDS kernels; any other cap: global workspace ws (ws_bytes per block, ws_blocks blocks)
// list/count (host count) or list/count_ptr (device count): the streams of a class-lcls launch
// (list NULL: every stream, class 0); listed streams no longer in class lcls are skipped.
hipError_t gk_launch_ingest(int cap, int vpl, const GKState& st, const double* x, const int64_t* offs,
                            const int32_t* list, int64_t count, const int32_t* count_ptr, int lcls, int force,
                            unsigned char* ws, size_t ws_bytes,
                            int64_t ws_blocks, int32_t* ovf_count, int32_t* ovf_list, const GKQuery& q,
                            unsigned long long* work, const int32_t* prio, const int32_t* prio_count,
                            const double* psort, const int64_t* prio_ws, const int32_t* prio_skip, int fused_stats,
                            hipStream_t stream, hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr,
                            const struct GKPoolDev* pool = nullptr, int pmode = 0);
// (ev_start / ev_stop: the small-class launch records them as part of its
// dispatch -- hipExtLaunchKernel, the kernel's own start and end -- instead of
// two marker packets around it; other classes ignore them.  pool / pmode:
// the promotion rounds' fused steps, k_ingest's pmode)
// The unbounded class (tables beyond 32768 entries; every class when P > 1024):
// one wave per stream over ws (ws_bytes >= gk_big_ws_bytes(cap, P) per block,
// ws_blocks blocks); list / count / count_ptr / lcls / force / q as above;
// ctr: the set's GK_CTR_* counters (GK_CTR_FATAL: per-stream count limit).
hipError_t gk_launch_ingest_big(int cap, const GKState& st, const double* x, const int64_t* offs,
                                const int32_t* list, int64_t count, const int32_t* count_ptr, int lcls, int force,
                                unsigned char* ws, size_t ws_bytes, int64_t ws_blocks, int32_t* ovf_count,
                                int32_t* ovf_list, const GKQuery& q, unsigned long long* work, int32_t* ctr,
                                hipStream_t stream);
// `fused_stats` > 0: the small-class batch launch (x given, no list) also
// walks the gk:52-59 stats of every stream of at most GK_STATS_LONG values,
// in that many waves per CU (then requires the lengths-only k_lengths before).
// `prio` / `prio_count` (device, may be NULL): streams handed out first by the
// capacity-class kernels (the long streams of the batch, longest first);
// `psort` / `prio_ws`: their presorted flush batches (GKPresort), or NULL.
// k_stats over every stream; streams longer than GK_STATS_LONG values are put
// on long_list (S entries), sorted longest first, with their pre-call n in
// long_n, for gk_launch_stats_long, which may run on another HIP stream beside
// the ingest launches (it writes only _min/_max/_sum/_avg of listed streams).
// Presort of the long streams' automatic-flush batches (sets whose class 0 is
// a capacity-class kernel): per list slot the workspace offset (-1: none)
// and first global batch, the workspace (ws_cap doubles) and the size this
// call needed (host grows the workspace from it after the call).
struct GKPresort {
  int64_t* list_ws = nullptr;  // [S]
  int64_t* list_b0 = nullptr;  // [S + 1]
  double* ws = nullptr;
  int64_t ws_cap = 0;
  int64_t* ws_need = nullptr;  // device, 1 value
  int32_t* wg_count = nullptr; // device, 1 value: k_ingest_wg's streams (the head of the long list); NULL: none
  int wg_presort = 1;          // with wg_count: presort as without it (1) or nothing (0: k_ingest_wg ranks)
  int32_t* done = nullptr;     // device, 1 value: k_presort_reg's finished waves (k_ingest_wg runs beside
                               // the presort and takes presorted batches once all are done); NULL: after it
};
// one workgroup per stream for the first *wg_count streams of the long list
// (class lcls = 0 of the 2048 class only); the prio k_ingest launch skips them
hipError_t gk_launch_ingest_wg(const GKState& st, const double* x, const int64_t* offs, const int32_t* long_list,
                               const int32_t* wg_count, int lcls, int force, int32_t* ovf_count, int32_t* ovf_list,
                               unsigned long long* work, const GKPresort& ps, hipStream_t stream,
                               const int32_t* go = nullptr);
// the long-stream list + every stream's pre-call n (k_lengths)
hipError_t gk_launch_stats(const GKState& st, const int64_t* offs, int32_t* long_list, int32_t* long_count,
                           hipStream_t stream);
// the long list sorted longest first, the listed streams' pre-call n, the
// presort plan and k_ingest_wg's stream count (k_long_prep)
hipError_t gk_launch_long_prep(const GKState& st, const int64_t* offs, int32_t* long_list, int64_t* long_n,
                               int32_t* long_count, const GKPresort& ps, hipStream_t stream, int32_t* go = nullptr);
// gk:52-59 chains of the streams up to GK_STATS_LONG values (k_stats_short; the
// long ones are k_stats_long's), when class 0 is not the small class
hipError_t gk_launch_stats_short(const GKState& st, const double* x, const int64_t* offs, hipStream_t stream);
// k_presort over the plan k_long_prep wrote (no-op without a workspace)
// k_presort_reg's grid (waves); k_ingest_wg compares *ps.done with it
int gk_presort_reg_grid(const GKState& st);
hipError_t gk_launch_presort(const GKState& st, const double* x, const int64_t* offs, const int32_t* long_list,
                             const int64_t* long_n, const int32_t* long_count, const GKPresort& ps,
                             hipStream_t stream);
// hc_count (device, may be NULL): the first *hc_count list entries are
// walked on host cores (gk_launch_hc_prep) and skipped here
hipError_t gk_launch_stats_long(const GKState& st, const double* x, const int64_t* offs, const int32_t* long_list,
                                const int64_t* long_n, const int32_t* long_count, const int32_t* hc_count,
                                hipStream_t stream);
// Host-walked chains: the longest streams of the sorted
// long list whose gk:52-59 chains run on host cores.  One record per stream:
// the pre-call state from gk_launch_hc_prep, the final one written back by
// the host and applied by gk_launch_hc_apply.
struct GKHostChainRec {
  int64_t s, xo, len, n;
  double sum, avg, mn, mx;
};
#define GK_HC_MAX 256
// takes list entries while len >= min_len and len >= rel_pct % of the
// longest, at most GK_HC_MAX of them and budget_factor x (the longest length)
// values in all, and only when the list is walked one wave per stream
// (<= GK_SL_BCAST streams); min_len <= 0: none
hipError_t gk_launch_hc_prep(const GKState& st, const int64_t* offs, const int32_t* long_list, const int64_t* long_n,
                             const int32_t* long_count, int64_t min_len, int rel_pct, int64_t budget_factor,
                             GKHostChainRec* recs, int32_t* hc_count, hipStream_t stream);
// fail (device, may be NULL): set by gk_launch_hc_wait; nonzero = the host
// walk failed and gk_launch_hc_fallback walks the picked streams instead
hipError_t gk_launch_hc_apply(const GKState& st, const GKHostChainRec* recs, const int32_t* hc_count,
                              const int32_t* fail, hipStream_t stream);
// waits (one thread, s_sleep) until *flag >> 2 >= seq, at most timeout_s
// seconds; *fail = 0 iff the flag is (seq << 2) | 1
hipError_t gk_launch_hc_wait(const unsigned long long* flag, unsigned long long seq, int32_t* fail,
                             double timeout_s, hipStream_t stream);
hipError_t gk_launch_hc_fallback(const GKState& st, const double* x, const int64_t* offs, const int32_t* long_list,
                                 const int64_t* long_n, const int32_t* hc_count, const int32_t* fail,
                                 hipStream_t stream);
// quantiles of the listed streams from their committed tables (after the
// join); qfix: also resolve the _min/_max markers of a small-class launch
// that carried the stats role (every stream's answers)
hipError_t gk_launch_query_list(const GKState& st, const int32_t* list, const int32_t* count, const GKQuery& q,
                                bool qfix, hipStream_t stream);
size_t gk_merge_lds_bytes(int cap, int pmax);
hipError_t gk_launch_merge(const MergeArgsHost& h, hipStream_t stream);
// every stream back to an empty sketch in class 0; ctr: also zero the set's
// counter words [0, GK_CTR_FATAL) (slots used, member-list lengths) and the
// per-call block [GK_CTR_CALL, GK_CALL_BYTES) (what begin_call's memset zeroes)
hipError_t gk_launch_reset(const GKState& st, hipStream_t stream, int32_t* ctr = nullptr);
// fills st.rtab (reciprocals 1.0/k, k < st.rtab_n)
hipError_t gk_launch_rtab(const GKState& st, hipStream_t stream);
hipError_t gk_launch_export(const GKState& st, const int64_t* offs, double* v, int32_t* g, int32_t* d,
                            hipStream_t stream);
hipError_t gk_launch_export_pending(const GKState& st, const int64_t* offs, double* v, hipStream_t stream);
// counts into *bad the streams whose pending count p is not one add() can leave (p > n mod P)
hipError_t gk_launch_check_pending(int64_t S, int P, const int64_t* n, const int64_t* poffs, int32_t* bad,
                                  hipStream_t stream);
hipError_t gk_launch_import(const GKState& st, const int64_t* offs, const double* v, const int32_t* g,
                            const int32_t* d, const int64_t* poffs, const double* pv, int32_t* ovf_count,
                            int32_t* ovf_list, hipStream_t stream);
hipError_t gk_launch_promote(const GKState& st, const int32_t* list, int64_t count, const int32_t* slots, int ncls,
                             hipStream_t stream);

// Device-side capacity-class bookkeeping: counters (slots used, member list
// lengths, re-run list lengths, streams that found no class / slot) and, per
// class c > 0, its member list and this round's re-run list (S entries each).
// Layout of the set's counter block (int32 words; one allocation):
//   persistent:  [0..3] slots used per class, [4..7] member-list lengths,
//                [12] streams with no class left, [13] the largest such id
//   per call (zeroed by ONE memset at the start of every call, from word
//   GK_CTR_CALL -- 16, a 64-byte boundary: one fill -- to GK_CALL_BYTES):
//   [16] deferred streams, [17] long-stream list length, [20 + 4r + c] round
//   r's re-run list length of class c, [40 + r] round r's overflow count,
//   then (byte GK_CALL_WORK) the launches' stream hand-out counters.
// The host reads words [0, GK_CTR_WORDS) back after every call.
#define GK_CTR_USED 0
#define GK_CTR_LCNT 4
#define GK_CTR_FATAL 12   // [12] count, [13] largest such stream id
#define GK_CTR_DEFER 16   // streams whose class had no free slot this call (re-run by the host later)
#define GK_CTR_LONG 17    // streams longer than GK_STATS_LONG values (k_stats)
#define GK_CTR_RCNT 20    // [20 + 4*round + class]
#define GK_CTR_OVFC 40    // [40 + round]
#define GK_CTR_BADPEND 48 // gk_import: streams with an unreachable pending count
#define GK_CTR_WG 50      // k_ingest_wg's stream count this call (k_long_prep)
#define GK_CTR_WGGO 53    // k_long_prep done: k_ingest_wg, launched ahead of it, starts its streams
#define GK_CTR_PSDONE 51  // k_presort_reg's finished waves this call (k_ingest_wg beside it)
#define GK_CTR_WORDS 18
#define GK_CTR_CALL 16
#define GK_CALL_WORK 256                          // bytes: the small-class launch's GK_WORK_BYTES, then
#define GK_CALL_SLOTS 16                          //   16 counters of 128 bytes for the other launches
#define GK_CALL_BYTES (GK_CALL_WORK + GK_WORK_BYTES + GK_CALL_SLOTS * 128)
static_assert(GK_CTR_RCNT + 4 * (GK_MAX_CLASSES + 1) <= GK_CTR_OVFC, "re-run counts fit below the overflow counts");
static_assert(GK_CTR_PSDONE < GK_CALL_WORK / 4, "counters fit below the hand-out block");
static_assert((GK_CTR_CALL * 4) % 64 == 0 && (GK_CALL_BYTES - GK_CTR_CALL * 4) % 16 == 0, "aligned per-call memset");
struct GKPoolDev {
  int32_t* ctr;
  int32_t* rcnt;  // this round's re-run list lengths (one per class)
  int32_t* list[GK_MAX_CLASSES];
  int32_t* rerun[GK_MAX_CLASSES];
  int32_t* defer;  // S entries
};
// k_promote_dev over list[0 .. *count): level -1 -> class cls+1 (ingest
// overflow: joins the re-run list, or the defer list when that class has no
// free slot), -2 -> class cls+1 (import), level >= 0 -> class `level` if below it
hipError_t gk_launch_promote_dev(const GKState& st, const int32_t* count, const int32_t* list, int level,
                                 const GKPoolDev& pool, hipStream_t stream);
