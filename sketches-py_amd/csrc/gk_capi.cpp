// gk_capi.cpp -- C ABI runtime of the MI355X batched GKArray engine.
//
// Owns the per-set device state (header arrays, table arenas, pending
// buffers), decides flush modes and table-capacity classes, and launches the
// kernels of gk_kernels.hip on the caller's HIP stream.  Every entry point is
// declared in include/gk_capi.h with the reference method it replaces.
#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gk_capi.h"
#include "gk_pack.h"
#include "gk_format.h"
#include "gk_launch.h"
#include "gk_state.h"
#include "gk_host_stats.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail(GK_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

constexpr int kCapSmall = GK_SMALL_CAP;  // LDS class (gk_launch.h)
constexpr int kCapLarge = 2048;  // LDS class, ~92 KB per wave
constexpr int kCapHuge = 32768;  // global-workspace class (k_ingest)
constexpr int kCapBig = 1 << 20;  // first unbounded class (k_ingest_big) after kCapHuge
constexpr int kCapMax = 1 << 27;  // largest class (2 GiB per table)
constexpr int kPMax = 1 << 24;    // largest flush period (eps >= 6e-8)
constexpr int64_t kRecipTable = (int64_t)1 << 17;  // entries of st.rtab (1 MiB)
constexpr int kMaxLdsCap = 2048;
constexpr int kRounds = GK_MAX_CLASSES + 1;  // overflow lists: launch round 0 + one per promotion level

int vpl_for(int P) {
  int v = 1;
  while (v * 64 < P) v <<= 1;
  return v;
}

}  // namespace

struct gk_set {
  // no stream is in a class above 0 (creation, gk_reset; cleared by every
  // enqueued promotion): the member-list launches of run_ingest are skipped
  bool no_members = true;
  int64_t S = 0;
  double eps = 0;
  int P = 0;
  int device = 0;
  int vpl = 1;
  GKState st{};
  // Capacity classes c > 0 live entirely on the device: slot counters, member
  // lists and re-run lists (GKPoolDev, k_promote_dev).  The host only sizes
  // the arenas (st.alloc) ahead of need, from counters read back
  // asynchronously at the end of each call (h_ctr, ev_done).
  int32_t* d_ctr = nullptr;                                  // GK_CTR_WORDS counters
  int32_t* d_list[GK_MAX_CLASSES] = {};
  int32_t* d_rerun[GK_MAX_CLASSES] = {};
  // kernel of each class: the unbounded k_ingest_big (classes beyond 32768
  // entries; every class when P > 1024) or the capacity-class kernels
  bool big[GK_MAX_CLASSES] = {};
  int32_t* d_defer = nullptr;  // streams whose next class had no free slot (S entries)
  int32_t* h_ctr = nullptr;  // pinned: the counters as of the end of the last call
  hipEvent_t ev_done = nullptr;
  bool done_pending = false;
  // the last ingest / flush call: its inputs, kept to re-run deferred streams
  // (the caller keeps them valid until the set's next call or gk_sync)
  struct {
    const double* x = nullptr;
    const int64_t* offs = nullptr;
    int force = 0;
    GKQuery q;
    bool may_defer = false;  // some class could run out of slots in it
  } last;
  // a gk_reset came after the call whose counters are still in flight: its
  // deferred streams are void (every stream was reset; nothing to re-run)
  bool void_defer = false;
  // the per-call counter block is known zero: gk_reset's k_reset zeroed it and
  // nothing has written it since (begin_call then skips its memset; cleared by
  // begin_call and by the paths that write the block without it: run_merge,
  // gk_import)
  bool ctr_clean = false;
  int32_t fatal_seen = 0;  // device FATAL count already reported
  int sticky = GK_OK;      // asynchronous error reported by the next call / gk_sync
  std::string sticky_msg;
  // global workspace of each class beyond LDS (allocated with its first slots)
  unsigned char* d_ws[GK_MAX_CLASSES] = {};
  size_t ws_bytes[GK_MAX_CLASSES] = {};
  int64_t ws_blocks[GK_MAX_CLASSES] = {};
  // overflow lists of the launch rounds (device); counts in one array
  int32_t* d_ovfc = nullptr;              // kRounds counts (words of d_ctr)
  int32_t* d_ovfl[kRounds] = {};
  int32_t* h_ovf = nullptr;               // pinned readback of a count (+ list) for merge / import
  int64_t* d_zero_offs = nullptr;  // S+1 zeros: offsets of flush-only launches
  unsigned long long* d_work = nullptr;  // the call's hand-out counters (bytes of d_ctr from GK_CALL_WORK)
  int next_work = 0;                     // next free 128-byte counter of this call
  int32_t* d_long_list = nullptr;        // streams k_stats hands to k_stats_long (longest first)
  int64_t* d_long_n = nullptr;           //   and their pre-call n
  int32_t* d_long_count = nullptr;       // (a word of d_ctr)
  // k_stats_long (the sequential _sum/_avg chains of long streams) runs on
  // this stream beside the ingest launches; ev_fork / ev_join order it
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_slgo = nullptr;  // aux has passed the fork: k_stats_long is next there
  // presorted flush batches of long streams (sets whose class 0 is the 2048
  // class): plan arrays, workspace, and the size the last call needed
  GKPresort ps;
  int64_t* h_ws_need = nullptr;  // pinned host copy of *ps.ws_need (valid once ev_done completed)
  // query scratch: pinned host copy of qs (the async H2D reads it), device copy
  double* h_qs = nullptr;
  double* d_qs = nullptr;
  int qs_alloc = 0;
  hipEvent_t ev_qs = nullptr;  // the last H2D copy out of h_qs
  int qs_n = 0;                // entries of the list last uploaded to d_qs (h_qs holds it)
  // eighths of a wave per CU of the small-class batch launch that walk the gk:52-59
  // stats chains first (0: separate k_stats launch); GK_FUSED_STATS overrides
  int fused_stats = 8;  // eighths of a wave per CU that start with the stats role (DESIGN 5 Stats)
  // gk_fold_packed: receives the packed states merged into this set (made on first use)
  gk_set* fold_scratch = nullptr;
  gk_set* self_scratch = nullptr;  // snapshot source of dst.merge(dst), only during that merge
  // Host-walked chains: the gk:52-59 chains of the
  // longest streams run on host cores beside the GPU ingest.  hc_min: shortest
  // stream taken (0: off; GK_HOST_CHAINS=0 / GK_HOST_CHAIN_MIN); hc_threads:
  // host threads (GK_HOST_CHAIN_THREADS); at most 4 x hc_threads x the
  // longest length values go to the host per call.
  int64_t hc_min = 0;
  int hc_rel = 75;  // ... and >= this % of the longest stream (GK_HOST_CHAIN_REL)
  int hc_threads = 1;
  GKHostChainRec* d_hc = nullptr;   // GK_HC_MAX records (device)
  int32_t* d_hc_count = nullptr;
  GKHostChainRec* h_hc = nullptr;   // pinned copies
  int32_t* h_hc_count = nullptr;
  hipEvent_t ev_hc = nullptr;       // the records' D2H copy
  bool hc_active = false;           // this call enqueued k_hc_prep
  const double* hc_x = nullptr;     // the call's values and offsets
  const int64_t* hc_offs = nullptr;
  bool forked = false;              // stats_fork launched on aux; stats_join / stats_abort joins it
  bool sl_inline = false;           // no fork: stats_join launches k_stats_long on the call's stream
  const double* sl_x = nullptr;     // (its arguments)
  const int64_t* sl_offs = nullptr;
  // one copy stream for every host thread's chunk copies, made at the first
  // host-walked chain (the box runs 4 hardware queues per process: a copy
  // stream sharing the ingest's or aux's queue waits behind their kernels --
  // 16 per-thread streams gave 12 GB/s instead of ~55); per host thread two
  // pinned chunk buffers and their events
  hipStream_t hc_copy = nullptr;
  // k_presort of the long streams' flush batches runs here beside the short
  // streams' chains (k_stats on the caller's stream); the ingest waits for it
  hipStream_t aux2 = nullptr;
  hipStream_t aux3 = nullptr;    // the presort when k_ingest_wg runs beside it (ps.done)
  bool presort_active = false;   // a presort of this call not yet joined on the caller's stream
  hipEvent_t ev_presort = nullptr;
  hipEvent_t ev_wg = nullptr;  // k_ingest_wg (on aux2, after the presort) done
  hipEvent_t ev_go = nullptr;  // the call's counters zeroed: k_ingest_wg may be launched (GK_WG_EARLY)
  bool wg_early = false;       // this call's k_ingest_wg was launched by stats_fork, ahead of the chain walks
  bool wg_trace = false;       // GK_WG_TRACE=1 at creation: its stream count per completed call on stderr (tests)
  std::vector<hipStream_t> hc_streams;
  std::vector<double*> hc_buf;
  std::vector<hipEvent_t> hc_ev;
  // The host walk is asynchronous (round 4): gk_ingest* only hands the call
  // to a worker thread of the set and enqueues the join on the caller's
  // stream (k_hc_wait on a pinned flag the worker writes, then the records'
  // copy, k_hc_apply, and k_hc_fallback which walks the picked chains on the
  // device if the host walk failed).  The next call on the set (or gk_sync /
  // gk_destroy) waits for the worker first, so the call's input buffers are
  // read by the worker no longer than the header's contract allows.
  std::thread hc_thr;
  std::mutex hc_mu;
  std::condition_variable hc_cv;
  std::deque<uint64_t> hc_jobs;             // calls whose chains wait for the worker
  bool hc_stop = false;
  uint64_t hc_seq = 0;                      // sequence number of the last handed-out call
  unsigned long long* h_hc_flag = nullptr;  // pinned, device-visible: (seq << 2) | 1 done / 2 failed
  int32_t* d_hc_fail = nullptr;             // device: this call's walk failed (set by k_hc_wait)
  int hc_fail_inject = 0;                   // GK_HC_FAIL=1 (tests): the worker reports a failure
  double hc_timeout_s = 20.0;               // k_hc_wait's bound on the host walk
  int64_t hc_last_taken = 0;                // streams the host walked in the last completed job
  int hc_last_rc = GK_OK;
  std::string hc_last_msg;
  // timing: event pairs recorded around the timed launches, summed at read
  bool timing = false;        // events around the class-0 ingest launch (gk_timing_enable bit 0)
  bool timing_stats = false;  // and around stats_fork's launches (bit 1: two more markers per call)
  std::vector<hipEvent_t> tev_flush, tev_stats;
  size_t n_flush = 0, n_stats = 0;
};

namespace {

// Every launch of the last class counts the streams that outgrow it as fatal
// itself (k_ingest pmode bit 1), so no promotion round is needed past it --
// unless that class runs k_ingest_big (or there is a single class).
bool fatal_direct(const gk_set* h) { return h->st.nclass >= 2 && !h->big[h->st.nclass - 1]; }

// What a launch of class c >= 1 (k_ingest) does itself with the streams that
// outgrow it, instead of listing them for the next promotion round: 2 =
// count them fatal (the last class), 4 = defer them (the next class has no
// slot during this call: the round would defer every one), 0 = list them.
int overflow_direct(const gk_set* h, int c) {
  const int R = h->st.nclass;
  if (c < 1 || c >= R || h->big[c]) return 0;
  if (c == R - 1) return fatal_direct(h) ? 2 : 0;
  return h->st.alloc[c + 1] == 0 ? 4 : 0;
}

GKPoolDev pool_args(const gk_set* h) {
  GKPoolDev p;
  p.ctr = h->d_ctr;
  p.rcnt = h->d_ctr + GK_CTR_RCNT;
  p.defer = h->d_defer;
  for (int c = 0; c < GK_MAX_CLASSES; ++c) {
    p.list[c] = h->d_list[c];
    p.rerun[c] = h->d_rerun[c];
  }
  return p;
}

// Global workspace of class c (ingest and merge share it), for classes beyond
// LDS; allocated when the class gets its first slots.
int ensure_ws(gk_set* h, int c) {
  const int cap = h->st.cap[c];
  if (h->d_ws[c] || (cap <= kMaxLdsCap && !h->big[c])) return GK_OK;
  size_t b = std::max(h->big[c] ? gk_big_ws_bytes(cap, h->P) : gk_ingest_ws_bytes(cap, h->vpl),
                      gk_merge_lds_bytes(cap, h->st.pmax));
  b = (b + 4095) & ~(size_t)4095;
  // class 0 holds every stream: many waves; a larger class only the rare
  // streams that outgrew the ones below, so a few blocks per 4096 streams.
  // At most ~2 GiB of workspace per class.
  const int64_t S = std::max<int64_t>(h->S, 1);
  int64_t blocks = c == 0 ? std::min<int64_t>(S, (int64_t)gk_num_cu() * 8)
                          : std::min<int64_t>(gk_num_cu(), std::max<int64_t>(8, S / 4096));
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, ((int64_t)2 << 30) / (int64_t)b));
  if (hipMalloc(&h->d_ws[c], b * blocks) != hipSuccess) {
    h->d_ws[c] = nullptr;
    return fail(GK_E_NOMEM, "class-%d workspace of %lld x %zu bytes failed", c, (long long)blocks, b);
  }
  h->ws_bytes[c] = b;
  h->ws_blocks[c] = blocks;
  return GK_OK;
}

// Slots a class starts with (grown on demand, see grow_pools): every stream
// while that costs at most 1 GiB (then no call can run out of slots), else a
// share of the streams.
int64_t initial_slots(const gk_set* h, int c) {
  const int64_t S = std::max<int64_t>(h->S, 1);
  if (c > 0 && h->st.cap[c] > kCapHuge) return 0;  // unbounded classes: on first use
  if (const char* e = getenv("GK_POOL_SLOTS"))  // tests: force tiny arenas (deferral / growth paths)
    return std::max<int64_t>(1, std::min<int64_t>(S, atoll(e)));
  const int64_t slot_bytes = (int64_t)h->st.cap[c] * (int64_t)sizeof(GKRec);
  if (S * slot_bytes <= ((int64_t)1 << 30)) return S;
  const int64_t n = h->st.cap[c] <= kCapLarge ? std::max<int64_t>(4096, S / 16) : std::max<int64_t>(64, S / 1024);
  return std::min<int64_t>(n, S);
}

// Grow class c's arena to `want` slots, keeping the slots handed out so far.
// Synchronises `s` (the arena may be in use by earlier launches).
int grow_class(gk_set* h, int c, int64_t want, hipStream_t s) {
  want = std::min<int64_t>(want, std::max<int64_t>(h->S, 1));
  if (want <= h->st.alloc[c]) return GK_OK;
  HIP_TRY(hipStreamSynchronize(s));
  if (ensure_ws(h, c) != GK_OK) return GK_E_NOMEM;
  int32_t used = 0;
  HIP_TRY(hipMemcpy(&used, h->d_ctr + GK_CTR_USED + c, sizeof(int32_t), hipMemcpyDeviceToHost));
  const int64_t keep = std::min<int64_t>(std::max(used, 0), h->st.alloc[c]);
  GKRec* nt = nullptr;
  if (hipMalloc(&nt, (size_t)want * h->st.cap[c] * sizeof(GKRec)) != hipSuccess)
    return fail(GK_E_NOMEM, "class-%d arena of %lld slots failed", c, (long long)want);
  if (h->st.tab[c] && keep) {
    HIP_TRY(hipMemcpy(nt, h->st.tab[c], (size_t)keep * h->st.cap[c] * sizeof(GKRec), hipMemcpyDeviceToDevice));
  }
  if (h->st.tab[c]) (void)hipFree(h->st.tab[c]);
  h->st.tab[c] = nt;
  h->st.alloc[c] = (int32_t)want;
  return GK_OK;
}

// Consume the counters read back at the end of the last call: report streams
// that found no class / slot (sticky GK_E_OVERFLOW), learn the presort
// workspace the last call needed.  block: wait for that call to finish.
void poll(gk_set* h, bool block) {
  if (!h->done_pending) return;
  if (block) {
    if (hipEventSynchronize(h->ev_done) != hipSuccess) return;
  } else if (hipEventQuery(h->ev_done) != hipSuccess) {
    return;
  }
  h->done_pending = false;
  if (h->void_defer) {
    h->h_ctr[GK_CTR_DEFER] = 0;
    h->void_defer = false;
  }
  if (h->ps.wg_count && h->wg_trace && h->h_ctr[GK_CTR_WORDS] > 0)
    fprintf(stderr, "[gk] k_ingest_wg: %d stream(s)\n", h->h_ctr[GK_CTR_WORDS]);
  const int32_t fatal = h->h_ctr[GK_CTR_FATAL];
  if (fatal > h->fatal_seen && h->sticky == GK_OK) {
    char buf[512];
    snprintf(buf, sizeof(buf),
             "%d stream(s) (largest id %d) outgrew every table capacity class (largest %d entries), found no "
             "free slot, or passed the per-stream count limit 2*eps*(n-1) <= 2^30: their values of that call "
             "were not added (past the last flush that fitted the smallest class, if one did)",
             fatal - h->fatal_seen, h->h_ctr[GK_CTR_FATAL + 1], h->st.cap[h->st.nclass - 1]);
    h->sticky = GK_E_OVERFLOW;
    h->sticky_msg = buf;
  }
  h->fatal_seen = fatal;
}

int promote_rounds(gk_set* h, const double* x, const int64_t* offs, int force, const GKQuery& q, hipStream_t s,
                   bool fresh = false);
int mark_done(gk_set* h, hipStream_t s, bool ingest = false);

// Start of a call's device work: ONE memset zeroes every per-call counter
// (deferred / long-stream counts, re-run and overflow list lengths, the
// launches' stream hand-out counters; gk_launch.h GK_CTR_*).
int begin_call(gk_set* h, hipStream_t s) {
  if (!h->ctr_clean)
    HIP_TRY(hipMemsetAsync(h->d_ctr + GK_CTR_CALL, 0, GK_CALL_BYTES - GK_CTR_CALL * sizeof(int32_t), s));
  h->ctr_clean = false;
  h->next_work = 0;
  return GK_OK;
}

// The zeroed hand-out counter of the call's next launch (the small-class
// launch has its own GK_WORK_BYTES block).
unsigned long long* work_counter(gk_set* h, bool small) {
  if (small) return h->d_work;
  if (h->next_work >= GK_CALL_SLOTS) return nullptr;  // (launches per call are bounded: 1 + R-1 + R(R-1)/2)
  return (unsigned long long*)((char*)h->d_work + GK_WORK_BYTES + 128 * (h->next_work++));
}

// GK_TRACE=1: the host runtime's slow-path decisions on stderr (debugging)
bool g_trace = getenv("GK_TRACE") != nullptr;
#define GK_TR(...)                      \
  do {                                  \
    if (g_trace) {                      \
      fprintf(stderr, "[gk] " __VA_ARGS__); \
      fputc('\n', stderr);              \
      fflush(stderr);                   \
    }                                   \
  } while (0)

// Grow the arenas for the `count` streams of device list `list`, each moving
// one class up (deferred ingest streams, import overflows): the target class
// of each is read back (synchronises), so only the classes they go to grow --
// the unbounded classes (MiB..GiB per slot) are allocated only when used.
int grow_targets(gk_set* h, const int32_t* list, int64_t count, hipStream_t s) {
  if (count <= 0) return GK_OK;
  std::vector<int32_t> ids(count), cls(std::max<int64_t>(h->S, 1));
  HIP_TRY(hipStreamSynchronize(s));
  HIP_TRY(hipMemcpy(ids.data(), list, count * sizeof(int32_t), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(cls.data(), h->st.cls, h->S * sizeof(int32_t), hipMemcpyDeviceToHost));
  int64_t need[GK_MAX_CLASSES] = {};
  for (int32_t id : ids) {
    const int t = cls[id] + 1;
    if (t < h->st.nclass) ++need[t];
  }
  for (int c = 1; c < h->st.nclass; ++c) {
    if (!need[c]) continue;
    int32_t used = 0;
    HIP_TRY(hipMemcpy(&used, h->d_ctr + GK_CTR_USED + c, sizeof(int32_t), hipMemcpyDeviceToHost));
    int64_t want = (int64_t)used + 2 * need[c];
    if (h->st.cap[c] <= kCapHuge) want = std::max<int64_t>(want, 2 * (int64_t)h->st.alloc[c]);
    GK_TR("grow_targets: class %d used %d need %lld -> want %lld", c, used, (long long)need[c], (long long)want);
    int rc = grow_class(h, c, want, s);
    if (rc) return rc;
  }
  return GK_OK;
}

// Streams the last call deferred (their next class had no free slot): grow
// the arenas and run them again, from that call's inputs, before anything
// else touches the set.
int replay_deferred(gk_set* h, hipStream_t s) {
  for (int guard = 0; guard < 2 * GK_MAX_CLASSES + 2; ++guard) {
    const int32_t nd = h->h_ctr[GK_CTR_DEFER];
    if (nd <= 0) return GK_OK;
    h->h_ctr[GK_CTR_DEFER] = 0;
    GK_TR("replay: %d deferred stream(s), round %d", nd, guard);
    int rc = grow_targets(h, h->d_defer, nd, s);
    GK_TR("replay: grown rc=%d", rc);
    if (rc) return rc;
    // the deferred list becomes round 0's overflow list of a fresh call
    HIP_TRY(hipMemcpyAsync(h->d_ovfl[0], h->d_defer, (size_t)nd * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
    int rb = begin_call(h, s);
    if (rb) return rb;
    h->h_ovf[0] = nd;  // pinned; the stream is synchronised below before it is reused
    HIP_TRY(hipMemcpyAsync(h->d_ovfc, h->h_ovf, sizeof(int32_t), hipMemcpyHostToDevice, s));
    rc = promote_rounds(h, h->last.x, h->last.offs, h->last.force, h->last.q, s);
    GK_TR("replay: enqueued rc=%d", rc);
    if (!rc) rc = mark_done(h, s);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    GK_TR("replay: done");
    poll(h, true);
  }
  return fail(GK_E_OVERFLOW, "deferred streams could not be placed in a capacity class");
}

void hc_drain(gk_set* h);

// Before a call (and in gk_sync): settle the previous call -- wait for it when
// it may have deferred streams (some class could run out of slots), re-run
// those, report its asynchronous errors.
int settle(gk_set* h, hipStream_t s, bool block) {
  hc_drain(h);  // the last call's host walk reads its inputs: done before anything else
  poll(h, block || h->last.may_defer);
  if (h->done_pending) return GK_OK;  // still running, and it cannot have deferred anything
  return replay_deferred(h, s);
}

// Before a call: keep every class's arena at least twice what is in use, so
// that the device-side promotions of the call find free slots.
int grow_pools(gk_set* h, hipStream_t s) {
  int rc = settle(h, s, false);
  if (rc) return rc;
  for (int c = 1; c < h->st.nclass; ++c) {
    const int64_t used = h->h_ctr ? h->h_ctr[GK_CTR_USED + c] : 0;
    if (2 * used > h->st.alloc[c]) {
      int rc = grow_class(h, c, std::max<int64_t>(4 * used, 2 * (int64_t)h->st.alloc[c]), s);
      if (rc) return rc;
    }
  }
  // presort workspace: what the last completed call needed (its long streams
  // flushed unsorted if it did not fit -- same results, slower)
  if (h->ps.ws_need && h->h_ws_need && *h->h_ws_need > h->ps.ws_cap) {
    const int64_t need = *h->h_ws_need;
    const int64_t cap = std::max<int64_t>(need + need / 8, 1 << 20);
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipStreamSynchronize(h->aux));
    if (h->aux2) HIP_TRY(hipStreamSynchronize(h->aux2));
    if (h->aux3) HIP_TRY(hipStreamSynchronize(h->aux3));
    if (h->ps.ws) (void)hipFree(h->ps.ws);
    h->ps.ws = nullptr;
    h->ps.ws_cap = 0;
    if (hipMalloc(&h->ps.ws, (size_t)cap * sizeof(double)) == hipSuccess) {
      h->ps.ws_cap = cap;
    } else {
      h->ps.ws = nullptr;  // not fatal: long streams flush unsorted
      (void)hipGetLastError();
    }
  }
  return GK_OK;
}

// Return (and clear) an asynchronous error of an earlier call.
int take_sticky(gk_set* h) {
  if (h->sticky == GK_OK) return GK_OK;
  const int rc = h->sticky;
  g_err = h->sticky_msg;
  h->sticky = GK_OK;
  h->sticky_msg.clear();
  return rc;
}

// End of a call's device work on `s`: counters -> pinned host memory.
// (ingest: the call listed the long streams -- word GK_CTR_LONG comes back
// too; every other call leaves the host copy of the last ingest's count, which
// stats_fork's fork decision reads)
static_assert(GK_CTR_LONG == GK_CTR_WORDS - 1, "the long-stream count is the last word read back");
int mark_done(gk_set* h, hipStream_t s, bool ingest) {
  HIP_TRY(hipMemcpyAsync(h->h_ctr, h->d_ctr, (GK_CTR_WORDS - (ingest ? 0 : 1)) * sizeof(int32_t),
                         hipMemcpyDeviceToHost, s));
  if (h->ps.wg_count && h->wg_trace)
    HIP_TRY(hipMemcpyAsync(h->h_ctr + GK_CTR_WORDS, h->ps.wg_count, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipEventRecord(h->ev_done, s));
  h->done_pending = true;
  h->void_defer = false;  // (the readback in flight is now this call's)
  return GK_OK;
}

int32_t* ovf_count(gk_set* h, int r) { return h->d_ovfc + r; }
int32_t* ovf_list(gk_set* h, int r) { return h->d_ovfl[r]; }

// Read back round r's overflow count and list (synchronises; merge / import only).
int64_t read_overflow(gk_set* h, int r, hipStream_t stream) {
  if (hipMemcpyAsync(h->h_ovf, h->d_ovfc + r, sizeof(int32_t), hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return fail(GK_E_HIP, "overflow readback failed: %s", hipGetErrorString(hipGetLastError()));
  return h->h_ovf[0];
}

int check_set(const gk_set* h) {
  if (!h) return fail(GK_E_ARG, "null set");
  return GK_OK;
}

hipEvent_t timing_event(std::vector<hipEvent_t>& v, size_t& n) {
  if (n == v.size()) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    v.push_back(e);
  }
  return v[n++];
}

bool stats_fused(const gk_set* h);

// One launch of class c: every stream (c == 0) or the streams of `list`
// whose length is *count_ptr (device).  Overflowing streams go to round r's list.
hipError_t launch_class(gk_set* h, int c, const double* x, const int64_t* offs, const int32_t* list,
                        const int32_t* count_ptr, int r, int force, const GKQuery& q, hipStream_t stream,
                        bool prio = false, bool wg = false, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr,
                        int pmode = 0) {
  if (c > 0 && h->st.alloc[c] == 0) return hipSuccess;  // no slot yet: no member
  unsigned long long* work = work_counter(h, c == 0 && h->st.cap[0] == GK_SMALL_CAP && !h->big[0]);
  if (!work) return hipErrorInvalidValue;
  const GKPoolDev pool = pool_args(h);
  if (h->big[c])
    return gk_launch_ingest_big(h->st.cap[c], h->st, x, offs, list, list ? 0 : h->S, count_ptr, c, force,
                                h->d_ws[c], h->ws_bytes[c], h->ws_blocks[c], ovf_count(h, r), ovf_list(h, r), q,
                                work, h->d_ctr, stream);
  return gk_launch_ingest(h->st.cap[c], h->vpl, h->st, x, offs, list, list ? 0 : h->S, count_ptr, c, force,
                          h->d_ws[c], h->ws_bytes[c], h->ws_blocks[c], ovf_count(h, r), ovf_list(h, r), q, work,
                          prio ? h->d_long_list : nullptr, prio ? h->d_long_count : nullptr,
                          prio && h->ps.ws ? h->ps.ws : nullptr, prio && h->ps.ws ? h->ps.list_ws : nullptr,
                          prio && wg ? h->ps.wg_count : nullptr,
                          (prio && c == 0 && stats_fused(h)) ? h->fused_stats : 0, stream, ev0, ev1, &pool,
                          pmode | overflow_direct(h, c));
}

// gk:52-59 for a batch: k_stats over every stream on `s` (it lists the
// streams longer than GK_STATS_LONG values, longest first), then the long
// streams' sequential _sum/_avg chains on h->aux, beside the ingest launches
// that follow on `s` (they touch neither _sum nor _avg).  stats_join makes
// `s` wait for them and, for a fused query, re-answers the long streams with
// their final _min/_max.
// the small-class batch launch walks the stats chains itself (k_stats then
// only lists the long streams)
bool stats_fused(const gk_set* h) { return h->fused_stats > 0 && h->st.cap[0] == GK_SMALL_CAP; }

// doubles per pinned chunk copy (GK_HOST_CHAIN_CHUNK_MB, default 8 MiB)
const int64_t kHcChunk = []() {
  int64_t mb = 8;
  if (const char* e = getenv("GK_HOST_CHAIN_CHUNK_MB")) mb = std::max<int64_t>(1, std::min<int64_t>(256, atoll(e)));
  return mb << 17;
}();

// Per-thread copy stream, chunk buffers and events for the first `t` host
// threads (made on first use, kept until gk_destroy).
int hc_ensure(gk_set* h, int t) {
  while ((int)h->hc_streams.size() < t) {
    h->hc_streams.push_back(h->hc_copy);
    for (int b = 0; b < 2; ++b) {
      double* p = nullptr;
      if (hipHostMalloc(&p, kHcChunk * sizeof(double)) != hipSuccess) return fail(GK_E_NOMEM, "host-chain buffer");
      h->hc_buf.push_back(p);
      hipEvent_t e = nullptr;
      HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      h->hc_ev.push_back(e);
    }
  }
  return GK_OK;
}

// Walk the chains k_hc_prep picked (blocking): the longest streams first,
// each on one host thread, its values streamed device -> pinned host in
// 2 MiB chunks (the next chunk's copy in flight while the chain walks this
// one) and fed to the host engine's gk:52-59 step.  The final state goes
// back into the pinned records (applied on the device by stats_join).
int run_host_chains(gk_set* h, int* taken) {
  *taken = 0;
  HIP_TRY(hipEventSynchronize(h->ev_hc));
  const int K = std::min(*h->h_hc_count, GK_HC_MAX);
  if (K <= 0) return GK_OK;
  if (!h->hc_copy) HIP_TRY(hipStreamCreateWithFlags(&h->hc_copy, hipStreamNonBlocking));
  // the picked records (k_hc_prep, complete: ev_hc followed it)
  HIP_TRY(hipMemcpyAsync(h->h_hc, h->d_hc, K * sizeof(GKHostChainRec), hipMemcpyDeviceToHost, h->hc_copy));
  HIP_TRY(hipStreamSynchronize(h->hc_copy));
  const int T = std::max(1, std::min(h->hc_threads, K));
  int rc = hc_ensure(h, T);
  if (rc) return rc;
  std::atomic<int> next{0};
  std::atomic<int> err{0};
  std::vector<std::string> msg(T);
  std::vector<double> t_walk(T, 0.0), t_wait(T, 0.0);
  std::vector<int64_t> v_done(T, 0);
  using clk = std::chrono::steady_clock;
  const auto t_start = clk::now();
  auto sec = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); };
  auto worker = [&](int t) {
    hipStream_t hs = h->hc_streams[t];
    double* buf[2] = {h->hc_buf[2 * t], h->hc_buf[2 * t + 1]};
    hipEvent_t ev[2] = {h->hc_ev[2 * t], h->hc_ev[2 * t + 1]};
    for (;;) {
      const int k = next.fetch_add(1);
      if (k >= K || err.load()) return;
      GKHostChainRec& r = h->h_hc[k];
      GKHostStats hs_state{r.n, r.sum, r.avg, r.mn, r.mx};
      const double* src = h->hc_x + r.xo;
      auto issue = [&](int64_t off, int b) -> bool {
        const int64_t c = std::min(kHcChunk, r.len - off);
        return hipMemcpyAsync(buf[b], src + off, c * sizeof(double), hipMemcpyDefault, hs) == hipSuccess &&
               hipEventRecord(ev[b], hs) == hipSuccess;
      };
      bool ok = r.len <= 0 || issue(0, 0);
      int cur = 0;
      for (int64_t off = 0; ok && off < r.len;) {
        const int64_t c = std::min(kHcChunk, r.len - off);
        if (off + c < r.len) ok = issue(off + c, cur ^ 1);
        const auto a = clk::now();
        ok = ok && hipEventSynchronize(ev[cur]) == hipSuccess;
        if (!ok) break;
        const auto b = clk::now();
        gk_host_stat_run(hs_state, buf[cur], c);
        t_wait[t] += sec(a, b);
        t_walk[t] += sec(b, clk::now());
        v_done[t] += c;
        off += c;
        cur ^= 1;
      }
      if (!ok) {
        msg[t] = hipGetErrorString(hipGetLastError());
        err.store(1);
        (void)hipStreamSynchronize(hs);
        return;
      }
      r.sum = hs_state.sum;
      r.avg = hs_state.avg;
      r.mn = hs_state.mn;
      r.mx = hs_state.mx;
    }
  };
  std::vector<std::thread> pool;
  pool.reserve(T - 1);
  for (int t = 1; t < T; ++t) pool.emplace_back(worker, t);
  worker(0);
  for (auto& th : pool) th.join();
  static const bool hc_trace = getenv("GK_HC_TRACE") != nullptr;
  if (hc_trace) {
    double w = 0, q = 0;
    int64_t v = 0;
    for (int t = 0; t < T; ++t) {
      w += t_walk[t];
      q += t_wait[t];
      v += v_done[t];
    }
    fprintf(stderr, "[gk] host chains: %d streams, %lld values on %d threads in %.1f ms (walk %.1f ms = %.2f ns/value, "
            "copy waits %.1f ms, summed over threads)\n", K, (long long)v, T, 1e3 * sec(t_start, clk::now()), 1e3 * w,
            v ? 1e9 * w / (double)v : 0.0, 1e3 * q);
  }
  if (err.load()) {
    for (const std::string& m : msg)
      if (!m.empty()) return fail(GK_E_HIP, "host-walked chains: chunk copy failed: %s", m.c_str());
    return fail(GK_E_HIP, "host-walked chains: chunk copy failed");
  }
  *taken = K;
  return GK_OK;
}

// The set's host-walk worker: walks the chains of each handed-out call (in
// order), then publishes (seq << 2) | status in the pinned flag that the
// call's k_hc_wait reads -- always, on failure too (status 2: k_hc_fallback
// then walks those streams on the device).
void hc_worker_main(gk_set* h) {
  (void)hipSetDevice(h->device);
  for (;;) {
    uint64_t seq = 0;
    {
      std::unique_lock<std::mutex> lk(h->hc_mu);
      h->hc_cv.wait(lk, [h] { return h->hc_stop || !h->hc_jobs.empty(); });
      if (h->hc_jobs.empty()) return;  // stop, nothing left
      seq = h->hc_jobs.front();
    }
    int taken = 0;
    int rc = run_host_chains(h, &taken);
    std::string msg = rc ? g_err : std::string();
    if (!rc && h->hc_fail_inject) {
      rc = GK_E_HIP;
      taken = 0;
      msg = "host-walked chains: failure injected (GK_HC_FAIL)";
    }
    __atomic_store_n(h->h_hc_flag, (unsigned long long)((seq << 2) | (rc == GK_OK ? 1u : 2u)), __ATOMIC_RELEASE);
    {
      std::lock_guard<std::mutex> lk(h->hc_mu);
      h->hc_jobs.pop_front();
      h->hc_last_taken = taken;
      h->hc_last_rc = rc;
      h->hc_last_msg = msg;
    }
    h->hc_cv.notify_all();
  }
}

// Wait until the worker has walked every handed-out call (start of the next
// call, gk_sync, gk_destroy).  A failed walk is not an error of the set: the
// device walked those chains instead (k_hc_fallback).
void hc_drain(gk_set* h) {
  if (!h->hc_thr.joinable()) return;
  std::unique_lock<std::mutex> lk(h->hc_mu);
  h->hc_cv.wait(lk, [h] { return h->hc_jobs.empty(); });
}

void hc_shutdown(gk_set* h) {
  if (!h->hc_thr.joinable()) return;
  {
    std::lock_guard<std::mutex> lk(h->hc_mu);
    h->hc_stop = true;
  }
  h->hc_cv.notify_all();
  h->hc_thr.join();
}

// A call that fails between stats_fork and stats_join: best effort, `s` still
// waits for the aux work, and chains the host would have walked are walked on
// the device (k_hc_fallback with the fail word set).
void stats_abort(gk_set* h, hipStream_t s) {
  if (h->wg_early) (void)hipStreamWaitEvent(s, h->ev_wg, 0);  // (launched by stats_fork: joined here too)
  h->wg_early = false;
  if (h->forked) (void)hipStreamWaitEvent(s, h->ev_join, 0);
  if (h->sl_inline)
    (void)gk_launch_stats_long(h->st, h->sl_x, h->sl_offs, h->d_long_list, nullptr, h->d_long_count, nullptr, s);
  h->sl_inline = false;
  if (h->presort_active) (void)hipStreamWaitEvent(s, h->ev_presort, 0);
  h->presort_active = false;
  if (h->hc_active) {
    const int32_t one = 1;
    if (hipMemcpyAsync(h->d_hc_fail, &one, sizeof(one), hipMemcpyHostToDevice, s) == hipSuccess)
      (void)gk_launch_hc_fallback(h->st, h->hc_x, h->hc_offs, h->d_long_list, h->d_long_n, h->d_hc_count,
                                  h->d_hc_fail, s);
    (void)hipStreamSynchronize(s);  // (`one` lives on this stack frame)
  }
  h->forked = false;
  h->hc_active = false;
}

int stats_fork(gk_set* h, const double* x, const int64_t* offs, hipStream_t s, int force) {
  hipEvent_t t0 = h->timing_stats ? timing_event(h->tev_stats, h->n_stats) : nullptr;
  if (t0) HIP_TRY(hipEventRecord(t0, s));
  // k_ingest_wg ahead of everything else of the call (GK_WG_EARLY, default
  // 1): launched behind the call's counter reset only, its workgroups take
  // their CUs (128 KiB of LDS and 8 waves each) while the chip is still
  // empty and wait on the device for k_long_prep's word; queued behind it,
  // they found the CUs held by the chain walks and the presort and started
  // 3.1-4.2 ms into a 38.9 ms cfg5 call (profiles/r05/r05AF3_*).  Launched
  // only after k_long_prep is enqueued, so that the word is always written.
  // The early workgroups spin on the device until k_long_prep has run, so
  // they are launched early only when the device keeps CUs free for it
  // (gk_wg_early_ok: at least 2 x GK_WG_MAX CUs; a partitioned device or
  // several sets sharing one could otherwise fill every CU with spinning
  // workgroups).  Read per call, like the other GK_WG switches.
  const char* early_s = getenv("GK_WG_EARLY");
  const int early_env = early_s ? atoi(early_s) : 1;
  h->wg_early = false;
  const bool early = early_env && x && h->ps.done && h->ps.wg_count && h->aux2 && h->ps.list_ws && gk_wg_early_ok();
  if (early) HIP_TRY(hipEventRecord(h->ev_go, s));
  // the long-stream list (k_lengths) + k_long_prep, then the fork
  // (k_stats_long needs only the sorted list and the pre-call n: the longest
  // chains start at once), then on `s` the short streams' chains (k_stats,
  // unless the small-class launch walks them) and the presort of the long
  // streams' flush batches
  HIP_TRY(gk_launch_stats(h->st, offs, h->d_long_list, h->d_long_count, s));
  // k_long_prep sorts the list (longest first) and plans the presort /
  // workgroups -- unless the small-class launch carries the stats role
  // (P <= 128: no presort, no workgroups) and no host chain is picked from
  // the sorted list: then it is not needed at all (k_stats_long reads the
  // list in k_lengths' order and the pre-call n from k_lengths' snapshot).
  // k_stats_long must be the first work on `aux` after the fork: queued behind
  // anything, its waves reach the CUs after the persistent ingest grid and run
  // ~3x longer beside it (round 5's k_long_prep on aux: cfg4 x 8 shards
  // 84 -> 118 ms per step, profiles/r05/r05E_*)
  const bool prep = !(stats_fused(h) && !(h->hc_min > 0));
  if (prep)
    HIP_TRY(gk_launch_long_prep(h->st, offs, h->d_long_list, h->d_long_n, h->d_long_count, h->ps, s,
                                early ? h->d_ctr + GK_CTR_WGGO : nullptr));
  unsigned long long* wwork_early = nullptr;
  if (early && prep) {
    wwork_early = work_counter(h, false);
    if (!wwork_early) return fail(GK_E_HIP, "no hand-out counter left for k_ingest_wg");
    HIP_TRY(hipStreamWaitEvent(h->aux2, h->ev_go, 0));
    HIP_TRY(gk_launch_ingest_wg(h->st, x, offs, h->d_long_list, h->ps.wg_count, 0, force, ovf_count(h, 0),
                                ovf_list(h, 0), wwork_early, h->ps, h->aux2, h->d_ctr + GK_CTR_WGGO));
    HIP_TRY(hipEventRecord(h->ev_wg, h->aux2));
    h->wg_early = true;
  }
  // the longest chains to host cores: k_hc_prep picks them (k_stats_long
  // skips them) ahead of the fork, so that `aux` holds nothing but
  // k_stats_long and its waves reach the CUs before the ingest grid of this
  // call (queued behind the pick and its copies they lost that race and ran
  // ~3x longer beside the ingest: cfg4 x8 shards 82 -> 110 ms per step).  The
  // records go to the host on the copy stream; the host walks the chains in
  // stats_join, while the GPU ingests.
  h->hc_active = false;
  // (not while `s` is being captured into a graph: a replay would not hand
  // the call to the worker; the device walks every chain then)
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (h->hc_min > 0 && s && hipStreamIsCapturing(s, &cap) != hipSuccess) cap = hipStreamCaptureStatusNone;
  const bool hc_on = h->hc_min > 0 && cap == hipStreamCaptureStatusNone;
  if (hc_on) {
    // (only the pick's count comes back here; the records follow in
    // run_host_chains when there are any -- every stream of the process
    // shares 4 hardware queues, and copies queued beside `aux` delayed it)
    HIP_TRY(gk_launch_hc_prep(h->st, offs, h->d_long_list, h->d_long_n, h->d_long_count, h->hc_min, h->hc_rel,
                              4 * (int64_t)h->hc_threads, h->d_hc, h->d_hc_count, s));
    HIP_TRY(hipMemcpyAsync(h->h_hc_count, h->d_hc_count, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(h->ev_hc, s));
    h->hc_x = x;
    h->hc_offs = offs;
  }
  const bool presort = h->ps.list_ws && h->ps.ws && h->ps.ws_cap > 0;
  // No fork when nothing but k_stats_long would go to the aux streams and the
  // set's last ingest call listed no long stream (its count comes back with
  // that call's counters): k_stats_long then runs on `s` behind the ingest
  // (stats_join).  Forked, its workgroups must reach the CUs before the
  // persistent ingest grid -- the fork's cross-queue wake-up (~13 us) is then
  // on the step's critical path, and a k_stats_long dispatched beside the
  // ingest grid cost the cfg3 launch 8 % (profiles/r06/r06q_*).  A wrong
  // guess costs time only: the walk is the same on either stream.
  h->sl_inline = stats_fused(h) && !prep && !early && !hc_on && !presort && !h->aux2 && h->h_ctr &&
                 h->h_ctr[GK_CTR_LONG] == 0 && !getenv("GK_SL_FORK");
  if (h->sl_inline) {
    h->sl_x = x;
    h->sl_offs = offs;
  } else {
    HIP_TRY(hipEventRecord(h->ev_fork, s));
  }
  if (wwork_early) {
    // behind k_long_prep, on the same hand-out counter: the streams of any
    // early workgroup that gave up waiting for k_long_prep's word (bounded
    // spin, GK_WG_GO_TICKS); normally none are left and its workgroups leave
    // at once
    HIP_TRY(hipStreamWaitEvent(h->aux2, h->ev_fork, 0));
    HIP_TRY(gk_launch_ingest_wg(h->st, x, offs, h->d_long_list, h->ps.wg_count, 0, force, ovf_count(h, 0),
                                ovf_list(h, 0), wwork_early, h->ps, h->aux2, nullptr));
    HIP_TRY(hipEventRecord(h->ev_wg, h->aux2));
  }
  // Forked ahead of the small-class launch (nothing else between them on
  // `s`): `s` waits until aux has passed the fork, so that k_stats_long's
  // waves reach the CUs before the persistent ingest grid -- dispatched beside
  // it they ran 2x longer and slowed the ingest (cfg4 x 8 shards 79 -> 84 ms
  // per step, profiles/r06/r07i_*).  Costs one cross-queue wake-up (~13 us)
  // on calls that fork (long streams: steps of tens of ms).
  const bool sl_order = !h->sl_inline && stats_fused(h) && !presort && !h->aux2;
  if (!h->sl_inline) {
    HIP_TRY(hipStreamWaitEvent(h->aux, h->ev_fork, 0));
    h->forked = true;
    if (sl_order) HIP_TRY(hipEventRecord(h->ev_slgo, h->aux));
    HIP_TRY(gk_launch_stats_long(h->st, x, offs, h->d_long_list, prep ? h->d_long_n : nullptr, h->d_long_count,
                                 hc_on ? h->d_hc_count : nullptr, h->aux));
    h->hc_active = hc_on;  // (stats_join hands the picked chains to the worker)
    HIP_TRY(hipEventRecord(h->ev_join, h->aux));
  }
  if (sl_order) HIP_TRY(hipStreamWaitEvent(s, h->ev_slgo, 0));
  if (presort) {
    // with k_ingest_wg beside it (ps.done): on its own stream, joined by
    // stats_join; else on aux2 ahead of k_ingest_wg
    hipStream_t ps_s = h->ps.done ? h->aux3 : h->aux2;
    HIP_TRY(hipStreamWaitEvent(ps_s, h->ev_fork, 0));
    HIP_TRY(gk_launch_presort(h->st, x, offs, h->d_long_list, h->d_long_n, h->d_long_count, h->ps, ps_s));
    HIP_TRY(hipEventRecord(h->ev_presort, ps_s));
    h->presort_active = true;
  }
  if (!stats_fused(h)) HIP_TRY(gk_launch_stats_short(h->st, x, offs, s));
  // (with k_ingest_wg every presorted stream is one of its streams: the
  // one-wave launch runs beside the presort; k_ingest_wg is ordered after it
  // on aux2)
  if (presort && !h->ps.wg_count) HIP_TRY(hipStreamWaitEvent(s, h->ev_presort, 0));
  if (h->ps.ws_need) HIP_TRY(hipMemcpyAsync(h->h_ws_need, h->ps.ws_need, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  hipEvent_t t1 = h->timing_stats ? timing_event(h->tev_stats, h->n_stats) : nullptr;
  if (t1) HIP_TRY(hipEventRecord(t1, s));
  return GK_OK;
}

int stats_join(gk_set* h, hipStream_t s, const GKQuery& q) {
  if (h->wg_early) {  // (run_ingest returned before joining the early k_ingest_wg)
    h->wg_early = false;
    HIP_TRY(hipStreamWaitEvent(s, h->ev_wg, 0));
  }
  if (h->sl_inline) {
    h->sl_inline = false;
    HIP_TRY(gk_launch_stats_long(h->st, h->sl_x, h->sl_offs, h->d_long_list, nullptr, h->d_long_count, nullptr, s));
  } else {
    HIP_TRY(hipStreamWaitEvent(s, h->ev_join, 0));
  }
  h->forked = false;
  if (h->presort_active) {
    h->presort_active = false;
    HIP_TRY(hipStreamWaitEvent(s, h->ev_presort, 0));
  }
  if (h->hc_active) {
    h->hc_active = false;
    // hand the call to the worker (it walks while the GPU ingests) and join
    // it on `s`: nothing here waits on the host
    if (!h->hc_thr.joinable()) {
      h->hc_stop = false;
      try {
        h->hc_thr = std::thread(hc_worker_main, h);
      } catch (...) {
        return fail(GK_E_HIP, "cannot start the host-chain worker thread");
      }
    }
    const uint64_t seq = ++h->hc_seq;
    {
      std::lock_guard<std::mutex> lk(h->hc_mu);
      h->hc_jobs.push_back(seq);
    }
    h->hc_cv.notify_all();
    HIP_TRY(gk_launch_hc_wait(h->h_hc_flag, seq, h->d_hc_fail, h->hc_timeout_s, s));
    // (the copy engine reads the pinned records once k_hc_wait has seen the
    // worker's flag; the next call's readback of them is ordered after it:
    // its fork waits on `s`, and the next call first drains the worker)
    HIP_TRY(hipMemcpyAsync(h->d_hc, h->h_hc, GK_HC_MAX * sizeof(GKHostChainRec), hipMemcpyHostToDevice, s));
    HIP_TRY(gk_launch_hc_apply(h->st, h->d_hc, h->d_hc_count, h->d_hc_fail, s));
    HIP_TRY(gk_launch_hc_fallback(h->st, h->hc_x, h->hc_offs, h->d_long_list, h->d_long_n, h->d_hc_count,
                                  h->d_hc_fail, s));
  }
  // (+ the _min/_max markers of the small-class launch's answers when it
  // carried the stats role: its chains are final here)
  HIP_TRY(gk_launch_query_list(h->st, h->d_long_list, h->d_long_count, q, stats_fused(h), s));
  return GK_OK;
}

// The ingest / flush launches of one call, with no host round trip: class 0
// over every stream and each larger class over its member list; a stream
// that outgrows its class is not committed, moves one class up on the device
// (k_promote_dev) and runs again there, at most once per class; a stream
// with no class left is counted as fatal (reported by a later call).
// Promotion rounds of a call: round r-1's overflow list moves one class up
// on the device and runs again in its new class (round r).  fresh: every
// stream started the call in class 0 (gk_create / gk_reset, nothing promoted
// since), so after r rounds no stream is above class r: round r re-runs
// class r only (the launches of the classes above would find their re-run
// lists empty).
int promote_rounds(gk_set* h, const double* x, const int64_t* offs, int force, const GKQuery& q, hipStream_t stream,
                   bool fresh) {
  const int R = h->st.nclass;
  GKPoolDev pool = pool_args(h);
  bool ran = true;  // a launch ran in the previous round (round 0: class 0)
  for (int r = 1; r <= R; ++r) {
    // (fresh: round r-1 re-ran class r-1 only; a class with no slots has no
    // launch, and then round r has nothing to promote)
    if (fresh && !ran) break;
    // (past the last class only fatal streams are left to count, and with
    // fatal_direct its launches counted them; fresh: round r-1 re-ran class
    // r-1 only, which counted or deferred its overflows itself)
    if (r == R && fatal_direct(h)) break;
    if (fresh && overflow_direct(h, r - 1)) break;
    int32_t* rcnt = h->d_ctr + GK_CTR_RCNT + GK_MAX_CLASSES * r;  // zeroed at the start of the call
    pool.rcnt = rcnt;
    h->no_members = false;
    // Fused round: every class launched this round has slots and runs
    // k_ingest, so each launch promotes the streams of round r-1's overflow
    // list whose next class is its own (k_ingest pmode bit 0) -- no
    // k_promote_dev launch and no re-run list.  GK_PROMOTE_FUSE=0: always the
    // separate promotion.
    const int c_end = fresh ? std::min(r + 1, R) : R;
    const bool fuse_env = !getenv("GK_PROMOTE_FUSE") || atoi(getenv("GK_PROMOTE_FUSE")) != 0;  // (per call: A/B, tests)
    bool fuse = fuse_env && r < R;
    for (int c = r; c < c_end; ++c) fuse = fuse && h->st.alloc[c] > 0 && !h->big[c];
    if (fuse) {
      ran = false;
      for (int c = r; c < c_end; ++c) {
        ran = true;
        HIP_TRY(launch_class(h, c, x, offs, ovf_list(h, r - 1), ovf_count(h, r - 1), r, force, q, stream, false, false,
                             nullptr, nullptr, 1));
        if (g_trace) {
          HIP_TRY(hipStreamSynchronize(stream));
          GK_TR("round %d: class %d promoted + re-run (fused)", r, c);
        }
      }
      continue;
    }
    HIP_TRY(gk_launch_promote_dev(h->st, ovf_count(h, r - 1), ovf_list(h, r - 1), -1, pool, stream));
    if (g_trace) {
      HIP_TRY(hipStreamSynchronize(stream));
      GK_TR("round %d: promoted", r);
    }
    if (r == R) break;  // the last promotion only counts what no class can hold
    ran = false;
    for (int c = r; c < (fresh ? r + 1 : R); ++c) {
      ran |= h->st.alloc[c] > 0;  // (launch_class launches nothing without slots)
      HIP_TRY(launch_class(h, c, x, offs, h->d_rerun[c], rcnt + c, r, force, q, stream));
      if (g_trace) {
        HIP_TRY(hipStreamSynchronize(stream));
        GK_TR("round %d: class %d re-run done", r, c);
      }
    }
  }
  return GK_OK;
}

int run_ingest(gk_set* h, const double* x, const int64_t* offs, int force, hipStream_t stream,
               const GKQuery& q = GKQuery(), bool prio = false) {
  if (!offs) offs = h->d_zero_offs;
  const int R = h->st.nclass;
  const bool fresh = h->no_members;  // (promote_rounds clears it)
  h->last.x = x;
  h->last.offs = offs;
  h->last.force = force;
  h->last.q = q;
  h->last.may_defer = false;
  for (int c = 1; c < R; ++c) h->last.may_defer |= h->st.alloc[c] < h->S;
  // (the call's counters were zeroed by begin_call)
  // timing covers the class-0 batch launch of gk_ingest (x given) only
  const bool timed = h->timing && x != nullptr;
  // the longest presorted streams of an ingest: one workgroup each, on aux2
  // right behind their presort, beside the class-0 launch (which skips them)
  // (a stream whose batches are not presorted -- no workspace yet, or it did
  // not fit -- is ranked unsorted there)
  const bool wg = prio && x != nullptr && h->ps.wg_count && h->aux2 && h->ps.list_ws;
  // The small-class launch alone records the pair as part of its dispatch
  // (the kernel's own start and end; two marker packets around it cost the
  // step ~12 us of dispatch gaps); with k_ingest_wg beside it the markers
  // span both launches.
  bool ext = timed && !wg && h->st.cap[0] == GK_SMALL_CAP && !h->big[0];
  hipEvent_t t0 = timed ? timing_event(h->tev_flush, h->n_flush) : nullptr;
  hipEvent_t t1x = (ext && t0) ? timing_event(h->tev_flush, h->n_flush) : nullptr;
  if (ext && !t1x) {  // (no second event: markers, paired as before)
    ext = false;
    if (t0) --h->n_flush;
    t0 = timed ? timing_event(h->tev_flush, h->n_flush) : nullptr;
  }
  if (t0 && !ext) HIP_TRY(hipEventRecord(t0, stream));
  if (wg && !h->wg_early) {
    unsigned long long* wwork = work_counter(h, false);
    if (!wwork) return fail(GK_E_HIP, "no hand-out counter left for k_ingest_wg");
    // (behind k_long_prep, which counts its streams, and the call's counter
    // reset: the fork point; the presort, when there is one, is already
    // ordered after it on aux2)
    HIP_TRY(hipStreamWaitEvent(h->aux2, h->ev_fork, 0));
    HIP_TRY(gk_launch_ingest_wg(h->st, x, offs, h->d_long_list, h->ps.wg_count, 0, force, ovf_count(h, 0),
                                ovf_list(h, 0), wwork, h->ps, h->aux2));
    HIP_TRY(hipEventRecord(h->ev_wg, h->aux2));
  }
  const hipError_t lc = launch_class(h, 0, x, offs, nullptr, nullptr, 0, force, q, stream, prio && x != nullptr, wg,
                                     ext ? t0 : nullptr, ext ? t1x : nullptr);
  // (its overflow entries feed the promotion rounds below).  k_ingest_wg is
  // joined on every path once launched: the next call's begin_call zeroes the
  // counter block it adds to
  if (wg) HIP_TRY(hipStreamWaitEvent(stream, h->ev_wg, 0));
  h->wg_early = false;
  HIP_TRY(lc);
  // (with k_ingest_wg beside it, the timed span is both: the call's batch ingest)
  hipEvent_t t1 = (timed && !ext) ? timing_event(h->tev_flush, h->n_flush) : nullptr;
  if (t1) HIP_TRY(hipEventRecord(t1, stream));
  if (!h->no_members)
    for (int c = 1; c < R; ++c)
      HIP_TRY(launch_class(h, c, x, offs, h->d_list[c], h->d_ctr + GK_CTR_LCNT + c, 0, force, q, stream));
  return promote_rounds(h, x, offs, force, q, stream, fresh);
}

// Merge / explicit merge_compress at LDS capacity level 0, then the streams
// that did not fit at increasing levels (their class raised on the device).
// Synchronous (one readback per level).
int run_merge(gk_set* dst, const MergeArgsHost& base, hipStream_t s) {
  MergeArgsHost a = base;
  const GKPoolDev pool = pool_args(dst);
  int64_t todo = 0;
  dst->ctr_clean = false;
  HIP_TRY(hipMemsetAsync(dst->d_ovfc, 0, kRounds * sizeof(int32_t), s));
  for (int level = 0; level < dst->st.nclass; ++level) {
    const int cap = dst->st.cap[level];
    if (level > 0) {
      if (todo == 0) return GK_OK;
      // streams below this class move up so that their output may grow
      int rc = grow_class(dst, level, (int64_t)dst->st.alloc[level] + todo, s);
      if (rc) return rc;
      dst->no_members = false;
      HIP_TRY(gk_launch_promote_dev(dst->st, ovf_count(dst, level - 1), ovf_list(dst, level - 1), level, pool, s));
    }
    a.dst = dst->st;
    a.cap = cap;
    a.list = level == 0 ? nullptr : ovf_list(dst, level - 1);
    a.count = level == 0 ? dst->S : todo;
    a.ovf_count = ovf_count(dst, level);
    a.ovf_list = ovf_list(dst, level);
    if (cap > kMaxLdsCap) {
      int rc = ensure_ws(dst, level);
      if (rc) return rc;
      a.ws = dst->d_ws[level];
      a.ws_bytes = dst->ws_bytes[level];
      a.ws_blocks = dst->ws_blocks[level];
    } else {
      a.ws = nullptr;
      a.ws_bytes = 0;
      a.ws_blocks = 0;
    }
    HIP_TRY(gk_launch_merge(a, s));
    todo = read_overflow(dst, level, s);
    if (todo < 0) return (int)todo;
    if (todo == 0) return GK_OK;
  }
  return fail(GK_E_OVERFLOW, "%lld stream(s) exceed %d table entries in merge, or the per-stream count limit "
              "2*eps*(n-1) <= 2^30", (long long)todo, dst->st.cap[dst->st.nclass - 1]);
}

}  // namespace

extern "C" {

int gk_version(void) { return 100; }

const char* gk_last_error(void) { return g_err.c_str(); }

int gk_create(int64_t num_streams, double eps, int64_t cap_hint, int device, gk_set** out) {
  if (!out) return fail(GK_E_ARG, "out is null");
  *out = nullptr;
  if (num_streams < 0 || num_streams > INT32_MAX) return fail(GK_E_ARG, "num_streams out of range");
  // any finite eps > 0, as the reference (gk:21); eps > 1 gives P = 1 (gk:60)
  if (!std::isfinite(eps) || !(eps > 0.0)) return fail(GK_E_ARG, "eps must be finite and > 0");
  const double inv = 1.0 / eps;
  if (inv >= (double)kPMax)
    return fail(GK_E_UNSUPPORTED, "eps=%g: flush period int(1/eps)+1 beyond %d is not supported", eps, kPMax);
  if (cap_hint < 0 || cap_hint >= kCapMax) return fail(GK_E_UNSUPPORTED, "cap_hint %lld out of range", (long long)cap_hint);
  std::vector<int> caps;
  std::vector<bool> force_big;
  if (const char* e = getenv("GK_CAPS")) {  // tests: an explicit ladder, "128,2048,4096b" (b: k_ingest_big)
    for (const char* t = e; *t;) {
      char* end = nullptr;
      const long v = strtol(t, &end, 10);
      if (end == t) return fail(GK_E_ARG, "GK_CAPS=%s: bad list", e);
      caps.push_back((int)v);
      force_big.push_back(*end == 'b');
      t = end + (*end == 'b');
      if (*t == ',') ++t;
    }
    const double P0 = (double)((int)inv + 1);
    bool okc = !caps.empty() && (int)caps.size() <= GK_MAX_CLASSES;
    for (size_t c = 0; okc && c < caps.size(); ++c) {
      okc = caps[c] >= 64 && caps[c] <= kCapMax && (c == 0 || caps[c] > caps[c - 1]);
      if (caps[c] == kCapSmall) okc = okc && c == 0 && P0 <= 128;
    }
    if (!okc) return fail(GK_E_ARG, "GK_CAPS=%s: increasing capacities in [64, %d], 128 only first", e, kCapMax);
  }
  int dev_count = 0;
  if (hipGetDeviceCount(&dev_count) != hipSuccess || dev_count <= 0)
    return fail(GK_E_HIP, "no HIP device available");
  if (device < 0 || device >= dev_count) return fail(GK_E_ARG, "device %d out of range", device);
  HIP_TRY(hipSetDevice(device));

  gk_set* h = new gk_set();
  h->S = num_streams;
  h->eps = eps;
  h->P = (int)inv + 1;  // gk:60
  h->device = device;
  h->vpl = h->P <= 1024 ? vpl_for(h->P) : 0;  // (registers of the capacity-class kernels)
  if (const char* fs = getenv("GK_FUSED_STATS")) h->fused_stats = std::max(0, std::min(64, atoi(fs)));
  // host-walked chains: off by default since round 4 (the device's
  // speculative walk of k_stats_long runs a 10^7-value chain in a few ms,
  // faster than a host core plus the PCIe copy of its values).  GK_HOST_CHAINS=1
  // turns them on for streams of >= 2^20 values (GK_HOST_CHAIN_MIN sets the
  // length and turns them on too; GK_HOST_CHAINS=0 wins) on up to 16 host
  // threads (GK_HOST_CHAIN_THREADS; the process's CPU share: its affinity
  // set, OMP_NUM_THREADS if lower)
  h->hc_min = 0;
  if (const char* e = getenv("GK_HOST_CHAINS"))
    if (atoi(e) != 0) h->hc_min = (int64_t)1 << 20;
  if (const char* e = getenv("GK_HOST_CHAIN_MIN")) h->hc_min = std::max<int64_t>(0, atoll(e));
  if (const char* e = getenv("GK_HOST_CHAINS"))
    if (atoi(e) == 0) h->hc_min = 0;
  if (const char* e = getenv("GK_HOST_CHAIN_REL")) h->hc_rel = std::max(0, std::min(100, atoi(e)));
  {
    int t = 16;
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0 && CPU_COUNT(&cs) > 0) t = std::min(t, CPU_COUNT(&cs));
    if (const char* e = getenv("OMP_NUM_THREADS"))
      if (atoi(e) > 0) t = std::min(t, atoi(e));
    if (const char* e = getenv("GK_HOST_CHAIN_THREADS"))
      if (atoi(e) > 0) t = atoi(e);
    h->hc_threads = std::max(1, std::min(t, GK_HC_MAX));
  }
  GKState& st = h->st;
  st.S = num_streams;
  st.eps = eps;
  st.two_eps = 2.0 * eps;
  st.inv_eps = inv;
  st.P = h->P;
  st.pmax = h->P;
  // Capacity ladder.  Class 0 (every stream) is the 128-entry LDS class when
  // a flush period fits two values per lane (iid tables at eps=0.01 stay at
  // <= ~106 entries); adversarial streams are promoted to 2048
  // (LDS), 32768 (global workspace) and then the unbounded classes of
  // k_ingest_big.  With P > 1024 (eps < 1/1023) every class is k_ingest_big:
  // class 0 of 2P entries (iid tables hold ~P/2..P), then x16 steps.
  auto pow2_at_least = [](int64_t v) {
    int64_t c = 1;
    while (c < v) c <<= 1;
    return c;
  };
  if (caps.empty()) {
    if (h->P <= 1024) {
      if (h->P <= 128 && cap_hint <= kCapSmall) caps = {kCapSmall, kCapLarge, kCapHuge, kCapBig};
      else if (cap_hint <= kCapLarge) caps = {kCapLarge, kCapHuge, kCapBig};
      else if (cap_hint < kCapHuge) caps = {kCapHuge, kCapBig};
    }
    if (caps.empty()) {
      int64_t c = std::max<int64_t>({4096, pow2_at_least(2 * (int64_t)h->P), pow2_at_least(cap_hint + 1)});
      for (; (int)caps.size() < GK_MAX_CLASSES && c <= kCapMax; c *= 16) caps.push_back((int)c);
      if (caps.back() < kCapMax && (int)caps.size() < GK_MAX_CLASSES) caps.push_back(kCapMax);
    }
  }
  st.nclass = (int)caps.size();
  for (int c = 0; c < GK_MAX_CLASSES; ++c) {
    st.cap[c] = c < st.nclass ? caps[c] : 0;
    const bool lds = (st.cap[c] == kCapSmall && c == 0) || st.cap[c] == kCapLarge;
    h->big[c] = c < st.nclass && (h->P > 1024 || st.cap[c] > kCapHuge || (!force_big.empty() && force_big[c]) ||
                                  (st.cap[c] <= kMaxLdsCap && !lds));
  }
  const int64_t S = std::max<int64_t>(num_streams, 1);
  bool okm = true;
  okm &= hipMalloc(&st.n, S * sizeof(int64_t)) == hipSuccess;
  okm &= hipMalloc(&st.E, S * sizeof(int32_t)) == hipSuccess;
  okm &= hipMalloc(&st.pend, S * sizeof(int32_t)) == hipSuccess;
  okm &= hipMalloc(&st.mn, S * sizeof(double)) == hipSuccess;
  okm &= hipMalloc(&st.mx, S * sizeof(double)) == hipSuccess;
  okm &= hipMalloc(&st.sum, S * sizeof(double)) == hipSuccess;
  okm &= hipMalloc(&st.avg, S * sizeof(double)) == hipSuccess;
  okm &= hipMalloc(&st.cls, S * sizeof(int32_t)) == hipSuccess;
  okm &= hipMalloc(&st.slot, S * sizeof(int32_t)) == hipSuccess;
  okm &= hipMalloc(&st.tab[0], (size_t)S * st.cap[0] * sizeof(GKRec)) == hipSuccess;
  okm &= hipMalloc(&st.pbuf, (size_t)S * st.pmax * sizeof(double)) == hipSuccess;
  st.rtab_n = kRecipTable;
  okm &= hipMalloc(&st.rtab, (size_t)st.rtab_n * sizeof(double)) == hipSuccess;
  okm &= hipMalloc(&st.n0, S * sizeof(int64_t)) == hipSuccess;

  for (int r = 0; r < kRounds; ++r) okm &= hipMalloc(&h->d_ovfl[r], S * sizeof(int32_t)) == hipSuccess;
  okm &= hipHostMalloc(&h->h_ovf, 16 * sizeof(int32_t)) == hipSuccess;
  okm &= hipMalloc(&h->d_ctr, GK_CALL_BYTES) == hipSuccess;
  if (h->d_ctr) {
    h->d_ovfc = h->d_ctr + GK_CTR_OVFC;
    h->d_long_count = h->d_ctr + GK_CTR_LONG;
    h->d_work = (unsigned long long*)((char*)h->d_ctr + GK_CALL_WORK);
  }
  okm &= hipHostMalloc(&h->h_ctr, (GK_CTR_WORDS + 1) * sizeof(int32_t)) == hipSuccess;  // + the call's wg count
  okm &= hipMalloc(&h->d_defer, S * sizeof(int32_t)) == hipSuccess;
  if (h->h_ctr) memset(h->h_ctr, 0, GK_CTR_WORDS * sizeof(int32_t));
  okm &= hipEventCreateWithFlags(&h->ev_done, hipEventDisableTiming) == hipSuccess;
  okm &= hipEventCreateWithFlags(&h->ev_qs, hipEventDisableTiming) == hipSuccess;
  st.alloc[0] = (int32_t)S;
  for (int c = 1; c < st.nclass; ++c) {
    okm &= hipMalloc(&h->d_list[c], S * sizeof(int32_t)) == hipSuccess;
    okm &= hipMalloc(&h->d_rerun[c], S * sizeof(int32_t)) == hipSuccess;
    const int64_t n = initial_slots(h, c);
    if (n > 0) okm &= hipMalloc(&st.tab[c], (size_t)n * st.cap[c] * sizeof(GKRec)) == hipSuccess;
    st.alloc[c] = (int32_t)n;
  }
  okm &= hipMalloc(&h->d_zero_offs, (S + 1) * sizeof(int64_t)) == hipSuccess;

  okm &= hipMalloc(&h->d_long_list, S * sizeof(int32_t)) == hipSuccess;
  okm &= hipMalloc(&h->d_long_n, S * sizeof(int64_t)) == hipSuccess;

  okm &= hipStreamCreateWithFlags(&h->aux, hipStreamNonBlocking) == hipSuccess;
  // (hc_copy is made on first use, run_host_chains: an idle stream still
  // takes a slot in the round-robin over the box's 4 hardware queues, and
  // with 8 sets the long chains' `aux` then shared the caller's queue more
  // often)
  // (aux2 only where the presort runs: every stream of a process shares the
  // box's 4 hardware queues, and a set's idle stream still takes a slot in
  // their round-robin -- with 8 sets of 3 streams the cfg4 shards' long
  // chains landed behind the next shard's ingest)
  if (h->P > 128 && !h->big[0]) okm &= hipStreamCreateWithFlags(&h->aux2, hipStreamNonBlocking) == hipSuccess;
  okm &= hipEventCreateWithFlags(&h->ev_presort, hipEventDisableTiming) == hipSuccess;
  okm &= hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) == hipSuccess;
  okm &= hipEventCreateWithFlags(&h->ev_slgo, hipEventDisableTiming) == hipSuccess;
  okm &= hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) == hipSuccess;
  okm &= hipMalloc(&h->d_hc, GK_HC_MAX * sizeof(GKHostChainRec)) == hipSuccess;
  okm &= hipMalloc(&h->d_hc_count, sizeof(int32_t)) == hipSuccess;
  okm &= hipHostMalloc(&h->h_hc, GK_HC_MAX * sizeof(GKHostChainRec)) == hipSuccess;
  okm &= hipHostMalloc(&h->h_hc_count, sizeof(int32_t)) == hipSuccess;
  // the worker's flag: coherent pinned memory that k_hc_wait polls
  okm &= hipHostMalloc(&h->h_hc_flag, sizeof(unsigned long long), hipHostMallocCoherent | hipHostMallocMapped) ==
         hipSuccess;
  okm &= hipMalloc(&h->d_hc_fail, sizeof(int32_t)) == hipSuccess;
  okm &= h->d_hc_fail && hipMemset(h->d_hc_fail, 0, sizeof(int32_t)) == hipSuccess;
  if (h->h_hc_flag) *h->h_hc_flag = 0;
  if (const char* e = getenv("GK_HC_FAIL")) h->hc_fail_inject = atoi(e) != 0;
  okm &= hipEventCreateWithFlags(&h->ev_hc, hipEventDisableTiming) == hipSuccess;
  if (h->P > 128 && !h->big[0]) {  // class 0 is a capacity-class kernel: presort long streams' batches
    okm &= hipMalloc(&h->ps.list_ws, S * sizeof(int64_t)) == hipSuccess;
    okm &= hipMalloc(&h->ps.list_b0, (S + 1) * sizeof(int64_t)) == hipSuccess;
    okm &= hipMalloc(&h->ps.ws_need, sizeof(int64_t)) == hipSuccess;
    okm &= hipHostMalloc(&h->h_ws_need, sizeof(int64_t)) == hipSuccess;
    if (h->h_ws_need) *h->h_ws_need = 0;
    // the longest streams: one workgroup each (k_ingest_wg, 2048 class,
    // P <= 1024; GK_WG=0 turns it off); their count is a per-call word.
    // Their batches are presorted (GK_WG_PRESORT=0: not; k_ingest_wg then
    // ranks each value among its gap's members)
    bool wg = st.cap[0] == 2048 && h->P <= 1024;
    if (const char* e = getenv("GK_WG")) wg = wg && atoi(e) != 0;
    if (wg) h->ps.wg_count = h->d_ctr + GK_CTR_WG;
    h->ps.wg_presort = 1;
    if (const char* e = getenv("GK_WG_PRESORT")) h->ps.wg_presort = atoi(e) != 0;
    // the register presort beside k_ingest_wg (which takes presorted batches
    // once it is done and ranks unsorted ones until then); GK_WG_CONC=0: the
    // workgroups wait for the presort
    bool conc = wg && h->ps.wg_presort && gk_presort_reg_grid(st) > 0;
    if (const char* e = getenv("GK_WG_CONC")) conc = conc && atoi(e) != 0;
    if (conc) {
      h->ps.done = h->d_ctr + GK_CTR_PSDONE;
      okm &= hipStreamCreateWithFlags(&h->aux3, hipStreamNonBlocking) == hipSuccess;
    }
    h->wg_trace = getenv("GK_WG_TRACE") != nullptr;
    okm &= hipEventCreateWithFlags(&h->ev_wg, hipEventDisableTiming) == hipSuccess;
    okm &= hipEventCreateWithFlags(&h->ev_go, hipEventDisableTiming) == hipSuccess;
  }
  if (!okm) {
    gk_destroy(h);
    return fail(GK_E_NOMEM, "device allocation for %lld streams failed", (long long)num_streams);
  }
  for (int c = 0; c < st.nclass; ++c) {  // classes with slots: their workspace (entered inside any call)
    if (st.alloc[c] > 0 && ensure_ws(h, c) != GK_OK) {
      gk_destroy(h);
      return GK_E_NOMEM;
    }
  }
  if (hipMemset(st.cls, 0, S * sizeof(int32_t)) != hipSuccess ||
      hipMemset(h->d_ctr, 0, GK_CALL_BYTES) != hipSuccess ||
      hipMemset(h->d_zero_offs, 0, (S + 1) * sizeof(int64_t)) != hipSuccess ||
      hipMemset(st.slot, 0, S * sizeof(int32_t)) != hipSuccess || gk_launch_reset(st, nullptr) != hipSuccess ||
      gk_launch_rtab(st, nullptr) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    gk_destroy(h);
    return fail(GK_E_HIP, "state initialisation failed");
  }
  *out = h;
  return GK_OK;
}

int gk_destroy(gk_set* h) {
  if (!h) return GK_OK;
  hc_shutdown(h);  // the worker finishes its handed-out walks (their joins may be waiting on the device)
  (void)hipDeviceSynchronize();  // launches of this set may still be running on the caller's stream
  if (h->fold_scratch) gk_destroy(h->fold_scratch);
  if (h->self_scratch) gk_destroy(h->self_scratch);
  GKState& st = h->st;
  void* ptrs[] = {st.n,       st.E,          st.pend,        st.mn,          st.mx,          st.sum,
                  st.avg,     st.cls,        st.slot,        st.pbuf,        h->d_qs,
                  h->d_ctr,   h->d_zero_offs, h->d_long_list, h->d_long_n,
                  h->ps.list_ws, h->ps.list_b0, h->ps.ws,    h->ps.ws_need,  st.rtab,        st.n0,
                  h->d_defer, h->d_hc,       h->d_hc_count,  h->d_hc_fail};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (int c = 0; c < GK_MAX_CLASSES; ++c)
    for (void* p : {(void*)st.tab[c], (void*)h->d_list[c], (void*)h->d_rerun[c], (void*)h->d_ws[c]})
      if (p) (void)hipFree(p);
  for (int r = 0; r < kRounds; ++r)
    if (h->d_ovfl[r]) (void)hipFree(h->d_ovfl[r]);
  for (auto* v : {&h->tev_flush, &h->tev_stats})
    for (hipEvent_t e : *v) (void)hipEventDestroy(e);
  for (hipEvent_t e : {h->ev_fork, h->ev_join, h->ev_slgo, h->ev_done, h->ev_qs, h->ev_hc})
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : h->hc_ev) (void)hipEventDestroy(e);
  if (h->hc_copy) (void)hipStreamDestroy(h->hc_copy);
  if (h->aux2) (void)hipStreamDestroy(h->aux2);
  if (h->aux3) (void)hipStreamDestroy(h->aux3);
  if (h->ev_presort) (void)hipEventDestroy(h->ev_presort);
  if (h->ev_wg) (void)hipEventDestroy(h->ev_wg);
  if (h->ev_go) (void)hipEventDestroy(h->ev_go);
  for (double* p : h->hc_buf) (void)hipHostFree(p);
  if (h->aux) (void)hipStreamDestroy(h->aux);
  for (void* p : {(void*)h->h_ws_need, (void*)h->h_ovf, (void*)h->h_ctr, (void*)h->h_qs, (void*)h->h_hc,
                  (void*)h->h_hc_count, (void*)h->h_hc_flag})
    if (p) (void)hipHostFree(p);
  delete h;
  return GK_OK;
}

int gk_reset(gk_set* h, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  // No wait for the last call: streams it deferred for
  // want of a slot would only be re-run to be reset; their re-run is void.
  // (Waiting here put the host's enqueueing of every step on the GPU's
  // critical path: ~90 us of idle GPU per step, 10 % of a 125k-stream rank
  // share.)  The last call's counters are consumed when they arrive: its
  // sticky errors are still reported, its deferred list is dropped.
  hc_drain(h);  // (the host walk reads the last call's inputs)
  poll(h, false);
  if (h->done_pending) h->void_defer = true;
  else h->h_ctr[GK_CTR_DEFER] = 0;
  h->last.may_defer = false;
  // (k_reset puts every stream back in class 0: cls = slot = 0)
  // slots, member lists and re-run lists start over (FATAL stays cumulative:
  // a readback still in flight carries it)
  // (+ counter words [0, GK_CTR_FATAL) and the per-call block: no separate
  // memset, and none at the next call's begin_call)
  HIP_TRY(gk_launch_reset(h->st, s, h->d_ctr));
  h->no_members = true;
  h->ctr_clean = true;
  return GK_OK;
}

int gk_ingest(gk_set* h, const double* values, const int64_t* offsets, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!offsets) return fail(GK_E_ARG, "offsets is null");
  if (!values) return fail(GK_E_ARG, "values is null");
  if (h->S == 0) return GK_OK;
  hipStream_t s = (hipStream_t)stream;
  rc = grow_pools(h, s);
  if (!rc) rc = take_sticky(h);
  if (!rc) rc = begin_call(h, s);
  if (rc) return rc;
  rc = stats_fork(h, values, offsets, s, 0);
  if (rc) {
    stats_abort(h, s);
    return rc;
  }
  rc = run_ingest(h, values, offsets, 0, s, GKQuery(), true);
  const int rj = stats_join(h, s, GKQuery());  // joined on every path
  const int rd = mark_done(h, s, true);
  return rc ? rc : (rj ? rj : rd);
}

int gk_flush(gk_set* h, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (h->S == 0) return GK_OK;
  hipStream_t s = (hipStream_t)stream;
  rc = grow_pools(h, s);
  if (!rc) rc = take_sticky(h);
  if (!rc) rc = begin_call(h, s);
  if (rc) return rc;
  rc = run_ingest(h, nullptr, nullptr, 1, s);
  const int rd = mark_done(h, s);
  return rc ? rc : rd;
}

int gk_sync(gk_set* h, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  rc = settle(h, (hipStream_t)stream, true);
  return rc ? rc : take_sticky(h);
}

// quantile arguments -> device copy of qs and the effective mode
static int prepare_query(gk_set* h, const double* qs, int nq, double* out, int mode, hipStream_t s, GKQuery* q) {
  if (nq < 0 || (nq > 0 && (!qs || !out))) return fail(GK_E_ARG, "bad quantile arguments");
  if (mode != GK_Q_LIST && mode != GK_Q_SINGLE) return fail(GK_E_ARG, "bad mode %d", mode);
  for (int i = 0; i < nq; ++i)
    if (std::isnan(qs[i])) return fail(GK_E_ARG, "cannot convert float NaN to integer");
  // gk:205-206: an unsorted list is answered q by q with quantile()
  int eff_mode = mode;
  if (mode == GK_Q_LIST) {
    for (int i = 1; i < nq; ++i)
      if (qs[i] < qs[i - 1]) {
        eff_mode = GK_Q_SINGLE;
        break;
      }
  }
  // the previous call's copy out of h_qs (and its kernels' reads of d_qs,
  // ordered on the same stream) must not see the new values
  HIP_TRY(hipEventSynchronize(h->ev_qs));
  if (nq > h->qs_alloc) {
    HIP_TRY(hipStreamSynchronize(s));
    if (h->d_qs) (void)hipFree(h->d_qs);
    if (h->h_qs) (void)hipHostFree(h->h_qs);
    h->d_qs = nullptr;
    h->h_qs = nullptr;
    const int cap = std::max(nq, 64);
    if (hipMalloc(&h->d_qs, cap * sizeof(double)) != hipSuccess ||
        hipHostMalloc(&h->h_qs, cap * sizeof(double)) != hipSuccess)
      return fail(GK_E_NOMEM, "qs allocation failed");
    h->qs_alloc = cap;
    h->qs_n = 0;
  }
  // (the same list as the last upload -- every step of a serving loop --
  // is already on the device: no copy, no blit launch)
  if (nq && !(nq == h->qs_n && memcmp(h->h_qs, qs, nq * sizeof(double)) == 0)) {
    memcpy(h->h_qs, qs, nq * sizeof(double));
    HIP_TRY(hipMemcpyAsync(h->d_qs, h->h_qs, nq * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(h->ev_qs, s));
    h->qs_n = nq;
  }
  q->qs = nq ? h->d_qs : nullptr;
  q->nq = nq;
  q->out = out;
  q->mode = eff_mode;
  return GK_OK;
}

int gk_quantiles(gk_set* h, const double* qs, int nq, double* out, int mode, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  // settle the previous call first: a deferred stream of it is re-run with
  // that call's query (h->last.q reads d_qs), which the upload below replaces
  rc = grow_pools(h, s);
  if (rc) return rc;
  GKQuery q;
  rc = prepare_query(h, qs, nq, out, mode, s, &q);
  if (rc) return rc;
  if (nq == 0 || h->S == 0) return GK_OK;
  rc = take_sticky(h);
  if (!rc) rc = begin_call(h, s);
  if (rc) return rc;
  // gk:197-198: pending values are flushed first (state mutation); the
  // quantiles are answered in the same launch from the flushed table
  rc = run_ingest(h, nullptr, nullptr, 1, s, q);
  const int rd = mark_done(h, s);
  return rc ? rc : rd;
}

int gk_ingest_quantiles(gk_set* h, const double* values, const int64_t* offsets, const double* qs, int nq,
                        double* out, int mode, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!offsets) return fail(GK_E_ARG, "offsets is null");
  if (!values) return fail(GK_E_ARG, "values is null");
  hipStream_t s = (hipStream_t)stream;
  rc = grow_pools(h, s);  // before d_qs is rewritten (see gk_quantiles)
  if (rc) return rc;
  GKQuery q;
  rc = prepare_query(h, qs, nq, out, mode, s, &q);
  if (rc) return rc;
  if (h->S == 0) return GK_OK;
  if (nq == 0) return gk_ingest(h, values, offsets, stream);
  rc = take_sticky(h);
  if (!rc) rc = begin_call(h, s);
  if (rc) return rc;
  rc = stats_fork(h, values, offsets, s, 1);
  if (rc) {
    stats_abort(h, s);
    return rc;
  }
  // add every value (gk:49-61), then quantiles() (gk:187-232): flush the
  // leftover pending values and answer from the LDS-resident table
  rc = run_ingest(h, values, offsets, 1, s, q, true);
  const int rj = stats_join(h, s, q);  // joined on every path
  const int rd = mark_done(h, s, true);
  return rc ? rc : (rj ? rj : rd);
}

int gk_stats(gk_set* h, int64_t* n, double* mn, double* mx, double* sum, double* avg, int32_t* table_size,
             int32_t* pending, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  rc = settle(h, (hipStream_t)stream, false);  // a deferred stream of the last call is re-run first
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const int64_t S = h->S;
  if (S == 0) return GK_OK;
  if (n) HIP_TRY(hipMemcpyAsync(n, h->st.n, S * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
  if (mn) HIP_TRY(hipMemcpyAsync(mn, h->st.mn, S * sizeof(double), hipMemcpyDeviceToDevice, s));
  if (mx) HIP_TRY(hipMemcpyAsync(mx, h->st.mx, S * sizeof(double), hipMemcpyDeviceToDevice, s));
  if (sum) HIP_TRY(hipMemcpyAsync(sum, h->st.sum, S * sizeof(double), hipMemcpyDeviceToDevice, s));
  if (avg) HIP_TRY(hipMemcpyAsync(avg, h->st.avg, S * sizeof(double), hipMemcpyDeviceToDevice, s));
  if (table_size) HIP_TRY(hipMemcpyAsync(table_size, h->st.E, S * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  if (pending) HIP_TRY(hipMemcpyAsync(pending, h->st.pend, S * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  return GK_OK;
}

static int merge_self(gk_set* dst, hipStream_t s, void* stream);

int gk_merge(gk_set* dst, gk_set* const* srcs, int nsrcs, void* stream) {
  int rc = check_set(dst);
  if (rc) return rc;
  if (nsrcs < 0 || (nsrcs > 0 && !srcs)) return fail(GK_E_ARG, "bad source list");
  for (int k = 0; k < nsrcs; ++k) {
    if (!srcs[k]) return fail(GK_E_ARG, "null source %d", k);
    if (srcs[k]->eps != dst->eps)  // gk:118-119
      return fail(GK_E_EPS_MISMATCH, "Cannot merge two GKArrays with different epsilon values");
    if (srcs[k]->S != dst->S)
      return fail(GK_E_ARG, "stream counts differ (%lld vs %lld)", (long long)srcs[k]->S, (long long)dst->S);
  }
  hipStream_t s = (hipStream_t)stream;
  rc = gk_sync(dst, stream);
  if (rc) return rc;
  for (int k = 0; k < nsrcs; ++k) {
    gk_set* src = srcs[k];
    if (src == dst) {  // dst.merge(dst): the reference accepts it (gk:111-154)
      rc = merge_self(dst, s, stream);
      if (rc) return rc;
      continue;
    }
    // a repeated source is flushed again at each of its merges (gk:137)
    rc = gk_sync(src, stream);
    if (rc) return rc;
    // other.merge_compress() -- unconditional in the reference (gk:126, 137)
    rc = begin_call(src, s);
    if (!rc) rc = run_ingest(src, nullptr, nullptr, 2, s);
    if (!rc) rc = mark_done(src, s);
    if (!rc) rc = gk_sync(src, stream);
    if (rc) return rc;
    MergeArgsHost a{};
    a.src = src->st;
    a.mode = 0;
    rc = run_merge(dst, a, s);
    if (rc) return rc;
  }
  HIP_TRY(hipStreamSynchronize(s));
  return GK_OK;
}

int gk_merge_compress(gk_set* h, const double* v, const int32_t* g, const int32_t* d, const int64_t* eoffs,
                      void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!eoffs || !v || !g || !d) return fail(GK_E_ARG, "null record arrays");
  hipStream_t s = (hipStream_t)stream;
  rc = gk_sync(h, stream);
  if (rc) return rc;
  MergeArgsHost a{};
  a.src = h->st;
  a.ev = v;
  a.eg = g;
  a.ed = d;
  a.eoffs = eoffs;
  a.mode = 1;
  rc = run_merge(h, a, s);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s));
  return GK_OK;
}

int gk_export_sizes(gk_set* h, int32_t* sizes, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  rc = settle(h, (hipStream_t)stream, false);  // a deferred stream of the last call is re-run first
  if (rc) return rc;
  if (!sizes) return fail(GK_E_ARG, "sizes is null");
  if (h->S)
    HIP_TRY(hipMemcpyAsync(sizes, h->st.E, h->S * sizeof(int32_t), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return GK_OK;
}

int gk_export(gk_set* h, const int64_t* offs, double* v, int32_t* g, int32_t* d, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  rc = settle(h, (hipStream_t)stream, false);  // a deferred stream of the last call is re-run first
  if (rc) return rc;
  if (!offs) return fail(GK_E_ARG, "offs is null");
  HIP_TRY(gk_launch_export(h->st, offs, v, g, d, (hipStream_t)stream));
  return GK_OK;
}

int gk_export_pending_sizes(gk_set* h, int32_t* sizes, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  rc = settle(h, (hipStream_t)stream, false);  // a deferred stream of the last call is re-run first
  if (rc) return rc;
  if (!sizes) return fail(GK_E_ARG, "sizes is null");
  if (h->S)
    HIP_TRY(hipMemcpyAsync(sizes, h->st.pend, h->S * sizeof(int32_t), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return GK_OK;
}

int gk_export_pending(gk_set* h, const int64_t* poffs, double* pv, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  rc = settle(h, (hipStream_t)stream, false);  // a deferred stream of the last call is re-run first
  if (rc) return rc;
  if (!poffs || !pv) return fail(GK_E_ARG, "null pointer");
  HIP_TRY(gk_launch_export_pending(h->st, poffs, pv, (hipStream_t)stream));
  return GK_OK;
}

int gk_import(gk_set* h, const int64_t* offs, const double* v, const int32_t* g, const int32_t* d,
              const int64_t* poffs, const double* pv, const int64_t* n, const double* mn, const double* mx,
              const double* sum, const double* avg, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!offs || !poffs || !n || !mn || !mx || !sum || !avg) return fail(GK_E_ARG, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int64_t S = h->S;
  if (S == 0) return GK_OK;
  rc = gk_sync(h, stream);
  if (rc) return rc;
  h->ctr_clean = false;  // (writes words of the per-call block below)
  {
    int32_t* bad = h->d_ctr + GK_CTR_BADPEND;
    HIP_TRY(hipMemsetAsync(bad, 0, sizeof(int32_t), s));
    HIP_TRY(gk_launch_check_pending(S, h->P, n, poffs, bad, s));
    HIP_TRY(hipMemcpyAsync(h->h_ovf, bad, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (h->h_ovf[0] != 0)
      return fail(GK_E_ARG, "%d stream(s) hold more pending values than add() leaves (pending <= n %% %d)",
                  h->h_ovf[0], h->P);
  }
  HIP_TRY(hipMemcpyAsync(h->st.n, n, S * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemcpyAsync(h->st.mn, mn, S * sizeof(double), hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemcpyAsync(h->st.mx, mx, S * sizeof(double), hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemcpyAsync(h->st.sum, sum, S * sizeof(double), hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemcpyAsync(h->st.avg, avg, S * sizeof(double), hipMemcpyDeviceToDevice, s));
  // tables that do not fit their stream's class: one class up (on the
  // device) and import again, until every table fits
  const GKPoolDev pool = pool_args(h);
  for (int round = 0; round <= h->st.nclass; ++round) {
    HIP_TRY(hipMemsetAsync(h->d_ovfc, 0, sizeof(int32_t), s));
    HIP_TRY(gk_launch_import(h->st, offs, v, g, d, poffs, pv, ovf_count(h, 0), ovf_list(h, 0), s));
    const int64_t c = read_overflow(h, 0, s);
    if (c < 0) return (int)c;
    if (c == 0) return GK_OK;
    rc = grow_targets(h, ovf_list(h, 0), c, s);
    if (rc) return rc;
    h->no_members = false;
    HIP_TRY(gk_launch_promote_dev(h->st, ovf_count(h, 0), ovf_list(h, 0), -2, pool, s));
    rc = mark_done(h, s);
    if (!rc) rc = gk_sync(h, stream);
    if (rc) return rc;
  }
  return fail(GK_E_OVERFLOW, "import did not converge");
}

// ---- versioned state files (gk_format.h) ------------------------------------
namespace {

int fmt_error(int rc, const char* path) {
  switch (rc) {
    case gkfmt::E_IO: return fail(GK_E_IO, "cannot read/write state file %s", path);
    case gkfmt::E_VERSION: return fail(GK_E_FORMAT, "%s: unsupported state format version", path);
    case gkfmt::E_CHECKSUM: return fail(GK_E_FORMAT, "%s: checksum mismatch (corrupt state file)", path);
    default: return fail(GK_E_FORMAT, "%s: not a GKSTATE file or truncated", path);
  }
}

// device scratch freed on scope exit (after the stream was synchronised)
struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  bool alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 8) == hipSuccess; }
};

}  // namespace

int gk_save(gk_set* h, const char* path, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!path) return fail(GK_E_ARG, "path is null");
  rc = gk_sync(h, stream);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const int64_t S = h->S;
  gkfmt::State st;
  st.eps = h->eps;
  st.resize_streams(S);
  if (S) {
    HIP_TRY(hipMemcpyAsync(st.sizes.data(), h->st.E, S * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(st.psizes.data(), h->st.pend, S * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(st.n.data(), h->st.n, S * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(st.mn.data(), h->st.mn, S * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(st.mx.data(), h->st.mx, S * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(st.sum.data(), h->st.sum, S * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(st.avg.data(), h->st.avg, S * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  std::vector<int64_t> offs(S + 1, 0), poffs(S + 1, 0);
  for (int64_t k = 0; k < S; ++k) {
    offs[k + 1] = offs[k] + st.sizes[k];
    poffs[k + 1] = poffs[k] + st.psizes[k];
  }
  const int64_t E = offs[S], P = poffs[S];
  st.v.resize(E);
  st.g.resize(E);
  st.d.resize(E);
  st.pv.resize(P);
  if (S) {
    DevBuf d_offs, d_poffs, d_v, d_g, d_d, d_pv;
    if (!d_offs.alloc((S + 1) * 8) || !d_poffs.alloc((S + 1) * 8) || !d_v.alloc(E * 8) || !d_g.alloc(E * 4) ||
        !d_d.alloc(E * 4) || !d_pv.alloc(P * 8))
      return fail(GK_E_NOMEM, "save: device scratch of %lld records failed", (long long)E);
    HIP_TRY(hipMemcpyAsync(d_offs.p, offs.data(), (S + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_poffs.p, poffs.data(), (S + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(gk_launch_export(h->st, (const int64_t*)d_offs.p, (double*)d_v.p, (int32_t*)d_g.p, (int32_t*)d_d.p, s));
    HIP_TRY(gk_launch_export_pending(h->st, (const int64_t*)d_poffs.p, (double*)d_pv.p, s));
    if (E) {
      HIP_TRY(hipMemcpyAsync(st.v.data(), d_v.p, E * 8, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipMemcpyAsync(st.g.data(), d_g.p, E * 4, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipMemcpyAsync(st.d.data(), d_d.p, E * 4, hipMemcpyDeviceToHost, s));
    }
    if (P) HIP_TRY(hipMemcpyAsync(st.pv.data(), d_pv.p, P * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  rc = gkfmt::write(path, st);
  return rc ? fmt_error(rc, path) : GK_OK;
}

int gk_peek(const char* path, double* eps, int64_t* num_streams) {
  if (!path) return fail(GK_E_ARG, "path is null");
  gkfmt::Header hd;
  const int rc = gkfmt::peek(path, &hd);
  if (rc) return fmt_error(rc, path);
  if (eps) *eps = hd.eps;
  if (num_streams) *num_streams = hd.S;
  return GK_OK;
}

int gk_load(gk_set* h, const char* path, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!path) return fail(GK_E_ARG, "path is null");
  gkfmt::State st;
  rc = gkfmt::read(path, &st);
  if (rc) return fmt_error(rc, path);
  if (st.S != h->S)
    return fail(GK_E_ARG, "%s holds %lld streams, the set has %lld", path, (long long)st.S, (long long)h->S);
  if (st.eps != h->eps) return fail(GK_E_EPS_MISMATCH, "%s was saved with eps=%.17g, the set has eps=%.17g", path,
                                   st.eps, h->eps);
  const int64_t S = st.S;
  if (S == 0) return GK_OK;
  hipStream_t s = (hipStream_t)stream;
  std::vector<int64_t> offs(S + 1, 0), poffs(S + 1, 0);
  for (int64_t k = 0; k < S; ++k) {
    offs[k + 1] = offs[k] + st.sizes[k];
    poffs[k + 1] = poffs[k] + st.psizes[k];
    if (st.psizes[k] < 0 || st.n[k] < 0 || st.psizes[k] > st.n[k] % h->P)
      return fail(GK_E_FORMAT, "%s: stream %lld holds %d pending values at n=%lld (at most n mod %d)", path,
                  (long long)k, st.psizes[k], (long long)st.n[k], h->P);
  }
  const int64_t E = offs[S], P = poffs[S];
  DevBuf d_offs, d_poffs, d_v, d_g, d_d, d_pv, d_hdr;
  if (!d_offs.alloc((S + 1) * 8) || !d_poffs.alloc((S + 1) * 8) || !d_v.alloc(E * 8) || !d_g.alloc(E * 4) ||
      !d_d.alloc(E * 4) || !d_pv.alloc(P * 8) || !d_hdr.alloc(5 * S * 8))
    return fail(GK_E_NOMEM, "load: device scratch of %lld records failed", (long long)E);
  int64_t* d_n = (int64_t*)d_hdr.p;
  double* d_f = (double*)d_hdr.p + S;
  HIP_TRY(hipMemcpyAsync(d_offs.p, offs.data(), (S + 1) * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_poffs.p, poffs.data(), (S + 1) * 8, hipMemcpyHostToDevice, s));
  if (E) {
    HIP_TRY(hipMemcpyAsync(d_v.p, st.v.data(), E * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_g.p, st.g.data(), E * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_d.p, st.d.data(), E * 4, hipMemcpyHostToDevice, s));
  }
  if (P) HIP_TRY(hipMemcpyAsync(d_pv.p, st.pv.data(), P * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_n, st.n.data(), S * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_f, st.mn.data(), S * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_f + S, st.mx.data(), S * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_f + 2 * S, st.sum.data(), S * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_f + 3 * S, st.avg.data(), S * 8, hipMemcpyHostToDevice, s));
  rc = gk_import(h, (const int64_t*)d_offs.p, (const double*)d_v.p, (const int32_t*)d_g.p, (const int32_t*)d_d.p,
                 (const int64_t*)d_poffs.p, (const double*)d_pv.p, d_n, d_f, d_f + S, d_f + 2 * S, d_f + 3 * S,
                 stream);
  const hipError_t e = hipStreamSynchronize(s);  // the scratch above is freed on return
  if (rc) return rc;
  if (e != hipSuccess) return fail(GK_E_HIP, "load: %s", hipGetErrorString(e));
  return GK_OK;
}

// ---- packed state (gk_pack.h): device buffers ------------------------------
namespace {
struct DevMem {
  static int to_host(void* host, const void* src, size_t n, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (hipMemcpyAsync(host, src, n, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
      return fail(GK_E_HIP, "packed state: device-to-host copy failed");
    return GK_OK;
  }
  static int from_host(void* dst, const void* host, size_t n, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (hipMemcpyAsync(dst, host, n, hipMemcpyHostToDevice, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
      return fail(GK_E_HIP, "packed state: host-to-device copy failed");
    return GK_OK;
  }
};
}  // namespace

// The size arrays borrow two of the set's S-entry overflow lists (idle
// outside an ingest call; the calls below synchronise first).
int gk_pack_bytes(gk_set* h, int64_t* bytes, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!bytes) return fail(GK_E_ARG, "bytes is null");
  rc = gk_sync(h, stream);
  if (rc) return rc;
  return gkpack::pack_bytes<DevMem>(h, h->d_ovfl[1], h->d_ovfl[2], bytes, stream);
}

int gk_pack(gk_set* h, void* buf, int64_t bytes, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!buf) return fail(GK_E_ARG, "buf is null");
  rc = gk_sync(h, stream);
  if (rc) return rc;
  std::string err;
  rc = gkpack::pack<DevMem>(h, h->d_ovfl[1], h->d_ovfl[2], buf, bytes, stream, err);
  return (rc && !err.empty()) ? fail(rc, "%s", err.c_str()) : rc;
}

// dst.merge(dst), gk:111-154 with `other` IS self: gk:137 flushes dst itself
// (emptying its incoming), gk:138-147 convert that flushed table, gk:149
// doubles n, and gk:154 merges the converted records back.  k_merge reads the
// source table while it rewrites the destination's, so the source is a
// snapshot of the flushed dst: packed into a device buffer and imported into
// a scratch set that is NOT flushed again (a second compress at the same
// threshold is not a no-op).  Its pending count is 0 and its n equals dst's,
// so k_merge takes the general branch (n > 0) or, for an empty stream, the
// "other empty" branch whose flush of an empty stream changes nothing.
static int merge_self(gk_set* dst, hipStream_t s, void* stream) {
  int rc = gk_sync(dst, stream);
  if (!rc) rc = begin_call(dst, s);
  if (!rc) rc = run_ingest(dst, nullptr, nullptr, 2, s);  // other.merge_compress() (gk:137)
  if (!rc) rc = mark_done(dst, s);
  if (!rc) rc = gk_sync(dst, stream);
  if (rc) return rc;
  int64_t bytes = 0;
  rc = gk_pack_bytes(dst, &bytes, stream);
  if (rc) return rc;
  DevBuf buf;
  if (!buf.alloc((size_t)bytes)) return fail(GK_E_NOMEM, "self-merge: snapshot of %lld bytes", (long long)bytes);
  rc = gk_pack(dst, buf.p, bytes, stream);
  if (!rc && !dst->self_scratch) rc = gk_create(dst->S, dst->eps, 0, dst->device, &dst->self_scratch);
  if (rc) return rc;
  std::string err;
  gkpack::Header hd{};
  rc = gkpack::read_header<DevMem>(dst->self_scratch, buf.p, &hd, stream, err);
  if (!rc) rc = gkpack::import_packed<DevMem>(dst->self_scratch, buf.p, hd, stream);
  if (!rc) rc = gk_sync(dst->self_scratch, stream);
  if (rc) return (!err.empty()) ? fail(rc, "%s", err.c_str()) : rc;
  MergeArgsHost a{};
  a.src = dst->self_scratch->st;
  a.mode = 0;
  rc = run_merge(dst, a, s);
  // the snapshot set (a full copy of dst's state) is not kept beyond the
  // merge: the set's memory stays what it was before
  const int rs = gk_sync(dst, stream);
  gk_destroy(dst->self_scratch);
  dst->self_scratch = nullptr;
  return rc ? rc : rs;
}

int gk_fold_packed(gk_set* dst, const void* const* bufs, int nbufs, void* stream) {
  int rc = check_set(dst);
  if (rc) return rc;
  rc = gk_sync(dst, stream);
  if (rc) return rc;
  std::string err;
  auto make = [&](gk_set** out) { return gk_create(dst->S, dst->eps, 0, dst->device, out); };
  rc = gkpack::fold<DevMem>(dst, bufs, nbufs, &dst->fold_scratch, make, stream, err);
  return (rc && !err.empty()) ? fail(rc, "%s", err.c_str()) : rc;
}

int64_t gk_num_streams(const gk_set* h) { return h ? h->S : -1; }
double gk_eps(const gk_set* h) { return h ? h->eps : 0.0; }
int gk_flush_period(const gk_set* h) { return h ? h->P : -1; }
int gk_capacity(const gk_set* h, int cls) {
  return (h && cls >= 0 && cls < h->st.nclass) ? h->st.cap[cls] : -1;
}
int64_t gk_host_chains_taken(gk_set* h) {
  if (!h) return -1;
  hc_drain(h);
  // the device's verdict on the last host-walked call: k_hc_wait sets the
  // fail word when the worker reported a failure or its flag came too late
  // (the chains were then walked on the device: k_hc_fallback), even if the
  // worker finished OK afterwards
  // (on the set's device, after the set's last call: ev_done follows its
  // k_hc_wait; nothing else on the device is waited for -- ADVICE r05)
  int32_t dev_fail = 0;
  int prev = 0;
  (void)hipGetDevice(&prev);
  bool ok = hipSetDevice(h->device) == hipSuccess && hipEventSynchronize(h->ev_done) == hipSuccess &&
            hipMemcpy(&dev_fail, h->d_hc_fail, sizeof(dev_fail), hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipSetDevice(prev);
  if (!ok) return -1;
  std::lock_guard<std::mutex> lk(h->hc_mu);
  return (h->hc_last_rc == GK_OK && dev_fail == 0) ? h->hc_last_taken : 0;
}

int64_t gk_num_promoted(const gk_set* h) {
  if (!h) return -1;
  if (h->S == 0) return 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (settle(const_cast<gk_set*>(h), nullptr, true) != GK_OK) return -1;  // deferred streams placed first
  std::vector<int32_t> cls(h->S);
  if (hipMemcpy(cls.data(), h->st.cls, h->S * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  int64_t n = 0;
  for (int32_t c : cls) n += c > 0;
  return n;
}

int gk_timing_enable(gk_set* h, int on) {
  int rc = check_set(h);
  if (rc) return rc;
  h->timing = (on & 1) != 0;
  h->timing_stats = (on & 2) != 0;
  return GK_OK;
}

int gk_timing_read(gk_set* h, double* flush_ms, double* stats_ms, int64_t* launches) {
  int rc = check_set(h);
  if (rc) return rc;
  double f = 0, st = 0;
  for (size_t k = 0; k + 1 < h->n_flush; k += 2) {
    float ms = 0;
    HIP_TRY(hipEventSynchronize(h->tev_flush[k + 1]));
    HIP_TRY(hipEventElapsedTime(&ms, h->tev_flush[k], h->tev_flush[k + 1]));
    f += ms;
  }
  for (size_t k = 0; k + 1 < h->n_stats; k += 2) {
    float ms = 0;
    HIP_TRY(hipEventSynchronize(h->tev_stats[k + 1]));
    HIP_TRY(hipEventElapsedTime(&ms, h->tev_stats[k], h->tev_stats[k + 1]));
    st += ms;
  }
  if (flush_ms) *flush_ms = f;
  if (stats_ms) *stats_ms = st;
  if (launches) *launches = (int64_t)(h->n_flush / 2);
  h->n_flush = h->n_stats = 0;
  return GK_OK;
}

}  // extern "C"
