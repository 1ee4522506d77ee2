// gk_capi.cpp -- C ABI runtime of the MI355X batched GKArray engine.
//
// Owns the per-set device state (header arrays, table arenas, pending
// buffers), decides flush modes and table-capacity classes, and launches the
// kernels of gk_kernels.hip on the caller's HIP stream.  Every entry point is
// declared in include/gk_capi.h with the reference method it replaces.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gk_capi.h"
#include "gk_launch.h"
#include "gk_state.h"

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
constexpr int64_t kOvfPrefix = 4096;     // overflow entries read back with the count
constexpr int kCapLarge = 2048;  // LDS class, ~92 KB per wave
constexpr int kCapHuge = 32768;  // global-workspace class
constexpr int64_t kRecipTable = (int64_t)1 << 17;  // entries of st.rtab (1 MiB)
constexpr int kMaxLdsCap = 2048;

int vpl_for(int P) {
  int v = 1;
  while (v * 64 < P) v <<= 1;
  return v;
}

}  // namespace

struct gk_set {
  int64_t S = 0;
  double eps = 0;
  int P = 0;
  int device = 0;
  int vpl = 1;
  GKState st{};
  std::vector<int8_t> h_cls;  // host mirror of st.cls
  // per class c >= 1: arena bookkeeping and member list (host + device copy)
  int64_t slots_alloc[GK_MAX_CLASSES] = {0, 0, 0};
  int64_t slots_used[GK_MAX_CLASSES] = {0, 0, 0};
  std::vector<int32_t> members[GK_MAX_CLASSES];
  int32_t* d_list[GK_MAX_CLASSES] = {nullptr, nullptr, nullptr};
  int64_t list_alloc[GK_MAX_CLASSES] = {0, 0, 0};
  // global workspace for classes beyond LDS
  unsigned char* d_ws = nullptr;
  size_t ws_bytes = 0;
  int64_t ws_blocks = 0;
  // overflow reporting
  int32_t* d_ovf_count = nullptr;  // d_ovf[0]
  int32_t* d_ovf_list = nullptr;   // d_ovf + 1: one buffer, so count + list come back in one copy
  int32_t* d_ovf = nullptr;
  int32_t* h_ovf = nullptr;        // pinned: count + the first kOvfPrefix list entries
  std::vector<int32_t> h_slots[GK_MAX_CLASSES];  // promotion slots per target class (kept until the next sync)
  int64_t* d_zero_offs = nullptr;  // S+1 zeros: offsets of flush-only launches
  unsigned long long* d_work = nullptr;  // stream hand-out counter of the small-class kernel
  int32_t* d_long_list = nullptr;        // streams k_stats hands to k_stats_long (longest first)
  int64_t* d_long_n = nullptr;           //   and their pre-call n
  int32_t* d_long_count = nullptr;
  // k_stats_long (the sequential _sum/_avg chains of long streams) runs on
  // this stream beside the ingest launches; ev_fork / ev_join order it
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // presorted flush batches of long streams (sets whose class 0 is the 2048
  // class): plan arrays, workspace, and the size the last call needed
  GKPresort ps;
  int64_t* h_ws_need = nullptr;  // pinned host copy of *ps.ws_need
  // scratch
  double* d_qs = nullptr;
  int qs_alloc = 0;
  int32_t* d_tmp_list = nullptr;
  int32_t* d_tmp_slots = nullptr;
  int64_t tmp_alloc = 0;
  // eighths of a wave per CU of the small-class batch launch that walk the gk:52-59
  // stats chains first (0: separate k_stats launch); GK_FUSED_STATS overrides
  int fused_stats = 7;
  // timing
  bool timing = false;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  double flush_ms = 0, stats_ms = 0;
  int64_t launches = 0;
};

namespace {

int ensure_tmp(gk_set* h, int64_t n) {
  if (n <= h->tmp_alloc) return GK_OK;
  if (h->d_tmp_list) (void)hipFree(h->d_tmp_list);
  if (h->d_tmp_slots) (void)hipFree(h->d_tmp_slots);
  h->d_tmp_list = nullptr;
  h->d_tmp_slots = nullptr;
  const int64_t cap = std::max<int64_t>(n, 1024);
  if (hipMalloc(&h->d_tmp_list, cap * sizeof(int32_t)) != hipSuccess ||
      hipMalloc(&h->d_tmp_slots, cap * sizeof(int32_t)) != hipSuccess)
    return fail(GK_E_NOMEM, "scratch allocation of %lld entries failed", (long long)cap);
  h->tmp_alloc = cap;
  return GK_OK;
}

int ensure_ws(gk_set* h) {
  if (h->d_ws) return GK_OK;
  const int cap = h->st.cap[h->st.nclass - 1];
  if (cap <= kMaxLdsCap) return GK_OK;
  size_t b = std::max(gk_ingest_ws_bytes(cap, h->vpl), gk_merge_lds_bytes(cap, h->st.pmax));
  b = (b + 4095) & ~(size_t)4095;
  int64_t blocks = std::min<int64_t>(gk_num_cu(), 256);
  if (hipMalloc(&h->d_ws, b * blocks) != hipSuccess)
    return fail(GK_E_NOMEM, "workspace of %lld x %zu bytes failed", (long long)blocks, b);
  h->ws_bytes = b;
  h->ws_blocks = blocks;
  return GK_OK;
}

// Grow the arena of class c so that `need` slots exist (copying live slots).
int ensure_slots(gk_set* h, int c, int64_t need, hipStream_t stream) {
  if (need <= h->slots_alloc[c]) return GK_OK;
  int64_t cap = std::max<int64_t>(h->slots_alloc[c] * 2, std::max<int64_t>(need, c == 1 ? 256 : 16));
  GKRec* nt = nullptr;
  if (hipMalloc(&nt, (size_t)cap * h->st.cap[c] * sizeof(GKRec)) != hipSuccess)
    return fail(GK_E_NOMEM, "class-%d arena of %lld slots failed", c, (long long)cap);
  if (h->st.tab[c]) {
    HIP_TRY(hipMemcpyAsync(nt, h->st.tab[c], (size_t)h->slots_used[c] * h->st.cap[c] * sizeof(GKRec),
                           hipMemcpyDeviceToDevice, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    (void)hipFree(h->st.tab[c]);
  }
  h->st.tab[c] = nt;
  h->slots_alloc[c] = cap;
  return GK_OK;
}

int sync_list(gk_set* h, int c, hipStream_t stream) {
  const int64_t n = (int64_t)h->members[c].size();
  if (n > h->list_alloc[c]) {
    if (h->d_list[c]) (void)hipFree(h->d_list[c]);
    h->d_list[c] = nullptr;
    const int64_t cap = std::max<int64_t>(n * 2, 256);
    if (hipMalloc(&h->d_list[c], cap * sizeof(int32_t)) != hipSuccess)
      return fail(GK_E_NOMEM, "class-%d list allocation failed", c);
    h->list_alloc[c] = cap;
  }
  if (n)
    HIP_TRY(hipMemcpyAsync(h->d_list[c], h->members[c].data(), n * sizeof(int32_t), hipMemcpyHostToDevice, stream));
  return GK_OK;
}

// Read back the overflow list of the last launch(es); returns count (>= 0) or
// error.  The count and the first kOvfPrefix entries come back in one copy
// (one synchronisation); a longer list takes a second copy.
int64_t read_overflow(gk_set* h, std::vector<int32_t>& out, hipStream_t stream) {
  const int64_t pre = std::min<int64_t>(h->S, kOvfPrefix);
  if (hipMemcpyAsync(h->h_ovf, h->d_ovf, (1 + pre) * sizeof(int32_t), hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return fail(GK_E_HIP, "overflow readback failed: %s", hipGetErrorString(hipGetLastError()));
  const int32_t cnt = h->h_ovf[0];
  out.resize(cnt);
  if (cnt) {
    if (cnt <= pre) {
      std::copy(h->h_ovf + 1, h->h_ovf + 1 + cnt, out.begin());
    } else if (hipMemcpyAsync(out.data(), h->d_ovf_list, cnt * sizeof(int32_t), hipMemcpyDeviceToHost, stream) !=
                   hipSuccess ||
               hipStreamSynchronize(stream) != hipSuccess) {
      return fail(GK_E_HIP, "overflow list readback failed");
    }
    std::sort(out.begin(), out.end());
  }
  return cnt;
}

// Move the listed streams (all currently below class `ncls`) to class `ncls`.
int promote(gk_set* h, const std::vector<int32_t>& ids, int ncls, hipStream_t stream) {
  if (ids.empty()) return GK_OK;
  if (ncls >= h->st.nclass)
    return fail(GK_E_OVERFLOW, "%zu stream(s) exceed the largest table capacity (%d entries)", ids.size(),
                h->st.cap[h->st.nclass - 1]);
  int rc = ensure_slots(h, ncls, h->slots_used[ncls] + (int64_t)ids.size(), stream);
  if (rc) return rc;
  rc = ensure_tmp(h, (int64_t)ids.size());
  if (rc) return rc;
  if (h->st.cap[ncls] > kMaxLdsCap) {
    rc = ensure_ws(h);
    if (rc) return rc;
  }
  // host sources of the copies below stay alive until the caller's next
  // synchronisation (ids: the caller's list; slots: h_slots)
  std::vector<int32_t>& slots = h->h_slots[ncls];
  slots.resize(ids.size());
  for (size_t k = 0; k < ids.size(); ++k) slots[k] = (int32_t)(h->slots_used[ncls] + (int64_t)k);
  HIP_TRY(hipMemcpyAsync(h->d_tmp_list, ids.data(), ids.size() * sizeof(int32_t), hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemcpyAsync(h->d_tmp_slots, slots.data(), slots.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                         stream));
  HIP_TRY(gk_launch_promote(h->st, h->d_tmp_list, (int64_t)ids.size(), h->d_tmp_slots, ncls, stream));
  h->slots_used[ncls] += (int64_t)ids.size();
  for (int32_t s : ids) {
    const int old = h->h_cls[s];
    if (old > 0) {  // leaves its old class list (its old slot is not reused)
      auto& m = h->members[old];
      m.erase(std::remove(m.begin(), m.end(), s), m.end());
    }
    h->h_cls[s] = (int8_t)ncls;
    h->members[ncls].push_back(s);
  }
  for (int c = 1; c < h->st.nclass; ++c) {
    rc = sync_list(h, c, stream);
    if (rc) return rc;
  }
  return GK_OK;
}

int check_set(const gk_set* h) {
  if (!h) return fail(GK_E_ARG, "null set");
  return GK_OK;
}

bool stats_fused(const gk_set* h);

hipError_t launch_class(gk_set* h, int c, const double* x, const int64_t* offs, const int32_t* list, int64_t count,
                        int force, const GKQuery& q, hipStream_t stream, bool prio = false) {
  return gk_launch_ingest(h->st.cap[c], h->vpl, h->st, x, offs, list, count, force, h->d_ws, h->ws_bytes,
                          h->ws_blocks, h->d_ovf_count, h->d_ovf_list, q, h->d_work,
                          prio ? h->d_long_list : nullptr, prio ? h->d_long_count : nullptr,
                          prio && h->ps.ws ? h->ps.ws : nullptr, prio && h->ps.ws ? h->ps.list_ws : nullptr,
                          (prio && c == 0 && stats_fused(h)) ? h->fused_stats : 0, stream);
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

int stats_fork(gk_set* h, const double* x, const int64_t* offs, hipStream_t s) {
  if (h->timing) HIP_TRY(hipEventRecord(h->ev[2], s));
  // k_stats + k_long_prep, then the fork (k_stats_long needs only the
  // sorted list and the pre-call n), then the presort of the long streams'
  // flush batches on `s`
  HIP_TRY(gk_launch_stats(h->st, x, offs, h->d_long_list, h->d_long_n, h->d_long_count, h->ps,
                          stats_fused(h) ? 1 : 0, s));
  HIP_TRY(hipEventRecord(h->ev_fork, s));
  HIP_TRY(hipStreamWaitEvent(h->aux, h->ev_fork, 0));
  HIP_TRY(gk_launch_stats_long(h->st, x, offs, h->d_long_list, h->d_long_n, h->d_long_count, h->aux));
  HIP_TRY(hipEventRecord(h->ev_join, h->aux));
  HIP_TRY(gk_launch_presort(h->st, x, offs, h->d_long_list, h->d_long_n, h->d_long_count, h->ps, s));
  if (h->ps.ws_need) HIP_TRY(hipMemcpyAsync(h->h_ws_need, h->ps.ws_need, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  if (h->timing) HIP_TRY(hipEventRecord(h->ev[3], s));
  return GK_OK;
}

int grow_presort(gk_set* h, hipStream_t s);

int stats_join(gk_set* h, hipStream_t s, const GKQuery& q) {
  HIP_TRY(hipStreamWaitEvent(s, h->ev_join, 0));
  int rc = grow_presort(h, s);
  if (rc) return rc;
  HIP_TRY(gk_launch_query_list(h->st, h->d_long_list, h->d_long_count, q, s));
  if (h->timing) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, h->ev[2], h->ev[3]));
    h->stats_ms += ms;
  }
  return GK_OK;
}

// Launch the ingest/flush kernel over every stream (class 0 over all, each
// larger class over its member list); streams that overflow their class were
// not committed, so they are promoted one class up and run again.
// The presort workspace is sized from what the previous call needed (read
// back after the call; a call whose batches do not fit runs those streams
// unsorted -- same results, slower flushes).
int grow_presort(gk_set* h, hipStream_t s) {
  if (!h->ps.ws_need) return GK_OK;
  HIP_TRY(hipStreamSynchronize(s));  // the ingest launches synchronise anyway
  const int64_t need = *h->h_ws_need;
  if (need <= h->ps.ws_cap) return GK_OK;
  const int64_t cap = std::max<int64_t>(need + need / 8, 1 << 20);
  if (h->ps.ws) (void)hipFree(h->ps.ws);
  h->ps.ws = nullptr;
  h->ps.ws_cap = 0;
  if (hipMalloc(&h->ps.ws, (size_t)cap * sizeof(double)) != hipSuccess) {
    h->ps.ws = nullptr;  // not fatal: long streams flush unsorted
    (void)hipGetLastError();
    return GK_OK;
  }
  h->ps.ws_cap = cap;
  return GK_OK;
}

int run_ingest(gk_set* h, const double* x, const int64_t* offs, int force, hipStream_t stream,
               const GKQuery& q = GKQuery(), bool prio = false) {
  if (!offs) offs = h->d_zero_offs;
  HIP_TRY(hipMemsetAsync(h->d_ovf_count, 0, sizeof(int32_t), stream));
  // timing covers the class-0 batch launch of gk_ingest (force == 0) only
  const bool timed = h->timing && x != nullptr;
  if (timed) HIP_TRY(hipEventRecord(h->ev[0], stream));
  HIP_TRY(launch_class(h, 0, x, offs, nullptr, h->S, force, q, stream, prio && x != nullptr));
  if (timed) HIP_TRY(hipEventRecord(h->ev[1], stream));
  for (int c = 1; c < h->st.nclass; ++c)
    if (!h->members[c].empty())
      HIP_TRY(launch_class(h, c, x, offs, h->d_list[c], (int64_t)h->members[c].size(), force, q, stream));
  std::vector<int32_t> ovf;
  int64_t cnt = read_overflow(h, ovf, stream);
  if (cnt < 0) return (int)cnt;
  if (timed) {
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    h->flush_ms += ms;
    h->launches += 1;
  }
  while (!ovf.empty()) {
    // group by target class
    std::vector<int32_t> by[GK_MAX_CLASSES];
    for (int32_t s : ovf) {
      const int nc = h->h_cls[s] + 1;
      if (nc >= h->st.nclass)
        return fail(GK_E_OVERFLOW, "stream %d exceeds the largest table capacity (%d entries)", s,
                    h->st.cap[h->st.nclass - 1]);
      by[nc].push_back(s);
    }
    HIP_TRY(hipMemsetAsync(h->d_ovf_count, 0, sizeof(int32_t), stream));
    for (int c = 1; c < h->st.nclass; ++c) {
      if (by[c].empty()) continue;
      int rc = promote(h, by[c], c, stream);  // leaves by[c] in d_tmp_list
      if (rc) return rc;
      HIP_TRY(launch_class(h, c, x, offs, h->d_tmp_list, (int64_t)by[c].size(), force, q, stream));
    }
    cnt = read_overflow(h, ovf, stream);
    if (cnt < 0) return (int)cnt;
  }
  return GK_OK;
}

// Merge / explicit merge_compress at LDS capacity level 0, then the streams
// that did not fit at increasing levels (promoting their dst class as needed).
int run_merge(gk_set* dst, const MergeArgsHost& base, hipStream_t s) {
  MergeArgsHost a = base;
  a.ovf_count = dst->d_ovf_count;
  a.ovf_list = dst->d_ovf_list;
  std::vector<int32_t> todo;
  // host source of promote()'s async copies: outlives them (the next
  // read_overflow synchronises the stream), like gk_import's `by`
  std::vector<int32_t> up;
  for (int level = 0; level < dst->st.nclass; ++level) {
    const int cap = dst->st.cap[level];
    if (level > 0 && todo.empty()) break;
    if (level > 0) {
      // streams below this class are promoted so that their output may grow
      up.clear();
      for (int32_t id : todo)
        if (dst->h_cls[id] < level) up.push_back(id);
      int rc = promote(dst, up, level, s);
      if (rc) return rc;
      rc = ensure_tmp(dst, (int64_t)todo.size());
      if (rc) return rc;
      HIP_TRY(hipMemcpyAsync(dst->d_tmp_list, todo.data(), todo.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
    }
    a.dst = dst->st;
    a.cap = cap;
    a.list = level == 0 ? nullptr : dst->d_tmp_list;
    a.count = level == 0 ? dst->S : (int64_t)todo.size();
    if (cap > kMaxLdsCap) {
      int rc = ensure_ws(dst);
      if (rc) return rc;
      a.ws = dst->d_ws;
      a.ws_bytes = dst->ws_bytes;
      a.ws_blocks = dst->ws_blocks;
    } else {
      a.ws = nullptr;
      a.ws_bytes = 0;
      a.ws_blocks = 0;
    }
    HIP_TRY(hipMemsetAsync(dst->d_ovf_count, 0, sizeof(int32_t), s));
    HIP_TRY(gk_launch_merge(a, s));
    int64_t c = read_overflow(dst, todo, s);
    if (c < 0) return (int)c;
    if (c == 0) return GK_OK;
  }
  return fail(GK_E_OVERFLOW, "%zu stream(s) exceed %d table entries in merge", todo.size(),
              dst->st.cap[dst->st.nclass - 1]);
}

}  // namespace

extern "C" {

int gk_version(void) { return 100; }

const char* gk_last_error(void) { return g_err.c_str(); }

int gk_create(int64_t num_streams, double eps, int64_t cap_hint, int device, gk_set** out) {
  if (!out) return fail(GK_E_ARG, "out is null");
  *out = nullptr;
  if (num_streams < 0 || num_streams > INT32_MAX) return fail(GK_E_ARG, "num_streams out of range");
  if (std::isnan(eps) || !(eps > 0.0) || !(eps <= 1.0)) return fail(GK_E_ARG, "eps must be in (0, 1]");
  const double inv = 1.0 / eps;
  if (inv > 1023.0) return fail(GK_E_UNSUPPORTED, "eps=%g: flush period int(1/eps)+1 > 1024 is not supported", eps);
  if (cap_hint < 0 || cap_hint > kCapHuge) return fail(GK_E_UNSUPPORTED, "cap_hint %lld out of range", (long long)cap_hint);
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
  h->vpl = vpl_for(h->P);
  if (const char* fs = getenv("GK_FUSED_STATS")) h->fused_stats = std::max(0, std::min(64, atoi(fs)));
  GKState& st = h->st;
  st.S = num_streams;
  st.eps = eps;
  st.two_eps = 2.0 * eps;
  st.inv_eps = inv;
  st.P = h->P;
  st.pmax = h->P;
  // Capacity ladder.  Class 0 (every stream) is the 256-entry LDS class when
  // a flush period fits two values per lane (iid tables at eps=0.01 stay at
  // <= ~106 entries); adversarial streams are promoted to 2048
  // (LDS) and then 32768 (global workspace).
  if (h->P <= 128 && cap_hint <= kCapSmall) {
    st.nclass = 3;
    st.cap[0] = kCapSmall;
    st.cap[1] = kCapLarge;
    st.cap[2] = kCapHuge;
  } else if (cap_hint <= kCapLarge) {
    st.nclass = 2;
    st.cap[0] = kCapLarge;
    st.cap[1] = kCapHuge;
    st.cap[2] = 0;
  } else {
    st.nclass = 1;
    st.cap[0] = kCapHuge;
    st.cap[1] = st.cap[2] = 0;
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
  okm &= hipMalloc(&h->d_ovf, (S + 1) * sizeof(int32_t)) == hipSuccess;
  okm &= hipHostMalloc(&h->h_ovf, (std::min<int64_t>(S, kOvfPrefix) + 1) * sizeof(int32_t)) == hipSuccess;
  h->d_ovf_count = h->d_ovf;
  h->d_ovf_list = h->d_ovf ? h->d_ovf + 1 : nullptr;
  okm &= hipMalloc(&h->d_zero_offs, (S + 1) * sizeof(int64_t)) == hipSuccess;
  okm &= hipMalloc(&h->d_work, GK_WORK_BYTES) == hipSuccess;
  okm &= hipMalloc(&h->d_long_list, S * sizeof(int32_t)) == hipSuccess;
  okm &= hipMalloc(&h->d_long_n, S * sizeof(int64_t)) == hipSuccess;
  okm &= hipMalloc(&h->d_long_count, sizeof(int32_t)) == hipSuccess;
  okm &= hipStreamCreateWithFlags(&h->aux, hipStreamNonBlocking) == hipSuccess;
  okm &= hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) == hipSuccess;
  okm &= hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) == hipSuccess;
  if (h->P > 128) {  // class 0 is a capacity-class kernel: presort long streams' batches
    okm &= hipMalloc(&h->ps.list_ws, S * sizeof(int64_t)) == hipSuccess;
    okm &= hipMalloc(&h->ps.list_b0, (S + 1) * sizeof(int64_t)) == hipSuccess;
    okm &= hipMalloc(&h->ps.ws_need, sizeof(int64_t)) == hipSuccess;
    okm &= hipHostMalloc(&h->h_ws_need, sizeof(int64_t)) == hipSuccess;
    if (h->h_ws_need) *h->h_ws_need = 0;
  }
  if (!okm) {
    gk_destroy(h);
    return fail(GK_E_NOMEM, "device allocation for %lld streams failed", (long long)num_streams);
  }
  h->h_cls.assign((size_t)S, 0);
  if (st.cap[0] > kMaxLdsCap && ensure_ws(h) != GK_OK) {
    gk_destroy(h);
    return GK_E_NOMEM;
  }
  if (hipMemset(st.cls, 0, S * sizeof(int32_t)) != hipSuccess ||
      hipMemset(h->d_zero_offs, 0, (S + 1) * sizeof(int64_t)) != hipSuccess ||
      hipMemset(st.slot, 0, S * sizeof(int32_t)) != hipSuccess || gk_launch_reset(st, nullptr) != hipSuccess ||
      gk_launch_rtab(st, nullptr) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    gk_destroy(h);
    return fail(GK_E_HIP, "state initialisation failed");
  }
  for (auto& e : h->ev) (void)hipEventCreate(&e);
  *out = h;
  return GK_OK;
}

int gk_destroy(gk_set* h) {
  if (!h) return GK_OK;
  if (h->aux) (void)hipStreamSynchronize(h->aux);  // k_stats_long may still read the set
  GKState& st = h->st;
  void* ptrs[] = {st.n,       st.E,           st.pend,          st.mn,          st.mx,         st.sum,
                  st.avg,     st.cls,         st.slot,          st.tab[0],      st.tab[1],     st.tab[2],
                  st.pbuf,    h->d_list[0],   h->d_list[1],     h->d_list[2],   h->d_qs,       h->d_ovf,
                  h->d_tmp_list, h->d_tmp_slots, h->d_ws, h->d_zero_offs, h->d_work,
                  h->d_long_list, h->d_long_n, h->d_long_count, h->ps.list_ws, h->ps.list_b0, h->ps.ws,
                  h->ps.ws_need, st.rtab, st.n0};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
  if (h->aux) (void)hipStreamDestroy(h->aux);
  if (h->h_ws_need) (void)hipHostFree(h->h_ws_need);
  if (h->h_ovf) (void)hipHostFree(h->h_ovf);
  delete h;
  return GK_OK;
}

int gk_reset(gk_set* h, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const int64_t S = std::max<int64_t>(h->S, 1);
  HIP_TRY(hipMemsetAsync(h->st.cls, 0, S * sizeof(int32_t), s));
  HIP_TRY(hipMemsetAsync(h->st.slot, 0, S * sizeof(int32_t), s));
  HIP_TRY(gk_launch_reset(h->st, s));
  for (int c = 0; c < GK_MAX_CLASSES; ++c) {
    h->members[c].clear();
    h->slots_used[c] = 0;
  }
  std::fill(h->h_cls.begin(), h->h_cls.end(), 0);
  return GK_OK;
}

int gk_ingest(gk_set* h, const double* values, const int64_t* offsets, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!offsets) return fail(GK_E_ARG, "offsets is null");
  if (!values) return fail(GK_E_ARG, "values is null");
  if (h->S == 0) return GK_OK;
  hipStream_t s = (hipStream_t)stream;
  rc = stats_fork(h, values, offsets, s);
  if (rc) return rc;
  rc = run_ingest(h, values, offsets, 0, s, GKQuery(), true);
  const int rj = stats_join(h, s, GKQuery());  // joined on every path
  return rc ? rc : rj;
}

int gk_flush(gk_set* h, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (h->S == 0) return GK_OK;
  return run_ingest(h, nullptr, nullptr, 1, (hipStream_t)stream);
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
  if (nq > h->qs_alloc) {
    if (h->d_qs) (void)hipFree(h->d_qs);
    h->d_qs = nullptr;
    const int cap = std::max(nq, 64);
    if (hipMalloc(&h->d_qs, cap * sizeof(double)) != hipSuccess) return fail(GK_E_NOMEM, "qs allocation failed");
    h->qs_alloc = cap;
  }
  if (nq) HIP_TRY(hipMemcpyAsync(h->d_qs, qs, nq * sizeof(double), hipMemcpyHostToDevice, s));
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
  GKQuery q;
  rc = prepare_query(h, qs, nq, out, mode, s, &q);
  if (rc) return rc;
  if (nq == 0 || h->S == 0) return GK_OK;
  // gk:197-198: pending values are flushed first (state mutation); the
  // quantiles are answered in the same launch from the flushed table
  rc = run_ingest(h, nullptr, nullptr, 1, s, q);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s));
  return GK_OK;
}

int gk_ingest_quantiles(gk_set* h, const double* values, const int64_t* offsets, const double* qs, int nq,
                        double* out, int mode, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!offsets) return fail(GK_E_ARG, "offsets is null");
  if (!values) return fail(GK_E_ARG, "values is null");
  hipStream_t s = (hipStream_t)stream;
  GKQuery q;
  rc = prepare_query(h, qs, nq, out, mode, s, &q);
  if (rc) return rc;
  if (h->S == 0) return GK_OK;
  if (nq == 0) return gk_ingest(h, values, offsets, stream);
  rc = stats_fork(h, values, offsets, s);
  if (rc) return rc;
  // add every value (gk:49-61), then quantiles() (gk:187-232): flush the
  // leftover pending values and answer from the LDS-resident table
  rc = run_ingest(h, values, offsets, 1, s, q, true);
  const int rj = stats_join(h, s, q);  // joined on every path
  if (rc) return rc;
  if (rj) return rj;
  HIP_TRY(hipStreamSynchronize(s));
  return GK_OK;
}

int gk_stats(gk_set* h, int64_t* n, double* mn, double* mx, double* sum, double* avg, int32_t* table_size,
             int32_t* pending, void* stream) {
  int rc = check_set(h);
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

int gk_merge(gk_set* dst, gk_set* const* srcs, int nsrcs, void* stream) {
  int rc = check_set(dst);
  if (rc) return rc;
  if (nsrcs < 0 || (nsrcs > 0 && !srcs)) return fail(GK_E_ARG, "bad source list");
  for (int k = 0; k < nsrcs; ++k) {
    if (!srcs[k]) return fail(GK_E_ARG, "null source %d", k);
    if (srcs[k] == dst) return fail(GK_E_ARG, "a set cannot be merged into itself");
    if (srcs[k]->eps != dst->eps)  // gk:118-119
      return fail(GK_E_EPS_MISMATCH, "Cannot merge two GKArrays with different epsilon values");
    if (srcs[k]->S != dst->S)
      return fail(GK_E_ARG, "stream counts differ (%lld vs %lld)", (long long)srcs[k]->S, (long long)dst->S);
  }
  hipStream_t s = (hipStream_t)stream;
  for (int k = 0; k < nsrcs; ++k) {
    gk_set* src = srcs[k];
    // other.merge_compress() -- unconditional in the reference (gk:126, 137)
    rc = run_ingest(src, nullptr, nullptr, 2, s);
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
  if (!sizes) return fail(GK_E_ARG, "sizes is null");
  if (h->S)
    HIP_TRY(hipMemcpyAsync(sizes, h->st.E, h->S * sizeof(int32_t), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return GK_OK;
}

int gk_export(gk_set* h, const int64_t* offs, double* v, int32_t* g, int32_t* d, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!offs) return fail(GK_E_ARG, "offs is null");
  HIP_TRY(gk_launch_export(h->st, offs, v, g, d, (hipStream_t)stream));
  return GK_OK;
}

int gk_export_pending_sizes(gk_set* h, int32_t* sizes, void* stream) {
  int rc = check_set(h);
  if (rc) return rc;
  if (!sizes) return fail(GK_E_ARG, "sizes is null");
  if (h->S)
    HIP_TRY(hipMemcpyAsync(sizes, h->st.pend, h->S * sizeof(int32_t), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return GK_OK;
}

int gk_export_pending(gk_set* h, const int64_t* poffs, double* pv, void* stream) {
  int rc = check_set(h);
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
  HIP_TRY(hipMemcpyAsync(h->st.n, n, S * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemcpyAsync(h->st.mn, mn, S * sizeof(double), hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemcpyAsync(h->st.mx, mx, S * sizeof(double), hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemcpyAsync(h->st.sum, sum, S * sizeof(double), hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemcpyAsync(h->st.avg, avg, S * sizeof(double), hipMemcpyDeviceToDevice, s));
  std::vector<int32_t> ovf;
  std::vector<int32_t> by[GK_MAX_CLASSES];  // outlives the copies promote() enqueues from it
  for (int round = 0; round <= h->st.nclass; ++round) {
    HIP_TRY(hipMemsetAsync(h->d_ovf_count, 0, sizeof(int32_t), s));
    HIP_TRY(gk_launch_import(h->st, offs, v, g, d, poffs, pv, h->d_ovf_count, h->d_ovf_list, s));
    int64_t c = read_overflow(h, ovf, s);
    if (c < 0) return (int)c;
    if (c == 0) return GK_OK;
    for (auto& b : by) b.clear();
    for (int32_t id : ovf) {
      const int nc = h->h_cls[id] + 1;
      if (nc >= h->st.nclass)
        return fail(GK_E_OVERFLOW, "imported table of stream %d exceeds %d entries", id, h->st.cap[h->st.nclass - 1]);
      by[nc].push_back(id);
    }
    for (int c2 = 1; c2 < h->st.nclass; ++c2) {
      rc = promote(h, by[c2], c2, s);
      if (rc) return rc;
    }
  }
  return fail(GK_E_OVERFLOW, "import did not converge");
}

int64_t gk_num_streams(const gk_set* h) { return h ? h->S : -1; }
double gk_eps(const gk_set* h) { return h ? h->eps : 0.0; }
int gk_flush_period(const gk_set* h) { return h ? h->P : -1; }
int gk_capacity(const gk_set* h, int cls) {
  return (h && cls >= 0 && cls < h->st.nclass) ? h->st.cap[cls] : -1;
}
int64_t gk_num_promoted(const gk_set* h) {
  if (!h) return -1;
  int64_t n = 0;
  for (int c = 1; c < GK_MAX_CLASSES; ++c) n += (int64_t)h->members[c].size();
  return n;
}

int gk_timing_enable(gk_set* h, int on) {
  int rc = check_set(h);
  if (rc) return rc;
  h->timing = on != 0;
  return GK_OK;
}

int gk_timing_read(gk_set* h, double* flush_ms, double* stats_ms, int64_t* launches) {
  int rc = check_set(h);
  if (rc) return rc;
  if (flush_ms) *flush_ms = h->flush_ms;
  if (stats_ms) *stats_ms = h->stats_ms;
  if (launches) *launches = h->launches;
  h->flush_ms = h->stats_ms = 0;
  h->launches = 0;
  return GK_OK;
}

}  // extern "C"
