// gk_kernels.hip -- CDNA4 (gfx950) kernels of the batched GKArray engine.
//
// Reference: githomin/sketches-py gkarray/gkarray.py ("gk:N" = line N).
// Every kernel reproduces the reference's integer decisions and float64
// comparisons exactly ("Bit-exactness").  Built with
// -ffp-contract=off: no FMA contraction of the reference's float64 formulas.
//
// Kernels
//   k_stats_short / k_stats_long / stats role  gk:52-59   lane per stream: n/_sum/_avg sequential chain, min/max
//   k_ingest     gk:60-109  wave per stream: flush schedule + closed-form
//                           merge_compress of each flush, table kept in LDS
//                           for the whole call
//                           + optional fused quantiles (gk:156-232) answered
//                           from the LDS table after the final flush: rank walk
//                           as a count over the running max of prefix(g)+delta
//   k_merge      gk:111-154 wave per stream: convert `other`, stable merge of
//                           the incoming list, general four-rule walk (gk:76-106)
//   k_export / k_import / k_reset: state movement
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <math.h>

#include <algorithm>
#include <atomic>
#include <limits>
#include <type_traits>

#include "gk_state.h"
#include "gk_launch.h"
#include "gk_xor.h"

#define GK_PROF_NSEC 12
#ifndef GK_PROF_FIRST
#define GK_PROF_FIRST 1  // k_ingest_small: a wave's first stream's loop tops in section 11
#endif
#ifdef GK_PROF
__device__ unsigned long long gk_prof_acc[GK_PROF_NSEC];
__device__ __forceinline__ uint32_t gk_cycles() { return (uint32_t)__builtin_amdgcn_s_memtime(); }
#define GK_MARK(L, sec)                                      \
  do {                                                       \
    if (threadIdx.x == 0) {                                  \
      const uint32_t t_ = gk_cycles();                       \
      (L).prof[sec] += (uint32_t)(t_ - (L).prof_t);         \
      (L).prof_t = t_;                                       \
    }                                                        \
  } while (0)
#else
#define GK_MARK(L, sec) do { } while (0)
#endif
// capacity-class kernels (k_ingest<CAP>): one LDS accumulator set per block,
// marked by lane 0 (GK_BMARK), summed into gk_prof_acc at the end
#ifdef GK_PROF
struct GKBigProf {
  unsigned long long acc[GK_PROF_NSEC];
  uint32_t t;
};
__device__ __forceinline__ GKBigProf& gk_big_prof() {
  __shared__ GKBigProf p;
  return p;
}
#define GK_BMARK(sec)                                        \
  do {                                                       \
    if (threadIdx.x == 0) {                                  \
      GKBigProf& p_ = gk_big_prof();                         \
      const uint32_t t_ = gk_cycles();                       \
      p_.acc[sec] += (uint32_t)(t_ - p_.t);                  \
      p_.t = t_;                                             \
    }                                                        \
  } while (0)
// k_ingest_wg, per wave (profiling builds): every wave's lane 0 adds the
// cycles since its previous mark to [wave][point], so that each stretch of a
// flush is split into its work and its barrier wait, wave by wave
// (tools/prof_sections.py --workload wg --per-wave)
#define GK_WP_N 16
#define GK_WP_W 8
__device__ unsigned long long gk_wprof_acc[GK_WP_W][GK_WP_N];
struct GKWaveProf {
  unsigned long long acc[GK_WP_W][GK_WP_N];
  uint32_t t[GK_WP_W];
};
__device__ __forceinline__ GKWaveProf& gk_wave_prof() {
  __shared__ GKWaveProf p;
  return p;
}
#define GK_WMARK(pt)                                                   \
  do {                                                                 \
    if ((threadIdx.x & 63) == 0 && (threadIdx.x >> 6) < GK_WP_W) {     \
      GKWaveProf& p_ = gk_wave_prof();                                 \
      const int w_ = threadIdx.x >> 6;                                 \
      const uint32_t t_ = gk_cycles();                                 \
      p_.acc[w_][pt] += (uint32_t)(t_ - p_.t[w_]);                     \
      p_.t[w_] = t_;                                                   \
    }                                                                  \
  } while (0)
#else
#define GK_BMARK(sec) do { } while (0)
#define GK_WMARK(pt) do { } while (0)
#endif

// quantile answers that are the stream's _min / _max while the stats role of
// the launch may still be writing them (the join, k_query_list, replaces them)
#define GK_QMARK_MIN 0x7ff4000000000001LL  // quantile = _min of the stream (gk:182-183, 220)
#define GK_QMARK_MAX 0x7ff4000000000002LL  // quantile = _max of the stream (gk:229)
#define GK_KEEP_BIT 0x40000000

// Largest T handled in int32 fields: T = floor(2 eps (n-1)) <= 2^30, i.e.
// n <= 2^29/eps values in ONE stream (5.4e10 at eps = 0.01).  No result is
// ever computed with a clamped T: the ingest kernels check the stream's count
// after the call first (gk_count_ok) and refuse a stream that would pass it
// (overflow -> promotion -> the unbounded class reports it, GK_E_OVERFLOW).
#define GK_T_CLAMP (1 << 30)

// T of every flush up to count `n_final` fits GK_T_CLAMP
__device__ __forceinline__ bool gk_count_ok(const GKState& st, int64_t n_final) {
  return st.two_eps * (double)(n_final - 1) < (double)GK_T_CLAMP + 1.0;
}

__device__ __forceinline__ int gk_threshold(const GKState& st, int64_t n) {
  // np.floor(2.0*self.eps*(self._n - 1))  (gk:70): (2.0*eps) * float(n-1)
  double t = floor(st.two_eps * (double)(n - 1));
  if (t > (double)GK_T_CLAMP) t = (double)GK_T_CLAMP;
  if (t < -1.0) t = -1.0;
  return (int)t;
}

__device__ __forceinline__ int clampi(int x, int lo, int hi) { return x < lo ? lo : (x > hi ? hi : x); }

// clamp(x, 0, m) for m >= 0 in one VALU op (the median of x, 0, m)
__device__ __forceinline__ int clamp0(int x, int m) {
  int r;
  asm("v_med3_i32 %0, %1, 0, %2" : "=v"(r) : "v"(x), "v"(m));
  return r;
}

// ---------------------------------------------------------------------------
// wave helpers (wave64)
// ---------------------------------------------------------------------------
// DPP controls (GFX9 family, gfx950 included)
#define DPP_ROW_SHR(n) (0x110 + (n))
#define DPP_WAVE_SHR1 0x138
#define DPP_WAVE_SHL1 0x130
#define DPP_ROW_BCAST15 0x142
#define DPP_ROW_BCAST31 0x143

// Inclusive wave64 prefix sum in 12 VALU ops: Hillis-Steele inside each row
// of 16 lanes, then the row_bcast15/31 carries across rows.  Lanes whose DPP
// source is outside the row (or rows masked off) receive 0.
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, int /*lane*/) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_SHR(1), 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_SHR(2), 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_SHR(4), 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_SHR(8), 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_BCAST15, 0xa, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_BCAST31, 0xc, 0xf, false);
  return v;
}

// inclusive wave64 running max of int32 (lanes without a DPP source take INT_MIN)
__device__ __forceinline__ int32_t wave_incl_max_i32(int32_t v) {
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, DPP_ROW_SHR(1), 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, DPP_ROW_SHR(2), 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, DPP_ROW_SHR(4), 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, DPP_ROW_SHR(8), 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, DPP_ROW_BCAST15, 0xa, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, DPP_ROW_BCAST31, 0xc, 0xf, false));
  return v;
}

// value of lane-1 (lane 0 gets `fill`)
__device__ __forceinline__ int wave_shr1(int v, int fill) {
  return __builtin_amdgcn_update_dpp(fill, v, DPP_WAVE_SHR1, 0xf, 0xf, false);
}

// 64-bit DPP move: both halves through the same control; lanes whose
// source is masked off or outside the row receive `old`
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int64_t dpp64(int64_t v, int64_t old) {
  const int lo = __builtin_amdgcn_update_dpp((int)(uint32_t)(uint64_t)old, (int)(uint32_t)(uint64_t)v, CTRL,
                                             ROWMASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(uint32_t)((uint64_t)old >> 32),
                                             (int)(uint32_t)((uint64_t)v >> 32), CTRL, ROWMASK, 0xf, false);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// inclusive wave64 prefix sum / running max of int64 on DPP (no LDS-pipe
// instruction: the flush's table traffic bounds the LDS)
__device__ __forceinline__ int64_t wave_incl_scan_i64(int64_t v, int /*lane*/) {
  v += dpp64<DPP_ROW_SHR(1), 0xf>(v, 0);
  v += dpp64<DPP_ROW_SHR(2), 0xf>(v, 0);
  v += dpp64<DPP_ROW_SHR(4), 0xf>(v, 0);
  v += dpp64<DPP_ROW_SHR(8), 0xf>(v, 0);
  v += dpp64<DPP_ROW_BCAST15, 0xa>(v, 0);
  v += dpp64<DPP_ROW_BCAST31, 0xc>(v, 0);
  return v;
}

__device__ __forceinline__ int64_t wave_incl_max_i64(int64_t v, int /*lane*/) {
  v = max(v, dpp64<DPP_ROW_SHR(1), 0xf>(v, INT64_MIN));
  v = max(v, dpp64<DPP_ROW_SHR(2), 0xf>(v, INT64_MIN));
  v = max(v, dpp64<DPP_ROW_SHR(4), 0xf>(v, INT64_MIN));
  v = max(v, dpp64<DPP_ROW_SHR(8), 0xf>(v, INT64_MIN));
  v = max(v, dpp64<DPP_ROW_BCAST15, 0xa>(v, INT64_MIN));
  v = max(v, dpp64<DPP_ROW_BCAST31, 0xc>(v, INT64_MIN));
  return v;
}

// the value of lane-1 (lane 0: fill)
__device__ __forceinline__ int64_t wave_shr1_i64(int64_t v, int64_t fill) { return dpp64<DPP_WAVE_SHR1, 0xf>(v, fill); }

__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Ordering point for a ONE-WAVE workgroup.  The LDS executes a wave's
// instructions in issue order, so a ds_write is visible to every later
// ds_read of the same wave; only the compiler must not move LDS accesses
// across this point.  Unlike __syncthreads() it does not wait for vmcnt, so
// global-memory prefetches stay in flight.  The global-workspace variant
// (GLOBAL = true) needs the memory counters drained and keeps __syncthreads.
template <bool GLOBAL>
__device__ __forceinline__ void wsync() {
  if constexpr (GLOBAL) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}


// ---------------------------------------------------------------------------
// Loads of flush values.  All loads are ordinary (compiler-visible): the
// compiler then places the vmcnt wait at the first use.  The prefetch of the
// next flush is issued after the gap search of the current one, so its first
// use -- the select at the end of the flush -- lands after the flush's LDS
// work.  (Inline-asm loads were tried and rejected: the compiler may copy an
// asm output register before the load lands; tools/check_async_loads.py.)
// ---------------------------------------------------------------------------
// A flush's values: the first p come from the stream's pending buffer, the
// rest from the batch.
template <int VPL>
__device__ __forceinline__ void gk_load_flush_values(double (&xv)[VPL], const double* pb, int p,
                                                     const double* xs, int cnt, int lane) {
  if (cnt <= 0) {
#pragma unroll
    for (int r = 0; r < VPL; ++r) xv[r] = 0.0;
    return;
  }
#pragma unroll
  for (int r = 0; r < VPL; ++r) {
    const int ic = min(lane + 64 * r, cnt - 1);
    const double* a = (ic < p) ? pb + ic : xs + (ic - p);
    xv[r] = *a;
  }
#pragma unroll
  for (int r = 0; r < VPL; ++r) xv[r] = (lane + 64 * r < cnt) ? xv[r] : 0.0;
}

// Per-stream header, loaded for the NEXT stream while the current one is
// processed (uniform addresses: one request each).
struct GKHdrV {
  int32_t cls, slot, pend, E;
  int64_t n, xo, xe;
  double mn, mx;
};

template <bool MINMAX = true>
__device__ __forceinline__ void gk_hdr_issue(GKHdrV& h, const GKState& st, const int64_t* offs, int64_t s) {
  h.cls = st.cls[s];
  h.slot = st.slot[s];
  h.pend = st.pend[s];
  h.E = st.E[s];
  h.n = st.n[s];
  h.xo = offs[s];
  h.xe = offs[s + 1];
  if constexpr (MINMAX) {
    h.mn = st.mn[s];
    h.mx = st.mx[s];
  } else {
    h.mn = h.mx = 0.0;
  }
}

// The same header spread over the lanes of ONE register (lane k loads word
// k: 0 cls, 1 slot, 2 pend, 3 E, 4-5 n, 6-7 xo, 8-9 xe, 10-11 mn, 12-13 mx)
// for k_ingest_small, where the prefetch stays live across the whole stream:
// one VGPR instead of 10-14.  Read back with gk_hdr1_word/_dword.
template <bool MINMAX>
__device__ __forceinline__ uint32_t gk_hdr1_issue(const GKState& st, const int64_t* offs, int64_t s, int lane) {
  constexpr int NW = MINMAX ? 14 : 10;
  const uint32_t* p = (const uint32_t*)(st.cls + s);
  if (lane == 1) p = (const uint32_t*)(st.slot + s);
  if (lane == 2) p = (const uint32_t*)(st.pend + s);
  if (lane == 3) p = (const uint32_t*)(st.E + s);
  if (lane >= 4) p = (const uint32_t*)(st.n + s) + (lane - 4);
  if (lane >= 6) p = (const uint32_t*)(offs + s) + (lane - 6);  // xo, then xe (offs[s + 1])
  if constexpr (MINMAX) {
    if (lane >= 10) p = (const uint32_t*)(st.mn + s) + (lane - 10);
    if (lane >= 12) p = (const uint32_t*)(st.mx + s) + (lane - 12);
  }
  uint32_t w = 0;
  if (lane < NW) w = *p;
  return w;
}
__device__ __forceinline__ int32_t gk_hdr1_word(uint32_t w, int k) { return __builtin_amdgcn_readlane((int)w, k); }
__device__ __forceinline__ int64_t gk_hdr1_dword(uint32_t w, int k) {
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)w, k + 1) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)w, k));
}

__device__ __forceinline__ int64_t rfl64(int64_t v) {
  const int lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)v);
  const int hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ GKRec* gk_table_ptr_cs(const GKState& st, int64_t s, int32_t c, int32_t slot) {
  return c == 0 ? st.tab[0] + s * (int64_t)st.cap[0] : st.tab[c] + (int64_t)slot * st.cap[c];
}

// Streams up to GK_STATS_LONG values have their gk:52-59 chains walked by the
// stats role of the small-class launch (P <= 128) or by k_stats_short;
// longer ones by k_stats_long (or on host cores), beside the ingest.
#ifndef GK_STATS_LONG
#define GK_STATS_LONG 16384  // longer streams go to k_stats_long (64 per wave, on a second HIP stream)
#endif

// The long-stream list (streams past GK_STATS_LONG values, for k_long_prep /
// k_stats_long) and the pre-call n snapshot st.n0 (read by the small-class
// launch's stats role while its ingest waves rewrite st.n): one stream per
// thread, no LDS (~6 us per 10^6 streams; as part of the former k_stats, whose 35 KiB
// chain tile holds it to 4 blocks per CU, it took 28 us).
#ifdef GK_TIMELINE
// timeline builds only: s_memrealtime when the call's first kernel starts
// (k_lengths) and when its join answers (k_query_list)
__device__ unsigned long long gk_tl_call[2];
#endif
__global__ __launch_bounds__(256) void k_lengths(GKState st, const int64_t* __restrict__ offs,
                                                 int32_t* __restrict__ long_list, int32_t* __restrict__ long_count) {
#ifdef GK_TIMELINE
  if (blockIdx.x == 0 && threadIdx.x == 0) gk_tl_call[0] = __builtin_amdgcn_s_memrealtime();
#endif
  const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (s >= st.S) return;
  st.n0[s] = st.n[s];
  if (offs[s + 1] - offs[s] > GK_STATS_LONG) long_list[atomicAdd(long_count, 1)] = (int32_t)s;
}

// ===========================================================================
// k_long_prep: the long-stream list k_lengths built (in atomic order) sorted by
// length, longest first (ties: lower stream id first), so that k_ingest and
// k_stats_long start the longest sequential chains first; and the pre-call n
// of every listed stream saved for k_stats_long, which runs beside k_ingest
// (k_ingest rewrites n).  One 1024-thread block, bitonic sort of 64-bit keys
// in LDS; lists longer than GK_SORT_LONG_MAX keep their arrival order (still
// correct, only less balanced).  Runs before k_ingest on the same HIP stream.
// ===========================================================================
#define GK_SORT_LONG_MAX 4096
// k_ingest_wg (below): at most this many streams per call, each with at least
// GK_WG_MIN_FLUSHES presorted flushes
#ifndef GK_WG_MAX
#define GK_WG_MAX 64
#endif
#ifndef GK_WG_MIN_FLUSHES
#define GK_WG_MIN_FLUSHES 256
#endif
#define GK_WG_CAP 2048
#define GK_WG_PMAX 1024
#ifndef GK_PRESORT_REL
#define GK_PRESORT_REL 3  // presort streams with >= 1/GK_PRESORT_REL of the longest one's flushes
#endif
// ... and with k_ingest_wg on (the longest streams walk ~3x faster there), the
// one-wave path's critical length shrinks: presort down to 1/GK_PRESORT_REL_WG
#ifndef GK_PRESORT_REL_WG
#define GK_PRESORT_REL_WG 5
#endif

__global__ __launch_bounds__(1024) void k_long_prep(GKState st, const int64_t* __restrict__ offs,
                                                    int32_t* __restrict__ list, int64_t* __restrict__ list_n,
                                                    const int32_t* __restrict__ count,
                                                    int64_t* __restrict__ list_ws, int64_t* __restrict__ list_b0,
                                                    int64_t ws_cap, int64_t* __restrict__ ws_need,
                                                    int32_t* __restrict__ wg_count, int wg_presort,
                                                    int32_t* __restrict__ go) {
  __shared__ uint64_t key[GK_SORT_LONG_MAX];
  const int cnt = *count;
  const int t = threadIdx.x;
  if (cnt > 1 && cnt <= GK_SORT_LONG_MAX) {
    int N = 2;
    while (N < cnt) N <<= 1;
    constexpr uint64_t LMAX = (1ull << 33) - 1;
    for (int i = t; i < N; i += 1024) {
      uint64_t k = ~0ull;
      if (i < cnt) {
        const int64_t s = list[i];
        uint64_t L = (uint64_t)(offs[s + 1] - offs[s]);
        if (L > LMAX) L = LMAX;
        // ascending key = descending length, then ascending stream id
        k = ((LMAX - L) << 31) | (uint64_t)s;
      }
      key[i] = k;
    }
    __syncthreads();
    for (int k = 2; k <= N; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int pp = t; pp < N / 2; pp += 1024) {
          const int i = ((pp & ~(j - 1)) << 1) | (pp & (j - 1));
          const int l = i + j;
          const uint64_t a = key[i], b = key[l];
          if ((a > b) == ((i & k) == 0)) {
            key[i] = b;
            key[l] = a;
          }
        }
        __syncthreads();
      }
    }
    for (int i = t; i < cnt; i += 1024) list[i] = (int32_t)(key[i] & 0x7fffffffu);
    __syncthreads();
  }
  // (the pre-call n from k_lengths' snapshot: with the stats role fused, this
  // kernel runs beside the ingest launch, which rewrites st.n)
  for (int i = t; i < cnt; i += 1024) list_n[i] = st.n0[list[i]];
  if (!list_ws) return;
  __syncthreads();
  // Presort plan (k_presort): every automatic flush of a listed class-0
  // stream in this call gets a slot of P doubles in the workspace; list_ws[i]
  // = first slot offset (in doubles) or -1 (not presorted: the workspace is
  // too small -- the host grows it from *ws_need after the call), list_b0[i]
  // = the stream's first global batch index (for k_presort's block mapping).
  // Only streams within a factor GK_PRESORT_REL of the longest one's flush
  // count are presorted: they alone can be the call's critical path (an
  // unsorted flush costs ~2-3x a presorted one), and sorting every listed
  // stream's batches cost cfg5 ~17 ms ahead of the ingest.
  __shared__ int64_t part[1024];
  __shared__ unsigned long long nbmax;
  if (t == 0) nbmax = 0;
  __syncthreads();
  const int per = (cnt + 1023) / 1024;
  const int i0 = t * per, i1 = min(i0 + per, cnt);
  for (int i = i0; i < i1; ++i) {
    const int64_t s = list[i];
    int64_t nb = 0;
    if (st.cls[s] == 0) {
      const int64_t L = offs[s + 1] - offs[s];
      const int64_t need = st.P - (list_n[i] % st.P);
      nb = L >= need ? 1 + (L - need) / st.P : 0;
    }
    list_b0[i] = nb;  // count for now
    atomicMax(&nbmax, (unsigned long long)nb);
  }
  __syncthreads();
  // k_ingest_wg takes the head of the list (longest first): every stream with
  // at least GK_WG_MIN_FLUSHES flushes, at most GK_WG_MAX of them.  Only its
  // streams are presorted then (GK_WG_PRESORT=0: none; k_ingest_wg ranks
  // unsorted batches itself), so that the one-wave launch, whose streams are
  // short enough to flush unsorted, need not wait for the presort
  __shared__ int wk;
  if (wg_count) {
    if (t == 0) {
      int k = 0;
      while (k < cnt && k < GK_WG_MAX && list_b0[k] >= GK_WG_MIN_FLUSHES) ++k;
      if (!(st.cap[0] == GK_WG_CAP && st.P <= GK_WG_PMAX)) k = 0;
      *wg_count = k;
      wk = wg_presort ? k : 0;
    }
    __syncthreads();
  }
  const int64_t nb_min = (int64_t)(nbmax / (wg_count ? GK_PRESORT_REL_WG : GK_PRESORT_REL));
  int64_t mine = 0;
  for (int i = i0; i < i1; ++i) {
    // flushed unsorted (with k_ingest_wg: all but its streams)
    if (list_b0[i] < nb_min || (wg_count && i >= wk)) list_b0[i] = 0;
    mine += list_b0[i];
  }
  part[t] = mine;
  __syncthreads();
  if (t == 0) {
    int64_t acc = 0;
    for (int k = 0; k < 1024; ++k) {
      const int64_t v = part[k];
      part[k] = acc;
      acc += v;
    }
    *ws_need = acc * st.P;
    list_b0[cnt] = acc;  // total batches (k_presort's grid bound)
  }
  __syncthreads();
  int64_t b = part[t];
  for (int i = i0; i < i1; ++i) {
    const int64_t nb = list_b0[i];
    list_b0[i] = b;
    list_ws[i] = (nb > 0 && (b + nb) * st.P <= ws_cap) ? b * st.P : -1;
    b += nb;
  }
  // k_ingest_wg, launched ahead of this kernel (its workgroups hold their CUs
  // before the chain walks and the presort fill the chip), waits for this
  // word: every write above released first
  if (go) {
    __syncthreads();
    if (t == 0) {
      __threadfence();
      __hip_atomic_store(go, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ===========================================================================
// k_presort: the batch of every automatic flush of a listed long stream
// (list_ws >= 0), sorted by (value, insertion index) -- Python's stable
// sorted() of gk:71-72 -- into its workspace slot, ahead of k_ingest, so that
// the flush (sequential per stream, on the critical path of long streams)
// skips its in-gap ranking.  Batch 0 is the pre-call pending values followed
// by the first `need` values; batch b > 0 is the next P values.  One
// 256-thread block per batch (global batch id -> stream by binary search over
// list_b0), bitonic sort of up to 1024 keys in LDS.
// ===========================================================================
__global__ __launch_bounds__(256) void k_presort(GKState st, const double* __restrict__ x,
                                                 const int64_t* __restrict__ offs,
                                                 const int32_t* __restrict__ list, const int32_t* __restrict__ count,
                                                 const int64_t* __restrict__ list_n,
                                                 const int64_t* __restrict__ list_ws,
                                                 const int64_t* __restrict__ list_b0, double* __restrict__ ws) {
  __shared__ double kv[1024];
  __shared__ uint32_t ki[1024];
  const int cnt = *count;
  if (cnt <= 0) return;
  const int64_t total = list_b0[cnt];
  const int t = threadIdx.x;
  const int P = st.P;
  // a contiguous range of global batches per block: one binary search for
  // its first stream slot, then the slot advances along the (ascending)
  // list_b0 -- a search per batch was ~10 dependent global loads
  const int64_t g0 = total * blockIdx.x / gridDim.x, g1 = total * (blockIdx.x + 1) / gridDim.x;
  if (g0 >= g1) return;
  int i = 0;
  {
    int lo = 0, hi = cnt - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (list_b0[mid] <= g0) lo = mid;
      else hi = mid - 1;
    }
    i = lo;
  }
  int64_t bnext = i + 1 < cnt ? list_b0[i + 1] : INT64_MAX;  // first global batch of slot i + 1
  int ci = -1;  // the slot whose parameters are loaded
  int64_t wso = -1, b0 = 0, s = 0, xo = 0, need = 0;
  int p = 0;
  for (int64_t gb = g0; gb < g1; ++gb) {
    while (gb >= bnext) {  // (slots without batches are passed over)
      ++i;
      bnext = i + 1 < cnt ? list_b0[i + 1] : INT64_MAX;
    }
    if (i != ci) {
      ci = i;
      wso = list_ws[i];
      b0 = list_b0[i];
      s = list[i];
      xo = offs[s];
      p = st.pend[s];
      need = P - (list_n[i] % P);
    }
    if (wso < 0) continue;  // block-uniform
    const int64_t b = gb - b0;
    const double* pb = st.pbuf + s * (int64_t)st.pmax;
    const int m = b == 0 ? p + (int)need : P;
    const int64_t xb = b == 0 ? xo : xo + need + (b - 1) * P;  // first x value of the batch (after pending)
    int N = 64;
    while (N < m) N <<= 1;
    for (int k = t; k < N; k += 256) {
      double v = __longlong_as_double(0x7ff0000000000000LL);
      if (k < m) v = (b == 0 && k < p) ? pb[k] : x[xb + (b == 0 ? k - p : k)];
      kv[k] = v;
      ki[k] = k < m ? (uint32_t)k : 0xffffffffu;
    }
    __syncthreads();
    for (int k = 2; k <= N; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int pp = t; pp < N / 2; pp += 256) {
          const int a = ((pp & ~(j - 1)) << 1) | (pp & (j - 1));
          const int c = a + j;
          const double va = kv[a], vc = kv[c];
          const uint32_t ia = ki[a], ic = ki[c];
          const bool a_gt = (va > vc) || (!(va < vc) && ia > ic);
          if (a_gt == ((a & k) == 0)) {
            kv[a] = vc;
            kv[c] = va;
            ki[a] = ic;
            ki[c] = ia;
          }
        }
        __syncthreads();
      }
    }
    double* out = ws + wso + b * P;
    for (int k = t; k < m; k += 256) out[k] = kv[k];
    __syncthreads();
  }
}

// streams walked one wave each by k_stats_long (more: 64 per wave); also the
// host-walked chains' limit
#ifndef GK_SL_BCAST
#define GK_SL_BCAST 1024
#endif

// ===========================================================================
// Host-walked chains.  The gk:54 `_avg` update is three dependent float64
// roundings per value: ~37 cycles per value on one gfx950 lane (15.7 ns), so
// a 10^7-value stream is a 157 ms chain however the batch is spread.  A host
// core runs the same three roundings at ~3 cycles each, so the longest
// streams' chains go to host cores (gk_capi.cpp, over pinned chunk copies)
// while the GPU ingests; k_hc_prep picks them and snapshots their pre-call
// state, k_hc_apply writes the host's results back.
// ===========================================================================
__global__ __launch_bounds__(256) void k_hc_prep(GKState st, const int64_t* __restrict__ offs,
                                                 const int32_t* __restrict__ list,
                                                 const int64_t* __restrict__ list_n,
                                                 const int32_t* __restrict__ count, int64_t min_len, int rel_pct,
                                                 int64_t budget_factor, GKHostChainRec* __restrict__ recs,
                                                 int32_t* __restrict__ hc_count) {
  __shared__ int64_t pre[GK_HC_MAX];
  __shared__ int64_t lmax;
  const int t = threadIdx.x;
  const int cnt = *count;
  // (the list is sorted longest first: k_long_prep sorts up to
  // GK_SORT_LONG_MAX >= GK_SL_BCAST entries, so eligibility is a prefix)
  const bool on = min_len > 0 && cnt > 0 && cnt <= GK_SL_BCAST;
  if (t == 0) lmax = on ? offs[(int64_t)list[0] + 1] - offs[list[0]] : 0;
  __syncthreads();
  // a chain shorter than rel_pct % of the longest finishes on the device
  // under the longest stream's flushes anyway
  const int64_t need = max(min_len, (int64_t)((double)lmax * (double)rel_pct / 100.0));
  int64_t s = 0, xo = 0, L = 0;
  if (on && t < cnt) {
    s = list[t];
    xo = offs[s];
    L = offs[s + 1] - xo;
  }
  pre[t] = (on && t < cnt && L >= need) ? L : 0;
  __syncthreads();
  // inclusive prefix sums of the eligible lengths (Hillis-Steele)
  for (int o = 1; o < GK_HC_MAX; o <<= 1) {
    const int64_t a = t >= o ? pre[t - o] : 0;
    __syncthreads();
    pre[t] += a;
    __syncthreads();
  }
  const int64_t budget = budget_factor * lmax;
  const bool take = on && t < cnt && L >= need && pre[t] <= budget;
  // a prefix: count it with a block-wide ballot of `take`
  __shared__ int32_t k;
  if (t == 0) k = 0;
  __syncthreads();
  if (take) {
    recs[t] = GKHostChainRec{s, xo, L, list_n[t], st.sum[s], st.avg[s], st.mn[s], st.mx[s]};
    atomicAdd(&k, 1);
  }
  __syncthreads();
  if (t == 0) *hc_count = k;
}

// The join of an asynchronous host walk (round 4): one thread waits until the
// set's host worker has published this call's sequence number in the pinned
// flag word ((seq << 2) | 1 done / 2 failed; gk_capi.cpp hc_worker), with a
// wall-clock bound (s_memrealtime, 100 MHz) after which the walk counts as
// failed.  `fail` tells k_hc_apply / k_hc_fallback which of them applies the
// picked streams' chains.  (Loads only: the flag is written by the host.)
__global__ void k_hc_wait(const unsigned long long* __restrict__ flag, unsigned long long seq,
                          int32_t* __restrict__ fail, unsigned long long timeout_ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int f = 1;
  for (;;) {
    const unsigned long long w = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((w >> 2) >= seq) {
      f = ((w >> 2) == seq && (w & 3) == 1) ? 0 : 1;
      break;
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) break;
    __builtin_amdgcn_s_sleep(127);
  }
  *fail = f;
}

__global__ __launch_bounds__(256) void k_hc_apply(GKState st, const GKHostChainRec* __restrict__ recs,
                                                  const int32_t* __restrict__ hc_count,
                                                  const int32_t* __restrict__ fail) {
  const int t = threadIdx.x;
  if ((fail && *fail) || t >= *hc_count) return;
  const GKHostChainRec r = recs[t];
  st.sum[r.s] = r.sum;
  st.avg[r.s] = r.avg;
  st.mn[r.s] = r.mn;
  st.mx[r.s] = r.mx;
}

// ===========================================================================
// k_stats_long: gk:52-59 for the streams k_lengths lists (longer than
// GK_STATS_LONG values).  The _avg update is three dependent float64
// roundings per value, so a long stream's time is its chain latency.  Two
// layouts, chosen on the device from the list length (the list comes sorted
// longest first from k_long_prep):
//  * up to GK_SL_BCAST streams: one wave per stream.  The 64 lanes load 64
//    consecutive values at a time (coalesced, SL_BCAST_DEPTH chunks in
//    flight) and compute 64 reciprocals 1.0/n and the first-occurrence
//    min/max in parallel; every lane walks the chain over LDS broadcast reads
//    of (v, 1/n), so the chain runs at its latency (~16 ns/value).
//  * more streams: 64 streams per wave, one per lane, each streaming its own
//    values into registers (chunks of 16 values as 8 aligned 16-byte loads,
//    SL_DEPTH chunks in flight).  A step costs ~25 VALU for 64 chains, so
//    throughput beats one wave per stream once there are more streams than
//    wave slots (10 000 streams of 10^6 values: cfg4 on one GPU).
// This kernel runs on a second HIP stream beside k_ingest, which rewrites n:
// the pre-call n of every listed stream comes from list_n.
// ===========================================================================
#define SL_BCAST_DEPTH 4
#ifndef SL_DEPTH
#define SL_DEPTH 7  // chunks in flight: 7 x 8 loads = 56 <= the 63 vmcnt can count
#endif

__device__ __forceinline__ void gk_stat_step(double v, int64_t& n, double& sm, double& av, double& mn, double& mx) {
  n += 1;                                   // gk:52
  sm = sm + v;                              // gk:53
  av = av + (v - av) * (1.0 / (double)n);   // gk:54 (no FMA: -ffp-contract=off)
  if (v < mn) mn = v;                       // gk:56-57 (strict: first occurrence kept)
  if (v > mx) mx = v;                       // gk:58-59
}


// ---------------------------------------------------------------------------
// Speculative walk of one stream's _sum/_avg chains (round 4).  The chains
// are sequential (gk:53-54: every value's update reads the previous result,
// three float64 roundings per _avg step), so one lane walks them at the
// latency of its dependent ops, ~16 ns/value.  A superstep of 64 x W values
// runs them on all 64 lanes at once instead:
//  1. lane j takes values j*W .. j*W+W-1 and starts from an ESTIMATE of the
//     chain at its first value (lane 0: the true value; lane j > 0: the
//     running mean/sum continued with a tree sum of the lanes before it);
//  2. each lane walks its W steps from its estimate (spec values X[0..W]);
//  3. the spec values are shifted onto the true chain: lane j's offset D_j
//     from a lane scan of X_{j-1}[W] - X_j[0] (lane 0: D = 0), b_t = X_t + D_j;
//  4. every step is CHECKED in parallel, bit for bit: f(b_t) == b_{t+1}
//     (lane j's b_W is lane j+1's b_0).  If every check passes, by induction
//     from the true b_0 every b_t is the sequential chain's value.  At the
//     first failing step the true value there is f(b_t): the checks restart
//     from it (only the steps after it), so each round makes progress and
//     the result is bit-exact whatever the data; usually one round suffices
//     (an offset keeps the _avg roundings unless the update crosses a
//     rounding boundary; the _sum's only at a binade change or a tie).
// tools/mb/spec_chain.c is the host prototype (rounds per superstep:
// lognormal 1.01-1.10, Pareto 1.08, signed e^+-50 3.3, all bit-exact).
// ---------------------------------------------------------------------------
#ifndef GK_SPEC_W
#define GK_SPEC_W 16
#endif
#ifndef GK_SPEC
#define GK_SPEC 1
#endif
#ifndef GK_SPEC_ROUNDS
#define GK_SPEC_ROUNDS 16
#endif
#ifndef GK_SPEC_GIVEUP
#define GK_SPEC_GIVEUP 4
#endif

// inclusive wave64 prefix sum of doubles on DPP (lanes without a source add
// +0.0); the addition order is the scan's, not a sequential one
__device__ __forceinline__ double wave_incl_scan_f64(double v) {
#define GK_SCAN_STEP(C, M) v = v + __longlong_as_double(dpp64<C, M>(__double_as_longlong(v), 0))
  GK_SCAN_STEP(DPP_ROW_SHR(1), 0xf);
  GK_SCAN_STEP(DPP_ROW_SHR(2), 0xf);
  GK_SCAN_STEP(DPP_ROW_SHR(4), 0xf);
  GK_SCAN_STEP(DPP_ROW_SHR(8), 0xf);
  GK_SCAN_STEP(DPP_ROW_BCAST15, 0xa);
  GK_SCAN_STEP(DPP_ROW_BCAST31, 0xc);
#undef GK_SCAN_STEP
  return v;
}
// the value of lane-1 / lane+1 (lane 0 / lane 63: fill)
__device__ __forceinline__ double wave_shr1_f64(double v, double fill) {
  return __longlong_as_double(dpp64<DPP_WAVE_SHR1, 0xf>(__double_as_longlong(v), __double_as_longlong(fill)));
}
__device__ __forceinline__ double wave_shl1_f64(double v, double fill) {
  return __longlong_as_double(dpp64<DPP_WAVE_SHL1, 0xf>(__double_as_longlong(v), __double_as_longlong(fill)));
}

__device__ __forceinline__ double rdlane_f64(double v, int l) {
  const int64_t b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double((int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

// KIND 0: _avg (b + (v - b) * r), 1: _sum (b + v).  X: this lane's spec
// values, K: the true value before the superstep.  Returns the true value
// after it (wave-uniform), or ok = false after GK_SPEC_ROUNDS rounds.
template <int KIND, int W>
__device__ __forceinline__ double spec_verify(const double (&X)[W + 1], const double (&v)[W], const double (&r)[W],
                                              double K, int lane, bool& ok) {
  int jo = 0, to = 0;  // first step not yet verified (lane, step); K = the true value there
  for (int round = 0;; ++round) {
    if (round == GK_SPEC_ROUNDS) {  // pathological data (infinities, NaNs): the caller walks it one at a time
      ok = false;
      return K;
    }
    double xt = X[0];
#pragma unroll
    for (int t = 1; t < W; ++t)
      if (t == to) xt = X[t];
    const double xprev = wave_shr1_f64(X[W], 0.0);
    const double D = wave_incl_scan_f64(lane < jo ? 0.0 : (lane == jo ? K - xt : xprev - X[0]));
    const double b0 = (lane == jo && to == 0) ? K : X[0] + D;
    const double bnx = wave_shl1_f64(b0, 0.0);  // lane j+1's b_0
    int ft = W;
    double fv = 0.0;
    double b = b0;
#pragma unroll
    for (int t = 0; t < W; ++t) {
      double bn = (t + 1 < W || lane == 63) ? X[t + 1] + D : bnx;
      if (lane == jo && t + 1 == to) bn = K;
      const double f = KIND == 0 ? b + (v[t] - b) * r[t] : b + v[t];
      const bool act = lane > jo || (lane == jo && t >= to);
      if (act && ft == W && __double_as_longlong(f) != __double_as_longlong(bn)) {
        ft = t;
        fv = f;
      }
      b = bn;
    }
    const uint64_t bad = __builtin_amdgcn_ballot_w64(ft < W);
    if (!bad) return rdlane_f64(X[W] + D, 63);
    const int jf = __builtin_amdgcn_readfirstlane(__builtin_ffsll((long long)bad) - 1);
    const int tf = __builtin_amdgcn_readlane(ft, jf);
    K = rdlane_f64(fv, jf);
    jo = jf;
    to = tf + 1;
    if (to == W) {
      ++jo;
      to = 0;
      if (jo == 64) return K;
    }
  }
}

// the gk:52-59 chain of values [k0, k1) of a stream one value at a time:
// chunks of 64 loaded per lane, then broadcast through LDS (buf) and walked in
// order by every lane (the chain's latency, ~16 ns per value)
__device__ __forceinline__ void bcast_walk(const double* __restrict__ x, const int64_t xo, const int64_t k0,
                                           const int64_t k1, int64_t& n, double& sm, double& av, double& lmn,
                                           double& lmx, int64_t& imn, int64_t& imx, const int lane, double2* buf) {
  double q[SL_BCAST_DEPTH];
#pragma unroll
  for (int d = 0; d < SL_BCAST_DEPTH; ++d) q[d] = (k0 + 64 * d + lane < k1) ? x[xo + k0 + 64 * d + lane] : 0.0;
  for (int64_t kc = k0; kc < k1; kc += 64 * SL_BCAST_DEPTH) {
#pragma unroll
    for (int d = 0; d < SL_BCAST_DEPTH; ++d) {
      const int64_t c0 = kc + 64 * d;  // first index of this chunk
      if (c0 < k1) {
        const int cn = (int)min((int64_t)64, k1 - c0);
        const double v = q[d];
        if (lane < cn) {
          const int64_t idx = c0 + lane;
          if (v < lmn) { lmn = v; imn = idx; }
          if (v > lmx) { lmx = v; imx = idx; }
        }
        buf[lane] = make_double2(v, 1.0 / (double)(n + 1 + lane));
        const int64_t nx = c0 + 64 * SL_BCAST_DEPTH + lane;  // refill: the chunk SL_BCAST_DEPTH ahead
        q[d] = (nx < k1) ? x[xo + nx] : 0.0;
        wsync<false>();
        if (cn == 64) {
          // keep GK_SL_AHEAD broadcast reads in flight (a ring of registers
          // refilled as each entry is consumed; sched_barrier pins each
          // refill before the chain step it hides)
#ifndef GK_SL_AHEAD
#define GK_SL_AHEAD 12
#endif
          double2 ring[GK_SL_AHEAD];
#pragma unroll
          for (int k = 0; k < GK_SL_AHEAD; ++k) ring[k] = buf[k];
#pragma unroll
          for (int j = 0; j < 64; ++j) {
            const double2 e = ring[j % GK_SL_AHEAD];
            if (j + GK_SL_AHEAD < 64) ring[j % GK_SL_AHEAD] = buf[j + GK_SL_AHEAD];
            __builtin_amdgcn_sched_barrier(0);
            sm = sm + e.x;                    // gk:53
            av = av + (e.x - av) * e.y;       // gk:54
          }
        } else {
          for (int j = 0; j < cn; ++j) {
            const double2 e = buf[j];
            sm = sm + e.x;
            av = av + (e.x - av) * e.y;
          }
        }
        n += cn;  // gk:52
        wsync<false>();
      }
    }
  }
}

// one wave walks stream list[w] (the broadcast layout): supersteps of 64 x
// GK_SPEC_W values by the speculative walk above, the rest one value at a
// time over LDS broadcasts
__device__ __forceinline__ void stats_long_bcast(const GKState& st, const double* __restrict__ x,
                                                 const int64_t* __restrict__ offs, const int32_t* __restrict__ list,
                                                 const int64_t* __restrict__ list_n, int w, int lane, double2* buf) {
  const int64_t s = list[w];
  const int64_t xo = offs[s];
  const int64_t L = offs[s + 1] - xo;
  int64_t n = list_n ? list_n[w] : st.n0[s];  // (no list_n: k_lengths' pre-call snapshot)
  double sm = st.sum[s], av = st.avg[s];
  double lmn = __longlong_as_double(0x7ff0000000000000LL), lmx = -lmn;
  int64_t imn = INT64_MAX, imx = INT64_MAX;
  int64_t kb = 0;  // first value of the one-at-a-time walk
#if GK_SPEC
  {
    constexpr int W = GK_SPEC_W;
    constexpr int SS = 64 * W;
    double vn[W];
    if (L >= SS) {
#pragma unroll
      for (int t = 0; t < W; ++t) vn[t] = x[xo + lane * W + t];
    }
    int fails = 0;  // failed supersteps in a row
    for (; kb + SS <= L; kb += SS) {
      double v[W], r[W];
#pragma unroll
      for (int t = 0; t < W; ++t) v[t] = vn[t];
      if (kb + 2 * SS <= L) {  // the next superstep's values, one superstep ahead
#pragma unroll
        for (int t = 0; t < W; ++t) vn[t] = x[xo + kb + SS + lane * W + t];
      }
      const int64_t i0 = kb + lane * W;  // this lane's first value (stream-relative)
#pragma unroll
      for (int t = 0; t < W; ++t) {
        r[t] = 1.0 / (double)(n + i0 + t + 1 - kb);  // gk:54's 1.0/n
        if (v[t] < lmn) { lmn = v[t]; imn = i0 + t; }  // gk:56-57 (first occurrence)
        if (v[t] > lmx) { lmx = v[t]; imx = i0 + t; }  // gk:58-59
      }
      // estimates of both chains at this lane's first value
      double p = 0.0;
      {
        double tr[W];
#pragma unroll
        for (int t = 0; t < W; ++t) tr[t] = v[t];
#pragma unroll
        for (int h = W / 2; h > 0; h >>= 1)
#pragma unroll
          for (int t = 0; t < h; ++t) tr[t] = tr[t] + tr[t + h];
        p = tr[0];
      }
      // exclusive (an estimate: any value is correct, a close one saves rounds)
      const double q = wave_incl_scan_f64(p) - p;
      const int64_t nl = n + lane * W;
      double ea = lane == 0 ? av : (av * (double)n + q) / (double)nl;
      double es = lane == 0 ? sm : sm + q;
      double XA[W + 1], XS[W + 1];
      XA[0] = ea;
      XS[0] = es;
#pragma unroll
      for (int t = 0; t < W; ++t) {
        es = es + v[t];                // gk:53
        ea = ea + (v[t] - ea) * r[t];  // gk:54
        XA[t + 1] = ea;
        XS[t + 1] = es;
      }
      bool ok = true;
      const double av1 = spec_verify<0, W>(XA, v, r, av, lane, ok);
      const double sm1 = ok ? spec_verify<1, W>(XS, v, r, sm, lane, ok) : sm;
      if (!ok) {
        // this superstep one value at a time (min/max re-seen: same indices,
        // no change); after GK_SPEC_GIVEUP failed supersteps in a row (the
        // chains at +-inf or NaN), the rest of the stream too
        bcast_walk(x, xo, kb, kb + SS, n, sm, av, lmn, lmx, imn, imx, lane, buf);
        if (++fails == GK_SPEC_GIVEUP) {
          kb += SS;
          break;
        }
        continue;  // (vn already holds the next superstep's values)
      }
      fails = 0;
      av = av1;
      sm = sm1;
      n += SS;  // gk:52
    }
  }
#endif
  bcast_walk(x, xo, kb, L, n, sm, av, lmn, lmx, imn, imx, lane, buf);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double omn = __shfl_xor(lmn, o, 64), omx = __shfl_xor(lmx, o, 64);
    const int64_t oin = __shfl_xor(imn, o, 64), oix = __shfl_xor(imx, o, 64);
    if (omn < lmn || (omn == lmn && oin < imn)) { lmn = omn; imn = oin; }
    if (omx > lmx || (omx == lmx && oix < imx)) { lmx = omx; imx = oix; }
  }
  if (lane == 0) {
    double mn = st.mn[s], mx = st.mx[s];
    if (lmn < mn) mn = lmn;  // gk:56-57: the pre-call value wins ties
    if (lmx > mx) mx = lmx;  // gk:58-59
    st.mn[s] = mn;
    st.mx[s] = mx;
    st.sum[s] = sm;
    st.avg[s] = av;
  }
  wsync<false>();
}

// The group walk of the stats kernels: lane l walks the gk:52-59 chain of
// stream s (act), starting at pre-call count n0, from a register ring of
// aligned 16-byte loads (SL_DEPTH chunks of 16 values in flight).  A step
// costs ~25 VALU for 64 chains.
__device__ __forceinline__ void stats_group_walk(const GKState& st, const double* __restrict__ x,
                                                 const int64_t* __restrict__ offs, const int64_t s, const bool act,
                                                 const int64_t n0, const int lane, double* rtile) {
  {
    const int64_t xo = act ? offs[s] : 0;
    int64_t rem = act ? offs[s + 1] - xo : 0;
    int64_t n = n0;
    double mn = 0, mx = 0, sm = 0, av = 0;
    if (act) {
      mn = st.mn[s];
      mx = st.mx[s];
      sm = st.sum[s];
      av = st.avg[s];
    }
    // peel one value when the stream starts off 16-byte alignment (pointer
    // arithmetic on x throughout, so the loads stay global_load, not flat)
    const int64_t peel = (rem > 0 && (((uintptr_t)(x + xo)) & 8)) ? 1 : 0;
    if (peel) {
      gk_stat_step(x[xo], n, sm, av, mn, mx);
      --rem;
    }
    const double* p = x + xo + peel;
    const int64_t nch = rem / 16;  // full chunks of this lane
    int64_t maxch = nch;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxch = max(maxch, (int64_t)__shfl_xor(maxch, o, 64));
    const double2* __restrict__ p2 = (const double2*)p;
    // loads past a lane's last chunk read the start of st.rtab instead (1 MiB
    // the set owns, 16-byte aligned; the values are never used), so every
    // refill load is unconditional and the wait before a slot is consumed
    // stays partial
    const double2* __restrict__ dummy = (const double2*)st.rtab;
    double2 ring[SL_DEPTH][8];
#pragma unroll
    for (int d = 0; d < SL_DEPTH; ++d) {
      const double2* src = (d < nch) ? p2 + d * 8 : dummy;
#pragma unroll
      for (int j = 0; j < 8; ++j) ring[d][j] = src[j];
    }
    // Uniform group: every active lane starts at the same n with the same
    // number of full chunks (cfg4: equal-length rows).  Then the gk:54
    // factors 1.0/n are the same for all lanes: the wave computes 64 of them
    // at once (lane j: 1.0/(n+1+j), one IEEE division per 64 values) into
    // LDS every 4 chunks, and a chunk reads its 16 as broadcast LDS loads --
    // instead of 16 divisions per lane and chunk (~15 of a step's ~27 VALU).
    const uint64_t am = __builtin_amdgcn_ballot_w64(act);
    const int fl = am ? __builtin_amdgcn_readfirstlane(__builtin_ffsll((long long)am) - 1) : 0;
    const int64_t n_f = __shfl(n, fl, 64), nch_f = __shfl(nch, fl, 64);
    const bool uni = __builtin_amdgcn_ballot_w64(act && (n != n_f || nch != nch_f)) == 0;
    for (int64_t c0 = 0; c0 < maxch; c0 += SL_DEPTH) {
#pragma unroll
      for (int d = 0; d < SL_DEPTH; ++d) {
        const int64_t c = c0 + d;
        if (uni && c < nch_f && (c & 3) == 0) {
          rtile[lane] = 1.0 / (double)(n_f + 16 * c + 1 + lane);
          wsync<false>();
        }
        if (c < nch) {
          // reciprocals 1.0/n off the chain (IEEE divisions), then the chain
          double rc[16];
          if (uni) {
#pragma unroll
            for (int k = 0; k < 16; ++k) rc[k] = rtile[16 * (int)(c & 3) + k];
          } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) rc[k] = 1.0 / (double)(n + 1 + k);
          }
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const double v = (k & 1) ? ring[d][k >> 1].y : ring[d][k >> 1].x;
            sm = sm + v;                    // gk:53
            av = av + (v - av) * rc[k];     // gk:54
            if (v < mn) mn = v;             // gk:56-57
            if (v > mx) mx = v;             // gk:58-59
          }
          n += 16;                          // gk:52
        }
        if (uni && (c & 3) == 3) wsync<false>();  // rtile is rewritten at the next chunk
        // refill this slot with the chunk SL_DEPTH ahead (unconditional load)
        const int64_t nx = c + SL_DEPTH;
        const double2* src = (nx < nch) ? p2 + nx * 8 : dummy;
#pragma unroll
        for (int j = 0; j < 8; ++j) ring[d][j] = src[j];
      }
    }
    const int tail = (int)(rem - nch * 16);
    for (int k = 0; k < tail; ++k) gk_stat_step(p[nch * 16 + k], n, sm, av, mn, mx);
    if (act) {
      st.mn[s] = mn;
      st.mx[s] = mx;
      st.sum[s] = sm;
      st.avg[s] = av;
    }
  }
}

// A failed host walk: the picked streams' chains on the device instead (the
// one-wave-per-stream walk of k_stats_long), so their _sum/_avg/_min/_max are
// exact either way.  Exits at once when the host walk succeeded.
__global__ __launch_bounds__(64) void k_hc_fallback(GKState st, const double* __restrict__ x,
                                                    const int64_t* __restrict__ offs,
                                                    const int32_t* __restrict__ list,
                                                    const int64_t* __restrict__ list_n,
                                                    const int32_t* __restrict__ hc_count,
                                                    const int32_t* __restrict__ fail) {
  __shared__ double2 buf[64];
  if (*fail == 0) return;
  const int k = *hc_count;
  for (int w = blockIdx.x; w < k; w += gridDim.x) stats_long_bcast(st, x, offs, list, list_n, w, threadIdx.x, buf);
}

__global__ __launch_bounds__(64) void k_stats_long(GKState st, const double* __restrict__ x,
                                                   const int64_t* __restrict__ offs,
                                                   const int32_t* __restrict__ list,
                                                   const int64_t* __restrict__ list_n,
                                                   const int32_t* __restrict__ count,
                                                   const int32_t* __restrict__ hc_count, int prio) {
  __shared__ double2 buf[64];
  __shared__ double rtile[64];
  const int lane = threadIdx.x;
  const int cnt = *count;
  if (cnt <= GK_SL_BCAST) {
    if (prio) __builtin_amdgcn_s_setprio(3);
    // the first *hc_count streams are walked on host cores (k_hc_prep)
    const int w0 = hc_count ? *hc_count : 0;
    for (int w = w0 + blockIdx.x; w < cnt; w += gridDim.x) stats_long_bcast(st, x, offs, list, list_n, w, lane, buf);
    return;
  }
  const int ngroups = (cnt + 63) / 64;
  for (int gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
    const int w = gi * 64 + lane;
    const bool act = w < cnt;
    stats_group_walk(st, x, offs, act ? (int64_t)list[w] : 0, act, act ? (list_n ? list_n[w] : st.n0[list[w]]) : 0,
                     lane, rtile);
  }
}

// k_stats_short: the short streams' chains (up to GK_STATS_LONG values; the
// longer ones are k_stats_long's) when the small-class launch does not walk
// them (P > 128: cfg5), 64 consecutive streams per wave with the group walk
// of k_stats_long.  A wave's trip count is its own longest stream, not a
// 256-stream block's (Zipf lengths: the former k_stats block-uniform chunk loop took
// ~9 ms of a cfg5 step ahead of the ingest launch).  Runs before k_ingest on
// the same HIP stream: st.n is the pre-call n.
__global__ __launch_bounds__(64) void k_stats_short(GKState st, const double* __restrict__ x,
                                                    const int64_t* __restrict__ offs) {
  __shared__ double rtile[64];
  const int lane = threadIdx.x;
  const int64_t ngroups = (st.S + 63) / 64;
  for (int64_t gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
    const int64_t s = gi * 64 + lane;
    bool act = s < st.S;
    if (act) {
      const int64_t L = offs[s + 1] - offs[s];
      act = L > 0 && L <= GK_STATS_LONG;
    }
    stats_group_walk(st, x, offs, act ? s : 0, act, act ? st.n[s] : 0, lane, rtile);
  }
}

// ===========================================================================
// k_ingest: the add-driven flush path.
//
// One wave owns one stream for the whole call.  The stream's table is loaded
// into LDS once, every flush of the call (gk:60-61: when n % P == 0) runs
// against it there, and the final table is written back once.
//
// A flush (merge_compress with only raw pending values, gk:63-109) is
// evaluated in closed form: every pending value x
// is placed in gap j = #{entries <= x}; with m_j values in gap j and an
// integer carry c from a removed predecessor,
//     G = g_j + c + k,   k = clamp(T - d_j - (g_j + c), 0, m_j)
// the k smallest gap values are absorbed into entry j (rule R3 true branch),
// the remaining m_j - k are emitted as (x, 1, G + d_j - 1) (R3 false branch),
// and entry j is removed (carry G) iff G + g_{j+1} + d_{j+1} <= T (R1/R4).
// The tail (values >= the last entry, rule R2) is cut into chunks of
// max(T,1) values, each emitting (last value, chunk size, 0).
// ===========================================================================
// Working storage of one flush: the table (single-buffered for the 256
// class, whose entries a lane caches in registers; double-buffered above),
// per-gap scratch and the pending values (members / sort area).  LDS for the
// 256 / 2048 classes, a per-block global workspace for the largest class
// (same code; the address space is known at compile time, so LDS accesses
// stay ds_* instructions).
struct FlushBuf {
  double* tv[2];     // table values: old buffer tv[cur], new buffer tv[cur^1]
  int32_t* tg[2];    //   (both the same array when single-buffered)
  int32_t* td[2];
  uint32_t* gpk;     // per gap: count, then packed (gap base << 16) | out base
  int32_t* gk;       // per entry: absorbed count k | KEEP bit
  int32_t* gdel;     // per entry: G, then delta of emitted gap values G+d-1
  double* mv;        // pending values: grouped by gap, or the sort keys
  uint32_t* mp;      // their payload (insertion index << 16) | gap
};

template <int CAP, int VPL>
struct FlushLDS {
  static constexpr int NB = CAP <= 256 ? 1 : 2;
  double tv[NB][CAP];
  int32_t tg[NB][CAP];
  int32_t td[NB][CAP];
  uint32_t gpk[CAP + 1];
  int32_t gk[CAP + 1];
  int32_t gdel[CAP + 1];
  double mv[64 * VPL];
  uint32_t mp[64 * VPL];
};

// bytes of one block's global workspace for capacity `cap`
__host__ __device__ inline size_t gk_flush_ws_bytes(int cap, int vpl) {
  size_t b = 2 * (size_t)cap * 8 + 4 * (size_t)cap * 4 + 3 * ((size_t)cap + 1) * 4 + 64 * (size_t)vpl * 12;
  return (b + 255) & ~(size_t)255;
}

__device__ inline FlushBuf flush_buf_global(unsigned char* base, int cap, int vpl) {
  FlushBuf b;
  double* dp = (double*)base;
  b.tv[0] = dp; dp += cap;
  b.tv[1] = dp; dp += cap;
  b.mv = dp; dp += 64 * vpl;
  int32_t* ip = (int32_t*)dp;
  b.tg[0] = ip; ip += cap;
  b.tg[1] = ip; ip += cap;
  b.td[0] = ip; ip += cap;
  b.td[1] = ip; ip += cap;
  b.gpk = (uint32_t*)ip; ip += cap + 1;
  b.gk = ip; ip += cap + 1;
  b.gdel = ip; ip += cap + 1;
  b.mp = (uint32_t*)ip;
  return b;
}

template <int CAP, int VPL>
__device__ inline FlushBuf flush_buf_lds(FlushLDS<CAP, VPL>& L) {
  constexpr int NB = FlushLDS<CAP, VPL>::NB;
  FlushBuf b;
  b.tv[0] = L.tv[0]; b.tv[1] = L.tv[NB - 1];
  b.tg[0] = L.tg[0]; b.tg[1] = L.tg[NB - 1];
  b.td[0] = L.td[0]; b.td[1] = L.td[NB - 1];
  b.gpk = L.gpk; b.gk = L.gk; b.gdel = L.gdel; b.mv = L.mv; b.mp = L.mp;
  return b;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_SHR(1), 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_SHR(2), 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_SHR(4), 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_SHR(8), 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_BCAST15, 0xa, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_BCAST31, 0xc, 0xf, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// smallest power of two strictly above e (e >= 0)
__device__ __forceinline__ int gk_pow2_above(int e) { return 1 << (32 - __clz(e)); }

// +inf into tv[E .. pow2_above(E)-2]: the probes of the branch-free search
__device__ __forceinline__ void gk_pad_table(double* tv, int E, int lane) {
  const int hi = gk_pow2_above(E) - 1;
  for (int j = E + lane; j < hi; j += 64) tv[j] = __longlong_as_double(0x7ff0000000000000LL);
}

// Gap sizes above this use the bitonic sort instead of the per-gap rank loop.
#define GK_RANK_LOOP_MAX 24
#define GK_PAD_PAYLOAD 0xFFFF0000u  // sorts after every real value (idx < 0xFFFF)

// x (insertion index i, gap `gap`, rank `rk` inside its gap): gk:93-99 for
// gap < E (the k smallest are absorbed, the rest emitted as (x, 1, G+d-1)),
// gk:85-92 for the tail (chunks of max(T,1): emit each chunk's last value).
__device__ __forceinline__ void emit_value(const FlushBuf& L, double* nv, int32_t* ng, int32_t* nd, int E,
                                           int totm, int cs, double x, int gap, int rk) {
  const uint32_t pk = L.gpk[gap];
  if (gap < E) {
    const int k = L.gk[gap] & ~GK_KEEP_BIT;
    if (rk >= k) {
      const int pos = (int)(pk & 0xffffu) + rk - k;
      nv[pos] = x;
      ng[pos] = 1;
      nd[pos] = L.gdel[gap];
    }
  } else {
    const int m = totm - (int)(pk >> 16);
    const int q = rk / cs;
    const int rr = rk - q * cs;
    if (rr == cs - 1 || rk == m - 1) {
      const int pos = (int)(pk & 0xffffu) + q;
      nv[pos] = x;
      ng[pos] = rr + 1;
      nd[pos] = 0;
    }
  }
}

// Returns the new table size, or -1 if it would exceed `cap` (nothing is
// written to the table in that case).  `cur` selects the old buffer; on
// success the new table is in buffer cur^1.  (The 256 class has its own
// flush, flush_small, below.)
// `after_search` runs once every lane has read the old table for the gap
// search; k_ingest issues the next flush's value loads there, so that the
// compiler's first vmcnt wait for them lands in the NEXT flush.
template <int VPL, bool GLOBAL, typename AfterSearch>
__device__ __forceinline__ int flush_wave(const FlushBuf& L, const int cap, const int cur, const int E,
                                          const double (&xv)[VPL], const int cnt, const int T,
                                          const int lane, AfterSearch&& after_search, const bool presorted) {
  // selects, not L.tv[cur]: a runtime index into the pointer pair would put
  // the pair in scratch memory
  const double* __restrict__ tv = cur ? L.tv[1] : L.tv[0];
  const int32_t* __restrict__ tg = cur ? L.tg[1] : L.tg[0];
  const int32_t* __restrict__ td = cur ? L.td[1] : L.td[0];
  double* __restrict__ nv = cur ? L.tv[0] : L.tv[1];
  int32_t* __restrict__ ng = cur ? L.tg[0] : L.tg[1];
  int32_t* __restrict__ nd = cur ? L.td[0] : L.td[1];

  // ---- gap of each pending value: number of entries <= x (gk:93 '<' puts
  //      a value equal to an entry after that entry); the VPL searches
  //      advance in lock step so their LDS reads overlap -------------------
  // The table is padded with +inf up to index pow2ceil(E+1)-2, so every probe
  // is in range and the search is branch-free; a value of +inf can step into
  // the padding, hence the final min with E.
  int xg[VPL];
#pragma unroll
  for (int r = 0; r < VPL; ++r) xg[r] = 0;
  for (int step = gk_pow2_above(E) >> 1; step > 0; step >>= 1) {
    double tvv[VPL];
#pragma unroll
    for (int r = 0; r < VPL; ++r) tvv[r] = tv[xg[r] + step - 1];
#pragma unroll
    for (int r = 0; r < VPL; ++r) xg[r] += (tvv[r] <= xv[r]) ? step : 0;
  }
#pragma unroll
  for (int r = 0; r < VPL; ++r) xg[r] = min(xg[r], E);
  GK_BMARK(1);
  after_search();
  for (int j = lane; j <= E; j += 64) L.gpk[j] = 0u;
  wsync<GLOBAL>();
  uint32_t xs[VPL];
#pragma unroll
  for (int r = 0; r < VPL; ++r) {
    const int i = lane + 64 * r;
    xs[r] = (i < cnt) ? atomicAdd(&L.gpk[xg[r]], 1u) : 0u;
  }
  wsync<GLOBAL>();
  uint32_t mloc = 0;
#pragma unroll
  for (int r = 0; r < VPL; ++r) mloc = max(mloc, xs[r] + 1u);
  const bool use_sort = !presorted && wave_max_u32(mloc) > GK_RANK_LOOP_MAX;
  GK_BMARK(2);

  // ---- carry walk over the entries (closed form of gk:93-106) --------------
  // Lane l owns the contiguous block [l*K, l*K+K).  A lane can run its block
  // once its carry-in is known: lane 0, or a lane whose predecessor entry is
  // kept even with carry 0 (then it is kept for any carry, because G grows
  // with c).  Remaining lanes wait for their left neighbour (rounds).
  const int K = (E + 63) >> 6;
  const int j0 = lane * K;
  const int jend = min(j0 + K, E);
  const bool has = j0 < E;
  const int cs = T > 1 ? T : 1;
  const int tail_lane = E == 0 ? 0 : (E - 1) / K;
  bool known = (lane == 0) || !has;
  if (has && lane > 0) {
    const int jp = j0 - 1;
    const int g = tg[jp], d = td[jp], m = (int)L.gpk[jp];
    const int G0 = g + clampi(T - d - g, 0, m);
    known = !(G0 + tg[j0] + td[j0] <= T);
  }
  bool done = !has;
  int cin = 0, cout = 0;
  uint32_t incl, total;
  int newE;
  {
    for (;;) {
      if (known && !done) {
        int c = cin;
        for (int j = j0; j < jend; ++j) {
          const int g = tg[j], d = td[j], m = (int)L.gpk[j];
          const int Gp = g + c;
          const int k = clampi(T - d - Gp, 0, m);
          const int G = Gp + k;
          const bool rem = (j + 1 < E) && (G + tg[j + 1] + td[j + 1] <= T);
          L.gk[j] = k | (rem ? 0 : GK_KEEP_BIT);
          L.gdel[j] = G;
          c = rem ? G : 0;
        }
        cout = c;
        done = true;
      }
      const int pc = wave_shr1(cout, 0);
      const int pd = wave_shr1((int)done, 1);
      if (!known && pd) {
        known = true;
        cin = pc;
      }
      if (__all(done)) break;
    }
    GK_BMARK(3);
    uint32_t sm = 0, so = 0;
    for (int j = j0; j < jend; ++j) {
      const int m = (int)L.gpk[j];
      const int kk = L.gk[j];
      sm += (uint32_t)m;
      so += (uint32_t)(m - (kk & ~GK_KEEP_BIT) + ((kk & GK_KEEP_BIT) ? 1 : 0));
    }
    if (lane == tail_lane) {
      const int mE = (int)L.gpk[E];
      sm += (uint32_t)mE;
      so += (uint32_t)((mE + cs - 1) / cs);
    }
    incl = wave_incl_scan_u32((sm << 16) | so, lane);
    total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    newE = (int)(total & 0xffffu);
    if (newE > cap - 1) return -1;  // one slot stays free for the search padding
    uint32_t base = incl - ((sm << 16) | so);
    for (int j = j0; j < jend; ++j) {
      const int m = (int)L.gpk[j];
      const int kk = L.gk[j];
      const int k = kk & ~GK_KEEP_BIT;
      const int G = L.gdel[j];
      const int d = td[j];
      L.gpk[j] = base;
      L.gdel[j] = G + d - 1;
      if (kk & GK_KEEP_BIT) {
        const int pos = (int)(base & 0xffffu) + m - k;
        nv[pos] = tv[j];
        ng[pos] = G;
        nd[pos] = d;
      }
      base += ((uint32_t)m << 16) | (uint32_t)(m - k + ((kk & GK_KEEP_BIT) ? 1 : 0));
    }
    if (lane == tail_lane) L.gpk[E] = base;
  }
  const int totm = (int)(total >> 16);
  wsync<GLOBAL>();
  GK_BMARK(4);

  // ---- stable order inside each gap (gk:72), then emit --------------------
  if (presorted) {
    // values arrive in (value, insertion index) order (k_presort): the rank
    // inside the gap is the position minus the gap's base
#pragma unroll
    for (int r = 0; r < VPL; ++r) {
      const int q = lane + 64 * r;
      if (q < cnt) emit_value(L, nv, ng, nd, E, totm, cs, xv[r], xg[r], q - (int)(L.gpk[xg[r]] >> 16));
    }
    GK_BMARK(5);
  } else if (!use_sort) {
    // small gaps: scatter by gap, rank by comparison with the gap's members
#pragma unroll
    for (int r = 0; r < VPL; ++r) {
      const int i = lane + 64 * r;
      if (i < cnt) {
        const int pos = (int)(L.gpk[xg[r]] >> 16) + (int)xs[r];
        L.mv[pos] = xv[r];
        L.mp[pos] = (uint32_t)i;
      }
    }
    wsync<GLOBAL>();
#pragma unroll
    for (int r = 0; r < VPL; ++r) {
      const int i = lane + 64 * r;
      if (i < cnt) {
        const int gap = xg[r];
        const int gb = (int)(L.gpk[gap] >> 16);
        const int ge = gap < E ? (int)(L.gpk[gap + 1] >> 16) : totm;
        const double x = xv[r];
        int rk = 0;
        int t = gb;
        for (; t + 1 < ge; t += 2) {
          const double y0 = L.mv[t], y1 = L.mv[t + 1];
          const int i0 = (int)L.mp[t], i1 = (int)L.mp[t + 1];
          rk += (int)((y0 < x) | ((y0 == x) & (i0 < i)));
          rk += (int)((y1 < x) | ((y1 == x) & (i1 < i)));
        }
        if (t < ge) {
          const double y0 = L.mv[t];
          rk += (int)((y0 < x) | ((y0 == x) & ((int)L.mp[t] < i)));
        }
        emit_value(L, nv, ng, nd, E, totm, cs, x, gap, rk);
      }
    }
    GK_BMARK(5);
  } else {
    // a large gap (first flush: everything is tail; adversarial orders):
    // bitonic sort of all values by (value, insertion index); all values of
    // gap g precede those of gap g+1, so rank = sorted position - gap base
    constexpr int N = 64 * VPL;
#pragma unroll
    for (int r = 0; r < VPL; ++r) {
      const int i = lane + 64 * r;
      L.mv[i] = (i < cnt) ? xv[r] : __longlong_as_double(0x7ff0000000000000LL);
      L.mp[i] = (i < cnt) ? (((uint32_t)i << 16) | (uint32_t)xg[r]) : GK_PAD_PAYLOAD;
    }
    wsync<GLOBAL>();
    for (int k = 2; k <= N; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int pp = lane; pp < N / 2; pp += 64) {
          const int i = ((pp & ~(j - 1)) << 1) | (pp & (j - 1));
          const int l = i + j;
          const double a = L.mv[i], b = L.mv[l];
          const uint32_t pa = L.mp[i], pb = L.mp[l];
          const bool a_gt = (a > b) || (a == b && (pa >> 16) > (pb >> 16));
          const bool asc = (i & k) == 0;
          if (a_gt == asc) {
            L.mv[i] = b;
            L.mv[l] = a;
            L.mp[i] = pb;
            L.mp[l] = pa;
          }
        }
        wsync<GLOBAL>();
      }
    }
#pragma unroll
    for (int r = 0; r < VPL; ++r) {
      const int q = lane + 64 * r;
      if (q < cnt) {
        const double x = L.mv[q];
        const int gap = (int)(L.mp[q] & 0xffffu);
        const int rk = q - (int)(L.gpk[gap] >> 16);
        emit_value(L, nv, ng, nd, E, totm, cs, x, gap, rk);
      }
    }
    GK_BMARK(6);
  }
  gk_pad_table(nv, newE, lane);
  wsync<GLOBAL>();
  GK_BMARK(7);
  return newE;
}


// ===========================================================================
// Quantiles of one stream from its table (gk:156-232), wave-parallel.
//   large n: the reference walks i = 0.. while prefix_g(i) + d_i - 1 <=
//   rank + spread; the first i that breaks is the number of i whose RUNNING
//   MAX of prefix_g + d - 1 is <= rank + spread (the running max is
//   monotone), so each q is one count over the table.
//   small n (n < 1/eps, gk:169): numpy.percentile(values, q*100), linear.
// qmode 0 (quantiles, sorted qs): no break -> _max (gk:225-230)
// qmode 1 (quantile / unsorted qs): no break -> entries[-1].val (gk:185)
// ===========================================================================
__device__ __forceinline__ double gk_nan() { return __longlong_as_double(0x7ff8000000000000LL); }

// SV / SI: element strides of the value / g,d arrays (1 for the split
// arrays of the large classes, 2 / 4 for the GKRec table of the 256 class)
template <typename At>
__device__ __forceinline__ double percentile_linear_at(int E, double q, At at) {
  // numpy 2.2.6 _function_base_impl.py: q/100 (l.4257), (n-1)*q (l.107),
  // bounds (l.4748-4750), gamma (l.4632), _lerp (l.4653-4657)
  const double qq = (q * 100.0) / 100.0;
  const double vi = (double)(E - 1) * qq;
  double prev;
  double a, b;
  if (vi >= (double)(E - 1)) {
    prev = -1.0;
    a = at(E - 1);
    b = a;
  } else if (vi < 0.0) {
    prev = 0.0;
    a = at(0);
    b = a;
  } else {
    prev = floor(vi);
    const int pi = (int)prev;
    a = at(pi);
    b = at(pi + 1);
  }
  const double gamma = vi - prev;
  const double diff = b - a;
  if (gamma >= 0.5) return b - diff * (1.0 - gamma);
  return a + diff * gamma;
}

template <int SV>
__device__ double percentile_linear_arr(const double* __restrict__ tv, int E, double q) {
  return percentile_linear_at(E, q, [&](int i) { return tv[i * SV]; });
}

template <int SV, int SI>
__device__ __attribute__((noinline)) void wave_quantiles(const double* __restrict__ tv, const int32_t* __restrict__ tg,
                               const int32_t* __restrict__ td, int E, int64_t n, double mn, double mx,
                               const GKState& st, const double* __restrict__ qs, int nq, int qmode,
                               double* __restrict__ out, int lane) {
  if (n == 0 || E == 0) {
    for (int q = lane; q < nq; q += 64) out[q] = gk_nan();
    return;
  }
  if ((double)n < st.inv_eps) {  // gk:169 / gk:200
    for (int q = lane; q < nq; q += 64) {
      const double qv = qs[q];
      out[q] = (qv >= 0.0 && qv <= 1.0) ? percentile_linear_arr<SV>(tv, E, qv) : gk_nan();
    }
    return;
  }
  const int K = (E + 63) >> 6;
  const int j0 = lane * K;
  const int jend = min(j0 + K, E);
  int64_t bsum = 0;
  for (int j = j0; j < jend; ++j) bsum += tg[j * SI];
  const int64_t bex = wave_incl_scan_i64(bsum, lane) - bsum;
  int64_t acc = bex, bmax = INT64_MIN;
  for (int j = j0; j < jend; ++j) {
    acc += tg[j * SI];
    const int64_t a = acc + td[j * SI] - 1;
    if (a > bmax) bmax = a;
  }
  const int64_t pmax_incl = wave_incl_max_i64(bmax, lane);
  int64_t pmax_ex = __shfl_up(pmax_incl, 1, 64);
  if (lane == 0) pmax_ex = INT64_MIN;
  const int64_t spread = (int64_t)(st.eps * (double)(n - 1));  // gk:174 / gk:210
  for (int q = 0; q < nq; ++q) {
    const double qv = qs[q];
    const bool valid = (qv >= 0.0 && qv <= 1.0);
    const int64_t rank = valid ? (int64_t)(qv * (double)(n - 1) + 1.0) : 0;  // gk:173
    const int64_t th = rank + spread;
    int c = 0;
    int64_t run = pmax_ex, a2 = bex;
    for (int j = j0; j < jend; ++j) {
      a2 += tg[j * SI];
      const int64_t a = a2 + td[j * SI] - 1;
      if (a > run) run = a;
      c += (run <= th) ? 1 : 0;
    }
    const int i = wave_sum_i32(c);
    if (lane == 0) {
      double r;
      if (!valid) r = gk_nan();
      else if (i == 0) r = mn;                          // gk:182-183 / gk:220
      else if (i < E) r = tv[(i - 1) * SV];                    // gk:185 / gk:220
      else r = (qmode == 0) ? mx : tv[(E - 1) * SV];           // gk:229 / gk:185
      out[q] = r;
    }
  }
}

// k_query_list: quantiles (gk:156-232) of the listed streams from their
// committed tables in HBM, one wave per stream.  The fused ingest+query
// launch answers every stream before k_stats_long (running beside it) has
// produced the final _min/_max of the long streams (gk:183, 220, 229); this
// launch re-answers exactly those streams once it has joined.
// The join of a fused ingest + query (one wave per block):
//  * qfix (the small-class launch carried the stats role): an answer that is
//    _min or _max (gk:182-183, gk:229) was written as a marker NaN while the
//    stats role could still be writing them; now they are final.  One answer
//    per thread (the grid covers S*nq; no loop: every load in flight at once).
//  * the long streams (`list`), answered again from their final _min/_max
//    (k_stats_long ran beside the ingest), one per wave.  (A long stream
//    whose answer the qfix part also resolves gets the same bits from both.)
__global__ __launch_bounds__(256) void k_query_list(GKState st, const int32_t* __restrict__ list,
                                                    const int32_t* __restrict__ count,
                                                    const double* __restrict__ qs, int nq, int qmode,
                                                    double* __restrict__ qout, int qfix) {
  const int lane = threadIdx.x & 63;
#ifdef GK_TIMELINE
  if (blockIdx.x == 0 && threadIdx.x == 0) gk_tl_call[1] = __builtin_amdgcn_s_memrealtime();
#endif
  if (qfix) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < st.S * (int64_t)nq) {
      const long long b = __double_as_longlong(qout[i]);
      if (b == GK_QMARK_MIN || b == GK_QMARK_MAX) {
        const int64_t s = i / nq;
        qout[i] = b == GK_QMARK_MIN ? st.mn[s] : st.mx[s];
      }
    }
  }
  const int cnt = *count;
  const int wid = (int)(blockIdx.x * 4 + (threadIdx.x >> 6)), nwv = (int)(gridDim.x * 4);
  for (int w = wid; w < cnt; w += nwv) {
    const int64_t s = list[w];
    const GKRec* tab = gk_table_ptr(st, s);
    wave_quantiles<2, 4>(&tab->v, &tab->g, &tab->d, st.E[s], st.n[s], st.mn[s], st.mx[s], st, qs, nq, qmode,
                         qout + s * (int64_t)nq, lane);
  }
}

// CAP > 0: LDS working storage of that capacity (class 256 / 2048).
// CAP == 0: global workspace `ws` (ws_bytes per block) of capacity `cap`.
// list == NULL: every class-0 stream; else the listed streams (class c > 0).
// count_ptr (device, may be NULL): the list length is read from there (lists
// built on the device: promotion re-runs, class member lists).  lcls: the
// class this launch serves; a listed stream now in another class (promoted
// further since it was listed) is skipped.
template <int CAP, int VPL>
__global__ __launch_bounds__(64) void k_ingest(GKState st, const double* __restrict__ x,
                                               const int64_t* __restrict__ offs,
                                               const int32_t* __restrict__ list, int64_t count,
                                               const int32_t* __restrict__ count_ptr, int lcls,
                                               int force, int cap, unsigned char* ws, size_t ws_bytes,
                                               int32_t* __restrict__ ovf_count,
                                               int32_t* __restrict__ ovf_list, const double* __restrict__ qs,
                                               int nq, double* __restrict__ qout, int qmode,
                                               unsigned long long* __restrict__ work,
                                               const int32_t* __restrict__ prio,
                                               const int32_t* __restrict__ prio_count,
                                               const double* __restrict__ psort,
                                               const int64_t* __restrict__ prio_ws,
                                               const int32_t* __restrict__ prio_skip, GKPoolDev pool, int pmode) {
  // pmode (promotion rounds, gk_capi.cpp promote_rounds): bit 0 -- `list` is
  // the previous round's overflow list and this launch moves each stream
  // whose next class is lcls into it first (k_promote_dev's level -1 step,
  // one launch fewer per round); bit 1 -- lcls is the last class: a stream
  // that outgrows it is counted fatal here instead of listed for a promotion
  // round that could only count it; bit 2 -- the next class has no slot: a
  // stream that outgrows lcls is deferred here (what that round would do)
  // the first *prio_skip streams of `prio` are k_ingest_wg's: skipped here,
  // and as many blocks leave at once so that its workgroups find free CUs
  const int skip = prio_skip ? *prio_skip : 0;
  if (skip > 0 && (int)blockIdx.x >= (int)gridDim.x - skip && gridDim.x > (unsigned)skip) return;
  constexpr int LCAP = CAP > 0 ? CAP : 1;
  constexpr int LVPL = CAP > 0 ? VPL : 1;
  __shared__ FlushLDS<LCAP, LVPL> Ls;
  FlushBuf B;
  if constexpr (CAP > 0) {
    B = flush_buf_lds<LCAP, LVPL>(Ls);
    cap = CAP;
  } else {
    B = flush_buf_global(ws + (size_t)blockIdx.x * ws_bytes, cap, VPL);
  }
  const int lane = threadIdx.x;
  const int P = st.P;
#ifdef GK_PROF
  if (lane == 0) {
    for (int i = 0; i < GK_PROF_NSEC; ++i) gk_big_prof().acc[i] = 0;
    gk_big_prof().t = gk_cycles();
  }
#endif
  // headers are prefetched one stream ahead; flush-only launches pass
  // x == NULL and an all-zero offs array
  // Streams are handed out dynamically (one atomic per stream on `work`,
  // zeroed before the launch).  Work items [0, npri) are the streams of
  // `prio` -- the streams longer than GK_STATS_LONG values, longest first
  // (k_sort_long) -- so that the long sequential flush chains start at once;
  // items [npri, npri+count) are the launch's streams in order, minus those
  // already taken from `prio` (the same length test k_lengths applied).
  if (count_ptr) count = *count_ptr;
  const int64_t npri = prio ? max((int64_t)*prio_count - skip, (int64_t)0) : 0;
  const int64_t total = npri + count;
  // blocks past the item count leave before the hand-out (the ones below it
  // take every item): an empty or short re-run list costs no atomics
  if ((int64_t)blockIdx.x >= total) return;
  auto grab = [&]() -> int64_t {
    unsigned long long v = 0;
    if (lane == 0) v = atomicAdd(work, 1ull);
    return rfl64((int64_t)v);
  };
  auto sid = [&](int64_t w) -> int64_t {
    return w < npri ? (int64_t)prio[w + skip] : (list ? (int64_t)list[w - npri] : w - npri);
  };
  GKHdrV hv;
  int64_t w = grab();
  if (w < total) gk_hdr_issue(hv, st, offs, sid(w));
  for (; w < total;) {
    const int64_t s = sid(w);
    const bool from_prio = w < npri;
    // presorted automatic-flush batches of this stream (k_presort), or none
    const int64_t wso = (from_prio && prio_ws) ? rfl64(prio_ws[w + skip]) : -1;
    const int64_t wn = grab();
    const int32_t scls = __builtin_amdgcn_readfirstlane(hv.cls);
    const int32_t sslot = __builtin_amdgcn_readfirstlane(hv.slot);
    int p = __builtin_amdgcn_readfirstlane(hv.pend);
    int E = __builtin_amdgcn_readfirstlane(hv.E);
    int64_t n = rfl64(hv.n);
    const int64_t xo0 = rfl64(hv.xo);
    const int64_t xe = rfl64(hv.xe);
    const double smn = __longlong_as_double(rfl64(__double_as_longlong(hv.mn)));
    const double smx = __longlong_as_double(rfl64(__double_as_longlong(hv.mx)));
    if (wn < total) gk_hdr_issue(hv, st, offs, sid(wn));
    w = wn;
    int32_t ucls = scls, uslot = sslot;  // the stream's class and slot from here on
    if (pmode & 1) {
      if (scls + 1 != lcls) continue;  // another class's launch promotes it
      int slot = -1;
      if (lane == 0) {
        slot = atomicAdd(&pool.ctr[GK_CTR_USED + lcls], 1);
        if (slot >= st.alloc[lcls]) {
          atomicSub(&pool.ctr[GK_CTR_USED + lcls], 1);
          slot = -1;
          pool.defer[atomicAdd(&pool.ctr[GK_CTR_DEFER], 1)] = (int32_t)s;  // (re-run by the host)
        }
      }
      slot = __builtin_amdgcn_readfirstlane(__shfl(slot, 0, 64));
      if (slot < 0) continue;
      // the pre-call table moves to the new slot (the LDS load below reads
      // the old one): an overflow in this class leaves it there for the
      // next round
      const GKRec* __restrict__ osrc = gk_table_ptr_cs(st, s, scls, sslot);
      GKRec* __restrict__ odst = st.tab[lcls] + (int64_t)slot * st.cap[lcls];
      const int oE = min(E, st.cap[scls]);
      for (int j = lane; j < oE; j += 64) odst[j] = osrc[j];
      if (lane == 0) {
        st.cls[s] = lcls;
        st.slot[s] = slot;
        pool.list[lcls][atomicAdd(&pool.ctr[GK_CTR_LCNT + lcls], 1)] = (int32_t)s;
      }
      ucls = lcls;
      uslot = slot;
    } else if (scls != lcls) {
      continue;  // in another class: handled by that class's launch
    }
    // a promoted stream continues from value n - n0 of the call (the flushes
    // its smaller class made before overflowing are committed: k_ingest_small)
    const int64_t xo = xo0 + ((lcls > 0 && x) ? n - rfl64(st.n0[s]) : 0);
    const int64_t Lx = xe - xo;
    if (prio && !from_prio && Lx > GK_STATS_LONG) continue;  // taken from `prio`

    // force 1: flush only if values are pending (size/quantile, gk:45, 166, 197)
    // force 2: unconditional merge_compress() (merge, gk:122, 126, 137)
    // a query launch (qs != NULL, force 1) answers every stream
    if (Lx <= 0 && !((force == 1 && p > 0) || (force == 2 && n > 0)) && !qs) continue;
    GKRec* __restrict__ tab = gk_table_ptr_cs(st, s, ucls, uslot);
    const GKRec* __restrict__ ltab = gk_table_ptr_cs(st, s, scls, sslot);  // (pre-call table: tab unless just promoted)
    double* __restrict__ pb = st.pbuf + s * (int64_t)st.pmax;
    int cur = 0;
    // table -> LDS: all of a lane's loads are issued before the first wait
    constexpr int TL = CAP > 0 ? CAP / 64 : 8;
    for (int j0 = 0; j0 < E; j0 += 64 * TL) {
      GKRec rc[TL];
#pragma unroll
      for (int r = 0; r < TL; ++r) {
        const int j = j0 + lane + 64 * r;
        if (j < E) rc[r] = ltab[j];
      }
#pragma unroll
      for (int r = 0; r < TL; ++r) {
        const int j = j0 + lane + 64 * r;
        if (j < E) {
          B.tv[0][j] = rc[r].v;
          B.tg[0][j] = rc[r].g;
          B.td[0][j] = rc[r].d;
        }
      }
    }
    if (E <= cap - 1) gk_pad_table(B.tv[0], E, lane);
    wsync<CAP == 0>();
    GK_BMARK(0);

    // an imported / merged table with no room for the search padding, or a
    // stream past the count limit, goes straight to the overflow path
    bool ok = E <= cap - 1 && gk_count_ok(st, n + (Lx > 0 ? Lx : 0));
    bool flushed = false;  // at least one automatic flush in this call
    int64_t used = 0;
    int64_t need = P - (n % P);  // adds until n hits the next multiple of P (gk:60)
    // The values of the next flush (or the leftover tail of the batch) are
    // loaded one flush ahead: their HBM latency hides under the current
    // flush's LDS work.
    double xv[VPL];
    // presorted batch b lives at psort + wso + b*P (k_presort, same values)
    const double* __restrict__ sb = wso >= 0 ? psort + wso : nullptr;
    if (ok && used + need <= Lx) {
      if (sb) {
#pragma unroll
        for (int r = 0; r < VPL; ++r) xv[r] = sb[min(lane + 64 * r, p + (int)need - 1)];
      } else {
        gk_load_flush_values<VPL>(xv, pb, p, x + xo, p + (int)need, lane);
      }
    }
    while (ok && used + need <= Lx) {
      const int cnt = p + (int)need;
      const int64_t nused = used + need;
      const int navail = (int)min((int64_t)P, Lx - nused);  // next flush, or the leftover tail
      const bool cur_sorted = sb != nullptr;
      double xn[VPL];
#pragma unroll
      for (int r = 0; r < VPL; ++r) xn[r] = 0.0;
      auto prefetch = [&]() {
        if (navail > 0) {
          // a full next batch comes presorted; the leftover tail does not
          const double* base = (sb && navail == P) ? sb + P : x + xo + nused;
#pragma unroll
          for (int r = 0; r < VPL; ++r) xn[r] = base[min(lane + 64 * r, navail - 1)];
        }
      };
      n += need;
      GK_BMARK(8);
      const int nE = flush_wave<VPL, CAP == 0>(B, cap, cur, E, xv, cnt, gk_threshold(st, n), lane, prefetch,
                                               cur_sorted);
      if (nE < 0) {
        ok = false;
        break;
      }
      E = nE;
      cur ^= 1;
      used = nused;
      p = 0;
      need = P;
      flushed = true;
      if (sb) sb = navail == P ? sb + P : nullptr;
#pragma unroll
      for (int r = 0; r < VPL; ++r) xv[r] = (lane + 64 * r < navail) ? xn[r] : 0.0;
    }
    if (ok) {
      const int64_t rem = Lx - used;  // < need: no automatic flush for these
      // after an automatic flush the leftover values are already in xv
      if ((force == 1 && p + rem > 0) || force == 2) {
        const int cnt = p + (int)rem;
        if (!flushed) gk_load_flush_values<VPL>(xv, pb, p, x ? x + xo + used : pb, cnt, lane);
        n += rem;
        const int nE = flush_wave<VPL, CAP == 0>(B, cap, cur, E, xv, cnt, gk_threshold(st, n), lane, [] {}, false);
        if (nE < 0) {
          ok = false;
        } else {
          E = nE;
          cur ^= 1;
          p = 0;
        }
      } else {
        if (flushed) {
#pragma unroll
          for (int r = 0; r < VPL; ++r)
            if (lane + 64 * r < rem) pb[lane + 64 * r] = xv[r];
        } else {
          for (int64_t i = lane; i < rem; i += 64) pb[p + i] = x[xo + used + i];
        }
        p += (int)rem;
        n += rem;
      }
    }
    if (!ok) {
      // nothing was written back: the stream keeps its pre-call state and
      // is re-run by the host after promotion to the next capacity class
      // (past the last class: counted fatal, as k_promote_dev would)
      if (lane == 0) {
        if (pmode & 2) {
          atomicAdd(&pool.ctr[GK_CTR_FATAL], 1);
          atomicMax(&pool.ctr[GK_CTR_FATAL + 1], (int)s);
        } else if (pmode & 4) {
          pool.defer[atomicAdd(&pool.ctr[GK_CTR_DEFER], 1)] = (int32_t)s;
        } else {
          const int k = atomicAdd(ovf_count, 1);
          ovf_list[k] = (int32_t)s;
        }
      }
      wsync<CAP == 0>();
      continue;
    }
    {
      const double* fv = cur ? B.tv[1] : B.tv[0];
      const int32_t* fg = cur ? B.tg[1] : B.tg[0];
      const int32_t* fd = cur ? B.td[1] : B.td[0];
      if (qs) wave_quantiles<1, 1>(fv, fg, fd, E, n, smn, smx, st, qs, nq, qmode, qout + s * (int64_t)nq, lane);
      for (int j = lane; j < E; j += 64) {
        GKRec rc;
        rc.v = fv[j];
        rc.g = fg[j];
        rc.d = fd[j];
        tab[j] = rc;
      }
    }
    if (lane == 0) {
      st.n[s] = n;
      st.E[s] = E;
      st.pend[s] = p;
    }
    wsync<CAP == 0>();
    GK_BMARK(9);
  }
#ifdef GK_PROF
  if (lane == 0)
    for (int i = 0; i < GK_PROF_NSEC; ++i) atomicAdd(&gk_prof_acc[i], gk_big_prof().acc[i]);
#endif
}

// ===========================================================================
// k_ingest_wg: the longest streams of a batch, one WORKGROUP per stream
// (round 4).  A Zipf head (cfg5: one stream of 10^7
// values at eps = 0.001, 9 990 dependent flushes of 1 001 values) is a
// sequential chain of flushes; one wave walked it at ~11.4 us per presorted
// flush, the whole batch's critical path.  Here GK_WG_WAVES waves share each
// flush: one or two batch values per thread, a few table entries per thread,
// the carry walk resolved wave by wave (DPP) and across waves through LDS,
// one workgroup scan for the output offsets.  Same closed form and results
// as flush_wave (bit-exact; tests/test_gpu_wg.py).  Streams: the first
// *wg_count entries of the long list (k_long_prep: presorted streams with
// at least 1/GK_PRESORT_REL of the longest one's flushes, at most
// GK_WG_MAX); class-0 sets of the 2048 class (128 < P <= 1024) only.
// Batches arrive presorted (k_presort); a batch that is not (the call's
// final partial flush) is sorted here by (value, insertion index) first.
// The fused query of these streams is answered after the join by
// k_query_list (their _min/_max are final only then), so none here.
// ===========================================================================
#ifndef GK_WG_WAVES
#define GK_WG_WAVES 8
#endif
#define GK_WG_T (64 * GK_WG_WAVES)
#define GK_WG_VPT ((GK_WG_PMAX + GK_WG_T - 1) / GK_WG_T)
#define GK_WG_KMAX ((GK_WG_CAP + GK_WG_T - 1) / GK_WG_T)  // table entries per thread

// s_waitcnt vmcnt(0) (expcnt / lgkmcnt left at their maxima; gfx9 encoding):
// every outstanding vector-memory load of the wave has returned
__device__ __forceinline__ void gk_wait_vmem() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// (g, d) pairs: a thread's two entries in one 16-byte read (separate g / d
// arrays: 0.85 ms more per cfg5 step, profiles/r05/r05B_*; value slots padded
// against the search probes' bank conflicts -- half the conflict cycles, but
// slower: 40.4 vs 38.4 ms).  The value buffers are GK_WG_TVN apart, not
// GK_WG_CAP: a table's slot j and the next table's slot j then fall on
// different banks (exactly 16 KiB apart: 38.95-39.0 vs 38.4-38.5 ms, r05C)
#define GK_WG_TVN (GK_WG_CAP + 68)
struct WgLDS {
  double tv[2][GK_WG_TVN];
  alignas(16) int2 tgd[2][GK_WG_CAP + 2];
  alignas(16) uint32_t gpk[2][GK_WG_CAP + 4];  // per gap: count, then (member base << 16) | out base; by table parity
  int32_t gk[GK_WG_CAP + 1];    // per entry: absorbed count | KEEP bit
  int32_t gdel[GK_WG_CAP + 1];  // per entry: G, then G + d - 1
  double sv[GK_WG_PMAX];        // sort area of a batch with a crowded gap
  uint32_t si[GK_WG_PMAX];
  double2 mem[GK_WG_PMAX];      // an unsorted batch's values by gap: (value, insertion index bits)
  uint32_t wsum[GK_WG_WAVES];   // the scan's wave totals
  int psflag_pub[2];            // k_ingest_wg: the presort-done flag thread 0 saw, by flush parity
  int32_t xdone[GK_WG_WAVES], xc[GK_WG_WAVES];  // the carry walk's wave-boundary states
  alignas(16) int32_t xall[GK_WG_WAVES];  // per wave: every lane's carry-in resolved (the walk's vote)
  alignas(16) int32_t xbig[GK_WG_WAVES];  // per wave: a gap with GK_WG_RANK_MAX members or more
  alignas(16) int32_t xcrowd[GK_WG_WAVES];  // per wave: a thread with > GK_WG_EMIT_MAX gap survivors
  uint32_t total;
  int go_ok;  // k_ingest_wg launched early: k_long_prep's word came in time
};
#ifndef GK_WG_GO_TICKS
#define GK_WG_GO_TICKS 100000000ull  // 1 s of s_memrealtime (100 MHz)
#endif

// The workgroup flush's value table in BFS (Eytzinger) order (GK_WG_EYTZ):
// sorted position j (0-based) of a table padded to 2^H - 1 entries lives at
// node (j + 1 + 2^H) >> (ctz(j + 1) + 1), the root at 1.  A search level's
// probes are then one contiguous row of nodes (2^l of them), so lanes with
// different values hit consecutive slots -- distinct LDS banks -- where the
// sorted layout's probes of a deep level are 2^(H-l) slots apart and share
// one bank (the 423 conflict cycles per wave and flush of round 5).
#ifndef GK_WG_EYTZ
#define GK_WG_EYTZ 1
#endif
__device__ __forceinline__ int wg_slot(int j, int H) {
#if GK_WG_EYTZ
  const int p1 = j + 1;
  return (p1 + (1 << H)) >> (__builtin_ctz((unsigned)p1) + 1);
#else
  (void)H;
  return j;
#endif
}
// tree height of a table of E entries: its padded size is pow2_above(E) - 1
__device__ __forceinline__ int wg_height(int E) { return 32 - __clz(E); }

// AND / OR over the workgroup of a per-wave flag (each wave's lane 0 has
// stored it in f[w] before a plain barrier): two 16-byte LDS reads, where
// __syncthreads_and / _or are a workgroup reduction with barriers of their own
static_assert(GK_WG_WAVES % 4 == 0, "per-wave flags are read as int4");
__device__ __forceinline__ int wg_flags_all(const int32_t* f) {
  int r = 1;
#pragma unroll
  for (int i = 0; i < GK_WG_WAVES; i += 4) {
    const int4 a = *(const int4*)(f + i);
    r &= a.x & a.y & a.z & a.w;
  }
  return r;
}
__device__ __forceinline__ int wg_flags_any(const int32_t* f) {
  int r = 0;
#pragma unroll
  for (int i = 0; i < GK_WG_WAVES; i += 4) {
    const int4 a = *(const int4*)(f + i);
    r |= a.x | a.y | a.z | a.w;
  }
  return r;
}

// values q = t + GK_WG_T * r of a batch of cnt in ascending (value, insertion
// index) order: Python's stable sorted() of gk:71-72
__device__ __forceinline__ void wg_sort(WgLDS& L, double (&xv)[GK_WG_VPT], int cnt, int t) {
  int N = 64;
  while (N < cnt) N <<= 1;
#pragma unroll
  for (int r = 0; r < GK_WG_VPT; ++r) {
    const int q = t + GK_WG_T * r;
    if (q < N) {
      L.sv[q] = q < cnt ? xv[r] : __longlong_as_double(0x7ff0000000000000LL);
      L.si[q] = q < cnt ? (uint32_t)q : 0xffffffffu;
    }
  }
  __syncthreads();
  for (int k = 2; k <= N; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int pp = t; pp < N / 2; pp += GK_WG_T) {
        const int a = ((pp & ~(j - 1)) << 1) | (pp & (j - 1));
        const int c = a + j;
        const double va = L.sv[a], vc = L.sv[c];
        const uint32_t ia = L.si[a], ic = L.si[c];
        const bool a_gt = (va > vc) || (!(va < vc) && ia > ic);
        if (a_gt == ((a & k) == 0)) {
          L.sv[a] = vc;
          L.sv[c] = va;
          L.si[a] = ic;
          L.si[c] = ia;
        }
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int r = 0; r < GK_WG_VPT; ++r) {
    const int q = t + GK_WG_T * r;
    xv[r] = q < cnt ? L.sv[q] : 0.0;
  }
  __syncthreads();
}

// One flush of a batch (value q of the batch in xv[r], q = t + GK_WG_T*r)
// into the table in buffer `cur`; the new table goes to cur^1.  A presorted
// batch (sorted: ascending (value, insertion index)) places value q at rank
// q - (its gap's first position); an unsorted one ranks each value among its
// gap's members (stored by gap in the sort area; gaps hold ~P/E values, ~1 for
// iid data), or, when some gap holds GK_WG_RANK_MAX or more, is sorted first.
// Returns the new size, or -1 if it would not fit GK_WG_CAP - 1 (nothing is
// written to the global table then; the caller promotes the stream).
#ifndef GK_WG_RANK_MAX
#define GK_WG_RANK_MAX 32
#endif
#ifndef GK_WG_RK_UNROLL
#define GK_WG_RK_UNROLL 4
#endif
// a sorted batch's gap survivors are stored by the thread of their entry
// (read from the sort area, GK_WG_EMIT_U per trip) unless some thread owns
// more than GK_WG_EMIT_MAX of them (crowded gaps: the per-gap records path)
#ifndef GK_WG_EMIT_MAX
#define GK_WG_EMIT_MAX 16
#endif
#ifndef GK_WG_EMIT_U
#define GK_WG_EMIT_U 4
#endif
// KM: table entries per thread, >= ceil(E / GK_WG_T) (2 up to 1024 entries)
template <int KM>
__device__ int flush_wg(WgLDS& L, const int cur, const int E, double (&xv)[GK_WG_VPT], const int cnt,
                        const int T, const int t, bool sorted) {
  const int lane = t & 63, w = t >> 6;
  const double* __restrict__ tv = L.tv[cur];
  const int2* __restrict__ tgd = L.tgd[cur];
  double* __restrict__ nv = L.tv[cur ^ 1];
  int2* __restrict__ ngd = L.tgd[cur ^ 1];
  // per-gap counts / bases: two buffers by table parity; this flush's was
  // zeroed during the previous one (or at stream setup), the other is zeroed
  // now for the next flush (no zeroing pass + barrier before the atomics)
  uint32_t* __restrict__ gpk = L.gpk[cur];
  {
    uint4* __restrict__ gz = (uint4*)L.gpk[cur ^ 1];
    for (int j = t; j < (GK_WG_CAP + 4) / 4; j += GK_WG_T) gz[j] = make_uint4(0u, 0u, 0u, 0u);
  }
  // this thread's block of entries for the carry walk below: their g, d (and
  // those of the entries either side) read now, under the search; only the
  // member counts wait for the atomics
  static_assert(KM >= 1 && KM <= GK_WG_KMAX, "entries per thread");
  const int K = (E + GK_WG_T - 1) / GK_WG_T;
  const int j0 = t * K;
  const int jend = min(j0 + K, E);
  const int nk = max(jend - j0, 0);
  const bool has = j0 < E;
  const int cs = T > 1 ? T : 1;
  const int tail_t = E == 0 ? 0 : (E - 1) / K;
  int eg[KM], ed[KM];
  {
    int2 gd[KM];
    if (K % 2 == 0) {  // (j0 even: 16-byte reads of two entries)
#pragma unroll
      for (int k = 0; k < KM; k += 2) {
        const int4 a = *(const int4*)&tgd[j0 + k];
        gd[k] = make_int2(a.x, a.y);
        if (k + 1 < KM) gd[k + 1] = make_int2(a.z, a.w);
      }
    } else {
#pragma unroll
      for (int k = 0; k < KM; ++k) gd[k] = tgd[j0 + k];
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const bool in = k < nk;
      eg[k] = in ? gd[k].x : 0;
      ed[k] = in ? gd[k].y : 0;
    }
  }
  const bool nx = has && jend < E;  // the entry after this block (the last entry's removal test)
  const int2 gdn = nx ? tgd[jend] : make_int2(0, 0);
  const int gnx = gdn.x, dnx = gdn.y;
  const int2 gdp = (has && t > 0) ? tgd[j0 - 1] : make_int2(0, 0);  // the entry before
  const int gp_ = gdp.x, dp_ = gdp.y;
  if (sorted) {  // the batch in order in the sort area, for the entry-side emit (a sort leaves it there too)
#pragma unroll
    for (int r = 0; r < GK_WG_VPT; ++r)
      if (t + GK_WG_T * r < cnt) L.sv[t + GK_WG_T * r] = xv[r];
  }
  GK_WMARK(1);  // setup: zeroing, the entries' g/d loads issued
  // ---- gap = #entries <= x (gk:93), branch-free over the +inf-padded table
  int xg[GK_WG_VPT];
  uint32_t slot[GK_WG_VPT];  // an unsorted value's member slot in its gap
  for (int pass = 0;; ++pass) {
#if GK_WG_EYTZ
    {
      const int H = wg_height(E);
#pragma unroll
      for (int r = 0; r < GK_WG_VPT; ++r) xg[r] = 1;
      for (int l = 0; l < H; ++l) {
        double tt[GK_WG_VPT];
#pragma unroll
        for (int r = 0; r < GK_WG_VPT; ++r) tt[r] = tv[xg[r]];
#pragma unroll
        for (int r = 0; r < GK_WG_VPT; ++r) xg[r] = 2 * xg[r] + ((tt[r] <= xv[r]) ? 1 : 0);
      }
#pragma unroll
      for (int r = 0; r < GK_WG_VPT; ++r) xg[r] = min(xg[r] - (1 << H), E);
    }
#else
#pragma unroll
    for (int r = 0; r < GK_WG_VPT; ++r) xg[r] = 0;
    for (int step = gk_pow2_above(E) >> 1; step > 0; step >>= 1) {
      double tt[GK_WG_VPT];
#pragma unroll
      for (int r = 0; r < GK_WG_VPT; ++r) tt[r] = tv[xg[r] + step - 1];
#pragma unroll
      for (int r = 0; r < GK_WG_VPT; ++r) xg[r] += (tt[r] <= xv[r]) ? step : 0;
    }
#pragma unroll
    for (int r = 0; r < GK_WG_VPT; ++r) xg[r] = min(xg[r], E);
#endif
    if (pass > 0) {  // (the re-search of a sorted batch: counts start over)
      for (int j = t; j <= E; j += GK_WG_T) gpk[j] = 0u;
      __syncthreads();
    }
    GK_WMARK(2);  // gap search
    bool big = false;
    if (sorted) {
      // (no slot needed: no-return atomics)
#pragma unroll
      for (int r = 0; r < GK_WG_VPT; ++r)
        if (t + GK_WG_T * r < cnt) (void)atomicAdd(&gpk[xg[r]], 1u);
    } else {
#pragma unroll
      for (int r = 0; r < GK_WG_VPT; ++r) {
        slot[r] = 0;
        if (t + GK_WG_T * r < cnt) {
          slot[r] = atomicAdd(&gpk[xg[r]], 1u);
          big |= slot[r] >= GK_WG_RANK_MAX;
        }
      }
    }
    if (sorted) {
      GK_WMARK(3);  // count atomics (issued)
      __syncthreads();
      GK_WMARK(4);  // count barrier (atomics drained + wait)
      break;
    }
    {
      const bool wbig = __builtin_amdgcn_ballot_w64(big) != 0;
      if (lane == 0) L.xbig[w] = wbig ? 1 : 0;
      __syncthreads();
      if (!wg_flags_any(L.xbig)) break;  // (xbig is written again only after the sort's barriers)
    }
    GK_BMARK(2);
    wg_sort(L, xv, cnt, t);  // a crowded gap: sort, then search again
    sorted = true;
    GK_BMARK(10);
  }
  GK_BMARK(2);

  // ---- carry walk (closed form of gk:93-106) -----------------------------
  // thread t owns entries [t*K, t*K+K) (K <= GK_WG_KMAX); their g, d and
  // member counts are read into registers once, so that a carry chain that
  // crosses many threads costs a few VALU per thread it crosses, not an LDS
  // round trip.  A thread's carry-in is known at once when its predecessor
  // entry is kept even at carry 0 (G grows with the carry); otherwise it
  // waits for its left neighbour: inside a wave over DPP, across waves through
  // LDS (one barrier per round; rounds are the longest chain of removed
  // entries crossing a wave boundary, usually none)
  int em[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) em[k] = k < nk ? (int)gpk[j0 + k] : 0;
  bool known = (t == 0) || !has;
  if (has && t > 0) {
    const int m = (int)gpk[j0 - 1];
    const int G0 = gp_ + clampi(T - dp_ - gp_, 0, m);
    known = !(G0 + eg[0] + ed[0] <= T);
  }
  bool done = !has;
  int cin = 0, cout = 0;
  int ek[KM], eG[KM];  // per entry: absorbed count | KEEP bit, G
#pragma unroll
  for (int k = 0; k < KM; ++k) ek[k] = eG[k] = 0;
  const int mEa = (int)gpk[E];            // the tail gap's members
  const int mE = t == tail_t ? mEa : 0;  // (counted by its thread)
  uint32_t v = 0, incl = 0;
#ifdef GK_PROF
  int prof_rounds = 0;  // DPP rounds of the carry walk (profiling builds: point 7 counts them)
#endif
  for (;;) {
    for (;;) {
#ifdef GK_PROF
      ++prof_rounds;
#endif
      if (known && !done) {
        int c = cin;
#pragma unroll
        for (int k = 0; k < KM; ++k) {
          if (k < nk) {
            const int Gp = eg[k] + c;
            const int kk = clampi(T - ed[k] - Gp, 0, em[k]);
            const int G = Gp + kk;
            const bool last = k + 1 >= nk;
            const int gn = last ? gnx : eg[k + 1 < KM ? k + 1 : k];
            const int dn = last ? dnx : ed[k + 1 < KM ? k + 1 : k];
            const bool rem = (!last || nx) && (G + gn + dn <= T);
            ek[k] = kk | (rem ? 0 : GK_KEEP_BIT);
            eG[k] = G;
            c = rem ? G : 0;
          }
        }
        cout = c;
        done = true;
      }
      const int pc = wave_shr1(cout, 0);
      const int pd = wave_shr1((int)done, 1);
      const bool nkn = !known && lane > 0 && pd;
      if (nkn) {
        known = true;
        cin = pc;
      }
      if (__builtin_amdgcn_ballot_w64(nkn) == 0) break;
    }
    // ---- output offsets: the wave scan of (members << 16 | outputs) of this
    //      round's results, published with the carry flags: when every
    //      carry is resolved (the common case, one round) the totals are
    //      final after this one barrier
    uint32_t sm = 0, so = 0;
    int ns = 0;  // gap survivors of this thread's entries
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k < nk) {
        const int m = em[k], kk = ek[k];
        sm += (uint32_t)m;
        so += (uint32_t)(m - (kk & ~GK_KEEP_BIT) + ((kk & GK_KEEP_BIT) ? 1 : 0));
        ns += m - (kk & ~GK_KEEP_BIT);
      }
    }
    if (t == tail_t) {
      sm += (uint32_t)mE;
      so += (uint32_t)((mE + cs - 1) / cs);
    }
    v = (sm << 16) | so;
    incl = wave_incl_scan_u32(v, lane);
    const bool wall = __builtin_amdgcn_ballot_w64(!done) == 0;
    const bool crowd = __builtin_amdgcn_ballot_w64(ns > GK_WG_EMIT_MAX) != 0;
    if (lane == 63) {
      L.xdone[w] = done ? 1 : 0;
      L.xc[w] = cout;
      L.xall[w] = wall ? 1 : 0;
      L.xcrowd[w] = crowd ? 1 : 0;
      L.wsum[w] = incl;
    }
    GK_WMARK(5);  // carry walk (counts read, DPP rounds) + sums + wave scan
    // (one barrier when no chain crosses a wave boundary: the common case)
    __syncthreads();
    const int cdone = wg_flags_all(L.xall);
    GK_WMARK(6);  // carry + scan barrier
#ifdef GK_PROF
    if ((t & 63) == 0) gk_wave_prof().acc[w][7] += (unsigned long long)prof_rounds * 1000ull;
    prof_rounds = 0;
#endif
    if (cdone) break;
    if (lane == 0 && w > 0 && !known && L.xdone[w - 1]) {
      known = true;
      cin = L.xc[w - 1];
    }
    __syncthreads();  // (xdone / xc / wsum are rewritten by the next round)
  }
  GK_BMARK(3);
  uint32_t pre = 0, total = 0;
#pragma unroll
  for (int k = 0; k < GK_WG_WAVES; ++k) {
    const uint32_t s = L.wsum[k];
    pre += k < w ? s : 0u;
    total += s;
  }
  const int newE = (int)(total & 0xffffu);
  if (newE > GK_WG_CAP - 1) return -1;  // (uniform: total comes from LDS) one slot stays free for the padding
  const int totm = (int)(total >> 16);
  const int Ho = wg_height(E), Hn = wg_height(newE);  // the old / new table's tree heights
  if (sorted && !wg_flags_any(L.xcrowd)) {
    // ---- entry-side emit (sorted, no crowded thread): each thread stores its
    //      entries' gap survivors (sorted positions member base + absorbed ..
    //      member base + m - 1, gk:93-99) and kept entries, flattened over its
    //      entries; the tail's values are stored by their own threads
    //      (gk:85-92).  No per-gap records and no placement barrier.
    uint32_t base = pre + incl - v;
    int soff[KM], doff[KM], sb[KM], dl[KM];
    int st_ = 0;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      soff[k] = doff[k] = dl[k] = 0;
      sb[k] = 1 << 30;
      if (k < nk) {
        const int j = j0 + k;
        const int m = em[k], kk = ek[k];
        const int ka = kk & ~GK_KEEP_BIT;
        const int ob = (int)(base & 0xffffu);
        if (kk & GK_KEEP_BIT) {
          const int pos = ob + m - ka;
          nv[wg_slot(pos, Hn)] = tv[wg_slot(j, Ho)];
          ngd[pos] = make_int2(eG[k], ed[k]);
        }
        sb[k] = st_;
        soff[k] = (int)(base >> 16) + ka - st_;
        doff[k] = ob - st_;
        dl[k] = eG[k] + ed[k] - 1;
        st_ += m - ka;
        base += ((uint32_t)m << 16) | (uint32_t)(m - ka + ((kk & GK_KEEP_BIT) ? 1 : 0));
      }
    }
    for (int o0 = 0; o0 < st_; o0 += GK_WG_EMIT_U) {
      double xs[GK_WG_EMIT_U];
      int dpos[GK_WG_EMIT_U], dd[GK_WG_EMIT_U];
#pragma unroll
      for (int u = 0; u < GK_WG_EMIT_U; ++u) {
        const int o = o0 + u;
        int so_ = soff[0], do_ = doff[0], dl_ = dl[0];
#pragma unroll
        for (int k = 1; k < KM; ++k)
          if (o >= sb[k]) {
            so_ = soff[k];
            do_ = doff[k];
            dl_ = dl[k];
          }
        xs[u] = L.sv[min(o + so_, GK_WG_PMAX - 1)];
        dpos[u] = o + do_;
        dd[u] = dl_;
      }
#pragma unroll
      for (int u = 0; u < GK_WG_EMIT_U; ++u) {
        if (o0 + u < st_) {
          nv[wg_slot(dpos[u], Hn)] = xs[u];
          ngd[dpos[u]] = make_int2(1, dd[u]);
        }
      }
    }
    const int mbE = totm - mEa, obE = newE - (mEa + cs - 1) / cs;
#pragma unroll
    for (int r = 0; r < GK_WG_VPT; ++r) {
      const int q = t + GK_WG_T * r;
      if (q < cnt && xg[r] == E) {
        const int rk = q - mbE;
        const int qq = rk / cs;
        const int rr = rk - qq * cs;
        if (rr == cs - 1 || rk == mEa - 1) {
          const int pos = obE + qq;
          nv[wg_slot(pos, Hn)] = xv[r];
          ngd[pos] = make_int2(rr + 1, 0);
        }
      }
    }
    const int hi = gk_pow2_above(newE) - 1;
    for (int j = newE + t; j < hi; j += GK_WG_T) nv[wg_slot(j, Hn)] = __longlong_as_double(0x7ff0000000000000LL);
    GK_WMARK(11);
    __syncthreads();
    GK_WMARK(12);
    GK_BMARK(6);
    return newE;
  }
  {
    uint32_t base = pre + incl - v;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k < nk) {
        const int j = j0 + k;
        const int m = em[k], kk = ek[k];
        const int ka = kk & ~GK_KEEP_BIT;
        const int G = eG[k];
        const int d = ed[k];
        gpk[j] = base;
        L.gk[j] = kk;
        L.gdel[j] = G + d - 1;
        if (kk & GK_KEEP_BIT) {
          const int pos = (int)(base & 0xffffu) + m - ka;
          nv[wg_slot(pos, Hn)] = tv[wg_slot(j, Ho)];
          ngd[pos] = make_int2(G, d);
        }
        base += ((uint32_t)m << 16) | (uint32_t)(m - ka + ((kk & GK_KEEP_BIT) ? 1 : 0));
      }
    }
    if (t == tail_t) gpk[E] = base;
  }
  GK_WMARK(9);  // wave totals, kept entries and per-gap records stored
  __syncthreads();
  GK_WMARK(10);  // placement barrier
  GK_BMARK(4);
  if (!sorted) {  // members by gap, in slot order
#pragma unroll
    for (int r = 0; r < GK_WG_VPT; ++r) {
      const int q = t + GK_WG_T * r;
      if (q < cnt) {
        const int pos = (int)(gpk[xg[r]] >> 16) + (int)slot[r];
        L.mem[pos] = make_double2(xv[r], __longlong_as_double((int64_t)q));
      }
    }
    __syncthreads();
  }
  GK_BMARK(5);

  // ---- the values: the rank inside a gap is the position minus the gap's
  //      member base when sorted, else the count of its members before it in
  //      (value, insertion index) order (gk:71-72); gk:93-99 for a gap before
  //      an entry, gk:85-92 for the tail: chunks of max(T,1), each emitting
  //      its last value
  uint32_t pkv[GK_WG_VPT];
  int rkv[GK_WG_VPT];
#pragma unroll
  for (int r = 0; r < GK_WG_VPT; ++r) {
    const int q = t + GK_WG_T * r;
    pkv[r] = q < cnt ? gpk[xg[r]] : 0u;
    rkv[r] = q - (int)(pkv[r] >> 16);
  }
  if (!sorted) {
    // both values' member lists walked side by side, one 16-byte read each
    int mb[GK_WG_VPT], mn[GK_WG_VPT], nmax = 0;
#pragma unroll
    for (int r = 0; r < GK_WG_VPT; ++r) {
      const int q = t + GK_WG_T * r;
      mb[r] = (int)(pkv[r] >> 16);
      mn[r] = q < cnt ? (xg[r] < E ? (int)(gpk[xg[r] + 1] >> 16) : totm) - mb[r] : 0;
      nmax = max(nmax, mn[r]);
      rkv[r] = 0;
    }
    // (GK_WG_RK_UNROLL members per value and trip: their reads are issued
    // together, the compares masked past the value's own members)
    for (int i = 0; i < nmax; i += GK_WG_RK_UNROLL) {
      double2 e[GK_WG_VPT][GK_WG_RK_UNROLL];
#pragma unroll
      for (int r = 0; r < GK_WG_VPT; ++r)
#pragma unroll
        for (int u = 0; u < GK_WG_RK_UNROLL; ++u) e[r][u] = L.mem[min(mb[r] + i + u, GK_WG_PMAX - 1)];
#pragma unroll
      for (int r = 0; r < GK_WG_VPT; ++r) {
        const double xq = xv[r];
        const int q = t + GK_WG_T * r;
#pragma unroll
        for (int u = 0; u < GK_WG_RK_UNROLL; ++u)
          rkv[r] += (i + u < mn[r] &&
                     (e[r][u].x < xq || (!(xq < e[r][u].x) && (int)__double_as_longlong(e[r][u].y) < q))) ? 1 : 0;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < GK_WG_VPT; ++r) {
    const int q = t + GK_WG_T * r;
    if (q < cnt) {
      const int gap = xg[r];
      const uint32_t pk = pkv[r];
      const int rk = rkv[r];
      if (gap < E) {
        const int k = L.gk[gap] & ~GK_KEEP_BIT;
        if (rk >= k) {
          const int pos = (int)(pk & 0xffffu) + rk - k;
          nv[wg_slot(pos, Hn)] = xv[r];
          ngd[pos] = make_int2(1, L.gdel[gap]);
        }
      } else {
        const int m = totm - (int)(pk >> 16);
        const int qq = rk / cs;
        const int rr = rk - qq * cs;
        if (rr == cs - 1 || rk == m - 1) {
          const int pos = (int)(pk & 0xffffu) + qq;
          nv[wg_slot(pos, Hn)] = xv[r];
          ngd[pos] = make_int2(rr + 1, 0);
        }
      }
    }
  }
  // +inf padding for the next search, up to pow2_above(newE) - 2
  const int hi = gk_pow2_above(newE) - 1;
  for (int j = newE + t; j < hi; j += GK_WG_T) nv[wg_slot(j, Hn)] = __longlong_as_double(0x7ff0000000000000LL);
  GK_WMARK(11);  // values: records read, survivors stored, padding
  __syncthreads();
  GK_WMARK(12);  // end barrier
  GK_BMARK(6);
  return newE;
}

#ifdef GK_TIMELINE
// timeline builds only: per workgroup of k_ingest_wg, s_memrealtime and
// s_memtime at its start and end, and its flushes (tools/launch_timeline.py)
__device__ unsigned long long gk_tl_wg[5 * GK_WG_MAX];
#endif
__global__ __launch_bounds__(GK_WG_T) void k_ingest_wg(GKState st, const double* __restrict__ x,
                                                       const int64_t* __restrict__ offs,
                                                       const int32_t* __restrict__ prio,
                                                       const int32_t* __restrict__ wg_count, int lcls, int force,
                                                       int32_t* __restrict__ ovf_count,
                                                       int32_t* __restrict__ ovf_list,
                                                       unsigned long long* __restrict__ work,
                                                       const double* __restrict__ psort,
                                                       const int64_t* __restrict__ prio_ws,
                                                       const int32_t* __restrict__ ps_done, int ps_grid,
                                                       int hi_prio, const int32_t* __restrict__ go) {
  __shared__ WgLDS L;
  if (hi_prio) __builtin_amdgcn_s_setprio(3);  // (GK_WG_PRIO: the critical chains win the SIMD's issue arbitration)
#ifdef GK_TIMELINE
  if (threadIdx.x == 0 && blockIdx.x < GK_WG_MAX) {
    gk_tl_wg[5 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    gk_tl_wg[5 * blockIdx.x + 1] = __builtin_amdgcn_s_memtime();
  }
#endif
  __shared__ int64_t item;
  // ps_done: the presort runs beside this launch; a presorted batch is used
  // only once every presort wave has finished (seen by thread 0 with a
  // relaxed load during one flush, published in LDS at its end, taken by all
  // threads after the next flush's barriers with an acquire load of their
  // own); before that batches are ranked unsorted.  Workgroup-uniform,
  // monotone.
  bool ps_ok = ps_done == nullptr;
  int fk = 0;  // flushes of this workgroup (the LDS slot parity)
  const int t = threadIdx.x;
  if (t == 0) L.psflag_pub[0] = L.psflag_pub[1] = 0;
  const int P = st.P;
  if (go) {
    // launched ahead of k_long_prep (the stream list, the presort plan and
    // this launch's stream count): wait for its word, then every thread
    // acquires it (the list was written on another CU).  Bounded: if the word
    // does not come within GK_WG_GO_TICKS (kernels serialised -- a profiler's
    // counter passes, AMD_SERIALIZE_KERNEL -- or no CU left for k_long_prep)
    // the workgroup leaves without taking a stream, and the launch the call
    // enqueues behind k_long_prep (gk_capi.cpp stats_fork) takes them all.
    if (t == 0) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      int ok = 1;
      while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > GK_WG_GO_TICKS) {
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(8);
      }
      L.go_ok = ok;
    }
    __syncthreads();
    if (!L.go_ok) return;  // (workgroup-uniform)
    (void)__hip_atomic_load(go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  }
  const int64_t K = *wg_count;
#ifdef GK_PROF
  if (t == 0) {
    for (int i = 0; i < GK_PROF_NSEC; ++i) gk_big_prof().acc[i] = 0;
    gk_big_prof().t = gk_cycles();
  }
  if ((t & 63) == 0 && (t >> 6) < GK_WP_W) {
    for (int i = 0; i < GK_WP_N; ++i) gk_wave_prof().acc[t >> 6][i] = 0;
    gk_wave_prof().t[t >> 6] = gk_cycles();
  }
#endif
  for (;;) {
    if (t == 0) item = (int64_t)atomicAdd(work, 1ull);
    __syncthreads();
    const int64_t wi = item;
    __syncthreads();  // (item is rewritten by the next grab)
    if (wi >= K) break;
    const int64_t s = prio[wi];
    const int32_t scls = st.cls[s];
    if (scls != lcls) continue;  // in another class: handled by that class's launch
    const int32_t sslot = st.slot[s];
    int p = st.pend[s];
    int E = st.E[s];
    int64_t n = st.n[s];
    const int64_t xo = offs[s];
    const int64_t Lx = offs[s + 1] - xo;
    const int64_t wso = prio_ws ? prio_ws[wi] : -1;
    if (Lx <= 0 && !((force == 1 && p > 0) || (force == 2 && n > 0))) continue;
    GKRec* __restrict__ tab = gk_table_ptr_cs(st, s, scls, sslot);
    double* __restrict__ pb = st.pbuf + s * (int64_t)st.pmax;
    bool ok = E <= GK_WG_CAP - 1 && P <= GK_WG_PMAX && gk_count_ok(st, n + (Lx > 0 ? Lx : 0));
    int cur = 0;
    if (ok) {
      const int H = wg_height(E);
      for (int j = t; j < E; j += GK_WG_T) {
        const GKRec rc = tab[j];
        L.tv[0][wg_slot(j, H)] = rc.v;
        L.tgd[0][j] = make_int2(rc.g, rc.d);
      }
      const int hi = gk_pow2_above(E) - 1;
      for (int j = E + t; j < hi; j += GK_WG_T) L.tv[0][wg_slot(j, H)] = __longlong_as_double(0x7ff0000000000000LL);
      for (int j = t; j <= GK_WG_CAP; j += GK_WG_T) L.gpk[0][j] = 0u;  // (flush_wg zeroes the other)
    }
    __syncthreads();
    int64_t used = 0;
    int64_t need = P - (n % P);  // adds until n hits the next multiple of P (gk:60)
    bool flushed = false;
    // presorted batch b of this call at psort + wso + b*P (k_presort)
    const double* __restrict__ sb = wso >= 0 ? psort + wso : nullptr;
    double xv[GK_WG_VPT];
    // the next batch is loaded one flush ahead (its HBM latency under the
    // current flush); xn holds it
    double xn[GK_WG_VPT];
    bool have_next = false, next_sorted = false;
    GK_BMARK(0);
    while (ok && used + need <= Lx) {
      const int cnt = p + (int)need;
      bool cur_sorted;
      int pf = 0;
      if (have_next) {
#pragma unroll
        for (int r = 0; r < GK_WG_VPT; ++r) xv[r] = xn[r];
        cur_sorted = next_sorted;
#ifdef GK_PROF
        // (profiling builds: point 13 = the wait for the prefetched batch)
        __builtin_amdgcn_s_waitcnt(0x0F70);
        GK_WMARK(13);
#endif
      } else if (sb && ps_ok && (flushed || !ps_done)) {
        // (beside the presort, batch 0 is never sorted: k_presort_reg)
        cur_sorted = true;
#pragma unroll
        for (int r = 0; r < GK_WG_VPT; ++r) {
          const int q = t + GK_WG_T * r;
          xv[r] = q < cnt ? sb[q] : 0.0;
        }
      } else {
        cur_sorted = false;
#pragma unroll
        for (int r = 0; r < GK_WG_VPT; ++r) {
          const int q = t + GK_WG_T * r;
          xv[r] = q < cnt ? (q < p ? pb[q] : x[xo + used + (q - p)]) : 0.0;
        }
      }
      n += need;
      // this batch's loads (if any) complete here, BEFORE the prefetch is
      // issued: the flush's first use of xv would otherwise wait (vmcnt(0):
      // the compiler cannot count loads over the three paths above) for the
      // next batch's loads as well, a full memory latency per flush
      gk_wait_vmem();
      // prefetch: the next automatic flush's batch (P values: presorted at
      // sb + P, or the call's next P values)
      have_next = used + need + P <= Lx;
      next_sorted = sb != nullptr && ps_ok;
      if (have_next) {
#pragma unroll
        for (int r = 0; r < GK_WG_VPT; ++r) {
          const int q = t + GK_WG_T * r;
          xn[r] = q < P ? (next_sorted ? sb[P + q] : x[xo + used + need + q]) : 0.0;
        }
      }
      // (after the prefetch: read after the flush)
      if (t == 0 && !ps_ok) pf = __hip_atomic_load(ps_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      GK_BMARK(1);
      GK_WMARK(0);  // between flushes: batch loads, flags
      const int nE = E <= 2 * GK_WG_T ? flush_wg<2>(L, cur, E, xv, cnt, gk_threshold(st, n), t, cur_sorted)
                                      : flush_wg<GK_WG_KMAX>(L, cur, E, xv, cnt, gk_threshold(st, n), t, cur_sorted);
      if (!ps_ok) {
        // the flag thread 0 saw at the start of the previous flush (published
        // before this flush's barriers); this flush's reading for the next one
        if (L.psflag_pub[fk & 1]) {
          // (every thread's own acquire of the finished count: the presort's
          // stores are visible to its later loads; the count only grows, so
          // all threads agree)
          ps_ok = __hip_atomic_load(ps_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= ps_grid;
        }
        if (t == 0) L.psflag_pub[(fk + 1) & 1] = pf >= ps_grid;
      }
      ++fk;
      if (nE < 0) {
        ok = false;
        break;
      }
      E = nE;
      cur ^= 1;
      used += need;
      p = 0;
      need = P;
      flushed = true;
      if (sb) sb += P;  // batch b at wso + b*P (k_presort)
      GK_BMARK(7);
    }
    (void)flushed;
    if (ok) {
      const int64_t rem = Lx - used;  // < need: no automatic flush for these
      if ((force == 1 && p + rem > 0) || force == 2) {
        const int cnt = p + (int)rem;
#pragma unroll
        for (int r = 0; r < GK_WG_VPT; ++r) {
          const int q = t + GK_WG_T * r;
          xv[r] = q < cnt ? (q < p ? pb[q] : x[xo + used + (q - p)]) : 0.0;
        }
        n += rem;
        const int nE = E <= 2 * GK_WG_T ? flush_wg<2>(L, cur, E, xv, cnt, gk_threshold(st, n), t, false)
                                        : flush_wg<GK_WG_KMAX>(L, cur, E, xv, cnt, gk_threshold(st, n), t, false);
        if (nE < 0) {
          ok = false;
        } else {
          E = nE;
          cur ^= 1;
          p = 0;
        }
      } else {
        for (int64_t i = t; i < rem; i += GK_WG_T) pb[p + i] = x[xo + used + i];
        p += (int)rem;
        n += rem;
      }
    }
    if (!ok) {
      // nothing written back: the stream keeps its pre-call state and is
      // re-run in the next capacity class
      if (t == 0) {
        const int k = atomicAdd(ovf_count, 1);
        ovf_list[k] = (int32_t)s;
      }
      __syncthreads();
      continue;
    }
    const int Hw = wg_height(E);
    for (int j = t; j < E; j += GK_WG_T) {
      GKRec rc;
      rc.v = L.tv[cur][wg_slot(j, Hw)];
      const int2 gd = L.tgd[cur][j];
      rc.g = gd.x;
      rc.d = gd.y;
      tab[j] = rc;
    }
    if (t == 0) {
      st.n[s] = n;
      st.E[s] = E;
      st.pend[s] = p;
    }
    __syncthreads();
    GK_BMARK(9);
  }
#ifdef GK_PROF
  if (t == 0)
    for (int i = 0; i < GK_PROF_NSEC; ++i) atomicAdd(&gk_prof_acc[i], gk_big_prof().acc[i]);
  if ((t & 63) == 0 && (t >> 6) < GK_WP_W)
    for (int i = 0; i < GK_WP_N; ++i) atomicAdd(&gk_wprof_acc[t >> 6][i], gk_wave_prof().acc[t >> 6][i]);
#endif
#ifdef GK_TIMELINE
  if (t == 0 && blockIdx.x < GK_WG_MAX) {
    gk_tl_wg[5 * blockIdx.x + 2] = __builtin_amdgcn_s_memrealtime();
    gk_tl_wg[5 * blockIdx.x + 3] = __builtin_amdgcn_s_memtime();
    gk_tl_wg[5 * blockIdx.x + 4] = (unsigned long long)fk;
  }
#endif
}

// ===========================================================================
// k_ingest_big: the add-driven flush (gk:49-109) with no size limit -- the
// class for tables beyond 32768 entries and, for eps < 1/1023 (flush period
// P > 1024), every class.  Same stream loop and closed form as k_ingest, but
// nothing lives in registers or in 16-bit fields: one wave per stream works
// in a per-block global workspace (BigBuf) of `cap` entries and NP >= P values.
// Per flush the batch (pending values, then the call's values, in insertion
// order) is sorted by (value, insertion index) -- Python's stable sorted() of
// gk:71-72 -- with a wave bitonic sort; A_j = #{values < v_j} splits it into
// gaps (gap j = sorted positions [A_{j-1}, A_j): gk:93 puts a value equal to an
// entry after it); then the carry walk and the emit of flush_wave in 32/64-bit
// arithmetic.  T = floor(2 eps (n-1)) stays exact: a stream whose count would
// take T past GK_T_CLAMP is refused before any work (GK_CTR_FATAL).
// ===========================================================================
struct BigBuf {
  double* tv[2];
  int32_t* tg[2];
  int32_t* td[2];
  int32_t* ga;    // [cap+1] A_j: sorted values below entry j
  int32_t* gk;    // [cap+1] absorbed count k | KEEP bit
  int32_t* gG;    // [cap+1] G, then the delta G + d - 1 of emitted gap values
  uint32_t* gob;  // [cap+1] first output position of gap j (j == E: the tail)
  double* mv;     // [NP] the batch: values, sorted in place
  uint32_t* mi;   //      their insertion index
};

// sort slots of the batch: a power of two >= 2P (a flush takes p + need <= P
// values of a consistent state; an imported one may hold up to P-1 pending
// values more, which must not run past the buffer)
__host__ __device__ inline int gk_big_np(int P) {
  int n = 64;
  while (n < 2 * P) n <<= 1;
  return n;
}

__host__ __device__ inline size_t gk_big_ws_bytes_dev(int cap, int P) {
  const size_t np = (size_t)gk_big_np(P);
  const size_t b = (2 * (size_t)cap + np) * 8 + (4 * (size_t)cap + 4 * ((size_t)cap + 1) + np) * 4;
  return (b + 255) & ~(size_t)255;
}

__device__ inline BigBuf big_buf(unsigned char* base, int cap, int np) {
  BigBuf b;
  double* dp = (double*)base;
  b.tv[0] = dp; dp += cap;
  b.tv[1] = dp; dp += cap;
  b.mv = dp; dp += np;
  int32_t* ip = (int32_t*)dp;
  b.tg[0] = ip; ip += cap;
  b.tg[1] = ip; ip += cap;
  b.td[0] = ip; ip += cap;
  b.td[1] = ip; ip += cap;
  b.ga = ip; ip += cap + 1;
  b.gk = ip; ip += cap + 1;
  b.gG = ip; ip += cap + 1;
  b.gob = (uint32_t*)ip; ip += cap + 1;
  b.mi = (uint32_t*)ip;
  return b;
}

// One flush of the `cnt` values in B.mv / B.mi (insertion order) into the
// table in buffer `cur` (E entries).  Returns the new size (table in buffer
// cur^1), or -1 if it would exceed cap-1 (nothing written to the table).
__device__ int big_flush(const BigBuf& B, const int cap, const int cur, const int E, const int cnt, const int T,
                         const int lane) {
  const double* __restrict__ tv = cur ? B.tv[1] : B.tv[0];
  const int32_t* __restrict__ tg = cur ? B.tg[1] : B.tg[0];
  const int32_t* __restrict__ td = cur ? B.td[1] : B.td[0];
  double* __restrict__ nv = cur ? B.tv[0] : B.tv[1];
  int32_t* __restrict__ ng = cur ? B.tg[0] : B.tg[1];
  int32_t* __restrict__ nd = cur ? B.td[0] : B.td[1];
  double* __restrict__ mv = B.mv;
  uint32_t* __restrict__ mi = B.mi;

  // ---- stable order of the batch (gk:71-72) ---------------------------------
  int N = 1;
  while (N < cnt) N <<= 1;
  for (int i = cnt + lane; i < N; i += 64) {
    mv[i] = __longlong_as_double(0x7ff0000000000000LL);
    mi[i] = 0xffffffffu;  // after every real value, +inf included
  }
  wsync<true>();
  for (int k = 2; k <= N; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int pp = lane; pp < N / 2; pp += 64) {
        const int i = ((pp & ~(j - 1)) << 1) | (pp & (j - 1));
        const int l = i + j;
        const double a = mv[i], b = mv[l];
        const uint32_t pa = mi[i], pb = mi[l];
        const bool a_gt = (a > b) || (a == b && pa > pb);
        if (a_gt == ((i & k) == 0)) {
          mv[i] = b;
          mv[l] = a;
          mi[i] = pb;
          mi[l] = pa;
        }
      }
      wsync<true>();
    }
  }
  // ---- gap boundaries: A_j = #{sorted values < v_j} --------------------------
  for (int j = lane; j < E; j += 64) {
    const double t = tv[j];
    int lo = 0, hi = cnt;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (mv[mid] < t) lo = mid + 1;
      else hi = mid;
    }
    B.ga[j] = lo;
  }
  wsync<true>();
  auto gap_m = [&](int j) -> int { return B.ga[j] - (j ? B.ga[j - 1] : 0); };

  // ---- carry walk (closed form of gk:93-106, see flush_wave) -----------------
  const int K = (E + 63) >> 6;
  const int j0 = lane * K;
  const int jend = min(j0 + K, E);
  const bool has = j0 < E;
  const int64_t T64 = T;
  const int cs = T > 1 ? T : 1;
  const int tail_lane = E == 0 ? 0 : (E - 1) / K;
  bool known = (lane == 0) || !has;
  if (has && lane > 0) {
    const int jp = j0 - 1;
    const int64_t g = tg[jp], d = td[jp];
    const int64_t G0 = g + min(max(T64 - d - g, (int64_t)0), (int64_t)gap_m(jp));
    known = !(G0 + tg[j0] + td[j0] <= T64);
  }
  bool done = !has;
  int64_t cin = 0, cout = 0;
  for (;;) {
    if (known && !done) {
      int64_t c = cin;
      for (int j = j0; j < jend; ++j) {
        const int64_t g = tg[j], d = td[j];
        const int m = gap_m(j);
        const int64_t Gp = g + c;
        const int k = (int)min(max(T64 - d - Gp, (int64_t)0), (int64_t)m);
        const int64_t G = Gp + k;
        const bool rem = (j + 1 < E) && (G + tg[j + 1] + td[j + 1] <= T64);
        B.gk[j] = k | (rem ? 0 : GK_KEEP_BIT);
        B.gG[j] = (int32_t)G;
        c = rem ? G : 0;
      }
      cout = c;
      done = true;
    }
    int64_t pc = __shfl_up(cout, 1, 64);
    const int pd = wave_shr1((int)done, 1);
    if (!known && pd) {
      known = true;
      cin = pc;
    }
    if (__all(done)) break;
  }
  // ---- output positions (a wave scan of the per-lane counts), kept entries --
  uint32_t so = 0;
  for (int j = j0; j < jend; ++j) {
    const int kk = B.gk[j];
    so += (uint32_t)(gap_m(j) - (kk & ~GK_KEEP_BIT) + ((kk & GK_KEEP_BIT) ? 1 : 0));
  }
  const int tb = E ? B.ga[E - 1] : 0;  // first sorted position of the tail
  const int mE = cnt - tb;
  if (lane == tail_lane) so += (uint32_t)((mE + cs - 1) / cs);
  const uint32_t incl = wave_incl_scan_u32(so, lane);
  const int newE = __builtin_amdgcn_readlane((int)incl, 63);
  if (newE > cap - 1) return -1;  // (uniform)
  uint32_t base = incl - so;
  for (int j = j0; j < jend; ++j) {
    const int m = gap_m(j);
    const int kk = B.gk[j];
    const int k = kk & ~GK_KEEP_BIT;
    const int G = B.gG[j];
    const int d = td[j];
    B.gob[j] = base;
    B.gG[j] = G + d - 1;
    if (kk & GK_KEEP_BIT) {
      const uint32_t pos = base + (uint32_t)(m - k);
      nv[pos] = tv[j];
      ng[pos] = G;
      nd[pos] = d;
    }
    base += (uint32_t)(m - k + ((kk & GK_KEEP_BIT) ? 1 : 0));
  }
  if (lane == tail_lane) B.gob[E] = base;
  wsync<true>();
  // ---- the batch values: R3 false branch in the gaps, R2 chunks in the tail --
  for (int q = lane; q < cnt; q += 64) {
    const double x = mv[q];
    int lo = 0, hi = E;  // gap j = #{j' : A_j' <= q}
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (B.ga[mid] <= q) lo = mid + 1;
      else hi = mid;
    }
    const int j = lo;
    if (j < E) {
      const int rk = q - (j ? B.ga[j - 1] : 0);
      const int k = B.gk[j] & ~GK_KEEP_BIT;
      if (rk >= k) {
        const uint32_t pos = B.gob[j] + (uint32_t)(rk - k);
        nv[pos] = x;
        ng[pos] = 1;
        nd[pos] = B.gG[j];
      }
    } else {
      const int rk = q - tb;
      const int qq = rk / cs;
      const int rr = rk - qq * cs;
      if (rr == cs - 1 || rk == mE - 1) {
        const uint32_t pos = B.gob[E] + (uint32_t)qq;
        nv[pos] = x;
        ng[pos] = rr + 1;
        nd[pos] = 0;
      }
    }
  }
  wsync<true>();
  return newE;
}

// The batch of a flush into B.mv / B.mi: p pending values, then c - p values of x.
__device__ __forceinline__ void big_load(const BigBuf& B, const double* __restrict__ pb, int p,
                                         const double* __restrict__ xs, int c, int lane) {
  for (int i = lane; i < c; i += 64) {
    B.mv[i] = i < p ? pb[i] : xs[i - p];
    B.mi[i] = (uint32_t)i;
  }
  wsync<true>();
}

// Arguments as k_ingest (CAP == 0); `ctr`: the set's device counters
// (GK_CTR_FATAL: streams over the per-stream count limit).
__global__ __launch_bounds__(64) void k_ingest_big(GKState st, const double* __restrict__ x,
                                                   const int64_t* __restrict__ offs,
                                                   const int32_t* __restrict__ list, int64_t count,
                                                   const int32_t* __restrict__ count_ptr, int lcls, int force,
                                                   int cap, unsigned char* ws, size_t ws_bytes,
                                                   int32_t* __restrict__ ovf_count, int32_t* __restrict__ ovf_list,
                                                   const double* __restrict__ qs, int nq,
                                                   double* __restrict__ qout, int qmode,
                                                   unsigned long long* __restrict__ work, int32_t* __restrict__ ctr) {
  const int lane = threadIdx.x;
  const int P = st.P;
  const BigBuf B = big_buf(ws + (size_t)blockIdx.x * ws_bytes, cap, gk_big_np(P));
  if (count_ptr) count = *count_ptr;
  if ((int64_t)blockIdx.x >= count) return;  // (the blocks below the count take every item)
  for (;;) {
    unsigned long long wv = 0;
    if (lane == 0) wv = atomicAdd(work, 1ull);
    const int64_t w = rfl64((int64_t)wv);
    if (w >= count) break;
    const int64_t s = list ? (int64_t)list[w] : w;
    if (__builtin_amdgcn_readfirstlane(st.cls[s]) != lcls) continue;  // in another class
    int p = __builtin_amdgcn_readfirstlane(st.pend[s]);
    int E = __builtin_amdgcn_readfirstlane(st.E[s]);
    int64_t n = rfl64(st.n[s]);
    // a promoted stream continues from value n - n0 of the call (the flushes
    // its smaller class made before overflowing are committed: k_ingest_small)
    const int64_t xo = rfl64(offs[s]) + ((lcls > 0 && x) ? n - rfl64(st.n0[s]) : 0);
    const int64_t Lx = rfl64(offs[s + 1]) - xo;
    if (Lx <= 0 && !((force == 1 && p > 0) || (force == 2 && n > 0)) && !qs) continue;
    // a stream past the per-stream count limit is refused like an overflow,
    // but counted as fatal (no class can take it)
    const bool over = !gk_count_ok(st, n + (Lx > 0 ? Lx : 0));
    const double smn = st.mn[s], smx = st.mx[s];
    GKRec* __restrict__ tab = gk_table_ptr(st, s);
    double* __restrict__ pb = st.pbuf + s * (int64_t)st.pmax;
    bool ok = !over && E <= cap - 1;
    if (ok) {
      for (int j = lane; j < E; j += 64) {
        const GKRec rc = tab[j];
        B.tv[0][j] = rc.v;
        B.tg[0][j] = rc.g;
        B.td[0][j] = rc.d;
      }
    }
    wsync<true>();
    int cur = 0;
    int64_t used = 0;
    int64_t need = P - (n % P);  // adds until n hits the next multiple of P (gk:60)
    while (ok && used + need <= Lx) {
      big_load(B, pb, p, x + xo + used, p + (int)need, lane);
      n += need;
      const int nE = big_flush(B, cap, cur, E, p + (int)need, gk_threshold(st, n), lane);
      if (nE < 0) {
        ok = false;
        break;
      }
      E = nE;
      cur ^= 1;
      used += need;
      p = 0;
      need = P;
    }
    if (ok) {
      const int64_t rem = Lx - used;  // < need: no automatic flush for these
      if ((force == 1 && p + rem > 0) || force == 2) {
        big_load(B, pb, p, rem > 0 ? x + xo + used : pb, p + (int)rem, lane);
        n += rem;
        const int nE = big_flush(B, cap, cur, E, p + (int)rem, gk_threshold(st, n), lane);
        if (nE < 0) {
          ok = false;
        } else {
          E = nE;
          cur ^= 1;
          p = 0;
        }
      } else {
        for (int64_t i = lane; i < rem; i += 64) pb[p + i] = x[xo + used + i];
        p += (int)rem;
        n += rem;
      }
    }
    if (!ok) {
      // nothing was written back: the stream keeps its pre-call state and is
      // re-run after promotion to the next capacity class (or, past the count
      // limit, reported: GK_CTR_FATAL)
      if (lane == 0) {
        if (over) {
          atomicAdd(&ctr[GK_CTR_FATAL], 1);
          atomicMax(&ctr[GK_CTR_FATAL + 1], (int)s);
        } else {
          const int k = atomicAdd(ovf_count, 1);
          ovf_list[k] = (int32_t)s;
        }
      }
      wsync<true>();
      continue;
    }
    const double* fv = cur ? B.tv[1] : B.tv[0];
    const int32_t* fg = cur ? B.tg[1] : B.tg[0];
    const int32_t* fd = cur ? B.td[1] : B.td[0];
    if (qs) wave_quantiles<1, 1>(fv, fg, fd, E, n, smn, smx, st, qs, nq, qmode, qout + s * (int64_t)nq, lane);
    for (int j = lane; j < E; j += 64) {
      GKRec rc;
      rc.v = fv[j];
      rc.g = fg[j];
      rc.d = fd[j];
      tab[j] = rc;
    }
    if (lane == 0) {
      st.n[s] = n;
      st.E[s] = E;
      st.pend[s] = p;
    }
    wsync<true>();
  }
}

// ===========================================================================
// k_ingest_small: k_ingest for the small LDS class (E <= SMALL_CAP-1 entries,
// P <= 128), which holds every stream at eps >= 1/127 until its table
// outgrows the class.  Same algorithm as flush_wave, laid out for the
// instruction and LDS budget of a flush of ~100 values:
//  * the table is structure-of-arrays in LDS: values `tv` (8 B) and (g, d)
//    pairs `tgd` (8 B).  The value array is bank-padded: logical slot i lives
//    at i + i/32.  The probes of one binary-search level are the slots
//    S-1 + 2S*m, which without padding all share i mod 32 for S >= 32 (and
//    crowd onto 2-8 banks below), i.e. up to 32-way LDS bank conflicts; with
//    the padding every level's probes fall on distinct banks.  The padded
//    base of a search only changes by S + S/32, so every probe is still an
//    LDS load with an immediate offset;
//  * K (entries per lane) is a compile-time 2 or 4 (4 only when the class
//    holds more than 127 entries), so a lane's entries live in registers
//    without per-entry branches (reads past E stay inside the arrays and are
//    masked);
//  * the gap search is unrolled from the table's power-of-two size (a switch
//    that falls through);
//  * divisions by the tail chunk size max(T,1) are multiplications;
//  * quantiles are answered from registers: a lane's K running maxima of
//    prefix(g) + d - 1, one ballot + popcount per entry slot and quantile.
// ===========================================================================
#define SMALL_CAP GK_SMALL_CAP
// values of one stream in one call that k_ingest_small takes (32-bit call
// counters; the flush plan's (f + 63) * P stays below 2^31)
#define GK_SMALL_LX_MAX (((int64_t)1 << 31) - ((int64_t)1 << 15))
// Round-4 variants of the small class were measured on MI355X and removed
// ((g, d) packed in 32 bits, T one flush ahead, selective
// count zeroing, masked in-gap rank reads, every batch register-sorted).
#ifndef GK_SMALL_WAVES
// min waves per SIMD asked of the register allocator: 7 (72 VGPRs) since
// round 6 -- the round-6 flush fits without a spill inside the flush loop
// (the few left are per stream and per stats batch), and the seventh wave
// hides latency: cfg3 launch 5.54 -> 5.35 ms (profiles/r06/r07a_*; round 2's
// 7-wave build spilled in the flush and lost)
#define GK_SMALL_WAVES 7
#endif
// largest gap handled by the in-gap rank loop; larger gaps rank by counting
#ifndef GK_SMALL_RANK_MAX
#define GK_SMALL_RANK_MAX 16
#endif
// Compiler-only barrier between two LDS accesses: keeps adjacent 8-byte
// reads as separate ds_read_b64 (2 LDS cycles each, banks over 64 dwords)
// instead of one ds_read2_b64 (8 cycles, 32 banks; MI355X_MICROARCH.md LDS
// table).  Emits no instruction and no wait.
__device__ __forceinline__ void gk_lds_order() { __asm__ volatile("" ::: "memory"); }

// LDS attribution builds only (-DGK_DUP=mask; scripts/lds_attrib.sh): group g
// of the flush's LDS accesses is issued a second time -- reads through a
// volatile pointer, stores with the same data to the same address -- so the
// SQ_LDS_* counter deltas against the product build price that group alone.
// Results are unchanged.  Never set in the product library.
#ifndef GK_DUP
#define GK_DUP 0
#endif
#define GK_DUPG(g) ((GK_DUP >> (g)) & 1)
template <typename T>
__device__ __forceinline__ void dup_ld(const T* p) {
  const uint32_t a = (uint32_t)(uintptr_t)p;  // LDS byte address
  if constexpr (sizeof(T) == 16) {
    __attribute__((ext_vector_type(4))) uint32_t w;
    __asm__ volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(a) : "memory");
  } else if constexpr (sizeof(T) == 8) {
    __attribute__((ext_vector_type(2))) uint32_t w;
    __asm__ volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(a) : "memory");
  } else {
    uint32_t w;
    __asm__ volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(a) : "memory");
  }
}
template <typename T>
__device__ __forceinline__ void dup_st(T* p, T v) {
  static_assert(sizeof(T) == 8, "8-byte stores only");
  unsigned long long u;
  __builtin_memcpy(&u, &v, 8);
  *(volatile unsigned long long*)p = u;
}

// padded index of logical table slot i in the value array
__device__ __forceinline__ int pidx(int i) { return i + (i >> 5); }
#define SMALL_TVN (SMALL_CAP + (SMALL_CAP >> 5) + 4)

// Section profiler (profiling builds only, -DGK_PROF; tools/prof_sections.py):
// lane 0 adds the s_memtime delta since the previous mark to a per-block
// LDS counter; the block adds its counters to gk_prof_acc when it ends.

// Gaps are indexed by the PADDED slot of their entry (pidx(j), j = 0..E): the
// gap search yields that index directly, so it addresses the counts and the
// per-gap records without a conversion.  Padded slots 32, 65, 98 (i % 33 ==
// 32) are never a gap.  Conditional LDS stores of the flush are branch-free:
// a lane with nothing to store writes to a slot nobody reads (GK_SMALL_TRASH
// in tv/tgd, the lane's own word past the counts, the last mv slot), which
// spares the exec-mask save / restore / branch of every divergent store.
// (One shared slot is right: stores of one address from several lanes of a
// group merge, while a slot per lane -- tried, GK_TRASH_LANES in round 3 --
// lands on the live stores' banks: +14% bank-conflict cycles, no gain;
// profiles/r03q_trash_slots_ab.txt.)
#define GK_SMALL_TRASH (SMALL_CAP + 1)  // logical slot: tv[pidx(129)], tgd[129]
static_assert(SMALL_CAP == 128, "k_ingest_small is laid out for the 128-entry class (K = 2 entries per lane)");
template <int VPL>
struct SmallLDS {
  // first, at LDS address 0: the rank loop's reads of mv take their offsets
  // as ds_read2_b64 immediates
  alignas(16) double mv[64 * VPL + 64 + 2];  // values grouped by gap, +inf after the last; [last] trash
  alignas(16) double tv[SMALL_TVN];        // entry values at pidx(i); +inf from E up to E+63 (<= 127)
  alignas(16) int2 tgd[SMALL_CAP + 2];     // entry (g, d) at i; [j0+2] read as successor; [129] trash
  union {
    // per gap (padded index): first the member count (.x, the count atomics),
    // then the record (m<<24 | k<<16 | member base<<8 | out base, G+d-1)
    alignas(16) int2 gi[SMALL_TVN];
    // exact rank pass: a member's insertion index; [last] trash.  It shares
    // the records' bytes: the values hold their records in registers by then,
    // and the records are reset (zeroed) after the pass.
    int32_t mi[64 * VPL + 2];
  };
#ifdef GK_PROF
  unsigned long long prof[GK_PROF_NSEC];
  uint32_t prof_t;
#endif
};

// gap counters of the next flush (gi[].x, read and written only inside a
// flush): padded indices 0 .. pidx(127) = 130 of the SMALL_TVN = 136 records
static_assert(SMALL_CAP + (SMALL_CAP >> 5) + 4 == 136, "gi zeroing covers 136 records");
static_assert(sizeof(int32_t) * (64 * 2 + 2) <= sizeof(int2) * 136, "mi fits in the records");
// (The zero is made at each use: hoisted out of the stream loop, the compiler
// keeps a 4-VGPR zero alive across the flush and, short of registers, spills
// it -- its reload's vmcnt wait then stalls on the in-flight LDS-DMA.)
__device__ __forceinline__ void small_zero_counts(int2* gi, int lane) {
  // two v_mov_b64 (a 4-VGPR zero for the 16-byte store, its low half for the
  // 8-byte one), not one v_mov_b32 and five copies
  typedef uint32_t gk_v4u __attribute__((ext_vector_type(4)));
  gk_v4u z;
  __asm__ volatile("v_mov_b64 %0, 0" : "=v"(z.xy));
  __asm__ volatile("v_mov_b64 %0, 0" : "=v"(z.zw));
  // (lane & 7 made opaque: hoisted out of the stream loop, its address was
  // spilled at 8 waves per SIMD and reloaded from scratch every flush)
  int l7 = lane & 7;
  __asm__ volatile("" : "+v"(l7));
  ((gk_v4u*)gi)[lane] = z;                          // records 0..127
  ((uint2*)gi)[128 + l7] = make_uint2(z.x, z.y);  // records 128..135
}

__device__ __forceinline__ void small_pad(double* tv, int E, int lane) {
  // the gap search always runs its 7 levels (first probe: slot 63); slots
  // E .. E+63 (clamped to 127, which never holds an entry) are +inf, so every
  // probe it makes at or above E reads +inf (for E <= 63 it never passes
  // slot 63 unless x is +inf, whose gap is clamped to E)
  tv[pidx(min(E + lane, SMALL_CAP - 1))] = __longlong_as_double(0x7ff0000000000000LL);
}

// a / cs for 0 <= a < 256, cs = max(T,1) >= 1, in two full-rate VALU ops:
// (a * m) >> 23 with m = ceil(2^23 / cs) (a 24-bit operand: v_mul_u32_u24).
// Exact: m*cs = 2^23 + e with 0 <= e < cs, so a*m / 2^23 = a/cs + a*e/(cs 2^23)
// and a*e < 2^16 < 2^23 keeps the floor; cs == 1: m = 2^23 gives a;
// cs >= 256: m = 1 gives 0 = a / cs.
struct CsDiv {
  int cs;
  uint32_t m;
  __device__ __forceinline__ int div(int a) const { return (int)(__umul24((uint32_t)a, m) >> 23); }
  // a - (a / cs) * cs (q * cs: q = 0 whenever cs >= 2^24)
  __device__ __forceinline__ int rem(int a, int q) const { return a - (int)__umul24((uint32_t)q, (uint32_t)cs); }
};

struct CsMagicTable {
  uint32_t m[256];
  constexpr CsMagicTable() : m() {
    for (uint32_t c = 1; c < 256; ++c) m[c] = ((1u << 23) + c - 1u) / c;
  }
};
__constant__ CsMagicTable gk_cs_magic = CsMagicTable();

__device__ __forceinline__ CsDiv make_csdiv(int T) {
  CsDiv c;
  c.cs = T > 1 ? T : 1;
  c.m = c.cs < 256 ? gk_cs_magic.m[c.cs] : 1u;
  return c;
}

// (g, d) <-> the packed LDS word: g in bits 0-15, d in bits 16-31 (one v_perm_b32)
__device__ __forceinline__ uint32_t gd_pack(int g, int d) { return __builtin_amdgcn_perm((uint32_t)d, (uint32_t)g, 0x05040100u); }
__device__ __forceinline__ int gd_g(uint32_t w) { return (int)(w & 0xffffu); }
__device__ __forceinline__ int gd_d(uint32_t w) { return (int)(w >> 16); }

template <int VPL, int DUPG = -1>
__device__ __forceinline__ void small_put(SmallLDS<VPL>& L, int pos, double v, int g, int d) {
  L.tv[pidx(pos)] = v;
  L.tgd[pos] = make_int2(g, d);
  if constexpr (DUPG >= 0 && GK_DUPG(DUPG)) {
    dup_st(&L.tv[pidx(pos)], v);
    dup_st(&L.tgd[pos], make_int2(g, d));
  }
}

// gi[gap].x = m << 24 | k << 16 | member base << 8 | out base (m, k <= 128)
__device__ __forceinline__ int gi_ob(int x) { return x & 0xff; }
__device__ __forceinline__ int gi_mb(int x) { return (x >> 8) & 0xff; }
__device__ __forceinline__ int gi_k(int x) { return (x >> 16) & 0xff; }
__device__ __forceinline__ int gi_m(int x) { return (int)((uint32_t)x >> 24); }

// One value x of a gap (its record gi) at rank `rk` inside the gap: gk:93-99
// for an entry's gap, gk:85-92 for the tail.  Both rules evaluated, one store:
// an absorbed value (or an empty slot, !valid) goes to the trash slot.  (A
// branch-free keep decision measured 14% slower on cfg3: the compiler's exec
// branches skip the tail rule for most waves; profiles/r03f_ab_dma_emit_variants.txt.)
template <int VPL, bool NOTAIL = false>
__device__ __forceinline__ void small_emit(SmallLDS<VPL>& L, bool in_gap, const CsDiv& cd, double x, int2 gi,
                                           int rk, bool valid) {
  const int k = gi_k(gi.x);
  if constexpr (NOTAIL) {
    // no value of the flush is in the tail gap (a wave-uniform fact): only
    // the entry-gap rule, no chunk division
    small_put<VPL, 8>(L, (valid && rk >= k) ? gi_ob(gi.x) + rk - k : GK_SMALL_TRASH, x, 1, gi.y);
    return;
  }
  const int q = cd.div(rk);
  const int rr = cd.rem(rk, q);
  const int pos = gi_ob(gi.x) + (in_gap ? rk - k : q);
  const bool keep = valid && (in_gap ? rk >= k : (rr == cd.cs - 1 || rk == gi_m(gi.x) - 1));
  small_put<VPL, 8>(L, keep ? pos : GK_SMALL_TRASH, x, in_gap ? 1 : rr + 1, in_gap ? gi.y : 0);
}

// ---- in-register sort of 128 doubles, two per lane ------------------------
// Position i = lane + 64*r holds a[r].  Bitonic merge sort in the form whose
// every compare-exchange keeps the smaller key at the lower position: a merge
// of two ascending runs of KB/2 starts with a mirror stage (i against
// i ^ (KB-1)), then half-cleaners (i against i ^ J, J = KB/4 .. 1).  The
// partner lane comes from DPP row / quad permutations and the permlane16 /
// permlane32 swaps (gk_xor.h) -- VALU instructions: the LDS pipe, which the
// table traffic of the flush keeps ~70% busy (SQ_LDS_IDX_ACTIVE,
// profiles/r02i_*), stays free; a stage is one compare and two selects per value.  Equal keys may land in either order
// (callers only use this when equal keys are bit-identical).
template <int J>
__device__ __forceinline__ int lane_xor_i32(int v, int lane) {
  // DPP / permlane on the VALU (gk_xor.h): the LDS pipe is the flush's bottleneck
  return lane_xor_dpp<J>(v, lane);
}

template <int J>
__device__ __forceinline__ double lane_xor_f64(double v, int lane) {
  // (round 4: one 64-bit DPP move per pair instead of two 32-bit ones saved a
  // v_mov per compare-exchange but gave wrong sorts on the GPU -- reverted)
  typedef int gk_v2i __attribute__((ext_vector_type(2)));
  const gk_v2i a = __builtin_bit_cast(gk_v2i, v);
  gk_v2i r;
  r.x = lane_xor_i32<J>(a.x, lane);
  r.y = lane_xor_i32<J>(a.y, lane);
  return __builtin_bit_cast(double, r);
}

// a[r] against the value at lane ^ X (same r); the lower lane (bit LB of the
// lane clear) keeps the minimum
template <int X, int LB>
__device__ __forceinline__ void cx_stage2(double (&a)[2], int lane) {
  const bool lower = (lane & LB) == 0;
  if constexpr (X == LB && (X == 16 || X == 32)) {
    // lane ^ 16 / lane ^ 32 by ONE permlane swap per half and no partner
    // select: the swap of (A, B) = (a, a) leaves A = own, B = partner in the
    // lower rows (halves) and A = partner, B = own in the upper ones, so
    // "B < A" decides both sides: lower keeps B iff B < A (the min), upper
    // keeps B iff not (the max); equal keys are bit-identical.
    typedef int gk_v2i __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const gk_v2i v = __builtin_bit_cast(gk_v2i, a[r]);
      gk_v2i A, B;
      if constexpr (X == 16) {
        const auto lo = __builtin_amdgcn_permlane16_swap(v.x, v.x, false, false);
        const auto hi = __builtin_amdgcn_permlane16_swap(v.y, v.y, false, false);
        A.x = (int)lo[0]; B.x = (int)lo[1]; A.y = (int)hi[0]; B.y = (int)hi[1];
      } else {
        const auto lo = __builtin_amdgcn_permlane32_swap(v.x, v.x, false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap(v.y, v.y, false, false);
        A.x = (int)lo[0]; B.x = (int)lo[1]; A.y = (int)hi[0]; B.y = (int)hi[1];
      }
      const double da = __builtin_bit_cast(double, A), db = __builtin_bit_cast(double, B);
      a[r] = ((db < da) == lower) ? db : da;
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const double p = lane_xor_f64<X>(a[r], lane);
    const bool take = (p < a[r]) == lower;
    a[r] = take ? p : a[r];
  }
}

template <int J>
__device__ __forceinline__ void half_cleaners2(double (&a)[2], int lane) {
  cx_stage2<J, J>(a, lane);
  if constexpr (J > 1) half_cleaners2<J / 2>(a, lane);
}

template <int KB>
__device__ __forceinline__ void sort_runs2(double (&a)[2], int lane) {
  // sorts every aligned run of KB positions (KB <= 64: within each r)
  if constexpr (KB > 2) sort_runs2<KB / 2>(a, lane);
  cx_stage2<KB - 1, KB / 2>(a, lane);  // mirror
  if constexpr (KB >= 4) half_cleaners2<KB / 4>(a, lane);
}

__device__ __forceinline__ void sort128_2(double (&a)[2], int lane) {
  sort_runs2<64>(a, lane);  // a[0] and a[1] each ascending over the lanes
  {
    // mirror of the full 128: position lane (r=0) against 127-lane, i.e.
    // lane ^ 63 of r=1; r=0 keeps the minimum
    const double p0 = lane_xor_f64<63>(a[1], lane);
    const double p1 = lane_xor_f64<63>(a[0], lane);
    const bool t0 = p0 < a[0];
    const bool t1 = a[1] < p1;
    a[0] = t0 ? p0 : a[0];
    a[1] = t1 ? p1 : a[1];
  }
  half_cleaners2<32>(a, lane);
}

// ===========================================================================
// k_presort_reg (round 4): the presort of long streams' flush batches, one
// WAVE per batch, in registers.  k_presort sorts a 1024-key batch with 256
// threads through LDS (55 stages, two compare-exchanges per thread and stage
// plus a barrier each): cfg5's 378k batches took 13.6 ms ahead of the
// critical stream's ingest.  Here element e = lane*16 + r of the (padded)
// batch lives in register a[r] of its lane; the bitonic network is run in the
// form whose compare-exchanges always keep the minimum at the lower position
// (a merge of two ascending runs of KB/2 = a mirror stage e ^ (KB-1), then
// half-cleaners e ^ J): distances below 16 are inside a lane (one compare and
// four selects per pair), 16 and up are lane exchanges on the VALU (DPP and
// the permlane swaps of gk_xor.h).  Keys are values alone: equal values are
// bit-identical, so their order cannot change a flush -- except +0.0 and
// -0.0.  A batch holding both has its run of zeros rewritten after the sort
// with the zeros' signs in insertion order (Python's stable sorted() of
// gk:71-72 keeps equal keys in insertion order).
// ===========================================================================
#define GK_PS_R 16  // keys per lane (1024 per wave)

template <bool KEYED>
__device__ __forceinline__ bool ps_less(double a, uint32_t ia, double b, uint32_t ib) {
  if constexpr (KEYED) return a < b || (!(b < a) && ia < ib);
  else return a < b;
}

// intra-lane compare-exchange: position R1 (< R2) keeps the minimum
template <bool KEYED>
__device__ __forceinline__ void ps_ce(double& a1, double& a2, uint32_t& i1, uint32_t& i2) {
  const bool sw = ps_less<KEYED>(a2, i2, a1, i1);
  const double lo = sw ? a2 : a1, hi = sw ? a1 : a2;
  a1 = lo;
  a2 = hi;
  if constexpr (KEYED) {
    const uint32_t il = sw ? i2 : i1, ih = sw ? i1 : i2;
    i1 = il;
    i2 = ih;
  }
}

// half-cleaners of distance J < 16 (inside every lane), J, J/2, .., 1
template <bool KEYED, int J>
__device__ __forceinline__ void ps_half_intra(double (&a)[GK_PS_R], uint32_t (&ix)[GK_PS_R]) {
#pragma unroll
  for (int r = 0; r < GK_PS_R; ++r)
    if ((r & J) == 0) ps_ce<KEYED>(a[r], a[r | J], ix[r], ix[r | J]);
  if constexpr (J > 1) ps_half_intra<KEYED, J / 2>(a, ix);
}

// merge of ascending runs of KB/2 into runs of KB, KB <= 16 (inside lanes)
template <bool KEYED, int KB>
__device__ __forceinline__ void ps_merge_intra(double (&a)[GK_PS_R], uint32_t (&ix)[GK_PS_R]) {
#pragma unroll
  for (int r = 0; r < GK_PS_R; ++r)
    if ((r & (KB / 2)) == 0) ps_ce<KEYED>(a[r], a[r ^ (KB - 1)], ix[r], ix[r ^ (KB - 1)]);
  if constexpr (KB >= 4) ps_half_intra<KEYED, KB / 4>(a, ix);
}

template <int M>
__device__ __forceinline__ uint32_t ps_xor_u32(uint32_t v, int lane) { return (uint32_t)lane_xor_i32<M>((int)v, lane); }

// half-cleaner of distance J >= 16: lanes l and l ^ (J/16), same r
template <bool KEYED, int J>
__device__ __forceinline__ void ps_half_cross(double (&a)[GK_PS_R], uint32_t (&ix)[GK_PS_R], int lane) {
  constexpr int M = J / 16;
  const bool lower = (lane & M) == 0;
#pragma unroll
  for (int r = 0; r < GK_PS_R; ++r) {
    const double p = lane_xor_f64<M>(a[r], lane);
    uint32_t ip = 0;
    if constexpr (KEYED) ip = ps_xor_u32<M>(ix[r], lane);
    const bool take = lower ? ps_less<KEYED>(p, ip, a[r], ix[r]) : ps_less<KEYED>(a[r], ix[r], p, ip);
    a[r] = take ? p : a[r];
    if constexpr (KEYED) ix[r] = take ? ip : ix[r];
  }
}

// merge into runs of KB >= 32: the mirror stage pairs (l, r) with
// (l ^ M, 15 - r), M = (KB - 1) / 16, then the half-cleaners
template <bool KEYED, int KB>
__device__ __forceinline__ void ps_merge_cross(double (&a)[GK_PS_R], uint32_t (&ix)[GK_PS_R], int lane) {
  constexpr int M = (KB - 1) >> 4;
  const bool lower = (lane & (KB / 32)) == 0;
#pragma unroll
  for (int r = 0; r < GK_PS_R / 2; ++r) {
    const int r2 = GK_PS_R - 1 - r;
    const double p1 = lane_xor_f64<M>(a[r2], lane), p2 = lane_xor_f64<M>(a[r], lane);
    uint32_t i1 = 0, i2 = 0;
    if constexpr (KEYED) {
      i1 = ps_xor_u32<M>(ix[r2], lane);
      i2 = ps_xor_u32<M>(ix[r], lane);
    }
    const bool t1 = lower ? ps_less<KEYED>(p1, i1, a[r], ix[r]) : ps_less<KEYED>(a[r], ix[r], p1, i1);
    const bool t2 = lower ? ps_less<KEYED>(p2, i2, a[r2], ix[r2]) : ps_less<KEYED>(a[r2], ix[r2], p2, i2);
    a[r] = t1 ? p1 : a[r];
    a[r2] = t2 ? p2 : a[r2];
    if constexpr (KEYED) {
      ix[r] = t1 ? i1 : ix[r];
      ix[r2] = t2 ? i2 : ix[r2];
    }
  }
  if constexpr (KB / 4 >= 16) ps_half_cross<KEYED, KB / 4>(a, ix, lane);
  if constexpr (KB / 8 >= 16) ps_half_cross<KEYED, KB / 8>(a, ix, lane);
  if constexpr (KB / 16 >= 16) ps_half_cross<KEYED, KB / 16>(a, ix, lane);
  if constexpr (KB / 32 >= 16) ps_half_cross<KEYED, KB / 32>(a, ix, lane);
  if constexpr (KB / 64 >= 16) ps_half_cross<KEYED, KB / 64>(a, ix, lane);
  ps_half_intra<KEYED, 8>(a, ix);
}

template <bool KEYED>
__device__ __forceinline__ void ps_sort1024(double (&a)[GK_PS_R], uint32_t (&ix)[GK_PS_R], int lane) {
  ps_merge_intra<KEYED, 2>(a, ix);
  ps_merge_intra<KEYED, 4>(a, ix);
  ps_merge_intra<KEYED, 8>(a, ix);
  ps_merge_intra<KEYED, 16>(a, ix);
  ps_merge_cross<KEYED, 32>(a, ix, lane);
  ps_merge_cross<KEYED, 64>(a, ix, lane);
  ps_merge_cross<KEYED, 128>(a, ix, lane);
  ps_merge_cross<KEYED, 256>(a, ix, lane);
  ps_merge_cross<KEYED, 512>(a, ix, lane);
  ps_merge_cross<KEYED, 1024>(a, ix, lane);
}

__device__ void presort_reg_range(const GKState& st, const double* __restrict__ x, const int64_t* __restrict__ offs,
                                  const int32_t* __restrict__ list, const int cnt,
                                  const int64_t* __restrict__ list_n, const int64_t* __restrict__ list_ws,
                                  const int64_t* __restrict__ list_b0, double* __restrict__ ws, uint8_t* zs,
                                  const int lane, const bool skip0);

__global__ __launch_bounds__(64) void k_presort_reg(GKState st, const double* __restrict__ x,
                                                    const int64_t* __restrict__ offs,
                                                    const int32_t* __restrict__ list,
                                                    const int32_t* __restrict__ count,
                                                    const int64_t* __restrict__ list_n,
                                                    const int64_t* __restrict__ list_ws,
                                                    const int64_t* __restrict__ list_b0, double* __restrict__ ws,
                                                    int32_t* __restrict__ done) {
  __shared__ uint8_t zs[64 * GK_PS_R];
  const int cnt = *count;
  const int lane = threadIdx.x;
  // Beside k_ingest_wg (done != null) a stream's batch 0 is not sorted: it
  // holds the stream's pre-call pending values, and k_ingest_wg may finish
  // that stream -- rewriting st.pend and its pbuf -- before this launch reaches
  // it; k_ingest_wg ranks every call's first batch unsorted then.
  // Batches b >= 1 are P values of the call's input: read-only here and there.
  if (cnt > 0) presort_reg_range(st, x, offs, list, cnt, list_n, list_ws, list_b0, ws, zs, lane, done != nullptr);
  // (k_ingest_wg, running beside this launch, takes presorted batches once
  // every wave has counted itself here: release of this wave's stores)
  if (done) {
    __threadfence();
    if (lane == 0) atomicAdd(done, 1);
  }
}

__device__ void presort_reg_range(const GKState& st, const double* __restrict__ x, const int64_t* __restrict__ offs,
                                  const int32_t* __restrict__ list, const int cnt,
                                  const int64_t* __restrict__ list_n, const int64_t* __restrict__ list_ws,
                                  const int64_t* __restrict__ list_b0, double* __restrict__ ws, uint8_t* zs,
                                  const int lane, const bool skip0) {
  const int64_t total = list_b0[cnt];
  const int P = st.P;
  // a contiguous range of global batches per wave (as k_presort)
  const int64_t g0 = total * blockIdx.x / gridDim.x, g1 = total * (blockIdx.x + 1) / gridDim.x;
  if (g0 >= g1) return;
  int i = 0;
  {
    int lo = 0, hi = cnt - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (list_b0[mid] <= g0) lo = mid;
      else hi = mid - 1;
    }
    i = lo;
  }
  int64_t bnext = i + 1 < cnt ? list_b0[i + 1] : INT64_MAX;
  int ci = -1;
  int64_t wso = -1, b0 = 0, s = 0, xo = 0, need = 0;
  int p = 0;
  for (int64_t gb = g0; gb < g1; ++gb) {
    while (gb >= bnext) {
      ++i;
      bnext = i + 1 < cnt ? list_b0[i + 1] : INT64_MAX;
    }
    if (i != ci) {
      ci = i;
      wso = list_ws[i];
      b0 = list_b0[i];
      s = list[i];
      xo = offs[s];
      need = P - (list_n[i] % P);
    }
    if (wso < 0) continue;
    const int64_t b = gb - b0;
    if (b == 0) {
      if (skip0) continue;  // wave-uniform
      p = st.pend[s];  // the pre-call pending values: nothing writes them during this launch
    }
    const double* pb = st.pbuf + s * (int64_t)st.pmax;
    const int m = b == 0 ? p + (int)need : P;
    const int64_t xb = b == 0 ? xo : xo + need + (b - 1) * P;
    double a[GK_PS_R];
    uint32_t ix[GK_PS_R];
    bool pz = false, nz = false;
#pragma unroll
    for (int r = 0; r < GK_PS_R; ++r) {
      const int e = lane * GK_PS_R + r;
      double v = __longlong_as_double(0x7ff0000000000000LL);
      if (e < m) v = (b == 0 && e < p) ? pb[e] : x[xb + (b == 0 ? e - p : e)];
      a[r] = v;
      ix[r] = (uint32_t)e;
      const bool z = e < m && v == 0.0;
      pz |= z && !signbit(v);
      nz |= z && signbit(v);
    }
    const bool mixed = __builtin_amdgcn_ballot_w64(pz) != 0 && __builtin_amdgcn_ballot_w64(nz) != 0;
    int zneg = 0;  // values below zero (the zero run starts there after the sort)
    if (mixed) {
      // the zeros' signs by their rank among the zeros in insertion order
      int zc = 0;
#pragma unroll
      for (int r = 0; r < GK_PS_R; ++r) {
        const int e = lane * GK_PS_R + r;
        zc += (e < m && a[r] == 0.0) ? 1 : 0;
        zneg += (e < m && a[r] < 0.0) ? 1 : 0;
      }
      int zr = (int)wave_incl_scan_u32((uint32_t)zc, lane) - zc;
#pragma unroll
      for (int r = 0; r < GK_PS_R; ++r) {
        const int e = lane * GK_PS_R + r;
        if (e < m && a[r] == 0.0) zs[zr++] = signbit(a[r]) ? 1 : 0;
      }
      zneg = wave_sum_i32(zneg);
      wsync<false>();
    }
    ps_sort1024<false>(a, ix, lane);
    if (mixed) {
#pragma unroll
      for (int r = 0; r < GK_PS_R; ++r)
        if (a[r] == 0.0) a[r] = zs[lane * GK_PS_R + r - zneg] ? -0.0 : 0.0;
      wsync<false>();  // (zs is rewritten by the next batch)
    }
    double* out = ws + wso + b * P;
#pragma unroll
    for (int r = 0; r < GK_PS_R; ++r) {
      const int e = lane * GK_PS_R + r;
      if (e < m) out[e] = a[r];
    }
  }
}

// One flush of the small class; K entries per lane (E <= 64*K - 1).  Returns
// the new table size, or -1 if it would exceed SMALL_CAP-1 (the table is then
// untouched... except for the counts, which the caller discards).
template <int VPL, int K, typename AfterSearch>
__device__ __forceinline__ int flush_small(SmallLDS<VPL>& L, const int E, const double (&xv_in)[VPL], const int cnt,
                                           const int T, const CsDiv cd, const int lane, AfterSearch&& after_search) {
  static_assert(K == 2, "the 128-entry class holds 2 entries per lane");
  const double (&xv)[VPL] = xv_in;
  // cd = make_csdiv(T): the chunk-size divider, made by the caller
  if constexpr (VPL == 2) {
    // ---- empty table (every stream's first flush): all values are tail
    //      (gk:85-92), so the flush is a sort and a cut into chunks of
    //      max(T,1).  Sorted in registers; a flush holding both +0.0 and
    //      -0.0 (equal keys that differ) takes the exact path below.
    if (E == 0) {
      bool pz = false, nz = false;
#pragma unroll
      for (int r = 0; r < VPL; ++r) {
        const bool z = (lane + 64 * r < cnt) && xv[r] == 0.0;
        pz |= z && !signbit(xv[r]);
        nz |= z && signbit(xv[r]);
      }
      if (!(__builtin_amdgcn_ballot_w64(pz) != 0 && __builtin_amdgcn_ballot_w64(nz) != 0)) {
        after_search();
        const int newE = cd.cs > 128 ? (cnt > 0 ? 1 : 0) : cd.div(cnt + cd.cs - 1);
        if (newE > SMALL_CAP - 1) return -1;
        double a[2];
#pragma unroll
        for (int r = 0; r < 2; ++r)
          a[r] = (lane + 64 * r < cnt) ? xv[r] : __longlong_as_double(0x7ff0000000000000LL);
        sort128_2(a, lane);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const int q = lane + 64 * r;  // rank in the tail
          const int c = cd.div(q);
          const int rr = cd.rem(q, c);
          const bool keep = q < cnt && (rr == cd.cs - 1 || q == cnt - 1);
          small_put<VPL, 10>(L, keep ? c : GK_SMALL_TRASH, a[r], rr + 1, 0);
        }
        small_pad(L.tv, newE, lane);
        wsync<false>();
        GK_MARK(L, 6);
        return newE;
      }
    }
  }
  // ---- gap = #entries <= x (gk:93): 7 levels over the padded table ---------
  // (slots E .. E+63 hold +inf, small_pad).  xb: byte offset of the padded
  // slot of the gap's entry; x = +inf may step into the padding: clamped to
  // the tail gap.  The gap's padded index addresses the counts (xb/2) and the
  // per-gap records (xb) directly.
  int xb[VPL];
#pragma unroll
  for (int r = 0; r < VPL; ++r) xb[r] = 0;
  const char* tb = (const char*)L.tv;
#define GK_PROBE(S_)                                                                                   \
  {                                                                                                    \
    constexpr int off_ = ((S_) - 1 + (((S_) - 1) >> 5)) * (int)sizeof(double);                         \
    constexpr int step_ = ((S_) + ((S_) >> 5)) * (int)sizeof(double);                                  \
    double t_[VPL];                                                                                    \
    _Pragma("unroll") for (int r = 0; r < VPL; ++r) t_[r] = *(const double*)(tb + xb[r] + off_);       \
    if constexpr (GK_DUPG((S_) >= 8 ? 1 : 2))                                                          \
      _Pragma("unroll") for (int r = 0; r < VPL; ++r) dup_ld((const double*)(tb + xb[r] + off_));      \
    _Pragma("unroll") for (int r = 0; r < VPL; ++r) xb[r] += (t_[r] <= xv[r]) ? step_ : 0;             \
  }
  GK_PROBE(64)
  GK_PROBE(32)
  GK_PROBE(16)
  GK_PROBE(8)
  GK_PROBE(4)
  GK_PROBE(2)
  GK_PROBE(1)
#undef GK_PROBE
  const int pE = pidx(E);           // padded index of the tail gap
  const int pE8 = pE * (int)sizeof(double);
#pragma unroll
  for (int r = 0; r < VPL; ++r) xb[r] = min(xb[r], pE8);
  after_search();
  GK_MARK(L, 1);

  // ---- the lane's 2 entries (+ successor) into registers ------------------
  // (the table is not written before the scan below: these reads are issued
  // beside the count atomics instead of after them)
  const int j0 = 2 * lane;
  const int pj0 = j0 + (lane >> 4);  // pidx(j0); j0 and j0+1 share a 32-slot block
  double ev[K];
  int eg[K + 1], ed[K + 1], em[K];
  {
    int2 gd[K + 1];
    const int4 a = *(const int4*)&L.tgd[j0];
    gd[0] = make_int2(a.x, a.y);
    gd[1] = make_int2(a.z, a.w);
    gd[2] = L.tgd[j0 + 2];
    if constexpr (GK_DUPG(4)) {
      dup_ld((const int4*)&L.tgd[j0]);
      dup_ld(&L.tgd[j0 + 2]);
      dup_ld(&L.tv[pj0]);
      dup_ld(&L.tv[pj0 + 1]);
    }
#pragma unroll
    for (int e = 0; e <= K; ++e) {
      const bool v = j0 + e < E;  // past E: stale LDS, masked
      if (e < K) {
        ev[e] = L.tv[pj0 + e];
        gk_lds_order();  // two ds_read_b64, not one ds_read2_b64
      }
      eg[e] = v ? gd[e].x : 0;
      ed[e] = v ? gd[e].y : 0;
    }
  }

  // ---- gap counts and each value's slot in its gap ------------------------
  // (the counters were zeroed at the end of the previous flush / stream
  // setup; an empty value slot counts into its lane's trash word)
  // (exec-masked, not redirected: an idle lane's trash word would share the
  // LDS banks of the live counters and add conflicts)
  uint32_t xs[VPL];
#pragma unroll
  for (int r = 0; r < VPL; ++r)
    xs[r] = (lane + 64 * r < cnt) ? atomicAdd((uint32_t*)((char*)L.gi + xb[r]), 1u) : 0u;
  if constexpr (GK_DUPG(3))
#pragma unroll
    for (int r = 0; r < VPL; ++r)
      if (lane + 64 * r < cnt) dup_ld((const uint32_t*)((const char*)L.gi + xb[r]));
  wsync<false>();
  uint32_t mloc = 0;
#pragma unroll
  for (int r = 0; r < VPL; ++r) mloc = max(mloc, xs[r] + 1u);
  // a gap of more than GK_SMALL_RANK_MAX members: rank by counting (exact,
  // ties by insertion index, like the in-gap exact pass below)
  const bool use_sort = __builtin_amdgcn_ballot_w64(mloc > (uint32_t)GK_SMALL_RANK_MAX) != 0;
  GK_MARK(L, 2);

  {
    const uint32_t m0 = (uint32_t)L.gi[pj0].x;
    gk_lds_order();
    const uint32_t m1 = (uint32_t)L.gi[pj0 + 1].x;
    if constexpr (GK_DUPG(4)) {
      dup_ld(&L.gi[pj0].x);
      dup_ld(&L.gi[pj0 + 1].x);
    }
    em[0] = (j0 < E) ? (int)m0 : 0;
    em[1] = (j0 + 1 < E) ? (int)m1 : 0;
  }
  int eh[K];  // g + d of the successor, -1 if none
#pragma unroll
  for (int e = 0; e < K; ++e) eh[e] = (j0 + e + 1 < E) ? eg[e + 1] + ed[e + 1] : -1;

  // ---- carry walk (closed form of gk:93-106), as in flush_wave ------------
  // Per entry, with carry c: k = clamp(a - c, 0, m) (a = T - d - g),
  // G = g + c + k, removed iff G <= b (b = T - g' - d' of the successor,
  // INT_MIN without one); the carry out is G if removed, else 0.  Rounds only
  // propagate carries (5 VALU per entry); k, G and keep are evaluated once
  // from the resolved carry-in afterwards.
  int ea[K], eb[K];
#pragma unroll
  for (int e = 0; e < K; ++e) {
    ea[e] = T - ed[e] - eg[e];
    eb[e] = eh[e] >= 0 ? T - eh[e] : INT_MIN;
  }
  // lane l+1's carry-in is known at once if lane l's last entry is kept with
  // carry 0 (G grows with c: then it is kept for any carry)
  const bool has = j0 < E;
  const bool known = (wave_shr1((int)!(eg[K - 1] + clamp0(ea[K - 1], em[K - 1]) <= eb[K - 1]), 1) != 0) || !has;
  // Lane l's carry-in is final once every lane of the run of unknown lanes
  // ending at l has been re-evaluated: the number of extra rounds is the
  // longest run of unknown lanes (scalar bit arithmetic on the lane mask).
  int rounds = 0;
  for (uint64_t u = ~__builtin_amdgcn_ballot_w64(known); u; u &= u << 1) ++rounds;
  int cin = 0;
  for (int r = 0; r < rounds; ++r) {
    int c = cin;
#pragma unroll
    for (int e = 0; e < K; ++e) {
      const int G = eg[e] + c + clamp0(ea[e] - c, em[e]);
      c = G <= eb[e] ? G : 0;
    }
    const int pc = wave_shr1(c, 0);
    cin = known ? 0 : pc;
  }
  int eG[K], ek[K];
  bool ekeep[K];
  {
    int c = cin;
#pragma unroll
    for (int e = 0; e < K; ++e) {
      ek[e] = clamp0(ea[e] - c, em[e]);
      eG[e] = eg[e] + c + ek[e];
      ekeep[e] = !(eG[e] <= eb[e]);
      c = ekeep[e] ? 0 : eG[e];
    }
  }
  uint32_t sm = 0, so = 0;
#pragma unroll
  for (int e = 0; e < K; ++e) {
    const bool v = j0 + e < E;
    sm += (uint32_t)em[e];  // 0 past E
    so += v ? (uint32_t)(em[e] - ek[e] + (ekeep[e] ? 1 : 0)) : 0u;
  }
  // the tail gap (uniform: one broadcast read), counted by the lane holding
  // the last entry
  const int tail_lane = E == 0 ? 0 : (E - 1) >> 1;
  const int mE = __builtin_amdgcn_readfirstlane(L.gi[pE].x);
  const int tail_out = cd.cs > 128 ? (mE > 0 ? 1 : 0) : cd.div(mE + cd.cs - 1);
  sm += lane == tail_lane ? (uint32_t)mE : 0u;
  so += lane == tail_lane ? (uint32_t)tail_out : 0u;
  const uint32_t incl = wave_incl_scan_u32((sm << 16) | so, lane);
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  const int newE = (int)(total & 0xffffu);
  if (newE > SMALL_CAP - 1) return -1;  // one slot stays free for the search padding
  const int totm = (int)(total >> 16);
  wsync<false>();                        // every lane has read the table and the counts
  GK_MARK(L, 3);

  // ---- per-gap results, kept entries (in place: all entries are in registers)
  {
    uint32_t base = incl - ((sm << 16) | so);  // (member base << 16) | out base
    int2 gk[K];
#pragma unroll
    for (int e = 0; e < K; ++e) {
      const bool v = j0 + e < E;
      gk[e] = make_int2((em[e] << 24) | (ek[e] << 16) | (int)((base >> 8) & 0xff00u) | (int)(base & 0xffu),
                        eG[e] + ed[e] - 1);
      small_put<VPL, 5>(L, (v && ekeep[e]) ? (int)(base & 0xffffu) + em[e] - ek[e] : GK_SMALL_TRASH, ev[e], eG[e], ed[e]);
      base += v ? (((uint32_t)em[e] << 16) | (uint32_t)(em[e] - ek[e] + (ekeep[e] ? 1 : 0))) : 0u;
    }
    L.gi[pj0] = gk[0];
    L.gi[pj0 + 1] = gk[1];
    if constexpr (GK_DUPG(11)) {
      dup_st(&L.gi[pj0], gk[0]);
      dup_st(&L.gi[pj0 + 1], gk[1]);
    }
    // the tail gap's record (it is last: member base totm - mE, out base
    // newE - tail_out); a later store, so it wins over the block store of the
    // lane owning padded index pE
    if (lane == 0) L.gi[pE] = make_int2((mE << 24) | ((totm - mE) << 8) | (newE - tail_out), 0);
  }
  wsync<false>();
  GK_MARK(L, 4);

  // ---- stable order inside each gap (gk:72), then emit --------------------
  if (!use_sort) {
    // Members of a gap are stored in slot order (the atomic slot xs).  A
    // value's rank in its gap counts the members below it.  Fast pass:
    // strict counts over every member (self included: never below itself);
    // they are the ranks iff no gap holds equal values, i.e. iff the rank sum
    // reaches sum m(m-1)/2 -- otherwise an exact pass (ties broken by
    // insertion index, Python's stable sort: also orders +0.0 / -0.0 like the
    // reference) reruns.  The reads run past a value's own members into the
    // next gaps (whose values are all above it: gaps partition the value
    // range, and x < v_j <= every member of gap j+1) and, after the last
    // member, into +inf padding: no index clamps, no member-count tests in
    // the loop.
    int2 gv[VPL];
    int gb[VPL], mm[VPL], me[VPL];
    int omax = 0;  // this lane's largest member count; the loop runs while any lane needs it
    int dsum = 0;  // sum over this lane's values of (members - 1)
    constexpr int MV_TRASH = 64 * VPL + 64 + 1;
#pragma unroll
    for (int r = 0; r < VPL; ++r) {
      const bool v = lane + 64 * r < cnt;
      gv[r] = *(const int2*)((const char*)L.gi + xb[r]);
      if constexpr (GK_DUPG(7)) dup_ld((const int2*)((const char*)L.gi + xb[r]));
      gb[r] = gi_mb(gv[r].x);
      const int m = v ? gi_m(gv[r].x) : 0;
      dsum += v ? m - 1 : 0;
      mm[r] = m >= 2 ? m : 0;  // a lone member has rank 0
      me[r] = (int)xs[r];
      L.mv[v ? gb[r] + me[r] : MV_TRASH] = xv[r];
      if constexpr (GK_DUPG(6)) dup_st(&L.mv[v ? gb[r] + me[r] : MV_TRASH], xv[r]);
      omax = max(omax, mm[r]);
    }
    L.mv[totm + lane] = __longlong_as_double(0x7ff0000000000000LL);  // (>= GK_SMALL_RANK_MAX slots)
    if constexpr (GK_DUPG(6)) dup_st(&L.mv[totm + lane], __longlong_as_double(0x7ff0000000000000LL));
    wsync<false>();
    int rk[VPL];
#pragma unroll
    for (int r = 0; r < VPL; ++r) rk[r] = 0;
#pragma unroll
    for (int u0 = 0; u0 < GK_SMALL_RANK_MAX; u0 += 2) {
      if (__builtin_amdgcn_ballot_w64(u0 < omax) == 0) break;
      // (mv sits at LDS address 0: the reads take immediate offsets; kept as
      // two ds_read_b64 -- 2 LDS cycles each over 64 banks -- instead of the
      // ds_read2_b64 the compiler would merge them into: 8 cycles, 32 banks)
      double y[VPL][2];
#pragma unroll
      for (int r = 0; r < VPL; ++r) {
        y[r][0] = L.mv[gb[r] + u0];
        gk_lds_order();
        y[r][1] = L.mv[gb[r] + u0 + 1];
        gk_lds_order();
        if constexpr (GK_DUPG(9)) {
          dup_ld(&L.mv[gb[r] + u0]);
          dup_ld(&L.mv[gb[r] + u0 + 1]);
        }
      }
#pragma unroll
      for (int r = 0; r < VPL; ++r) rk[r] += ((y[r][0] < xv[r]) ? 1 : 0) + ((y[r][1] < xv[r]) ? 1 : 0);
    }
    int rsum = 0;
#pragma unroll
    for (int r = 0; r < VPL; ++r) rsum += (lane + 64 * r < cnt) ? rk[r] : 0;
    // (DPP scan: the sum wraps mod 2^32, exact for these small counts)
    if (__builtin_amdgcn_readlane((int)wave_incl_scan_u32((uint32_t)(2 * rsum - dsum), lane), 63) != 0) {
      // equal values in some gap: exact ranks, ties broken by insertion index
      constexpr int MI_TRASH = 64 * VPL + 1;
#pragma unroll
      for (int r = 0; r < VPL; ++r) L.mi[(lane + 64 * r < cnt) ? gb[r] + me[r] : MI_TRASH] = lane + 64 * r;
      wsync<false>();
#pragma unroll
      for (int r = 0; r < VPL; ++r) rk[r] = 0;
      for (int u0 = 0; __builtin_amdgcn_ballot_w64(u0 < omax) != 0; u0 += 2) {
#pragma unroll
        for (int r = 0; r < VPL; ++r)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int u = u0 + h;
            const int iu = gb[r] + min(u, max(mm[r] - 1, 0));
            const double yy = L.mv[iu];
            const int ii = L.mi[iu];
            const bool below = (yy < xv[r]) | ((yy == xv[r]) & (ii < lane + 64 * r));
            rk[r] += (u < mm[r] && below) ? 1 : 0;
          }
      }
    }
    // (mE: the tail gap's members.  Most flushes have none -- a value past
    // the table's last entry is a new maximum -- and skip the tail rule.)
    if (mE == 0) {
#pragma unroll
      for (int r = 0; r < VPL; ++r) small_emit<VPL, true>(L, true, cd, xv[r], gv[r], rk[r], lane + 64 * r < cnt);
    } else {
#pragma unroll
      for (int r = 0; r < VPL; ++r) small_emit(L, xb[r] < pE8, cd, xv[r], gv[r], rk[r], lane + 64 * r < cnt);
    }
    GK_MARK(L, 5);
  } else {
    // A large gap (the first flush, where every value is tail, or an
    // adversarial order): each value's rank among all the flush's values, by
    // counting in registers -- every value is broadcast from its lane
    // (v_readlane into SGPRs) and compared with the lane's own values.  No
    // LDS traffic.  Gap members are contiguous in the stable order (gaps
    // partition the value range), so the rank inside the gap is the global
    // rank minus the gap's member base.  Equal values (the stable order's
    // tie-break on insertion index) are rare: strict counting gives tied
    // values the same rank, which shows as a rank sum below cnt*(cnt-1)/2,
    // and only then is the exact comparison run.
    int q[VPL];
#pragma unroll
    for (int r = 0; r < VPL; ++r) q[r] = 0;
#pragma unroll
    for (int r2 = 0; r2 < VPL; ++r2) {
      if (64 * r2 >= cnt) break;
      // slots past cnt compare as +inf (never below a value)
      const double y2 = (lane + 64 * r2 < cnt) ? xv[r2] : __longlong_as_double(0x7ff0000000000000LL);
      const int lo2 = __double2loint(y2), hi2 = __double2hiint(y2);
#pragma unroll
      for (int jl = 0; jl < 64; ++jl) {
        const double y = __hiloint2double(__builtin_amdgcn_readlane(hi2, jl), __builtin_amdgcn_readlane(lo2, jl));
#pragma unroll
        for (int r = 0; r < VPL; ++r) q[r] += (y < xv[r]) ? 1 : 0;
      }
    }
    uint32_t qsum = 0;
#pragma unroll
    for (int r = 0; r < VPL; ++r) qsum += (lane + 64 * r < cnt) ? (uint32_t)q[r] : 0u;
    qsum = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_u32(qsum, lane), 63);
    if (qsum != (uint32_t)(cnt * (cnt - 1) / 2)) {
      // ties: (y < x) or (y == x and earlier), gk:72's stable sort
#pragma unroll
      for (int r = 0; r < VPL; ++r) q[r] = 0;
#pragma unroll
      for (int r2 = 0; r2 < VPL; ++r2) {
        const int nj = min(64, cnt - 64 * r2);
        const int lo2 = __double2loint(xv[r2]), hi2 = __double2hiint(xv[r2]);
        for (int jl = 0; jl < nj; ++jl) {
          const double y = __hiloint2double(__builtin_amdgcn_readlane(hi2, jl), __builtin_amdgcn_readlane(lo2, jl));
          const int j = jl + 64 * r2;
#pragma unroll
          for (int r = 0; r < VPL; ++r) q[r] += ((y < xv[r]) | ((y == xv[r]) & (j < lane + 64 * r))) ? 1 : 0;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < VPL; ++r) {
      const int2 gv = *(const int2*)((const char*)L.gi + xb[r]);
      small_emit(L, xb[r] < pE8, cd, xv[r], gv, q[r] - gi_mb(gv.x), lane + 64 * r < cnt);
    }
    GK_MARK(L, 6);
  }
  small_pad(L.tv, newE, lane);
  small_zero_counts(L.gi, lane);
  if constexpr (GK_DUPG(12)) {
    dup_st(&L.tv[pidx(min(newE + lane, SMALL_CAP - 1))], __longlong_as_double(0x7ff0000000000000LL));
    small_zero_counts(L.gi, lane);
  }
  wsync<false>();
  GK_MARK(L, 7);
  return newE;
}

// Quantiles of one stream from the small-class table (gk:156-232): the same
// rule as wave_quantiles, with the lane's K entries in registers.  The
// running max of prefix(g) + d - 1 is monotone, so the reference's break
// index for a threshold th is the number of entries whose running max is
// <= th: one ballot + popcount per entry slot.
// Quantiles of one stream from the small-class table (gk:156-232): the same
// rule as wave_quantiles, with the lane's 2 entries in registers.  The
// running max of prefix(g) + d - 1 is monotone, so the reference's break
// index for a threshold th is the number of entries whose running max is
// <= th: one ballot + popcount per entry slot and quantile.  One chunk of up
// to 64 quantiles: lane l holds q value `qv` of quantile l (qe of them, the
// same for every stream: loaded once per wave by the caller) and gets its
// answer back -- no memory access besides the LDS table (a callee reaches
// global memory only through flat accesses, each a full memory wait).
// Prefix sums in 32 bits while n < 2^31 (always, short of 2^31-value
// streams), else 64.
template <typename I, int VPL>
__device__ __forceinline__ int small_rank_count(SmallLDS<VPL>& L, int E, int64_t n, double spread_d, double qv,
                                                int qe, int lane) {
  const int j0 = 2 * lane;
  I run[2];
  {
    const int4 gd = *(const int4*)&L.tgd[j0];
    const int g0 = (j0 < E) ? gd.x : 0, g1 = (j0 + 1 < E) ? gd.z : 0;
    const I lsum = (I)g0 + (I)g1;
    I bex;
    if constexpr (sizeof(I) == 4) bex = (I)wave_incl_scan_u32((uint32_t)lsum, lane) - lsum;
    else bex = wave_incl_scan_i64(lsum, lane) - lsum;
    const I a0 = bex + g0 + gd.y - 1, a1 = bex + g0 + g1 + gd.w - 1;
    const I lo = std::numeric_limits<I>::min();
    I m = (j0 < E) ? a0 : lo;
    run[0] = m;
    if (j0 + 1 < E && a1 > m) m = a1;
    run[1] = m;
    I pm;
    if constexpr (sizeof(I) == 4) pm = (I)wave_incl_max_i32((int32_t)m);
    else pm = wave_incl_max_i64(m, lane);
    I pex;
    if constexpr (sizeof(I) == 4) pex = (I)wave_shr1((int)pm, (int)lo);
    else pex = wave_shr1_i64(pm, lo);
    const I hi = std::numeric_limits<I>::max();
    run[0] = (j0 < E) ? (run[0] > pex ? run[0] : pex) : hi;
    run[1] = (j0 + 1 < E) ? (run[1] > pex ? run[1] : pex) : hi;
  }
  const double nm1 = (double)(n - 1);
  int myi = 0;
  for (int qq = 0; qq < qe; ++qq) {
    const double q = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(qv), qq),
                                      __builtin_amdgcn_readlane(__double2loint(qv), qq));
    const bool valid = (q >= 0.0 && q <= 1.0);
    // rank = int(q*(n-1) + 1) (gk:173), threshold rank + spread (gk:174-178)
    const int64_t th = valid ? (int64_t)(q * nm1 + 1.0) + (int64_t)spread_d : 0;
    const I t = (I)th;
    const int c = __popcll(__builtin_amdgcn_ballot_w64(run[0] <= t)) + __popcll(__builtin_amdgcn_ballot_w64(run[1] <= t));
    if (lane == qq) myi = c;
  }
  return myi;
}

template <int VPL>
__device__ __attribute__((noinline)) double small_quantiles(SmallLDS<VPL>& L, int E, int64_t n, double mn, double mx,
                                                            double inv_eps, double eps, double qv, int qe, int qmode,
                                                            int lane) {
  const bool valid = (qv >= 0.0 && qv <= 1.0);
  if (n == 0 || E == 0) return gk_nan();
  if ((double)n < inv_eps)  // gk:169 / gk:200
    return valid ? percentile_linear_at(E, qv, [&](int i) { return L.tv[pidx(i)]; }) : gk_nan();
  const double spread_d = floor(eps * (double)(n - 1));  // int(eps*(n-1)) (gk:174 / gk:210), >= 0
  // prefix(g) + d <= n + T < 2^31 - 1 in 32 bits
  const int myi = n < ((int64_t)1 << 30) ? small_rank_count<int32_t>(L, E, n, spread_d, qv, qe, lane)
                                         : small_rank_count<int64_t>(L, E, n, spread_d, qv, qe, lane);
  if (!valid) return gk_nan();
  if (myi == 0) return mn;                          // gk:182-183 / gk:220
  if (myi < E) return L.tv[pidx(myi - 1)];          // gk:185 / gk:220
  return (qmode == 0) ? mx : L.tv[pidx(E - 1)];     // gk:229 / gk:185
}

// ---- stats role of the small-class launch (gk:52-59) ----------------------
// The ingest waves are VALU/SALU-issue-bound and leave most of the HBM
// bandwidth idle, while k_stats is a pure stream of the same values; run as a
// separate launch it cost ~19% of a cfg3 step and cannot share the CUs with
// the persistent ingest grid (profiles/r01c_ab_concurrent_stats.txt).  So the
// first `nstat` waves (GK_FUSED_STATS/8 per CU) of the small-class launch walk the _sum/_avg chains
// first -- 64 streams per wave, one per lane, from a register ring of aligned
// 16-byte loads (the k_stats_long layout, shallower) -- and then join the
// ingest hand-out.  Batches of 64 streams are handed out through `swork`.
// Streams longer than GK_STATS_LONG are k_stats_long's (listed beforehand by
// the lengths-only k_lengths).  The ingest waves do not read _min/_max: a fused
// query that needs them writes a marker that the join (k_query_list) resolves.
#ifndef GK_FS_DEPTH
#define GK_FS_DEPTH 2  // chunks of 8 values in flight per lane
#endif
#define GK_SWORK_IDX 128  // the stats batch counters in `work` (after the 8 ingest parts), one per part
#ifndef GK_FS_LAG_DEFAULT
#define GK_FS_LAG_DEFAULT 256  // streams the ingest hand-out runs ahead of a stats batch (GK_FS_LAG overrides)
#endif
#ifndef GK_FS_DRAIN
#define GK_FS_DRAIN 1  // ingest waves walk their part's unclaimed stats batches once its streams run out
#endif
#ifndef GK_FS_SPIN_MAX
#define GK_FS_SPIN_MAX (1 << 16)  // pacing waits at most this many s_sleeps per batch (no deadlock by construction)
#endif

// Part-aligned and paced (pace > 0): a stats wave serves the streams of its
// own hand-out part (blockIdx % nparts: the XCD whose ingest waves take that
// part's streams), 64 consecutive streams per batch, and starts a batch only
// once the part's ingest hand-out has passed its last stream by `lag`
// streams -- so its reads of the values hit the L2 lines the ingest waves
// (same XCD, same moment) fetched, instead of reading the batch from HBM a
// second time.  pace == 0: no waiting (every wave may be a stats wave).
template <int DEPTH = GK_FS_DEPTH>
__device__ __forceinline__ void fused_stats_role(const GKState& st, const double* __restrict__ x,
                                                 const int64_t* __restrict__ offs,
                                                 unsigned long long* __restrict__ work, int part, int lgp,
                                                 int64_t count, int pace, int lag, int lane) {
  const int64_t pbeg = (count * part) >> lgp, pend = (count * (part + 1)) >> lgp;
  const int64_t nb = (pend - pbeg + 63) / 64;
  unsigned long long* __restrict__ swork = work + GK_SWORK_IDX + 16 * part;
  unsigned long long* __restrict__ iwork = work + 16 * part;  // the part's ingest hand-out counter
  // refills past a lane's last chunk read this instead (st.rtab: 1 MiB the set
  // owns, 16-byte aligned; the values are never used)
  const double2* __restrict__ dummy = (const double2*)st.rtab;
  for (;;) {
    unsigned long long v = 0;
    if (lane == 0) v = atomicAdd(swork, 1ull);
    const int64_t b = rfl64((int64_t)v);
    if (b >= nb) break;
    if (pace) {
      const int64_t want = min((b + 1) * 64 + (int64_t)lag, pend - pbeg);
      for (int spin = 0; spin < GK_FS_SPIN_MAX; ++spin) {
        unsigned long long got = 0;
        if (lane == 0) got = __hip_atomic_load(iwork, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (rfl64((int64_t)got) >= want) break;
        __builtin_amdgcn_s_sleep(8);
      }
    }
    // (stream ids fit in 32 bits; a 64-bit pbeg + lane hoisted out of the
    // batch loop was the launch's one remaining scratch spill)
    const int64_t s = (int64_t)((int)(pbeg + b * 64) + lane);
    const bool live = s < pend;
    const int64_t xo = live ? offs[s] : 0;
    int64_t rem = live ? offs[s + 1] - xo : 0;
    if (rem > GK_STATS_LONG) rem = 0;  // k_stats_long's
    const bool act = rem > 0;
    int64_t n = 0;
    double mn = 0, mx = 0, sm = 0, av = 0;
    if (act) {
      n = st.n0[s];  // pre-call n (k_lengths snapshot): st.n[s] may already be the ingest's
      mn = st.mn[s];
      mx = st.mx[s];
      sm = st.sum[s];
      av = st.avg[s];
    }
    // peel one value when the stream starts off 16-byte alignment
    const int64_t peel = (act && (((uintptr_t)(x + xo)) & 8)) ? 1 : 0;
    if (peel) {
      gk_stat_step(x[xo], n, sm, av, mn, mx);
      --rem;
    }
    const double* p = x + xo + peel;
    const int64_t nch = rem / 8;  // full chunks of 8 values
    int64_t maxch = nch;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxch = max(maxch, (int64_t)__shfl_xor(maxch, o, 64));
    const double2* __restrict__ p2 = (const double2*)p;
    // Streams of one batch usually share n (same history): the gk:54 factors
    // 1.0/n are then wave-uniform and read from st.rtab (scalar loads)
    // instead of ~10 VALU of IEEE division per value.  n of the active lanes
    // stays equal chunk by chunk (each adds 8 per chunk while active).
    int64_t nlo = act ? n : INT64_MAX, nhi = act ? n : INT64_MIN;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      nlo = min(nlo, (int64_t)__shfl_xor(nlo, o, 64));
      nhi = max(nhi, (int64_t)__shfl_xor(nhi, o, 64));
    }
    const int64_t nu = rfl64(nlo);
    const bool uni = nu == rfl64(nhi) && nu >= 0 && nu + 8 * maxch + 8 < st.rtab_n;
    // loads past a lane's last chunk read the first aligned values of the
    // batch instead, so every refill is unconditional
    double2 ring[DEPTH][4];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const double2* src = (d < nch) ? p2 + d * 4 : dummy;
#pragma unroll
      for (int j = 0; j < 4; ++j) ring[d][j] = src[j];
    }
    auto walk = [&](auto tab) {
      constexpr bool TAB = decltype(tab)::value;
      for (int64_t c0 = 0; c0 < maxch; c0 += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
          const int64_t c = c0 + d;
          if (c < nch) {
            const double* __restrict__ rt = st.rtab + (nu + 8 * c + 1);  // uniform (TAB)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const double v = (k & 1) ? ring[d][k >> 1].y : ring[d][k >> 1].x;
              const double rc = TAB ? rt[k] : 1.0 / (double)(n + 1 + k);  // off the chain
              sm = sm + v;                    // gk:53
              av = av + (v - av) * rc;        // gk:54
              if (v < mn) mn = v;             // gk:56-57
              if (v > mx) mx = v;             // gk:58-59
            }
            n += 8;                           // gk:52
          }
          const int64_t nx = c + DEPTH;
          const double2* src = (nx < nch) ? p2 + nx * 4 : dummy;
#pragma unroll
          for (int j = 0; j < 4; ++j) ring[d][j] = src[j];
        }
      }
    };
    if (uni) walk(std::true_type{});
    else walk(std::false_type{});
    const int tail = (int)(rem - nch * 8);
    for (int k = 0; k < tail; ++k) gk_stat_step(p[nch * 8 + k], n, sm, av, mn, mx);
    if (act) {
      st.mn[s] = mn;
      st.mx[s] = mx;
      st.sum[s] = sm;
      st.avg[s] = av;
    }
  }
}

// fused-stats launches: quantiles that are _min / _max (markers) resolved
// FS: the launch carries the stats role (nstat > 0): _min/_max are not final
// during it, so the header prefetch skips them and fused quantiles use markers.
// Class 0 over every stream only (promoted streams are skipped: their class's
// launch runs them).
#ifdef GK_TIMELINE
// timeline builds only (tools/launch_timeline.py): s_memrealtime (100 MHz,
// chip-wide) per wave (start, stats role done, end) and per stream (start, end)
#define GK_TL_MAXS (1 << 20)
#define GK_TL_MAXW 16384
__device__ unsigned long long gk_tl_wave[5 * GK_TL_MAXW];
__device__ unsigned long long gk_tl_sbeg[GK_TL_MAXS];
__device__ unsigned long long gk_tl_send[GK_TL_MAXS];
#endif
template <int VPL, bool FS, int W = GK_SMALL_WAVES>
__global__ __launch_bounds__(64, W) void k_ingest_small(GKState st, const double* __restrict__ x,
                                                     const int64_t* __restrict__ offs, int64_t count, int force,
                                                     int32_t* __restrict__ ovf_count, int32_t* __restrict__ ovf_list,
                                                     const double* __restrict__ qs, int nq,
                                                     double* __restrict__ qout, int qmode,
                                                     unsigned long long* __restrict__ work, int nstat,
                                                     int fs_pace, int fs_lag) {
  __shared__ __attribute__((aligned(16))) SmallLDS<VPL> L;
  const int lane = threadIdx.x;
  const int P = st.P;
#ifdef GK_PROF
  if (lane == 0) {
    for (int i = 0; i < GK_PROF_NSEC; ++i) L.prof[i] = 0;
    L.prof_t = gk_cycles();
  }
#endif
  // Streams are handed out dynamically (one atomic per stream on `work`,
  // zeroed before the launch), so waves on slower CUs simply take fewer
  // streams; the next stream's id and header are fetched one stream ahead.
  uint32_t hv = 0;  // the next stream's header, one word per lane (gk_hdr1_issue)
#ifndef GK_WORK_PARTS
#define GK_WORK_PARTS 8  // counters (one 128-B line each); a wave uses blockIdx % parts
#endif
#ifndef GK_WORK_CHUNK
#define GK_WORK_CHUNK 2  // streams per grab
#endif
  // parts: a power of two, at most GK_WORK_PARTS and the grid (every part
  // has a wave), so that the part bounds are scalar shifts (a 64-bit division
  // here was VALU code whose results the flush loop's register pressure
  // spilled to scratch -- and a launch with scratch costs the step two
  // dispatch gaps of ~5 us)
  static_assert((GK_WORK_PARTS & (GK_WORK_PARTS - 1)) == 0, "a power of two");
  int lgp = 0;
  while ((2 << lgp) <= GK_WORK_PARTS && (2u << lgp) <= gridDim.x) ++lgp;
  const int part = (int)(blockIdx.x & ((1u << lgp) - 1u));
#ifdef GK_TIMELINE
  if (lane == 0 && blockIdx.x < GK_TL_MAXW) {
    gk_tl_wave[5 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    gk_tl_wave[5 * blockIdx.x + 3] = __builtin_amdgcn_s_memtime();
  }
#endif
  if (FS && (int)blockIdx.x < nstat) fused_stats_role(st, x, offs, work, part, lgp, count, fs_pace, fs_lag, lane);
#ifdef GK_TIMELINE
  if (lane == 0 && blockIdx.x < GK_TL_MAXW) gk_tl_wave[5 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
#endif
  const int64_t pbeg = (count * part) >> lgp, pend = (count * (part + 1)) >> lgp;
  // the query's q values, the same for every stream: lane l holds q l
  const double qpre = (qs && lane < nq) ? qs[lane] : 0.0;
  int64_t cur = 0, cend = 0;
  auto grab = [&]() -> int64_t {
    if (cur >= cend) {
      unsigned long long v = 0;
      if (lane == 0) v = atomicAdd(work + 16 * part, (unsigned long long)GK_WORK_CHUNK);
      cur = pbeg + rfl64((int64_t)v);
      cend = min(cur + GK_WORK_CHUNK, pend);
      if (cur >= pend) return count;
    }
    return cur++;
  };
  int64_t w = grab();
  if (w < count) hv = gk_hdr1_issue<!FS>(st, offs, w, lane);
#ifdef GK_PROF
  bool prof_done_any = false;  // a stream of this wave has been written back
#endif
  for (; w < count;) {
    const int64_t s = w;
    const int64_t wn = grab();
    const int32_t scls = gk_hdr1_word(hv, 0);
    const int32_t sslot = gk_hdr1_word(hv, 1);
    int p = gk_hdr1_word(hv, 2);
    int E = gk_hdr1_word(hv, 3);
    int64_t n = gk_hdr1_dword(hv, 4);
    const int64_t xo = gk_hdr1_dword(hv, 6);
    const int64_t xe = gk_hdr1_dword(hv, 8);
    // with the stats role in this launch, _min/_max are not final yet: markers
    const double smn = __longlong_as_double(FS ? GK_QMARK_MIN : gk_hdr1_dword(hv, 10));
    const double smx = __longlong_as_double(FS ? GK_QMARK_MAX : gk_hdr1_dword(hv, 12));
    if (wn < count) hv = gk_hdr1_issue<!FS>(st, offs, wn, lane);
    w = wn;
    if (scls != 0) continue;  // promoted: handled by its class launch
#ifdef GK_TIMELINE
    if (lane == 0 && s < GK_TL_MAXS) gk_tl_sbeg[s] = __builtin_amdgcn_s_memrealtime();
#endif
    const int64_t Lx = xe - xo;
    // force 1: flush only if values are pending (size/quantile, gk:45, 166, 197)
    // force 2: unconditional merge_compress() (merge, gk:122, 126, 137)
    if (Lx <= 0 && !((force == 1 && p > 0) || (force == 2 && n > 0)) && !qs) continue;
    GKRec* __restrict__ tab = gk_table_ptr_cs(st, s, scls, sslot);
    double* __restrict__ pb = st.pbuf + s * (int64_t)st.pmax;
    // an imported / merged table without room for the padding, a stream
    // past the count limit, or one with 2^31 - 2^15 or more values in this
    // call (the flush loop counts in 32 bits; k_ingest counts in 64):
    // promotion
    bool ok = E <= SMALL_CAP - 1 && gk_count_ok(st, n + (Lx > 0 ? Lx : 0)) && Lx < GK_SMALL_LX_MAX;
    if (ok) {
      // 16-byte records moved as int4: all loads issued before the first wait
      const int4* __restrict__ t4 = (const int4*)tab;
      int4 rc[SMALL_CAP / 64];
#pragma unroll
      for (int r = 0; r < SMALL_CAP / 64; ++r)
        rc[r] = (lane + 64 * r < E) ? t4[lane + 64 * r] : make_int4(0, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < SMALL_CAP / 64; ++r) {
        const int j = lane + 64 * r;
        if (j < E) {
          L.tv[pidx(j)] = __hiloint2double(rc[r].y, rc[r].x);
          L.tgd[j] = make_int2(rc[r].z, rc[r].w);
        }
      }
      small_pad(L.tv, E, lane);
      small_zero_counts(L.gi, lane);
    }
    wsync<false>();
    GK_MARK(L, 0);

    bool flushed = false;  // at least one flush in this call
    bool final_done = false;
    // Per-call counters in 32 bits (ok: Lx < GK_SMALL_LX_MAX), so that the
    // loop's tests are scalar compares, not 64-bit VALU ones.
    const int L32 = (int)Lx;
    int used = 0;
    const int need0 = P - (int)(n % P);  // adds until n hits the next multiple of P (gk:60)
    int need = need0;
    // T = floor((2 eps) * float(n - 1)) (gk:70) and the chunk divider of
    // every flush of the call, 64 flushes at a time, lane f for flush f: n at
    // flush f is n + min(need0 + f P, Lx) (the last term for the requested
    // flush that ends the call), float(n - 1) exact (integers < 2^53), and
    // gk_count_ok above bounds T by GK_T_CLAMP (no clamps).  The flush reads
    // its T and magic number with two v_readlane.
    const double nm1c = (double)(n - 1);
    int fl = 0;  // flushes made in this call
    int tT = 0;
    uint32_t tM = 0;
    auto plan_t = [&]() {
      const int k = min(need0 + (fl + lane) * P, L32);
      tT = (int)(st.two_eps * (nm1c + (double)k));
      const uint32_t cs = (uint32_t)max(tT, 1);
      tM = cs < 256u ? ((1u << 23) + cs - 1u) / cs : 1u;
    };
    // the stream's values from x + xo as a buffer resource: the prefetch of
    // the next flush reads lanes past its count as 0 (range check), with no
    // address clamps or 64-bit address arithmetic on the VALU
    const double* const xs = x ? x + xo : pb;
    double xv[VPL];
#pragma unroll
    for (int r = 0; r < VPL; ++r) xv[r] = 0.0;
    while (ok) {
      const bool autof = need <= L32 - used;
      int nadd;
      if (autof) {
        nadd = need;
      } else {
        nadd = L32 - used;  // < need: only a requested flush takes these now
        if (!((force == 1 && p + nadd > 0) || force == 2)) break;
      }
      const int cnt = p + nadd;
      if (!flushed) gk_load_flush_values<VPL>(xv, pb, p, xs, cnt, lane);
      const int nused = used + nadd;
      // the next flush's values (or the leftover tail), loaded one flush ahead
      const int navail = autof ? min(P, L32 - nused) : 0;
      double xn[VPL];
      auto prefetch = [&]() {
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(xs + nused), 0, navail * (int)sizeof(double), 0x00020000);
#pragma unroll
        for (int r = 0; r < VPL; ++r)
          xn[r] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, (lane + 64 * r) * 8, 0, 0));
      };
      if ((fl & 63) == 0) plan_t();
      n += nadd;
      const int T = __builtin_amdgcn_readlane(tT, fl & 63);
      CsDiv cd;
      cd.cs = max(T, 1);
      cd.m = (uint32_t)__builtin_amdgcn_readlane((int)tM, fl & 63);
      ++fl;
      // (profiling builds: the loop top of a wave's FIRST stream counts apart, in 11)
      // (GK_PROF_FIRST 1: a wave's first stream's loop tops; 2: every
      // stream's first loop top -- its first values' load -- in section 11)
      GK_MARK(L, (GK_PROF_FIRST == 2 ? !flushed : (GK_PROF_FIRST && !prof_done_any)) ? 11 : 8);
      int nE;
      if constexpr (SMALL_CAP > 128)
        nE = E <= 127 ? flush_small<VPL, 2>(L, E, xv, cnt, T, cd, lane, prefetch)
                      : flush_small<VPL, 4>(L, E, xv, cnt, T, cd, lane, prefetch);
      else
        nE = flush_small<VPL, 2>(L, E, xv, cnt, T, cd, lane, prefetch);
      if (nE < 0) {
        n -= nadd;  // (this flush is not made here: the state stays that of the last flush that fitted)
        ok = false;
        break;
      }
      E = nE;
      used = nused;
      p = 0;
      need = P;
      flushed = true;
#pragma unroll
      for (int r = 0; r < VPL; ++r) xv[r] = xn[r];  // 0.0 past navail (range check)
      GK_MARK(L, 10);  // (profiling builds: the wait for the prefetched values)
      if (!autof) {
        final_done = true;
        break;
      }
    }
    if (ok && !final_done) {
      const int rem = L32 - used;  // < need: stays pending
      if (flushed) {
#pragma unroll
        for (int r = 0; r < VPL; ++r)
          if (lane + 64 * r < rem) pb[lane + 64 * r] = xv[r];
      } else {
        for (int i = lane; i < rem; i += 64) pb[p + i] = xs[used + i];
      }
      p += rem;
      n += rem;
    }
    // the table (E <= 127: two records per lane, all LDS reads before the
    // 16-byte stores) and the header words
    auto write_back = [&]() {
      double v[2];
      int2 gd[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        v[r] = L.tv[pidx(lane + 64 * r)];
        gd[r] = L.tgd[lane + 64 * r];
      }
#pragma unroll
      for (int r = 0; r < 2; ++r)
        if (lane + 64 * r < E) ((int4*)tab)[lane + 64 * r] = make_int4(__double2loint(v[r]), __double2hiint(v[r]), gd[r].x, gd[r].y);
      if (lane == 0) {
        st.n[s] = n;
        st.E[s] = E;
        st.pend[s] = p;
      }
    };
    if (!ok) {
      // The flush that outgrew the class is not made.  The flushes before it
      // are committed (table, n, no pending value): the stream is promoted to
      // the next class on the device and continues there from value n - n0
      // of this call (st.n0: the pre-call n, k_lengths) instead of re-running
      // the whole call.  Without a flush in this call the pre-call state
      // stays as it was.
      if (flushed) write_back();
      if (lane == 0) {
        const int k = atomicAdd(ovf_count, 1);
        ovf_list[k] = (int32_t)s;
      }
      wsync<false>();
      continue;
    }
    if (qs) {
      for (int q0 = 0; q0 < nq; q0 += 64) {
        // (the lane made opaque per chunk: its 64-bit address math is not
        // hoisted out of the stream loop, where it was spilled to scratch)
        int ql = lane;
        __asm__ volatile("" : "+v"(ql));
        const double qv = nq <= 64 ? qpre : ((q0 + ql < nq) ? qs[q0 + ql] : 0.0);
        const double r = small_quantiles<VPL>(L, E, n, smn, smx, st.inv_eps, st.eps, qv, min(nq - q0, 64), qmode, lane);
        if (q0 + ql < nq) qout[s * (int64_t)nq + q0 + ql] = r;
      }
    }
    write_back();
    wsync<false>();
    GK_MARK(L, 9);
#ifdef GK_TIMELINE
    if (lane == 0 && s < GK_TL_MAXS) gk_tl_send[s] = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef GK_PROF
    prof_done_any = true;
#endif
  }
  // The part's streams have run out: its stats batches still unclaimed are
  // walked by every wave of the part as it gets here, not by the stats waves
  // alone (which trail the hand-out: until round 6 they ended the launch up
  // to ~200 us after the last ingest wave).  The part's hand-out is past its
  // end, so the pacing never waits here.
  if (FS && GK_FS_DRAIN) fused_stats_role(st, x, offs, work, part, lgp, count, fs_pace, fs_lag, lane);
#ifdef GK_PROF
  if (lane == 0)
    for (int i = 0; i < GK_PROF_NSEC; ++i) atomicAdd(&gk_prof_acc[i], L.prof[i]);
#endif
#ifdef GK_TIMELINE
  if (lane == 0 && blockIdx.x < GK_TL_MAXW) {
    gk_tl_wave[5 * blockIdx.x + 2] = __builtin_amdgcn_s_memrealtime();
    gk_tl_wave[5 * blockIdx.x + 4] = __builtin_amdgcn_s_memtime();
  }
#endif
}

// ===========================================================================
// k_merge: GKArray.merge (gk:111-154) and merge_compress(entries), stream by
// stream.  The incoming list (self's raw pending values, then the converted
// records of `other` or the caller's records) is stably ordered by value and
// the four-rule walk of gk:76-106 runs wave-parallel over LDS: incoming
// records carry g > 1 here, so the add-path closed form does not apply; each
// lane re-walks its block of entries from its neighbour's carry until no
// carry-in changes (k_merge).
// `other` has already been flushed by the caller (gk:126, gk:137).
// ===========================================================================
struct MergeArgs {
  GKState dst;
  GKState src;            // mode 0: the other set (already flushed, gk:126/137)
  const double* ev;       // mode 1: explicit records (v, g, d) in CSR
  const int32_t* eg;
  const int32_t* ed;
  const int64_t* eoffs;
  int mode;               // 0 = merge(other), 1 = merge_compress(entries)
  int cap;                // LDS capacity for tables / records
  const int32_t* list;    // streams to process (NULL = all)
  int64_t count;
  int32_t* ovf_count;
  int32_t* ovf_list;
  unsigned char* ws;      // global workspace (largest class), NULL = dynamic LDS
  size_t ws_bytes;        // per block
};

struct MergeLDS {
  double *tv, *rv, *sp, *iv, *ov;
  int32_t *tg, *td, *rg, *rd, *ig, *id, *og, *od;
};

__device__ __forceinline__ MergeLDS merge_carve(unsigned char* smem, int cap, int pm) {
  const int MR = cap + 1, MI = cap + 1 + pm;
  MergeLDS m;
  double* dp = (double*)smem;
  m.tv = dp; dp += cap;
  m.rv = dp; dp += MR;
  m.sp = dp; dp += pm;
  m.iv = dp; dp += MI;
  m.ov = dp; dp += cap;
  int32_t* ip = (int32_t*)dp;
  m.tg = ip; ip += cap;
  m.td = ip; ip += cap;
  m.rg = ip; ip += MR;
  m.rd = ip; ip += MR;
  m.ig = ip; ip += MI;
  m.id = ip; ip += MI;
  m.og = ip; ip += cap;
  m.od = ip; ip += cap;
  return m;
}

__device__ __forceinline__ void flag_overflow(int32_t* cnt, int32_t* list, int64_t s, int lane) {
  if (lane == 0) {
    const int k = atomicAdd(cnt, 1);
    list[k] = (int32_t)s;
  }
}

#define GK_MERGE_RANK_MAX 256  // pending values ranked by comparison up to this many; bitonic above

template <bool GLOBAL>
__global__ __launch_bounds__(64) void k_merge(MergeArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int sh_out;
  const int lane = threadIdx.x;
  const int CAPL = a.cap;
  const int PM = a.dst.pmax;
  unsigned char* base = GLOBAL ? a.ws + (size_t)blockIdx.x * a.ws_bytes : smem;
  const MergeLDS m = merge_carve(base, CAPL, PM);
  const GKState& st = a.dst;
  for (int64_t w = blockIdx.x; w < a.count; w += gridDim.x) {
    const int64_t s = a.list ? (int64_t)a.list[w] : w;
    GKRec* __restrict__ tab = gk_table_ptr(st, s);
    const int outcap = min(st.cap[st.cls[s]], CAPL) - 1;  // k_ingest keeps one slot for padding
    int64_t n = st.n[s];
    const int E = st.E[s];
    const int p = st.pend[s];
    const double* __restrict__ pb = st.pbuf + s * (int64_t)st.pmax;

    // ---- branch of gk:121-133 -------------------------------------------------
    int nrec = 0;
    if (a.mode == 0) {
      const GKState& os = a.src;
      const int64_t on = os.n[s];
      const int oE = os.E[s];
      const GKRec* __restrict__ otab = gk_table_ptr(os, s);
      if (on != 0 && n == 0) {  // gk:125-133: take a copy of (flushed) other
        if (oE > outcap) {
          flag_overflow(a.ovf_count, a.ovf_list, s, lane);
          __syncthreads();
          continue;
        }
        for (int j = lane; j < oE; j += 64) tab[j] = otab[j];
        if (lane == 0) {
          st.n[s] = on;
          st.E[s] = oE;
          st.pend[s] = 0;
          st.mn[s] = os.mn[s];
          st.mx[s] = os.mx[s];
          st.sum[s] = os.sum[s];
          st.avg[s] = os.avg[s];
        }
        __syncthreads();
        continue;
      }
      if (on != 0) {
        // gk:136-147: spread from other's n, then the converted records
        //   (other._min, g0+d0-spread-1), (v_k, g_{k+1}+d_{k+1}-d_k),
        //   (v_{L-1}, spread+1-d_{L-1}); only g > 0 is kept.
        const int64_t spread = (int64_t)(os.eps * (double)(on - 1));
        const int ncand = oE + 1;
        if (ncand > CAPL + 1) {
          flag_overflow(a.ovf_count, a.ovf_list, s, lane);
          __syncthreads();
          continue;
        }
        int base = 0;
        for (int c0 = 0; c0 < ncand; c0 += 64) {
          const int c = c0 + lane;
          int64_t gv = 0;
          double vv = 0.0;
          if (c < ncand) {
            if (c == 0) {
              gv = (int64_t)otab[0].g + otab[0].d - spread - 1;
              vv = os.mn[s];
            } else if (c < oE) {
              gv = (int64_t)otab[c].g + otab[c].d - otab[c - 1].d;
              vv = otab[c - 1].v;
            } else {
              gv = spread + 1 - otab[oE - 1].d;
              vv = otab[oE - 1].v;
            }
          }
          const bool keep = (c < ncand) && gv > 0;
          const unsigned long long bal = __ballot(keep);
          const int before = __popcll(bal & ((1ull << lane) - 1ull));
          if (keep) {
            m.rv[base + before] = vv;
            m.rg[base + before] = (int32_t)gv;
            m.rd[base + before] = 0;
          }
          base += __popcll(bal);
        }
        nrec = base;
        n += on;  // gk:149
        if (lane == 0) {  // gk:151-152: min()/max() keep self's value on ties
          const double omn = os.mn[s], omx = os.mx[s];
          if (omn < st.mn[s]) st.mn[s] = omn;
          if (omx > st.mx[s]) st.mx[s] = omx;
        }
      }
      // on == 0: gk:121-123, self.merge_compress() with no records
    } else {
      const int64_t eo = a.eoffs[s];
      nrec = (int)(a.eoffs[s + 1] - eo);
      if (nrec > CAPL + 1) {
        flag_overflow(a.ovf_count, a.ovf_list, s, lane);
        __syncthreads();
        continue;
      }
      for (int c = lane; c < nrec; c += 64) {
        m.rv[c] = a.ev[eo + c];
        m.rg[c] = a.eg[eo + c];
        m.rd[c] = a.ed[eo + c];
      }
    }
    if (E > CAPL || !gk_count_ok(st, n)) {  // (n: after the merge, gk:149)
      flag_overflow(a.ovf_count, a.ovf_list, s, lane);
      __syncthreads();
      continue;
    }
    // ---- stable order of self's raw pending values (gk:72) ------------------
    if (p <= GK_MERGE_RANK_MAX) {
      // few values: each lane ranks its values against all of them
      for (int i = lane; i < p; i += 64) m.ov[i] = pb[i];
      __syncthreads();
      for (int i = lane; i < p; i += 64) {
        const double x = m.ov[i];
        int rk = 0;
        for (int t = 0; t < p; ++t) {
          const double y = m.ov[t];
          rk += (y < x) || (y == x && t < i);
        }
        m.sp[rk] = x;
      }
    } else {
      // a large flush period (eps < 1/256): bitonic sort of (value, index)
      // in the output arrays (free here; cap >= pow2 above p for every class)
      int N = 1;
      while (N < p) N <<= 1;
      for (int i = lane; i < N; i += 64) {
        m.ov[i] = i < p ? pb[i] : __longlong_as_double(0x7ff0000000000000LL);
        m.og[i] = i < p ? i : INT32_MAX;
      }
      __syncthreads();
      for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int pp = lane; pp < N / 2; pp += 64) {
            const int i = ((pp & ~(j - 1)) << 1) | (pp & (j - 1));
            const int l = i + j;
            const double a = m.ov[i], b = m.ov[l];
            const int ia = m.og[i], ib = m.og[l];
            const bool a_gt = (a > b) || (a == b && ia > ib);
            if (a_gt == ((i & k) == 0)) {
              m.ov[i] = b;
              m.ov[l] = a;
              m.og[i] = ib;
              m.og[l] = ia;
            }
          }
          __syncthreads();
        }
      }
      for (int i = lane; i < p; i += 64) m.sp[i] = m.ov[i];
    }
    __syncthreads();
    // ---- merged incoming list: `self.incoming + entries` sorted stably, so on
    //      equal values the raw pending values come first (gk:71-72) ----------
    for (int r = lane; r < p; r += 64) {
      const double x = m.sp[r];
      int lo = 0, hi = nrec;  // records strictly below x
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (m.rv[mid] < x) lo = mid + 1; else hi = mid;
      }
      m.iv[r + lo] = x;
      m.ig[r + lo] = 1;
      m.id[r + lo] = 0;
    }
    for (int t = lane; t < nrec; t += 64) {
      const double y = m.rv[t];
      int lo = 0, hi = p;  // pending values <= y
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (m.sp[mid] <= y) lo = mid + 1; else hi = mid;
      }
      m.iv[t + lo] = y;
      m.ig[t + lo] = m.rg[t];
      m.id[t + lo] = m.rd[t];
    }
    for (int j = lane; j < E; j += 64) {
      const GKRec rc = tab[j];
      m.tv[j] = rc.v;
      m.tg[j] = rc.g;
      m.td[j] = rc.d;
    }
    __syncthreads();
    // ---- the four-rule walk of gk:76-106, wave-parallel ----------------------
    // Incoming records (sorted) fall into gaps: record i precedes entry j iff
    // iv[i] < tv[j] (gk:93), so gap j holds [a_{j-1}, a_j) with a_j = #{i :
    // iv[i] < tv[j]}, and the tail [a_{E-1}, M) follows the last entry.  Entry
    // j with carry-in c (the g of removed predecessors, gk:80/102) starts at
    // G = g_j + c and walks its gap in order: record i is absorbed iff
    // g_i + G + d_j <= T (G += g_i), else emitted as (v_i, g_i, G + d_j - g_i)
    // (gk:94-99); the entry is then removed (carry G) iff j+1 < E and
    // G + g_{j+1} + d_{j+1} <= T (gk:79/101), else emitted as (v_j, G, d_j).
    // The tail chains records (gk:86-92).  Lane l owns entries [lK, lK+K); the
    // carries are resolved by rounds (each lane re-walks its block from its
    // left neighbour's last carry-out) until no carry-in changes -- lane 0's is
    // fixed, so the fixpoint is the sequential walk.  Then counts, a wave scan
    // and a second walk write the records in order.
    {
      const int64_t T = (int64_t)floor(st.two_eps * (double)(n - 1));  // gk:70
      const int M = p + nrec;
      int32_t* ga = m.rg;  // a_j (records are in iv/ig/id by now)
      for (int j = lane; j < E; j += 64) {
        const double tvj = m.tv[j];
        int lo = 0, hi = M;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (m.iv[mid] < tvj) lo = mid + 1; else hi = mid;
        }
        ga[j] = lo;
      }
      __syncthreads();
      const int K = (E + 63) >> 6;
      const int j0 = lane * K;
      const int jend = min(j0 + K, E);
      // walk of the lane's block from carry-in c; returns the carry-out and
      // the number of records it emits (out != NULL: also writes them)
      auto walk = [&](int64_t c, int& cnt_out, int obase, bool write) -> int64_t {
        int no_l = 0;
        for (int j = j0; j < jend; ++j) {
          int64_t G = (int64_t)m.tg[j] + c;
          const int64_t dj = m.td[j];
          const int ib = j == 0 ? 0 : ga[j - 1];
          const int ie = ga[j];
          for (int i = ib; i < ie; ++i) {
            const int64_t gi = m.ig[i];
            if (gi + G + dj <= T) {
              G += gi;
            } else {
              if (write) {
                m.ov[obase + no_l] = m.iv[i];
                m.og[obase + no_l] = (int32_t)gi;
                m.od[obase + no_l] = (int32_t)(G + dj - gi);
              }
              ++no_l;
            }
          }
          const bool rem = (j + 1 < E) && (G + m.tg[j + 1] + m.td[j + 1] <= T);
          if (rem) {
            c = G;
          } else {
            if (write) {
              m.ov[obase + no_l] = m.tv[j];
              m.og[obase + no_l] = (int32_t)G;
              m.od[obase + no_l] = (int32_t)dj;
            }
            ++no_l;
            c = 0;
          }
        }
        cnt_out = no_l;
        return c;
      };
      int64_t cin = 0;
      int cnt_blk = 0;
      for (int round = 0; round <= 64; ++round) {
        const int64_t cout = walk(cin, cnt_blk, 0, false);
        int64_t ncin = __shfl_up(cout, 1, 64);
        if (lane == 0) ncin = 0;
        if (__ballot(ncin != cin) == 0) break;
        cin = ncin;
      }
      // the tail (gk:85-92), on the lane owning the last entry
      const int tail_lane = E == 0 ? 0 : (E - 1) / K;
      const int t0 = E == 0 ? 0 : ga[E - 1];
      int cnt_tail = 0;
      if (lane == tail_lane) {
        int64_t acc = 0;
        for (int i = t0; i < M; ++i) {
          acc += m.ig[i];
          if (i + 1 < M && acc + m.ig[i + 1] + m.id[i + 1] <= T) continue;  // into record i+1
          ++cnt_tail;
          acc = 0;
        }
      }
      const int mine = (j0 < E ? cnt_blk : 0) + cnt_tail;
      const uint32_t incl = wave_incl_scan_u32((uint32_t)mine, lane);
      const int total = __builtin_amdgcn_readlane((int)incl, 63);
      if (total > outcap) {
        if (lane == 0) sh_out = -1;
      } else {
        const int obase = (int)incl - mine;
        int wrote = 0;
        if (j0 < E) walk(cin, wrote, obase, true);
        if (lane == tail_lane) {
          int o = obase + wrote;
          int64_t acc = 0;
          for (int i = t0; i < M; ++i) {
            acc += m.ig[i];
            if (i + 1 < M && acc + m.ig[i + 1] + m.id[i + 1] <= T) continue;
            m.ov[o] = m.iv[i];
            m.og[o] = (int32_t)acc;
            m.od[o] = m.id[i];
            ++o;
            acc = 0;
          }
        }
        if (lane == 0) sh_out = total;
      }
    }
    __syncthreads();
    const int no = sh_out;
    if (no < 0) {
      flag_overflow(a.ovf_count, a.ovf_list, s, lane);
      __syncthreads();
      continue;
    }
    for (int j = lane; j < no; j += 64) {
      GKRec rc;
      rc.v = m.ov[j];
      rc.g = m.og[j];
      rc.d = m.od[j];
      tab[j] = rc;
    }
    if (lane == 0) {
      st.n[s] = n;
      st.E[s] = no;
      st.pend[s] = 0;
    }
    __syncthreads();
  }
}

// ===========================================================================
// state movement
// ===========================================================================
// ctr (gk_reset): the set's slot and member-list counters start over too
// (words [0, GK_CTR_FATAL); FATAL stays cumulative)
__global__ void k_reset(GKState st, int32_t* __restrict__ ctr) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // (+ the per-call block [GK_CTR_CALL, GK_CALL_BYTES): the next call's
  // begin_call then skips its memset -- one dispatch fewer per step)
  if (ctr && (s < GK_CTR_FATAL || (s >= GK_CTR_CALL && s < GK_CALL_BYTES / 4))) ctr[s] = 0;
  if (s >= st.S) return;
  st.n[s] = 0;
  st.E[s] = 0;
  st.pend[s] = 0;
  st.mn[s] = __longlong_as_double(0x7ff0000000000000LL);   // +inf (gk:25)
  st.mx[s] = __longlong_as_double((long long)0xfff0000000000000ULL);  // -inf (gk:26)
  st.sum[s] = 0.0;
  st.avg[s] = 0.0;
  st.cls[s] = 0;  // every stream back in class 0
  st.slot[s] = 0;
}

__global__ void k_export(GKState st, const int64_t* __restrict__ offs, double* __restrict__ v,
                         int32_t* __restrict__ g, int32_t* __restrict__ d) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s = wave; s < st.S; s += nw) {
    const GKRec* tab = gk_table_ptr(st, s);
    const int E = st.E[s];
    const int64_t o = offs[s];
    for (int j = lane; j < E; j += 64) {
      const GKRec rc = tab[j];
      if (v) v[o + j] = rc.v;
      if (g) g[o + j] = rc.g;
      if (d) d[o + j] = rc.d;
    }
  }
}

__global__ void k_export_pending(GKState st, const int64_t* __restrict__ offs, double* __restrict__ v) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s = wave; s < st.S; s += nw) {
    const int p = st.pend[s];
    const double* pb = st.pbuf + s * (int64_t)st.pmax;
    const int64_t o = offs[s];
    for (int j = lane; j < p; j += 64) v[o + j] = pb[j];
  }
}

// gk_import's argument check, before any state is written: a stream's
// pending count p must be one that add() can leave behind -- the values added
// since n last crossed a multiple of P (gk:60), so p <= n mod P (and p = 0
// when n mod P = 0).  A flush batch is then at most P values.
__global__ void k_check_pending(int64_t S, int P, const int64_t* __restrict__ n, const int64_t* __restrict__ poffs,
                                int32_t* __restrict__ bad) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const int64_t p = poffs[s + 1] - poffs[s];
  const int64_t ns = n[s];
  if (p < 0 || ns < 0 || p > ns % P) atomicAdd(bad, 1);
}

__global__ void k_import(GKState st, const int64_t* __restrict__ offs, const double* __restrict__ v,
                         const int32_t* __restrict__ g, const int32_t* __restrict__ d,
                         const int64_t* __restrict__ poffs, const double* __restrict__ pv,
                         int32_t* __restrict__ ovf_count, int32_t* __restrict__ ovf_list) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s = wave; s < st.S; s += nw) {
    const int cap = st.cap[st.cls[s]] - 1;  // k_ingest keeps one slot for padding
    const int64_t o = offs[s];
    const int E = (int)(offs[s + 1] - o);
    const int64_t po = poffs[s];
    const int p = (int)(poffs[s + 1] - po);
    if (E > cap || p > st.pmax) {
      if (lane == 0) {
        const int k = atomicAdd(ovf_count, 1);
        ovf_list[k] = (int32_t)s;
      }
      continue;
    }
    GKRec* tab = gk_table_ptr(st, s);
    for (int j = lane; j < E; j += 64) {
      GKRec rc;
      rc.v = v[o + j];
      rc.g = g[o + j];
      rc.d = d[o + j];
      tab[j] = rc;
    }
    double* pb = st.pbuf + s * (int64_t)st.pmax;
    for (int j = lane; j < p; j += 64) pb[j] = pv[po + j];
    if (lane == 0) {
      st.E[s] = E;
      st.pend[s] = p;
    }
  }
}

// move each listed stream's table into its (already assigned) slot of class `ncls`
__global__ void k_promote(GKState st, const int32_t* __restrict__ list, int64_t count,
                          const int32_t* __restrict__ slots, int ncls) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t w = wave; w < count; w += nw) {
    const int64_t s = list[w];
    const int32_t slot = slots[w];
    const GKRec* src = gk_table_ptr(st, s);
    GKRec* dst = st.tab[ncls] + (int64_t)slot * st.cap[ncls];
    const int E = st.E[s];
    for (int j = lane; j < E; j += 64) dst[j] = src[j];
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      st.cls[s] = ncls;
      st.slot[s] = slot;
    }
  }
}

// Device-side promotion (no host round trip): every stream on the list
// (count from the device) moves to class t = cls+1 (level < 0: an ingest
// overflow) or t = level when it is below that class (level >= 0: a merge at
// capacity level `level`).  Its slot comes from the class's device counter;
// the table is copied over, the stream joins the class member list and, for
// ingest, the re-run list of this round.  The stream's state was not
// committed, so it stays as it is when it cannot move: no free slot in its
// next class -> the defer list (the host grows the arena and re-runs it before
// the set's next call); no class above -> ctr[GK_CTR_FATAL], reported as a
// (sticky) GK_E_OVERFLOW.
__global__ void k_promote_dev(GKState st, const int32_t* __restrict__ count, const int32_t* __restrict__ list,
                              int level, GKPoolDev pool) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t cnt = *count;
  for (int64_t w = wave; w < cnt; w += nw) {
    const int64_t s = list[w];
    const int c = st.cls[s];
    const int t = level < 0 ? c + 1 : level;  // -1: ingest overflow, -2: import overflow
    if (level >= 0 && c >= t) continue;      // already large enough
    int slot = -1;
    if (lane == 0) {
      if (t < st.nclass) {
        slot = atomicAdd(&pool.ctr[GK_CTR_USED + t], 1);
        if (slot >= st.alloc[t]) {
          atomicSub(&pool.ctr[GK_CTR_USED + t], 1);
          slot = -1;
          if (level == -1) pool.defer[atomicAdd(&pool.ctr[GK_CTR_DEFER], 1)] = (int32_t)s;
          else atomicAdd(&pool.ctr[GK_CTR_FATAL], 1);  // (merge / import grow the arena first)
        }
      } else {
        atomicAdd(&pool.ctr[GK_CTR_FATAL], 1);
        atomicMax(&pool.ctr[GK_CTR_FATAL + 1], (int)s);
      }
    }
    slot = __shfl(slot, 0, 64);
    if (slot < 0) continue;
    const GKRec* src = gk_table_ptr(st, s);
    GKRec* dst = st.tab[t] + (int64_t)slot * st.cap[t];
    const int E = min(st.E[s], st.cap[c]);
    for (int j = lane; j < E; j += 64) dst[j] = src[j];
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      st.cls[s] = t;
      st.slot[s] = slot;
      pool.list[t][atomicAdd(&pool.ctr[GK_CTR_LCNT + t], 1)] = (int32_t)s;
      if (level == -1) pool.rerun[t][atomicAdd(&pool.rcnt[t], 1)] = (int32_t)s;
    }
  }
}

// ===========================================================================
// host-side launchers (called from gk_capi.cpp)
// ===========================================================================
// Host-side values cached per device (a set's calls run on its own device,
// made current by the caller): the CU count and each launcher's occupancy
// query (a host API call of several us), one relaxed atomic slot per device.
#define GK_MAX_DEV 64
template <typename Q>
static int per_device(std::atomic<int> (&cache)[GK_MAX_DEV], Q query) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::atomic<int>& c = cache[(unsigned)dev % GK_MAX_DEV];
  int v = c.load(std::memory_order_relaxed);
  if (v <= 0) {
    v = query(dev);
    if (v <= 0) v = 1;
    c.store(v, std::memory_order_relaxed);
  }
  return v;
}

static int num_cu() {
  static std::atomic<int> cache[GK_MAX_DEV];
  return per_device(cache, [](int dev) {
    hipDeviceProp_t prop;
    return hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0 ? prop.multiProcessorCount
                                                                                           : 256;
  });
}

int gk_num_cu() { return num_cu(); }

// GK_WG_EARLY: k_ingest_wg's GK_WG_MAX workgroups (one per CU: 128 KiB of
// LDS each) are launched ahead of k_long_prep and spin until it has run, so
// the device must keep CUs free for it: at least as many again as the early
// grid holds (else the call launches them behind k_long_prep, as with
// GK_WG_EARLY=0).
int gk_wg_early_ok() { return num_cu() >= 2 * GK_WG_MAX; }

template <int CAP, int VPL>
static hipError_t launch_ingest_t(const GKState& st, const double* x, const int64_t* offs,
                                  const int32_t* list, int64_t count, const int32_t* count_ptr, int lcls,
                                  int force, int cap,
                                  unsigned char* ws, size_t ws_bytes, int64_t ws_blocks,
                                  int32_t* ovf_count, int32_t* ovf_list, const GKQuery& q,
                                  unsigned long long* work, const int32_t* prio, const int32_t* prio_count,
                                  const double* psort, const int64_t* prio_ws, const int32_t* prio_skip, hipStream_t stream,
                                  const GKPoolDev& pool, int pmode) {
  if (count <= 0 && !count_ptr) return hipSuccess;
  if (!work) return hipErrorInvalidValue;
  int64_t grid;
  if (CAP > 0) {
    // one resident wave per slot; streams are handed out through `work`
    // (the occupancy query is a host API call of several us: once per kernel)
    static std::atomic<int> occ_cache[GK_MAX_DEV];
    const int occ = per_device(occ_cache, [](int) {
      int o = 0;
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_ingest<CAP, VPL>, 64, 0);
      return o;
    });
    grid = (int64_t)num_cu() * occ;
  } else {
    grid = ws_blocks;
  }
  if (!prio && !count_ptr && grid > count) grid = count;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((k_ingest<CAP, VPL>), dim3((unsigned)grid), dim3(64), 0, stream, st, x, offs, list,
                     count, count_ptr, lcls, force, cap, ws, ws_bytes, ovf_count, ovf_list, q.qs, q.nq, q.out,
                     q.mode, work, prio, prio_count, psort, prio_ws, prio_skip, pool, pmode);
  return hipGetLastError();
}

template <int CAP>
static hipError_t launch_ingest_vpl(int vpl, const GKState& st, const double* x, const int64_t* offs,
                                    const int32_t* list, int64_t count, const int32_t* count_ptr, int lcls,
                                    int force, int cap, unsigned char* ws,
                                    size_t ws_bytes, int64_t ws_blocks, int32_t* ovf_count, int32_t* ovf_list,
                                    const GKQuery& q, unsigned long long* work, const int32_t* prio,
                                    const int32_t* prio_count, const double* psort, const int64_t* prio_ws, const int32_t* prio_skip,
                                    hipStream_t stream, const GKPoolDev& pool, int pmode) {
#define GK_L(V) launch_ingest_t<CAP, V>(st, x, offs, list, count, count_ptr, lcls, force, cap, ws, ws_bytes, ws_blocks, \
                                        ovf_count, ovf_list, q, work, prio, prio_count, psort, prio_ws, prio_skip, stream, \
                                        pool, pmode)
  switch (vpl) {
    case 1: return GK_L(1);
    case 2: return GK_L(2);
    case 4: return GK_L(4);
    case 8: return GK_L(8);
    case 16: return GK_L(16);
    default: return hipErrorInvalidValue;
  }
#undef GK_L
}

template <int VPL>
static hipError_t launch_ingest_small(const GKState& st, const double* x, const int64_t* offs, const int32_t* list,
                                      int64_t count, int force, int32_t* ovf_count, int32_t* ovf_list,
                                      const GKQuery& q, unsigned long long* work, int fused_stats,
                                      hipStream_t stream, hipEvent_t ev0, hipEvent_t ev1) {
  if (count <= 0) return hipSuccess;
  if (!work) return hipErrorInvalidValue;
  const bool fs_launch = fused_stats > 0 && x && !list;
  // Two builds of each kernel: GK_SMALL_WAVES (7) waves per SIMD, and 6 for
  // launches of few streams per wave (occupancy queried once per device and
  // kernel: the register counts may differ).
  static std::atomic<int> occ_cache[2][2][GK_MAX_DEV];
  auto occ_of = [&](bool fs, bool w6) -> int {
    return per_device(occ_cache[fs][w6], [fs, w6](int) {
      int o = 0;
      if (fs) {
        if (w6) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_ingest_small<VPL, true, 6>, 64, 0);
        else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_ingest_small<VPL, true>, 64, 0);
      } else {
        if (w6) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_ingest_small<VPL, false, 6>, 64, 0);
        else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k_ingest_small<VPL, false>, 64, 0);
      }
      return o;
    });
  };
  // one resident wave per slot; streams are handed out through `work`
  auto full_grid = [&](bool w6) -> int64_t {
    int64_t g = (int64_t)num_cu() * occ_of(fs_launch, w6);
    return std::max<int64_t>(1, std::min<int64_t>(g, count));
  };
  // Few streams per wave (cfg4: 10^4 streams of 10^6 values, 1.4 per wave at
  // 7 waves per SIMD): the launch lasts a wave's share of streams, and the
  // 6-wave build runs each faster (cfg4 80.4 -> 71.2 ms per step); many
  // (cfg3: 140 per wave) -- the 7-wave build's latency hiding wins
  // (profiles/r06/r07_waves_per_simd_ab.txt).  GK_SMALL_W=6|7 forces one.
  static const int w_env = getenv("GK_SMALL_W") ? atoi(getenv("GK_SMALL_W")) : 0;
  static const int few_rounds = getenv("GK_FEW_ROUNDS") ? atoi(getenv("GK_FEW_ROUNDS")) : 4;
  int64_t grid = full_grid(false);
  const int64_t rounds7 = (count + grid - 1) / grid;
  const bool w6 = w_env ? w_env == 6 : (GK_SMALL_WAVES != 6 && rounds7 <= few_rounds);
  if (w6) grid = full_grid(true);
  // stats role: fused_stats/8 waves per CU start with the _sum/_avg chains
  // (only for the batch launch over every stream: x given, no list)
  int nstat = 0;
  if (fs_launch) {
    const int64_t want = std::max<int64_t>(1, (int64_t)num_cu() * fused_stats / 8);  // eighths of a wave per CU
    nstat = (int)(grid < want ? grid : want);
  }
  // pacing needs ingest-only waves in every part (stats waves wait for them)
  const int pace = nstat > 0 && grid >= 4 * (int64_t)nstat && grid >= 8 * GK_WORK_PARTS ? 1 : 0;
  static const int lag = getenv("GK_FS_LAG") ? atoi(getenv("GK_FS_LAG")) : GK_FS_LAG_DEFAULT;
  if (list) return hipErrorInvalidValue;  // class 0 over every stream only
  // (ev0 / ev1: recorded by the dispatch itself -- the kernel's own start and
  // end -- when given)
#define GK_SMALL_LAUNCH(FS_, W_)                                                                              \
  hipExtLaunchKernelGGL((k_ingest_small<VPL, FS_, W_>), dim3((unsigned)grid), dim3(64), 0, stream, ev0, ev1, 0, st, x, \
                        offs, count, force, ovf_count, ovf_list, q.qs, q.nq, q.out, q.mode, work, nstat, pace, lag)
  if (nstat > 0) {
    if (w6) GK_SMALL_LAUNCH(true, 6);
    else GK_SMALL_LAUNCH(true, GK_SMALL_WAVES);
  } else {
    if (w6) GK_SMALL_LAUNCH(false, 6);
    else GK_SMALL_LAUNCH(false, GK_SMALL_WAVES);
  }
#undef GK_SMALL_LAUNCH
  return hipGetLastError();
}

size_t gk_ingest_ws_bytes(int cap, int vpl) { return gk_flush_ws_bytes(cap, vpl); }
size_t gk_big_ws_bytes(int cap, int P) { return gk_big_ws_bytes_dev(cap, P); }

hipError_t gk_launch_ingest_big(int cap, const GKState& st, const double* x, const int64_t* offs,
                                const int32_t* list, int64_t count, const int32_t* count_ptr, int lcls, int force,
                                unsigned char* ws, size_t ws_bytes, int64_t ws_blocks, int32_t* ovf_count,
                                int32_t* ovf_list, const GKQuery& q, unsigned long long* work, int32_t* ctr,
                                hipStream_t stream) {
  if (count <= 0 && !count_ptr) return hipSuccess;
  if (!ws || ws_blocks <= 0 || !work || !ctr || ws_bytes < gk_big_ws_bytes_dev(cap, st.P)) return hipErrorInvalidValue;
  int64_t grid = ws_blocks;
  if (!count_ptr && grid > count) grid = count;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_ingest_big, dim3((unsigned)grid), dim3(64), 0, stream, st, x, offs, list, count, count_ptr,
                     lcls, force, cap, ws, ws_bytes, ovf_count, ovf_list, q.qs, q.nq, q.out, q.mode, work, ctr);
  return hipGetLastError();
}

hipError_t gk_launch_ingest(int cap, int vpl, const GKState& st, const double* x, const int64_t* offs,
                            const int32_t* list, int64_t count, const int32_t* count_ptr, int lcls, int force,
                            unsigned char* ws, size_t ws_bytes,
                            int64_t ws_blocks, int32_t* ovf_count, int32_t* ovf_list, const GKQuery& q,
                            unsigned long long* work, const int32_t* prio, const int32_t* prio_count,
                            const double* psort, const int64_t* prio_ws, const int32_t* prio_skip, int fused_stats,
                            hipStream_t stream, hipEvent_t ev_start, hipEvent_t ev_stop, const GKPoolDev* pool,
                            int pmode) {
  const GKPoolDev nopool{};
  const GKPoolDev& pl = pool ? *pool : nopool;
  if (pmode && !pool) return hipErrorInvalidValue;
  switch (cap) {
    case SMALL_CAP:
      if (list || count_ptr || lcls != 0 || pmode) return hipErrorInvalidValue;  // class 0 over every stream only
      if (vpl == 1)
        return launch_ingest_small<1>(st, x, offs, list, count, force, ovf_count, ovf_list, q, work, fused_stats, stream,
                                      ev_start, ev_stop);
      if (vpl == 2)
        return launch_ingest_small<2>(st, x, offs, list, count, force, ovf_count, ovf_list, q, work, fused_stats, stream,
                                      ev_start, ev_stop);
      return hipErrorInvalidValue;
    case 2048:
      return launch_ingest_vpl<2048>(vpl, st, x, offs, list, count, count_ptr, lcls, force, cap, nullptr, 0, 0,
                                     ovf_count, ovf_list, q, work, prio, prio_count, psort, prio_ws, prio_skip, stream,
                                     pl, pmode);
    default:
      if (!ws || ws_blocks <= 0) return hipErrorInvalidValue;
      return launch_ingest_vpl<0>(vpl, st, x, offs, list, count, count_ptr, lcls, force, cap, ws, ws_bytes,
                                  ws_blocks, ovf_count, ovf_list, q, work, prio, prio_count, psort, prio_ws, prio_skip, stream,
                                  pl, pmode);
  }
}

hipError_t gk_launch_ingest_wg(const GKState& st, const double* x, const int64_t* offs, const int32_t* long_list,
                               const int32_t* wg_count, int lcls, int force, int32_t* ovf_count, int32_t* ovf_list,
                               unsigned long long* work, const GKPresort& ps, hipStream_t stream,
                               const int32_t* go) {
  if (st.S <= 0 || !ps.wg_count || !work) return hipSuccess;
  // (at most GK_WG_MAX streams: the count is only known on the device; the
  // spare workgroups find the hand-out exhausted and leave)
  // raised wave priority (GK_WG_PRIO=0: off): the workgroups' flush chains
  // are the cfg5 critical path; co-resident waves of the one-wave launch and
  // the chain walks wait (cfg5 39.4 -> 39.15 ms, profiles/r05/r05x_*)
  static const int wg_prio = getenv("GK_WG_PRIO") ? atoi(getenv("GK_WG_PRIO")) : 1;
  hipLaunchKernelGGL(k_ingest_wg, dim3(GK_WG_MAX), dim3(GK_WG_T), 0, stream, st, x, offs, long_list, wg_count, lcls,
                     force, ovf_count, ovf_list, work, (const double*)ps.ws, (const int64_t*)ps.list_ws,
                     (const int32_t*)ps.done, ps.done ? gk_presort_reg_grid(st) : 0, wg_prio, go);
  return hipGetLastError();
}

hipError_t gk_launch_stats(const GKState& st, const int64_t* offs, int32_t* long_list, int32_t* long_count,
                           hipStream_t stream) {
  if (st.S <= 0) return hipSuccess;
  const int64_t grid = (st.S + 255) / 256;
  // the long-stream list first (k_lengths, a few us), so that the caller can
  // fork k_stats_long -- the sequential chains of the longest streams, the
  // critical path of a Zipf batch -- before the short streams' chains
  // (gk_launch_stats_short) run on this stream
  hipLaunchKernelGGL(k_lengths, dim3((unsigned)grid), dim3(256), 0, stream, st, offs, long_list, long_count);
  return hipGetLastError();
}

hipError_t gk_launch_long_prep(const GKState& st, const int64_t* offs, int32_t* long_list, int64_t* long_n,
                               int32_t* long_count, const GKPresort& ps, hipStream_t stream, int32_t* go) {
  if (st.S <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_long_prep, dim3(1), dim3(1024), 0, stream, st, offs, long_list, long_n,
                     (const int32_t*)long_count, ps.list_ws, ps.list_b0, ps.ws_cap, ps.ws_need, ps.wg_count,
                     ps.wg_presort, go);
  return hipGetLastError();
}

hipError_t gk_launch_stats_short(const GKState& st, const double* x, const int64_t* offs, hipStream_t stream) {
  if (st.S <= 0) return hipSuccess;
  const int64_t ngroups = (st.S + 63) / 64;
  const int64_t grid = std::min<int64_t>(ngroups, (int64_t)num_cu() * 16);
  hipLaunchKernelGGL(k_stats_short, dim3((unsigned)grid), dim3(64), 0, stream, st, x, offs);
  return hipGetLastError();
}

int gk_presort_reg_grid(const GKState& st) {
  static const int reg = getenv("GK_PRESORT_REG") ? atoi(getenv("GK_PRESORT_REG")) : 1;
  return (reg && st.P <= 64 * GK_PS_R) ? num_cu() * 16 : 0;
}

hipError_t gk_launch_presort(const GKState& st, const double* x, const int64_t* offs, const int32_t* long_list,
                             const int64_t* long_n, const int32_t* long_count, const GKPresort& ps,
                             hipStream_t stream) {
  if (st.S <= 0 || !ps.list_ws || !ps.ws || ps.ws_cap <= 0) return hipSuccess;
  // one wave per batch in registers (k_presort_reg, P <= 1024); GK_PRESORT_REG=0
  // or larger batches: the LDS sort of k_presort
  if (gk_presort_reg_grid(st) > 0)
    hipLaunchKernelGGL(k_presort_reg, dim3((unsigned)gk_presort_reg_grid(st)), dim3(64), 0, stream, st, x, offs,
                       long_list, long_count, long_n, (const int64_t*)ps.list_ws, (const int64_t*)ps.list_b0, ps.ws,
                       ps.done);
  else
    hipLaunchKernelGGL(k_presort, dim3((unsigned)(num_cu() * 8)), dim3(256), 0, stream, st, x, offs, long_list,
                       long_count, long_n, (const int64_t*)ps.list_ws, (const int64_t*)ps.list_b0, ps.ws);
  return hipGetLastError();
}

hipError_t gk_launch_stats_long(const GKState& st, const double* x, const int64_t* offs, const int32_t* long_list,
                                const int64_t* long_n, const int32_t* long_count, const int32_t* hc_count,
                                hipStream_t stream) {
  if (st.S <= 0) return hipSuccess;
  // the long-stream count is only known on the device: a fixed grid of waves
  // reads it (an empty list costs one short launch)
  // (GK_SL_PRIO=0: the one-wave-per-stream walk without raised wave
  // priority; with it the critical chains' waves win the SIMD's issue
  // arbitration over the co-resident ingest waves)
  static const int sl_prio = getenv("GK_SL_PRIO") ? atoi(getenv("GK_SL_PRIO")) : 1;
  hipLaunchKernelGGL(k_stats_long, dim3((unsigned)(num_cu() * 4)), dim3(64), 0, stream, st, x, offs, long_list,
                     long_n, long_count, hc_count, sl_prio);
  return hipGetLastError();
}

hipError_t gk_launch_hc_prep(const GKState& st, const int64_t* offs, const int32_t* long_list, const int64_t* long_n,
                             const int32_t* long_count, int64_t min_len, int rel_pct, int64_t budget_factor,
                             GKHostChainRec* recs, int32_t* hc_count, hipStream_t stream) {
  static_assert(GK_HC_MAX == 256, "k_hc_prep: one thread per record");
  if (st.S <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hc_prep, dim3(1), dim3(GK_HC_MAX), 0, stream, st, offs, long_list, long_n, long_count, min_len,
                     rel_pct, budget_factor, recs, hc_count);
  return hipGetLastError();
}

hipError_t gk_launch_hc_apply(const GKState& st, const GKHostChainRec* recs, const int32_t* hc_count,
                              const int32_t* fail, hipStream_t stream) {
  if (st.S <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hc_apply, dim3(1), dim3(GK_HC_MAX), 0, stream, st, recs, hc_count, fail);
  return hipGetLastError();
}

hipError_t gk_launch_hc_wait(const unsigned long long* flag, unsigned long long seq, int32_t* fail,
                             double timeout_s, hipStream_t stream) {
  hipLaunchKernelGGL(k_hc_wait, dim3(1), dim3(64), 0, stream, flag, seq, fail,
                     (unsigned long long)(timeout_s * 1e8));
  return hipGetLastError();
}

hipError_t gk_launch_hc_fallback(const GKState& st, const double* x, const int64_t* offs, const int32_t* long_list,
                                 const int64_t* long_n, const int32_t* hc_count, const int32_t* fail,
                                 hipStream_t stream) {
  if (st.S <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hc_fallback, dim3(GK_HC_MAX), dim3(64), 0, stream, st, x, offs, long_list, long_n, hc_count,
                     fail);
  return hipGetLastError();
}

hipError_t gk_launch_query_list(const GKState& st, const int32_t* list, const int32_t* count, const GKQuery& q,
                                bool qfix, hipStream_t stream) {
  if (st.S <= 0 || !q.qs || q.nq <= 0) return hipSuccess;
  // (4 waves per block: num_cu() blocks = 4 waves per CU for the list; the
  // marker fix needs one thread per answer)
  const int64_t grid = std::max<int64_t>(num_cu(), qfix ? (st.S * (int64_t)q.nq + 255) / 256 : 0);
  hipLaunchKernelGGL(k_query_list, dim3((unsigned)grid), dim3(256), 0, stream, st, list, count, q.qs, q.nq,
                     q.mode, q.out, qfix ? 1 : 0);
  return hipGetLastError();
}

size_t gk_merge_lds_bytes(int cap, int pmax) {
  const size_t MR = (size_t)cap + 1, MI = (size_t)cap + 1 + pmax;
  size_t b = 8 * ((size_t)cap + MR + pmax + MI + cap) + 4 * (2 * (size_t)cap + 2 * MR + 2 * MI + 2 * (size_t)cap) + 16;
  return (b + 255) & ~(size_t)255;
}

hipError_t gk_launch_merge(const MergeArgsHost& h, hipStream_t stream) {
  if (h.count <= 0) return hipSuccess;
  MergeArgs a;
  a.dst = h.dst;
  a.src = h.src;
  a.ev = h.ev;
  a.eg = h.eg;
  a.ed = h.ed;
  a.eoffs = h.eoffs;
  a.mode = h.mode;
  a.cap = h.cap;
  a.list = h.list;
  a.count = h.count;
  a.ovf_count = h.ovf_count;
  a.ovf_list = h.ovf_list;
  a.ws = h.ws;
  a.ws_bytes = h.ws_bytes;
  const size_t lds = gk_merge_lds_bytes(h.cap, h.dst.pmax);
  if (h.ws) {
    if (h.ws_bytes < lds || h.ws_blocks <= 0) return hipErrorInvalidValue;
    int64_t grid = h.ws_blocks;
    if (grid > h.count) grid = h.count;
    hipLaunchKernelGGL(k_merge<true>, dim3((unsigned)grid), dim3(64), 0, stream, a);
    return hipGetLastError();
  }
  if (lds > 160 * 1024 - 64) return hipErrorInvalidValue;
  if (lds > 48 * 1024)
    (void)hipFuncSetAttribute((const void*)k_merge<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int64_t grid = (int64_t)num_cu() * 8;
  if (grid > h.count) grid = h.count;
  hipLaunchKernelGGL(k_merge<false>, dim3((unsigned)grid), dim3(64), lds, stream, a);
  return hipGetLastError();
}

__global__ void k_rtab(GKState st) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < st.rtab_n) st.rtab[k] = k == 0 ? 0.0 : 1.0 / (double)k;  // same IEEE division as gk_stat_step
}

hipError_t gk_launch_rtab(const GKState& st, hipStream_t stream) {
  if (!st.rtab || st.rtab_n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_rtab, dim3((unsigned)((st.rtab_n + 255) / 256)), dim3(256), 0, stream, st);
  return hipGetLastError();
}

hipError_t gk_launch_reset(const GKState& st, hipStream_t stream, int32_t* ctr) {
  if (st.S <= 0 && !ctr) return hipSuccess;
  const int64_t grid = (std::max<int64_t>(st.S, GK_CALL_BYTES / 4) + 255) / 256;
  hipLaunchKernelGGL(k_reset, dim3((unsigned)grid), dim3(256), 0, stream, st, ctr);
  return hipGetLastError();
}

static int64_t wave_grid(int64_t S) {
  int64_t g = (S + 3) / 4;
  const int64_t cap = (int64_t)num_cu() * 16;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return g;
}

hipError_t gk_launch_export(const GKState& st, const int64_t* offs, double* v, int32_t* g, int32_t* d,
                            hipStream_t stream) {
  if (st.S <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_export, dim3((unsigned)wave_grid(st.S)), dim3(256), 0, stream, st, offs, v, g, d);
  return hipGetLastError();
}

hipError_t gk_launch_export_pending(const GKState& st, const int64_t* offs, double* v, hipStream_t stream) {
  if (st.S <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_export_pending, dim3((unsigned)wave_grid(st.S)), dim3(256), 0, stream, st, offs, v);
  return hipGetLastError();
}

hipError_t gk_launch_check_pending(int64_t S, int P, const int64_t* n, const int64_t* poffs, int32_t* bad,
                                  hipStream_t stream) {
  if (S <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_check_pending, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, stream, S, P, n, poffs, bad);
  return hipGetLastError();
}

hipError_t gk_launch_import(const GKState& st, const int64_t* offs, const double* v, const int32_t* g,
                            const int32_t* d, const int64_t* poffs, const double* pv, int32_t* ovf_count,
                            int32_t* ovf_list, hipStream_t stream) {
  if (st.S <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_import, dim3((unsigned)wave_grid(st.S)), dim3(256), 0, stream, st, offs, v, g, d,
                     poffs, pv, ovf_count, ovf_list);
  return hipGetLastError();
}

hipError_t gk_launch_promote_dev(const GKState& st, const int32_t* count, const int32_t* list, int level,
                                 const GKPoolDev& pool, hipStream_t stream) {
  hipLaunchKernelGGL(k_promote_dev, dim3((unsigned)(num_cu() * 2)), dim3(256), 0, stream, st, count, list, level,
                     pool);
  return hipGetLastError();
}

hipError_t gk_launch_promote(const GKState& st, const int32_t* list, int64_t count, const int32_t* slots, int ncls,
                             hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_promote, dim3((unsigned)wave_grid(count)), dim3(256), 0, stream, st, list, count, slots,
                     ncls);
  return hipGetLastError();
}

#ifdef GK_TIMELINE
// timeline builds only (tools/launch_timeline.py; not part of include/gk_capi.h)
extern "C" int gk_tl_read(unsigned long long* wave, unsigned long long* sbeg, unsigned long long* send) {
  if (hipDeviceSynchronize() != hipSuccess) return -4;
  if (hipMemcpyFromSymbol(wave, HIP_SYMBOL(gk_tl_wave), sizeof(unsigned long long) * 5 * GK_TL_MAXW) != hipSuccess) return -4;
  if (hipMemcpyFromSymbol(sbeg, HIP_SYMBOL(gk_tl_sbeg), sizeof(unsigned long long) * GK_TL_MAXS) != hipSuccess) return -4;
  return hipMemcpyFromSymbol(send, HIP_SYMBOL(gk_tl_send), sizeof(unsigned long long) * GK_TL_MAXS) == hipSuccess ? 0 : -4;
}
extern "C" int gk_tl_call_read(unsigned long long* c) {
  if (hipDeviceSynchronize() != hipSuccess) return -4;
  return hipMemcpyFromSymbol(c, HIP_SYMBOL(gk_tl_call), sizeof(unsigned long long) * 2) == hipSuccess ? 0 : -4;
}
extern "C" int gk_tl_wg_read(unsigned long long* wg) {
  if (hipDeviceSynchronize() != hipSuccess) return -4;
  return hipMemcpyFromSymbol(wg, HIP_SYMBOL(gk_tl_wg), sizeof(unsigned long long) * 5 * GK_WG_MAX) == hipSuccess ? 0 : -4;
}
#endif
#ifdef GK_PROF
// profiling builds only (not part of include/gk_capi.h)
extern "C" int gk_prof_read(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(gk_prof_acc), sizeof(unsigned long long) * GK_PROF_NSEC) == hipSuccess ? 0 : -4;
}
extern "C" int gk_prof_reset() {
  unsigned long long z[GK_PROF_NSEC] = {0};
  unsigned long long zw[GK_WP_W * GK_WP_N] = {0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(gk_wprof_acc), zw, sizeof(zw)) != hipSuccess) return -4;
  return hipMemcpyToSymbol(HIP_SYMBOL(gk_prof_acc), z, sizeof(z)) == hipSuccess ? 0 : -4;
}
// k_ingest_wg's per-wave marks: [wave][point], GK_WP_W x GK_WP_N
extern "C" int gk_wprof_read(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(gk_wprof_acc), sizeof(unsigned long long) * GK_WP_W * GK_WP_N) == hipSuccess
             ? 0 : -4;
}
#endif
