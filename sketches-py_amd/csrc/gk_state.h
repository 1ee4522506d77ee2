// gk_state.h -- device-side layout of a set of GKArray streams (shared by the
// HIP kernels and the host runtime).  See DESIGN.md "Data layout in HBM".
#pragma once
#include <stdint.h>

// One GK tuple (gk:8-16): value, g, delta.  16 bytes, so a wave moves 64
// records (1 KiB) per coalesced dwordx4 access.
struct GKRec {
  double v;
  int32_t g;
  int32_t d;
};

#define GK_MAX_CLASSES 4

// Per-set device pointers, passed by value to every kernel.
struct GKState {
  int64_t S;        // number of streams
  double eps;       // gk:22
  double two_eps;   // 2.0*eps, the first product of gk:70
  double inv_eps;   // 1.0/eps, the small-n cutoff of gk:169 / gk:200
  int32_t P;        // flush period int(1.0/eps)+1 (gk:60)
  int32_t pmax;     // pending slots per stream (== P)

  // header, structure of arrays [S]
  int64_t* n;       // _n
  int32_t* E;       // len(entries)
  int32_t* pend;    // len(incoming)
  double* mn;       // _min
  double* mx;       // _max
  double* sum;      // _sum
  double* avg;      // _avg

  // tables by capacity class: class 0 = tab[0] + s*cap[0] (every stream has
  // one); class c > 0 = tab[c] + slot[s]*cap[c] for promoted streams.
  int32_t* cls;     // capacity class of stream s
  int32_t* slot;    // slot of stream s inside its class arena
  GKRec* tab[GK_MAX_CLASSES];
  int32_t cap[GK_MAX_CLASSES];
  int32_t alloc[GK_MAX_CLASSES];  // slots allocated in tab[c] (c > 0; class 0: S)
  int32_t nclass;

  double* pbuf;     // pending values: pbuf + s*pmax, insertion order

  // rtab[k] = 1.0/(double)k for 1 <= k < rtab_n (IEEE division, made once on
  // the device): the gk:54 factor of a wave whose streams share n
  double* rtab;
  int64_t rtab_n;

  // pre-call n of every stream, written by k_stats before an ingest launch:
  // the stats role of k_ingest_small reads it while ingest waves of the same
  // launch rewrite n (scratch, S entries)
  int64_t* n0;
};

__host__ __device__ inline GKRec* gk_table_ptr(const GKState& st, int64_t s) {
  const int32_t c = st.cls[s];
  return c == 0 ? st.tab[0] + s * (int64_t)st.cap[0] : st.tab[c] + (int64_t)st.slot[s] * st.cap[c];
}
