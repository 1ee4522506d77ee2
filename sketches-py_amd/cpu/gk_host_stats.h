// gk:52-59 on host cores: the product host engine's per-value stats step,
// shared by the host engine (gk_cpu.cpp, every stream) and the HIP engine's
// host-walked chains (gk_capi.cpp: the few longest streams of a batch, whose
// dependent float64 `_avg` chain runs ~6x faster on a CPU core than on one
// gfx950 lane; DESIGN.md section 5, "host-walked chains").
//
// Compiled with -ffp-contract=off and without fast-math (both Makefiles): the
// three roundings of gk:54 stay three IEEE roundings, so the results are the
// reference's bit for bit, whichever engine walks the chain.
#pragma once
#include <cstdint>

struct GKHostStats {
  int64_t n;   // _n (gk:52)
  double sum;  // _sum (gk:53)
  double avg;  // _avg (gk:54)
  double mn;   // _min (gk:56-57)
  double mx;   // _max (gk:58-59)
};

// one value (gk:52-59)
inline void gk_host_stat_step(int64_t& n, double& sum, double& avg, double& mn, double& mx, double v) {
  n += 1;
  sum += v;
  avg += (v - avg) * (1.0 / (double)n);
  if (v < mn) mn = v;  // strict: the first occurrence (and a NaN never) wins
  if (v > mx) mx = v;
}

// a run of values in insertion order (the state kept in locals: registers)
inline void gk_host_stat_run(GKHostStats& s, const double* v, int64_t len) {
  int64_t n = s.n;
  double sum = s.sum, avg = s.avg, mn = s.mn, mx = s.mx;
  for (int64_t i = 0; i < len; ++i) gk_host_stat_step(n, sum, avg, mn, mx, v[i]);
  s.n = n;
  s.sum = sum;
  s.avg = avg;
  s.mn = mn;
  s.mx = mx;
}
