// cpu_selftest.cpp -- TEST INFRASTRUCTURE: drives the host engine
// (sketches-py_amd/cpu/gk_cpu.cpp, through include/gk_capi.h + gk_cpu.h) and
// the C oracle (oracle/gk_oracle.c) on the same seeded random workloads and
// requires identical state.  Built with ASan + UBSan by
// `make -C sketches-py_amd/cpu sanitize` (sanitizers on the host
// code); tests/test_cpu_sanitize.py runs it.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <random>
#include <vector>

#include "gk_cpu.h"

extern "C" {
typedef struct gko_set gko_set;
gko_set* gko_create(int64_t S, double eps);
void gko_destroy(gko_set* h);
int gko_ingest(gko_set* h, const double* values, const int64_t* offs, int nthreads);
int gko_flush(gko_set* h, int force, int nthreads);
int gko_quantiles(gko_set* h, const double* qs, int nq, double* out, int mode, int nthreads);
int gko_merge(gko_set* dst, gko_set* src, int nthreads);
void gko_stats(const gko_set* h, int64_t* n, double* mn, double* mx, double* sum, double* avg, int32_t* E,
               int32_t* p);
void gko_export(const gko_set* h, const int64_t* offs, double* v, int64_t* g, int64_t* d);
void gko_export_pending(const gko_set* h, const int64_t* offs, double* v);
}

static int failures = 0;
#define CHECK(c, ...)                   \
  do {                                  \
    if (!(c)) {                         \
      fprintf(stderr, __VA_ARGS__);     \
      fprintf(stderr, "\n");            \
      ++failures;                       \
      return;                           \
    }                                   \
  } while (0)

static bool same_bits(double a, double b) { return memcmp(&a, &b, 8) == 0 || (std::isnan(a) && std::isnan(b)); }

static void compare(gk_set* a, gko_set* o, int64_t S, const char* what) {
  std::vector<int64_t> n1(S), n2(S);
  std::vector<double> f1(4 * S), f2(4 * S);
  std::vector<int32_t> e1(S), e2(S), p1(S), p2(S);
  gk_stats(a, n1.data(), f1.data(), f1.data() + S, f1.data() + 2 * S, f1.data() + 3 * S, e1.data(), p1.data(),
           nullptr);
  gko_stats(o, n2.data(), f2.data(), f2.data() + S, f2.data() + 2 * S, f2.data() + 3 * S, e2.data(), p2.data());
  for (int64_t s = 0; s < S; ++s) {
    CHECK(n1[s] == n2[s] && e1[s] == e2[s] && p1[s] == p2[s], "%s: stream %lld sizes", what, (long long)s);
    for (int k = 0; k < 4; ++k) CHECK(same_bits(f1[k * S + s], f2[k * S + s]), "%s: stream %lld stat %d", what,
                                      (long long)s, k);
  }
  std::vector<int64_t> off(S + 1, 0), poff(S + 1, 0);
  for (int64_t s = 0; s < S; ++s) {
    off[s + 1] = off[s] + e1[s];
    poff[s + 1] = poff[s] + p1[s];
  }
  const int64_t E = off[S], P = poff[S];
  std::vector<double> v1(E + 1), v2(E + 1), pv1(P + 1), pv2(P + 1);
  std::vector<int32_t> g1(E + 1), d1(E + 1);
  std::vector<int64_t> g2(E + 1), d2(E + 1);
  gk_export(a, off.data(), v1.data(), g1.data(), d1.data(), nullptr);
  gko_export(o, off.data(), v2.data(), g2.data(), d2.data());
  gk_export_pending(a, poff.data(), pv1.data(), nullptr);
  gko_export_pending(o, poff.data(), pv2.data());
  for (int64_t k = 0; k < E; ++k)
    CHECK(same_bits(v1[k], v2[k]) && g1[k] == g2[k] && d1[k] == d2[k], "%s: record %lld", what, (long long)k);
  for (int64_t k = 0; k < P; ++k) CHECK(same_bits(pv1[k], pv2[k]), "%s: pending %lld", what, (long long)k);
}

static std::vector<double> gen(std::mt19937_64& rng, int dist, int64_t L) {
  std::vector<double> x(L);
  std::uniform_real_distribution<double> u(0, 1);
  std::lognormal_distribution<double> ln(0, 1);
  std::uniform_int_distribution<int> small(0, 4);
  for (int64_t i = 0; i < L; ++i) {
    switch (dist) {
      case 0: x[i] = u(rng); break;
      case 1: x[i] = ln(rng); break;
      case 2: x[i] = (double)(L - i); break;  // descending
      case 3: x[i] = (double)small(rng); break;
      default: x[i] = (small(rng) & 1) ? 0.0 : -0.0; break;
    }
  }
  return x;
}

static void run(double eps, int64_t S, uint64_t seed) {
  std::mt19937_64 rng(seed);
  const int64_t P = (int64_t)(1.0 / eps) + 1;
  gk_set* a = nullptr;
  gk_set* b = nullptr;
  if (gk_create(S, eps, 0, -1, &a) != GK_OK || gk_create(S, eps, 0, -1, &b) != GK_OK) {
    ++failures;
    return;
  }
  gk_cpu_set_threads(a, 4);
  gko_set* o = gko_create(S, eps);
  gko_set* ob = gko_create(S, eps);
  char what[64];
  for (int part = 0; part < 3; ++part) {
    std::vector<double> flat;
    std::vector<int64_t> offs(S + 1, 0);
    std::vector<double> fb;
    std::vector<int64_t> ob_offs(S + 1, 0);
    for (int64_t s = 0; s < S; ++s) {
      auto x = gen(rng, (int)(rng() % 5), (int64_t)(rng() % (4 * P)));
      flat.insert(flat.end(), x.begin(), x.end());
      offs[s + 1] = (int64_t)flat.size();
      auto y = gen(rng, (int)(rng() % 5), (int64_t)(rng() % (3 * P)));
      fb.insert(fb.end(), y.begin(), y.end());
      ob_offs[s + 1] = (int64_t)fb.size();
    }
    flat.push_back(0);
    fb.push_back(0);
    gk_ingest(a, flat.data(), offs.data(), nullptr);
    gko_ingest(o, flat.data(), offs.data(), 1);
    gk_ingest(b, fb.data(), ob_offs.data(), nullptr);
    gko_ingest(ob, fb.data(), ob_offs.data(), 1);
    snprintf(what, sizeof(what), "eps=%g ingest %d", eps, part);
    compare(a, o, S, what);
    const double qs[4] = {0.01, 0.5, 0.9, 1.0};
    std::vector<double> q1(4 * S), q2(4 * S);
    gk_quantiles(a, qs, 4, q1.data(), GK_Q_LIST, nullptr);
    gko_flush(o, 1, 1);  // the oracle's caller flushes (gk:197-198)
    gko_quantiles(o, qs, 4, q2.data(), 0, 1);
    for (int64_t k = 0; k < 4 * S; ++k) {
      if (!same_bits(q1[k], q2[k])) {
        fprintf(stderr, "%s: quantile %lld\n", what, (long long)k);
        ++failures;
        break;
      }
    }
    gk_set* srcs[1] = {b};
    gk_merge(a, srcs, 1, nullptr);
    gko_merge(o, ob, 1);
    snprintf(what, sizeof(what), "eps=%g merge %d", eps, part);
    compare(a, o, S, what);
    compare(b, ob, S, "merge source");
  }
  gk_destroy(a);
  gk_destroy(b);
  gko_destroy(o);
  gko_destroy(ob);
}

int main() {
  const double eps[] = {0.2, 0.05, 0.01, 0.001};
  for (int k = 0; k < 4; ++k) run(eps[k], eps[k] >= 0.01 ? 300 : 40, 1000 + k);
  if (failures) {
    fprintf(stderr, "cpu_selftest: %d failure(s)\n", failures);
    return 1;
  }
  printf("cpu_selftest: ok\n");
  return 0;
}
