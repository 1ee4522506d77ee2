/* Host prototype of the speculative gk:52-54 chain walk (design check for
 * k_stats_long's superstep kernel): 64 "lanes" x W steps per superstep, each
 * lane runs its sub-chunk's _sum/_avg chain from an estimated start, then
 * the spec values are shifted by per-lane offsets (a lane scan) and every
 * step is checked f(b[t]) == b[t+1] bit for bit; the first failure restarts
 * from the true value there.  Compares with the plain sequential chain and
 * counts verification rounds.  gcc -O2 -ffp-contract=off spec_chain.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define L 64
static int W = 32;

static uint64_t bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static double fa(double a, double v, double r) { return a + (v - a) * r; }
static double fs(double s, double v) { return s + v; }

static uint64_t rng = 88172645463325252ull;
static double urand(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return (rng >> 11) * (1.0 / 9007199254740992.0); }
static double lognorm(void) { double u1 = urand(), u2 = urand(); if (u1 < 1e-300) u1 = 1e-300; return exp(sqrt(-2 * log(u1)) * cos(2 * M_PI * u2)); }

/* one chain kind: 0 = avg, 1 = sum.  Returns rounds used. */
static int verify(int kind, double X[L][65], const double* v, const double* r, double T0, double* out_end) {
  /* override: lane jo, step to, true value K */
  int jo = 0, to = 0, rounds = 0;
  double K = T0;
  for (;;) {
    ++rounds;
    double D[L], b[L][65];
    /* lane offsets: lane jo from K, lanes after by a scan of e_j */
    D[jo] = K - X[jo][to];
    for (int j = jo + 1; j < L; ++j) D[j] = D[j - 1] + (X[j - 1][W] - X[j][0]);
    for (int j = jo; j < L; ++j)
      for (int t = (j == jo ? to : 0); t <= W; ++t) b[j][t] = X[j][t] + D[j];
    b[jo][to] = K;
    int fj = -1, ft = -1;
    for (int j = jo; j < L && fj < 0; ++j)
      for (int t = (j == jo ? to : 0); t < W; ++t) {
        const double nxt = (t + 1 < W || j == L - 1) ? b[j][t + 1] : b[j + 1][0];
        const int idx = j * W + t;
        const double f = kind == 0 ? fa(b[j][t], v[idx], r[idx]) : fs(b[j][t], v[idx]);
        if (bits(f) != bits(nxt)) { fj = j; ft = t; K = f; break; }
      }
    if (fj < 0) { *out_end = b[L - 1][W]; return rounds; }
    jo = fj; to = ft + 1;
    if (to == W) { jo++; to = 0; if (jo == L) { *out_end = K; return rounds; } }
  }
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 10000000;
  if (argc > 2) W = atoi(argv[2]);
  const int dist = argc > 3 ? atoi(argv[3]) : 0;
  const int SS = L * W;
  double* x = malloc(sizeof(double) * N);
  for (int64_t i = 0; i < N; ++i) x[i] = dist == 0 ? lognorm() : dist == 1 ? (double)(i % 7) : dist == 2 ? (double)(N - i) : dist == 3 ? pow(urand() + 1e-12, -1.0 / 1.5) : dist == 4 ? (urand() < 0.5 ? -1 : 1) * exp(100 * (urand() - 0.5)) : (urand() < 0.3 ? -0.0 : urand() < 0.5 ? 0.0 : lognorm() - 1.0);
  /* reference chain */
  double ra = 0, rsum = 0;
  for (int64_t i = 0; i < N; ++i) { rsum = rsum + x[i]; ra = ra + (x[i] - ra) * (1.0 / (double)(i + 1)); }
  double A = 0, S = 0;
  int64_t n = 0, ra_rounds = 0, rs_rounds = 0, steps = 0;
  static double XA[L][65], XS[L][65];
  double r[L * 65];
  for (int64_t k0 = 0; k0 + SS <= N; k0 += SS, n += SS) {
    const double* v = x + k0;
    for (int i = 0; i < SS; ++i) r[i] = 1.0 / (double)(n + i + 1);
    /* estimates: lane partial sums, exclusive scan */
    double P[L], Q[L];
    for (int j = 0; j < L; ++j) { double p = 0; for (int t = 0; t < W; ++t) p += v[j * W + t]; P[j] = p; }
    Q[0] = 0; for (int j = 1; j < L; ++j) Q[j] = Q[j - 1] + P[j - 1];
    for (int j = 0; j < L; ++j) {
      double a = j == 0 ? A : (A * (double)n + Q[j]) / (double)(n + (int64_t)j * W);
      double s = S + Q[j];
      XA[j][0] = a; XS[j][0] = s;
      for (int t = 0; t < W; ++t) {
        const int idx = j * W + t;
        a = fa(a, v[idx], r[idx]); s = fs(s, v[idx]);
        XA[j][t + 1] = a; XS[j][t + 1] = s;
      }
    }
    double ea, es;
    ra_rounds += verify(0, XA, v, r, A, &ea);
    rs_rounds += verify(1, XS, v, r, S, &es);
    A = ea; S = es; steps++;
  }
  for (int64_t i = n; i < N; ++i) { S = S + x[i]; A = A + (x[i] - A) * (1.0 / (double)(i + 1)); }
  printf("N=%lld W=%d dist=%d supersteps=%lld avg rounds/superstep: avg %.3f sum %.3f  exact avg %d sum %d\n",
         (long long)N, W, dist, (long long)steps, (double)ra_rounds / steps, (double)rs_rounds / steps,
         bits(A) == bits(ra), bits(S) == bits(rsum));
  return 0;
}
