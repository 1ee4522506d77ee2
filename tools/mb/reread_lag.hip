// Is a second read of the same values, a given data distance later, served
// by the caches (L2 / Infinity Cache) or by HBM?  (the
// fused stats role of k_ingest_small re-reads every value of cfg3 some
// distance behind the ingest waves; PMC FETCH_SIZE counts Infinity-Cache
// hits too, so it cannot tell.)
//
// 10^6 "streams" x 1000 doubles (8.0 GB, far beyond the 256 MiB Infinity
// Cache), taken in order by persistent waves (one wave per stream, 64 lanes x
// 16 B per load, all 8 KB in flight at once).  (A first version handed the
// streams out through one atomic counter: at 10^6 hand-outs that counter
// alone held the launch to 12 ms.)
// Mode D = 0: every stream read once.  Mode D > 0: the wave that takes
// stream c also reads stream c - D, i.e. every stream is read a second time
// after D more streams (D x 8 KB of fresh data chip-wide) were handed out.
// If the second read hits a cache the launch takes about as long as D = 0;
// if it goes to HBM, about twice as long (the D = 0 launch streams at close
// to HBM speed).  Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/mb/reread_lag tools/mb/reread_lag.hip
// Result: profiles/r03n_reread_lag.txt
#include <hip/hip_runtime.h>
#include <cstdio>

#define NS 1000000L
#define LEN 1000L

__global__ __launch_bounds__(64) void rd(const double2* __restrict__ x, double* __restrict__ out, long D) {
  // wave w takes streams w, w + G, w + 2G, ...: all waves advance together, so
  // stream c is read at about time c / G x (time per round of G streams)
  double acc = 0.0;
  const long G = gridDim.x;
  for (long c = blockIdx.x; c < NS; c += G) {
    const double2* p = x + c * (LEN / 2);
    const double2* q = x + (c >= D ? c - D : c) * (LEN / 2);
    double2 v[8], w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = j * 64 + threadIdx.x;
      v[j] = k < LEN / 2 ? p[k] : make_double2(0, 0);
    }
    if (D > 0 && c >= D) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = j * 64 + threadIdx.x;
        w[j] = k < LEN / 2 ? q[k] : make_double2(0, 0);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += w[j].x + w[j].y;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j].x + v[j].y;
  }
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}

int main() {
  double* x = nullptr;
  double* out = nullptr;
  unsigned long long* ctr = nullptr;
  if (hipMalloc(&x, NS * LEN * sizeof(double)) != hipSuccess) return 1;
  const int grid = 256 * 24;  // 6 waves per SIMD, like k_ingest_small (one per 64-thread block)
  if (hipMalloc(&out, grid * 64 * sizeof(double)) != hipSuccess) return 1;
  if (hipMalloc(&ctr, 8) != hipSuccess) return 1;
  (void)hipMemset(x, 0, NS * LEN * sizeof(double));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const long Ds[] = {0, 256, 1024, 4096, 8192, 16384, 32768, 65536, 262144};
  printf("8.0 GB streamed by %d waves; D = streams handed out between a stream's two reads\n", grid);
  for (int rep = 0; rep < 2; ++rep) {
    for (long D : Ds) {
            (void)hipEventRecord(a);
      hipLaunchKernelGGL(rd, dim3(grid), dim3(64), 0, 0, (const double2*)x, out, D);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      const double gb = (NS + (D > 0 && D < NS ? NS - D : 0)) * LEN * 8.0 / 1e9;  // streams c >= D are read twice
      if (rep)
        printf("D=%6ld (%7.1f MB between reads)  %7.3f ms  %6.2f TB/s of reads (%s)\n", D, D * LEN * 8.0 / 1e6, ms,
               gb / ms, D ? "streams past D twice" : "each value once");
    }
  }
  return 0;
}
