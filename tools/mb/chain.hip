// Microbenchmark: latency of the dependent float64 chain of gk:53-54 (_sum / _avg)
// on one wave.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o chain chain.hip
// Result: profiles/r01u_dp_chain_microbench.txt
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void chain(double* out, const double* in, long iters) {
  double av = in[threadIdx.x], sm = 0.0;
  double v0 = in[64 + threadIdx.x], r0 = in[128 + threadIdx.x];
  double v1 = v0 * 1.0000001, r1 = r0 * 0.9999999;
  for (long i = 0; i < iters; i += 2) {
    sm = sm + v0; av = av + (v0 - av) * r0;
    sm = sm + v1; av = av + (v1 - av) * r1;
  }
  out[threadIdx.x] = av + sm;
}
__global__ void chain3(double* out, const double* in, long iters) {  // only the avg chain
  double av = in[threadIdx.x];
  double v0 = in[64 + threadIdx.x], r0 = in[128 + threadIdx.x];
  for (long i = 0; i < iters; ++i) { av = av + (v0 - av) * r0; }
  out[threadIdx.x] = av;
}
__global__ void add1(double* out, const double* in, long iters) {  // one dependent add
  double a = in[threadIdx.x], b = in[64 + threadIdx.x];
  for (long i = 0; i < iters; ++i) { a = a + b; }
  out[threadIdx.x] = a;
}
int main() {
  double *in, *out; hipMalloc(&in, 4096); hipMalloc(&out, 4096);
  double h[512]; for (int i = 0; i < 512; ++i) h[i] = 1.0 + i * 1e-3;
  hipMemcpy(in, h, 4096, hipMemcpyHostToDevice);
  long iters = 10000000;
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  float ms;
  for (int k = 0; k < 2; ++k) {
    hipEventRecord(a); chain<<<1, 64>>>(out, in, iters); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b); printf("sum+avg chain: %.3f ns/value\n", ms * 1e6 / iters);
    hipEventRecord(a); chain3<<<1, 64>>>(out, in, iters); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b); printf("avg chain only: %.3f ns/value\n", ms * 1e6 / iters);
    hipEventRecord(a); add1<<<1, 64>>>(out, in, iters); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b); printf("dependent v_add_f64: %.3f ns/op\n", ms * 1e6 / iters);
  }
  return 0;
}
