// Microbenchmark: issue cost on gfx950 of the compare +
// select step of the flush's gap search, on float64 keys against 64- and
// 32-bit integer keys.  One step = xb += (t <= x) ? S : 0 (v_cmp, v_cndmask,
// v_add), 4 independent chains per lane, 8 waves per SIMD, every CU busy.
// Reported per SIMD: cycles per step (s_memtime), so 2 cycles ~ one full-rate
// wave64 VALU instruction.
// Build: hipcc --offload-arch=gfx950 -O3 -o cmp_cost cmp_cost.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <typename T>
__device__ __forceinline__ void opaque(T& v) {
  if constexpr (sizeof(T) == 8) asm volatile("" : "+v"(v));
  else asm volatile("" : "+v"(v));
}

// KIND 0: search step (cmp + select + add); KIND 1: bare compares feeding a
// popcount-free sum (cmp + addc); KIND 2: select only (baseline)
template <typename K, int KIND>
__global__ __launch_bounds__(256) void k_steps(const K* __restrict__ in, uint32_t* __restrict__ out,
                                               unsigned long long* __restrict__ cyc, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  K x = in[tid & 1023];
  K t0 = in[(tid + 1) & 1023], t1 = in[(tid + 7) & 1023], t2 = in[(tid + 13) & 1023], t3 = in[(tid + 29) & 1023];
  uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  const uint32_t S = 8u + (uint32_t)(tid & 3);
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      opaque(t0); opaque(t1); opaque(t2); opaque(t3);
      if constexpr (KIND == 0) {
        a0 += (t0 <= x) ? S : 0u;
        a1 += (t1 <= x) ? S : 0u;
        a2 += (t2 <= x) ? S : 0u;
        a3 += (t3 <= x) ? S : 0u;
      } else {
        a0 += (t0 <= x);
        a1 += (t1 <= x);
        a2 += (t2 <= x);
        a3 += (t3 <= x);
      }
    }
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  out[tid] = a0 + a1 + a2 + a3;
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, c1 - c0);
}

template <typename K, int KIND>
void run(const char* name, const void* din, uint32_t* out, unsigned long long* cyc, int iters) {
  const int blocks = 256 * 8, threads = 256;  // 2048 threads per CU = 8 waves per SIMD
  unsigned long long h = 0;
  for (int rep = 0; rep < 2; ++rep) {
    hipMemset(cyc, 0, 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    k_steps<K, KIND><<<blocks, threads>>>((const K*)din, out, cyc, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    const double waves = blocks * threads / 64.0;
    const double steps_per_wave = (double)iters * 8 * 4;
    const double wave_cyc = h / waves;                    // elapsed cycles of one wave
    const double per_simd = wave_cyc / (8.0 * steps_per_wave);  // 8 waves share a SIMD
    const double wall_per_simd = ms * 1e-3 * 2.4e9 * 1024 / (waves * steps_per_wave);
    if (rep) printf("%-34s %6.2f cycles/step/SIMD (s_memtime)  %6.2f (wall @2.4GHz)  %.3f ms\n", name, per_simd,
                    wall_per_simd, ms);
  }
}

int main() {
  void* din;
  uint32_t* out;
  unsigned long long* cyc;
  hipMalloc(&din, 1024 * 8);
  hipMalloc(&out, 256 * 8 * 256 * 4);
  hipMalloc(&cyc, 8);
  double h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = 1.0 + (i * 7919 % 1024) * 1e-3;
  hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  const int iters = 4000;
  run<double, 0>("f64 search step (cmp+sel+add)", din, out, cyc, iters);
  run<unsigned long long, 0>("u64 search step (cmp+sel+add)", din, out, cyc, iters);
  run<uint32_t, 0>("u32 search step (cmp+sel+add)", din, out, cyc, iters);
  run<double, 1>("f64 compare + count", din, out, cyc, iters);
  run<unsigned long long, 1>("u64 compare + count", din, out, cyc, iters);
  run<uint32_t, 1>("u32 compare + count", din, out, cyc, iters);
  return 0;
}
