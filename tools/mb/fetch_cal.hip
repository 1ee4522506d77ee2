// Calibration of rocprofv3 FETCH_SIZE for the two read patterns of the
// small-class launch (k_ingest_small), over an 8 GB buffer far larger than
// the 256 MiB Infinity Cache (every byte comes from HBM once):
//   mode 0 "ingest": a wave per stream, 64 lanes x 8 B contiguous per load
//                    (the flush values: 512 B per wave-instruction);
//   mode 1 "stats":  a lane per stream, 64 streams per wave, aligned 16-byte
//                    loads walking each stream in order, 2 x 64 B in flight
//                    per lane (the fused stats role's register ring).
// Each mode reads 10^6 streams x 1000 doubles = 8.0 GB exactly once; FETCH
// of one launch / 8.0 GB is the counting factor of that pattern (the
// guide's 1/2 holds for wide coalesced reads).  Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/mb/fetch_cal tools/mb/fetch_cal.hip
// Run: rocprofv3 --pmc FETCH_SIZE --kernel-trace -- tools/mb/fetch_cal
// Result: profiles/r02Ze_fetch_calibration.txt
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define NS 1000000L
#define LEN 1000L

__global__ __launch_bounds__(64) void rd_ingest(const double* __restrict__ x, double* __restrict__ out) {
  // grid-stride over streams, one wave per stream (like the ingest waves)
  double acc = 0.0;
  for (long s = blockIdx.x; s < NS; s += gridDim.x) {
    const double* p = x + s * LEN;
    for (int k = threadIdx.x; k < LEN; k += 64) acc += p[k];
  }
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(64) void rd_stats(const double* __restrict__ x, double* __restrict__ out) {
  // 64 streams per wave, one per lane; 16-byte loads, ring of 2 x 4 loads
  double acc = 0.0;
  for (long g = blockIdx.x; g < NS / 64; g += gridDim.x) {
    const double2* p = (const double2*)(x + (g * 64 + threadIdx.x) * LEN);
    double2 r0[4], r1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) r0[j] = p[j];
#pragma unroll
    for (int j = 0; j < 4; ++j) r1[j] = p[4 + j];
    for (int c = 0; c < LEN / 8; c += 2) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc += r0[j].x + r0[j].y;
      if (c + 2 < LEN / 8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) r0[j] = p[(c + 2) * 4 + j];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc += r1[j].x + r1[j].y;
      if (c + 3 < LEN / 8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) r1[j] = p[(c + 3) * 4 + j];
      }
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}

int main() {
  double *x = nullptr, *out = nullptr;
  const size_t bytes = (size_t)NS * LEN * sizeof(double);
  const int grid_i = 256 * 24, grid_s = 256 * 4;  // out holds one double per thread of the larger grid
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&out, (size_t)grid_i * 64 * sizeof(double)) != hipSuccess) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  hipError_t e = hipMemset(x, 0, bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    fprintf(stderr, "memset: %s\n", hipGetErrorString(e));
    return 1;
  }
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int rep = 0; rep < 2; ++rep) {
    float ms = 0;
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(rd_ingest, dim3(grid_i), dim3(64), 0, 0, x, out);
    if ((e = hipGetLastError()) != hipSuccess) {
      fprintf(stderr, "rd_ingest: %s\n", hipGetErrorString(e));
      return 1;
    }
    (void)hipEventRecord(b);
    if ((e = hipEventSynchronize(b)) != hipSuccess) {
      fprintf(stderr, "sync: %s\n", hipGetErrorString(e));
      return 1;
    }
    (void)hipEventElapsedTime(&ms, a, b);
    printf("rd_ingest %.3f ms  %.1f GB/s\n", ms, bytes / (ms * 1e6));
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(rd_stats, dim3(grid_s), dim3(64), 0, 0, x, out);
    if ((e = hipGetLastError()) != hipSuccess) {
      fprintf(stderr, "rd_stats: %s\n", hipGetErrorString(e));
      return 1;
    }
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    printf("rd_stats  %.3f ms  %.1f GB/s\n", ms, bytes / (ms * 1e6));
  }
  (void)hipFree(x);
  (void)hipFree(out);
  return 0;
}
