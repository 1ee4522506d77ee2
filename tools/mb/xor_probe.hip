// Probe: lane-exchange helpers built from DPP / permlane (gk_kernels.hip
// lane_xor_dpp) against ds_bpermute, for every partner distance the
// first-flush sort uses.  Prints "ok" or the first mismatch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define GK_XOR_PROBE
#include "../../sketches-py_amd/csrc/gk_xor.h"

template <int J>
__global__ void probe(int* bad) {
  const int lane = threadIdx.x;
  const int v = lane * 7 + 1000;
  const int got = lane_xor_dpp<J>(v, lane);
  const int want = __builtin_amdgcn_ds_bpermute((lane ^ J) << 2, v);
  if (got != want) atomicMin(bad, J * 100 + lane);
}

int main() {
  int* d;
  hipMalloc(&d, 4);
  int h = 1 << 30;
  hipMemcpy(d, &h, 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe<1>, 1, 64, 0, 0, d);
  hipLaunchKernelGGL(probe<2>, 1, 64, 0, 0, d);
  hipLaunchKernelGGL(probe<3>, 1, 64, 0, 0, d);
  hipLaunchKernelGGL(probe<4>, 1, 64, 0, 0, d);
  hipLaunchKernelGGL(probe<7>, 1, 64, 0, 0, d);
  hipLaunchKernelGGL(probe<8>, 1, 64, 0, 0, d);
  hipLaunchKernelGGL(probe<15>, 1, 64, 0, 0, d);
  hipLaunchKernelGGL(probe<16>, 1, 64, 0, 0, d);
  hipLaunchKernelGGL(probe<31>, 1, 64, 0, 0, d);
  hipLaunchKernelGGL(probe<32>, 1, 64, 0, 0, d);
  hipLaunchKernelGGL(probe<63>, 1, 64, 0, 0, d);
  hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  if (h == (1 << 30)) printf("xor probe: ok\n");
  else printf("xor probe: mismatch J=%d lane=%d\n", h / 100, h % 100);
  return h == (1 << 30) ? 0 : 1;
}
