// gk_xor.h -- lane exchanges (the value of lane ^ J, wave64) on the VALU: DPP
// row / quad permutations and the gfx950 permlane16 / permlane32 swaps, no
// LDS-pipe instruction (ds_swizzle / ds_bpermute share the LDS with the
// flush's table traffic, which bounds k_ingest_small).  Verified against
// ds_bpermute by tools/mb/xor_probe.hip.
#pragma once
#include <hip/hip_runtime.h>

#define GK_DPP_QPERM(a, b, c, d) ((a) | ((b) << 2) | ((c) << 4) | ((d) << 6))
#define GK_DPP_ROW_MIRROR 0x140
#define GK_DPP_ROW_HALF_MIRROR 0x141
#define GK_DPP_ROW_ROR8 0x128


// full permutations (every lane has a source): no `old` operand to
// initialise (v_mov_b32_dpp with bound_ctrl, one instruction)
template <int CTRL>
__device__ __forceinline__ int gk_dppmov(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, true);
}

// lane ^ 16: permlane16_swap exchanges the odd rows of its first operand with
// the even rows of its second; with both = v, row 2k+1 of the first result
// holds row 2k and row 2k of the second holds row 2k+1
__device__ __forceinline__ int gk_xor16(int v, int lane) {
  const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return (lane & 16) ? (int)r[0] : (int)r[1];
}

// lane ^ 32: the same with the two halves of the wave
__device__ __forceinline__ int gk_xor32(int v, int lane) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (lane & 32) ? (int)r[0] : (int)r[1];
}

template <int J>
__device__ __forceinline__ int lane_xor_dpp(int v, int lane) {
  if constexpr (J == 1) return gk_dppmov<GK_DPP_QPERM(1, 0, 3, 2)>(v);
  else if constexpr (J == 2) return gk_dppmov<GK_DPP_QPERM(2, 3, 0, 1)>(v);
  else if constexpr (J == 3) return gk_dppmov<GK_DPP_QPERM(3, 2, 1, 0)>(v);
  else if constexpr (J == 7) return gk_dppmov<GK_DPP_ROW_HALF_MIRROR>(v);
  else if constexpr (J == 15) return gk_dppmov<GK_DPP_ROW_MIRROR>(v);
  else if constexpr (J == 8) return gk_dppmov<GK_DPP_ROW_ROR8>(v);
  else if constexpr (J == 4) return gk_dppmov<GK_DPP_QPERM(3, 2, 1, 0)>(gk_dppmov<GK_DPP_ROW_HALF_MIRROR>(v));
  else if constexpr (J == 16) return gk_xor16(v, lane);
  else if constexpr (J == 31) return gk_xor16(gk_dppmov<GK_DPP_ROW_MIRROR>(v), lane);
  else if constexpr (J == 32) return gk_xor32(v, lane);
  else if constexpr (J == 63) return gk_xor32(gk_xor16(gk_dppmov<GK_DPP_ROW_MIRROR>(v), lane), lane);
  else return __builtin_amdgcn_ds_bpermute((lane ^ J) << 2, v);
}
