// Cross-lane exchange for one 64-wide wavefront on VALU paths (DPP and the gfx950
// permlane swaps) instead of LDS (ds_bpermute): a few cycles per exchange.
#pragma once

#include <hip/hip_runtime.h>

namespace fs {

template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}
// value of lane (lane ^ off), off a power of two <= 32 (a compile-time constant after unrolling)
__device__ __forceinline__ float xor_get(float x, int off, int lane) {
  switch (off) {
    case 1: return dpp<0xB1>(x);                                  // quad_perm [1,0,3,2]
    case 2: return dpp<0x4E>(x);                                  // quad_perm [2,3,0,1]
    case 4: {                                                     // row_shr:4 / row_shl:4
      // both DPP moves run with the full wave active (a branch would leave the source lanes
      // of each move disabled); the pick is bitwise
      const int up = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x114, 0xf, 0xf, false);
      const int dn = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x104, 0xf, 0xf, false);
      const int msk = -((lane >> 2) & 1);
      return __builtin_bit_cast(float, (up & msk) | (dn & ~msk));
    }
    case 8: return dpp<0x128>(x);                                 // row_ror:8
    case 16: {
      const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, x),
                                                      false, false);
      return __builtin_bit_cast(float, (lane & 16) ? r[0] : r[1]);
    }
    default: {
      const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, x),
                                                      false, false);
      return __builtin_bit_cast(float, (lane & 32) ? r[0] : r[1]);
    }
  }
}
// one reduce-scatter level over lane pairs (l, l ^ off): lanes with (lane & off) keep the
// upper element `b`, the others the lower `a`; returns keep + partner's copy of it.
// (Summing both outputs of one permlane swap of (a, b) would save the selects, but this
// compiler folds that sum to r0 + r0 -- verified by scripts/probe/xorget.hip; mixture.hip's
// rs_level issues the swap as inline asm instead, where both outputs survive.)
__device__ __forceinline__ float rs_pair(float a, float b, int off, int lane) {
  const bool h = (lane & off) != 0;
  return (h ? b : a) + xor_get(h ? a : b, off, lane);
}

// Reduce-scatter + all-reduce of CP per-lane partials (CP a power of two <= 32): returns,
// in lane l, the wave-wide sum of v[l / (64/CP)] -- i.e. lanes 4c..4c+3 hold class c's total
// for CP = 16.  Every lane of a class group holds the bitwise same value.
template <int CP>
__device__ __forceinline__ float class_totals(float (&v)[CP], int lane) {
  constexpr int LPC = 64 / CP;
#pragma unroll
  for (int off = 32, L = CP; off >= LPC; off >>= 1, L >>= 1) {
#pragma unroll
    for (int i = 0; i < L / 2; ++i) v[i] = rs_pair(v[i], v[i + L / 2], off, lane);
  }
  float o = v[0];
#pragma unroll
  for (int off = LPC / 2; off >= 1; off >>= 1) o += xor_get(o, off, lane);
  return o;
}
// wave-wide sum, xor butterfly 32 .. 1 (the same order, so the same bits, as the ds_bpermute
// form of common.h's wave_sum); every lane must be active
__device__ __forceinline__ float wave_sum_dpp(float v, int lane) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += xor_get(v, off, lane);
  return v;
}

// max / sum over the class groups of a class_totals layout (lanes l, l^LPC, l^2LPC, ...)
template <int LPC>
__device__ __forceinline__ float class_max(float x, int lane) {
#pragma unroll
  for (int off = LPC; off < 64; off <<= 1) x = fmaxf(x, xor_get(x, off, lane));
  return x;
}
template <int LPC>
__device__ __forceinline__ float class_sum(float x, int lane) {
#pragma unroll
  for (int off = LPC; off < 64; off <<= 1) x += xor_get(x, off, lane);
  return x;
}

}  // namespace fs
