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

// reduce-scatter level at lane distance OFF over pairs (a, b): lanes with (lane & OFF) keep b
template <int OFF, bool SWAP>
__device__ __forceinline__ float rs_level(float a, float b, int lane) {
  if constexpr (SWAP && (OFF == 32 || OFF == 16)) {
    // inline asm, not the builtin: with a constant-zero partner (padding classes) hipcc
    // 7.2 drops the builtin's second result and sums r0 + 0.  The pad inside the string is
    // the 2 wait states a VALU write of either operand needs before v_permlane*_swap reads it.
    if constexpr (OFF == 32)
      asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    else
      asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    return a + b;
  } else {
    return rs_pair(a, b, OFF, lane);
  }
}

// one reduce-scatter level of a 16-lane row at lane distance 8 or 4: two DPP adds, each
// writing the lanes (DPP banks) that keep one element of the pair: dst = partner's copy of
// that element + own copy (lanes with the OFF bit clear keep lo, the others hi)
template <int OFF>
__device__ __forceinline__ float rs_bank(float lo, float hi) {
  float r;
  if constexpr (OFF == 8)
    asm volatile(
        "s_nop 1\n\t"
        "v_add_f32_dpp %0, %1, %1 row_ror:8 row_mask:0xf bank_mask:0x3\n\t"
        "v_add_f32_dpp %0, %2, %2 row_ror:8 row_mask:0xf bank_mask:0xc"
        : "=&v"(r)
        : "v"(lo), "v"(hi));
  else
    asm volatile(
        "s_nop 1\n\t"
        "v_add_f32_dpp %0, %1, %1 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
        "v_add_f32_dpp %0, %2, %2 row_shr:4 row_mask:0xf bank_mask:0xa"
        : "=&v"(r)
        : "v"(lo), "v"(hi));
  return r;
}

// max / sum over the 16 lanes of a DPP row (rotations 8 and 4, then the quad butterflies:
// every lane of the row ends with bitwise the same value)
template <bool MAX>
__device__ __forceinline__ float row16_all(float x) {
  x = MAX ? fmaxf(x, dpp<0x128>(x)) : x + dpp<0x128>(x);   // row_ror:8
  x = MAX ? fmaxf(x, dpp<0x124>(x)) : x + dpp<0x124>(x);   // row_ror:4
  x = MAX ? fmaxf(x, dpp<0x4E>(x)) : x + dpp<0x4E>(x);     // quad xor 2
  x = MAX ? fmaxf(x, dpp<0xB1>(x)) : x + dpp<0xB1>(x);     // quad xor 1
  return x;
}

// x of lane c of this lane's 16-lane row (gfx950 DPP row_newbcast:c; c a compile-time
// constant after unrolling)
__device__ __forceinline__ float row_get(float x, int c) {
  switch (c) {
    case 0: return dpp<0x150>(x);
    case 1: return dpp<0x151>(x);
    case 2: return dpp<0x152>(x);
    case 3: return dpp<0x153>(x);
    case 4: return dpp<0x154>(x);
    case 5: return dpp<0x155>(x);
    case 6: return dpp<0x156>(x);
    case 7: return dpp<0x157>(x);
    case 8: return dpp<0x158>(x);
    case 9: return dpp<0x159>(x);
    case 10: return dpp<0x15A>(x);
    case 11: return dpp<0x15B>(x);
    case 12: return dpp<0x15C>(x);
    case 13: return dpp<0x15D>(x);
    case 14: return dpp<0x15E>(x);
    default: return dpp<0x15F>(x);
  }
}

// the two values of a permlane swap of x with itself: lo = x of the lane group with the
// OFF bit clear, hi = x of the group with it set (OFF = 16: rows; 32: halves)
template <int OFF>
__device__ __forceinline__ void gather_pair(float x, float& lo, float& hi) {
  float a = x, b = x;
  if constexpr (OFF == 32)
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  else
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  lo = a;
  hi = b;
}

}  // namespace fs
