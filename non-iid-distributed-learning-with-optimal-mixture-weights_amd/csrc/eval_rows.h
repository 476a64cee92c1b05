// Test-set evaluation of one 16-row group -- THE evaluation body: fs_eval's workgroups
// (eval.hip) and the fused evaluation blocks of local_train_split.hip both run exactly this
// code, so a row's logits, cross-entropy and arg-max are the same bits either way.  NWV waves
// split the 64-column feature tiles, v_mfma_f32_16x16x4_f32 logits over CT class tiles of 16
// (C <= 16 * CT), partials summed through LDS, wave 0 accumulates the rows' cross-entropy and
// correct count (tools.py:218-237).
#pragma once

#include "common.h"

namespace fs {

// zt: NWV * 16 * (16 CT + 1) floats of LDS.  ce / cor accumulate in wave 0's lanes 0-15.
template <int NWV, int CT = 1>
__device__ __forceinline__ void eval_group16(const float* __restrict__ phi, int64_t ld, const int32_t* __restrict__ y,
                                             int n, const float* __restrict__ W, int C, int r0, float* zt, double& ce,
                                             double& cor) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l16 = lane & 15, lg = lane >> 4;
  const int NT = (int)(ld >> 6);
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool rok = r0 + l16 < n;
  const float* xr = phi + (int64_t)(rok ? r0 + l16 : 0) * ld;
  constexpr int ZS = CT * 16 + 1;                  // LDS row stride of the partial logits
  floatx4 acc[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) acc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int T0 = w; T0 < NT; T0 += 2 * NWV) {
    const bool ok1 = T0 + NWV < NT;
    const int T1 = ok1 ? T0 + NWV : T0;
    float4 xv[2][4], wv[2][4][CT];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t dof = 64 * (h ? T1 : T0) + 16 * lg;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        xv[h][q] = ld4(xr + dof + 4 * q);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) wv[h][q][ct] = ld4(W + min(ct * 16 + l16, C - 1) * ld + dof + 4 * q);
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !ok1) break;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = rok ? xv[h][q] : zero4;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const float4 wq = ct * 16 + l16 < C ? wv[h][q][ct] : zero4;
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) acc[ct] = mfma4(comp(x, e4), comp(wq, e4), acc[ct]);
        }
      }
    }
  }
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int i = 0; i < 4; ++i) zt[(w * 16 + 4 * lg + i) * ZS + ct * 16 + l16] = acc[ct][i];
  __syncthreads();
  if (w == 0 && lane < 16 && r0 + lane < n) {
    const int r = lane;
    const int yy = y[r0 + r];
    float m = -INFINITY;
    int am = 0;
    for (int c = 0; c < C; ++c) {
      float z = zt[r * ZS + c];
#pragma unroll
      for (int k = 1; k < NWV; ++k) z += zt[(k * 16 + r) * ZS + c];
      zt[r * ZS + c] = z;
      if (z > m) { m = z; am = c; }
    }
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += expf(zt[r * ZS + c] - m);
    ce += (double)(-(zt[r * ZS + yy] - m - logf(se)));
    cor += (am == yy) ? 1.0 : 0.0;
  }
  __syncthreads();                                 // zt is rewritten by the next group
}

// block e of E walks the row groups e, e + E, ... and writes its two partial sums to part[2e]
template <int NWV>
__device__ void eval_persistent(const float* __restrict__ phi, int64_t ld, const int32_t* __restrict__ y, int n,
                                const float* __restrict__ W, int C, int e, int E, float* zt,
                                double* __restrict__ part) {
  double ce = 0.0, cor = 0.0;
  for (int rg = e; rg * 16 < n; rg += E) eval_group16<NWV>(phi, ld, y, n, W, C, rg * 16, zt, ce, cor);
  if ((threadIdx.x >> 6) == 0) {
    ce = wave_sum(ce);
    cor = wave_sum(cor);
    if ((threadIdx.x & 63) == 0) {
      part[2 * e] = ce;
      part[2 * e + 1] = cor;
    }
  }
}

}  // namespace fs
