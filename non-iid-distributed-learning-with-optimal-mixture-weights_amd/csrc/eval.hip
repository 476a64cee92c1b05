// fs_eval -- test-set cross-entropy and top-1 accuracy of the global model.
//
// Replaces test_loop + comp_accuracy + Meter (/root/reference/functions/tools.py:218-237,
// 82-96, 99-148).  The reference walks shuffled batches of 32 and averages per-batch
// means weighted by batch size, which equals the plain mean over all rows up to fp32
// rounding; the shuffle only matters for the RNG stream, which the host replays.
//
// Each 8-wave workgroup owns 16 test rows; its waves split the 64-column feature tiles
// (2 tiles of loads in flight per wave, ~2,500 waves for 10k rows so every CU streams),
// computing logits (16 x classes) with v_mfma_f32_16x16x4_f32; the partials are summed
// through LDS and wave 0 computes CE and arg-max per row.  Per-block partial
// sums go to a workspace and a one-block finalizer folds them in a fixed order, so the
// result is bitwise reproducible run to run.  HBM-bound: one read of the test features.
#include "common.h"

namespace fs {

constexpr int EV_WAVES = 4;
constexpr int EV_ROWS = 16;   // rows per workgroup; its 4 waves split the feature tiles

// RTW row tiles of 16 per workgroup: each wave's W fragments are loaded once per tile pair
// and reused for all RTW row tiles (W is re-read by every workgroup: RTW = 2 halves those
// reads, 10k rows then still give ~1.2 workgroups per CU)
template <int CT, int RTW, int NWV>
__global__ __launch_bounds__(NWV * 64) void eval_kernel(const float* __restrict__ phi, int64_t ld,
                                                           const int32_t* __restrict__ y, int n,
                                                           const float* __restrict__ W, int C,
                                                           double* __restrict__ part) {
  constexpr int ROWS = 16 * RTW;
  __shared__ float zt[NWV][ROWS][CT * 16 + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l16 = lane & 15, lg = lane >> 4;
  const int NT = (int)(ld >> 6);
  const int r0 = blockIdx.x * ROWS;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  bool rok[RTW];
  const float* xr[RTW];
#pragma unroll
  for (int rt = 0; rt < RTW; ++rt) {
    rok[rt] = r0 + 16 * rt + l16 < n;
    xr[rt] = phi + (int64_t)(rok[rt] ? r0 + 16 * rt + l16 : 0) * ld;   // unconditional loads, zeroed below
  }
  floatx4 acc[RTW][CT];
#pragma unroll
  for (int rt = 0; rt < RTW; ++rt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int T0 = w; T0 < NT; T0 += 2 * NWV) {
    const bool ok1 = T0 + NWV < NT;
    const int T1 = ok1 ? T0 + NWV : T0;
    float4 xv[RTW][2][4], wv[2][4][CT];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t dof = 64 * (h ? T1 : T0) + 16 * lg;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int rt = 0; rt < RTW; ++rt) xv[rt][h][q] = ld4(xr[rt] + dof + 4 * q);
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) wv[h][q][ct] = ld4(W + min(ct * 16 + l16, C - 1) * ld + dof + 4 * q);
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !ok1) break;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const float4 wq = (ct * 16 + l16 < C) ? wv[h][q][ct] : zero4;
#pragma unroll
          for (int rt = 0; rt < RTW; ++rt) {
            const float4 x = rok[rt] ? xv[rt][h][q] : zero4;
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) acc[rt][ct] = mfma4(comp(x, e4), comp(wq, e4), acc[rt][ct]);
          }
        }
      }
    }
  }
#pragma unroll
  for (int rt = 0; rt < RTW; ++rt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int i = 0; i < 4; ++i) zt[w][16 * rt + 4 * lg + i][ct * 16 + l16] = acc[rt][ct][i];
  __syncthreads();
  if (w == 0) {
    double ce = 0.0, cor = 0.0;
    if (lane < ROWS && r0 + lane < n) {
      const int r = lane;
      const int yy = y[r0 + r];
      float m = -INFINITY;
      int am = 0;
      for (int c = 0; c < C; ++c) {
        float z = zt[0][r][c];
#pragma unroll
        for (int k = 1; k < NWV; ++k) z += zt[k][r][c];
        zt[0][r][c] = z;
        if (z > m) { m = z; am = c; }
      }
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += expf(zt[0][r][c] - m);
      ce = (double)(-(zt[0][r][yy] - m - logf(se)));
      cor = (am == yy) ? 1.0 : 0.0;
    }
    ce = wave_sum(ce);
    cor = wave_sum(cor);
    if (lane == 0) {
      part[2 * blockIdx.x] = ce;
      part[2 * blockIdx.x + 1] = cor;
    }
  }
}

__global__ __launch_bounds__(256) void eval_finalize(const double* __restrict__ part, int nb, int n,
                                                    double* __restrict__ out) {
  __shared__ double s[2][256];
  double a = 0.0, b = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) { a += part[2 * i]; b += part[2 * i + 1]; }
  s[0][threadIdx.x] = a;
  s[1][threadIdx.x] = b;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      s[0][threadIdx.x] += s[0][threadIdx.x + h];
      s[1][threadIdx.x] += s[1][threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = s[0][0] / (double)n;
    out[1] = 100.0 * s[1][0] / (double)n;
  }
}

int eval_finalize_launch(const double* part, int nb, int n, double* out, hipStream_t st) {
  hipLaunchKernelGGL(eval_finalize, dim3(1), dim3(256), 0, st, part, nb, n, out);
  FS_LAUNCH_CHECK();
  return FS_OK;
}

}  // namespace fs

using namespace fs;

extern "C" int64_t fs_eval_ws_doubles(int n) { return 2 * (int64_t)((n + EV_ROWS - 1) / EV_ROWS) + 2; }

extern "C" int fs_eval(const float* d_phi, int64_t ld, const int32_t* d_labels, int n, const float* d_W, int C,
                       double* d_out, double* d_ws, void* stream) {
  FS_REQUIRE(n >= 1, "n must be >= 1");
  FS_REQUIRE(C >= 1 && C <= 32, "num_classes must be in [1, 32]");
  FS_REQUIRE(ld >= 64 && ld % 64 == 0, "ld must be a positive multiple of 64");
  FS_REQUIRE(d_phi && d_labels && d_W && d_out && d_ws, "null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // row tiles per workgroup (FS_EVAL_RTW = 1 | 2 | 4 for diagnostics; 2 and 4 measured slower:
  // config 2 26.6 / 32.0 / 34.8 us, config 3 163 / 184 / 218 us -- r02s2ev)
  const char* er = getenv("FS_EVAL_RTW");
  int rtw = er ? atoi(er) : 1;
  if (rtw != 2 && rtw != 4) rtw = 1;
  const int nb = (n + EV_ROWS * rtw - 1) / (EV_ROWS * rtw);
  // waves per workgroup splitting the feature tiles (FS_EVAL_WAVES = 4 | 8, default 8)
  const char* ew = getenv("FS_EVAL_WAVES");
  const int nwv = ew && atoi(ew) == 4 ? 4 : 8;   // 8: 24.3 vs 26.2 us at config 2, 158 vs 164 at config 3 (r02s2ev3)
#define EV_LAUNCH(CT_, RTW_)                                                                                       \
  do {                                                                                                             \
    if (nwv == 8)                                                                                                  \
      hipLaunchKernelGGL((eval_kernel<CT_, RTW_, 8>), dim3(nb), dim3(8 * 64), 0, st, d_phi, ld, d_labels, n, d_W, C, d_ws); \
    else                                                                                                           \
      hipLaunchKernelGGL((eval_kernel<CT_, RTW_, 4>), dim3(nb), dim3(4 * 64), 0, st, d_phi, ld, d_labels, n, d_W, C, d_ws); \
  } while (0)
  if (C <= 16) {
    if (rtw == 4) EV_LAUNCH(1, 4);
    else if (rtw == 2) EV_LAUNCH(1, 2);
    else EV_LAUNCH(1, 1);
  } else {
    if (rtw == 4) EV_LAUNCH(2, 4);
    else if (rtw == 2) EV_LAUNCH(2, 2);
    else EV_LAUNCH(2, 1);
  }
#undef EV_LAUNCH
  hipLaunchKernelGGL(eval_finalize, dim3(1), dim3(256), 0, st, d_ws, nb, n, d_out);
  FS_LAUNCH_CHECK();
  return FS_OK;
}
