// Data heterogeneity of a partition (exp.py:67-74):
//
//   C   = Phi^T Phi / n                     (all n rows)
//   C_j = Phi_j^T Phi_j / n_j               (client j's rows)
//   hete = sum_j n_j / n * || C - C_j ||_F
//
// Two MFMA kernels over the client-packed feature buffer (rows CSR by client, row stride ld):
//   fs_gram    G = Phi^T Phi, D x D, upper-triangle 64 x 64 tiles (K = all rows), each tile
//              written to both halves (exactly symmetric);
//   fs_hetero  per (upper tile, client): the client's Gram tile G_j on the fly (K = n_j rows),
//              then sum over the tile of (G/n - G_j/n_j)^2 (fp32 difference, as torch forms
//              it, accumulated in double) into S[j] -- G_j is never written to HBM.
// Both are SYRK-shaped: 2 * rows * D^2 flop (half of it skipped by symmetry), MFMA-bound.
// Tile: 256 threads, 64 x 64 output, K staged 16 rows at a time through LDS (row stride 80
// floats: the 4 k-rows x 16 columns an MFMA operand read touches land in 64 distinct banks),
// each wave a 32 x 32 quadrant = 2 x 2 v_mfma_f32_16x16x4_f32.
#include "common.h"

namespace fs {

constexpr int GR_T = 64, GR_BK = 16, GR_LDS = GR_T + 16;

// upper-triangle tile pair (I <= J) of linear index q over T tiles
__device__ __forceinline__ void tri_pair(int q, int T, int& I, int& J) {
  I = 0;
  int rowlen = T;
  while (q >= rowlen) {
    q -= rowlen;
    ++I;
    --rowlen;
  }
  J = I + q;
}

// acc[ti][tj][i] <- sum over rows [r0, r1) of phi[r][I*64 + i'] * phi[r][J*64 + j']
__device__ __forceinline__ void gram_tile(const float* __restrict__ phi, int64_t ld, int64_t r0, int64_t r1,
                                          int ci, int cj, int D, floatx4 (&acc)[2][2], float (*As)[GR_LDS],
                                          float (*Bs)[GR_LDS]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l16 = lane & 15, lg = lane >> 4;
  const int wr = (w >> 1) * 32, wc = (w & 1) * 32;
  const int lk = tid >> 4, lc = (tid & 15) * 4;     // loader: k-row, 4-column group
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t k0 = r0; k0 < r1; k0 += GR_BK) {
    const int64_t r = k0 + lk;
    float4 av = zero4, bv = zero4;
    if (r < r1) {
      const float* row = phi + r * ld;
      if (ci + lc < D) av = ld4(row + ci + lc);      // ld % 64 == 0 and the padding columns are 0
      if (cj + lc < D) bv = ld4(row + cj + lc);
    }
    __syncthreads();
    st4(&As[lk][lc], av);
    st4(&Bs[lk][lc], bv);
    __syncthreads();
#pragma unroll
    for (int kq = 0; kq < GR_BK / 4; ++kq) {
      float a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[t] = As[4 * kq + lg][wr + 16 * t + l16];
        b[t] = Bs[4 * kq + lg][wc + 16 * t + l16];
      }
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) acc[ti][tj] = mfma4(a[ti], b[tj], acc[ti][tj]);
    }
  }
}

__global__ __launch_bounds__(256) void gram_kernel(const float* __restrict__ phi, int64_t ld, int64_t rows, int D,
                                                  float* __restrict__ G, int64_t ldg) {
  __shared__ float As[GR_BK][GR_LDS];
  __shared__ float Bs[GR_BK][GR_LDS];
  const int T = (D + GR_T - 1) / GR_T;
  int I, J;
  tri_pair(blockIdx.x, T, I, J);
  floatx4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  gram_tile(phi, ld, 0, rows, I * GR_T, J * GR_T, D, acc, As, Bs);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, lg = lane >> 4;
  const int wr = (w >> 1) * 32, wc = (w & 1) * 32;
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int a = I * GR_T + wr + 16 * ti + 4 * lg + i;
        const int b = J * GR_T + wc + 16 * tj + l16;
        if (a < D && b < D) {
          G[(int64_t)a * ldg + b] = acc[ti][tj][i];
          if (I != J) G[(int64_t)b * ldg + a] = acc[ti][tj][i];
        }
      }
}

__global__ __launch_bounds__(256) void hetero_kernel(const float* __restrict__ phi, int64_t ld,
                                                    const int64_t* __restrict__ row_off, int D,
                                                    const float* __restrict__ G, int64_t ldg, float n_all,
                                                    double* __restrict__ S) {
  __shared__ float As[GR_BK][GR_LDS];
  __shared__ float Bs[GR_BK][GR_LDS];
  const int T = (D + GR_T - 1) / GR_T;
  int I, J;
  tri_pair(blockIdx.x, T, I, J);
  const int j = blockIdx.y;
  const int64_t r0 = row_off[j], r1 = row_off[j + 1];
  floatx4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  gram_tile(phi, ld, r0, r1, I * GR_T, J * GR_T, D, acc, As, Bs);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, lg = lane >> 4;
  const int wr = (w >> 1) * 32, wc = (w & 1) * 32;
  const float nj = (float)(r1 - r0);
  double s = 0.0;
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int a = I * GR_T + wr + 16 * ti + 4 * lg + i;
        const int b = J * GR_T + wc + 16 * tj + l16;
        if (a < D && b < D) {
          const float c = G[(int64_t)a * ldg + b] / n_all;   // torch: matmul(...) / len
          const float cj = acc[ti][tj][i] / nj;
          const float df = c - cj;
          s += (double)df * (double)df;
        }
      }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0 && r1 > r0) atomicAdd(&S[j], I == J ? s : 2.0 * s);
}

}  // namespace fs

using namespace fs;

extern "C" int fs_gram(const float* d_phi, int64_t ld, int64_t rows, int D, float* d_G, int64_t ldg, void* stream) {
  FS_REQUIRE(rows >= 0 && D >= 1, "bad sizes");
  FS_REQUIRE(ld >= 64 && ld % 64 == 0 && ld >= D, "ld must be a multiple of 64 covering D");
  FS_REQUIRE(ldg >= D, "ldg must cover D");
  FS_REQUIRE(d_phi && d_G, "null pointer");
  const int T = (D + GR_T - 1) / GR_T;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(gram_kernel, dim3(T * (T + 1) / 2), dim3(256), 0, st, d_phi, ld, rows, D, d_G, ldg);
  FS_LAUNCH_CHECK();
  return FS_OK;
}

extern "C" int fs_hetero(const float* d_phi, int64_t ld, const int64_t* d_row_off, int N, int D, const float* d_G,
                         int64_t ldg, int64_t n_total, double* d_S, void* stream) {
  FS_REQUIRE(N >= 1 && D >= 1 && n_total >= 1, "bad sizes");
  FS_REQUIRE(N <= 65535, "at most 65535 clients per launch");
  FS_REQUIRE(ld >= 64 && ld % 64 == 0 && ld >= D, "ld must be a multiple of 64 covering D");
  FS_REQUIRE(ldg >= D, "ldg must cover D");
  FS_REQUIRE(d_phi && d_row_off && d_G && d_S, "null pointer");
  const int T = (D + GR_T - 1) / GR_T;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(d_S, 0, sizeof(double) * N, st) != hipSuccess) return fail(FS_EHIP, "fs_hetero: memset");
  hipLaunchKernelGGL(hetero_kernel, dim3(T * (T + 1) / 2, N), dim3(256), 0, st, d_phi, ld, d_row_off, D, d_G, ldg,
                     (float)n_total, d_S);
  FS_LAUNCH_CHECK();
  return FS_OK;
}
