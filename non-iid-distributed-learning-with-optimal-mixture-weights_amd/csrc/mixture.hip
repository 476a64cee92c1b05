// FedAMW mixture-weight estimation (/root/reference/functions/tools.py:435-453).
//
// fs_mix_z:     Z[v][c*N + n] = X_val[v] . W_n[c]          -- fp32 MFMA GEMM, MFMA-bound
//               (M = n_val, N = C*clients, K = D).  The reference recomputes this matmul
//               for every 16-row batch of every inner epoch (tools.py:448); W is fixed
//               during the p-solve, so it is computed once per round here.
// fs_mix_solve: all `epochs * ceil(n_val/Bv)` dependent p-SGD steps of one round in ONE
//               persistent workgroup (a grid-wide barrier per step would cost more than
//               the step): out = Z_b p, CE, grad_p = Z_b^T g, momentum update.
#include "common.h"

namespace fs {

// ----------------------------------------------------------------------------
// Z GEMM: 64 x 64 output tile per 256-thread workgroup, BK = 16, LDS-staged,
// each wave a 32 x 32 quadrant = 2 x 2 tiles of v_mfma_f32_16x16x4_f32.
// ----------------------------------------------------------------------------
constexpr int MZ_BM = 64, MZ_BN = 64, MZ_BK = 16, MZ_PAD = 4;

__global__ __launch_bounds__(256) void mix_z_kernel(const float* __restrict__ W, const float* __restrict__ X,
                                                   int64_t ld, int N, int C, int nv, float* __restrict__ Z) {
  __shared__ float As[MZ_BM][MZ_BK + MZ_PAD];
  __shared__ float Bs[MZ_BN][MZ_BK + MZ_PAD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l16 = lane & 15, lg = lane >> 4;
  const int CN = C * N;
  const int v0 = blockIdx.y * MZ_BM;
  const int c0 = blockIdx.x * MZ_BN;
  // loader mapping: thread -> (row, 4-float group) of a 64 x 16 tile
  const int lr = tid >> 2, lk = (tid & 3) * 4;
  const int va = v0 + lr;
  const float* arow = va < nv ? X + (int64_t)va * ld : nullptr;
  const int cb = c0 + lr;
  const float* brow = nullptr;
  if (cb < CN) {
    const int c = cb / N, n = cb - c * N;
    brow = W + ((int64_t)n * C + c) * ld;
  }
  const int wr = (w >> 1) * 32, wc = (w & 1) * 32;
  floatx4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t k0 = 0; k0 < ld; k0 += MZ_BK) {
    const float4 av = arow ? ld4(arow + k0 + lk) : zero4;
    const float4 bv = brow ? ld4(brow + k0 + lk) : zero4;
    __syncthreads();
    st4(&As[lr][lk], av);
    st4(&Bs[lr][lk], bv);
    __syncthreads();
#pragma unroll
    for (int kq = 0; kq < MZ_BK / 4; ++kq) {
      float a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[t] = As[wr + 16 * t + l16][4 * kq + lg];
        b[t] = Bs[wc + 16 * t + l16][4 * kq + lg];
      }
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) acc[ti][tj] = mfma4(a[ti], b[tj], acc[ti][tj]);
    }
  }
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int v = v0 + wr + 16 * ti + 4 * lg + i;
        const int col = c0 + wc + 16 * tj + l16;
        if (v < nv && col < CN) Z[(int64_t)v * CN + col] = acc[ti][tj][i];
      }
}

// ----------------------------------------------------------------------------
// p-solve: one workgroup of 1024 threads.  p and the momentum buffer live in LDS.
// ----------------------------------------------------------------------------
constexpr int MS_THREADS = 1024;
constexpr int MS_WAVES = MS_THREADS / 64;
constexpr int MS_MAXB = 64;

__global__ __launch_bounds__(MS_THREADS) void mix_solve_kernel(const float* __restrict__ Z,
                                                              const int32_t* __restrict__ y,
                                                              const int32_t* __restrict__ perms, int N, int C,
                                                              int nv, int epochs, int Bv, float lr, float mom,
                                                              float* __restrict__ p, float* __restrict__ buf,
                                                              int* __restrict__ first_flag) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* ps = smem;                       // [N]
  float* bs = ps + N;                     // [N]
  float* outs = bs + N;                   // [MS_MAXB][C]
  float* gs = outs + MS_MAXB * C;         // [MS_MAXB][C]
  int* vid = reinterpret_cast<int*>(gs + MS_MAXB * C);  // [MS_MAXB]
  int* vy = vid + MS_MAXB;                              // [MS_MAXB]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int CN = C * N;
  for (int n = tid; n < N; n += MS_THREADS) { ps[n] = p[n]; bs[n] = buf[n]; }
  int first = *first_flag;
  const int nbat = (nv + Bv - 1) / Bv;
  for (int ep = 0; ep < epochs; ++ep) {
    for (int s = 0; s < nbat; ++s) {
      const int b0 = s * Bv;
      const int bc = min(Bv, nv - b0);
      if (tid < bc) {
        const int v = perms[(int64_t)ep * nv + b0 + tid];
        vid[tid] = v;
        vy[tid] = y[v];
      }
      __syncthreads();
      // out[b][c] = sum_n p_n Z[v_b][c*N + n]
      for (int q = w; q < bc * C; q += MS_WAVES) {
        const int b = q / C, c = q - b * C;
        const float* zr = Z + (int64_t)vid[b] * CN + (int64_t)c * N;
        float a = 0.f;
        for (int n = lane; n < N; n += 64) a += ps[n] * zr[n];
        a = wave_sum(a);
        if (lane == 0) outs[b * C + c] = a;
      }
      __syncthreads();
      // softmax / CE gradient (CrossEntropyLoss mean over the batch)
      if (w == 0 && lane < bc) {
        const int b = lane;
        const int yy = vy[b];
        float m = -INFINITY;
        for (int c = 0; c < C; ++c) m = fmaxf(m, outs[b * C + c]);
        float se = 0.f;
        for (int c = 0; c < C; ++c) se += expf(outs[b * C + c] - m);
        const float lse = logf(se);
        const float invb = 1.0f / (float)bc;
        for (int c = 0; c < C; ++c) {
          const float lp = outs[b * C + c] - m - lse;
          gs[b * C + c] = (c == yy ? -invb : 0.f) + expf(lp) * invb;
        }
      }
      __syncthreads();
      // grad_p[n] = sum_{b,c} g[b][c] Z[v_b][c*N+n];  SGD momentum (torch.optim.SGD semantics)
      for (int n = tid; n < N; n += MS_THREADS) {
        float gp = 0.f;
        for (int b = 0; b < bc; ++b) {
          const float* zr = Z + (int64_t)vid[b] * CN + n;
          for (int c = 0; c < C; ++c) gp += gs[b * C + c] * zr[(int64_t)c * N];
        }
        {
#pragma clang fp contract(off)
          const float nb = first ? gp : mom * bs[n] + gp;   // buf.mul_(0.9).add_(grad), two roundings
          bs[n] = nb;
          ps[n] = ps[n] + (-lr) * nb;                         // p.add_(buf, alpha=-lr)
        }
      }
      first = 0;
      __syncthreads();
    }
  }
  for (int n = tid; n < N; n += MS_THREADS) { p[n] = ps[n]; buf[n] = bs[n]; }
  if (tid == 0 && epochs > 0 && nbat > 0) *first_flag = 0;
}

}  // namespace fs

using namespace fs;

extern "C" int fs_mix_z(const float* d_W_all, const float* d_X_val, int64_t ld, int N, int C, int n_val, float* d_Z,
                        void* stream) {
  FS_REQUIRE(N >= 1 && C >= 1 && n_val >= 1, "bad sizes");
  FS_REQUIRE(ld >= 64 && ld % 64 == 0, "ld must be a positive multiple of 64");
  FS_REQUIRE(d_W_all && d_X_val && d_Z, "null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int CN = C * N;
  dim3 grid((CN + MZ_BN - 1) / MZ_BN, (n_val + MZ_BM - 1) / MZ_BM);
  hipLaunchKernelGGL(mix_z_kernel, grid, dim3(256), 0, st, d_W_all, d_X_val, ld, N, C, n_val, d_Z);
  FS_LAUNCH_CHECK();
  return FS_OK;
}

extern "C" int fs_mix_solve(const float* d_Z, const int32_t* d_labels, const int32_t* d_perms, int N, int C,
                            int n_val, int epochs, int Bv, float lr_p, float momentum, float* d_p, float* d_buf,
                            int* d_first, void* stream) {
  FS_REQUIRE(N >= 1 && C >= 1 && n_val >= 1 && epochs >= 0, "bad sizes");
  FS_REQUIRE(Bv >= 1 && Bv <= MS_MAXB, "valid batch size must be in [1, 64]");
  FS_REQUIRE(d_Z && d_labels && d_perms && d_p && d_buf && d_first, "null pointer");
  const size_t lds = sizeof(float) * (2 * (size_t)N + 2 * MS_MAXB * (size_t)C) + sizeof(int) * 2 * MS_MAXB;
  FS_REQUIRE(lds <= 160 * 1024, "N too large for the LDS-resident mixture solve");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mix_solve_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_mix_solve: ") + hipGetErrorString(e));
  }
  hipLaunchKernelGGL(mix_solve_kernel, dim3(1), dim3(MS_THREADS), lds, st, d_Z, d_labels, d_perms, N, C, n_val,
                     epochs, Bv, lr_p, momentum, d_p, d_buf, d_first);
  FS_LAUNCH_CHECK();
  return FS_OK;
}
