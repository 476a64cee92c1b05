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

// ----------------------------------------------------------------------------
// p-solve, LDS-staged form (used whenever two batches of Z rows fit in LDS):
// wave w owns batch rows b = w, w+16, ...; its lanes split the clients n.  Per row the
// wave reduces the C logits out[b][c] = sum_n p_n Z[v_b][c][n] with xor butterflies (all
// lanes end up holding them), computes the softmax-CE gradient g[b][:] redundantly in
// every lane, and accumulates sum_c g[b][c] Z[v_b][c][n] for its own n; the 16 waves'
// partial gradients are summed in wave order, then the momentum step.  The next batch's
// rows are loaded into registers at the top of the step and written to the other LDS
// buffer at its end, so Z streams from L2/MALL behind the arithmetic.  Two barriers per
// step; a step costs ~1 us instead of three dependent global round trips.
// ----------------------------------------------------------------------------
constexpr int MS2_PER_THREAD = 4;     // float4 of staged rows per thread (one batch <= 64 KB)
constexpr int MS2_NK = 4;             // clients per lane (N <= 256 on this path)

template <int CMAX>
__global__ __launch_bounds__(MS_THREADS) void mix_solve_staged_kernel(const float* __restrict__ Z,
                                                                     const int32_t* __restrict__ y,
                                                                     const int32_t* __restrict__ perms, int N,
                                                                     int C, int nv, int epochs, int Bv, float lr,
                                                                     float mom, float* __restrict__ p,
                                                                     float* __restrict__ buf,
                                                                     int* __restrict__ first_flag) {
  extern __shared__ __attribute__((aligned(16))) float smem2[];
  const int CN = C * N;
  const int CN4 = (CN + 3) & ~3;                   // row stride in LDS (float4 aligned)
  float* zb = smem2;                               // [2][Bv][CN4]
  float* ps = zb + 2 * Bv * CN4;                   // [N]
  float* bs = ps + N;                              // [N]
  float* gpart = bs + N;                           // [MS_WAVES][N]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int n = tid; n < N; n += MS_THREADS) { ps[n] = p[n]; bs[n] = buf[n]; }
  int first = *first_flag;
  const int nbat = (nv + Bv - 1) / Bv;
  const int total = epochs * nbat;
  const int F4 = CN4 / 4;                          // float4 per staged row
  float4 stg[MS2_PER_THREAD];
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // stage batch `st` (global step) rows into registers / LDS slot
  auto batch_row = [&](int st, int b) -> int {
    const int ep = st / nbat, s = st - ep * nbat;
    return perms[(int64_t)ep * nv + s * Bv + b];
  };
  auto batch_size = [&](int st) -> int {
    const int s = st % nbat;
    return min(Bv, nv - s * Bv);
  };
#define MS2_LOAD(ST_)                                                                 \
  {                                                                                   \
    const int bcn_ = batch_size(ST_);                                                 \
    _Pragma("unroll") for (int i = 0; i < MS2_PER_THREAD; ++i) {                      \
      const int idx = tid + MS_THREADS * i;                                           \
      const int b = idx / F4, f = idx - b * F4;                                       \
      stg[i] = zero4;                                                                 \
      if (b < bcn_) {                                                                 \
        const float* zr = Z + (int64_t)batch_row(ST_, b) * CN;                        \
        if (4 * f + 3 < CN) stg[i] = ld4(zr + 4 * f);                                 \
        else {                                                                        \
          float t_[4] = {0.f, 0.f, 0.f, 0.f};                                         \
          for (int k = 0; k < 4; ++k) if (4 * f + k < CN) t_[k] = zr[4 * f + k];      \
          stg[i] = make_float4(t_[0], t_[1], t_[2], t_[3]);                           \
        }                                                                             \
      }                                                                               \
    }                                                                                 \
  }
#define MS2_STORE(SLOT_)                                                              \
  {                                                                                   \
    _Pragma("unroll") for (int i = 0; i < MS2_PER_THREAD; ++i) {                      \
      const int idx = tid + MS_THREADS * i;                                           \
      if (idx < Bv * F4) st4(zb + (int64_t)(SLOT_) * Bv * CN4 + (int64_t)idx * 4, stg[i]); \
    }                                                                                 \
  }
  if (total > 0) {
    MS2_LOAD(0);
    MS2_STORE(0);
  }
  __syncthreads();
  for (int st = 0; st < total; ++st) {
    const int cur = st & 1;
    const int bc = batch_size(st);
    const bool more = st + 1 < total;
    if (more) MS2_LOAD(st + 1);
    // per-lane gradient partials for n = lane + 64 k (k < MS2_NK, compile-time indexed)
    float gacc[MS2_NK];
#pragma unroll
    for (int k = 0; k < MS2_NK; ++k) gacc[k] = 0.f;
    for (int b = w; b < bc; b += MS_WAVES) {
      const float* zr = zb + (int64_t)cur * Bv * CN4 + (int64_t)b * CN4;
      float o[CMAX];
#pragma unroll
      for (int c = 0; c < CMAX; ++c) {
        float a = 0.f;
        if (c < C) {
#pragma unroll
          for (int k = 0; k < MS2_NK; ++k) {
            const int n = lane + 64 * k;
            if (n < N) a += ps[n] * zr[c * N + n];
          }
        }
        o[c] = wave_sum(a);                          // every lane holds out[b][c]
      }
      float m = -INFINITY;
#pragma unroll
      for (int c = 0; c < CMAX; ++c) if (c < C) m = fmaxf(m, o[c]);
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < CMAX; ++c) if (c < C) se += expf(o[c] - m);
      const float lse = logf(se);
      const float invb = 1.0f / (float)bc;
      const int yy = y[batch_row(st, b)];
#pragma unroll
      for (int c = 0; c < CMAX; ++c) {
        if (c < C) {
          const float gv = (c == yy ? -invb : 0.f) + expf(o[c] - m - lse) * invb;
#pragma unroll
          for (int k = 0; k < MS2_NK; ++k) {
            const int n = lane + 64 * k;
            if (n < N) gacc[k] += gv * zr[c * N + n];
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < MS2_NK; ++k) {
      const int n = lane + 64 * k;
      if (n < N) gpart[w * N + n] = gacc[k];
    }
    if (more) MS2_STORE(cur ^ 1);
    __syncthreads();
    for (int n = tid; n < N; n += MS_THREADS) {
      float gp = 0.f;
      for (int i = 0; i < MS_WAVES; ++i) gp += gpart[i * N + n];
      {
#pragma clang fp contract(off)
        const float nb = first ? gp : mom * bs[n] + gp;   // buf.mul_(0.9).add_(grad)
        bs[n] = nb;
        ps[n] = ps[n] + (-lr) * nb;                       // p.add_(buf, alpha=-lr)
      }
    }
    first = 0;
    __syncthreads();
  }
#undef MS2_LOAD
#undef MS2_STORE
  for (int n = tid; n < N; n += MS_THREADS) { p[n] = ps[n]; buf[n] = bs[n]; }
  if (tid == 0 && total > 0) *first_flag = 0;
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
  hipStream_t st0 = reinterpret_cast<hipStream_t>(stream);
  {
    // LDS-staged solver: two batches of Z rows + p, buf and the wave partials must fit
    const int CN4 = (C * N + 3) & ~3;
    const size_t lds2 = sizeof(float) * (2 * (size_t)Bv * CN4 + 2 * (size_t)N + (size_t)MS_WAVES * N);
    if (N <= 64 * MS2_NK && C <= 32 && lds2 <= 150 * 1024 && (size_t)Bv * (CN4 / 4) <= (size_t)MS_THREADS * MS2_PER_THREAD) {
      const void* kfn = C <= 16 ? reinterpret_cast<const void*>(&mix_solve_staged_kernel<16>)
                                : reinterpret_cast<const void*>(&mix_solve_staged_kernel<32>);
      if (lds2 > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2);
        if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_mix_solve: ") + hipGetErrorString(e));
      }
      if (C <= 16)
        hipLaunchKernelGGL(mix_solve_staged_kernel<16>, dim3(1), dim3(MS_THREADS), lds2, st0, d_Z, d_labels, d_perms,
                           N, C, n_val, epochs, Bv, lr_p, momentum, d_p, d_buf, d_first);
      else
        hipLaunchKernelGGL(mix_solve_staged_kernel<32>, dim3(1), dim3(MS_THREADS), lds2, st0, d_Z, d_labels, d_perms,
                           N, C, n_val, epochs, Bv, lr_p, momentum, d_p, d_buf, d_first);
      FS_LAUNCH_CHECK();
      return FS_OK;
    }
  }
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
