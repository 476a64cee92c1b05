// fs_aggregate -- mixture-weighted model aggregation over the clients x params buffer.
//
// Replaces the inline fold of /root/reference/functions/tools.py:345-350 (also 372-377,
// 455-460):   global = p0*W0;  global = global + p_j*W_j  for j = 1..N-1,
// every product and every sum rounded separately (no fma contraction), so with one
// chunk the result is bitwise the reference's fold of the same W_j.
//
// HBM-bound streaming reduction: each thread owns one float4 of the C*ld parameters
// and walks the clients; consecutive threads read consecutive 16 B, so every client
// row is one coalesced sweep.  When C*ld/4 threads cannot fill the chip the client
// range is cut into `chunks` consecutive pieces folded in parallel (stage 1) and the
// partials are folded by a fixed tree (stage 2: strided in-order sums, then those in order).
#include "common.h"
#include "finalize.h"

namespace fs {

// No fma contraction anywhere in this file: the fold must round p*W and the sum separately
// (plain operators under this pragma; HIP's __fmul_rn/__fadd_rn are header functions whose
// instructions keep the default contract flag and still fuse after inlining).
#pragma clang fp contract(off)

__device__ __forceinline__ float4 fold_step(float4 acc, float p, float4 w) {
  return make_float4(acc.x + p * w.x, acc.y + p * w.y, acc.z + p * w.z, acc.w + p * w.w);
}

__global__ __launch_bounds__(256) void aggregate_kernel(const float* __restrict__ W, int64_t stride,
                                                       const float* __restrict__ p, int N, int64_t len4,
                                                       int per_chunk, float* __restrict__ out,
                                                       int64_t out_stride) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= len4) return;
  const int k = blockIdx.y;
  const int j0 = k * per_chunk;
  const int j1 = min(N, j0 + per_chunk);
  const float* base = W + 4 * i;
  const float4 w0 = ld4(base + (int64_t)j0 * stride);
  const float p0 = p[j0];
  float4 acc = make_float4(p0 * w0.x, p0 * w0.y, p0 * w0.z, p0 * w0.w);
  int j = j0 + 1;
  for (; j + 3 < j1; j += 4) {
    const float4 a = ld4(base + (int64_t)j * stride);
    const float4 b = ld4(base + (int64_t)(j + 1) * stride);
    const float4 c = ld4(base + (int64_t)(j + 2) * stride);
    const float4 d = ld4(base + (int64_t)(j + 3) * stride);
    acc = fold_step(acc, p[j], a);
    acc = fold_step(acc, p[j + 1], b);
    acc = fold_step(acc, p[j + 2], c);
    acc = fold_step(acc, p[j + 3], d);
  }
  for (; j < j1; ++j) acc = fold_step(acc, p[j], ld4(base + (int64_t)j * stride));
  st4(out + (int64_t)k * out_stride + 4 * i, acc);
}

// stage 2: FP_SUB threads per float4 position, thread s folding the partials k = s, s + FP_SUB,
// ... in order, then thread 0 of the position folding the FP_SUB sums in order (a fixed tree:
// the same bits every run).  One thread per position walking all K partials put only len4 / 256
// workgroups on the chip (config 4: 20 CUs, 20 us for 5 MB of partials).
constexpr int FP_SUB = 8, FP_POS = 256 / FP_SUB;

__global__ __launch_bounds__(256) void fold_partials_kernel(const float* __restrict__ part, int K, int64_t len4,
                                                           float* __restrict__ out) {
  __shared__ float4 sums[FP_SUB][FP_POS];
  const int sub = threadIdx.x / FP_POS, pl = threadIdx.x % FP_POS;
  const int64_t i = (int64_t)blockIdx.x * FP_POS + pl;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < len4 && sub < K) {
    acc = ld4(part + (int64_t)sub * 4 * len4 + 4 * i);
    for (int k = sub + FP_SUB; k < K; k += FP_SUB) {
      const float4 v = ld4(part + (int64_t)k * 4 * len4 + 4 * i);
      acc = make_float4(acc.x + v.x, acc.y + v.y, acc.z + v.z, acc.w + v.w);
    }
  }
  sums[sub][pl] = acc;
  __syncthreads();
  if (sub == 0 && i < len4) {
    float4 t = sums[0][pl];
    for (int s2 = 1; s2 < FP_SUB && s2 < K; ++s2) {
      const float4 v = sums[s2][pl];
      t = make_float4(t.x + v.x, t.y + v.y, t.z + v.z, t.w + v.w);
    }
    st4(out + 4 * i, t);
  }
}

// One-launch form (round 5, chunks <= 0 with 16 <= N <= AG_ONE_MAX_N): SUB consecutive client
// ranges per float4 position folded by SUB threads of one workgroup (stage 1, as
// aggregate_kernel's chunks), their partials folded in order in LDS (stage 2) -- one launch
// instead of two, no workspace.  The round plan also hands it the deferred evaluation's
// finaliser (one extra workgroup, eval.hip's eval_finalize arithmetic): config 2's round went
// from four launches after the training (finalise, aggregate, fold, next training) to two.
constexpr int AG_ONE_MAX_N = 512;   // above: 64 sub-ranges of 4 positions read 64-byte pieces of
                                    // each client row (N = 1000-1250: 34-38 vs 18-19 us, round 5)

template <int SUB>
__global__ __launch_bounds__(256) void aggregate_one_kernel(const float* __restrict__ W, int64_t stride,
                                                           const float* __restrict__ p, int N, int64_t len4, int per,
                                                           float* __restrict__ out, EvalFinalize fin) {
  constexpr int POS = 256 / SUB;
  __shared__ float4 sums[SUB][POS];
  if (fin.part && blockIdx.x == gridDim.x - 1) {
    eval_finalize_block(fin.part, fin.nb, fin.n, fin.out, reinterpret_cast<double(*)[256]>(&sums[0][0]));
    return;
  }
  static_assert(sizeof(sums) >= 2 * 256 * sizeof(double), "the finaliser reuses the partials' LDS");
  const int sub = threadIdx.x / POS, pl = threadIdx.x % POS;
  const int64_t i = (int64_t)blockIdx.x * POS + pl;
  const int j0 = sub * per, j1 = min(N, j0 + per);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < len4 && j0 < j1) {
    // every load of a group of 8 clients (the range's first included) issued before the first
    // fold: one round trip per 8 clients (round 6; the first client's load, then groups of 8 / 4,
    // then the tail one by one took 4 dependent round trips at config 2's 7 clients per range).
    // The same products and sums in the same order as the left fold of the range.
    const float* base = W + 4 * i;
    for (int j = j0; j < j1; j += 8) {
      const int n = min(8, j1 - j);
      float4 v[8];
      float pv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u < n) {
          v[u] = ld4(base + (int64_t)(j + u) * stride);
          pv[u] = p[j + u];
        }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u < n) {
          if (u == 0 && j == j0)
            acc = make_float4(pv[0] * v[0].x, pv[0] * v[0].y, pv[0] * v[0].z, pv[0] * v[0].w);
          else
            acc = fold_step(acc, pv[u], v[u]);
        }
    }
  }
  sums[sub][pl] = acc;
  __syncthreads();
  if (sub == 0 && i < len4) {
    float4 t = sums[0][pl];
    for (int s2 = 1; s2 < SUB && s2 * per < N; ++s2) {
      const float4 v = sums[s2][pl];
      t = make_float4(t.x + v.x, t.y + v.y, t.z + v.z, t.w + v.w);
    }
    st4(out + 4 * i, t);
  }
}

// sub-ranges per position: 1 below 16 clients (then the fold is the reference's, bitwise),
// else the largest power of two <= min(32, N / 6) (~6+ clients per thread: one or two round
// trips of 8 loads)
static int one_launch_sub(int N) {
  if (N < 16) return 1;
  int s = 1;
  while (s * 2 <= 32 && s * 2 <= N / 6) s *= 2;
  return s;
}

template <int SUB>
static void launch_one(const float* W, int64_t stride, const float* p, int N, int64_t len4, float* out,
                       const EvalFinalize& fin, hipStream_t st) {
  constexpr int POS = 256 / SUB;
  const int per = (N + SUB - 1) / SUB;
  const int64_t blocks = (len4 + POS - 1) / POS + (fin.part ? 1 : 0);
  hipLaunchKernelGGL((aggregate_one_kernel<SUB>), dim3((unsigned)blocks), dim3(256), 0, st, W, stride, p, N, len4, per,
                     out, fin);
}

int aggregate_launch(const float* d_W_all, int64_t stride, const float* d_p, int N, int64_t len, float* d_W_bar,
                     float* d_ws, int64_t ws_floats, int chunks, const EvalFinalize* fin, hipStream_t st) {
  FS_REQUIRE(N >= 1, "N must be >= 1");
  FS_REQUIRE(len >= 4 && len % 4 == 0 && stride % 4 == 0 && stride >= len, "len/stride must be multiples of 4");
  FS_REQUIRE(d_W_all && d_p && d_W_bar, "null pointer");
  const int64_t len4 = len / 4;
  const EvalFinalize none{nullptr, 0, 0, nullptr};
  if (chunks <= 0 && N <= AG_ONE_MAX_N) {
    const EvalFinalize& f = fin ? *fin : none;
    switch (one_launch_sub(N)) {
      case 1: launch_one<1>(d_W_all, stride, d_p, N, len4, d_W_bar, f, st); break;
      case 2: launch_one<2>(d_W_all, stride, d_p, N, len4, d_W_bar, f, st); break;
      case 4: launch_one<4>(d_W_all, stride, d_p, N, len4, d_W_bar, f, st); break;
      case 8: launch_one<8>(d_W_all, stride, d_p, N, len4, d_W_bar, f, st); break;
      case 16: launch_one<16>(d_W_all, stride, d_p, N, len4, d_W_bar, f, st); break;
      default: launch_one<32>(d_W_all, stride, d_p, N, len4, d_W_bar, f, st); break;
    }
    FS_LAUNCH_CHECK();
    return FS_OK;
  }
  if (fin) {
    const int rc = eval_finalize_launch(fin->part, fin->nb, fin->n, fin->out, st);
    if (rc != FS_OK) return rc;
  }
  const int64_t bx = (len4 + 255) / 256;
  if (chunks <= 0) {
    // 8 chunks (>= 8 clients each): at N = 1000-1250 every count from 8 to 16 measured within
    // 5 % of the best and the earlier "~2048 workgroups" rule (74-103 chunks) 10-20 % slower
    // (profiles/r05/agg_time.txt)
    chunks = (int)std::max<int64_t>(1, std::min<int64_t>(8, N / 8));
  }
  if (chunks > N) chunks = N;
  // as many chunks as the workspace holds partials for (without one: a single chunk); an
  // automatic count above that used to fall back to ONE chunk -- 8 % of HBM at config 4
  // (1250 clients, 80 KB each, 5,120 threads walking all of them: 161 us per round)
  if (chunks > 1) chunks = d_ws ? (int)std::min<int64_t>(chunks, ws_floats / len) : 1;
  if (chunks < 1) chunks = 1;
  const int per = (N + chunks - 1) / chunks;
  chunks = (N + per - 1) / per;
  if (chunks == 1) {
    hipLaunchKernelGGL(aggregate_kernel, dim3((unsigned)bx, 1), dim3(256), 0, st, d_W_all, stride, d_p, N, len4, per,
                       d_W_bar, (int64_t)0);
  } else {
    hipLaunchKernelGGL(aggregate_kernel, dim3((unsigned)bx, chunks), dim3(256), 0, st, d_W_all, stride, d_p, N, len4,
                       per, d_ws, len);
    hipLaunchKernelGGL(fold_partials_kernel, dim3((unsigned)((len4 + FP_POS - 1) / FP_POS)), dim3(256), 0, st, d_ws,
                       chunks, len4, d_W_bar);
  }
  FS_LAUNCH_CHECK();
  return FS_OK;
}

}  // namespace fs

using namespace fs;

extern "C" int fs_aggregate(const float* d_W_all, int64_t stride, const float* d_p, int N, int64_t len,
                            float* d_W_bar, float* d_ws, int64_t ws_floats, int chunks, void* stream) {
  return aggregate_launch(d_W_all, stride, d_p, N, len, d_W_bar, d_ws, ws_floats, chunks, nullptr,
                          reinterpret_cast<hipStream_t>(stream));
}
