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

}  // namespace fs

using namespace fs;

extern "C" int fs_aggregate(const float* d_W_all, int64_t stride, const float* d_p, int N, int64_t len,
                            float* d_W_bar, float* d_ws, int64_t ws_floats, int chunks, void* stream) {
  FS_REQUIRE(N >= 1, "N must be >= 1");
  FS_REQUIRE(len >= 4 && len % 4 == 0 && stride % 4 == 0 && stride >= len, "len/stride must be multiples of 4");
  FS_REQUIRE(d_W_all && d_p && d_W_bar, "null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t len4 = len / 4;
  const int64_t bx = (len4 + 255) / 256;
  if (chunks <= 0) {
    // aim for >= ~2048 workgroups of 256 threads while keeping >= 8 clients per chunk
    int64_t want = (2048 + bx - 1) / bx;
    want = std::min<int64_t>(want, std::max<int64_t>(1, N / 8));
    chunks = (int)std::max<int64_t>(1, want);
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
