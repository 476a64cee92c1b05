// Shared helpers for the gfx950 kernels and the C-ABI wrappers.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "../../include/fedsim.h"

namespace fs {

// ---- error plumbing (thread-local message, negative status codes) ----------
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

// ---- the process-wide tuning of fs_set_tuning (host.cpp), read at each launch ----
fs_tuning tuning();

#define FS_REQUIRE(cond, msg)                                                  \
  do {                                                                         \
    if (!(cond)) return ::fs::fail(FS_EINVAL, std::string(__func__) + ": " + (msg)); \
  } while (0)

#define FS_LAUNCH_CHECK()                                                      \
  do {                                                                         \
    hipError_t e_ = hipGetLastError();                                         \
    if (e_ != hipSuccess)                                                      \
      return ::fs::fail(FS_EHIP, std::string(__func__) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ---- local training parameters (shared by the single- and split-workgroup kernels) ----
struct LTParams {
  const float* phi;
  int64_t ld;
  const int64_t* row_off;
  const int32_t* labels;
  const int32_t* perms;
  const int32_t* order;
  int N, C, B, E;
  float lr, mu, lam;
  int prox, reg, chained;
  const float* W_start;
  float* W_out;
  double* loss;
  int64_t max_client_steps = 0;   // host bound on E * ceil(n_j / B) over the clients (0: unknown)
  // fused evaluation (parallel split launches only): fuse_E extra workgroups on the CUs the
  // groups leave idle evaluate W_start on the test set, partial sums into fuse_part[2E]
  const float* fuse_phi = nullptr;
  const int32_t* fuse_y = nullptr;
  int fuse_n = 0, fuse_E = 0;
  double* fuse_part = nullptr;
};

struct FuseEval {
  const float* phi;
  const int32_t* y;
  int n, E;
  double* part;
};

// workgroups a parallel split launch of this shape leaves idle (0: none, or not a split launch)
int split_idle_cus(int N, int C, int B, int64_t ld, int G, int chained);
// fs_eval's fold of nb partial pairs into out[0..1] (one workgroup)
int eval_finalize_launch(const double* part, int nb, int n, double* out, hipStream_t st);

// fs_local_train with a host bound on the steps of any client (the round plan knows the
// client sizes; with the bound the split kernel tags its hand-offs by launch generation
// instead of clearing its exchange buffer before every launch)
int local_train(const float* d_phi, int64_t ld, const int64_t* d_row_off, const int32_t* d_labels,
                const int32_t* d_perms, const int32_t* d_order, int N, int C, int B, int E, float lr, float mu,
                int prox, float lam, int reg, int chained, const float* d_W_start, float* d_W_out, double* d_loss,
                int G, void* d_ws, int64_t ws_bytes, hipStream_t st, int64_t max_client_steps,
                const FuseEval* fuse = nullptr);

// split-client launcher (local_train_split.hip): G workgroups per client
int launch_local_train_split(const LTParams& P, int G, void* ws, int64_t ws_bytes, hipStream_t st);
// the kernel the calling thread's last fs_local_train launched (FS_LT_*, fs_local_train_last_kernel)
void set_last_lt_kernel(int k);
// pair-client launcher (local_train_pair.hip): G workgroups per group, two clients per group
int launch_local_train_pair(const LTParams& P, int G, void* ws, int64_t ws_bytes, hipStream_t st);
// pipelined split launcher (local_train_pipe.hip): G workgroups per client, hand-off by row tile
int launch_local_train_pipe(const LTParams& P, int G, void* ws, int64_t ws_bytes, hipStream_t st);

// ---- device helpers ----------------------------------------------------------
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// v_mfma_f32_16x16x4_f32: A[i][k] lane l -> i = l&15, k = l>>4; B[k][j] -> k = l>>4,
// j = l&15; D[i][j] -> j = l&15, i = 4*(l>>4) + reg.  Exact f32 (k-ordered fma chain).
__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() carries a workgroup-scope
// release that drains vmcnt -- i.e. waits for every prefetch in flight; this waits for this
// wave's LDS operations (lgkmcnt) and nothing else.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

__device__ __forceinline__ float comp(const float4& v, int e) {
  return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

}  // namespace fs
