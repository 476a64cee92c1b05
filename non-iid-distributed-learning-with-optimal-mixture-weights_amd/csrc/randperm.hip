// fs_randperm_device -- the DataLoader shuffle replay on the GPU.
//
// For pass i: out[off[i] .. off[i]+n[i]) = torch.randperm(n[i], generator=g) with
// g.manual_seed(seed[i]) -- exactly what torch.utils.data.RandomSampler draws for one
// shuffled DataLoader pass (/root/reference/functions/tools.py:179, 220; exp.py:99).
// torch's CPU generator is MT19937 seeded with (uint32)seed; its randperm is a forward
// Fisher-Yates taking z = mt() % (n - k) (bit-exact with
// fs_randperm_batch and torch, tests/test_gpu_parity.py).
//
// One wave per pass.  The MT19937 seeding recurrence is serial (lane 0, 623 steps);
// each 624-word twist runs in four dependency phases across the wave's lanes
// (i in [0,227) reads only old words; [227,454) needs the new [0,227); [454,623) the
// new [227,396); i = 623 the new words 0 and 396); tempering is lane-parallel; the
// Fisher-Yates swaps are inherently serial and run on lane 0 out of LDS.  Passes are
// independent, so a round's hundreds of passes fill the chip; the replay never
// touches the host and costs one launch per round.  Passes of at most 64 rows run one per
// lane instead (randperm_lanes_kernel below).
#include "common.h"

namespace fs {

constexpr int MT_N = 624, MT_M = 397;
constexpr int RP_THREADS = 64;

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// in-place twist of mt[0..623]; all 64 lanes participate
__device__ void mt_twist(uint32_t* mt) {
  const int lane = threadIdx.x;
  uint32_t v[4];
  // phase A: i in [0, 227)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = lane + 64 * k;
    if (i < MT_N - MT_M) v[k] = mt_mix(mt[i], mt[i + 1], mt[i + MT_M]);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = lane + 64 * k;
    if (i < MT_N - MT_M) mt[i] = v[k];
  }
  __syncthreads();
  // phase B: i in [227, 454)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = (MT_N - MT_M) + lane + 64 * k;
    if (i < 2 * (MT_N - MT_M)) v[k] = mt_mix(mt[i], mt[i + 1], mt[i + MT_M - MT_N]);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = (MT_N - MT_M) + lane + 64 * k;
    if (i < 2 * (MT_N - MT_M)) mt[i] = v[k];
  }
  __syncthreads();
  // phase C: i in [454, 623)
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int i = 2 * (MT_N - MT_M) + lane + 64 * k;
    if (i < MT_N - 1) v[k] = mt_mix(mt[i], mt[i + 1], mt[i + MT_M - MT_N]);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int i = 2 * (MT_N - MT_M) + lane + 64 * k;
    if (i < MT_N - 1) mt[i] = v[k];
  }
  __syncthreads();
  // phase D: i = 623
  if (lane == 0) mt[MT_N - 1] = mt_mix(mt[MT_N - 1], mt[0], mt[MT_M - 1]);
  __syncthreads();
}

// a pass longer than the launch's max_n (a caller breaking the contract, include/fedsim.h): its
// rows are written as the identity permutation (bounded, in global memory) and the error word
// is set, so the host raises instead of training on a silently unshuffled pass
__device__ __forceinline__ void rp_contract_broken(int32_t* dst, int n, int lane, int stride, uint32_t* err) {
  for (int i = lane; i < n; i += stride) dst[i] = i;
  if (err && lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool IN_LDS>
__global__ __launch_bounds__(RP_THREADS) void randperm_kernel(const int64_t* __restrict__ seeds,
                                                             const int64_t* __restrict__ ns,
                                                             const int64_t* __restrict__ offs,
                                                             int32_t* __restrict__ out, int64_t max_n,
                                                             uint32_t* err) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem_rp[];
  uint32_t* mt = smem_rp;             // [624]
  uint32_t* rnd = mt + MT_N;          // [624]
  const int lane = threadIdx.x;
  const int pass = blockIdx.x;
  const int64_t n64 = ns[pass];
  int32_t* dst = out + offs[pass];
  if (n64 > max_n) {                  // (wave-uniform)
    rp_contract_broken(dst, (int)n64, lane, RP_THREADS, err);
    return;
  }
  const int n = (int)n64;
  int32_t* perm = IN_LDS ? reinterpret_cast<int32_t*>(rnd + MT_N) : dst;
  for (int i = lane; i < n; i += RP_THREADS) perm[i] = i;
  if (lane == 0) {
    uint32_t x = (uint32_t)(uint64_t)seeds[pass];
    mt[0] = x;
    for (int i = 1; i < MT_N; ++i) {
      x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
      mt[i] = x;
    }
  }
  __syncthreads();
  for (int i0 = 0; i0 < n - 1; i0 += MT_N) {
    mt_twist(mt);
    for (int k = lane; k < MT_N; k += RP_THREADS) rnd[k] = mt_temper(mt[k]);
    __syncthreads();
    if (lane == 0) {
      const int i1 = min(n - 1, i0 + MT_N);
      for (int i = i0; i < i1; ++i) {
        const uint32_t z = rnd[i - i0] % (uint32_t)(n - i);
        const int32_t a = perm[i];
        perm[i] = perm[i + z];
        perm[i + z] = a;
      }
    }
    __syncthreads();
  }
  if (IN_LDS)
    for (int i = lane; i < n; i += RP_THREADS) dst[i] = perm[i];
}

// Short passes (every n <= RL_MAXN, config 4's 64-row clients): one LANE per pass, 64 passes
// per wave.  A pass of n rows draws n - 1 words, the first n - 1 of MT19937's first twist:
// word k = mix(mt[k], mt[k+1], mt[k+397]) (k < 227 needs no word the twist rewrote first), so
// the seeding recurrence runs to 397 + n - 2 and only mt[0..n-1] and mt[397..397+n-2] are kept
// -- in registers, the recurrence fully unrolled (compile-time slots).  Fisher-Yates on the
// lane's own LDS row (stride RL_MAXN + 1: the lanes' sequential accesses hit distinct banks).
// The one-wave-per-pass form above keeps 63 of 64 lanes idle through the serial seeding and
// swaps; next to a training launch its thousands of waves compete for the CUs.
constexpr int RL_MAXN = 64;

__global__ __launch_bounds__(64) void randperm_lanes_kernel(const int64_t* __restrict__ seeds,
                                                           const int64_t* __restrict__ ns,
                                                           const int64_t* __restrict__ offs, int64_t npasses,
                                                           int32_t* __restrict__ out, int max_n, uint32_t* err) {
  __shared__ int32_t perm_s[64][RL_MAXN + 1];
  const int lane = threadIdx.x;
  const int64_t pass = (int64_t)blockIdx.x * 64 + lane;
  const bool live = pass < npasses;
  const int n_req = live ? (int)ns[pass] : 0;
  // the contract (fedsim.h): every ns[pass] <= max_n; this form is chosen for max_n <= RL_MAXN.
  // A longer pass (a caller bug) must not shuffle into its neighbours' LDS rows: it is written
  // as the identity permutation -- valid row indices, memory-safe -- and the error word is set
  // (max_n <= RL_MAXN here)
  const int n = n_req <= max_n ? n_req : 0;
  if (n_req > max_n && err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int32_t* perm = perm_s[lane];
  uint32_t lo[RL_MAXN], hi[RL_MAXN - 1];
  {
    uint32_t x = live ? (uint32_t)(uint64_t)seeds[pass] : 0u;
    lo[0] = x;
#pragma unroll
    for (int i = 1; i <= MT_M + RL_MAXN - 2; ++i) {
      x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
      if (i < RL_MAXN) lo[i] = x;
      if (i >= MT_M) hi[i - MT_M] = x;
    }
  }
#pragma unroll
  for (int i = 0; i < RL_MAXN; ++i)
    if (i < n) perm[i] = i;
#pragma unroll
  for (int i = 0; i < RL_MAXN - 1; ++i) {
    if (i < n - 1) {
      const uint32_t r = mt_temper(mt_mix(lo[i], lo[i + 1], hi[i]));
      const int z = (int)(r % (uint32_t)(n - i));
      const int32_t a = perm[i];
      perm[i] = perm[i + z];
      perm[i + z] = a;
    }
  }
  if (live) {
    int32_t* dst = out + offs[pass];
    for (int i = 0; i < n; ++i) dst[i] = perm[i];
    for (int i = n; i < n_req; ++i) dst[i] = i;
  }
}

}  // namespace fs

using namespace fs;

extern "C" int fs_randperm_device(const int64_t* d_seeds, const int64_t* d_n, const int64_t* d_off, int64_t npasses,
                                  int64_t max_n, int32_t* d_out, uint32_t* d_err, void* stream) {
  FS_REQUIRE(npasses >= 0 && max_n >= 0 && max_n < ((int64_t)1 << 31), "bad sizes");
  if (npasses == 0) return FS_OK;
  FS_REQUIRE(d_seeds && d_n && d_off && d_out, "null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (max_n <= RL_MAXN) {
    hipLaunchKernelGGL(randperm_lanes_kernel, dim3((unsigned)((npasses + 63) / 64)), dim3(64), 0, st, d_seeds, d_n,
                       d_off, npasses, d_out, (int)max_n, d_err);
    FS_LAUNCH_CHECK();
    return FS_OK;
  }
  const size_t lds_small = sizeof(uint32_t) * 2 * MT_N;
  const size_t lds_full = lds_small + sizeof(int32_t) * (size_t)max_n;
  if (lds_full <= 160 * 1024) {
    if (lds_full > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&randperm_kernel<true>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_full);
      if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_randperm_device: ") + hipGetErrorString(e));
    }
    hipLaunchKernelGGL(randperm_kernel<true>, dim3((unsigned)npasses), dim3(RP_THREADS), lds_full, st, d_seeds, d_n,
                       d_off, d_out, max_n, d_err);
  } else {
    hipLaunchKernelGGL(randperm_kernel<false>, dim3((unsigned)npasses), dim3(RP_THREADS), lds_small, st, d_seeds, d_n,
                       d_off, d_out, max_n, d_err);
  }
  FS_LAUNCH_CHECK();
  return FS_OK;
}
