// Probe (round 6): the split form's forward MFMA stream at config 2 (8 waves = 2 per SIMD, one
// wave's tiles: 2 tiles x 2 row tiles x 16 columns-groups), as the 16x16x4 instances issue it
// (64 MFMAs per wave, 2 accumulators) and as the mb instances do (192 4x4x1_16b MFMAs per wave,
// 6 accumulators, cbsz 2 / abid q) -- cycles per forward per wave, operands from distinct
// registers as in the kernel.  (scripts/probe/mfma4x4.hip measured one register pair reused.)
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probe/mb_fwd_rate.hip -o /tmp/mb_fwd_rate && /tmp/mb_fwd_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__device__ __forceinline__ float comp(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }

template <int Q>
__device__ __forceinline__ void mbq(floatx4 (&acc)[2][3], const float4 (&xt)[2][4], const float4 (&wt)[3]) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int cb = 0; cb < 3; ++cb)
        acc[rt][cb] = __builtin_amdgcn_mfma_f32_4x4x1f32(comp(wt[cb], e), comp(xt[rt][Q], e), acc[rt][cb], 2, Q, 0);
}

template <int MB>
__global__ __launch_bounds__(512) void fwd_rate(const float* in, float* out, int iters, unsigned long long* cyc) {
  const int l = threadIdx.x & 63;
  float4 xf[2][2][4];
  float4 wr[2][4];
  for (int i = 0; i < 2; ++i)
    for (int rt = 0; rt < 2; ++rt)
      for (int q = 0; q < 4; ++q) xf[i][rt][q] = *reinterpret_cast<const float4*>(in + 4 * ((l + 16 * (i * 8 + rt * 4 + q)) & 255));
  for (int i = 0; i < 2; ++i)
    for (int q = 0; q < 4; ++q) wr[i][q] = *reinterpret_cast<const float4*>(in + 4 * ((l + 7 * (i * 4 + q)) & 255));
  floatx4 acc[2][3];
  floatx4 acc16[2];
  for (int rt = 0; rt < 2; ++rt) {
    acc16[rt] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int cb = 0; cb < 3; ++cb) acc[rt][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if constexpr (MB) {
        float4 wt[3] = {wr[i][0], wr[i][1], wr[i][2]};
        mbq<0>(acc, xf[i], wt);
        mbq<1>(acc, xf[i], wt);
        mbq<2>(acc, xf[i], wt);
        mbq<3>(acc, xf[i], wt);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
              acc16[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(xf[i][rt][q], e), comp(wr[i][q], e), acc16[rt], 0, 0, 0);
      }
    }
    asm volatile("" ::: "memory");
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  float s = 0.f;
  for (int rt = 0; rt < 2; ++rt) {
    s += acc16[rt][0] + acc16[rt][3];
    for (int cb = 0; cb < 3; ++cb) s += acc[rt][cb][0] + acc[rt][cb][1] + acc[rt][cb][2] + acc[rt][cb][3];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
}

template <int MB>
static void run(const float* din, float* dout, unsigned long long* dcyc, int threads, int iters, const char* name) {
  for (int k = 0; k < 2; ++k) {
    hipLaunchKernelGGL((fwd_rate<MB>), dim3(1), dim3(threads), 0, 0, din, dout, iters, dcyc);
    CK(hipDeviceSynchronize());
  }
  std::vector<unsigned long long> c(8);
  CK(hipMemcpy(c.data(), dcyc, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  double mx = 0;
  for (int w = 0; w < threads / 64; ++w) mx = c[w] > mx ? (double)c[w] : mx;
  printf("%-8s %d waves: %.0f cycles per wave-forward (%d MFMAs per wave)\n", name, threads / 64, mx / iters, MB ? 192 : 64);
}

int main() {
  float *din, *dout;
  unsigned long long* dcyc;
  CK(hipMalloc(&din, 1024 * sizeof(float)));
  CK(hipMalloc(&dout, 512 * sizeof(float)));
  CK(hipMalloc(&dcyc, 8 * sizeof(unsigned long long)));
  std::vector<float> h(1024);
  srand(3);
  for (auto& v : h) v = (float)((rand() % 2001) - 1000) / 1000.f;
  CK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  for (int threads : {64, 256, 512}) {
    run<0>(din, dout, dcyc, threads, 2000, "16x16x4");
    run<1>(din, dout, dcyc, threads, 2000, "4x4x1");
  }
  return 0;
}
