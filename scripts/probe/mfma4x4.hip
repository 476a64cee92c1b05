// Probe (round 6): v_mfma_f32_4x4x1_16b_f32 on gfx950 -- issue cycles and operand/result layouts.
//
// The split local-training form computes C = 10 classes on v_mfma_f32_16x16x4_f32, which pads
// the classes to 16 (37.5 % of its MFMA cycles do no work).  The 16-block 4x4x1 form pads them to
// 12 -- if it issues at the f32 rate (8 cycles per instruction per SIMD for 16 blocks x 4 x 4 x 1
// x 2 flop).  This probe measures
//   (1) cycles per instruction, back-to-back, 1..8 independent accumulators (and 16x16x4 beside);
//   (2) where each A / B lane lands in the result, with the CBSZ / ABID (A broadcast) and BLGP
//       (B lane-group) modifiers the kernel would use.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probe/mfma4x4.hip -o /tmp/mfma4x4 && /tmp/mfma4x4
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// ---------------- layouts ----------------
// out[(m * 64 + lane) * 4 + r] = result register r of lane `lane` for mode m.
template <int CBSZ, int ABID, int BLGP>
__device__ f4 mf(float a, float b) {
  f4 z = {0.f, 0.f, 0.f, 0.f};
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, z, CBSZ, ABID, BLGP);
}

__global__ void layout_kernel(float* out) {
  const int l = threadIdx.x;
  // a codes the lane in the units, b codes the lane in the thousands: A lane = v % 1000 - 1 when
  // b = 1, etc.  Run with one operand 1 and the other 1 + lane so each product names its lane.
  const float one = 1.f, lid = 1.f + (float)l;
  f4 r[12];
  r[0] = mf<0, 0, 0>(lid, one);   // A lane map
  r[1] = mf<0, 0, 0>(one, lid);   // B lane map
  r[2] = mf<3, 0, 0>(lid, one);   // A broadcast in groups of 8 blocks from block 0
  r[3] = mf<3, 5, 0>(lid, one);   // ... from block 5
  r[4] = mf<4, 9, 0>(lid, one);   // all 16 blocks from block 9
  r[5] = mf<0, 0, 1>(one, lid);   // BLGP 1
  r[6] = mf<0, 0, 2>(one, lid);   // BLGP 2
  r[7] = mf<0, 0, 3>(one, lid);   // BLGP 3
  r[8] = mf<0, 0, 4>(one, lid);   // BLGP 4
  r[9] = mf<0, 0, 5>(one, lid);   // BLGP 5
  r[10] = mf<2, 1, 0>(lid, one);  // groups of 4 blocks from block 1
  r[11] = mf<1, 1, 0>(lid, one);  // groups of 2 from block 1
  for (int m = 0; m < 12; ++m)
    for (int q = 0; q < 4; ++q) out[(m * 64 + l) * 4 + q] = r[m][q];
}

// ---------------- timing ----------------
template <int NACC, int KIND>
__global__ __launch_bounds__(512) void time_kernel(const float* in, float* out, int iters, unsigned long long* cyc) {
  const int l = threadIdx.x;
  float a = in[l & 63], b = in[64 + (l & 63)];
  f4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f4{0.f, 0.f, 0.f, (float)i};
  __syncthreads();
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      if (KIND == 0)
        acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
      else
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  f4 s = acc[0];
  for (int i = 1; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + l] = s[0] + s[1] + s[2] + s[3];
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NACC, int KIND>
static double time_one(const float* din, float* dout, unsigned long long* dcyc, int threads, int iters) {
  hipLaunchKernelGGL((time_kernel<NACC, KIND>), dim3(1), dim3(threads), 0, 0, din, dout, iters, dcyc);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL((time_kernel<NACC, KIND>), dim3(1), dim3(threads), 0, 0, din, dout, iters, dcyc);
  CK(hipDeviceSynchronize());
  unsigned long long c;
  CK(hipMemcpy(&c, dcyc, sizeof c, hipMemcpyDeviceToHost));
  return (double)c / ((double)iters * NACC);
}

int main() {
  float* dout;
  CK(hipMalloc(&dout, 12 * 64 * 4 * sizeof(float)));
  hipLaunchKernelGGL(layout_kernel, dim3(1), dim3(64), 0, 0, dout);
  CK(hipDeviceSynchronize());
  std::vector<float> h(12 * 64 * 4);
  CK(hipMemcpy(h.data(), dout, h.size() * sizeof(float), hipMemcpyDeviceToHost));
  const char* names[12] = {"A map (cbsz0)",  "B map (blgp0)", "A cbsz3 abid0", "A cbsz3 abid5", "A cbsz4 abid9", "B blgp1",
                           "B blgp2",        "B blgp3",       "B blgp4",       "B blgp5",       "A cbsz2 abid1", "A cbsz1 abid1"};
  for (int m = 0; m < 12; ++m) {
    printf("== %s: reg r of lane l holds (source lane); one line per register\n", names[m]);
    for (int q = 0; q < 4; ++q) {
      printf("r%d:", q);
      for (int l = 0; l < 64; ++l) printf(" %d", (int)h[(m * 64 + l) * 4 + q] - 1);
      printf("\n");
    }
  }
  float *din, *dt;
  unsigned long long* dcyc;
  CK(hipMalloc(&din, 128 * sizeof(float)));
  CK(hipMalloc(&dt, 512 * sizeof(float)));
  CK(hipMalloc(&dcyc, 8 * sizeof(unsigned long long)));
  std::vector<float> hin(128);
  for (int i = 0; i < 128; ++i) hin[i] = 0.001f * (float)(i % 17);
  CK(hipMemcpy(din, hin.data(), 128 * sizeof(float), hipMemcpyHostToDevice));
  const int iters = 4096;
  for (int threads : {64, 256, 512}) {
    printf("== cycles per MFMA per wave, %d threads (%d waves, 4 SIMDs)\n", threads, threads / 64);
    printf("4x4x1_16b  acc 1 %.2f  2 %.2f  4 %.2f  8 %.2f\n", time_one<1, 0>(din, dt, dcyc, threads, iters),
           time_one<2, 0>(din, dt, dcyc, threads, iters), time_one<4, 0>(din, dt, dcyc, threads, iters),
           time_one<8, 0>(din, dt, dcyc, threads, iters));
    printf("16x16x4    acc 1 %.2f  2 %.2f  4 %.2f  8 %.2f\n", time_one<1, 1>(din, dt, dcyc, threads, iters),
           time_one<2, 1>(din, dt, dcyc, threads, iters), time_one<4, 1>(din, dt, dcyc, threads, iters),
           time_one<8, 1>(din, dt, dcyc, threads, iters));
  }
  return 0;
}
