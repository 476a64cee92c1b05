// Probe (round 6): the 4x4x1 multi-block operand layouts of the split form's "mb" instances,
// checked on one wave against a CPU product before they go into the kernel.
//
// One 64-column tile, 16 batch rows (one row tile), C classes in CB = ceil(C / 4) blocks of 4:
//   X register (the split form's row layout): lane (l16, lg), component e of register q
//       = X[l16][16 q + 4 lg + e]
//   W register wm[cb] (new): lane 16 lg + 4 q + i, component e = W[4 cb + i][16 q + 4 lg + e]
//   forward: acc[cb] += mfma_4x4x1(A = wm[cb].e, B = x[q].e, cbsz 2, abid q)
//       -> lane 16 lg + l16, register i: partial z[l16][4 cb + i] over k-group lg
//   k-group sum: permlane32 / permlane16 swaps + adds, 4 registers -> 1:
//       lane 16 lg + l16 of out[cb] = z[l16][4 cb + perm(lg)], perm = {0, 2, 1, 3}
//   backward: ga[cb] += mfma_4x4x1(A = image row r at lane-column 16 q + 4 lg + e (lane 16 lg + 4 q + e),
//                                  B = g row r (lane 16 s + 4 x + j = g[r][4 s + j]), blgp 4 + cb)
//       -> lane 16 lg + 4 q + j, register e: grad[4 cb + j][16 q + 4 lg + e]  (= wm's layout)
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probe/mb_layout.hip -o /tmp/mb_layout && /tmp/mb_layout
#include <hip/hip_runtime.h>

#include <cmath>
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

constexpr int CB = 3;

template <int A, int Q, int BL>
__device__ __forceinline__ floatx4 mf(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, A, Q, BL);
}

__device__ __forceinline__ float comp(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }

__device__ __forceinline__ void swap32(float& a, float& b) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap16(float& a, float& b) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
// lanes 16 lg + l16 of the result: acc register perm(lg) summed over the four k-groups
__device__ __forceinline__ float kgroup_sum(floatx4 a) {
  float r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3];
  swap32(r0, r1);
  swap32(r2, r3);
  float s01 = r0 + r1, s23 = r2 + r3;
  swap16(s01, s23);
  return s01 + s23;
}

// X [16][64], W [CB*4][64], g [16][16] (classes padded), out: z [16][16], grad [16][64]
__global__ void probe(const float* X, const float* W, const float* g, float* z, float* grad, float* raw) {
  const int lane = threadIdx.x, l16 = lane & 15, lg = lane >> 4, mq = (lane >> 2) & 3, mi = lane & 3;
  __shared__ float img[16][64];
  float4 xf[4];
  for (int q = 0; q < 4; ++q) xf[q] = *reinterpret_cast<const float4*>(X + l16 * 64 + 16 * q + 4 * lg);
  float4 wm[CB];
  for (int cb = 0; cb < CB; ++cb) wm[cb] = *reinterpret_cast<const float4*>(W + (4 * cb + mi) * 64 + 16 * mq + 4 * lg);
  floatx4 acc[CB];
  for (int cb = 0; cb < CB; ++cb) acc[cb] = floatx4{0.f, 0.f, 0.f, 0.f};
#define FQ(Q)                                                                   \
  for (int e = 0; e < 4; ++e)                                                   \
    for (int cb = 0; cb < CB; ++cb) acc[cb] = mf<2, Q, 0>(comp(wm[cb], e), comp(xf[Q], e), acc[cb]);
  FQ(0) FQ(1) FQ(2) FQ(3)
#undef FQ
  for (int cb = 0; cb < CB; ++cb)
    for (int i = 0; i < 4; ++i) raw[(cb * 4 + i) * 64 + lane] = acc[cb][i];
  const int perm[4] = {0, 2, 1, 3};
  for (int cb = 0; cb < CB; ++cb) {
    const float s = kgroup_sum(acc[cb]);
    z[l16 * 16 + 4 * cb + perm[lg]] = s;
  }
  // image: row-major
  for (int q = 0; q < 4; ++q)
    for (int e = 0; e < 4; ++e) img[l16][16 * q + 4 * lg + e] = comp(xf[q], e);
  __syncthreads();
  floatx4 ga[CB];
  for (int cb = 0; cb < CB; ++cb) ga[cb] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < 16; ++r) {
    const float a = img[r][16 * mq + 4 * lg + mi];   // lane 16 lg + 4 q + e -> column 16 q + 4 lg + e
    const float gr = g[r * 16 + 4 * lg + mi];         // lane 16 s + 4 x + j -> g[r][4 s + j]
    ga[0] = mf<0, 0, 4>(a, gr, ga[0]);
    ga[1] = mf<0, 0, 5>(a, gr, ga[1]);
    ga[2] = mf<0, 0, 6>(a, gr, ga[2]);
  }
  for (int cb = 0; cb < CB; ++cb)
    for (int e = 0; e < 4; ++e) grad[(4 * cb + mi) * 64 + 16 * mq + 4 * lg + e] = ga[cb][e];
}

int main() {
  std::vector<float> X(16 * 64), W(CB * 4 * 64), g(16 * 16, 0.f);
  srand(7);
  auto rnd = []() { return (float)((rand() % 2001) - 1000) / 1000.f; };
  for (auto& v : X) v = rnd();
  for (auto& v : W) v = rnd();
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 4 * CB; ++c) g[r * 16 + c] = rnd();
  float *dX, *dW, *dg, *dz, *dgr, *draw;
  CK(hipMalloc(&dX, X.size() * 4));
  CK(hipMalloc(&dW, W.size() * 4));
  CK(hipMalloc(&dg, g.size() * 4));
  CK(hipMalloc(&dz, 256 * 4));
  CK(hipMalloc(&dgr, 16 * 64 * 4));
  CK(hipMalloc(&draw, CB * 4 * 64 * 4));
  CK(hipMemset(dz, 0, 256 * 4));
  CK(hipMemset(dgr, 0, 16 * 64 * 4));
  CK(hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dW, W.data(), W.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dg, g.data(), g.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dX, dW, dg, dz, dgr, draw);
  CK(hipDeviceSynchronize());
  std::vector<float> z(256), gr(16 * 64), raw(CB * 4 * 64);
  CK(hipMemcpy(z.data(), dz, 256 * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(gr.data(), dgr, 16 * 64 * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(raw.data(), draw, raw.size() * 4, hipMemcpyDeviceToHost));
  double ez = 0, eg = 0, eraw = 0;
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 4 * CB; ++c) {
      double s = 0;
      for (int k = 0; k < 64; ++k) s += (double)X[r * 64 + k] * W[c * 64 + k];
      ez = fmax(ez, fabs(s - z[r * 16 + c]));
      // raw: lane 16 lg + l16, register i of acc[cb]: partial over k-group lg
      for (int lg = 0; lg < 4; ++lg) {
        double p = 0;
        for (int q = 0; q < 4; ++q)
          for (int e = 0; e < 4; ++e) {
            const int k = 16 * q + 4 * lg + e;
            p += (double)X[r * 64 + k] * W[c * 64 + k];
          }
        eraw = fmax(eraw, fabs(p - raw[((c / 4) * 4 + (c % 4)) * 64 + 16 * lg + r]));
      }
    }
  for (int c = 0; c < 4 * CB; ++c)
    for (int k = 0; k < 64; ++k) {
      double s = 0;
      for (int r = 0; r < 16; ++r) s += (double)g[r * 16 + c] * X[r * 64 + k];
      eg = fmax(eg, fabs(s - gr[c * 64 + k]));
    }
  printf("forward raw partials max err %.3e\nforward summed logits max err %.3e\nbackward grad max err %.3e\n", eraw, ez, eg);
  printf("%s\n", (ez < 1e-4 && eg < 1e-4 && eraw < 1e-4) ? "LAYOUTS OK" : "LAYOUT MISMATCH");
  return 0;
}
