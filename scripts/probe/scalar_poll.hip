// Probe (round 6): can the split form's hand-off polls leave the vector-memory queue?
//
// A step of the split local-training form (csrc/local_train_split.hip, G = 2) publishes the
// workgroup's B x C partial logits as {tag, value} granules, polls the partner's, and streams
// 128 KB of next-step rows per CU.  The polls are vector loads: issued behind row loads they
// return only after them (one in-order vector-memory path per CU), so the rows are issued after
// the polls return.  This probe runs groups of 2 workgroups (8 waves, partners on one XCD) that
// per step publish 320 granules, issue NL of each wave's 16 row loads (1 KB each, gathered rows
// of a 400 MB table), poll the partner, issue the rest of the rows inside a dependent VALU
// "backward", and wait for them -- with the polls as
//   MODE 0: relaxed agent-scope vector loads (the shipped form), or
//   MODE 1: scalar loads with glc (scalar-cache miss), 40 granules per wave, tags checked on the
//           scalar unit, values moved into lanes with v_writelane_b32.
// Every value read is checked against what the partner published (err bit 2); every spin is bounded
// (err bit 1).
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probe/scalar_poll.hip -o /tmp/scalar_poll && /tmp/scalar_poll
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int WAVES = 8;
constexpr int NV = 320;   // granules per workgroup and step (B x C = 32 x 10)
constexpr int GPW = 40;   // granules per wave in the scalar form
constexpr unsigned SPIN_LIMIT = 1u << 20;
constexpr int ROWF = 2048;  // floats per row (D = 2048)

typedef unsigned u32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float pubval(unsigned tag, int g, int idx) { return (float)(tag * 3u + (unsigned)g * 7u) + 0.25f * idx; }

template <int MODE, int NL>
__global__ __launch_bounds__(WAVES * 64, 1) void probe_kernel(const float* phi, int nrows, unsigned long long* slots,
                                                            int ngroups, int steps, int delay, int work, unsigned* err,
                                                            unsigned long long* cyc, float* sink) {
  const int b = blockIdx.x, xcd = b % 8, r = b / 8, g = r & 1, grp = xcd + 8 * (r >> 1);
  if (grp >= ngroups) return;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  unsigned long long t0 = __builtin_readcyclecounter();
  float acc = 0.f;
  bool dead = false;
  unsigned bad = 0;
  for (int s = 0; s < steps; ++s) {
    const unsigned tag = (unsigned)s + 1u;
    const int par = s & 1;
    unsigned long long* mine = slots + (((int64_t)grp * 2 + par) * 2 + g) * NV;
    unsigned long long* peer = slots + (((int64_t)grp * 2 + par) * 2 + (g ^ 1)) * NV;
    const int idx = w * 64 + lane;
    if (idx < NV)
      __hip_atomic_store(mine + idx, ((unsigned long long)tag << 32) | __float_as_uint(pubval(tag, g, idx)),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the step's row stream: 16 loads of 1 KB per wave (gathered rows)
    float4 xr[16];
    auto issue = [&](int i) {
      const unsigned h = (unsigned)(s * 2654435761u) ^ (unsigned)(grp * 40503u + w * 977u + i * 131u + g * 7u);
      const int row = (int)(h % (unsigned)nrows);
      xr[i] = *reinterpret_cast<const float4*>(phi + (int64_t)row * ROWF + 1024 * g + 256 * (i & 3) + 4 * lane);
    };
#pragma unroll
    for (int i = 0; i < NL; ++i) issue(i);
    for (int d = 0; d < delay; ++d) __builtin_amdgcn_s_sleep(1);
    float got = 0.f;
    if constexpr (MODE == 0) {
      if (idx < NV) {
        unsigned long long v = 0;
        unsigned spins = 0;
        for (;;) {
          v = __hip_atomic_load(peer + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((unsigned)(v >> 32) == tag) break;
          if (dead || ++spins > SPIN_LIMIT) {
            dead = true;
            bad |= 1u;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        got = __uint_as_float((unsigned)v);
        if (!dead && got != pubval(tag, g ^ 1, idx)) bad |= 2u;
      }
    } else {
      const unsigned long long* q = peer + GPW * w;
      unsigned spins = 0;
      for (;;) {
        u32x16 a0, a1, a2, a3, a4;
        asm volatile(
            "s_load_dwordx16 %0, %5, 0x0 glc\n\t"
            "s_load_dwordx16 %1, %5, 0x40 glc\n\t"
            "s_load_dwordx16 %2, %5, 0x80 glc\n\t"
            "s_load_dwordx16 %3, %5, 0xc0 glc\n\t"
            "s_load_dwordx16 %4, %5, 0x100 glc\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=s"(a0), "=s"(a1), "=s"(a2), "=s"(a3), "=s"(a4)
            : "s"(q)
            : "memory");
        bool ok = true;
#pragma unroll
        for (int i = 0; i < 8; ++i) ok &= (a0[2 * i + 1] == tag) & (a1[2 * i + 1] == tag) & (a2[2 * i + 1] == tag) &
                                         (a3[2 * i + 1] == tag) & (a4[2 * i + 1] == tag);
        if (ok) {
          float v = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(a0[2 * i]), "n"(i));
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(a1[2 * i]), "n"(8 + i));
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(a2[2 * i]), "n"(16 + i));
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(a3[2 * i]), "n"(24 + i));
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(a4[2 * i]), "n"(32 + i));
          }
          got = v;
          const int gi = GPW * w + lane;
          if (lane < GPW && gi < NV && got != pubval(tag, g ^ 1, gi)) bad |= 2u;
          break;
        }
        if (dead || ++spins > SPIN_LIMIT) {
          dead = true;
          bad |= 1u;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    // the "softmax + backward": a dependent VALU chain with the rest of the rows issued inside it
    float x = got * 1e-9f + acc;
#pragma unroll
    for (int i = NL; i < 16; ++i) {
      issue(i);
      for (int k = 0; k < work; ++k) x = __builtin_fmaf(x, 0.999f, 1e-7f);
    }
    for (int k = 0; k < work * (NL + 1); ++k) x = __builtin_fmaf(x, 0.999f, 1e-7f);
#pragma unroll
    for (int i = 0; i < 16; ++i) x += (xr[i].x + xr[i].y + xr[i].z + xr[i].w) * 1e-12f;
    acc = x;
    __syncthreads();
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  if (bad) __hip_atomic_fetch_or(err, bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x == 0) cyc[grp * 2 + g] = t1 - t0;
  if (acc == 1234.5f) sink[threadIdx.x] = acc;
}

#define CHECK(x)                                                       \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));   \
      std::exit(1);                                                    \
    }                                                                  \
  } while (0)

template <int MODE, int NL>
static void run(const float* phi, int nrows, int ngroups, int steps, int delay, int work) {
  unsigned long long *slots, *cyc;
  unsigned* err;
  float* sink;
  const size_t ns = (size_t)ngroups * 2 * 2 * NV;
  CHECK(hipMalloc(&slots, ns * 8));
  CHECK(hipMalloc(&err, 4));
  CHECK(hipMalloc(&cyc, ngroups * 2 * 8));
  CHECK(hipMalloc(&sink, 512 * 4));
  const int grid = 8 * 2 * ((ngroups + 7) / 8);
  float best = 1e30f;
  double bc = 0;
  unsigned e = 0;
  for (int rep = 0; rep < 3 && !e; ++rep) {
    CHECK(hipMemset(slots, 0, ns * 8));
    CHECK(hipMemset(err, 0, 4));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((probe_kernel<MODE, NL>), dim3(grid), dim3(WAVES * 64), 0, 0, phi, nrows, slots, ngroups, steps,
                       delay, work, err, cyc, sink);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    std::vector<unsigned long long> c(ngroups * 2);
    CHECK(hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost));
    double mc = 0;
    for (auto x : c) mc += (double)x / c.size();
    if (ms < best) {
      best = ms;
      bc = mc / steps;
    }
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
  }
  std::printf("%s NL=%2d groups=%3d delay=%2d work=%3d: %7.3f us/step (event), %6.0f ticks/step, err=%u%s\n",
              MODE ? "scalar" : "vector", NL, ngroups, delay, work, 1e3 * best / steps, bc, e,
              e & 1 ? " (spin bound)" : (e & 2 ? " (WRONG VALUE)" : ""));
  std::fflush(stdout);
  CHECK(hipFree(slots));
  CHECK(hipFree(err));
  CHECK(hipFree(cyc));
  CHECK(hipFree(sink));
}

int main() {
  const int nrows = 51200;
  float* phi;
  CHECK(hipMalloc(&phi, (size_t)nrows * ROWF * 4));
  CHECK(hipMemset(phi, 0, (size_t)nrows * ROWF * 4));
  const int steps = 2000;
  // coherence first: one group, no rows
  run<1, 0>(phi, nrows, 1, steps, 0, 0);
  run<0, 0>(phi, nrows, 1, steps, 0, 0);
  for (int ng : {1, 100}) {
    for (int work : {0, 16}) {
      run<0, 0>(phi, nrows, ng, steps, 0, work);
      run<0, 6>(phi, nrows, ng, steps, 0, work);
      run<1, 0>(phi, nrows, ng, steps, 0, work);
      run<1, 6>(phi, nrows, ng, steps, 0, work);
      run<1, 10>(phi, nrows, ng, steps, 0, work);
      run<1, 16>(phi, nrows, ng, steps, 0, work);
    }
  }
  CHECK(hipFree(phi));
  return 0;
}
