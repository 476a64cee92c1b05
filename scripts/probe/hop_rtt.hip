// Probe: the floor of one all-to-all hand-off hop among K workgroups on one XCD -- the exchange
// the qmc p-solver (mixture.hip) and the split/pipe local-training forms run once per step, here
// with no other work: every step each workgroup publishes `vals` {tag, value} granules per wave
// (relaxed agent-scope stores, the data is its own flag) and polls its K - 1 partners' granules
// until every tag is the step's (relaxed agent-scope loads, re-polled in one batch per round trip),
// then goes on.  Time per step = one hop with zero skew and zero compute.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probe/hop_rtt.hip -o /tmp/hop_rtt && /tmp/hop_rtt
//
// Workgroups with blockIdx % 8 == 0 (one XCD under the round-robin dispatch) take part; the
// others exit at once.  Every spin is bounded (the grid drains even if a partner never arrives).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int WAVES = 4;
constexpr unsigned SPIN_LIMIT = 1u << 20;

template <int VALS>  // granules per lane per wave and partner (qmc at C = 10: 4 rows x 10 / 16 lanes ~ 3)
__global__ __launch_bounds__(WAVES * 64) void hop_kernel(unsigned long long* slots, int K, int steps, int sleep_first,
                                                         unsigned* err, unsigned long long* cycles) {
  if (blockIdx.x % 8 != 0) return;
  const int k = blockIdx.x / 8;
  if (k >= K) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // slot layout: [parity][workgroup][wave][VALS][64]
  auto at = [&](int par, int wg, int v) {
    return slots + ((((int64_t)par * K + wg) * WAVES + w) * VALS + v) * 64 + lane;
  };
  unsigned long long t0 = __builtin_readcyclecounter();  // s_memtime
  bool dead = false;
  float acc = 0.f;
  for (int s = 0; s < steps; ++s) {
    const unsigned tag = (unsigned)s + 1u;
    const int par = s & 1;
#pragma unroll
    for (int v = 0; v < VALS; ++v)
      __hip_atomic_store(at(par, k, v), ((unsigned long long)tag << 32) | __float_as_uint(acc + v),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (sleep_first > 0)
      for (int i = 0; i < sleep_first; ++i) __builtin_amdgcn_s_sleep(1);
    unsigned spins = 0;
    for (;;) {
      bool ok = true;
      float sum = 0.f;
      for (int p = 0; p < K; ++p) {
        if (p == k) continue;
#pragma unroll
        for (int v = 0; v < VALS; ++v) {
          const unsigned long long g = __hip_atomic_load(at(par, p, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok &= (unsigned)(g >> 32) == tag;
          sum += __uint_as_float((unsigned)g);
        }
      }
      if (__all(ok)) {
        acc = sum * 1e-9f;
        break;
      }
      if (dead || ++spins > SPIN_LIMIT) {
        if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dead = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) cycles[k] = t1 - t0 + (acc == 12345.f ? 1 : 0);
}

// The qmc-like hop: each lane polls VALS granules spread over the K - 1 partners (the qmc solver's
// lanes read ~10 each at K = 16, C = 10), and a re-poll reloads only the granules still stale
// (exec-masked loads), one batch per round trip.  Each wave publishes 256 granules per step.
template <int VALS>
__global__ __launch_bounds__(WAVES * 64) void hop_spread_kernel(unsigned long long* slots, int K, int steps,
                                                                int sleep_first, unsigned* err,
                                                                unsigned long long* cycles) {
  if (blockIdx.x % 8 != 0) return;
  const int k = blockIdx.x / 8;
  if (k >= K) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  auto at = [&](int par, int wg, int idx) { return slots + (((int64_t)par * K + wg) * WAVES + w) * 256 + idx; };
  int pp[VALS], pi[VALS];
#pragma unroll
  for (int v = 0; v < VALS; ++v) {
    const int i = lane * VALS + v;
    const int q = i % (K - 1);
    pp[v] = q + (q >= k ? 1 : 0);
    pi[v] = (i / (K - 1)) & 255;
  }
  unsigned long long t0 = __builtin_readcyclecounter();
  bool dead = false;
  float acc = 0.f;
  for (int s = 0; s < steps; ++s) {
    const unsigned tag = (unsigned)s + 1u;
    const int par = s & 1;
#pragma unroll
    for (int v = 0; v < 4; ++v)
      __hip_atomic_store(at(par, k, 64 * v + lane), ((unsigned long long)tag << 32) | __float_as_uint(acc + v),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int i = 0; i < sleep_first; ++i) __builtin_amdgcn_s_sleep(1);
    unsigned long long g[VALS];
#pragma unroll
    for (int v = 0; v < VALS; ++v) g[v] = __hip_atomic_load(at(par, pp[v], pi[v]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int v = 0; v < VALS; ++v) ok &= (unsigned)(g[v] >> 32) == tag;
      if (__all(ok)) break;
      if (dead || ++spins > SPIN_LIMIT) {
        if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dead = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int v = 0; v < VALS; ++v)
        if ((unsigned)(g[v] >> 32) != tag)
          g[v] = __hip_atomic_load(at(par, pp[v], pi[v]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    float sum = 0.f;
#pragma unroll
    for (int v = 0; v < VALS; ++v) sum += __uint_as_float((unsigned)g[v]);
    acc = sum * 1e-9f;
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) cycles[k] = t1 - t0 + (acc == 12345.f ? 1 : 0);
}

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

template <int VALS, bool SPREAD = false>
static void run(int K, int steps, int sleep_first) {
  unsigned long long* slots;
  unsigned* err;
  unsigned long long* cyc;
  const size_t n = (size_t)2 * K * WAVES * (SPREAD ? 256 : VALS * 64);
  CHECK(hipMalloc(&slots, n * 8));
  CHECK(hipMalloc(&err, 4));
  CHECK(hipMalloc(&cyc, K * 8));
  float best = 1e30f;
  double best_cyc = 0;
  for (int rep = 0; rep < 3; ++rep) {
    CHECK(hipMemset(slots, 0, n * 8));
    CHECK(hipMemset(err, 0, 4));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a));
    if (SPREAD)
      hipLaunchKernelGGL(hop_spread_kernel<VALS>, dim3(8 * K), dim3(WAVES * 64), 0, 0, slots, K, steps, sleep_first, err,
                         cyc);
    else
      hipLaunchKernelGGL(hop_kernel<VALS>, dim3(8 * K), dim3(WAVES * 64), 0, 0, slots, K, steps, sleep_first, err, cyc);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    unsigned e;
    CHECK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    if (e) {
      std::printf("K=%d vals=%d: a spin hit its bound\n", K, VALS);
      break;
    }
    std::vector<unsigned long long> c(K);
    CHECK(hipMemcpy(c.data(), cyc, K * 8, hipMemcpyDeviceToHost));
    double mc = 0;
    for (auto x : c) mc += (double)x / K;
    if (ms < best) {
      best = ms;
      best_cyc = mc / steps;
    }
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
  }
  std::printf("%s K=%2d granules/lane%s=%2d first-sleep=%2d: %.3f us per hop (event), %.0f s_memtime ticks per hop\n",
              SPREAD ? "spread" : "all   ", K, SPREAD ? "        " : "/partner", VALS, sleep_first, 1e3 * best / steps,
              best_cyc);
  CHECK(hipFree(slots));
  CHECK(hipFree(err));
  CHECK(hipFree(cyc));
}

int main() {
  const int steps = 20000;
  for (int K : {2, 4, 8, 16}) run<1>(K, steps, 0);
  for (int K : {2, 4, 8, 16}) run<3>(K, steps, 0);
  for (int sl : {4, 8, 16}) run<3>(16, steps, sl);
  for (int K : {2, 4, 8, 16}) run<1, true>(K, steps, 0);
  for (int K : {2, 4, 8, 16}) run<10, true>(K, steps, 0);
  for (int sl : {2, 4, 8, 12, 16, 20, 24, 32}) run<10, true>(16, steps, sl);
  for (int sl : {0, 8, 16, 24}) run<4, true>(16, steps, sl);
  return 0;
}
