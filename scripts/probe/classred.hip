// Probe: lanes.h class_totals / class_max / class_sum against host sums, every CP.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include "../../non-iid-distributed-learning-with-optimal-mixture-weights_amd/csrc/lanes.h"
using namespace fs;
__device__ float val(int l, int c) { return (float)((l * 7 + c * 13) % 17) + 0.25f * c; }
template <int CP>
__global__ void k(float* out) {
  const int l = threadIdx.x;
  float v[CP];
  for (int c = 0; c < CP; ++c) v[c] = val(l, c);
  const float o = class_totals<CP>(v, l);
  out[l] = o;
  out[64 + l] = class_max<64 / CP>(o, l);
  out[128 + l] = class_sum<64 / CP>(o, l);
}
static float hval(int l, int c) { return (float)((l * 7 + c * 13) % 17) + 0.25f * c; }
template <int CP>
int run() {
  float* d;
  (void)hipMalloc(&d, 3 * 64 * 4);
  hipLaunchKernelGGL(k<CP>, dim3(1), dim3(64), 0, 0, d);
  float h[192];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  int bad = 0;
  float tot[32], mx = -1e30f, sm = 0;
  for (int c = 0; c < CP; ++c) {
    tot[c] = 0;
    for (int l = 0; l < 64; ++l) tot[c] += hval(l, c);
    mx = fmaxf(mx, tot[c]);
    sm += tot[c];
  }
  for (int l = 0; l < 64; ++l) {
    const int c = l / (64 / CP);
    if (h[l] != tot[c]) { if (bad < 5) printf("CP=%d lane %d total %g want %g\n", CP, l, h[l], tot[c]); ++bad; }
    if (h[64 + l] != mx) { if (bad < 5) printf("CP=%d lane %d max %g want %g\n", CP, l, h[64 + l], mx); ++bad; }
    if (h[128 + l] != sm) { if (bad < 5) printf("CP=%d lane %d sum %g want %g\n", CP, l, h[128 + l], sm); ++bad; }
  }
  printf("CP=%d: %s\n", CP, bad ? "FAIL" : "ok");
  return bad;
}
int main() { return (run<2>() + run<4>() + run<8>() + run<16>() + run<32>()) ? 1 : 0; }
