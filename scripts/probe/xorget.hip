// Probe: lanes.h xor_get / rs_pair per offset.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../non-iid-distributed-learning-with-optimal-mixture-weights_amd/csrc/lanes.h"
using namespace fs;
__global__ void k(float* out) {
  const int l = threadIdx.x;
  const float x = (float)l;
#pragma unroll
  for (int i = 0, off = 1; off <= 32; ++i, off <<= 1) {
    out[i * 64 + l] = xor_get(x, off, l);
    out[(6 + i) * 64 + l] = rs_pair(x, 100.f + x, off, l);
  }
}
int main() {
  float* d;
  (void)hipMalloc(&d, 12 * 64 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float h[12 * 64];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 6; ++i) {
    const int off = 1 << i;
    for (int l = 0; l < 64; ++l) {
      const int p = l ^ off;
      const float want = (float)p, keep = (l & off) ? 100.f + l : (float)l, recv = (l & off) ? 100.f + p : (float)p;
      if (h[i * 64 + l] != want) { if (bad++ < 8) printf("xor_get off=%d lane %d got %g want %g\n", off, l, h[i * 64 + l], want); }
      if (h[(6 + i) * 64 + l] != keep + recv) { if (bad++ < 16) printf("rs_pair off=%d lane %d got %g want %g\n", off, l, h[(6 + i) * 64 + l], keep + recv); }
    }
  }
  printf("%s\n", bad ? "FAIL" : "ok");
  return bad != 0;
}
