// Probe: the cross-lane building blocks of the quarter-wave p-solver (lanes.h) on one wave,
// against their intended results computed on the host.  Prints "ok" / the mismatching lanes.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../non-iid-distributed-learning-with-optimal-mixture-weights_amd/csrc/lanes.h"

using namespace fs;

__global__ void k(float* out) {
  const int l = threadIdx.x;
  float v[16];
  for (int c = 0; c < 16; ++c) v[c] = (float)(1000 * c + l);
  for (int i = 0; i < 8; ++i) v[i] = rs_bank<8>(v[i], v[i + 8]);
  out[0 * 64 + l] = v[0];                                  // after level 8: class (l & 8) of slot 0
  for (int i = 0; i < 4; ++i) v[i] = rs_bank<4>(v[i], v[i + 4]);
  out[1 * 64 + l] = v[0];
  for (int i = 0; i < 2; ++i) v[i] = rs_pair(v[i], v[i + 2], 2, l);
  out[2 * 64 + l] = rs_pair(v[0], v[1], 1, l);             // class r's row total
  out[3 * 64 + l] = row16_all<false>((float)l);
  out[4 * 64 + l] = row16_all<true>((float)((l * 7) % 13));
  float lo, hi;
  gather_pair<16>((float)l, lo, hi);
  out[5 * 64 + l] = lo;
  out[6 * 64 + l] = hi;
  gather_pair<32>((float)l, lo, hi);
  out[7 * 64 + l] = lo;
  out[8 * 64 + l] = hi;
  out[9 * 64 + l] = rs_level<32, true>((float)l, (float)(100 + l), l);
  out[10 * 64 + l] = rs_level<16, true>((float)l, (float)(100 + l), l);
}

int main() {
  float* d;
  hipMalloc(&d, 11 * 64 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float h[11 * 64];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  auto chk = [&](int t, int l, double want, const char* nm) {
    if (h[t * 64 + l] != (float)want) {
      if (bad++ < 40) printf("%-10s lane %2d: got %g want %g\n", nm, l, h[t * 64 + l], want);
    }
  };
  for (int l = 0; l < 64; ++l) {
    const int q = l >> 4, r = l & 15;
    auto val = [&](int c, int lane) { return 1000.0 * c + lane; };
    const int c8 = (r & 8);                                  // level 8 keeps class 8*bit3 in slot 0
    chk(0, l, val(c8, l) + val(c8, l ^ 8), "rs8");
    const int c4 = c8 + (r & 4);
    double s4 = 0;
    for (int k = 0; k < 4; ++k) s4 += val(c4, (l & ~12) | (k << 2));
    chk(1, l, s4, "rs4");
    double s16 = 0;
    for (int k = 0; k < 16; ++k) s16 += val(r, 16 * q + k);
    chk(2, l, s16, "rs_full");
    double rs = 0;
    for (int k = 0; k < 16; ++k) rs += 16 * q + k;
    chk(3, l, rs, "row_sum");
    int mx = 0;
    for (int k = 0; k < 16; ++k) mx = mx > ((16 * q + k) * 7) % 13 ? mx : ((16 * q + k) * 7) % 13;
    chk(4, l, mx, "row_max");
    chk(5, l, l & ~16, "g16.lo");
    chk(6, l, l | 16, "g16.hi");
    chk(7, l, l & ~32, "g32.lo");
    chk(8, l, l | 32, "g32.hi");
    chk(9, l, l < 32 ? (double)(l + l + 32) : (double)(100 + l - 32 + 100 + l), "rsl32");
    chk(10, l, (l & 16) ? (double)(100 + (l & ~16) + 100 + l) : (double)(l + (l | 16)), "rsl16");
  }
  printf(bad ? "FAIL %d\n" : "ok\n", bad);
  return bad ? 1 : 0;
}
