// Probe: semantics of the gfx950 permlane swaps and the DPP controls used by mixture.hip.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL>
__device__ int dpp(int x) { return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false); }
__global__ void k(int* out) {
  const int l = threadIdx.x;
  const int a = l, b = 100 + l;
  auto r32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  auto r16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  out[0 * 64 + l] = r32[0];
  out[1 * 64 + l] = r32[1];
  out[2 * 64 + l] = r16[0];
  out[3 * 64 + l] = r16[1];
  out[4 * 64 + l] = dpp<0x104>(a);
  out[5 * 64 + l] = dpp<0x114>(a);
  out[6 * 64 + l] = dpp<0x128>(a);
  out[7 * 64 + l] = dpp<0xB1>(a);
  out[8 * 64 + l] = dpp<0x4E>(a);
}
int main() {
  int* d;
  hipMalloc(&d, 9 * 64 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[9 * 64];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[9] = {"p32[0]", "p32[1]", "p16[0]", "p16[1]", "row_shl4", "row_shr4", "row_ror8", "qp_B1", "qp_4E"};
  for (int r = 0; r < 9; ++r) {
    printf("%-9s", nm[r]);
    for (int l = 0; l < 64; ++l) printf(" %d", h[r * 64 + l]);
    printf("\n");
  }
  return 0;
}
