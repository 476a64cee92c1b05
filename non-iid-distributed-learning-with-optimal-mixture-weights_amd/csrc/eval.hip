// fs_eval -- test-set cross-entropy and top-1 accuracy of the global model.
//
// Replaces test_loop + comp_accuracy + Meter (/root/reference/functions/tools.py:218-237,
// 82-96, 99-148).  The reference walks shuffled batches of 32 and averages per-batch
// means weighted by batch size, which equals the plain mean over all rows up to fp32
// rounding; the shuffle only matters for the RNG stream, which the host replays.
//
// Each 8-wave workgroup owns 16 test rows (eval_rows.h, the body the training launch's fused
// evaluation blocks share); its waves split the 64-column feature tiles (2 tiles of loads in
// flight per wave, ~5,000 waves for 10k rows so every CU streams), computing logits (16 x
// classes) with v_mfma_f32_16x16x4_f32; the partials are summed through LDS and wave 0
// computes CE and arg-max per row.  Per-block partial
// sums go to a workspace and a one-block finalizer folds them in a fixed order, so the
// result is bitwise reproducible run to run.  HBM-bound: one read of the test features.
#include "common.h"
#include "finalize.h"
#include "eval_rows.h"

namespace fs {

constexpr int EV_WAVES = 8;   // waves per workgroup splitting the feature tiles (8: 24.3 vs 26.2 us
                              // with 4 at config 2, 158 vs 164 us at config 3 -- r02s2ev3)
constexpr int EV_ROWS = 16;   // rows per workgroup (32 or 64 measured slower: config 2 26.6 / 32.0 /
                              // 34.8 us, config 3 163 / 184 / 218 us -- r02s2ev)

// one 16-row group per workgroup: eval_rows.h's body (the fused evaluation blocks of the
// training launch run the same one), its two partial sums to part[2 * blockIdx.x]
template <int CT>
__global__ __launch_bounds__(EV_WAVES * 64) void eval_kernel(const float* __restrict__ phi, int64_t ld,
                                                              const int32_t* __restrict__ y, int n,
                                                              const float* __restrict__ W, int C,
                                                              double* __restrict__ part) {
  __shared__ float zt[EV_WAVES * 16 * (CT * 16 + 1)];
  double ce = 0.0, cor = 0.0;
  eval_group16<EV_WAVES, CT>(phi, ld, y, n, W, C, (int)blockIdx.x * EV_ROWS, zt, ce, cor);
  if ((threadIdx.x >> 6) == 0) {
    ce = wave_sum(ce);
    cor = wave_sum(cor);
    if ((threadIdx.x & 63) == 0) {
      part[2 * blockIdx.x] = ce;
      part[2 * blockIdx.x + 1] = cor;
    }
  }
}

__global__ __launch_bounds__(256) void eval_finalize(const double* __restrict__ part, int nb, int n,
                                                    double* __restrict__ out) {
  __shared__ double s[2][256];
  eval_finalize_block(part, nb, n, out, s);
}

int eval_finalize_launch(const double* part, int nb, int n, double* out, hipStream_t st) {
  hipLaunchKernelGGL(eval_finalize, dim3(1), dim3(256), 0, st, part, nb, n, out);
  FS_LAUNCH_CHECK();
  return FS_OK;
}

}  // namespace fs

using namespace fs;

extern "C" int64_t fs_eval_ws_doubles(int n) { return 2 * (int64_t)((n + EV_ROWS - 1) / EV_ROWS) + 2; }

extern "C" int fs_eval(const float* d_phi, int64_t ld, const int32_t* d_labels, int n, const float* d_W, int C,
                       double* d_out, double* d_ws, void* stream) {
  FS_REQUIRE(n >= 1, "n must be >= 1");
  FS_REQUIRE(C >= 1 && C <= 32, "num_classes must be in [1, 32]");
  FS_REQUIRE(ld >= 64 && ld % 64 == 0, "ld must be a positive multiple of 64");
  FS_REQUIRE(d_phi && d_labels && d_W && d_out && d_ws, "null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nb = (n + EV_ROWS - 1) / EV_ROWS;
  if (C <= 16)
    hipLaunchKernelGGL((eval_kernel<1>), dim3(nb), dim3(EV_WAVES * 64), 0, st, d_phi, ld, d_labels, n, d_W, C, d_ws);
  else
    hipLaunchKernelGGL((eval_kernel<2>), dim3(nb), dim3(EV_WAVES * 64), 0, st, d_phi, ld, d_labels, n, d_W, C, d_ws);
  hipLaunchKernelGGL(eval_finalize, dim3(1), dim3(256), 0, st, d_ws, nb, n, d_out);
  FS_LAUNCH_CHECK();
  return FS_OK;
}
