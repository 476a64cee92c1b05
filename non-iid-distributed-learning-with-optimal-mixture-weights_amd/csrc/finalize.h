// The test evaluation's finaliser: the fold of the per-workgroup fp64 (loss, correct) partials
// into (loss, accuracy %) by one 256-thread workgroup -- eval.hip's eval_finalize kernel, and the
// last workgroup of the one-launch aggregation that carries it (aggregate.hip).
#pragma once
#include "common.h"

namespace fs {

// the deferred evaluation's finaliser riding on the aggregation launch (aggregate.hip): the nb
// fp64 (loss, correct) partials at part folded into out[0..1] (eval.hip's arithmetic)
struct EvalFinalize {
  const double* part;
  int nb, n;
  double* out;
};
// fs_aggregate with an optional finaliser (nullptr: none); chunks <= 0 with 16 <= N <= 512 is
// one launch (the finaliser as its last workgroup)
int aggregate_launch(const float* d_W_all, int64_t stride, const float* d_p, int N, int64_t len, float* d_W_bar,
                     float* d_ws, int64_t ws_floats, int chunks, const EvalFinalize* fin, hipStream_t st);

__device__ __forceinline__ void eval_finalize_block(const double* __restrict__ part, int nb, int n,
                                                   double* __restrict__ out, double (*s)[256]) {
  double a = 0.0, b = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) { a += part[2 * i]; b += part[2 * i + 1]; }
  s[0][threadIdx.x] = a;
  s[1][threadIdx.x] = b;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      s[0][threadIdx.x] += s[0][threadIdx.x + h];
      s[1][threadIdx.x] += s[1][threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = s[0][0] / (double)n;
    out[1] = 100.0 * s[1][0] / (double)n;
  }
}

}  // namespace fs
