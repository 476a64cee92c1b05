// fs_local_train -- per-client local SGD for the whole round, fused in one launch.
//
// Replaces train_loop (/root/reference/functions/tools.py:177-215) as called by
// FedAvg / FedProx / FedAMW (tools.py:340-343, 367-370, 430-433).
//
// One 256-thread workgroup (4 waves, one per SIMD) owns one client and runs all of
// its E * ceil(n_j / B) dependent SGD steps without leaving the kernel.  Per step:
//   forward   z = X_b W^T        v_mfma_f32_16x16x4_f32, M = batch rows (16 per tile),
//                                N = classes (16 per tile), K = D split over the 4 waves;
//                                X rows gathered straight from HBM by the shuffled index.
//   softmax   g = (softmax(z) - onehot) / |b|,  CE mean           (wave 0, one row per lane)
//   backward  grad^T = X_b^T g   v_mfma_f32_16x16x4_f32, M = D (16 per tile), N = classes,
//                                K = batch rows; X_b re-read (L2-resident by now).
//   update    W -= lr * (grad + mu (W - W_a)/||W - W_a|| + lam W/||W||)
//             fused on the MFMA output fragments; the two norms for the next step are
//             reduced in the same pass.
// Lane <-> element ownership: the lane that produces grad[c][d] in the backward is
// the lane that reads W[c][d] as the forward's B operand, so W never crosses lanes
// and chained clients (reference semantics) need no inter-lane hand-off.
#include "common.h"

namespace fs {

constexpr int LT_WAVES = 4;
constexpr int LT_THREADS = LT_WAVES * kWave;

struct LTParams {
  const float* phi;
  int64_t ld;
  const int64_t* row_off;
  const int32_t* labels;
  const int32_t* perms;
  const int32_t* order;
  int N, C, B, E;
  float lr, mu, lam;
  int prox, reg, chained;
  const float* W_start;
  float* W_out;
  double* loss;
};

template <int RT, int CT>
struct LTShared {
  int rows[2][RT * 16];
  int ylab[2][RT * 16];
  float zpart[LT_WAVES][RT * 16][CT * 16 + 1];
  float g[RT * 16][CT * 16];
  float red[2][LT_WAVES][2];
  float pro[LT_WAVES];
};

template <int RT, int CT>
__global__ __launch_bounds__(LT_THREADS) void local_train_kernel(LTParams P) {
  __shared__ LTShared<RT, CT> sh;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int l16 = lane & 15;
  const int lg = lane >> 4;
  const int64_t ld = P.ld;
  const int NT = (int)(ld >> 6);
  const int C = P.C;
  const int B = P.B;
  const int E = P.E;
  const int nclients = P.chained ? P.N : 1;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  int it = 0;  // global step counter (parity of the double-buffered LDS slots)

  for (int k = 0; k < nclients; ++k) {
    const int j = P.chained ? k : (P.order ? P.order[blockIdx.x] : (int)blockIdx.x);
    const int64_t row0 = P.row_off[j];
    const int n = (int)(P.row_off[j + 1] - row0);
    const float* start = (P.chained && j > 0) ? P.W_out + (int64_t)(j - 1) * C * ld : P.W_start;
    const float* anchor = start;  // global_model = deepcopy(model)  (tools.py:180)
    float* Wj = P.W_out + (int64_t)j * C * ld;
    const int nb = (n + B - 1) / B;
    const int steps = E * nb;

    if (steps == 0) {
      for (int T = w; T < NT; T += LT_WAVES)
        for (int ct = 0; ct < CT; ++ct) {
          const int c = ct * 16 + l16;
          if (c < C)
            for (int q = 0; q < 4; ++q) {
              const int64_t off = c * ld + 64 * T + 16 * lg + 4 * q;
              st4(Wj + off, ld4(start + off));
            }
        }
      if (tid == 0) P.loss[j] = 0.0;
      __syncthreads();
      continue;
    }

    // ||W_start||^2 for the ridge term of the first step (the prox norm starts at 0).
    float wn2 = 0.f, pn2 = 0.f;
    if (P.reg) {
      float acc = 0.f;
      for (int T = w; T < NT; T += LT_WAVES)
        for (int ct = 0; ct < CT; ++ct) {
          const int c = ct * 16 + l16;
          if (c < C)
            for (int q = 0; q < 4; ++q) {
              const float4 v = ld4(start + c * ld + 64 * T + 16 * lg + 4 * q);
              acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
            }
        }
      acc = wave_sum(acc);
      if (lane == 0) sh.pro[w] = acc;
      __syncthreads();
      wn2 = sh.pro[0] + sh.pro[1] + sh.pro[2] + sh.pro[3];
    }

    const float* src = start;
    double lsum = 0.0;
    for (int e = 0; e < E; ++e) {
      for (int s = 0; s < nb; ++s, ++it) {
        const int par = it & 1;
        const int b0 = s * B;
        const int bc = min(B, n - b0);
        if (tid < bc) {
          const int li = P.perms[(int64_t)E * row0 + (int64_t)e * n + b0 + tid];
          sh.rows[par][tid] = (int)(row0 + li);
          sh.ylab[par][tid] = P.labels[row0 + li];
        }
        __syncthreads();  // B1: batch indices visible; previous step's norm partials visible
        if (s > 0 || e > 0) {
          pn2 = sh.red[par ^ 1][0][0] + sh.red[par ^ 1][1][0] + sh.red[par ^ 1][2][0] + sh.red[par ^ 1][3][0];
          wn2 = sh.red[par ^ 1][0][1] + sh.red[par ^ 1][1][1] + sh.red[par ^ 1][2][1] + sh.red[par ^ 1][3][1];
        }

        // ---------------- forward: z = X_b W^T ----------------
        const float* xr[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const int r = rt * 16 + l16;
          xr[rt] = r < bc ? P.phi + (int64_t)sh.rows[par][r] * ld : nullptr;
        }
        floatx4 acc[RT][CT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = floatx4{0.f, 0.f, 0.f, 0.f};

        for (int T = w; T < NT; T += LT_WAVES) {
          const int64_t dof = 64 * T + 16 * lg;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float4 wv[CT], xv[RT];
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
              const int c = ct * 16 + l16;
              wv[ct] = c < C ? ld4(src + c * ld + dof + 4 * q) : zero4;
            }
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) xv[rt] = xr[rt] ? ld4(xr[rt] + dof + 4 * q) : zero4;
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4)
#pragma unroll
              for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int ct = 0; ct < CT; ++ct)
                  acc[rt][ct] = mfma4(comp(xv[rt], e4), comp(wv[ct], e4), acc[rt][ct]);
          }
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int i = 0; i < 4; ++i) sh.zpart[w][rt * 16 + 4 * lg + i][ct * 16 + l16] = acc[rt][ct][i];
        __syncthreads();  // B2: partial logits from all waves

        // ---------------- softmax / CE (wave 0, row = lane) ----------------
        if (w == 0) {
          float ce = 0.f;
          if (lane < RT * 16) {
            const int r = lane;
            if (r < bc) {
              const int y = sh.ylab[par][r];
              float m = -INFINITY;
              for (int c = 0; c < C; ++c) {
                const float z = ((sh.zpart[0][r][c] + sh.zpart[1][r][c]) + sh.zpart[2][r][c]) + sh.zpart[3][r][c];
                sh.zpart[0][r][c] = z;
                m = fmaxf(m, z);
              }
              float se = 0.f;
              for (int c = 0; c < C; ++c) se += expf(sh.zpart[0][r][c] - m);
              const float lse = logf(se);
              const float invb = 1.0f / (float)bc;
              for (int c = 0; c < C; ++c) {
                const float lp = sh.zpart[0][r][c] - m - lse;
                sh.g[r][c] = (c == y ? -invb : 0.f) + expf(lp) * invb;
                if (c == y) ce = -lp;
              }
              for (int c = C; c < CT * 16; ++c) sh.g[r][c] = 0.f;
            } else {
              for (int c = 0; c < CT * 16; ++c) sh.g[r][c] = 0.f;
            }
          }
          ce = wave_sum(ce);
          if (lane == 0 && e == E - 1) {
            float loss = ce / (float)bc;                       // CrossEntropyLoss, mean
            if (P.prox) loss = loss + P.mu * sqrtf(pn2);       // + mu * ||W - W_a||_F  (tools.py:197, 203-205)
            if (P.reg) loss = loss + P.lam * sqrtf(wn2);       // + lambda * ||W||_F    (tools.py:201, 203, 207)
            lsum += (double)loss * (double)bc;                 // Meter.update(loss.item(), |b|)
          }
        }
        __syncthreads();  // B3: g visible

        // ---------------- backward + fused SGD/prox/ridge update ----------------
        float gB[4 * RT][CT];
        const float* xk[4 * RT];
#pragma unroll
        for (int kk = 0; kk < 4 * RT; ++kk) {
          const int r = 4 * kk + lg;
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) gB[kk][ct] = sh.g[r][ct * 16 + l16];
          xk[kk] = r < bc ? P.phi + (int64_t)sh.rows[par][r] * ld : nullptr;
        }
        const float sp = (P.prox && pn2 > 0.f) ? P.mu / sqrtf(pn2) : 0.f;
        const float sr = (P.reg && wn2 > 0.f) ? P.lam / sqrtf(wn2) : 0.f;
        const float lr = P.lr;
        float npn = 0.f, nwn = 0.f;
        for (int T = w; T < NT; T += LT_WAVES) {
          floatx4 ga[CT][4];
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) ga[ct][e4] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < 4 * RT; ++kk) {
            const float4 xv = xk[kk] ? ld4(xk[kk] + 64 * T + 4 * l16) : zero4;
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4)
#pragma unroll
              for (int ct = 0; ct < CT; ++ct) ga[ct][e4] = mfma4(comp(xv, e4), gB[kk][ct], ga[ct][e4]);
          }
          // ga[ct][e][q] = grad[c = ct*16 + l16][d = 64T + 16 lg + 4q + e]
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
            const int c = ct * 16 + l16;
            if (c < C) {
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const int64_t off = c * ld + 64 * T + 16 * lg + 4 * q;
                const float4 wv = ld4(src + off);
                const float4 av = P.prox ? ld4(anchor + off) : zero4;
                float o[4];
#pragma unroll
                for (int e4 = 0; e4 < 4; ++e4) {
                  const float wc = comp(wv, e4);
                  const float ac = comp(av, e4);
                  float gr = ga[ct][e4][q];
                  if (P.prox) gr = gr + (wc - ac) * sp;
                  if (P.reg) gr = gr + wc * sr;
                  o[e4] = wc - lr * gr;
                  const float dp = o[e4] - ac;
                  npn += dp * dp;
                  nwn += o[e4] * o[e4];
                }
                st4(Wj + off, make_float4(o[0], o[1], o[2], o[3]));
              }
            }
          }
        }
        npn = wave_sum(npn);
        nwn = wave_sum(nwn);
        if (lane == 0) {
          sh.red[par][w][0] = npn;
          sh.red[par][w][1] = nwn;
        }
        src = Wj;
      }
    }
    if (tid == 0) P.loss[j] = lsum / (double)n;
    __syncthreads();
  }
}

template <int RT, int CT>
static int launch_lt(const LTParams& P, int grid, hipStream_t st) {
  hipLaunchKernelGGL((local_train_kernel<RT, CT>), dim3(grid), dim3(LT_THREADS), 0, st, P);
  return 0;
}

}  // namespace fs

using namespace fs;

extern "C" int fs_local_train(const float* d_phi, int64_t ld, const int64_t* d_row_off, const int32_t* d_labels,
                              const int32_t* d_perms, const int32_t* d_order, int N, int C, int B, int E,
                              float lr, float mu, int prox, float lam, int reg, int chained,
                              const float* d_W_start, float* d_W_out, double* d_loss, void* stream) {
  FS_REQUIRE(N >= 1, "N must be >= 1");
  FS_REQUIRE(C >= 1 && C <= 32, "num_classes must be in [1, 32]");
  FS_REQUIRE(B >= 1 && B <= 64, "batch_size must be in [1, 64]");
  FS_REQUIRE(E >= 0, "epoch must be >= 0");
  FS_REQUIRE(ld >= 64 && ld % 64 == 0, "ld must be a positive multiple of 64");
  FS_REQUIRE(d_phi && d_row_off && d_labels && d_perms && d_W_start && d_W_out && d_loss, "null pointer");
  LTParams P{d_phi, ld, d_row_off, d_labels, d_perms, d_order, N, C, B, E, lr, mu, lam,
             prox ? 1 : 0, reg ? 1 : 0, chained ? 1 : 0, d_W_start, d_W_out, d_loss};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int grid = chained ? 1 : N;
  const int RT = B <= 16 ? 1 : (B <= 32 ? 2 : 4);
  const int CT = C <= 16 ? 1 : 2;
  if (RT == 1 && CT == 1) launch_lt<1, 1>(P, grid, st);
  else if (RT == 2 && CT == 1) launch_lt<2, 1>(P, grid, st);
  else if (RT == 4 && CT == 1) launch_lt<4, 1>(P, grid, st);
  else if (RT == 1 && CT == 2) launch_lt<1, 2>(P, grid, st);
  else if (RT == 2 && CT == 2) launch_lt<2, 2>(P, grid, st);
  else launch_lt<4, 2>(P, grid, st);
  FS_LAUNCH_CHECK();
  return FS_OK;
}
