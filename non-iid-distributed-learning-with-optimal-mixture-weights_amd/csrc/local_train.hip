// fs_local_train -- per-client local SGD for the whole round, fused in one launch.
//
// Replaces train_loop (/root/reference/functions/tools.py:177-215) as called by
// FedAvg / FedProx / FedAMW (tools.py:340-343, 367-370, 430-433).
//
// One 512-thread workgroup (8 waves, two per SIMD, up to 256 VGPRs each) owns one client and runs all of
// its E * ceil(n_j / B) dependent SGD steps without leaving the kernel.  The feature
// dimension is cut into 64-column tiles T, dealt round-robin to the 8 waves.  Per step:
//   forward   z = X_b W^T        v_mfma_f32_16x16x4_f32, M = batch rows (16 per tile),
//                                N = classes (16 per tile), K = the wave's columns; the
//                                batch rows are gathered straight from HBM by the shuffled
//                                index (16 B per lane, 64 contiguous bytes per row per
//                                instruction), all of a wave's loads issued before its MFMAs.
//   reduce    the 8 waves' partial logits are summed through LDS, one logit per thread.
//   softmax   g = (softmax(z) - onehot) / |b|,  CE mean           (wave 0, one row per lane)
//   backward  grad^T = X_b^T g   v_mfma_f32_16x16x4_f32, M = 16 columns, N = classes,
//                                K = batch rows; X_b re-read (L2-resident by now).
//   update    W -= lr * (grad + mu (W - W_a)/||W - W_a|| + lam W/||W||)
//             fused on the MFMA output fragments; the two squared norms for the next
//             step are reduced in the same pass.
// Lane <-> element ownership: the lane that produces grad[c][d] in the backward is the
// lane that reads W[c][d] as the forward's B operand, so W never crosses lanes and
// chained clients (reference semantics) need no inter-lane hand-off.
#include "common.h"

namespace fs {

constexpr int LT_WAVES = 8;
constexpr int LT_THREADS = LT_WAVES * kWave;

constexpr int LT_CHUNK = 2048;   // batch rows whose (row, label) are staged in LDS at once

template <int RT, int CT>
struct LTShared {
  int erow[LT_CHUNK];                 // global feature row of each staged batch position
  int elab[LT_CHUNK];                 // its label
  float zpart[LT_WAVES][RT * 16][CT * 16];
  float g[RT * 16][CT * 16];
  float red[2][LT_WAVES][2];
  float cep[2][LT_WAVES];
  float pro[LT_WAVES];
  float pad_[2];                      // keep sizeof a multiple of 16 B: the dynamic W image follows
};

__device__ __forceinline__ float4 mask4(float4 v, bool keep) {
  return keep ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}

template <int W>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int off = W / 2; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int off = W / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// WLDS: the client's weights live in LDS for the whole local training (row stride ld + 4
// floats, 16 B of skew per class row), so the forward's B operand and the update never touch
// the L1/L2 path; otherwise they stay in the (L2-resident) output buffer.
template <int RT, int CT, bool WLDS>
__global__ __launch_bounds__(LT_THREADS) void local_train_kernel(LTParams P) {
  __shared__ LTShared<RT, CT> sh;
  extern __shared__ __attribute__((aligned(16))) float sW[];   // [C][ld + 4] when WLDS
  constexpr int NC = CT * 16;           // padded classes
  constexpr int NZ = RT * 16 * NC;      // padded logits per step
  constexpr int UF = (RT * CT >= 4) ? 1 : 2;   // forward tiles per batch of loads (register budget)
  constexpr int UB = (RT >= 4) ? 1 : 2;        // backward tiles per batch of loads
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
  const int CH = (LT_CHUNK / B) * B;
  const int nclients = P.chained ? P.N : 1;
  const int64_t LDW = ld + 4;
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
      for (int i = 0; i < LT_WAVES; ++i) wn2 += sh.pro[i];
    }

    const float* src = start;
    if (WLDS) {
      // lane-owned copy: every lane later reads and writes exactly these elements
      for (int T = w; T < NT; T += LT_WAVES)
        for (int ct = 0; ct < CT; ++ct) {
          const int c = ct * 16 + l16;
          if (c < C)
            for (int q = 0; q < 4; ++q) {
              const int64_t off = 64 * T + 16 * lg + 4 * q;
              st4(sW + c * LDW + off, ld4(start + c * ld + off));
            }
        }
    }
    double lsum = 0.0;
    for (int e = 0; e < E; ++e) {
      for (int s = 0; s < nb; ++s, ++it) {
        const int par = it & 1;
        const int b0 = s * B;
        const int bc = min(B, n - b0);
        const int cb = b0 % CH;           // position of this batch inside the staged chunk
        if (cb == 0) {
          // stage the next CH shuffled rows of this epoch: (global row, label) into LDS
          __syncthreads();                // every wave is done with the previous chunk
          const int cn = min(CH, n - b0);
          const int32_t* pp = P.perms + (int64_t)E * row0 + (int64_t)e * n + b0;
          for (int i = tid; i < cn; i += LT_THREADS) {
            const int li = pp[i];
            sh.erow[i] = (int)(row0 + li);
            sh.elab[i] = P.labels[row0 + li];
          }
          __syncthreads();
        }

        // ---------------- forward: z = X_b W^T ----------------
        // invalid rows (>= bc) read a valid row and are zeroed after the load, so every
        // load is unconditional and the compiler can keep them all in flight.
        const float* xr[RT];
        bool xok[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const int r = rt * 16 + l16;
          xok[rt] = r < bc;
          xr[rt] = P.phi + (int64_t)sh.erow[cb + (xok[rt] ? r : 0)] * ld;
        }
        floatx4 acc[RT][CT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = floatx4{0.f, 0.f, 0.f, 0.f};

        // UF tiles per iteration: all UF x 4 x (RT + CT) 16-byte loads are issued before the MFMAs
        for (int T0 = w; T0 < NT; T0 += UF * LT_WAVES) {
          const bool ok1 = UF > 1 && T0 + LT_WAVES < NT;
          const int T1 = ok1 ? T0 + LT_WAVES : T0;
          float4 xv[UF][4][RT], wv[UF][4][CT];
#pragma unroll
          for (int h = 0; h < UF; ++h) {
            const int64_t dof = 64 * (h ? T1 : T0) + 16 * lg;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
              for (int rt = 0; rt < RT; ++rt) xv[h][q][rt] = ld4(xr[rt] + dof + 4 * q);
#pragma unroll
              for (int ct = 0; ct < CT; ++ct) {
                const int c = min(ct * 16 + l16, C - 1);
                wv[h][q][ct] = WLDS ? ld4(sW + c * LDW + dof + 4 * q) : ld4(src + c * ld + dof + 4 * q);
              }
            }
          }
#pragma unroll
          for (int h = 0; h < UF; ++h) {
            if (h == 1 && !ok1) break;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
              for (int rt = 0; rt < RT; ++rt) xv[h][q][rt] = mask4(xv[h][q][rt], xok[rt]);
#pragma unroll
              for (int ct = 0; ct < CT; ++ct) wv[h][q][ct] = mask4(wv[h][q][ct], ct * 16 + l16 < C);
#pragma unroll
              for (int e4 = 0; e4 < 4; ++e4)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                  for (int ct = 0; ct < CT; ++ct)
                    acc[rt][ct] = mfma4(comp(xv[h][q][rt], e4), comp(wv[h][q][ct], e4), acc[rt][ct]);
            }
          }
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int i = 0; i < 4; ++i) sh.zpart[w][rt * 16 + 4 * lg + i][ct * 16 + l16] = acc[rt][ct][i];
        __syncthreads();  // B1: partial logits of all waves; previous step's norm partials

        if (s > 0 || e > 0) {
          pn2 = 0.f;
          wn2 = 0.f;
#pragma unroll
          for (int i = 0; i < LT_WAVES; ++i) {
            pn2 += sh.red[par ^ 1][i][0];
            wn2 += sh.red[par ^ 1][i][1];
          }
        }

        // ------- logits (fixed-order sum of the wave partials) + softmax / CE, one logit per thread -------
        {
          const float invb = 1.0f / (float)bc;
          float cep = 0.f;
          for (int idx = tid; idx < NZ; idx += LT_THREADS) {   // NC lanes of one wave hold one row
            const int r = idx / NC, c = idx % NC;
            float z = 0.f;
#pragma unroll
            for (int i = 0; i < LT_WAVES; ++i) z += sh.zpart[i][r][c];
            const bool valid = r < bc && c < C;
            const float m = group_max<NC>(valid ? z : -INFINITY);
            const float se = group_sum<NC>(valid ? expf(z - m) : 0.f);
            float gv = 0.f;
            if (valid) {
              const float lp = z - m - logf(se);               // log_softmax
              const bool isy = c == sh.elab[cb + r];
              gv = (isy ? -invb : 0.f) + expf(lp) * invb;      // d CE_mean / d z
              if (isy) cep -= lp;
            }
            sh.g[r][c] = gv;
          }
          cep = wave_sum(cep);
          if (lane == 0) sh.cep[par][w] = cep;
        }
        __syncthreads();  // B2: g and the CE partials visible

        if (tid == 0 && e == E - 1) {
          float ce = 0.f;
          for (int i = 0; i < LT_WAVES; ++i) ce += sh.cep[par][i];
          float loss = ce / (float)bc;                       // CrossEntropyLoss, mean
          if (P.prox) loss = loss + P.mu * sqrtf(pn2);       // + mu * ||W - W_a||_F  (tools.py:197, 203-205)
          if (P.reg) loss = loss + P.lam * sqrtf(wn2);       // + lambda * ||W||_F    (tools.py:201, 203, 207)
          lsum += (double)loss * (double)bc;                 // Meter.update(loss.item(), |b|)
        }

        // ---------------- backward + fused SGD/prox/ridge update ----------------
        float gB[4 * RT][CT];
        const float* xk[4 * RT];
        bool kok[4 * RT];
#pragma unroll
        for (int kk = 0; kk < 4 * RT; ++kk) {
          const int r = 4 * kk + lg;
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) gB[kk][ct] = sh.g[r][ct * 16 + l16];
          kok[kk] = r < bc;
          xk[kk] = P.phi + (int64_t)sh.erow[cb + (kok[kk] ? r : 0)] * ld + 4 * l16;
        }
        const float sp = (P.prox && pn2 > 0.f) ? P.mu / sqrtf(pn2) : 0.f;
        const float sr = (P.reg && wn2 > 0.f) ? P.lam / sqrtf(wn2) : 0.f;
        const float lr = P.lr;
        float npn = 0.f, nwn = 0.f;
        for (int T0 = w; T0 < NT; T0 += UB * LT_WAVES) {
          const bool ok1 = UB > 1 && T0 + LT_WAVES < NT;
          const int T1 = ok1 ? T0 + LT_WAVES : T0;
          float4 xv[UB][4 * RT];
#pragma unroll
          for (int h = 0; h < UB; ++h)
#pragma unroll
            for (int kk = 0; kk < 4 * RT; ++kk) xv[h][kk] = ld4(xk[kk] + 64 * (h ? T1 : T0));
#pragma unroll
          for (int h = 0; h < UB; ++h) {
            if (h == 1 && !ok1) break;
            const int T = h ? T1 : T0;
            floatx4 ga[CT][4];
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
              for (int e4 = 0; e4 < 4; ++e4) ga[ct][e4] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < 4 * RT; ++kk) {
              const float4 x = mask4(xv[h][kk], kok[kk]);
#pragma unroll
              for (int e4 = 0; e4 < 4; ++e4)
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) ga[ct][e4] = mfma4(comp(x, e4), gB[kk][ct], ga[ct][e4]);
            }
            // ga[ct][e][q] = grad[c = ct*16 + l16][d = 64T + 16 lg + 4q + e]
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
              const int c = ct * 16 + l16;
              if (c < C) {
                float4 wv[4], av[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  const int64_t off = c * ld + 64 * T + 16 * lg + 4 * q;
                  wv[q] = WLDS ? ld4(sW + (off - c * ld) + c * LDW) : ld4(src + off);
                  av[q] = P.prox ? ld4(anchor + off) : zero4;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  const int64_t off = c * ld + 64 * T + 16 * lg + 4 * q;
                  float o[4];
#pragma unroll
                  for (int e4 = 0; e4 < 4; ++e4) {
                    const float wc = comp(wv[q], e4);
                    const float ac = comp(av[q], e4);
                    float gr = ga[ct][e4][q];
                    if (P.prox) gr = gr + (wc - ac) * sp;
                    if (P.reg) gr = gr + wc * sr;
                    o[e4] = wc - lr * gr;
                    const float dp = o[e4] - ac;
                    npn += dp * dp;
                    nwn += o[e4] * o[e4];
                  }
                  if (WLDS) st4(sW + (off - c * ld) + c * LDW, make_float4(o[0], o[1], o[2], o[3]));
                  else st4(Wj + off, make_float4(o[0], o[1], o[2], o[3]));
                }
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
    if (WLDS) {
      for (int T = w; T < NT; T += LT_WAVES)
        for (int ct = 0; ct < CT; ++ct) {
          const int c = ct * 16 + l16;
          if (c < C)
            for (int q = 0; q < 4; ++q) {
              const int64_t off = 64 * T + 16 * lg + 4 * q;
              st4(Wj + c * ld + off, ld4(sW + c * LDW + off));
            }
        }
    }
    if (tid == 0) P.loss[j] = lsum / (double)n;
    __syncthreads();
  }
}

template <int RT, int CT>
static int launch_lt(const LTParams& P, int grid, hipStream_t st) {
  const size_t wbytes = sizeof(float) * (size_t)P.C * (size_t)(P.ld + 4);
  const size_t budget = 160 * 1024 - sizeof(LTShared<RT, CT>);
  if (wbytes <= budget) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&local_train_kernel<RT, CT, true>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)wbytes);
    if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_local_train: ") + hipGetErrorString(e));
    hipLaunchKernelGGL((local_train_kernel<RT, CT, true>), dim3(grid), dim3(LT_THREADS), wbytes, st, P);
  } else {
    hipLaunchKernelGGL((local_train_kernel<RT, CT, false>), dim3(grid), dim3(LT_THREADS), 0, st, P);
  }
  return FS_OK;
}

}  // namespace fs

using namespace fs;

static thread_local int t_last_lt = 0;
void fs::set_last_lt_kernel(int k) { t_last_lt = k; }
extern "C" int fs_local_train_last_kernel(void) { return t_last_lt; }

extern "C" int fs_local_train(const float* d_phi, int64_t ld, const int64_t* d_row_off, const int32_t* d_labels,
                              const int32_t* d_perms, const int32_t* d_order, int N, int C, int B, int E,
                              float lr, float mu, int prox, float lam, int reg, int chained,
                              const float* d_W_start, float* d_W_out, double* d_loss, int G, void* d_ws,
                              int64_t ws_bytes, void* stream) {
  return fs::local_train(d_phi, ld, d_row_off, d_labels, d_perms, d_order, N, C, B, E, lr, mu, prox, lam, reg, chained,
                         d_W_start, d_W_out, d_loss, G, d_ws, ws_bytes, reinterpret_cast<hipStream_t>(stream), 0);
}

int fs::local_train(const float* d_phi, int64_t ld, const int64_t* d_row_off, const int32_t* d_labels,
                    const int32_t* d_perms, const int32_t* d_order, int N, int C, int B, int E, float lr, float mu,
                    int prox, float lam, int reg, int chained, const float* d_W_start, float* d_W_out,
                    double* d_loss, int G, void* d_ws, int64_t ws_bytes, hipStream_t st,
                    int64_t max_client_steps, const FuseEval* fuse) {
  FS_REQUIRE(N >= 1, "N must be >= 1");
  FS_REQUIRE(C >= 1 && C <= 32, "num_classes must be in [1, 32]");
  FS_REQUIRE(B >= 1 && B <= 64, "batch_size must be in [1, 64]");
  FS_REQUIRE(E >= 0, "epoch must be >= 0");
  FS_REQUIRE(ld >= 64 && ld % 64 == 0, "ld must be a positive multiple of 64");
  FS_REQUIRE(d_phi && d_row_off && d_labels && d_perms && d_W_start && d_W_out && d_loss, "null pointer");
  LTParams P{d_phi, ld, d_row_off, d_labels, d_perms, d_order, N, C, B, E, lr, mu, lam,
             prox ? 1 : 0, reg ? 1 : 0, chained ? 1 : 0, d_W_start, d_W_out, d_loss, max_client_steps};
  if (fuse && G > 1 && !chained) {
    P.fuse_phi = fuse->phi;
    P.fuse_y = fuse->y;
    P.fuse_n = fuse->n;
    P.fuse_E = fuse->E;
    P.fuse_part = fuse->part;
  }
  if (G > 1) {
    set_last_lt_kernel((G & FS_G_PIPE) ? FS_LT_PIPE : (G & FS_G_PAIR) ? FS_LT_PAIR : (G & FS_G_TEAMS) ? FS_LT_TEAMS : FS_LT_SPLIT);
    const int rc = (G & FS_G_PIPE)   ? launch_local_train_pipe(P, G & (FS_G_PAIR - 1), d_ws, ws_bytes, st)
                   : (G & FS_G_PAIR) ? launch_local_train_pair(P, G & (FS_G_PAIR - 1), d_ws, ws_bytes, st)
                                     : launch_local_train_split(P, G, d_ws, ws_bytes, st);
    if (rc != FS_OK) return rc;
    FS_LAUNCH_CHECK();
    return FS_OK;
  }
  set_last_lt_kernel(FS_LT_SINGLE);
  const int grid = chained ? 1 : N;
  const int RT = B <= 16 ? 1 : (B <= 32 ? 2 : 4);
  const int CT = C <= 16 ? 1 : 2;
  int rc;
  if (RT == 1 && CT == 1) rc = launch_lt<1, 1>(P, grid, st);
  else if (RT == 2 && CT == 1) rc = launch_lt<2, 1>(P, grid, st);
  else if (RT == 4 && CT == 1) rc = launch_lt<4, 1>(P, grid, st);
  else if (RT == 1 && CT == 2) rc = launch_lt<1, 2>(P, grid, st);
  else if (RT == 2 && CT == 2) rc = launch_lt<2, 2>(P, grid, st);
  else rc = launch_lt<4, 2>(P, grid, st);
  if (rc != FS_OK) return rc;
  FS_LAUNCH_CHECK();
  return FS_OK;
}
