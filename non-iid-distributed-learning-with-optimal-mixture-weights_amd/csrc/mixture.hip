// FedAMW mixture-weight estimation (/root/reference/functions/tools.py:435-453).
//
// fs_mix_z:     Z[v][c*ldN + n] = X_val[v] . W_n[c]: the fp32 MFMA GEMM in mix_z.hip
//               (the reference recomputes this matmul for every 16-row batch of every inner
//               epoch, tools.py:448; W is fixed during the p-solve, so once per round here).
// fs_mix_solve: all `epochs * ceil(n_val/Bv)` dependent p-SGD steps of one round in ONE
//               persistent workgroup (a grid-wide barrier per step would cost more than
//               the step): out = Z_b p, CE, grad_p = Z_b^T g, momentum update.
#include "common.h"
#include "lanes.h"

#include <cstdlib>

namespace fs {

// client stride of a Z row segment: N rounded up to 4 (16-byte aligned class segments)
__host__ __device__ __forceinline__ int mix_ldn(int N) { return (N + 3) & ~3; }

// ----------------------------------------------------------------------------
// p-solve: one workgroup of 1024 threads.  p and the momentum buffer live in LDS.
// ----------------------------------------------------------------------------
constexpr int MS_THREADS = 1024;
constexpr int MS_WAVES = MS_THREADS / 64;
constexpr int MS_MAXB = 64;

__global__ __launch_bounds__(MS_THREADS) void mix_solve_kernel(const float* __restrict__ Z,
                                                              const int32_t* __restrict__ y,
                                                              const int32_t* __restrict__ perms, int N, int C,
                                                              int nv, int epochs, int Bv, float lr, float mom,
                                                              float* __restrict__ p, float* __restrict__ buf,
                                                              int* __restrict__ first_flag) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int ldN = mix_ldn(N);
  float* ps = smem;                       // [N]
  float* bs = ps + N;                     // [N]
  float* outs = bs + N;                   // [MS_MAXB][C]
  float* gs = outs + MS_MAXB * C;         // [MS_MAXB][C]
  int* vid = reinterpret_cast<int*>(gs + MS_MAXB * C);  // [MS_MAXB]
  int* vy = vid + MS_MAXB;                              // [MS_MAXB]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int CN = C * ldN;
  for (int n = tid; n < N; n += MS_THREADS) { ps[n] = p[n]; bs[n] = buf[n]; }
  int first = *first_flag;
  const int nbat = (nv + Bv - 1) / Bv;
  for (int ep = 0; ep < epochs; ++ep) {
    for (int s = 0; s < nbat; ++s) {
      const int b0 = s * Bv;
      const int bc = min(Bv, nv - b0);
      if (tid < bc) {
        const int v = perms[(int64_t)ep * nv + b0 + tid];
        vid[tid] = v;
        vy[tid] = y[v];
      }
      __syncthreads();
      // out[b][c] = sum_n p_n Z[v_b][c*N + n]
      for (int q = w; q < bc * C; q += MS_WAVES) {
        const int b = q / C, c = q - b * C;
        const float* zr = Z + (int64_t)vid[b] * CN + (int64_t)c * ldN;
        float a = 0.f;
        for (int n = lane; n < N; n += 64) a += ps[n] * zr[n];
        a = wave_sum(a);
        if (lane == 0) outs[b * C + c] = a;
      }
      __syncthreads();
      // softmax / CE gradient (CrossEntropyLoss mean over the batch)
      if (w == 0 && lane < bc) {
        const int b = lane;
        const int yy = vy[b];
        float m = -INFINITY;
        for (int c = 0; c < C; ++c) m = fmaxf(m, outs[b * C + c]);
        float se = 0.f;
        for (int c = 0; c < C; ++c) se += expf(outs[b * C + c] - m);
        const float lse = logf(se);
        const float invb = 1.0f / (float)bc;
        for (int c = 0; c < C; ++c) {
          const float lp = outs[b * C + c] - m - lse;
          gs[b * C + c] = (c == yy ? -invb : 0.f) + expf(lp) * invb;
        }
      }
      __syncthreads();
      // grad_p[n] = sum_{b,c} g[b][c] Z[v_b][c*N+n];  SGD momentum (torch.optim.SGD semantics)
      for (int n = tid; n < N; n += MS_THREADS) {
        float gp = 0.f;
        for (int b = 0; b < bc; ++b) {
          const float* zr = Z + (int64_t)vid[b] * CN + n;
          for (int c = 0; c < C; ++c) gp += gs[b * C + c] * zr[(int64_t)c * ldN];
        }
        {
#pragma clang fp contract(off)
          const float nb = first ? gp : mom * bs[n] + gp;   // buf.mul_(0.9).add_(grad), two roundings
          bs[n] = nb;
          ps[n] = ps[n] + (-lr) * nb;                         // p.add_(buf, alpha=-lr)
        }
      }
      first = 0;
      __syncthreads();
    }
  }
  for (int n = tid; n < N; n += MS_THREADS) { p[n] = ps[n]; buf[n] = bs[n]; }
  if (tid == 0 && epochs > 0 && nbat > 0) *first_flag = 0;
}

// ----------------------------------------------------------------------------
// p-solve, LDS-staged form (used whenever two batches of Z rows fit in LDS):
// wave w owns batch rows b = w, w+16, ...; its lanes split the clients n.  Per row the
// wave reduces the C logits out[b][c] = sum_n p_n Z[v_b][c][n] with xor butterflies (all
// lanes end up holding them), computes the softmax-CE gradient g[b][:] redundantly in
// every lane, and accumulates sum_c g[b][c] Z[v_b][c][n] for its own n; the 16 waves'
// partial gradients are summed in wave order, then the momentum step.  The next batch's
// rows are loaded into registers at the top of the step and written to the other LDS
// buffer at its end, so Z streams from L2/MALL behind the arithmetic.  Two barriers per
// step; a step costs ~1 us instead of three dependent global round trips.
// ----------------------------------------------------------------------------
constexpr int MS2_PER_THREAD = 4;     // float4 of staged rows per thread (one batch <= 64 KB)
constexpr int MS2_NK = 4;             // clients per lane (N <= 256 on this path)

template <int CMAX>
__global__ __launch_bounds__(MS_THREADS) void mix_solve_staged_kernel(const float* __restrict__ Z,
                                                                     const int32_t* __restrict__ y,
                                                                     const int32_t* __restrict__ perms, int N,
                                                                     int C, int nv, int epochs, int Bv, float lr,
                                                                     float mom, float* __restrict__ p,
                                                                     float* __restrict__ buf,
                                                                     int* __restrict__ first_flag) {
  extern __shared__ __attribute__((aligned(16))) float smem2[];
  const int ldN = mix_ldn(N);
  const int CN = C * ldN;
  const int CN4 = CN;                              // row stride in LDS (ldN % 4 == 0: float4 aligned)
  float* zb = smem2;                               // [2][Bv][CN4]
  float* ps = zb + 2 * Bv * CN4;                   // [N]
  float* bs = ps + N;                              // [N]
  float* gpart = bs + N;                           // [MS_WAVES][N]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int n = tid; n < N; n += MS_THREADS) { ps[n] = p[n]; bs[n] = buf[n]; }
  int first = *first_flag;
  const int nbat = (nv + Bv - 1) / Bv;
  const int total = epochs * nbat;
  const int F4 = CN4 / 4;                          // float4 per staged row
  float4 stg[MS2_PER_THREAD];
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // stage batch `st` (global step) rows into registers / LDS slot
  auto batch_row = [&](int st, int b) -> int {
    const int ep = st / nbat, s = st - ep * nbat;
    return perms[(int64_t)ep * nv + s * Bv + b];
  };
  auto batch_size = [&](int st) -> int {
    const int s = st % nbat;
    return min(Bv, nv - s * Bv);
  };
#define MS2_LOAD(ST_)                                                                 \
  {                                                                                   \
    const int bcn_ = batch_size(ST_);                                                 \
    _Pragma("unroll") for (int i = 0; i < MS2_PER_THREAD; ++i) {                      \
      const int idx = tid + MS_THREADS * i;                                           \
      const int b = idx / F4, f = idx - b * F4;                                       \
      stg[i] = zero4;                                                                 \
      if (b < bcn_) {                                                                 \
        const float* zr = Z + (int64_t)batch_row(ST_, b) * CN;                        \
        if (4 * f + 3 < CN) stg[i] = ld4(zr + 4 * f);                                 \
        else {                                                                        \
          float t_[4] = {0.f, 0.f, 0.f, 0.f};                                         \
          for (int k = 0; k < 4; ++k) if (4 * f + k < CN) t_[k] = zr[4 * f + k];      \
          stg[i] = make_float4(t_[0], t_[1], t_[2], t_[3]);                           \
        }                                                                             \
      }                                                                               \
    }                                                                                 \
  }
#define MS2_STORE(SLOT_)                                                              \
  {                                                                                   \
    _Pragma("unroll") for (int i = 0; i < MS2_PER_THREAD; ++i) {                      \
      const int idx = tid + MS_THREADS * i;                                           \
      if (idx < Bv * F4) st4(zb + (int64_t)(SLOT_) * Bv * CN4 + (int64_t)idx * 4, stg[i]); \
    }                                                                                 \
  }
  if (total > 0) {
    MS2_LOAD(0);
    MS2_STORE(0);
  }
  __syncthreads();
  for (int st = 0; st < total; ++st) {
    const int cur = st & 1;
    const int bc = batch_size(st);
    const bool more = st + 1 < total;
    if (more) MS2_LOAD(st + 1);
    // per-lane gradient partials for n = lane + 64 k (k < MS2_NK, compile-time indexed)
    float gacc[MS2_NK];
#pragma unroll
    for (int k = 0; k < MS2_NK; ++k) gacc[k] = 0.f;
    for (int b = w; b < bc; b += MS_WAVES) {
      const float* zr = zb + (int64_t)cur * Bv * CN4 + (int64_t)b * CN4;
      float o[CMAX];
#pragma unroll
      for (int c = 0; c < CMAX; ++c) {
        float a = 0.f;
        if (c < C) {
#pragma unroll
          for (int k = 0; k < MS2_NK; ++k) {
            const int n = lane + 64 * k;
            if (n < N) a += ps[n] * zr[c * ldN + n];
          }
        }
        o[c] = wave_sum(a);                          // every lane holds out[b][c]
      }
      float m = -INFINITY;
#pragma unroll
      for (int c = 0; c < CMAX; ++c) if (c < C) m = fmaxf(m, o[c]);
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < CMAX; ++c) if (c < C) se += expf(o[c] - m);
      const float lse = logf(se);
      const float invb = 1.0f / (float)bc;
      const int yy = y[batch_row(st, b)];
#pragma unroll
      for (int c = 0; c < CMAX; ++c) {
        if (c < C) {
          const float gv = (c == yy ? -invb : 0.f) + expf(o[c] - m - lse) * invb;
#pragma unroll
          for (int k = 0; k < MS2_NK; ++k) {
            const int n = lane + 64 * k;
            if (n < N) gacc[k] += gv * zr[c * ldN + n];
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < MS2_NK; ++k) {
      const int n = lane + 64 * k;
      if (n < N) gpart[w * N + n] = gacc[k];
    }
    if (more) MS2_STORE(cur ^ 1);
    __syncthreads();
    for (int n = tid; n < N; n += MS_THREADS) {
      float gp = 0.f;
      for (int i = 0; i < MS_WAVES; ++i) gp += gpart[i * N + n];
      {
#pragma clang fp contract(off)
        const float nb = first ? gp : mom * bs[n] + gp;   // buf.mul_(0.9).add_(grad)
        bs[n] = nb;
        ps[n] = ps[n] + (-lr) * nb;                       // p.add_(buf, alpha=-lr)
      }
    }
    first = 0;
    __syncthreads();
  }
#undef MS2_LOAD
#undef MS2_STORE
  for (int n = tid; n < N; n += MS_THREADS) { p[n] = ps[n]; buf[n] = bs[n]; }
  if (tid == 0 && total > 0) *first_flag = 0;
}

// ----------------------------------------------------------------------------
// p-solve, register-resident form (Bv <= 16, N <= 64*NK): the latency-optimised path.
// Wave w owns batch row w of every step; lane l owns clients n = NK*l + j (j < NK) in EVERY
// wave, so p and the momentum buffer live in registers (each wave updates its copy
// redundantly, bitwise identically).  A step:
//   logits    lane partials v[c] = sum_j Z[v_b][c][n_j] p[n_j], then a reduce-scatter over
//             the 64 lanes on DPP / permlane swaps (lanes.h): lane l ends with the full
//             out[b][l / (64/CP)]
//   softmax   max / sum over the class groups (xor exchanges); the CE gradient of lane l's
//             class, g = (softmax - onehot) / bc (torch's log_softmax backward)
//   grad_p    g[c] broadcast by readlane; lane partial sum_c g[c] Z[v_b][c][n_j]; wave
//             partials through LDS; after a raw barrier each client's 16 partials are
//             folded ONCE (16/NK threads: NK partials each in wave order, then a fixed lane
//             tree), its owner thread takes the momentum step (torch.optim.SGD, two
//             roundings) and publishes p[n] in LDS; after a second barrier every wave reads
//             its lanes' p back.  (Round 2's form -- every wave folding all 16 x 64NK
//             partials itself, one barrier -- spent ~2,000 of a step's ~5,900 cycles in LDS
//             reads: 128 KB per step at N = 100; r02s2c stamps.)
// Z rows never touch LDS: each step's row segment is ONE dword / dwordx2 / dwordx4 load per
// class per lane into a 3-deep register ring (the loads of step s+3 are issued as soon as
// step s's data is consumed; CL + 2 loads per step keep 3 steps under the 63-deep vmcnt
// window); the batch's row indices and labels are fetched one step earlier still.
// ----------------------------------------------------------------------------
// torch.optim.SGD(momentum) on one element: buf = first ? g : mom*buf + g; p -= lr*buf,
// every product and sum rounded separately (no fma contraction)
__device__ __forceinline__ void momentum_step(float& p, float& b, float g, int first, float mom, float lr) {
#pragma clang fp contract(off)
  const float nb = first ? g : mom * b + g;   // buf.mul_(0.9).add_(grad)
  b = nb;
  p = p + (-lr) * nb;                         // p.add_(buf, alpha=-lr)
}

// the same step where lane condition `live` holds, p and b unchanged elsewhere (selects, no
// branch: the quarter-wave solvers' padding clients)
__device__ __forceinline__ void momentum_step_sel(float& p, float& b, float g, int first, float mom, float lr,
                                                  bool live) {
  float np = p, nb = b;
  momentum_step(np, nb, g, first, mom, lr);
  p = live ? np : p;
  b = live ? nb : b;
}

// max over the 16 lanes of a DPP row, one v_max_f32_dpp per level (hipcc's fmaxf over a DPP
// move costs a move, a canonicalising max and the max per level); every lane of the row ends
// with the same value.  Inputs are finite or -inf.
__device__ __forceinline__ float row16_max(float x) {
  float r;
  asm volatile(
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %1, %1 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
      : "=&v"(r)
      : "v"(x));
  return r;
}

// rs_bank<8> on the 8 pairs (v[i], v[i + 8]) and then rs_bank<4> on (v[i], v[i + 4]), i.e. the
// first two reduce-scatter levels of the quarter-wave solvers' 16 class partials, as two asm
// blocks with ONE hazard pad each (rs_bank pads every call: 12 x s_nop 1 per step).  Every DPP
// read in a block is of a block input, written before the block's pad; outputs are early-clobber.
__device__ __forceinline__ void rs_banks_8_4(float (&v)[16]) {
#define RSB8(o, a, b)                                                                        \
  "v_add_f32_dpp " o ", " a ", " a " row_ror:8 row_mask:0xf bank_mask:0x3\n\t"             \
  "v_add_f32_dpp " o ", " b ", " b " row_ror:8 row_mask:0xf bank_mask:0xc\n\t"
#define RSB4(o, a, b)                                                                        \
  "v_add_f32_dpp " o ", " a ", " a " row_shl:4 row_mask:0xf bank_mask:0x5\n\t"             \
  "v_add_f32_dpp " o ", " b ", " b " row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
  float w[8];
  asm volatile("s_nop 1\n\t" RSB8("%0", "%8", "%16") RSB8("%1", "%9", "%17") RSB8("%2", "%10", "%18")
               RSB8("%3", "%11", "%19") RSB8("%4", "%12", "%20") RSB8("%5", "%13", "%21")
               RSB8("%6", "%14", "%22") RSB8("%7", "%15", "%23")
               : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]), "=&v"(w[5]), "=&v"(w[6]),
                 "=&v"(w[7])
               : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]),
                 "v"(v[8]), "v"(v[9]), "v"(v[10]), "v"(v[11]), "v"(v[12]), "v"(v[13]), "v"(v[14]), "v"(v[15]));
  asm volatile("s_nop 1\n\t" RSB4("%0", "%4", "%8") RSB4("%1", "%5", "%9") RSB4("%2", "%6", "%10")
               RSB4("%3", "%7", "%11")
               : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
               : "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]));
#undef RSB8
#undef RSB4
}

// M permlane swaps (lane distance OFF = 32 or 16) of the pairs (a[i], b[i]) behind ONE hazard
// pad (rs_level / gather_pair pad every swap); the pairs are distinct registers, so no swap of
// the batch reads another's result
template <int OFF, int M>
__device__ __forceinline__ void swap_batch(float (&a)[M], float (&b)[M]) {
  static_assert((OFF == 32 || OFF == 16) && (M == 1 || M == 2 || M == 4), "swap batch");
  if constexpr (OFF == 32) {
    if constexpr (M == 1)
      asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a[0]), "+v"(b[0]));
    else if constexpr (M == 2)
      asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %2\n\tv_permlane32_swap_b32 %1, %3"
                   : "+v"(a[0]), "+v"(a[1]), "+v"(b[0]), "+v"(b[1]));
    else
      asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %4\n\tv_permlane32_swap_b32 %1, %5\n\t"
                   "v_permlane32_swap_b32 %2, %6\n\tv_permlane32_swap_b32 %3, %7"
                   : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]));
  } else {
    if constexpr (M == 1)
      asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a[0]), "+v"(b[0]));
    else if constexpr (M == 2)
      asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %2\n\tv_permlane16_swap_b32 %1, %3"
                   : "+v"(a[0]), "+v"(a[1]), "+v"(b[0]), "+v"(b[1]));
    else
      asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %4\n\tv_permlane16_swap_b32 %1, %5\n\t"
                   "v_permlane16_swap_b32 %2, %6\n\tv_permlane16_swap_b32 %3, %7"
                   : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]));
  }
}

constexpr int MR_WAVES = 16;

// Diagnostic build only (-DFS_MIX_STAMPS, `make stamps`): per-phase cycle sums of wave 0,
// written after the solver's buf[N] as buf[N + 8 + 2k] (uint64); never in the shipped library.
#ifdef FS_MIX_STAMPS
#define MR_STAMP(k)                                                                       \
  {                                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    unsigned long long t_;                                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    if (k > 0) mr_acc[k > 0 ? k - 1 : 0] += t_ - mr_prev;                                 \
    mr_prev = t_;                                                                         \
  }
#else
#define MR_STAMP(k)
#endif

// ----------------------------------------------------------------------------
// L2 prefetch helpers of the single-CU solvers.  One CU gathers random Z rows from the
// Infinity Cache at ~33.5 GB/s but from its XCD's L2 at 66-73 GB/s (MI355X_MICROARCH.md,
// "Indexed rows"); the register solver is bound by the former.  The
// step order is known before the launch (the perms), so H helper workgroups on the solver's
// XCD (blockIdx % 8 == 0 under round-robin placement) load the Z rows of the steps ahead
// of the solver into that L2: helper h takes steps h, h + H, ..., each wave one batch row,
// and stays at most `lead` steps ahead of the solver's progress word (wave 0 of the solver
// stores its step count every 4 steps).  Helpers change no bytes the solver reads or
// writes -- they only warm the cache -- so results are identical with any H (speed only).
// Every wait is bounded and a helper that starts late (after the solver) or falls behind
// skips to the solver's position; it exits once the solver's count reaches the total.
// ----------------------------------------------------------------------------
constexpr int PF_SPIN_LIMIT = 1 << 22;
constexpr int PF_INFLIGHT = 32;                   // 1-KB pieces a helper wave keeps in flight

__device__ __forceinline__ void mix_prefetch_helper(const float* __restrict__ Z, const int32_t* __restrict__ perms,
                                                 int N, int C, int nv, int epochs, int Bv, int h, int H, int lead,
                                                 const unsigned* prog, int zL = 0, int zR = 1) {
  // The loads only warm the caches: each is an LDS-DMA (global_load_lds_dwordx4, 1 KB per
  // wave instruction) into a sink no one reads, so a wave needs no registers for them and
  // keeps PF_INFLIGHT pieces in flight (a counted vmcnt throttle) instead of waiting for every
  // 4 KB (round 3's register form: at config 5's 40-KB rows, 10 dependent round trips per row,
  // ~5 us per step over 16 helpers -- slower than the solver, so the helpers fell behind)
  __shared__ __attribute__((aligned(1024))) char pf_sink[1024];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int nw = blockDim.x >> 6;
  // Z rows: zR blocks of zL clients (fs_mix_solve_blocked: [zR][n_val][C][zL]; else one block
  // of ldN): a row is zR segments of C * zL floats, nv * C * zL floats apart
  if (zL == 0) zL = mix_ldn(N);
  const int CN4 = C * zL / 4;                     // float4 per row segment (zL % 4 == 0)
  const int64_t bstride = (int64_t)nv * C * zL;
  const int nbat = (nv + Bv - 1) / Bv;
  const int total = epochs * nbat;
  unsigned seen = 0;
  int issued = 0;
  for (int t = h; t < total; t += H) {
    int spins = 0;
    while ((unsigned)t >= seen + (unsigned)lead) {   // pace: at most `lead` steps ahead
      seen = __builtin_amdgcn_readfirstlane(__hip_atomic_load(prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      if ((unsigned)t < seen + (unsigned)lead) break;
      if (++spins > PF_SPIN_LIMIT) return;
      __builtin_amdgcn_s_sleep(1);
    }
    if (seen >= (unsigned)total) return;           // the solver is done
    if ((unsigned)t < seen) {                      // fell behind: skip to the solver's step
      t += (int)((seen - (unsigned)t + H - 1) / H) * H;
      if (t >= total) return;
    }
    const int ep = t / nbat, sb = t - ep * nbat;
    const int bc = min(Bv, nv - sb * Bv);
    for (int r = w; r < bc * zR; r += nw) {
      const int rb = r / zR, blk = r - rb * zR;
      const int row = __builtin_amdgcn_readfirstlane(perms[(int64_t)ep * nv + sb * Bv + rb]);
      const float4* zr = reinterpret_cast<const float4*>(Z + blk * bstride + (int64_t)row * (4 * CN4));
      for (int i0 = 0; i0 < CN4; i0 += 64) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(zr + min(i0 + lane, CN4 - 1)),
                                         (__attribute__((address_space(3))) void*)pf_sink, 16, 0, 0);
        if (++issued == PF_INFLIGHT) {
          asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
          issued = 16;
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// the solver's side: publish the number of completed steps (vector store, relaxed agent scope)
__device__ __forceinline__ void mix_publish_progress(unsigned* prog, int s) {
  if (threadIdx.x == 0) __hip_atomic_store(prog, (unsigned)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NK> struct MRVec;
template <> struct MRVec<1> { typedef float T; };
template <> struct MRVec<2> { typedef float T __attribute__((ext_vector_type(2))); };
template <> struct MRVec<4> { typedef float T __attribute__((ext_vector_type(4))); };
template <int NK>
__device__ __forceinline__ float mr_el(const typename MRVec<NK>::T& v, int j) {
  if constexpr (NK == 1) return v;
  else return v[j];
}

template <int NK, int CP, int CL, int MR_DEPTH>
__global__ __launch_bounds__(MR_WAVES * 64) void mix_solve_reg_kernel(const float* __restrict__ Z,
                                                                     const int32_t* __restrict__ y,
                                                                     const int32_t* __restrict__ perms, int N,
                                                                     int C, int nv, int epochs, int Bv, float lr,
                                                                     float mom, float* __restrict__ p,
                                                                     float* __restrict__ buf,
                                                                     int* __restrict__ first_flag,
                                                                     unsigned* __restrict__ pf_prog, int pf_h,
                                                                     int pf_lead) {
  static_assert(CL <= CP && CP <= 32 && (CP & (CP - 1)) == 0, "class padding");
  static_assert(MR_DEPTH * (CL + 2) <= 63 && (MR_DEPTH == 2 || MR_DEPTH == 3), "ring vs the vmcnt window");
  if (blockIdx.x != 0) {                           // L2 prefetch helpers (speed only)
    if (pf_prog && blockIdx.x % 8 == 0)
      mix_prefetch_helper(Z, perms, N, C, nv, epochs, Bv, blockIdx.x / 8 - 1, pf_h, pf_lead, pf_prog);
    return;
  }
  typedef typename MRVec<NK>::T vec;
  constexpr int LPC = 64 / CP;                     // lanes per class after the reduce-scatter
  __shared__ __attribute__((aligned(16))) float gpart[MR_WAVES][NK * 64];
  __shared__ __attribute__((aligned(16))) float pnew[NK * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ldN = mix_ldn(N);
  const int CN = C * ldN;
  const int nbat = (nv + Bv - 1) / Bv;
  const int total = epochs * nbat;
  const int n0 = NK * lane;                        // this lane's first client
  float pr[NK];
#pragma unroll
  for (int j = 0; j < NK; ++j) pr[j] = n0 + j < N ? p[n0 + j] : 0.f;   // p stays 0 on padding clients
  // the update's owner of client `cn`: TPC = 16 / NK consecutive threads fold its 16 wave
  // partials (NK each, then a lane tree); the first of them keeps its p and momentum entry
  constexpr int TPC = MR_WAVES / NK;
  const int cn = tid / TPC, cq = tid % TPC;
  float po = (cq == 0 && cn < N) ? p[cn] : 0.f;
  float bo = (cq == 0 && cn < N) ? buf[cn] : 0.f;
  int first = *first_flag;
  const float invB = 1.0f / (float)Bv;            // 1/|batch| of every full batch
  // lane byte offset inside a class segment; lanes past ldN re-read the last vector (p = 0)
  const uint32_t nbyte = 4u * (uint32_t)min(n0, ldN - NK);
  vec zr[MR_DEPTH][CL];
  int lab[MR_DEPTH];
  int idxr[MR_DEPTH];                              // slot R: row indices (lanes < Bv) of step s + DEPTH
  // Every load below is unconditional (out-of-range lanes read a clamped, valid address and
  // their values are masked where used): a predicated load would make the compiler wait for
  // it at the join, which serialises the ring.
  auto row_of = [&](int st) -> int {               // perms entry of lane `lane` in step st
    const int ep = st / nbat, sb = st - ep * nbat;
    const int b = sb * Bv + lane;
    const int64_t at = (lane < Bv && b < nv && st < total) ? (int64_t)ep * nv + b : 0;
    return perms[at];                              // always a valid row of Z
  };
  auto bsize = [&](int st) -> int { return min(Bv, nv - (st % nbat) * Bv); };
  // issue the loads of one step (row indices in `idxv`, lanes < Bv) into ring slot R
#define MR_ISSUE(R_, IDXV_)                                                                \
  {                                                                                        \
    const int vrow_ = __builtin_amdgcn_readlane((IDXV_), w);                               \
    const char* zp_ = reinterpret_cast<const char*>(Z + (int64_t)vrow_ * CN);              \
    _Pragma("unroll") for (int c = 0; c < CL; ++c) {                                       \
      /* uniform class base (c >= C: masked in the softmax) + 32-bit lane byte offset */  \
      const char* zc_ = zp_ + 4 * (int64_t)(min(c, C - 1) * ldN);                          \
      zr[R_][c] = *reinterpret_cast<const vec*>(                                           \
          __builtin_assume_aligned(zc_ + nbyte, 4 * NK)); /* ldN % 4 == 0 */               \
    }                                                                                      \
    lab[R_] = y[(IDXV_)];                                                                  \
  }
  {
    const int i0 = row_of(0), i1 = row_of(1), i2 = row_of(2);
    idxr[0] = row_of(MR_DEPTH);
    idxr[1] = row_of(MR_DEPTH + 1);
    if constexpr (MR_DEPTH == 3) idxr[2] = row_of(MR_DEPTH + 2);
    MR_ISSUE(0, i0);
    MR_ISSUE(1, i1);
    if constexpr (MR_DEPTH == 3) MR_ISSUE(2, i2);
    // drain the prologue once, so the loop header inherits only the loop's own load order
    __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0)
  }
  // one step on ring slot R_
#define MR_STEP(R_)                                                                        \
  {                                                                                        \
    if (s >= total) break;                                                                 \
    MR_STAMP(0)                                                                            \
    /* indices of step s+DEPTH were loaded DEPTH steps ago; fetch those of s+2*DEPTH */   \
    const int idx_cur = idxr[R_];                                                          \
    idxr[R_] = row_of(s + 2 * MR_DEPTH);                                                   \
    const int bc = bsize(s);                                                               \
    float gme[NK];                                                                         \
    _Pragma("unroll") for (int j = 0; j < NK; ++j) gme[j] = 0.f;                           \
    MR_STAMP(1)                                                                            \
    if (w < bc) {                                                                          \
      float v[CP];                                                                         \
      _Pragma("unroll") for (int c = 0; c < CP; ++c) {                                     \
        float a = 0.f;                                                                     \
        if (c < CL) {                                                                      \
          _Pragma("unroll") for (int j = 0; j < NK; ++j) a += mr_el<NK>(zr[R_][c], j) * pr[j]; \
        }                                                                                  \
        v[c] = a;                                                                          \
      }                                                                                    \
      const float o = class_totals<CP>(v, lane);                                           \
      const int cls = lane / LPC;                                                          \
      const bool real = cls < C;                                                           \
      const float m = class_max<LPC>(real ? o : -INFINITY, lane);                          \
      const float e = class_sum<LPC>(real ? expf(o - m) : 0.f, lane);                      \
      const float lse = logf(e);                                                           \
      const float invb = bc == Bv ? invB : 1.0f / (float)bc;                               \
      const int yy = __builtin_amdgcn_readlane(lab[R_], w);                                \
      const float g = (cls == yy ? -invb : 0.f) + expf(o - m - lse) * invb;                \
      _Pragma("unroll") for (int c = 0; c < CL; ++c) {                                     \
        if (c < C) {                                                                       \
          const float gc = __builtin_bit_cast(float, __builtin_amdgcn_readlane(            \
              __builtin_bit_cast(int, g), c * LPC));                                       \
          _Pragma("unroll") for (int j = 0; j < NK; ++j) gme[j] += gc * mr_el<NK>(zr[R_][c], j); \
        }                                                                                  \
      }                                                                                    \
    }                                                                                      \
    MR_STAMP(2)                                                                            \
    _Pragma("unroll") for (int j = 0; j < NK; ++j) gpart[w][n0 + j] = gme[j];              \
    MR_ISSUE(R_, idx_cur);                                                                 \
    MR_STAMP(3)                                                                            \
    lds_barrier();                 /* not __syncthreads: that would drain the ring */     \
    MR_STAMP(4)                                                                            \
    {                              /* fold once per client, update at its owner */       \
      float gp = gpart[cq * NK][cn];                                                       \
      _Pragma("unroll") for (int i = 1; i < NK; ++i) gp += gpart[cq * NK + i][cn];         \
      _Pragma("unroll") for (int off = 1; off < TPC; off <<= 1) gp += xor_get(gp, off, lane); \
      if (cq == 0) {                                                                       \
        if (cn < N) momentum_step(po, bo, gp, first, mom, lr);                             \
        pnew[cn] = po;                                                                     \
      }                                                                                    \
    }                                                                                      \
    lds_barrier();                                                                         \
    if constexpr (NK == 1) pr[0] = pnew[n0];                                               \
    else {                                                                                 \
      const vec pv = *reinterpret_cast<const vec*>(&pnew[n0]);                             \
      _Pragma("unroll") for (int j = 0; j < NK; ++j) pr[j] = mr_el<NK>(pv, j);             \
    }                                                                                      \
    first = 0;                                                                             \
    MR_STAMP(5)                                                                            \
    ++s;                                                                                   \
    if (pf_prog && (s & 3) == 0) mix_publish_progress(pf_prog, s);                         \
  }
#ifdef FS_MIX_STAMPS
  unsigned long long mr_acc[5] = {0, 0, 0, 0, 0}, mr_prev = 0;
#endif
  int s = 0;
  for (;;) {
    MR_STEP(0)
    MR_STEP(1)
    if constexpr (MR_DEPTH == 3) MR_STEP(2)
  }
#undef MR_STEP
#undef MR_ISSUE
  if (pf_prog) mix_publish_progress(pf_prog, total);   // releases the helpers
  if (cq == 0 && cn < N) {
    p[cn] = po;
    buf[cn] = bo;
  }
  if (w == 0) {
    if (lane == 0 && total > 0) *first_flag = 0;
#ifdef FS_MIX_STAMPS
    if (lane < 5) reinterpret_cast<unsigned long long*>(buf + N + 8)[lane] = mr_acc[lane];
#endif
  }
}

struct MixPrefetch {
  unsigned* prog;   // progress word (null: no helpers)
  int h, lead;      // helper workgroups, steps ahead
};

template <int NK, int CP, int CL>
static void launch_mix_reg(hipStream_t st, const float* Z, const int32_t* y, const int32_t* perms, int N, int C,
                           int nv, int epochs, int Bv, float lr, float mom, float* p, float* buf, int* first,
                           const MixPrefetch& pf) {
  constexpr int depth = 3 * (CL + 2) <= 63 ? 3 : 2;   // CL + 2 loads per step stay in the vmcnt window
  const int blocks = pf.prog ? 8 * std::min(pf.h, 31) + 1 : 1;
  hipLaunchKernelGGL((mix_solve_reg_kernel<NK, CP, CL, depth>), dim3(blocks), dim3(MR_WAVES * 64), 0, st, Z, y,
                     perms, N, C, nv, epochs, Bv, lr, mom, p, buf, first, pf.prog, std::min(pf.h, 31), pf.lead);
}

// register-resident solver for (N, C, Bv) if an instance covers it
static bool mix_solve_reg(hipStream_t st, const float* Z, const int32_t* y, const int32_t* perms, int N, int C,
                          int nv, int epochs, int Bv, float lr, float mom, float* p, float* buf, int* first,
                          const MixPrefetch& pf) {
  if (Bv > MR_WAVES) return false;
  const int nk = N <= 64 ? 1 : (N <= 128 ? 2 : (N <= 256 ? 4 : 0));
#define MR_CASE(NK_, CP_, CL_)                                                                      \
  if (nk == NK_ && C <= CL_) {                                                                      \
    launch_mix_reg<NK_, CP_, CL_>(st, Z, y, perms, N, C, nv, epochs, Bv, lr, mom, p, buf, first, pf); \
    return true;                                                                                    \
  }
  // (the ring holds DEPTH * CL * NK floats per lane: larger shapes take the LDS-staged solver)
  MR_CASE(1, 2, 2) MR_CASE(1, 4, 4) MR_CASE(1, 8, 8) MR_CASE(1, 16, 10) MR_CASE(1, 16, 16) MR_CASE(1, 32, 24)
  MR_CASE(2, 2, 2) MR_CASE(2, 4, 4) MR_CASE(2, 8, 8) MR_CASE(2, 16, 10)
  MR_CASE(4, 2, 2) MR_CASE(4, 4, 4)
#undef MR_CASE
  return false;
}

// ----------------------------------------------------------------------------
// p-solve, register-resident form 2 (Bv <= 16, C <= CL <= 10, N <= 64*NK): the register
// solver above is VALU-bound (rocprofv3: the SIMDs' vector pipes ~80 % busy at config 2);
// this form does the same arithmetic in fewer vector instructions per step:
//   * 8 waves x 2 batch rows (rows w and w + 8): the per-step fixed work -- the cross-wave
//     gradient sum and the momentum step, which every wave repeats -- runs 8 times, not 16,
//     and the two rows' reductions interleave (independent DPP chains, fewer wait states);
//   * the batch's row indices and labels are wave-uniform: scalar loads, so the vector
//     memory queue holds only Z rows and the ring of in-flight steps stays DEPTH deep;
//   * Z rows through one buffer descriptor: row and class offsets are scalar (soffset), the
//     lane's client offset the only vector address operand;
//   * the two cross-half levels of the logits' reduce-scatter (lane distance 32 and 16) as
//     one v_permlane{32,16}_swap of (a, b) plus one add: after the swap every lane holds its
//     own and its partner's copy of the element it keeps (SWAP = 0 keeps the select form).
// ----------------------------------------------------------------------------
constexpr int M2_WAVES = 8;

// class_totals of lanes.h for two independent rows at once (the levels interleave)
template <int CP>
__device__ __forceinline__ void class_totals2(float (&v0)[CP], float (&v1)[CP], int lane, float& o0, float& o1) {
  constexpr int LPC = 64 / CP;
#define M2_LEVEL(OFF_)                                                              \
  if constexpr (CP >= 64 / (OFF_)) {                                               \
    constexpr int L_ = CP / (32 / (OFF_));                                         \
    _Pragma("unroll") for (int i = 0; i < L_ / 2; ++i) {                           \
      v0[i] = rs_level<OFF_, true>(v0[i], v0[i + L_ / 2], lane);                   \
      v1[i] = rs_level<OFF_, true>(v1[i], v1[i + L_ / 2], lane);                   \
    }                                                                              \
  }
  M2_LEVEL(32) M2_LEVEL(16) M2_LEVEL(8) M2_LEVEL(4) M2_LEVEL(2) M2_LEVEL(1)
#undef M2_LEVEL
  float a = v0[0], b = v1[0];
#pragma unroll
  for (int off = LPC / 2; off >= 1; off >>= 1) {
    a += xor_get(a, off, lane);
    b += xor_get(b, off, lane);
  }
  o0 = a;
  o1 = b;
}

template <int NK, int CP, int CL, int DEPTH>
__global__ __launch_bounds__(M2_WAVES * 64) void mix_solve_reg2_kernel(const float* __restrict__ Z,
                                                                      const int32_t* __restrict__ y,
                                                                      const int32_t* __restrict__ perms, int N, int C,
                                                                      int nv, int epochs, int Bv, float lr, float mom,
                                                                      float* __restrict__ p, float* __restrict__ buf,
                                                                      int* __restrict__ first_flag, int z_bytes) {
  static_assert(CL <= CP && CP <= 32 && (CP & (CP - 1)) == 0, "class padding");
  static_assert(2 * CL * DEPTH <= 63, "ring vs the vmcnt window");
  typedef typename MRVec<NK>::T vec;
  constexpr int LPC = 64 / CP;
  __shared__ __attribute__((aligned(16))) float gpart[2][M2_WAVES][NK * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ldN = mix_ldn(N);
  const int CN = C * ldN;
  const int nbat = (nv + Bv - 1) / Bv;
  const int total = epochs * nbat;
  const int n0 = NK * lane;
  float pr[NK], br[NK];
#pragma unroll
  for (int j = 0; j < NK; ++j) {
    const int n = n0 + j;
    pr[j] = n < N ? p[n] : 0.f;
    br[j] = n < N ? buf[n] : 0.f;
  }
  int first = *first_flag;
  const float invB = 1.0f / (float)Bv;
  // per-class lane byte offsets (VGPRs, computed once, so the row base is the only scalar
  // operand); lanes past ldN re-read the last vector (p = 0), classes c >= C re-read class
  // C - 1 (masked in the softmax)
  uint32_t cofs[CL];
#pragma unroll
  for (int c = 0; c < CL; ++c) cofs[c] = 4u * (uint32_t)(min(n0, ldN - NK) + min(c, C - 1) * ldN);
  const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Z), 0, z_bytes, 0x00020000);
  // fetch cursor: the step whose row indices are read next (stays on the last step at the end)
  int fst = 0, fep = 0, fsb = 0;
  auto fetch_rows = [&](int& i0, int& i1) {
    const int base = fep * nv + fsb * Bv;
    const int bc = min(Bv, nv - fsb * Bv);
    i0 = perms[base + (w < bc ? w : 0)];             // rows past the batch: its first row (masked)
    i1 = perms[base + (w + M2_WAVES < bc ? w + M2_WAVES : 0)];
    if (fst + 1 < total) {
      ++fst;
      if (++fsb == nbat) {
        fsb = 0;
        ++fep;
      }
    }
  };
  vec zr[DEPTH][2][CL];
  int idxq[DEPTH][2], labq[DEPTH][2];
#define M2_LOAD(DST_, ROW_, C_)                                                                    \
  {                                                                                                \
    const int so_ = (ROW_) * CN * 4;                                                               \
    if constexpr (NK == 1)                                                                         \
      DST_ = __builtin_bit_cast(vec, __builtin_amdgcn_raw_buffer_load_b32(zrs, cofs[C_], so_, 0));  \
    else if constexpr (NK == 2)                                                                    \
      DST_ = __builtin_bit_cast(vec, __builtin_amdgcn_raw_buffer_load_b64(zrs, cofs[C_], so_, 0));  \
    else                                                                                           \
      DST_ = __builtin_bit_cast(vec, __builtin_amdgcn_raw_buffer_load_b128(zrs, cofs[C_], so_, 0)); \
  }
#define M2_ISSUE(R_, I0_, I1_)                                                             \
  {                                                                                        \
    _Pragma("unroll") for (int c = 0; c < CL; ++c) {                                       \
      M2_LOAD(zr[R_][0][c], I0_, c)                                                        \
      M2_LOAD(zr[R_][1][c], I1_, c)                                                        \
    }                                                                                      \
  }
  // prologue: rows and labels of steps 0 .. DEPTH-1 in flight, row indices of DEPTH .. 2 DEPTH-1
#pragma unroll
  for (int k = 0; k < DEPTH; ++k) {
    int i0, i1;
    fetch_rows(i0, i1);
    labq[k][0] = y[i0];
    labq[k][1] = y[i1];
    M2_ISSUE(k, i0, i1);
  }
#pragma unroll
  for (int k = 0; k < DEPTH; ++k) fetch_rows(idxq[k][0], idxq[k][1]);
  // drain the prologue once, so the loop header inherits only the loop's own load order
  __builtin_amdgcn_s_waitcnt(0x0F70);              // vmcnt(0)
  int csb = 0;                                      // batch of step s within its epoch
  int s = 0;
#define M2_STEP(R_)                                                                        \
  {                                                                                        \
    if (s >= total) break;                                                                 \
    const int bc = min(Bv, nv - csb * Bv);                                                 \
    csb = csb + 1 == nbat ? 0 : csb + 1;                                                   \
    const bool ok0 = w < bc, ok1 = w + M2_WAVES < bc;                                      \
    float v0[CP], v1[CP];                                                                  \
    _Pragma("unroll") for (int c = 0; c < CP; ++c) {                                       \
      float a = 0.f, b = 0.f;                                                              \
      if (c < CL) {                                                                        \
        _Pragma("unroll") for (int j = 0; j < NK; ++j) {                                   \
          a += mr_el<NK>(zr[R_][0][c], j) * pr[j];                                         \
          b += mr_el<NK>(zr[R_][1][c], j) * pr[j];                                         \
        }                                                                                  \
      }                                                                                    \
      v0[c] = a;                                                                           \
      v1[c] = b;                                                                           \
    }                                                                                      \
    float o0, o1;                                                                          \
    class_totals2<CP>(v0, v1, lane, o0, o1);                                         \
    const int cls = lane / LPC;                                                            \
    const bool real = cls < C;                                                             \
    const float m0 = class_max<LPC>(real ? o0 : -INFINITY, lane);                          \
    const float m1 = class_max<LPC>(real ? o1 : -INFINITY, lane);                          \
    const float e0 = class_sum<LPC>(real ? expf(o0 - m0) : 0.f, lane);                     \
    const float e1 = class_sum<LPC>(real ? expf(o1 - m1) : 0.f, lane);                     \
    const float invb = bc == Bv ? invB : 1.0f / (float)bc;                                 \
    const float g0 = ok0 ? (cls == labq[R_][0] ? -invb : 0.f) + expf(o0 - m0 - logf(e0)) * invb : 0.f; \
    const float g1 = ok1 ? (cls == labq[R_][1] ? -invb : 0.f) + expf(o1 - m1 - logf(e1)) * invb : 0.f; \
    float gme[NK];                                                                         \
    _Pragma("unroll") for (int j = 0; j < NK; ++j) gme[j] = 0.f;                           \
    _Pragma("unroll") for (int c = 0; c < CL; ++c) {                                       \
      if (c < C) {                                                                         \
        const float gc0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, g0), c * LPC)); \
        const float gc1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, g1), c * LPC)); \
        _Pragma("unroll") for (int j = 0; j < NK; ++j) {                                   \
          gme[j] += gc0 * mr_el<NK>(zr[R_][0][c], j);                                      \
          gme[j] += gc1 * mr_el<NK>(zr[R_][1][c], j);                                      \
        }                                                                                  \
      }                                                                                    \
    }                                                                                      \
    const int par = s & 1;                                                                 \
    _Pragma("unroll") for (int j = 0; j < NK; ++j) gpart[par][w][n0 + j] = gme[j];         \
    /* the slot's rows are consumed: refill it with step s + DEPTH, label first */         \
    labq[R_][0] = y[idxq[R_][0]];                                                          \
    labq[R_][1] = y[idxq[R_][1]];                                                          \
    M2_ISSUE(R_, idxq[R_][0], idxq[R_][1]);                                                \
    lds_barrier();                 /* not __syncthreads: that would drain the ring */     \
    fetch_rows(idxq[R_][0], idxq[R_][1]);       /* step s + 2 DEPTH */                     \
    _Pragma("unroll") for (int j = 0; j < NK; ++j) {                                       \
      float gp = 0.f;                                                                      \
      _Pragma("unroll") for (int i = 0; i < M2_WAVES; ++i) gp += gpart[par][i][n0 + j];    \
      if (n0 + j < N) momentum_step(pr[j], br[j], gp, first, mom, lr);                     \
    }                                                                                      \
    first = 0;                                                                             \
    ++s;                                                                                   \
  }
  for (;;) {
    M2_STEP(0)
    if constexpr (DEPTH > 1) M2_STEP(1)
    if constexpr (DEPTH > 2) M2_STEP(2)
  }
#undef M2_STEP
#undef M2_ISSUE
#undef M2_LOAD
  if (w == 0) {
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int n = n0 + j;
      if (n < N) {
        p[n] = pr[j];
        buf[n] = br[j];
      }
    }
    if (lane == 0 && total > 0) *first_flag = 0;
  }
}

template <int NK, int CP, int CL>
static void launch_mix_reg2(hipStream_t st, const float* Z, const int32_t* y, const int32_t* perms, int N, int C,
                            int nv, int epochs, int Bv, float lr, float mom, float* p, float* buf, int* first,
                            int z_bytes) {
  constexpr int depth = 2 * CL * 3 <= 63 ? 3 : (2 * CL * 2 <= 63 ? 2 : 1);
  hipLaunchKernelGGL((mix_solve_reg2_kernel<NK, CP, CL, depth>), dim3(1), dim3(M2_WAVES * 64), 0, st, Z, y,
                     perms, N, C, nv, epochs, Bv, lr, mom, p, buf, first, z_bytes);
}

// register-resident solver, form 2, for (N, C, Bv) if an instance covers it
static bool mix_solve_reg2(hipStream_t st, const float* Z, const int32_t* y, const int32_t* perms, int N, int C,
                           int nv, int epochs, int Bv, float lr, float mom, float* p, float* buf, int* first) {
  if (Bv > 2 * M2_WAVES || C > 10) return false;
  const int64_t zb = (int64_t)nv * C * mix_ldn(N) * 4;
  if (zb >= ((int64_t)1 << 31) || (int64_t)epochs * nv >= ((int64_t)1 << 31)) return false;   // 32-bit offsets
  const int nk = N <= 64 ? 1 : (N <= 128 ? 2 : (N <= 256 ? 4 : 0));
#define M2_CASE(NK_, CP_, CL_)                                                                              \
  if (nk == NK_ && C <= CL_) {                                                                              \
    launch_mix_reg2<NK_, CP_, CL_>(st, Z, y, perms, N, C, nv, epochs, Bv, lr, mom, p, buf, first, (int)zb);       \
    return true;                                                                                            \
  }
  M2_CASE(1, 2, 2) M2_CASE(1, 4, 4) M2_CASE(1, 8, 8) M2_CASE(1, 16, 10)
  M2_CASE(2, 2, 2) M2_CASE(2, 4, 4) M2_CASE(2, 8, 8) M2_CASE(2, 16, 10)
  M2_CASE(4, 2, 2) M2_CASE(4, 4, 4)
#undef M2_CASE
  return false;
}

// ----------------------------------------------------------------------------
// p-solve, quarter-wave form "quad" (Bv <= 16, N <= 16*NK, C <= CL <= 16).  The register
// solvers above are bound by the vector ALU, not by the Z gather: at config 2 a step costs the
// same 2.36-2.46 us with Z = 51 MB (Infinity Cache) as with Z = 0.5 MB (L2), and with
// s_memtime stamps the first wave of each SIMD finishes its row ~2,500 cycles before the last
// (4 waves x ~270 VALU instructions per step on every SIMD; r02s2c/d).  Most of those
// instructions are the cross-lane reductions of ONE row over 64 lanes.  Here a row takes 16
// lanes (one DPP row), so one wave instruction advances 4 batch rows at once:
//   * 4 waves x 4 rows (batch row b = 4w + q for lane group q = lane / 16); lane (q, r) holds
//     clients n = NK*r + j of its row, every class: the logits' partials are NK-term dot
//     products, reduce-scattered over the 16 lanes (levels 8 and 4 as two bank-masked DPP
//     adds each, 2 and 1 in the select form) so that lane r ends with class r's logit;
//   * softmax max / sum as 4-level DPP all-reduces inside the row (bitwise-identical in
//     every lane of the row), the CE gradient g of lane r's class;
//   * the row's g values broadcast through 64 bytes of the wave's own LDS (16 lanes read one
//     address: no conflict, no barrier), the gradient partials of the NK clients in-lane;
//   * the 4 rows of a wave folded by a reduce-scatter over the row groups (permlane32 /
//     permlane16 swaps: lane keeps NK/4 clients), the 4 waves' partials through LDS (ONE
//     raw barrier per step, double-buffered by step parity), summed in wave order by every
//     wave -- the same bits everywhere -- then the momentum step on the kept clients and an
//     all-gather (the same swaps) returns p to the NK-per-lane layout;
//   * Z through one buffer descriptor (row offset per lane group, class offset scalar), a
//     DEPTH-deep register ring; row indices and labels per lane, DEPTH steps ahead.
// Optional L2 prefetch helpers as for the register solver (FS_MIX_PF_H).
// ----------------------------------------------------------------------------
constexpr int MQ_WAVES = 4;
// Diagnostic build only (`make probe`, -DFS_MIX_PROBE_NOLOAD): the quarter-wave solver skips
// its in-loop Z loads (the ring keeps its first rows: wrong p, timing only) -- what a step costs
// without the vector-memory issue.  Never in the shipped library.
#ifdef FS_MIX_PROBE_NOLOAD
constexpr bool kMixProbeNoLoad = true;
#else
constexpr bool kMixProbeNoLoad = false;
#endif

typedef float float2v __attribute__((ext_vector_type(2)));
// elements (2h, 2h+1) of a float4
__device__ __forceinline__ float2v half2(const floatx4& v, int h) {
  return h ? float2v{v[2], v[3]} : float2v{v[0], v[1]};
}

template <int NK, int CL, int DEPTH, int SPL, bool FASTX>
__global__ __launch_bounds__(MQ_WAVES * 64) void mix_solve_quad_kernel(
    const float* __restrict__ Z, const int32_t* __restrict__ y, const int32_t* __restrict__ perms, int N, int C,
    int nv, int epochs, int Bv, float lr, float mom, float* __restrict__ p, float* __restrict__ buf,
    int* __restrict__ first_flag, int z_bytes, unsigned* __restrict__ pf_prog, int pf_h, int pf_lead) {
  static_assert(NK == 4 || NK == 8, "clients per lane");
  static_assert(CL >= 1 && CL <= 16, "classes");
  static_assert(DEPTH * (CL * NK / 4 + 2) <= 63, "ring vs the vmcnt window");
  static_assert(SPL >= 1 && SPL <= CL, "issue split");
  if (blockIdx.x != 0) {                           // L2 prefetch helpers (speed only)
    if (pf_prog && blockIdx.x % 8 == 0)
      mix_prefetch_helper(Z, perms, N, C, nv, epochs, Bv, blockIdx.x / 8 - 1, pf_h, pf_lead, pf_prog);
    return;
  }
  constexpr int NV4 = NK / 4;                      // float4 chunks per class and lane
  constexpr int KP = NK / 4;                       // clients a lane keeps after the row fold
  __shared__ __attribute__((aligned(16))) float gx[2][MQ_WAVES][64 * KP];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r = lane & 15;
  const int brow = MQ_WAVES * w + q;               // this lane group's batch row
  const int ldN = mix_ldn(N);
  const int CN = C * ldN;
  const int nbat = (nv + Bv - 1) / Bv;
  const int total = epochs * nbat;
  const int bc_tail = nv - (nbat - 1) * Bv;
  const float invB = 1.0f / (float)Bv;
  const float invT = 1.0f / (float)bc_tail;
  const int n0 = NK * r;
  float pr[NK];
#pragma unroll
  for (int j = 0; j < NK; ++j) pr[j] = n0 + j < N ? p[n0 + j] : 0.f;   // p = 0 on padding clients
  // kept clients after the fold over the row groups: j = (q >> 1) NK/2 + (q & 1) NK/4 + i
  const int kj0 = (q >> 1) * (NK / 2) + (q & 1) * (NK / 4);
  float po[KP], bo[KP];
#pragma unroll
  for (int i = 0; i < KP; ++i) {
    const int n = n0 + kj0 + i;
    po[i] = n < N ? p[n] : 0.f;
    bo[i] = n < N ? buf[n] : 0.f;
  }
  int first = *first_flag;
  // lane byte offsets of its client chunks inside a class segment; a chunk wholly past ldN
  // gets an offset beyond the buffer's range: the load returns zeros without a memory access
  uint32_t lofs[NV4];
#pragma unroll
  for (int h = 0; h < NV4; ++h)
    lofs[h] = n0 + 4 * h < ldN ? 4u * (uint32_t)(n0 + 4 * h) : 0x80000000u;
  int sofs[CL];
#pragma unroll
  for (int c = 0; c < CL; ++c) sofs[c] = __builtin_amdgcn_readfirstlane(4 * min(c, C - 1) * ldN);
  const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Z), 0, z_bytes, 0x00020000);
  // fetch cursor: the step whose row indices are read next (stays on the last step at the end)
  int fst = 0, fep = 0, fsb = 0;
  auto fetch_row = [&]() -> int {
    const int base = fep * nv + fsb * Bv;
    const int bc = min(Bv, nv - fsb * Bv);
    const int row = perms[base + (brow < bc ? brow : 0)];   // rows past the batch: its first (masked)
    if (fst + 1 < total) {
      ++fst;
      if (++fsb == nbat) {
        fsb = 0;
        ++fep;
      }
    }
    return row;
  };
  floatx4 zr[DEPTH][CL][NV4];
  int idxq[DEPTH], labq[DEPTH];
#define MQ_ISSUE(R_, ROW_, C0_, C1_)                                                         \
  {                                                                                          \
    const uint32_t ro_ = (uint32_t)(ROW_) * (uint32_t)CN * 4u;                               \
    _Pragma("unroll") for (int c = (C0_); c < (C1_); ++c) {                                      \
      _Pragma("unroll") for (int h = 0; h < NV4; ++h) zr[R_][c][h] = __builtin_bit_cast(     \
          floatx4, __builtin_amdgcn_raw_buffer_load_b128(zrs, ro_ + lofs[h], sofs[c], 0));   \
    }                                                                                        \
  }
#pragma unroll
  for (int k = 0; k < DEPTH; ++k) {
    const int row = fetch_row();
    labq[k] = y[row];
    MQ_ISSUE(k, row, 0, CL);
  }
#pragma unroll
  for (int k = 0; k < DEPTH; ++k) idxq[k] = fetch_row();
  __builtin_amdgcn_s_waitcnt(0x0F70);              // vmcnt(0): the loop inherits only its own order
  int csb = 0;
  int s = 0;
  int late_row = 0;                                 // row of the step whose late classes are pending
#ifdef FS_MIX_STAMPS
  unsigned long long mr_acc[6] = {0, 0, 0, 0, 0, 0}, mr_prev = 0;
#endif
#define MQ_STEP(R_)                                                                          \
  {                                                                                          \
    if (s >= total) break;                                                                   \
    MR_STAMP(0)                                                                              \
    const int bc = min(Bv, nv - csb * Bv);                                                   \
    csb = csb + 1 == nbat ? 0 : csb + 1;                                                     \
    float v[16];                                                                             \
    {              /* packed pairs (v_pk_fma_f32): even and odd clients summed apart, then    \
                      joined; the classes' chains interleaved (independent accumulators) */   \
      float2v a2[CL];                                                                        \
      _Pragma("unroll") for (int c = 0; c < CL; ++c) a2[c] = float2v{0.f, 0.f};              \
      _Pragma("unroll") for (int j = 0; j < NK; j += 2) {                                    \
        _Pragma("unroll") for (int c = 0; c < CL; ++c) a2[c] = __builtin_elementwise_fma(   \
            half2(zr[R_][c][j >> 2], (j >> 1) & 1), float2v{pr[j], pr[j + 1]}, a2[c]);      \
      }                                                                                      \
      _Pragma("unroll") for (int c = 0; c < 16; ++c) v[c] = c < CL ? a2[c].x + a2[c].y : 0.f; \
    }                                                                                        \
    MR_STAMP(1)                                                                              \
    /* the late classes of step s - 1 + DEPTH (its early ones went out with the last step) */ \
    if constexpr (SPL < CL && !kMixProbeNoLoad) {                                            \
      if (s > 0) MQ_ISSUE((R_ + DEPTH - 1) % DEPTH, late_row, SPL, CL);                      \
    }                                                                                        \
    rs_banks_8_4(v);                                                                         \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) v[i] = rs_pair(v[i], v[i + 2], 2, lane);   \
    const float o = rs_pair(v[0], v[1], 1, lane);  /* class r's logit */                     \
    const bool real = r < C;                                                                 \
    const float m = row16_max(real ? o : -INFINITY);                                         \
    const float invb = bc == Bv ? invB : invT;                                               \
    float g;                                                                                 \
    if constexpr (FASTX) {         /* v_exp_f32 / v_rcp_f32: softmax = e / sum */            \
      const float e = real ? __expf(o - m) : 0.f;                                            \
      const float ssum = row16_all<false>(e);                                                \
      g = (real && brow < bc) ? (r == labq[R_] ? -invb : 0.f) + e * __builtin_amdgcn_rcpf(ssum) * invb : 0.f; \
    } else {                       /* torch's log_softmax backward: exp(o - m - log(sum)) */ \
      const float ssum = row16_all<false>(real ? expf(o - m) : 0.f);                         \
      g = (real && brow < bc) ? (r == labq[R_] ? -invb : 0.f) + expf(o - m - logf(ssum)) * invb : 0.f; \
    }                                                                                        \
    float gv[CL];                  /* g of class c of this row: DPP row broadcast */         \
    _Pragma("unroll") for (int c = 0; c < CL; ++c) gv[c] = row_get(g, c);                    \
    float2v gm2[NK / 2];                                                                      \
    _Pragma("unroll") for (int j = 0; j < NK / 2; ++j) gm2[j] = float2v{0.f, 0.f};            \
    _Pragma("unroll") for (int c = 0; c < CL; ++c) {                                         \
      _Pragma("unroll") for (int j = 0; j < NK / 2; ++j) gm2[j] = __builtin_elementwise_fma( \
          float2v{gv[c], gv[c]}, half2(zr[R_][c][j >> 1], j & 1), gm2[j]);                   \
    }                                                                                        \
    float gme[NK];                                                                           \
    _Pragma("unroll") for (int j = 0; j < NK / 2; ++j) {                                     \
      gme[2 * j] = gm2[j].x;                                                                 \
      gme[2 * j + 1] = gm2[j].y;                                                             \
    }                                                                                        \
    MR_STAMP(2)                                                                              \
    /* slot consumed: refill with step s + DEPTH, then fetch the rows of s + 2 DEPTH */      \
    labq[R_] = y[idxq[R_]];                                                                  \
    if constexpr (!kMixProbeNoLoad) MQ_ISSUE(R_, idxq[R_], 0, SPL);                          \
    late_row = idxq[R_];                                                                     \
    idxq[R_] = fetch_row();                                                                  \
    MR_STAMP(6)                                                                              \
    /* fold the wave's 4 rows: reduce-scatter over the row groups */                         \
    float t[NK / 2];               /* = rs_level<32> / <16>, one pad per level */            \
    {                                                                                        \
      float sa[NK / 2], sb[NK / 2];                                                          \
      _Pragma("unroll") for (int i = 0; i < NK / 2; ++i) {                                   \
        sa[i] = gme[i];                                                                      \
        sb[i] = gme[i + NK / 2];                                                             \
      }                                                                                      \
      swap_batch<32, NK / 2>(sa, sb);                                                        \
      _Pragma("unroll") for (int i = 0; i < NK / 2; ++i) t[i] = sa[i] + sb[i];               \
    }                                                                                        \
    float u[KP];                                                                             \
    {                                                                                        \
      float sa[KP], sb[KP];                                                                  \
      _Pragma("unroll") for (int i = 0; i < KP; ++i) {                                       \
        sa[i] = t[i];                                                                        \
        sb[i] = t[i + KP];                                                                   \
      }                                                                                      \
      swap_batch<16, KP>(sa, sb);                                                            \
      _Pragma("unroll") for (int i = 0; i < KP; ++i) u[i] = sa[i] + sb[i];                   \
    }                                                                                        \
    const int par = s & 1;                                                                   \
    _Pragma("unroll") for (int i = 0; i < KP; ++i) gx[par][w][lane * KP + i] = u[i];         \
    MR_STAMP(3)                                                                              \
    lds_barrier();                 /* not __syncthreads: that would drain the ring */       \
    MR_STAMP(4)                                                                              \
    _Pragma("unroll") for (int i = 0; i < KP; ++i) {                                         \
      float gs = gx[par][0][lane * KP + i];                                                  \
      _Pragma("unroll") for (int k = 1; k < MQ_WAVES; ++k) gs += gx[par][k][lane * KP + i];  \
      momentum_step_sel(po[i], bo[i], gs, first, mom, lr, n0 + kj0 + i < N);                 \
    }                                                                                        \
    first = 0;                                                                               \
    /* all-gather p back to NK clients per lane */                                           \
    {                              /* = gather_pair<16> / <32>, one pad per level */         \
      float sa[KP], sb[KP];                                                                  \
      _Pragma("unroll") for (int i = 0; i < KP; ++i) sa[i] = sb[i] = po[i];                  \
      swap_batch<16, KP>(sa, sb);                                                            \
      _Pragma("unroll") for (int i = 0; i < KP; ++i) {                                       \
        t[i] = sa[i];                                                                        \
        t[i + KP] = sb[i];                                                                   \
      }                                                                                      \
      float ga[NK / 2], gb2[NK / 2];                                                         \
      _Pragma("unroll") for (int i = 0; i < NK / 2; ++i) ga[i] = gb2[i] = t[i];              \
      swap_batch<32, NK / 2>(ga, gb2);                                                       \
      _Pragma("unroll") for (int i = 0; i < NK / 2; ++i) {                                   \
        pr[i] = ga[i];                                                                       \
        pr[i + NK / 2] = gb2[i];                                                             \
      }                                                                                      \
    }                                                                                        \
    MR_STAMP(5)                                                                              \
    ++s;                                                                                     \
    if (pf_prog && (s & 3) == 0) mix_publish_progress(pf_prog, s);                           \
  }
  for (;;) {
    MQ_STEP(0)
    if constexpr (DEPTH > 1) MQ_STEP(1)
    if constexpr (DEPTH > 2) MQ_STEP(2)
  }
#undef MQ_STEP
#undef MQ_ISSUE
  if (pf_prog) mix_publish_progress(pf_prog, total);   // releases the helpers
  if (w == 0) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      const int n = n0 + kj0 + i;
      if (n < N) {
        p[n] = po[i];
        buf[n] = bo[i];
      }
    }
    if (lane == 0 && total > 0) *first_flag = 0;
#ifdef FS_MIX_STAMPS
    if (lane < 6) reinterpret_cast<unsigned long long*>(buf + N + 8)[lane] = mr_acc[lane];
#endif
  }
}

// default issue split: about 3/10 of the classes at the end of a step, the rest after the next
// step's logits (r02s2j/k, config 2: 1.65 us per step unsplit, 1.42-1.47 split 3 or 5 without
// helpers, 1.35-1.43 with 4 helpers; split 3 also keeps the (8, 10) instance in 242 VGPRs)
template <int CL>
constexpr int quad_split() { return (3 * CL + 9) / 10; }

// ----------------------------------------------------------------------------
// The quarter-wave solver with LOADER WAVES (round 4, fs_tuning.mix_quad_loaders).  The
// no-load probe (`make probe`, profiles/r04/quad_noload_probe.txt) put a third of quad's step
// at config 2 in issuing its Z loads: 20 buffer_load_dwordx4 per wave per step, ~40 cycles
// each, in the compute waves' own instruction stream (1.25 -> 0.87 us per step without them).
// Here 4 more waves (one per SIMD) issue the late classes' loads as LDS-DMA
// (global_load_lds_dwordx4, 1 KB per instruction, the lane layout of the register ring) into a
// 2-slot LDS ring: loader L serves compute wave L's 4 rows.  Step s's slot is filled after the
// workgroup barrier of step s - 2 (whose compute waves had read it) and landed (vmcnt(0)) before
// the barrier of step s - 1; the compute waves read it with ds_read_b128 at step s.  The early
// classes stay in the compute waves' register ring as in quad.  Same values into the same
// arithmetic: bitwise quad's p (tests/test_gpu_parity.py).  Lanes past ldN (padding clients,
// p = 0 and never stepped) read column 0 instead of zeros: finite values times p = 0.
// ----------------------------------------------------------------------------
template <int NK, int CL, int SPL>
__global__ __launch_bounds__(2 * MQ_WAVES * 64) void mix_solve_quadl_kernel(
    const float* __restrict__ Z, const int32_t* __restrict__ y, const int32_t* __restrict__ perms, int N, int C,
    int nv, int epochs, int Bv, float lr, float mom, float* __restrict__ p, float* __restrict__ buf,
    int* __restrict__ first_flag, int z_bytes, unsigned* __restrict__ pf_prog, int pf_h, int pf_lead) {
  static_assert(NK == 4 || NK == 8, "clients per lane");
  static_assert(SPL >= 1 && SPL < CL && CL <= 16, "classes");
  constexpr int DEPTH = 2;
  constexpr int NV4 = NK / 4;
  constexpr int KP = NK / 4;
  constexpr int CLL = CL - SPL;                    // late classes, through LDS
  static_assert(DEPTH * MQ_WAVES * CLL * NV4 * 1024 <= 128 * 1024, "LDS ring");
  if (blockIdx.x != 0) {                           // L2 prefetch helpers (speed only)
    if (pf_prog && blockIdx.x % 8 == 0)
      mix_prefetch_helper(Z, perms, N, C, nv, epochs, Bv, blockIdx.x / 8 - 1, pf_h, pf_lead, pf_prog);
    return;
  }
  __shared__ __attribute__((aligned(1024))) char lz[DEPTH][MQ_WAVES][CLL][NV4][1024];
  __shared__ __attribute__((aligned(16))) float gx[2][MQ_WAVES][64 * KP];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int w = wv & (MQ_WAVES - 1);               // compute wave w, or the loader of wave w's rows
  const int q = lane >> 4, r = lane & 15;
  const int brow = MQ_WAVES * w + q;
  const int ldN = mix_ldn(N);
  const int CN = C * ldN;
  const int nbat = (nv + Bv - 1) / Bv;
  const int total = epochs * nbat;
  const int n0 = NK * r;
  int fst = 0, fep = 0, fsb = 0;
  auto fetch_row = [&]() -> int {
    const int base = fep * nv + fsb * Bv;
    const int bc = min(Bv, nv - fsb * Bv);
    const int row = perms[base + (brow < bc ? brow : 0)];
    if (fst + 1 < total) {
      ++fst;
      if (++fsb == nbat) {
        fsb = 0;
        ++fep;
      }
    }
    return row;
  };
  if (wv >= MQ_WAVES) {
    // ---- loader wave: the late classes of its compute wave's rows, two steps ahead ----
    int cofs[NV4];
#pragma unroll
    for (int h = 0; h < NV4; ++h) cofs[h] = n0 + 4 * h < ldN ? n0 + 4 * h : 0;
    auto issue = [&](int slot, int row) {
      const float* zrow = Z + (int64_t)row * CN;
#pragma unroll
      for (int c = 0; c < CLL; ++c) {
        const int cc = min(c + SPL, C - 1);
#pragma unroll
        for (int h = 0; h < NV4; ++h)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(zrow + cc * ldN + cofs[h]),
                                           (__attribute__((address_space(3))) void*)&lz[slot][w][c][h][0], 16, 0, 0);
      }
    };
    issue(0, fetch_row());
    issue(1, fetch_row());
    int next = fetch_row();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                  // B_init: slots 0 and 1 landed
    for (int s = 0; s < total; ++s) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // step s + 1's slot landed
      __builtin_amdgcn_s_barrier();                // B_s: the compute waves are done with slot s & 1
      asm volatile("" ::: "memory");
      if (s + 2 < total) {
        issue(s & 1, next);
        next = fetch_row();
      }
    }
    return;
  }
  // ---- compute wave: quad's step, the late classes from the LDS ring ----
  float pr[NK];
#pragma unroll
  for (int j = 0; j < NK; ++j) pr[j] = n0 + j < N ? p[n0 + j] : 0.f;
  const int kj0 = (q >> 1) * (NK / 2) + (q & 1) * (NK / 4);
  float po[KP], bo[KP];
#pragma unroll
  for (int i = 0; i < KP; ++i) {
    const int n = n0 + kj0 + i;
    po[i] = n < N ? p[n] : 0.f;
    bo[i] = n < N ? buf[n] : 0.f;
  }
  int first = *first_flag;
  const float invB = 1.0f / (float)Bv;
  const float invT = 1.0f / (float)(nv - (nbat - 1) * Bv);
  uint32_t lofs[NV4];
#pragma unroll
  for (int h = 0; h < NV4; ++h) lofs[h] = n0 + 4 * h < ldN ? 4u * (uint32_t)(n0 + 4 * h) : 0x80000000u;
  int sofs[SPL];
#pragma unroll
  for (int c = 0; c < SPL; ++c) sofs[c] = __builtin_amdgcn_readfirstlane(4 * min(c, C - 1) * ldN);
  const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Z), 0, z_bytes, 0x00020000);
  floatx4 zr[DEPTH][SPL][NV4];
  int idxq[DEPTH], labq[DEPTH];
#define QL_ISSUE(R_, ROW_)                                                                   \
  {                                                                                          \
    const uint32_t ro_ = (uint32_t)(ROW_) * (uint32_t)CN * 4u;                               \
    _Pragma("unroll") for (int c = 0; c < SPL; ++c) {                                        \
      _Pragma("unroll") for (int h = 0; h < NV4; ++h) zr[R_][c][h] = __builtin_bit_cast(     \
          floatx4, __builtin_amdgcn_raw_buffer_load_b128(zrs, ro_ + lofs[h], sofs[c], 0));   \
    }                                                                                        \
  }
#pragma unroll
  for (int k = 0; k < DEPTH; ++k) {
    const int row = fetch_row();
    labq[k] = y[row];
    QL_ISSUE(k, row);
  }
#pragma unroll
  for (int k = 0; k < DEPTH; ++k) idxq[k] = fetch_row();
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __builtin_amdgcn_s_barrier();                    // B_init
  asm volatile("" ::: "memory");
  int csb = 0;
  int s = 0;
#ifdef FS_MIX_STAMPS
  unsigned long long mr_acc[6] = {0, 0, 0, 0, 0, 0}, mr_prev = 0;
#endif
#define QL_STEP(R_)                                                                          \
  {                                                                                          \
    if (s >= total) break;                                                                   \
    MR_STAMP(0)                                                                              \
    floatx4 zl[CLL][NV4];          /* the late classes of this step, from the LDS ring */   \
    _Pragma("unroll") for (int c = 0; c < CLL; ++c) {                                        \
      _Pragma("unroll") for (int h = 0; h < NV4; ++h)                                        \
        zl[c][h] = *reinterpret_cast<const floatx4*>(&lz[R_][w][c][h][lane * 16]);           \
    }                                                                                        \
    const int bc = min(Bv, nv - csb * Bv);                                                   \
    csb = csb + 1 == nbat ? 0 : csb + 1;                                                     \
    float v[16];                                                                             \
    {                                                                                        \
      float2v a2[CL];                                                                        \
      _Pragma("unroll") for (int c = 0; c < CL; ++c) a2[c] = float2v{0.f, 0.f};              \
      _Pragma("unroll") for (int j = 0; j < NK; j += 2) {                                    \
        _Pragma("unroll") for (int c = 0; c < CL; ++c) a2[c] = __builtin_elementwise_fma(   \
            half2(c < SPL ? zr[R_][c < SPL ? c : 0][j >> 2] : zl[c < SPL ? 0 : c - SPL][j >> 2], \
                  (j >> 1) & 1),                                                             \
            float2v{pr[j], pr[j + 1]}, a2[c]);                                               \
      }                                                                                      \
      _Pragma("unroll") for (int c = 0; c < 16; ++c) v[c] = c < CL ? a2[c].x + a2[c].y : 0.f; \
    }                                                                                        \
    MR_STAMP(1)                                                                              \
    rs_banks_8_4(v);                                                                         \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) v[i] = rs_pair(v[i], v[i + 2], 2, lane);   \
    const float o = rs_pair(v[0], v[1], 1, lane);                                            \
    const bool real = r < C;                                                                 \
    const float m = row16_max(real ? o : -INFINITY);                                         \
    const float invb = bc == Bv ? invB : invT;                                               \
    const float e = real ? __expf(o - m) : 0.f;                                              \
    const float ssum = row16_all<false>(e);                                                  \
    const float g = (real && brow < bc) ? (r == labq[R_] ? -invb : 0.f) + e * __builtin_amdgcn_rcpf(ssum) * invb \
                                        : 0.f;                                               \
    float gv[CL];                                                                            \
    _Pragma("unroll") for (int c = 0; c < CL; ++c) gv[c] = row_get(g, c);                    \
    float2v gm2[NK / 2];                                                                     \
    _Pragma("unroll") for (int j = 0; j < NK / 2; ++j) gm2[j] = float2v{0.f, 0.f};           \
    _Pragma("unroll") for (int c = 0; c < CL; ++c) {                                         \
      _Pragma("unroll") for (int j = 0; j < NK / 2; ++j) gm2[j] = __builtin_elementwise_fma( \
          float2v{gv[c], gv[c]},                                                             \
          half2(c < SPL ? zr[R_][c < SPL ? c : 0][j >> 1] : zl[c < SPL ? 0 : c - SPL][j >> 1], j & 1), \
          gm2[j]);                                                                           \
    }                                                                                        \
    float gme[NK];                                                                           \
    _Pragma("unroll") for (int j = 0; j < NK / 2; ++j) {                                     \
      gme[2 * j] = gm2[j].x;                                                                 \
      gme[2 * j + 1] = gm2[j].y;                                                             \
    }                                                                                        \
    MR_STAMP(2)                                                                              \
    labq[R_] = y[idxq[R_]];                                                                  \
    QL_ISSUE(R_, idxq[R_]);                                                                  \
    idxq[R_] = fetch_row();                                                                  \
    MR_STAMP(6)                                                                              \
    float t[NK / 2];                                                                         \
    {                                                                                        \
      float sa[NK / 2], sb[NK / 2];                                                          \
      _Pragma("unroll") for (int i = 0; i < NK / 2; ++i) {                                   \
        sa[i] = gme[i];                                                                      \
        sb[i] = gme[i + NK / 2];                                                             \
      }                                                                                      \
      swap_batch<32, NK / 2>(sa, sb);                                                        \
      _Pragma("unroll") for (int i = 0; i < NK / 2; ++i) t[i] = sa[i] + sb[i];               \
    }                                                                                        \
    float u[KP];                                                                             \
    {                                                                                        \
      float sa[KP], sb[KP];                                                                  \
      _Pragma("unroll") for (int i = 0; i < KP; ++i) {                                       \
        sa[i] = t[i];                                                                        \
        sb[i] = t[i + KP];                                                                   \
      }                                                                                      \
      swap_batch<16, KP>(sa, sb);                                                            \
      _Pragma("unroll") for (int i = 0; i < KP; ++i) u[i] = sa[i] + sb[i];                   \
    }                                                                                        \
    const int par = s & 1;                                                                   \
    _Pragma("unroll") for (int i = 0; i < KP; ++i) gx[par][w][lane * KP + i] = u[i];         \
    MR_STAMP(3)                                                                              \
    lds_barrier();                 /* B_s: also releases slot R_ to the loaders */          \
    MR_STAMP(4)                                                                              \
    _Pragma("unroll") for (int i = 0; i < KP; ++i) {                                         \
      float gs = gx[par][0][lane * KP + i];                                                  \
      _Pragma("unroll") for (int k = 1; k < MQ_WAVES; ++k) gs += gx[par][k][lane * KP + i];  \
      momentum_step_sel(po[i], bo[i], gs, first, mom, lr, n0 + kj0 + i < N);                 \
    }                                                                                        \
    first = 0;                                                                               \
    {                                                                                        \
      float sa[KP], sb[KP];                                                                  \
      _Pragma("unroll") for (int i = 0; i < KP; ++i) sa[i] = sb[i] = po[i];                  \
      swap_batch<16, KP>(sa, sb);                                                            \
      _Pragma("unroll") for (int i = 0; i < KP; ++i) {                                       \
        t[i] = sa[i];                                                                        \
        t[i + KP] = sb[i];                                                                   \
      }                                                                                      \
      float ga[NK / 2], gb2[NK / 2];                                                         \
      _Pragma("unroll") for (int i = 0; i < NK / 2; ++i) ga[i] = gb2[i] = t[i];              \
      swap_batch<32, NK / 2>(ga, gb2);                                                       \
      _Pragma("unroll") for (int i = 0; i < NK / 2; ++i) {                                   \
        pr[i] = ga[i];                                                                       \
        pr[i + NK / 2] = gb2[i];                                                             \
      }                                                                                      \
    }                                                                                        \
    MR_STAMP(5)                                                                              \
    ++s;                                                                                     \
    if (pf_prog && (s & 3) == 0) mix_publish_progress(pf_prog, s);                           \
  }
  for (;;) {
    QL_STEP(0)
    QL_STEP(1)
  }
#undef QL_STEP
#undef QL_ISSUE
  if (pf_prog) mix_publish_progress(pf_prog, total);
  if (w == 0) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      const int n = n0 + kj0 + i;
      if (n < N) {
        p[n] = po[i];
        buf[n] = bo[i];
      }
    }
    if (lane == 0 && total > 0) *first_flag = 0;
#ifdef FS_MIX_STAMPS
    if (lane < 6) reinterpret_cast<unsigned long long*>(buf + N + 8)[lane] = mr_acc[lane];
#endif
  }
}

template <int NK, int CL, int SPL = quad_split<CL>()>
static void launch_mix_quad(hipStream_t st, const float* Z, const int32_t* y, const int32_t* perms, int N, int C,
                            int nv, int epochs, int Bv, float lr, float mom, float* p, float* buf, int* first,
                            int z_bytes, const MixPrefetch& pf) {
  // ring: DEPTH x CL x NK floats per lane (<= 160), CL*NK/4 + 2 loads per step in the vmcnt window
  constexpr int depth = (3 * CL * NK <= 160 && 3 * (CL * NK / 4 + 2) <= 63) ? 3 : 2;
  const int blocks = pf.prog ? 8 * std::min(pf.h, 31) + 1 : 1;   // helpers: the solver's XCD only
  // softmax on v_exp_f32 / v_rcp_f32 (e / sum) by default: config 2 1.28-1.29 -> 1.21-1.23 us per
  // step (r02s2fx), within the fp32 tolerance of the oracle like every other solver;
  // fs_tuning.mix_exact_softmax: torch's exp(o - m - log(sum)) form with libm expf / logf
  // loader waves (mix_solve_quadl_kernel): config 2's instance (NK = 8, CL = 10) by default,
  // fs_tuning.mix_quad_loaders = -1 off
  // (2 classes in the register ring, 8 through the LDS ring: 0.837-0.839 us per step against
  // 0.851-0.856 with 3 and 0.851-0.874 with 1, profiles/r04/quad_loader_split.txt)
  if constexpr (NK == 8 && CL == 10 && SPL < CL) {
    if (!tuning().mix_exact_softmax && tuning().mix_quad_loaders >= 0) {
      hipLaunchKernelGGL((mix_solve_quadl_kernel<NK, CL, 2>), dim3(blocks), dim3(2 * MQ_WAVES * 64), 0, st, Z, y,
                         perms, N, C, nv, epochs, Bv, lr, mom, p, buf, first, z_bytes, pf.prog, std::min(pf.h, 31),
                         pf.lead);
      return;
    }
  }
  if (!tuning().mix_exact_softmax)
    hipLaunchKernelGGL((mix_solve_quad_kernel<NK, CL, depth, SPL, true>), dim3(blocks), dim3(MQ_WAVES * 64), 0, st, Z,
                       y, perms, N, C, nv, epochs, Bv, lr, mom, p, buf, first, z_bytes, pf.prog, std::min(pf.h, 31),
                       pf.lead);
  else
    hipLaunchKernelGGL((mix_solve_quad_kernel<NK, CL, depth, SPL, false>), dim3(blocks), dim3(MQ_WAVES * 64), 0, st, Z,
                       y, perms, N, C, nv, epochs, Bv, lr, mom, p, buf, first, z_bytes, pf.prog, std::min(pf.h, 31),
                       pf.lead);
}

static bool quad_covers(int N, int C, int Bv, int nv, int epochs) {
  const int64_t zb = (int64_t)nv * C * mix_ldn(N) * 4;
  return Bv <= 16 && (N <= 64 ? C <= 16 : (N <= 128 && C <= 10)) && zb < ((int64_t)1 << 31) && (int64_t)epochs * nv < ((int64_t)1 << 31);
}

static bool mix_solve_quad(hipStream_t st, const float* Z, const int32_t* y, const int32_t* perms, int N, int C,
                           int nv, int epochs, int Bv, float lr, float mom, float* p, float* buf, int* first,
                           const MixPrefetch& pf) {
  if (!quad_covers(N, C, Bv, nv, epochs)) return false;
  const int zb = (int)((int64_t)nv * C * mix_ldn(N) * 4);
  const int nk = N <= 64 ? 4 : 8;
#define MQ_CASE(NK_, CL_)                                                                                    \
  if (nk == NK_ && C <= CL_) {                                                                               \
    launch_mix_quad<NK_, CL_>(st, Z, y, perms, N, C, nv, epochs, Bv, lr, mom, p, buf, first, zb, pf);         \
    return true;                                                                                             \
  }
  MQ_CASE(4, 2) MQ_CASE(4, 4) MQ_CASE(4, 8) MQ_CASE(4, 10) MQ_CASE(4, 16)
  MQ_CASE(8, 2) MQ_CASE(8, 4) MQ_CASE(8, 8) MQ_CASE(8, 10)
#undef MQ_CASE
  return false;
}

// ----------------------------------------------------------------------------
// p-solve, one wave (N <= 16, C <= 4, Bv <= 16: config 1's FedAMW, N = 10, C = 2).  At this
// size a step moves 16 x C x N floats; the workgroup solvers' fixed per-step cost (a barrier,
// LDS partial sums, one batch row per wave) is the whole of their ~1 us.  Here one wave holds
// the step: lane l = (row b = l / 4, class c = l % 4) holds its Z segment (16 clients, 4 float4);
// the logit is a 16-term dot product with p held in SGPRs; the softmax runs over the row's 4
// lanes (DPP); the gradient g_{b,c} * Z segment is reduce-scattered over the wave so that lanes
// 4n .. 4n+3 hold client n's total (lanes.h class_totals), which they use to step p_n and the
// momentum buffer; 16 readlanes return p to SGPRs.  No barrier, no LDS.  The next DEPTH steps'
// rows stream in behind (Z segments and labels, their row indices DEPTH steps earlier still).
// ----------------------------------------------------------------------------
constexpr int MW_DEPTH = 6;

__global__ __launch_bounds__(64) void mix_solve_wave_kernel(const float* __restrict__ Z,
                                                           const int32_t* __restrict__ y,
                                                           const int32_t* __restrict__ perms, int N, int C, int nv,
                                                           int epochs, int Bv, float lr, float mom,
                                                           float* __restrict__ p, float* __restrict__ buf,
                                                           int* __restrict__ first_flag) {
  const int lane = threadIdx.x;
  const int b = lane >> 2, c = lane & 3;
  const int ldN = mix_ldn(N);                      // <= 16
  const int CN = C * ldN;
  const int nbat = (nv + Bv - 1) / Bv;
  const int total = epochs * nbat;
  const int cc = min(c, C - 1);
  int coff[4];                                     // this lane's four float4 of its class segment
#pragma unroll
  for (int k = 0; k < 4; ++k) coff[k] = cc * ldN + min(4 * k, ldN - 4);   // (past ldN: p = 0 there)
  const int mn = lane >> 2;                        // the client this lane steps after the reduce-scatter
  float pr = mn < N ? p[mn] : 0.f;
  float br = mn < N ? buf[mn] : 0.f;
  float sp[16];
#pragma unroll
  for (int n = 0; n < 16; ++n)
    sp[n] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, pr), 4 * n));
  int first = *first_flag;
  // row index of the next step in fetch order (this lane's row; rows past the batch read its
  // first row, their gradient is 0); the cursor stays on the last step at the end
  int fst = 0, fep = 0, fsb = 0;
  auto next_row = [&]() -> int {
    const int bc = min(Bv, nv - fsb * Bv);
    const int r = perms[(int64_t)fep * nv + fsb * Bv + (b < bc ? b : 0)];
    if (fst + 1 < total) {
      ++fst;
      if (++fsb == nbat) {
        fsb = 0;
        ++fep;
      }
    }
    return r;
  };
  float4 zr[MW_DEPTH][4];
  int lab[MW_DEPTH], idx[MW_DEPTH];
#define MW_ISSUE(R_, ROW_)                                                                 \
  {                                                                                        \
    const float* zp_ = Z + (int64_t)(ROW_) * CN;                                           \
    _Pragma("unroll") for (int q_ = 0; q_ < 4; ++q_) zr[R_][q_] = ld4(zp_ + coff[q_]);    \
    lab[R_] = y[(ROW_)];                                                                   \
  }
#pragma unroll
  for (int r0 = 0; r0 < MW_DEPTH; ++r0) {          // steps 0 .. DEPTH-1: rows in flight
    const int r = next_row();
    MW_ISSUE(r0, r);
  }
#pragma unroll
  for (int r0 = 0; r0 < MW_DEPTH; ++r0) idx[r0] = next_row();   // steps DEPTH .. 2 DEPTH-1
  __builtin_amdgcn_s_waitcnt(0x0F70);              // vmcnt(0): the loop inherits only its own order
  int s = 0, csb = 0;
#define MW_STEP(R_)                                                                        \
  {                                                                                        \
    if (s >= total) break;                                                                 \
    const int bc = min(Bv, nv - csb * Bv);                                                 \
    csb = csb + 1 == nbat ? 0 : csb + 1;                                                   \
    float o0 = 0.f, o1 = 0.f;                                                              \
    _Pragma("unroll") for (int k = 0; k < 4; ++k) {                                        \
      o0 += zr[R_][k].x * sp[4 * k + 0];                                                   \
      o1 += zr[R_][k].y * sp[4 * k + 1];                                                   \
      o0 += zr[R_][k].z * sp[4 * k + 2];                                                   \
      o1 += zr[R_][k].w * sp[4 * k + 3];                                                   \
    }                                                                                      \
    const float o = o0 + o1;                                                               \
    const bool real = c < C;                                                               \
    float m = real ? o : -INFINITY;                                                        \
    m = fmaxf(m, xor_get(m, 1, lane));                                                     \
    m = fmaxf(m, xor_get(m, 2, lane));                                                     \
    float e = real ? expf(o - m) : 0.f;                                                    \
    e += xor_get(e, 1, lane);                                                              \
    e += xor_get(e, 2, lane);                                                              \
    const float invb = 1.0f / (float)bc;                                                   \
    const float g = (real && b < bc) ? (c == lab[R_] ? -invb : 0.f) + expf(o - m - logf(e)) * invb : 0.f; \
    float v[16];                                                                           \
    _Pragma("unroll") for (int k = 0; k < 4; ++k) {                                        \
      v[4 * k + 0] = g * zr[R_][k].x;                                                      \
      v[4 * k + 1] = g * zr[R_][k].y;                                                      \
      v[4 * k + 2] = g * zr[R_][k].z;                                                      \
      v[4 * k + 3] = g * zr[R_][k].w;                                                      \
    }                                                                                      \
    const float gp = class_totals<16>(v, lane);                                            \
    /* the slot is consumed: refill it with step s + DEPTH, fetch the rows of s + 2 DEPTH */ \
    MW_ISSUE(R_, idx[R_]);                                                                 \
    idx[R_] = next_row();                          /* step s + 2 DEPTH */                  \
    if (mn < N) momentum_step(pr, br, gp, first, mom, lr);                                 \
    first = 0;                                                                             \
    _Pragma("unroll") for (int n = 0; n < 16; ++n)                                         \
      sp[n] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, pr), 4 * n)); \
    ++s;                                                                                   \
  }
  for (;;) {
    MW_STEP(0) MW_STEP(1) MW_STEP(2) MW_STEP(3) MW_STEP(4) MW_STEP(5)
  }
#undef MW_STEP
#undef MW_ISSUE
  if ((lane & 3) == 0 && mn < N) {
    p[mn] = pr;
    buf[mn] = br;
  }
  if (lane == 0 && total > 0) *first_flag = 0;
}

// ----------------------------------------------------------------------------
// p-solve, one wave for two classes ("bin": N <= 16, C <= 2, Bv <= 16 -- config 1's FedAMW on
// a9a, N = 10, C = 2).  `wave` above gives half its lanes to padding classes and runs its
// softmax on libm; `quad` pays an LDS barrier per step for 4 waves.  Here lane l = (row b = l/4,
// class c = (l/2) & 1, half h = l & 1) holds 8 of the 16 client columns (8h .. 8h+7) of its
// (row, class) segment -- 2 float4 -- and p of those 8 clients in VGPRs:
//   * logit: a packed 8-term dot product plus one DPP add over the half pair (o_0 + o_1 in
//     both lanes: the same bits);
//   * softmax of two classes: the other class's logit by one DPP move, g = rcp(1 + exp(o' - o))
//     on v_exp_f32 / v_rcp_f32 (fs_tuning.mix_exact_softmax = 1: torch's exp(o - m - log(e0 +
//     e1)) on libm), minus the label's one-hot, over the batch size;
//   * gradient: 8 packed products reduce-scattered over row bits 5, 4 (permlane32 / 16 swaps)
//     and 3 (bank-masked DPP adds), then summed over row bit 2 and the class bit, so that lane
//     l ends with client 8h + 4 bit5 + 2 bit4 + bit3's total (4 lanes each, the same bits);
//   * the momentum step there, and the inverse moves (DPP, then the swaps) gather p back to
//     8 clients per lane.
// No LDS, no barrier, no SGPR round trip.  Z through a buffer descriptor (a chunk past ldN or
// a padding class reads zeros), a DEPTH-step register ring; row indices DEPTH steps earlier.
// ----------------------------------------------------------------------------
constexpr int MB_DEPTH = 8;

template <bool FASTX>
__global__ __launch_bounds__(64) void mix_solve_bin_kernel(const float* __restrict__ Z, const int32_t* __restrict__ y,
                                                           const int32_t* __restrict__ perms, int N, int C, int nv,
                                                           int epochs, int Bv, float lr, float mom,
                                                           float* __restrict__ p, float* __restrict__ buf,
                                                           int* __restrict__ first_flag, int z_bytes) {
  static_assert(MB_DEPTH * 4 <= 63, "ring vs the vmcnt window");
  const int lane = threadIdx.x;
  const int b = lane >> 2, c = (lane >> 1) & 1, h = lane & 1;
  const int ldN = mix_ldn(N);                      // <= 16
  const int CN = C * ldN;
  const int nbat = (nv + Bv - 1) / Bv;
  const int total = epochs * nbat;
  const int bc_tail = nv - (nbat - 1) * Bv;
  const float invB = 1.0f / (float)Bv;
  const float invT = 1.0f / (float)bc_tail;
  const bool real = c < C;
  uint32_t lofs[2];                                // byte offsets of the lane's chunks in a row
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int col = 8 * h + 4 * k;
    lofs[k] = (real && col < ldN) ? 4u * (uint32_t)(c * ldN + col) : 0x80000000u;
  }
  // the client this lane holds after the reduce-scatter; p of the lane's 8 dot-product clients
  const int kn = 8 * h + 4 * ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1);
  float po = kn < N ? p[kn] : 0.f;
  float bo = kn < N ? buf[kn] : 0.f;
  float pv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) pv[j] = 8 * h + j < N ? p[8 * h + j] : 0.f;   // p = 0 on padding
  int first = *first_flag;
  const bool b3 = (lane >> 3) & 1;
  const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Z), 0, z_bytes, 0x00020000);
  // fetch cursor: the step whose row indices are read next (stays on the last step at the end)
  int fst = 0, fep = 0, fsb = 0;
  auto fetch_row = [&]() -> int {
    const int base = fep * nv + fsb * Bv;
    const int bc = min(Bv, nv - fsb * Bv);
    const int row = perms[base + (b < bc ? b : 0)];   // rows past the batch: its first (masked)
    if (fst + 1 < total) {
      ++fst;
      if (++fsb == nbat) {
        fsb = 0;
        ++fep;
      }
    }
    return row;
  };
  floatx4 zr[MB_DEPTH][2];
  int idxq[MB_DEPTH], labq[MB_DEPTH];
#define MB_ISSUE(R_, ROW_)                                                                   \
  {                                                                                          \
    const uint32_t ro_ = (uint32_t)(ROW_) * (uint32_t)CN * 4u;                               \
    _Pragma("unroll") for (int k_ = 0; k_ < 2; ++k_) zr[R_][k_] =                            \
        __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(zrs, ro_ + lofs[k_], 0, 0)); \
  }
#pragma unroll
  for (int k = 0; k < MB_DEPTH; ++k) {
    const int row = fetch_row();
    labq[k] = y[row];
    MB_ISSUE(k, row);
  }
#pragma unroll
  for (int k = 0; k < MB_DEPTH; ++k) idxq[k] = fetch_row();
  __builtin_amdgcn_s_waitcnt(0x0F70);              // vmcnt(0): the loop inherits only its own order
  int csb = 0;
  int s = 0;
#define MB_STEP(R_, TAIL_)                                                                   \
  {                                                                                          \
    if (TAIL_ && s >= total) break;                                                          \
    const int bc = min(Bv, nv - csb * Bv);                                                   \
    const float invb = bc == Bv ? invB : invT;                                               \
    csb = csb + 1 == nbat ? 0 : csb + 1;                                                     \
    float2v a2 = {0.f, 0.f};                                                                 \
    _Pragma("unroll") for (int j = 0; j < 8; j += 2) a2 = __builtin_elementwise_fma(          \
        half2(zr[R_][j >> 2], (j >> 1) & 1), float2v{pv[j], pv[j + 1]}, a2);                 \
    const float op = a2.x + a2.y;                                                            \
    const float o = op + dpp<0xB1>(op);              /* the half pair: quad_perm [1,0,3,2] */ \
    const float oo = C > 1 ? dpp<0x4E>(o) : -INFINITY;   /* the other class: [2,3,0,1] */    \
    float sm;                                                                                \
    if constexpr (FASTX) {                                                                   \
      sm = __builtin_amdgcn_rcpf(1.f + __expf(oo - o));                                      \
    } else {                       /* torch's log_softmax backward: exp(o - m - log(sum)) */ \
      const float m = fmaxf(o, oo);                                                          \
      sm = expf(o - m - logf(expf(o - m) + expf(oo - m)));                                   \
    }                                                                                        \
    const float g = (real && b < bc) ? (c == labq[R_] ? -invb : 0.f) + sm * invb : 0.f;      \
    float v[8];                                                                              \
    _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                          \
      float2v t2 = float2v{g, g} * half2(zr[R_][j >> 1], j & 1);                             \
      asm volatile("" : "+v"(t2));                   /* computed here: the slot dies here */ \
      v[2 * j] = t2.x;                                                                       \
      v[2 * j + 1] = t2.y;                                                                   \
    }                                                                                        \
    /* slot consumed: refill with step s + DEPTH, then fetch the rows of s + 2 DEPTH (the   \
       scheduling fence keeps the refill below the slot's last use: one register per slot,   \
       no copies on the loop's back edge) */                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    labq[R_] = y[idxq[R_]];                                                                  \
    MB_ISSUE(R_, idxq[R_]);                                                                  \
    idxq[R_] = fetch_row();                                                                  \
    float t[4];                                                                              \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) t[i] = rs_level<32, true>(v[i], v[i + 4], lane); \
    const float u0 = rs_level<16, true>(t[0], t[2], lane);                                   \
    const float u1 = rs_level<16, true>(t[1], t[3], lane);                                   \
    float gs = rs_bank<8>(u0, u1);                                                           \
    gs = rs_bank<4>(gs, gs);                         /* over row bit 2 */                    \
    gs = gs + dpp<0x4E>(gs);                         /* over the class bit */                \
    if (kn < N) momentum_step(po, bo, gs, first, mom, lr);                                   \
    first = 0;                                                                               \
    /* gather p back: row bit 3 (row_ror:8), then bits 4 and 5 (swaps) */                   \
    const float px = dpp<0x128>(po);                                                         \
    float r4[4];                                                                             \
    gather_pair<16>(b3 ? px : po, r4[0], r4[2]);                                             \
    gather_pair<16>(b3 ? po : px, r4[1], r4[3]);                                             \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) gather_pair<32>(r4[i], pv[i], pv[i + 4]); \
    ++s;                                                                                     \
  }
  // whole ring turns without an exit inside (a break per step gives the loop a latch shared
  // with the exits, where hipcc copies the ring registers and waits for the newest loads),
  // then the last total % DEPTH steps
  for (int it = total / MB_DEPTH; it > 0; --it) {
    MB_STEP(0, false) MB_STEP(1, false) MB_STEP(2, false) MB_STEP(3, false)
    MB_STEP(4, false) MB_STEP(5, false) MB_STEP(6, false) MB_STEP(7, false)
  }
  do {
    MB_STEP(0, true) MB_STEP(1, true) MB_STEP(2, true) MB_STEP(3, true)
    MB_STEP(4, true) MB_STEP(5, true) MB_STEP(6, true)
  } while (false);
#undef MB_STEP
#undef MB_ISSUE
  if ((lane & 6) == 0 && kn < N) {                 // one of the 4 lanes holding client kn
    p[kn] = po;
    buf[kn] = bo;
  }
  if (lane == 0 && total > 0) *first_flag = 0;
}

static bool bin_covers(int N, int C, int Bv, int nv, int epochs) {
  const int64_t zb = (int64_t)nv * C * mix_ldn(N) * 4;
  return N <= 16 && C <= 2 && Bv <= 16 && zb < ((int64_t)1 << 31) && (int64_t)epochs * nv < ((int64_t)1 << 31);
}

// ----------------------------------------------------------------------------
// p-solve, multi-CU form (Bv <= 16, C <= 16, N <= 2048).  One workgroup on one CU cannot
// stream a batch of Z rows faster than ~33 GB/s (gathered rows from the Infinity Cache,
// MI355X_MICROARCH.md "Indexed rows"): at config 2 that is 64 KB per step, ~2 us -- the
// whole cost of the register solver.  Here K workgroups split the CLIENTS: workgroup k owns
// clients [k*S, k*S + S) and reads only that slice of every Z row, so each step moves
// 16*C*S*4 bytes per CU.  The only cross-CU dependence of a step is the logits
// out[b][c] = sum_n p_n Z[v_b][c][n]: every workgroup publishes its 16 x C partial logits
// as 8-byte {tag, value} granules (relaxed agent-scope stores: the data is its own flag,
// cdna_hip_programming.md Guideline 16, R2 form), reads all K partial vectors back and sums
// them in workgroup order -- identical bits everywhere, so every workgroup computes the same
// softmax gradient g[b][c] with no second exchange.  The gradient of its own clients,
// grad_n = sum_{b,c} g[b][c] Z[v_b][c][n], then needs only its own registers (a wave
// reduce-scatter + 4 wave partials through LDS), and the momentum step is local.
//
// Thread t = (row b = t / 16, class slot c = t % 16): 256 threads = 16 rows x 16 slots; slot
// c >= C loads a clamped class and carries g = 0.  The next step's Z slice (S floats per
// thread) is loaded at the top of the step, so it streams while the exchange waits.
// Placement: 8*K workgroups are launched and those with blockIdx % 8 == 0 participate, which
// under round-robin dispatch puts all K on one XCD (the exchange stays inside one L2); any
// other placement changes only speed.  Parity slots (step & 1) of the exchange buffer are
// zeroed before each launch; tags are step + 1.  Every spin is bounded: a timeout sets the
// error word and poisons p with NaN (the kernel still drains).
// ----------------------------------------------------------------------------
constexpr int MC_THREADS = 256;
constexpr int MC_XCDS = 8;
constexpr int MC_KMAX = 32;
constexpr int MC_SLOT = 256;                     // granules per workgroup per parity
constexpr int MC_TOT = 256;                      // hop-2 granules (logit totals) per parity
constexpr unsigned MC_SPIN_LIMIT = 1u << 20;

// spin on one granule until it carries `tag`; false (and the error word set) on a timeout
__device__ __forceinline__ bool mc_wait(const unsigned long long* g, unsigned tag, unsigned long long& out,
                                        unsigned spin_limit, unsigned* err) {
  unsigned spins = 0;
  for (;;) {
    out = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((unsigned)(out >> 32) == tag) return true;
    if (++spins > spin_limit) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
}

// HOPS = 1: every workgroup reads all K partial vectors (16 C K granules per workgroup and
// step).  HOPS = 2: reduce-scatter + all-gather -- value r = b*C + c of the 16 x C logits is
// owned by workgroup r % K, which folds the K partials of its ceil(16C/K) values in workgroup
// order (the same left fold as HOPS = 1, so the same bits) and publishes the totals; every
// workgroup then reads the 16 C totals.  About 2 x 16 C granules per workgroup and step
// instead of 16 C K: at K = 32 the exchange no longer out-reads the Z slice.
// ZAT: where the next step's Z slice is issued -- 0 at the top of the step (it streams while
// the exchange waits, but every poll queues behind it: a hop between streaming CUs costs ~3x
// an idle one, MI355X_MICROARCH.md handoff-1to1), 1 after hop 1 (HOPS = 2: hop 1 runs with
// an empty queue), 2 after the exchange (both hops idle, the slice's latency exposed).
template <int S, int HOPS>
__global__ __launch_bounds__(MC_THREADS) void mix_solve_mc_kernel(const float* __restrict__ Z,
                                                                 const int32_t* __restrict__ y,
                                                                 const int32_t* __restrict__ perms, int N, int C,
                                                                 int nv, int epochs, int Bv, float lr, float mom,
                                                                 float* __restrict__ p, float* __restrict__ buf,
                                                                 int* __restrict__ first_flag,
                                                                 unsigned long long* __restrict__ xbuf,
                                                                 unsigned* __restrict__ err, int K,
                                                                 unsigned spin_limit, unsigned* __restrict__ pf_prog,
                                                                 int pf_h, int pf_lead) {
  static_assert(S == 8 || S == 16 || S == 32 || S == 64, "slice width");
  static_assert(HOPS == 1 || HOPS == 2, "exchange form");
  if (blockIdx.x % MC_XCDS) {
    // the other XCDs' blocks: the first pf_h prefetch the Z rows of the steps ahead into the
    // Infinity Cache (shared by all XCDs; their own L2s are of no use to the solver's XCD)
    const int hidx = (int)blockIdx.x - (int)blockIdx.x / MC_XCDS - 1;
    if (pf_prog && hidx < pf_h) mix_prefetch_helper(Z, perms, N, C, nv, epochs, Bv, hidx, pf_h, pf_lead, pf_prog);
    return;
  }
  constexpr int LPV = 64 / S;                      // lanes per value after the reduce-scatter
  __shared__ __attribute__((aligned(16))) float ps[S];
  __shared__ float gp[MC_THREADS / 64][S];
  __shared__ float part[HOPS == 2 ? 2 * MC_THREADS : 1];   // hop 1: partials of owned values
  const int k = blockIdx.x / MC_XCDS;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int b = t >> 4, c = t & 15;
  const int ldN = mix_ldn(N);
  const int CN = C * ldN;
  const int n_lo = k * S;
  const int nbat = (nv + Bv - 1) / Bv;
  const int total = epochs * nbat;
  const int myn = n_lo + t;                        // client of thread t < S
  float pr = 0.f, br = 0.f;
  if (t < S && myn < N) {
    pr = p[myn];
    br = buf[myn];
  }
  if (t < S) ps[t] = pr;                           // p = 0 on padding clients
  int first = *first_flag;
  // this thread's column offsets inside a row: class min(c, C-1), float4 i of the slice
  // (past ldN: clamped to a valid vector, multiplied by p = 0 and its gradient discarded)
  const int cc = min(c, C - 1);
  int coff[S / 4];
#pragma unroll
  for (int i = 0; i < S / 4; ++i) coff[i] = cc * ldN + min(n_lo + 4 * i, ldN - 4);
  auto row_at = [&](int st) -> int {              // Z row of (step st, row b), clamped
    st = min(st, total - 1);
    const int ep = st / nbat, sb = st - ep * nbat;
    const int bc = min(Bv, nv - sb * Bv);
    return perms[(int64_t)ep * nv + sb * Bv + (b < bc ? b : 0)];
  };
  float4 zc[S / 4];
  int yc, vnext;
  {
    const int v0 = row_at(0);
    const float* zr = Z + (int64_t)v0 * CN;
#pragma unroll
    for (int i = 0; i < S / 4; ++i) zc[i] = ld4(zr + coff[i]);
    yc = y[v0];
    vnext = row_at(1);
  }
  bool dead = false;
  if (spin_limit == 0 && k == 0 && t == 0 && total > 0)   // test knob: report an injected timeout
    __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  lds_barrier();
  for (int st = 0; st < total; ++st) {
    // ---- next step's slice streams behind this step ----
    float4 zn[S / 4];
    int yn = 0;
    auto issue_next = [&]() {
      const float* zr = Z + (int64_t)vnext * CN;
#pragma unroll
      for (int i = 0; i < S / 4; ++i) zn[i] = ld4(zr + coff[i]);
      yn = y[vnext];
    };
    const int vn2 = row_at(st + 2);
    // ---- partial logits of this workgroup's clients ----
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < S / 4; ++i) {
      const float4 pv = *reinterpret_cast<const float4*>(&ps[4 * i]);
      a += zc[i].x * pv.x;
      a += zc[i].y * pv.y;
      a += zc[i].z * pv.z;
      a += zc[i].w * pv.w;
    }
    // ---- exchange: publish, then gather all K partials (workgroup order) ----
    const unsigned tag = (unsigned)st + 1u;
    unsigned long long* slot = xbuf + (int64_t)(st & 1) * K * MC_SLOT;
    const bool real = c < C;
    float o = 0.f;
    if (real)
      __hip_atomic_store(slot + (int64_t)k * MC_SLOT + t,
                         ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(a), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (HOPS == 1) {
      if (real) {
        unsigned long long gr[MC_KMAX];
        unsigned spins = 0;
        for (;;) {
#pragma unroll
          for (int q = 0; q < MC_KMAX; ++q)
            if (q < K) gr[q] = __hip_atomic_load(slot + (int64_t)q * MC_SLOT + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          bool ok = true;
#pragma unroll
          for (int q = 0; q < MC_KMAX; ++q)
            if (q < K) ok = ok && (unsigned)(gr[q] >> 32) == tag;
          if (ok || dead) break;
          if (++spins > spin_limit) {
            dead = true;
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
#pragma unroll
        for (int q = 0; q < MC_KMAX; ++q)
          if (q < K) o += __uint_as_float((unsigned)gr[q]);
      }
    } else {
      // hop 1: this workgroup owns values r = k + K i; thread u loads partner q = u % K's
      // partial of owned value i = u / K (two passes when 16 C + K > 256)
      const int nval = 16 * C;
      const int nown = (nval - k + K - 1) / K;     // values r = k + K i < 16 C
      unsigned long long* tots = xbuf + (int64_t)2 * K * MC_SLOT + (int64_t)(st & 1) * MC_TOT;
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        const int u = t + pass * MC_THREADS;
        const int i = u / K, q = u - (u / K) * K;
        if (i < nown) {
          const int r = k + K * i;
          const int tr = (r / C) * 16 + (r % C);   // thread slot of value r in a partial vector
          unsigned long long gv = 0;
          if (!dead && !mc_wait(slot + (int64_t)q * MC_SLOT + tr, tag, gv, spin_limit, err)) dead = true;
          part[u] = __uint_as_float((unsigned)gv);
        }
      }
      lds_barrier();
      if (t < nown) {                              // fold in workgroup order, publish the total
        float sum = 0.f;
        for (int q = 0; q < K; ++q) sum += part[t * K + q];
        const int r = k + K * t;
        __hip_atomic_store(tots + r, ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(sum),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      // hop 2: every real thread reads the total of its own value
      if (real) {
        unsigned long long gv = 0;
        if (!dead && !mc_wait(tots + (b * C + c), tag, gv, spin_limit, err)) dead = true;
        o = __uint_as_float((unsigned)gv);
      }
    }
    issue_next();
    // ---- softmax-CE gradient of row b (16-lane class groups) ----
    const int sb = st % nbat;
    const int bc = min(Bv, nv - sb * Bv);
    float m = real ? o : -INFINITY;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) m = fmaxf(m, xor_get(m, off, lane));
    float e = real ? expf(o - m) : 0.f;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) e += xor_get(e, off, lane);
    const float lse = logf(e);
    const float invb = 1.0f / (float)bc;
    const float g = (real && b < bc) ? (c == yc ? -invb : 0.f) + expf(o - m - lse) * invb : 0.f;
    // ---- gradient of this workgroup's clients ----
    float v[S];
#pragma unroll
    for (int i = 0; i < S / 4; ++i) {
      v[4 * i + 0] = g * zc[i].x;
      v[4 * i + 1] = g * zc[i].y;
      v[4 * i + 2] = g * zc[i].z;
      v[4 * i + 3] = g * zc[i].w;
    }
    const float tot = class_totals<S>(v, lane);    // lane l: wave sum of v[l / LPV]
    if ((lane & (LPV - 1)) == 0) gp[w][lane / LPV] = tot;
    lds_barrier();
    if (t < S) {
      const float gs = ((gp[0][t] + gp[1][t]) + gp[2][t]) + gp[3][t];
      if (myn < N) momentum_step(pr, br, gs, first, mom, lr);
      ps[t] = pr;
    }
    first = 0;
    lds_barrier();
#pragma unroll
    for (int i = 0; i < S / 4; ++i) zc[i] = zn[i];
    yc = yn;
    vnext = vn2;
    if (pf_prog && k == 0 && ((st + 1) & 3) == 0) mix_publish_progress(pf_prog, st + 1);
  }
  if (pf_prog && k == 0) mix_publish_progress(pf_prog, total);   // releases the helpers
  if (t < S && myn < N) {
    p[myn] = dead ? __int_as_float(0x7fc00000) : pr;
    buf[myn] = br;
  }
  if (k == 0 && t == 0 && total > 0) *first_flag = 0;
}

// caller-owned workspace of the multi-CU solver: [2][K][MC_SLOT] exchange granules (zeroed
// before every launch) followed by a 256-byte error block (sticky: only the caller clears it)
constexpr int64_t MC_ERR_BYTES = 256;

static int64_t mc_xbytes(int K) { return (int64_t)sizeof(unsigned long long) * 2 * (K * MC_SLOT + MC_TOT); }

// exchange form: two hops, except at S = 8 (one) -- r02n, N = 100, C = 10, us per step, one hop /
// two hops (Z issued after the exchange): S = 64 (K = 2) 5.50 / 4.14, S = 32 (K = 4) 4.43 / 2.90,
// S = 16 (K = 7) 3.95 / 2.87, S = 8 (K = 13) 3.25 / 3.79
static int mc_hops(int K, int S) { return (K >= 2 && S >= 16) ? 2 : 1; }

// the exchange kernels' spin bound (fs_tuning.spin_limit) and the injected-timeout test knob
// (the kernels report a timeout at the first exchange when the bound they get is 0)
static unsigned mc_spin_limit() {
  const fs_tuning t = tuning();
  if (t.inject_timeout) return 0u;
  return t.spin_limit ? t.spin_limit : MC_SPIN_LIMIT;
}

// slice width for N clients (0: not covered): S clients per workgroup, K = ceil(ldN / S) <= 32
static int mc_slice(int N) {
  const int ldN = mix_ldn(N);
  for (int s : {8, 16, 32, 64})
    if ((ldN + s - 1) / s <= MC_KMAX && (s > 8 || ldN <= 128)) return s;
  return 0;
}

static bool mc_covers(int N, int C, int Bv) { return mc_slice(N) != 0 && C <= 16 && Bv <= 16; }

static int mix_solve_mc(hipStream_t st, const float* Z, const int32_t* y, const int32_t* perms, int N, int C, int nv,
                        int epochs, int Bv, float lr, float mom, float* p, float* buf, int* first, void* d_ws,
                        int64_t ws_bytes, MixPrefetch pf) {
  if (!mc_covers(N, C, Bv)) return 1;            // not covered
  const int S = mc_slice(N);
  const int K = (mix_ldn(N) + S - 1) / S;
  const int64_t xbytes = mc_xbytes(K);
  if (!d_ws || ws_bytes < xbytes + MC_ERR_BYTES)
    return fail(FS_EINVAL, "fs_mix_solve: workspace too small (see fs_mix_solve_ws_bytes)");
  unsigned long long* ws = reinterpret_cast<unsigned long long*>(d_ws);
  unsigned* err = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(d_ws) + ws_bytes - MC_ERR_BYTES);
  hipError_t e = hipMemsetAsync(ws, 0, (size_t)xbytes, st);
  if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_mix_solve: ") + hipGetErrorString(e));
  const unsigned spin_limit = mc_spin_limit();
  const dim3 grid(MC_XCDS * K), block(MC_THREADS);
  const int hops = mc_hops(K, S);
  // the next Z slice is issued after the exchange -- r02i, us per step, (hops, issued at the top /
  // after hop 1 / after the exchange): N = 1000, C = 10, K = 32: (1, top) 6.61, (2, top) 6.03,
  // (2, hop 1) 5.45, (2, exchange) 5.44; N = 300, C = 4, K = 19: 4.33 / 4.34 / 4.08 / 3.38
  if (pf.prog) pf.h = std::min(pf.h, (MC_XCDS - 1) * K);   // helpers: the grid's other-XCD blocks
#define MC_CASE(S_, H_)                                                                                       \
  if (S == S_ && hops == H_)                                                                                  \
    hipLaunchKernelGGL((mix_solve_mc_kernel<S_, H_>), grid, block, 0, st, Z, y, perms, N, C, nv, epochs, Bv, lr,  \
                       mom, p, buf, first, ws, err, K, spin_limit, pf.prog, pf.h, pf.lead);
  MC_CASE(8, 1) MC_CASE(16, 2) MC_CASE(32, 2) MC_CASE(64, 2)
#undef MC_CASE
  return 0;
}

// ----------------------------------------------------------------------------
// p-solve, multi-CU quarter-wave form "qmc" (Bv <= 16, 128 < N <= 16 * 16 * NK, C <= CL):
// the quarter-wave layout on K <= 16 workgroups of 16*NK clients each (N = 1000: K = 16 of 64),
// all on one XCD.  A workgroup computes its clients' partial logits, publishes them (the
// 16 x C row/class values, 8-byte {tag, value} granules) and reads the K partials of every
// value back -- ONE hop -- summing them in workgroup order, so every workgroup holds the
// bitwise-same logits, softmax and CE gradient; the gradient of its own clients, the
// momentum step and p stay local (no second hop).  Its 16 x C x 16NK Z values per step come
// from L2, where H helper workgroups on the same XCD prefetch the rows of the next steps
// (fs_tuning.mix_prefetch; by default 24, at most the 32 - K CUs left on the XCD, 6 steps
// ahead).  Spins are bounded; a timeout sets the error
// word and poisons p with NaN.
// ----------------------------------------------------------------------------
constexpr int QMC_KMAX = 16;

template <int NK, int CL, int DEPTH, int SPL>
__global__ __launch_bounds__(MQ_WAVES * 64) void mix_solve_qmc_kernel(
    const float* __restrict__ Z, const int32_t* __restrict__ y, const int32_t* __restrict__ perms, int N, int C,
    int nv, int epochs, int Bv, float lr, float mom, float* __restrict__ p, float* __restrict__ buf,
    int* __restrict__ first_flag, int z_bytes, unsigned long long* __restrict__ xbuf, unsigned* __restrict__ err,
    int K, unsigned spin_limit, unsigned* __restrict__ pf_prog, int pf_h, int pf_lead, int zL, int zR,
    int poll_delay) {
  static_assert(NK == 4 || NK == 8, "clients per lane");
  static_assert(CL >= 1 && CL <= 16, "classes");
  static_assert(DEPTH * (CL * NK / 4 + 2) <= 63, "ring vs the vmcnt window");
  if (blockIdx.x % MC_XCDS) return;
  const int bk = blockIdx.x / MC_XCDS;
  if (bk >= K) {                                   // L2 prefetch helpers on the solvers' XCD
    if (pf_prog && bk - K < pf_h)
      mix_prefetch_helper(Z, perms, N, C, nv, epochs, Bv, bk - K, pf_h, pf_lead, pf_prog, zL, zR);
    return;
  }
  const int k = bk;
  constexpr int NV4 = NK / 4;
  constexpr int KP = NK / 4;
  __shared__ __attribute__((aligned(16))) float gx[2][MQ_WAVES][64 * KP];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r = lane & 15;
  const int brow = MQ_WAVES * w + q;
  const int ldN = mix_ldn(N);                      // = zR * zL
  const int CN = C * zL;                           // floats per row segment
  const int nbat = (nv + Bv - 1) / Bv;
  const int total = epochs * nbat;
  const int bc_tail = nv - (nbat - 1) * Bv;
  const float invB = 1.0f / (float)Bv;
  const float invT = 1.0f / (float)bc_tail;
  const int n0 = k * 16 * NK + NK * r;             // this lane's first client (global index)
  float pr[NK];
#pragma unroll
  for (int j = 0; j < NK; ++j) pr[j] = n0 + j < N ? p[n0 + j] : 0.f;
  const int kj0 = (q >> 1) * (NK / 2) + (q & 1) * (NK / 4);
  float po[KP], bo[KP];
#pragma unroll
  for (int i = 0; i < KP; ++i) {
    const int n = n0 + kj0 + i;
    po[i] = n < N ? p[n] : 0.f;
    bo[i] = n < N ? buf[n] : 0.f;
  }
  int first = *first_flag;
  // Z layout: zR blocks [n_val][C][zL] (client n = block n / zL, column n % zL; the standard
  // layout is one block of ldN); a lane's 4-client chunks never straddle a block (zL % 4 == 0)
  uint32_t lofs[NV4];                              // chunks past ldN: out of range (zeros, no access)
#pragma unroll
  for (int h = 0; h < NV4; ++h) {
    const int n = n0 + 4 * h;
    lofs[h] = n < ldN ? 4u * ((uint32_t)(n / zL) * (uint32_t)nv * (uint32_t)CN + (uint32_t)(n % zL)) : 0x80000000u;
  }
  int sofs[CL];
#pragma unroll
  for (int c = 0; c < CL; ++c) sofs[c] = __builtin_amdgcn_readfirstlane(4 * min(c, C - 1) * zL);
  const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Z), 0, z_bytes, 0x00020000);
  int fst = 0, fep = 0, fsb = 0;
  auto fetch_row = [&]() -> int {
    const int base = fep * nv + fsb * Bv;
    const int bcf = min(Bv, nv - fsb * Bv);
    const int row = perms[base + (brow < bcf ? brow : 0)];
    if (fst + 1 < total) {
      ++fst;
      if (++fsb == nbat) {
        fsb = 0;
        ++fep;
      }
    }
    return row;
  };
  floatx4 zr[DEPTH][CL][NV4];
  int idxq[DEPTH], labq[DEPTH];
#define QM_ISSUE(R_, ROW_, C0_, C1_)                                                         \
  {                                                                                          \
    const uint32_t ro_ = (uint32_t)(ROW_) * (uint32_t)CN * 4u;                               \
    _Pragma("unroll") for (int c = (C0_); c < (C1_); ++c) {                                      \
      _Pragma("unroll") for (int h = 0; h < NV4; ++h) zr[R_][c][h] = __builtin_bit_cast(     \
          floatx4, __builtin_amdgcn_raw_buffer_load_b128(zrs, ro_ + lofs[h], sofs[c], 0));   \
    }                                                                                        \
  }
#pragma unroll
  for (int kk = 0; kk < DEPTH; ++kk) {
    const int row = fetch_row();
    labq[kk] = y[row];
    QM_ISSUE(kk, row, 0, CL);
  }
#pragma unroll
  for (int kk = 0; kk < DEPTH; ++kk) idxq[kk] = fetch_row();
  __builtin_amdgcn_s_waitcnt(0x0F70);
  bool dead = false;
  if (spin_limit == 0 && k == 0 && tid == 0 && total > 0)   // test knob: report an injected timeout
    __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int csb = 0;
  int s = 0;
  int late_row = 0;
#ifdef FS_MIX_STAMPS
  unsigned long long mr_acc[6] = {0, 0, 0, 0, 0, 0}, mr_prev = 0;
#endif
#define QM_STEP(R_)                                                                          \
  {                                                                                          \
    if (s >= total) break;                                                                   \
    MR_STAMP(0)                                                                              \
    const int bc = min(Bv, nv - csb * Bv);                                                   \
    csb = csb + 1 == nbat ? 0 : csb + 1;                                                     \
    float v[16];                                                                             \
    {              /* packed pairs (v_pk_fma_f32): even and odd clients summed apart, then    \
                      joined; the classes' chains interleaved (independent accumulators) */   \
      float2v a2[CL];                                                                        \
      _Pragma("unroll") for (int c = 0; c < CL; ++c) a2[c] = float2v{0.f, 0.f};              \
      _Pragma("unroll") for (int j = 0; j < NK; j += 2) {                                    \
        _Pragma("unroll") for (int c = 0; c < CL; ++c) a2[c] = __builtin_elementwise_fma(   \
            half2(zr[R_][c][j >> 2], (j >> 1) & 1), float2v{pr[j], pr[j + 1]}, a2[c]);      \
      }                                                                                      \
      _Pragma("unroll") for (int c = 0; c < 16; ++c) v[c] = c < CL ? a2[c].x + a2[c].y : 0.f; \
    }                                                                                        \
    rs_banks_8_4(v);                                                                         \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) v[i] = rs_pair(v[i], v[i + 2], 2, lane);   \
    const float opart = rs_pair(v[0], v[1], 1, lane);   /* this workgroup's share */         \
    MR_STAMP(1)                                                                              \
    const bool real = r < C;                                                                 \
    /* one hop: publish, read the K partials, fold in workgroup order */                     \
    const unsigned tag = (unsigned)s + 1u;                                                   \
    unsigned long long* slot = xbuf + (int64_t)(s & 1) * K * MC_SLOT;                        \
    const int gi = brow * 16 + r;                                                            \
    float o = 0.f;                                                                           \
    if (real) {                                                                              \
      __hip_atomic_store(slot + (int64_t)k * MC_SLOT + gi,                                   \
                         ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(opart), \
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);                        \
      unsigned long long gr[QMC_KMAX];                                                       \
      /* wait ~64 poll_delay cycles before the first poll: the partners publish about then, \
         and the polls of 16 workgroups x 4 waves on the same lines clog the L2 while they \
         are early (profiles/r04/qmc_poll_delay_sweep.txt) */                                \
      for (int d_ = 0; d_ < poll_delay; ++d_) __builtin_amdgcn_s_sleep(1);                   \
      _Pragma("unroll") for (int kk = 0; kk < QMC_KMAX; ++kk)                                \
        if (kk < K) gr[kk] = __hip_atomic_load(slot + (int64_t)kk * MC_SLOT + gi, __ATOMIC_RELAXED, \
                                               __HIP_MEMORY_SCOPE_AGENT);                    \
      /* re-poll every partner still missing in ONE batch per round trip (round 3 spun on   \
         them one after another: a round trip per late partner) */                           \
      for (unsigned spins = 0; !dead;) {                                                     \
        bool miss = false;                                                                   \
        _Pragma("unroll") for (int kk = 0; kk < QMC_KMAX; ++kk)                              \
          miss |= kk < K && (unsigned)(gr[kk] >> 32) != tag;                                 \
        if (!miss) break;                                                                    \
        if (++spins > spin_limit) {                                                          \
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);           \
          dead = true;                                                                       \
          break;                                                                             \
        }                                                                                    \
        _Pragma("unroll") for (int kk = 0; kk < QMC_KMAX; ++kk)                              \
          if (kk < K && (unsigned)(gr[kk] >> 32) != tag)                                     \
            gr[kk] = __hip_atomic_load(slot + (int64_t)kk * MC_SLOT + gi, __ATOMIC_RELAXED,  \
                                       __HIP_MEMORY_SCOPE_AGENT);                            \
      }                                                                                      \
      _Pragma("unroll") for (int kk = 0; kk < QMC_KMAX; ++kk)                                \
        if (kk < K) o += __uint_as_float((unsigned)gr[kk]);                                  \
    }                                                                                        \
    MR_STAMP(2)                                                                              \
    /* the late classes of step s - 1 + DEPTH, behind the hop (its polls queue behind nothing) */ \
    if constexpr (SPL < CL) {                                                                \
      if (s > 0) QM_ISSUE((R_ + DEPTH - 1) % DEPTH, late_row, SPL, CL);                      \
    }                                                                                        \
    const float m = row16_max(real ? o : -INFINITY);                                         \
    const float invb = bc == Bv ? invB : invT;                                               \
    const float e = real ? __expf(o - m) : 0.f;                                              \
    const float ssum = row16_all<false>(e);                                                  \
    const float g = (real && brow < bc) ? (r == labq[R_] ? -invb : 0.f) + e * __builtin_amdgcn_rcpf(ssum) * invb \
                                        : 0.f;                                               \
    float gv[CL];                  /* g of class c of this row: DPP row broadcast */         \
    _Pragma("unroll") for (int c = 0; c < CL; ++c) gv[c] = row_get(g, c);                    \
    float2v gm2[NK / 2];                                                                     \
    _Pragma("unroll") for (int j = 0; j < NK / 2; ++j) gm2[j] = float2v{0.f, 0.f};           \
    _Pragma("unroll") for (int c = 0; c < CL; ++c) {                                         \
      _Pragma("unroll") for (int j = 0; j < NK / 2; ++j) gm2[j] = __builtin_elementwise_fma( \
          float2v{gv[c], gv[c]}, half2(zr[R_][c][j >> 1], j & 1), gm2[j]);                   \
    }                                                                                        \
    float gme[NK];                                                                           \
    _Pragma("unroll") for (int j = 0; j < NK / 2; ++j) {                                     \
      gme[2 * j] = gm2[j].x;                                                                 \
      gme[2 * j + 1] = gm2[j].y;                                                             \
    }                                                                                        \
    MR_STAMP(3)                                                                              \
    labq[R_] = y[idxq[R_]];                                                                  \
    QM_ISSUE(R_, idxq[R_], 0, SPL);                                                          \
    late_row = idxq[R_];                                                                     \
    idxq[R_] = fetch_row();                                                                  \
    float t[NK / 2];               /* = rs_level<32> / <16>, one pad per level */            \
    {                                                                                        \
      float sa[NK / 2], sb[NK / 2];                                                          \
      _Pragma("unroll") for (int i = 0; i < NK / 2; ++i) {                                   \
        sa[i] = gme[i];                                                                      \
        sb[i] = gme[i + NK / 2];                                                             \
      }                                                                                      \
      swap_batch<32, NK / 2>(sa, sb);                                                        \
      _Pragma("unroll") for (int i = 0; i < NK / 2; ++i) t[i] = sa[i] + sb[i];               \
    }                                                                                        \
    float u[KP];                                                                             \
    {                                                                                        \
      float sa[KP], sb[KP];                                                                  \
      _Pragma("unroll") for (int i = 0; i < KP; ++i) {                                       \
        sa[i] = t[i];                                                                        \
        sb[i] = t[i + KP];                                                                   \
      }                                                                                      \
      swap_batch<16, KP>(sa, sb);                                                            \
      _Pragma("unroll") for (int i = 0; i < KP; ++i) u[i] = sa[i] + sb[i];                   \
    }                                                                                        \
    const int par = s & 1;                                                                   \
    _Pragma("unroll") for (int i = 0; i < KP; ++i) gx[par][w][lane * KP + i] = u[i];         \
    MR_STAMP(4)                                                                              \
    lds_barrier();                                                                           \
    MR_STAMP(5)                                                                              \
    _Pragma("unroll") for (int i = 0; i < KP; ++i) {                                         \
      float gs = gx[par][0][lane * KP + i];                                                  \
      _Pragma("unroll") for (int kk = 1; kk < MQ_WAVES; ++kk) gs += gx[par][kk][lane * KP + i]; \
      momentum_step_sel(po[i], bo[i], gs, first, mom, lr, n0 + kj0 + i < N);                 \
    }                                                                                        \
    first = 0;                                                                               \
    {                              /* = gather_pair<16> / <32>, one pad per level */         \
      float sa[KP], sb[KP];                                                                  \
      _Pragma("unroll") for (int i = 0; i < KP; ++i) sa[i] = sb[i] = po[i];                  \
      swap_batch<16, KP>(sa, sb);                                                            \
      _Pragma("unroll") for (int i = 0; i < KP; ++i) {                                       \
        t[i] = sa[i];                                                                        \
        t[i + KP] = sb[i];                                                                   \
      }                                                                                      \
      float ga[NK / 2], gb2[NK / 2];                                                         \
      _Pragma("unroll") for (int i = 0; i < NK / 2; ++i) ga[i] = gb2[i] = t[i];              \
      swap_batch<32, NK / 2>(ga, gb2);                                                       \
      _Pragma("unroll") for (int i = 0; i < NK / 2; ++i) {                                   \
        pr[i] = ga[i];                                                                       \
        pr[i + NK / 2] = gb2[i];                                                             \
      }                                                                                      \
    }                                                                                        \
    MR_STAMP(6)                                                                              \
    ++s;                                                                                     \
    if (pf_prog && k == 0) mix_publish_progress(pf_prog, s);   /* every step: helpers pace on it */ \
  }
  for (;;) {
    QM_STEP(0)
    if constexpr (DEPTH > 1) QM_STEP(1)
    if constexpr (DEPTH > 2) QM_STEP(2)
  }
#undef QM_STEP
#undef QM_ISSUE
  if (pf_prog && k == 0) mix_publish_progress(pf_prog, total);
  if (w == 0) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      const int n = n0 + kj0 + i;
      if (n < N) {
        p[n] = dead ? __int_as_float(0x7fc00000) : po[i];
        buf[n] = bo[i];
      }
    }
    if (k == 0 && lane == 0 && total > 0) *first_flag = 0;
#ifdef FS_MIX_STAMPS
    if (k == 0 && lane < 6) reinterpret_cast<unsigned long long*>(buf + N + 8)[lane] = mr_acc[lane];
#endif
  }
}

// clients per lane: 4 (64 per workgroup) wherever K = ceil(N / 64) <= 16 workgroups, else 8
// (C <= 10 only).  Round 4 (profiles/r04/qmc_lane_ab*.txt, us per step, 8 vs 4): N = 1000
// C = 10 3.60-3.71 vs 3.30; N = 300 3.00 vs 2.50; N = 520 3.23 vs 2.73 -- half the gather per CU
// outweighs the hop's 16 partners since the hop re-polls all missing partners at once (round 2,
// polling them one after another, measured the two the same).  fs_tuning.mix_qmc_lane_clients
// forces one.
static int qmc_nk(int N, int C) {
  const int f = tuning().mix_qmc_lane_clients;
  if (C > 10 || f == 4) return 4;
  if (f == 8) return 8;
  return (mix_ldn(N) + 63) / 64 <= QMC_KMAX ? 4 : 8;
}

// s_sleep(1) units before a step's first poll (fs_tuning.mix_poll_delay: 0 = by shape, -1 =
// none, n > 0 = n).  By shape from the sweeps (profiles/r04/qmc_poll_delay*.txt, us per step,
// none / best, at helper lead 6): N = 1000, C = 10 (K = 16) 3.24 / 2.73 at 14 (12-16 within 1 %);
// N = 1000, C = 4 2.86 / 2.28 at 8 (2.49 at 16); N = 300 2.41 / 1.95 at 8; N = 520 2.68 / 2.07 at 8.
// At lead 8 (the qmc default since) the K = 16 optimum moved to 10: 2.48 vs 2.58 us at 14
// (profiles/r04/qmc_delay_lead_grid.txt).
static int qmc_poll_delay(int K, int C) {
  const int t = tuning().mix_poll_delay;
  if (t < 0) return 0;
  if (t > 0) return t;
  return (K >= 12 && C >= 8) ? 10 : 8;
}

static bool qmc_covers(int N, int C, int Bv, int nv, int epochs) {
  const int64_t zb = (int64_t)nv * C * mix_ldn(N) * 4;
  const int nk = qmc_nk(N, C);
  return Bv <= 16 && N > 128 && C <= 16 && (mix_ldn(N) + 16 * nk - 1) / (16 * nk) <= QMC_KMAX &&
         zb < ((int64_t)1 << 31) && (int64_t)epochs * nv < ((int64_t)1 << 31);
}

// the calling thread's last multi-CU launch layout (fs_mix_solve_last_layout): workgroups K and
// clients per lane NK of the qmc solver (0, 0 after any other solver)
static thread_local int t_last_k = 0, t_last_nk = 0;

// 1: not covered; 0: launched; < 0: error
static int mix_solve_qmc(hipStream_t st, const float* Z, const int32_t* y, const int32_t* perms, int N, int C, int nv,
                         int epochs, int Bv, float lr, float mom, float* p, float* buf, int* first, void* d_ws,
                         int64_t ws_bytes, MixPrefetch pf, int zR = 1) {
  if (!qmc_covers(N, C, Bv, nv, epochs)) return 1;
  const int zL = mix_ldn(N) / zR;
  const int nk = qmc_nk(N, C);
  const int K = (mix_ldn(N) + 16 * nk - 1) / (16 * nk);
  const int64_t xbytes = mc_xbytes(K);
  if (!d_ws || ws_bytes < xbytes + MC_ERR_BYTES)
    return fail(FS_EINVAL, "fs_mix_solve: workspace too small (see fs_mix_solve_ws_bytes)");
  unsigned long long* ws = reinterpret_cast<unsigned long long*>(d_ws);
  unsigned* err = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(d_ws) + ws_bytes - MC_ERR_BYTES);
  hipError_t e = hipMemsetAsync(ws, 0, (size_t)xbytes, st);
  if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_mix_solve: ") + hipGetErrorString(e));
  const unsigned spin_limit = mc_spin_limit();
  const int h = pf.prog ? std::min(pf.h, 32 - K) : 0;   // the solvers' XCD has 32 CUs
  const dim3 grid(MC_XCDS * (K + h)), block(MQ_WAVES * 64);
  const int zb = (int)((int64_t)nv * C * mix_ldn(N) * 4);
  const int pd = qmc_poll_delay(K, C);
  t_last_k = K;
  t_last_nk = nk;
  if (nk == 8)
    hipLaunchKernelGGL((mix_solve_qmc_kernel<8, 10, 2, quad_split<10>()>), grid, block, 0, st, Z, y, perms, N, C, nv,
                       epochs, Bv, lr, mom, p, buf, first, zb, ws, err, K, spin_limit, pf.prog, h, pf.lead, zL, zR,
                       pd);
  else if (C <= 10)
    hipLaunchKernelGGL((mix_solve_qmc_kernel<4, 10, 3, quad_split<10>()>), grid, block, 0, st, Z, y, perms, N, C, nv,
                       epochs, Bv, lr, mom, p, buf, first, zb, ws, err, K, spin_limit, pf.prog, h, pf.lead, zL, zR,
                       pd);
  else
    hipLaunchKernelGGL((mix_solve_qmc_kernel<4, 16, 2, quad_split<16>()>), grid, block, 0, st, Z, y, perms, N, C, nv,
                       epochs, Bv, lr, mom, p, buf, first, zb, ws, err, K, spin_limit, pf.prog, h, pf.lead, zL, zR,
                       pd);
  return 0;
}

}  // namespace fs

using namespace fs;

static thread_local int t_last_solver = 0;

extern "C" int fs_mix_solve_last_mode(void) { return t_last_solver; }

extern "C" int fs_mix_solve_last_layout(int* workgroups, int* lane_clients) {
  FS_REQUIRE(workgroups && lane_clients, "null pointer");
  const bool q = t_last_solver == FS_SOLVER_QMC;
  *workgroups = q ? fs::t_last_k : 0;
  *lane_clients = q ? fs::t_last_nk : 0;
  return FS_OK;
}

extern "C" int64_t fs_mix_solve_ws_bytes(int N, int C, int Bv) {
  if (N < 1) return MC_ERR_BYTES;
  const int S = mc_slice(N);
  const int K = S ? (mix_ldn(N) + S - 1) / S : 0;
  const int64_t mc = mc_covers(N, C, Bv) ? mc_xbytes(K) : 0;
  const int64_t qmc = mc_xbytes((mix_ldn(N) + 63) / 64);   // the larger K of either lane width
  return std::max(mc, (N > 128 && C <= 16 && Bv <= 16) ? qmc : (int64_t)0) + MC_ERR_BYTES;
}

// L2 prefetch helper setup of fs_mix_solve / fs_mix_solve_blocked (0, or an error status)
static int mix_prefetch_setup(const fs_tuning& tune, bool use_quad, bool use_qmc, int N, int C, int n_val, void* d_ws,
                              int64_t ws_bytes, hipStream_t st0, MixPrefetch& pf) {
  // L2 prefetch helpers (fs_tuning.mix_prefetch: 0 = by solver, -1 = none, n): 4 for the
  // quarter-wave solver, whose gather they speed up (r02s2k, 1.42-1.47 -> 1.35-1.43 us per step
  // at config 2), 16 for qmc, none for the others, where they measured nothing; they run
  // mix_prefetch_lead (0: 16) steps ahead; the progress word lives in the error block (byte 128)
  // (quad: only when Z outgrows the L2s -- at config 1's 0.6 MB the helpers cost 3 %, r02s2c1)
  const bool z_big = (int64_t)n_val * C * mix_ldn(N) * 4 > ((int64_t)16 << 20);
  const int h = tune.mix_prefetch > 0 ? tune.mix_prefetch
                : (tune.mix_prefetch < 0 ? 0 : ((use_quad && z_big) ? 4 : (use_qmc ? 24 : 0)));
  // default lead: 16 steps for the quarter-wave solver; 8 for qmc, whose helpers (round 4:
  // LDS-DMA pieces, the solver's progress published every step) keep a few steps of rows in
  // the XCD's 4 MB L2 ahead of the solver -- at config 5 before the first-poll delay, 24
  // helpers, leads 4 / 6 / 8 / 12: 3.85 / 3.62 / 3.76 / 3.81 us per step, none: 4.40
  // (profiles/r04/mix_solve_helper_sweep.txt); with it (16 helpers at K = 16), leads 6 / 8 / 10
  // / 12 / 16: 2.70-2.72 / 2.58 / 2.62-2.63 / 2.65 / 2.66, and at N = 300 1.96 for 6 and 8
  // (profiles/r04/qmc_lead_sweep.txt); at N = 800 (K = 13) 8 is faster (2.33 vs 2.38-2.40), at
  // N = 520 (K = 9) 6 (2.08 vs 2.18-2.24, profiles/r04/qmc_lead_sweep2.txt): 8 from K = 12, as
  // the first-poll delay's step (qmc_poll_delay)
  int qmc_k = 0;
  if (use_qmc) {
    const int lw = 16 * qmc_nk(N, C);
    qmc_k = (mix_ldn(N) + lw - 1) / lw;
  }
  const int lead = tune.mix_prefetch_lead > 0 ? tune.mix_prefetch_lead : (use_qmc ? (qmc_k >= 12 ? 8 : 6) : 16);
  if (h > 0 && d_ws && ws_bytes >= MC_ERR_BYTES) {
    pf.prog = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(d_ws) + ws_bytes - MC_ERR_BYTES + 128);
    pf.h = h;
    pf.lead = lead;
    hipError_t e = hipMemsetAsync(pf.prog, 0, sizeof(unsigned), st0);
    if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_mix_solve: ") + hipGetErrorString(e));
  }
  return 0;
}

extern "C" int fs_mix_solve(const float* d_Z, const int32_t* d_labels, const int32_t* d_perms, int N, int C,
                            int n_val, int epochs, int Bv, float lr_p, float momentum, float* d_p, float* d_buf,
                            int* d_first, void* d_ws, int64_t ws_bytes, void* stream) {
  FS_REQUIRE(N >= 1 && C >= 1 && n_val >= 1 && epochs >= 0, "bad sizes");
  FS_REQUIRE(Bv >= 1 && Bv <= MS_MAXB, "valid batch size must be in [1, 64]");
  FS_REQUIRE(d_Z && d_labels && d_perms && d_p && d_buf && d_first, "null pointer");
  hipStream_t st0 = reinterpret_cast<hipStream_t>(stream);
  // solver choice: by shape, or forced by fs_tuning.mix_solver (tests, diagnostics; a forced
  // solver that does not cover the shape falls through to the next one)
  const fs_tuning tune = tuning();
  const int want = tune.mix_solver;
  const bool aut = want == FS_SOLVER_AUTO;
  // two classes, N <= 16 (config 1): the one-wave binary solver; one wave where it measured
  // fastest (N <= 16, C = 3..4: 0.616 vs 0.62 us per step); else the quarter-wave solver
  const bool auto_wave = N <= 16 && C >= 3 && C <= 4 && Bv <= 16;
  const bool use_quad = (aut && !auto_wave && quad_covers(N, C, Bv, n_val, epochs)) || want == FS_SOLVER_QUAD;
  // the multi-CU quarter-wave solver where the single-workgroup register solvers end (N > 256)
  const bool use_qmc = want == FS_SOLVER_QMC || (aut && N > 256 && qmc_covers(N, C, Bv, n_val, epochs));
  MixPrefetch pf{nullptr, 0, 0};
  if (int rc = mix_prefetch_setup(tune, use_quad, use_qmc, N, C, n_val, d_ws, ws_bytes, st0, pf)) return rc;
  // by shape: one wave for N <= 16, C <= 4; the quarter-wave solver (+ L2 prefetch helpers) for
  // N <= 64, C <= 16 or N <= 128, C <= 10; the register solvers where an instance covers the
  // shape (no cross-CU exchange: ~1-2.5 us per step); for N > 256 the multi-CU quarter-wave
  // solver (one exchange hop per step; 3.9 us at N = 1000, C = 10) where it covers, else the
  // multi-CU solver (two hops, ~4-7 us per step, 7-11x the single-workgroup staged / global
  // solvers at N = 200..1000, C = 10); else those.
  if (((aut && N <= 16 && C <= 2) || want == FS_SOLVER_BIN) && bin_covers(N, C, Bv, n_val, epochs)) {
    const int zb = (int)((int64_t)n_val * C * mix_ldn(N) * 4);
    if (!tune.mix_exact_softmax)
      hipLaunchKernelGGL(mix_solve_bin_kernel<true>, dim3(1), dim3(64), 0, st0, d_Z, d_labels, d_perms, N, C, n_val,
                         epochs, Bv, lr_p, momentum, d_p, d_buf, d_first, zb);
    else
      hipLaunchKernelGGL(mix_solve_bin_kernel<false>, dim3(1), dim3(64), 0, st0, d_Z, d_labels, d_perms, N, C, n_val,
                         epochs, Bv, lr_p, momentum, d_p, d_buf, d_first, zb);
    t_last_solver = FS_SOLVER_BIN;
    FS_LAUNCH_CHECK();
    return FS_OK;
  }
  if (((aut && auto_wave) || want == FS_SOLVER_WAVE) && N <= 16 && C <= 4 && Bv <= 16) {
    hipLaunchKernelGGL(mix_solve_wave_kernel, dim3(1), dim3(64), 0, st0, d_Z, d_labels, d_perms, N, C, n_val, epochs,
                       Bv, lr_p, momentum, d_p, d_buf, d_first);
    t_last_solver = 6;
    FS_LAUNCH_CHECK();
    return FS_OK;
  }
  if (use_quad &&
      mix_solve_quad(st0, d_Z, d_labels, d_perms, N, C, n_val, epochs, Bv, lr_p, momentum, d_p, d_buf, d_first, pf)) {
    t_last_solver = 8;
    FS_LAUNCH_CHECK();
    return FS_OK;
  }
  // form 2 (two rows per wave) where it measured faster: N in (128, 256], NK = 4 (2.0 vs 4.1 us
  // per step at N = 256, C = 4); below that the one-row form is as fast or faster (r02g)
  if (((aut && N > 128) || want == FS_SOLVER_REG2) &&
      mix_solve_reg2(st0, d_Z, d_labels, d_perms, N, C, n_val, epochs, Bv, lr_p, momentum, d_p, d_buf, d_first)) {
    t_last_solver = 5;
    FS_LAUNCH_CHECK();
    return FS_OK;
  }
  if ((aut || want == FS_SOLVER_REG) &&
      mix_solve_reg(st0, d_Z, d_labels, d_perms, N, C, n_val, epochs, Bv, lr_p, momentum, d_p, d_buf, d_first,
                    pf)) {
    t_last_solver = 1;
    FS_LAUNCH_CHECK();
    return FS_OK;
  }
  if (use_qmc) {
    const int rc = mix_solve_qmc(st0, d_Z, d_labels, d_perms, N, C, n_val, epochs, Bv, lr_p, momentum, d_p, d_buf,
                                 d_first, d_ws, ws_bytes, pf);
    if (rc < 0) return rc;
    if (rc == 0) {
      t_last_solver = 9;
      FS_LAUNCH_CHECK();
      return FS_OK;
    }
  }
  if (aut || want == FS_SOLVER_MC) {
    const int rc = mix_solve_mc(st0, d_Z, d_labels, d_perms, N, C, n_val, epochs, Bv, lr_p, momentum, d_p, d_buf,
                                d_first, d_ws, ws_bytes, pf);
    if (rc < 0) return rc;
    if (rc == 0) {
      t_last_solver = 2;
      FS_LAUNCH_CHECK();
      return FS_OK;
    }
  }
  {
    // LDS-staged solver: two batches of Z rows + p, buf and the wave partials must fit
    const int CN4 = C * mix_ldn(N);
    const size_t lds2 = sizeof(float) * (2 * (size_t)Bv * CN4 + 2 * (size_t)N + (size_t)MS_WAVES * N);
    if (want != FS_SOLVER_GLOBAL && N <= 64 * MS2_NK && C <= 16 && lds2 <= 150 * 1024 && (size_t)Bv * (CN4 / 4) <= (size_t)MS_THREADS * MS2_PER_THREAD) {
      const void* kfn = reinterpret_cast<const void*>(&mix_solve_staged_kernel<16>);
      if (lds2 > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2);
        if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_mix_solve: ") + hipGetErrorString(e));
      }
      hipLaunchKernelGGL(mix_solve_staged_kernel<16>, dim3(1), dim3(MS_THREADS), lds2, st0, d_Z, d_labels, d_perms, N,
                         C, n_val, epochs, Bv, lr_p, momentum, d_p, d_buf, d_first);
      t_last_solver = 3;
      FS_LAUNCH_CHECK();
      return FS_OK;
    }
  }
  const size_t lds = sizeof(float) * (2 * (size_t)N + 2 * MS_MAXB * (size_t)C) + sizeof(int) * 2 * MS_MAXB;
  FS_REQUIRE(lds <= 160 * 1024, "N too large for the LDS-resident mixture solve");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mix_solve_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_mix_solve: ") + hipGetErrorString(e));
  }
  hipLaunchKernelGGL(mix_solve_kernel, dim3(1), dim3(MS_THREADS), lds, st, d_Z, d_labels, d_perms, N, C, n_val,
                     epochs, Bv, lr_p, momentum, d_p, d_buf, d_first);
  t_last_solver = 4;
  FS_LAUNCH_CHECK();
  return FS_OK;
}

extern "C" int fs_mix_solve_blocked_covers(int N, int C, int n_val, int epochs, int Bv) {
  const fs_tuning tune = tuning();
  const bool forced_other = tune.mix_solver != FS_SOLVER_AUTO && tune.mix_solver != FS_SOLVER_QMC;
  return !forced_other && N >= 1 && C >= 1 && n_val >= 1 && epochs >= 0 && qmc_covers(N, C, Bv, n_val, epochs) &&
         (tune.mix_solver == FS_SOLVER_QMC || N > 256);
}

extern "C" int fs_mix_solve_blocked(const float* d_Z, int blocks, const int32_t* d_labels, const int32_t* d_perms,
                                    int N, int C, int n_val, int epochs, int Bv, float lr_p, float momentum, float* d_p,
                                    float* d_buf, int* d_first, void* d_ws, int64_t ws_bytes, void* stream) {
  FS_REQUIRE(N >= 1 && C >= 1 && n_val >= 1 && epochs >= 0, "bad sizes");
  FS_REQUIRE(blocks >= 1 && N % (4 * blocks) == 0, "N must be a multiple of 4 * blocks");
  FS_REQUIRE(Bv >= 1 && Bv <= MS_MAXB, "valid batch size must be in [1, 64]");
  FS_REQUIRE(d_Z && d_labels && d_perms && d_p && d_buf && d_first, "null pointer");
  hipStream_t st0 = reinterpret_cast<hipStream_t>(stream);
  const fs_tuning tune = tuning();
  if (!fs_mix_solve_blocked_covers(N, C, n_val, epochs, Bv))
    return fail(FS_EUNSUPPORTED, "fs_mix_solve_blocked: the rank-blocked Z layout is read by the qmc solver only "
                                 "(N > 256, C <= 16, Bv <= 16); use fs_mix_solve on the standard layout");
  MixPrefetch pf{nullptr, 0, 0};
  if (int rc = mix_prefetch_setup(tune, false, true, N, C, n_val, d_ws, ws_bytes, st0, pf)) return rc;
  const int rc = mix_solve_qmc(st0, d_Z, d_labels, d_perms, N, C, n_val, epochs, Bv, lr_p, momentum, d_p, d_buf,
                               d_first, d_ws, ws_bytes, pf, blocks);
  if (rc < 0) return rc;
  if (rc != 0) return fail(FS_EUNSUPPORTED, "fs_mix_solve_blocked: shape not covered");
  t_last_solver = FS_SOLVER_QMC;
  FS_LAUNCH_CHECK();
  return FS_OK;
}
