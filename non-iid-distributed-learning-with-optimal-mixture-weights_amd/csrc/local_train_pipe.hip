// Pipelined split-client local training ("pipe" form, ABI 14, G | FS_G_PIPE): a GROUP of G
// workgroups trains one client at a time, each owning a 16-tile slice of the feature
// dimension -- the split form's arithmetic (local_train_split.hip) in the split form's order,
// so the two agree BITWISE -- with each step's hand-off pipelined by ROW TILE.
//
// Same math as train_loop (/root/reference/functions/tools.py:177-215).  The split form runs a
// step as one chain: forward (all 32 rows) -> S1 -> publish -> poll -> S2 -> softmax -> S3 ->
// backward, so the partners' round trip and the softmax run with the MFMA pipe and the row
// stream idle (round-4 stamps: ~6k of ~20k cycles at config 2).  The batch's two 16-row tiles
// are independent up to the gradient sum, so here:
//
//   F0 (forward, rows 0-15) -> B1a -> publish rt0 -> F1 (forward, rows 16-31) -> B1b ->
//   publish rt1 -> poll rt0 -> image -> next rows rt0 -> softmax rt0 -> K0 (backward, rows
//   0-15) -> poll rt1 -> next rows rt1 -> softmax rt1 -> K1 (backward, rows 16-31) + update
//
// rt0's round trip runs under F1, rt1's under K0 (the polls are issued after a whole MFMA
// phase and are normally fresh at once), and the next step's rows stream from the image write
// on (rt0) and from K0's end on (rt1) instead of only inside the backward.
//   * every wave computes the softmax of all 16 rows of a tile itself, in registers, in the
//     backward's operand layout (lane (class, lg) holds rows 4 kk + lg of the tile, kk = 0..3:
//     exactly the g values its backward MFMAs take), from the own slice's partial logits (an
//     LDS transpose of the 8 wave partials, summed in wave order) plus the partners' granules
//     it polls itself (G - 1 partners x 4 per lane) -- no S2 / S3 barrier, no LDS gbuf;
//   * two barriers per step (one per row tile: the wave partials); the LDS image is
//     wave-private (each wave reads back only its own tiles), so it needs none;
//   * the same {tag, value} granule hand-off as the split form (cdna_hip_programming.md
//     Guideline 16, R2: relaxed agent-scope store / load, the data is its own flag), the
//     partner sum in slice order with the own partial at position g, every spin bounded.
// Covered shapes: full slices (ld = 1024 G: 16 tiles per workgroup, 2 per wave), 16 < B <= 32,
// C <= 16, no FedProx anchor (FedAvg, FedAMW's ridge-regularised local training: configs 2, 4
// and 5).  The bitwise match with the split form is tested (tests/test_gpu_pipe.py).
#include <type_traits>

#include "common.h"
#include "eval_rows.h"
#include "lanes.h"
#include "split_common.h"

namespace fs {

constexpr int PP_WAVES = 8;
constexpr int PP_THREADS = PP_WAVES * 64;
constexpr int PP_TPW = 2;                 // 64-column tiles per wave (the slice is 16 tiles)
constexpr int PP_NTS = PP_WAVES * PP_TPW;
constexpr int PP_RS = PP_NTS * 64 + 8;    // LDS image row stride (floats)
constexpr int PP_NR = 32;                 // batch rows (two 16-row tiles)
constexpr int PP_SZ = 520;                // granules per (group, parity, slice): [rt][kk][lane] + 2 norms
constexpr int PP_ZS = 20;                 // transposed partial-logit block: floats per class (16 + pad)
constexpr int PP_ERR_BYTES = 256;

// In-loop loads are inline asm (tagged as the pair form's: `; pr-row`, `; pr-idx`, `; pr-poll`),
// invisible to hipcc's vmcnt bookkeeping -- which, merging the poll retry loop and the client
// start's weight reload into the step, drained the whole row stream before the forward and
// inside the backward -- and their waits are counted by hand from the fixed per-step issue
// pattern below; every destination is named "+v" (`; pr-own`) after the wait that retires it,
// and scripts/asm_audit.py checks the built code object for any touch of a destination in
// between (cdna_hip_programming.md 5.7 item 1, form ii).
template <int OFF>
__device__ __forceinline__ void pp_ld4(floatx4& d, const float* p) {
  asm volatile("global_load_dwordx4 %0, %1, off offset:%2 ; pr-row" : "=v"(d) : "v"(p), "n"(OFF) : "memory");
}
__device__ __forceinline__ void pp_ld1(int& d, const int32_t* p) {
  asm volatile("global_load_dword %0, %1, off ; pr-idx" : "=v"(d) : "v"(p) : "memory");
}
__device__ __forceinline__ void pp_poll(unsigned long long& d, const unsigned long long* p) {
  asm volatile("global_load_dwordx2 %0, %1, off sc1 ; pr-poll" : "=v"(d) : "v"(p) : "memory");
}
template <int N>
__device__ __forceinline__ void pp_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" : : "n"(N) : "memory");
}
template <typename T>
__device__ __forceinline__ void pp_own(T& x) {
  asm volatile("; pr-own %0" : "+v"(x));
}

template <int G, bool NRM>
__global__ __launch_bounds__(PP_THREADS, 1) void local_train_pipe_kernel(LTParams P, SplitWS X) {
  constexpr int NW = PP_WAVES, TPW = PP_TPW, RS = PP_RS, NC = 16;
  constexpr int GP = G > 1 ? G - 1 : 1;          // partners
  // wave partial logits, transposed: zpt[w][rt][class * ZS + 4 lg + kk] = the partial of row
  // 16 rt + 4 kk + lg -- one ds_read_b128 per wave gives a lane its four rows of the tile
  __shared__ __attribute__((aligned(16))) float zpt[NW][2][NC * PP_ZS];
  __shared__ int labw[NW][2][PP_NR];       // wave-private copies of the step's labels (by parity)
  __shared__ float wred[NW][2];            // ||W - W_a||^2 (always 0 here), ||W||^2 of the wave's slice
  extern __shared__ __attribute__((aligned(16))) float xs_dyn[];   // [32][RS] batch slice image

  const int tid = (int)threadIdx.x, lane = tid & 63, l16 = lane & 15, lg = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t ld = P.ld;
  const int C = P.C, B = P.B, E = P.E;

  // block -> (group, slice), fused evaluation blocks: as the split form
  const int nb = gridDim.x - P.fuse_E;
  if ((int)blockIdx.x >= nb) {
    eval_persistent<PP_WAVES>(P.fuse_phi, P.ld, P.fuse_y, P.fuse_n, P.W_start, P.C, (int)blockIdx.x - nb, P.fuse_E,
                              xs_dyn, P.fuse_part);
    return;
  }
  int lin;
  if (P.chained) {
    if (blockIdx.x % 8) return;
    lin = blockIdx.x / 8;
  } else {
    lin = blockIdx.x;
    if (nb % 8 == 0) lin = (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8;
  }
  const int ng = X.ngroups;
  const int grp = lin / G, g = lin % G;
  if (grp >= ng) return;
  const int T = P.chained ? P.N : (P.N + ng - 1) / ng;
  const int t0 = PP_NTS * g;                     // the host guarantees ld = 1024 G
  const float* start = P.W_start;
  unsigned long long* xb = X.xbuf + (int64_t)grp * 2 * G * PP_SZ;
  const floatx4 zero4 = floatx4{0.f, 0.f, 0.f, 0.f};

  // ---- weights of this slice in registers: lane (c, lg) holds W[c][64 T + 16 q + 4 lg + e] ----
  floatx4 wr[TPW][4];
  // (classes >= C read class C - 1's row -- every load unconditional -- and are zeroed)
  auto wsrc = [&]() {
    int64_t b = (int64_t)min(l16, C - 1) * ld + 64 * t0 + 4 * lg + 64 * w;
    asm volatile("" : "+v"(b));
    return start + b;
  };
  auto wnorm = [&]() {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (l16 >= C) wr[i][q] = zero4;
        s += wr[i][q][0] * wr[i][q][0] + wr[i][q][1] * wr[i][q][1] + wr[i][q][2] * wr[i][q][2] +
             wr[i][q][3] * wr[i][q][3];
      }
    return wave_sum_dpp(s, lane);
  };
  // the round-start model as counted loads, drained at once (client starts only)
  auto load_start = [&]() {
    const float* src = wsrc();
    pp_ld4<0>(wr[0][0], src); pp_ld4<64>(wr[0][1], src); pp_ld4<128>(wr[0][2], src); pp_ld4<192>(wr[0][3], src);
    pp_ld4<2048>(wr[1][0], src); pp_ld4<2112>(wr[1][1], src); pp_ld4<2176>(wr[1][2], src);
    pp_ld4<2240>(wr[1][3], src);
    pp_wait<0>();
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) pp_own(wr[i][q]);
    return wnorm();
  };
  auto wbase = [&]() {
    int64_t b = (int64_t)l16 * ld + 64 * t0 + 4 * lg;
    asm volatile("" : "+v"(b));
    return b;
  };
  auto store_w = [&](float* Wj) {
    const int64_t base = wbase();
    if (l16 < C)
#pragma unroll
      for (int i = 0; i < TPW; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          st4(Wj + base + 64 * (w + NW * i) + 16 * q, make_float4(wr[i][q][0], wr[i][q][1], wr[i][q][2], wr[i][q][3]));
  };
  const float nw0 = load_start();
  if (lane == 0) { wred[w][0] = 0.f; wred[w][1] = nw0; }

  // ---- rows: lane (l16, lg) holds row 16 rt + l16, columns 64 T + 16 q + 4 lg .. +3 ----
  floatx4 xf[TPW][2][4];
  int pn[2], pi[2], lb[2];
  int64_t prow0 = 0;
  bool pvalid = false;
  SpCur lc;
  bool lc_ok = sp_seek<true>(lc, P, grp, ng, T, 0);
  // the next step's row indices: 2 counted loads, issued whether or not there is a next step
  // (then from a valid dummy address) so every step issues the same pattern
  auto fetch_rows = [&]() {
    const int e_ = lc_ok ? lc.st / lc.nbat : 0, s_ = lc_ok ? lc.st - e_ * lc.nbat : 0;
    const int b0_ = s_ * B, bc_ = lc_ok ? min(B, lc.n - b0_) : 1;
    const int32_t* pp_ = lc_ok ? P.perms + (int64_t)E * lc.row0 + (int64_t)e_ * lc.n + b0_ : P.perms;
    prow0 = lc_ok ? lc.row0 : 0;
    pvalid = lc_ok;
    pp_ld1(pi[0], pp_ + (l16 < bc_ ? l16 : 0));
    pp_ld1(pi[1], pp_ + (16 + l16 < bc_ ? 16 + l16 : 0));
  };
  auto take_rows = [&]() {                       // (after the wait that retires pi)
    pp_own(pi[0]);
    pp_own(pi[1]);
    // (no next step: keep the current rows -- row 0 before the first -- rather than an index read
    // from the dummy address, which need not hold a row of this launch)
    pn[0] = pvalid ? (int)(prow0 + pi[0]) : pn[0];
    pn[1] = pvalid ? (int)(prow0 + pi[1]) : pn[1];
  };
  auto issue_labels = [&]() {
    pp_ld1(lb[0], P.labels + pn[0]);
    pp_ld1(lb[1], P.labels + pn[1]);
  };
  auto issue_rows = [&](int rt) {
    const float* src = P.phi + (int64_t)pn[rt] * ld + 64 * t0 + 4 * lg + 64 * w;
    pp_ld4<0>(xf[0][rt][0], src); pp_ld4<64>(xf[0][rt][1], src); pp_ld4<128>(xf[0][rt][2], src);
    pp_ld4<192>(xf[0][rt][3], src);
    pp_ld4<2048>(xf[1][rt][0], src); pp_ld4<2112>(xf[1][rt][1], src); pp_ld4<2176>(xf[1][rt][2], src);
    pp_ld4<2240>(xf[1][rt][3], src);
  };
  // prologue: the first step's labels and rows, the second step's indices; all landed
  pn[0] = pn[1] = 0;
  fetch_rows();
  pp_wait<0>();
  take_rows();
  issue_labels();
  issue_rows(0);
  issue_rows(1);
  if (lc_ok) lc_ok = sp_advance<true>(lc, P, grp, ng, T);
  fetch_rows();
  pp_wait<0>();
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    pp_own(lb[rt]);
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) pp_own(xf[i][rt][q]);
  }
  take_rows();
  lds_barrier();

  auto flush_empty = [&](int ka, int kb) {
    for (int k = ka; k < kb; ++k) {
      const int j = sp_client<true>(P, grp, ng, k);
      if (j < 0) continue;
      float* Wj = P.W_out + (int64_t)j * C * ld;
      if (P.chained) {
        store_w(Wj);
      } else {
        const int64_t base = wbase();
        if (l16 < C)
#pragma unroll
          for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int64_t off = base + 64 * (w + NW * i) + 16 * q;
              st4(Wj + off, ld4(start + off));
            }
      }
      if (g == 0 && tid == 0) P.loss[j] = 0.0;
    }
  };

  // Per step every wave issues, in this order (counted vector-memory operations):
  //   [client start: 8 weight loads, drained at once]  1 publish store (rt0)  NRM norm store
  //   1 publish store (rt1)  P0 polls (rt0: 4 (G-1) + NRM (G-1))  2 label loads  8 row loads (next
  //   step, rt0)  P1 polls (rt1: 4 (G-1))  8 row loads (next step, rt1)  2 index loads
  // -- so at the forward of rt0 its rows (issued one step ago) have P1 + 8 + 2 operations behind
  // them, the rows of rt1 2 + 1 + NRM, the indices 1 + NRM + 1 + P0, the rt0 polls 2 + 8, the
  // rt1 polls 8.  A re-poll drains everything (vmcnt(0)); other extra operations (client-end
  // stores, spills) only make a wait stricter.
  constexpr int P0 = 4 * (G - 1) + (NRM ? G - 1 : 0), P1 = 4 * (G - 1);
  constexpr int W_F0 = P1 + 8 + 2, W_F1 = 2 + 1 + (NRM ? 1 : 0), W_IDX = 1 + (NRM ? 1 : 0) + 1 + P0;
  constexpr int W_POLL0 = 2 + 8, W_POLL1 = 8;

  SpCur cc;
  bool cc_ok = sp_seek<true>(cc, P, grp, ng, T, 0);
  flush_empty(0, cc_ok ? cc.k : T);
  unsigned gs = 0;
  bool dead = false;
  double lsum = 0.0;
  const int rblk = 4 * (l16 & 3) + (l16 >> 2);
  unsigned long long pl[4][GP];
  unsigned long long pnrm[GP];
  for (; cc_ok; ++gs) {
    const int st = cc.st, n = cc.n, nbat = cc.nbat;
    if (st == 0) {
      if (!P.chained && gs > 0) {
        (void)load_start();
        if (lane == 0) { wred[w][0] = 0.f; wred[w][1] = nw0; }
      } else if (lane == 0) {
        wred[w][0] = 0.f;
      }
      lsum = 0.0;
    }
    const int e = st / nbat, s = st - e * nbat;
    const int bc = min(B, n - s * B);
    const int par = gs & 1;
    const unsigned tag32 = X.tag_base + gs + 1u;
    const unsigned long long tag = (unsigned long long)tag32 << 32;
    unsigned long long* slot = xb + (int64_t)par * G * PP_SZ;

    // ---- forward of one row tile; its wave partial goes to LDS transposed ----
    auto forward = [&](int rt) {
      floatx4 a = zero4;
#pragma unroll
      for (int i = 0; i < TPW; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) a = mfma4(xf[i][rt][q][e4], wr[i][q][e4], a);
      // a[j] = partial logit of (row 16 rt + 4 lg + j, class l16)
#pragma unroll
      for (int j = 0; j < 4; ++j) zpt[w][rt][l16 * PP_ZS + 4 * j + lg] = a[j];
    };
    // ---- the own slice's partials of one tile (wave order) ----
    auto own_sum = [&](int rt) {
      float4 p[NW];
#pragma unroll
      for (int i = 0; i < NW; ++i) p[i] = ld4(&zpt[i][rt][l16 * PP_ZS + 4 * lg]);
      floatx4 v = zero4;
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        v[0] += p[i].x; v[1] += p[i].y; v[2] += p[i].z; v[3] += p[i].w;
      }
      return v;
    };
    // (waves w and w + 4 publish the same component kk = w & 3: one unconditional store each)
    auto publish = [&](int rt, const floatx4& v) {
      const int kk = w & 3;
      const float x = kk == 0 ? v[0] : (kk == 1 ? v[1] : (kk == 2 ? v[2] : v[3]));
      __hip_atomic_store(slot + (int64_t)g * PP_SZ + rt * 256 + kk * 64 + lane, tag | __float_as_uint(x),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // ---- polls: the G - 1 partners' granules of this lane's four rows of a tile ----
    auto poll = [&](int rt) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int k = 0; k < G - 1; ++k) {
          const int h = k + (k >= g ? 1 : 0);
          pp_poll(pl[kk][k], slot + (int64_t)h * PP_SZ + rt * 256 + kk * 64 + lane);
        }
      if (NRM && rt == 0)
#pragma unroll
        for (int k = 0; k < G - 1; ++k) {
          const int h = k + (k >= g ? 1 : 0);
          pp_poll(pnrm[k], slot + (int64_t)h * PP_SZ + 512 + (lane & 1));
        }
    };
    auto own_polls = [&](int rt) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int k = 0; k < G - 1; ++k) pp_own(pl[kk][k]);
      if (NRM && rt == 0)
#pragma unroll
        for (int k = 0; k < G - 1; ++k) pp_own(pnrm[k]);
    };
    unsigned spins = 0;
    // (call after the counted wait and the own statements of the first poll; a stale partner
    // re-polls everything and drains the queue)
    auto wait_poll = [&](int rt) {
      if (X.spin_limit == 0 && gs == 0 && lane == 0)      // test knob: report an injected timeout
        __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int k = 0; k < G - 1; ++k) ok &= (l16 >= C) | ((unsigned)(pl[kk][k] >> 32) == tag32);
        if (NRM && rt == 0)
#pragma unroll
          for (int k = 0; k < G - 1; ++k) ok &= (unsigned)(pnrm[k] >> 32) == tag32;
        if (__all(ok)) break;
        if (dead || ++spins > X.spin_limit) {
          if (lane == 0) __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          dead = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        poll(rt);
        pp_wait<0>();
        own_polls(rt);
      }
    };
    // the slice-order sum (own partial at position g): every partner gets the same bits
    auto slice_sum = [&](float own, int kk) {
      float sum = 0.f;
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float pv = 0.f;
#pragma unroll
        for (int k = 0; k < G - 1; ++k)
          if (k + (k >= g ? 1 : 0) == h) pv = __uint_as_float((unsigned)pl[kk][k]);
        sum += (h == g) ? own : pv;
      }
      return sum;
    };
    // ---- softmax of one tile in the backward's operand layout ----
    const float invb = 1.0f / (float)bc;
    float gB[8], cep[8];
    auto softmax = [&](int rt, const floatx4& own) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int r = 16 * rt + 4 * kk + lg;
        const float z0 = slice_sum(own[kk], kk);
        const bool valid = r < bc && l16 < C;
        const float z = valid ? z0 : 0.f;
        float m = valid ? z : -INFINITY;
#pragma unroll
        for (int off = NC / 2; off > 0; off >>= 1) m = fmaxf(m, xor_get(m, off, lane));
        const float ex = valid ? __expf(z - m) : 0.f;
        float se = ex;
#pragma unroll
        for (int off = NC / 2; off > 0; off >>= 1) se += xor_get(se, off, lane);
        float gv = 0.f, ce = 0.f;
        if (valid) {
          const bool isy = l16 == labw[w][par][r];
          gv = (isy ? -invb : 0.f) + ex * __builtin_amdgcn_rcpf(se) * invb;
          if (isy) ce -= z - m - __logf(se);
        }
        gB[4 * rt + kk] = gv;
        cep[4 * rt + kk] = ce;
      }
    };

    // ================= row tile 0: forward, publish =================
    pp_wait<W_F0>();                                // this step's rt0 rows and labels landed
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) pp_own(lb[rt]);
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) pp_own(xf[i][0][q]);
    if (lg == 0) {
      labw[w][par][l16] = lb[0];
      labw[w][par][16 + l16] = lb[1];
    }
    forward(0);
    lds_barrier();                                  // B1a: wave partials of rt0 (and the norms)
    const floatx4 own0 = own_sum(0);
    float nown[2] = {0.f, 0.f};
    if (NRM) {
#pragma unroll
      for (int i = 0; i < NW; ++i) { nown[0] += wred[i][0]; nown[1] += wred[i][1]; }
    }
    publish(0, own0);
    if (NRM && lane < 2)
      __hip_atomic_store(slot + (int64_t)g * PP_SZ + 512 + lane, tag | __float_as_uint(nown[lane & 1]),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ================= row tile 1: forward (rt0's round trip runs under it), publish ========
    pp_wait<W_F1>();                                // this step's rt1 rows landed
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) pp_own(xf[i][1][q]);
    forward(1);
    lds_barrier();                                  // B1b
    const floatx4 own1 = own_sum(1);
    publish(1, own1);
    poll(0);
    pp_wait<W_IDX>();                               // the next step's row indices landed
    take_rows();
    // image of this wave's tiles for the backward (wave-private: no barrier); then the next
    // step's labels and row-tile-0 rows stream from here on, behind the polls
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          st4(xs_dyn + img_off(rt * 16 + l16, RS, w + NW * i, 4 * q + lg),
              make_float4(xf[i][rt][q][0], xf[i][rt][q][1], xf[i][rt][q][2], xf[i][rt][q][3]));
    // (the image has read xf before the loads below refill it)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    issue_labels();
    issue_rows(0);
    pp_wait<W_POLL0>();
    own_polls(0);
    wait_poll(0);
    float wn2 = 0.f;
    if (NRM) {
      // ||W||^2 at the start of this step: slice-order sum (lane 1; lane 0 holds ||W - W_a||^2)
      float ns = 0.f;
      const float mine = (lane & 1) ? nown[1] : nown[0];
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float pv = 0.f;
#pragma unroll
        for (int k = 0; k < G - 1; ++k)
          if (k + (k >= g ? 1 : 0) == h) pv = __uint_as_float((unsigned)pnrm[k]);
        ns += (h == g) ? mine : pv;
      }
      wn2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ns), 1));
    }
    softmax(0, own0);

    // ================= backward: image rows 4 kk + lg, kk = 0..7 =================
    floatx4 ga[TPW][4];
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) ga[i][e4] = zero4;
    auto bwd = [&](int kk0) {
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        const int Tl = w + NW * i;
        const float* ib0 = xs_dyn + lg * RS + 64 * Tl + 4 * (rblk ^ lg);
        const float* ib1 = xs_dyn + lg * RS + 64 * Tl + 4 * (rblk ^ (lg + 4));
#pragma unroll
        for (int kk = kk0; kk < kk0 + 4; ++kk) {
          const float4 x = ld4(((kk & 1) ? ib1 : ib0) + 4 * kk * RS);
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) ga[i][e4] = mfma4(comp(x, e4), gB[kk], ga[i][e4]);
        }
      }
    };
    bwd(0);                                         // K0 (rt1's round trip runs under it)
    poll(1);
    issue_rows(1);
    pp_wait<W_POLL1>();
    own_polls(1);
    wait_poll(1);
    softmax(1, own1);
    if (g == 0 && w == 0 && e == E - 1) {
      // the loss as the split form sums it: per 4-row group (split wave 4 rt + kk) a DPP wave
      // sum, then the eight in row order
      float ce = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) ce += wave_sum_dpp(cep[k], lane);
      if (lane == 0) {
        float loss = ce / (float)bc;
        if (P.reg) loss = loss + P.lam * sqrtf(wn2);
        lsum += (double)loss * (double)bc;
      }
    }
    bwd(4);                                         // K1
    // ---- update of the register-resident slice ----
    {
      const float sr = (P.reg && wn2 > 0.f) ? P.lam / sqrtf(wn2) : 0.f;
      const float lr = P.lr;
      if (l16 < C) {
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) {
              const float wc = wr[i][q][e4];
              float gr = ga[i][e4][q];
              if (P.reg) gr = gr + wc * sr;
              wr[i][q][e4] = wc - lr * gr;
            }
      }
    }
    if (NRM) {
      // ridge: ||W||^2 of the updated slice in the update's order (the split form's bits)
      float nwn = 0.f;
#pragma unroll
      for (int i = 0; i < TPW; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) nwn += wr[i][q][e4] * wr[i][q][e4];
      nwn = wave_sum_dpp(nwn, lane);
      if (lane == 0) { wred[w][0] = 0.f; wred[w][1] = nwn; }
    }
    if (lc_ok) lc_ok = sp_advance<true>(lc, P, grp, ng, T);
    fetch_rows();
    if (st == cc.steps - 1) {
      store_w(P.W_out + (int64_t)cc.j * C * ld);
      if (g == 0 && tid == 0) P.loss[cc.j] = lsum / (double)n;
    }
    const int kprev = cc.k;
    cc_ok = sp_advance<true>(cc, P, grp, ng, T);
    flush_empty(kprev + 1, cc_ok ? cc.k : T);
  }
  pp_wait<0>();                                     // nothing of ours is in flight at the exit
}

bool pipe_fits(int C, int B, int NT, int G, int prox) {
  // (G = 8 holds 4 x 7 polled granules per lane: ~200 VGPRs spilled; G = 16 more -- not built)
  if (!(G == 2 || G == 4)) return false;
  return !prox && C >= 1 && C <= 16 && B > 16 && B <= 32 && NT == PP_NTS * G;
}

static int64_t pipe_xbuf_bytes(int ngroups, int G) { return (int64_t)ngroups * 2 * G * PP_SZ * 8; }

int pipe_groups(int N, int G, int chained, int cus) { return chained ? 1 : std::max(1, std::min(N, cus / G)); }

int64_t pipe_ws_bytes(int N, int G, int chained, int cus) {
  return pipe_xbuf_bytes(pipe_groups(N, G, chained, cus), G) + PP_ERR_BYTES;
}

template <int G, bool NRM>
static void launch_pipe_s(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&local_train_pipe_kernel<G, NRM>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((local_train_pipe_kernel<G, NRM>), dim3(grid), dim3(PP_THREADS), lds, st, P, X);
}

template <int G>
static void launch_pipe_g(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  if (P.reg) launch_pipe_s<G, true>(P, X, grid, lds, st);
  else launch_pipe_s<G, false>(P, X, grid, lds, st);
}

unsigned split_spin_bound();   // local_train_split.hip: fs_tuning.spin_limit / the test knob

int launch_local_train_pipe(const LTParams& P, int G, void* ws, int64_t ws_bytes, hipStream_t st) {
  const int NT = (int)(P.ld >> 6);
  if (!pipe_fits(P.C, P.B, NT, G, P.prox))
    return fail(FS_EUNSUPPORTED, "fs_local_train: the pipe form needs ld = 1024 G (G = 2 or 4), 16 < B <= 32, "
                                 "C <= 16 and no prox term");
  const int cus = device_cus();
  if (cus <= 0) return fail(FS_EHIP, "fs_local_train: no device");
  if (G > cus) return fail(FS_EUNSUPPORTED, "fs_local_train: G exceeds the CU count");
  const int ng = pipe_groups(P.N, G, P.chained, cus);
  const int64_t xbytes = pipe_xbuf_bytes(ng, G);
  if (!ws || ws_bytes < xbytes + PP_ERR_BYTES) return fail(FS_EINVAL, "fs_local_train: workspace too small");
  char* base = reinterpret_cast<char*>(ws);
  SplitWS X;
  X.xbuf = reinterpret_cast<unsigned long long*>(base);
  X.err = reinterpret_cast<unsigned*>(base + ws_bytes - PP_ERR_BYTES);
  X.SZ = PP_SZ;
  X.ngroups = ng;
  X.spin_limit = split_spin_bound();
  X.poll_delay = 0;
  X.stamps = nullptr;
  // hand-off tags by launch generation (as the split form, local_train_split.hip)
  const int64_t groups_clients = P.chained ? P.N : (P.N + ng - 1) / ng;
  const bool long_launch = P.max_client_steps <= 0 || P.max_client_steps * groups_clients >= (1 << 20) - 1;
  const unsigned gen = exchange_generation(ws, long_launch);
  X.tag_base = gen << 20;
  if (gen <= 1) {
    hipError_t e = hipMemsetAsync(base, 0, (size_t)xbytes, st);
    if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_local_train: ") + hipGetErrorString(e));
  }
  const size_t lds = sizeof(float) * (size_t)PP_NR * PP_RS;
  if (P.fuse_E > 0 && (P.chained || ng * G + P.fuse_E > cus))
    return fail(FS_EINVAL, "fs_local_train: no room for the fused evaluation");
  const int grid = P.chained ? 8 * G : ng * G + P.fuse_E;
  switch (G) {
    case 2: launch_pipe_g<2>(P, X, grid, lds, st); break;
    case 4: launch_pipe_g<4>(P, X, grid, lds, st); break;
    default: launch_pipe_g<4>(P, X, grid, lds, st); break;
  }
  return FS_OK;
}

}  // namespace fs
