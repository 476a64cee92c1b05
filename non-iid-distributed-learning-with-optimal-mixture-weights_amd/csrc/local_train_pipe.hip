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
//   * each wave computes the softmax of ONE 16-lane-row column of a tile (row tile w / 4, rows
//     4 (w % 4) + lg) in registers, from the own slice's partial logits (an LDS transpose of the
//     8 wave partials, summed in wave order) plus the partners' granules it polls itself (G - 1
//     per lane), and hands its g values to the other waves through LDS with a tag flag per
//     column (no barrier): waves 0-3 finish tile 0's softmax while waves 4-7 still wait for
//     tile 1's partners;
//   * two barriers per step (one per row tile: the wave partials); the LDS image is
//     wave-private (each wave reads back only its own tiles), so it needs none;
//   * the same {tag, value} granule hand-off as the split form (cdna_hip_programming.md
//     Guideline 16, R2: relaxed agent-scope store / load, the data is its own flag), the
//     partner sum in slice order with the own partial at position g, every spin bounded.
// Covered shapes: full slices (ld = 1024 G: 16 tiles per workgroup, 2 per wave), 16 < B <= 32,
// C <= 16; the ridge and FedProx terms (the prox anchor's slice streamed per step, round 5).
// The bitwise match with the split form is tested (tests/test_gpu_pipe.py).  The planner picks
// it by shape only where it measured fastest (parallel clients at G <= 4 with more clients than
// groups and no prox term: config 4).
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
constexpr int PP_ZS = 16;                 // transposed partial-logit block: floats per class
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

// Diagnostic build only (-DFS_STAMPS): per-phase cycle sums of wave 0 of every workgroup
#ifdef FS_STAMPS
#define PP_STAMP(k)                                                                       \
  {                                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    unsigned long long t_;                                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    if (k > 0) stamp_acc[k > 0 ? k - 1 : 0] += t_ - stamp_prev;                           \
    stamp_prev = t_;                                                                      \
  }
#else
#define PP_STAMP(k)
#endif

// Wave issue priority (round 5): each SIMD issues its older wave first, so the second wave of
// every SIMD (waves 4-7) fell behind over a step and waves 0-3 waited at B1a (stamps, DESIGN.md
// 4.1).  PP_PRIO bit 2: from each tile's barrier to the end of its hand-off (own sum, publish,
// polls, image, softmax) a wave runs at priority 3, the MFMA phases at 0 -- the hand-off first
// whichever wave holds it (config 2: 311-314 -> 300-302 us per launch; config 4: 427-430 ->
// 421-427, profiles/r05/pipe_prio.txt); bit 1 (waves 4-7 at priority 1 throughout) measured no
// gain.  -DPP_PRIO=m selects the experiment (scripts/build_pipe_prio_variant.sh).
#ifndef PP_PRIO
#define PP_PRIO 2
#endif
#define PP_SETPRIO(n) __builtin_amdgcn_s_setprio(n)

__device__ __forceinline__ float invb_of(int bc) { return 1.0f / (float)bc; }

template <int G, bool NRM, bool PROX>
__global__ __launch_bounds__(PP_THREADS, 1) void local_train_pipe_kernel(LTParams P, SplitWS X) {
  static_assert(NRM || !PROX, "the prox term exchanges the norms");
  constexpr int NW = PP_WAVES, TPW = PP_TPW, RS = PP_RS, NC = 16;
  constexpr int GP = G > 1 ? G - 1 : 1;          // partners
  // wave partial logits, transposed: zpt[w][rt][class * ZS + 4 (kk ^ zsw(class)) + lg] = the partial
  // of row 16 rt + 4 lg + kk -- one ds_read_b128 per wave gives a lane its four rows of the tile.
  // The float4 slots of a class are XOR-swizzled by (class >> 1) & 3 (round 6): at a 20-float
  // class stride (unswizzled) the reads' 16-lane groups hit a bank twice, 22 % of the form's
  // LDS-array cycles in conflicts at config 4 (profiles/r06/pmc_c4.txt); now the reads are
  // conflict-free and the ds_write_b32 of the partials at most 2-way (free, MI355X_MICROARCH.md LDS)
  __shared__ __attribute__((aligned(16))) float zpt[NW][2][NC * PP_ZS];
  // softmax gradients of the step (by parity): gsm[par][rt][lane][kk] = g of (row 16 rt + 4 kk + lg,
  // class l16), written by wave 4 rt + kk, read back by every wave as one ds_read_b128; the
  // flags gfl[par][rt][kk] carry the step's tag once wave 4 rt + kk has written its column
  __shared__ __attribute__((aligned(16))) float gsm[2][2][64][4];
  __shared__ __attribute__((aligned(16))) unsigned gfl[2][2][4];
  __shared__ float cesm[2][8];             // per 4-row group CE wave sums (the reported loss)
  __shared__ float wn2sm[2][2];            // ||W - W_a||^2, ||W||^2 at the step's start, by wave 0
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
        s = sq4_acc(s, wr[i][q][0], wr[i][q][1], wr[i][q][2], wr[i][q][3]);
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
  if (PP_PRIO & 1) {
    if (w >= 4) PP_SETPRIO(1);                   // the SIMDs' second waves first
  }
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
  if (tid < 16) (&gfl[0][0][0])[tid] = 0u;       // (tag 0 is never a step's tag)
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

  // Per step, wave w publishes and polls like every other, but computes the softmax of ONE
  // 16-lane-row column: row tile h = w / 4, rows 4 kk + lg with kk = w % 4 -- 64 of the tile's
  // 256 (row, class) entries, as the split form spreads its softmax over its 8 waves -- and
  // hands the g values to the other waves through LDS (gsm + a tag flag per column, no
  // barrier): waves 0-3 finish tile 0's softmax while waves 4-7 still wait for tile 1's
  // partners, so a SIMD's two waves (one of each half) overlap one's round trip with the
  // other's backward MFMAs.  Every wave issues, in this order (counted vector-memory ops):
  //   [client start: 8 weight loads, drained at once]  1 publish store (rt0)  NRM norm store
  //   1 publish store (rt1)  [wait: the indices]  PH polls (its column: G - 1; wave 0 also the
  //   norms: G - 1)  [wait 0: every poll lands before any row is issued]  2 label loads
  //   8 row loads (next step, rt0: one per backward iteration of K0)  8 row loads (rt1, in K1)
  //   2 index loads
  // -- so at the forward of rt0 its rows (one step ago) have 8 + 2 operations behind them, the
  // rows of rt1 2 + 1 + NRM, the indices 1 + NRM + 1.  A stale poll is re-polled with nothing
  // else in flight.  Other extra operations (client-end stores, spills) only make a wait
  // stricter.
  // PROX: 8 anchor loads (the client's start W_a, tools.py:180; L2-resident) go out right after
  // the labels -- the update waits for them with the 16 row loads of K0 and K1 behind.
  constexpr int W_F0 = 8 + 2, W_F1 = 2 + 1 + (NRM ? 1 : 0), W_IDX = 1 + (NRM ? 1 : 0) + 1, W_ANC = 16;
  const int hrt = w >> 2, kcol = w & 3;          // this wave's softmax column: row tile, kk

  SpCur cc;
  bool cc_ok = sp_seek<true>(cc, P, grp, ng, T, 0);
  flush_empty(0, cc_ok ? cc.k : T);
  unsigned gs = 0;
  bool dead = false;
  double lsum = 0.0;
  const int rblk = 4 * (l16 & 3) + (l16 >> 2);
  unsigned long long pl[GP];
  unsigned long long pnrm[GP];
  floatx4 av[TPW][4];                            // PROX: the anchor slice of this step
  const float* anc = P.W_start;                  // PROX: the anchor of the current client
#ifdef FS_STAMPS
  unsigned long long stamp_acc[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, stamp_prev = 0;
#endif
  for (; cc_ok; ++gs) {
    PP_STAMP(0)
    const int st = cc.st, n = cc.n, nbat = cc.nbat;
    if (st == 0) {
      if (!P.chained && gs > 0) {
        (void)load_start();
        if (lane == 0) { wred[w][0] = 0.f; wred[w][1] = nw0; }
      } else if (lane == 0) {
        wred[w][0] = 0.f;
      }
      // the prox anchor is the client's start (tools.py:180): W_start, or in a chain the previous
      // client's result, which this workgroup stored at that client's end
      if (PROX) anc = (P.chained && cc.j > 0) ? P.W_out + (int64_t)(cc.j - 1) * C * ld : start;
      lsum = 0.0;
    }
    const int e = st / nbat, s = st - e * nbat;
    const int bc = min(B, n - s * B);
    const int par = gs & 1;
    const unsigned tag32 = X.tag_base + gs + 1u;
    const unsigned long long tag = (unsigned long long)tag32 << 32;
    unsigned long long* slot = xb + (int64_t)par * G * PP_SZ;
    const bool need_ce = g == 0 && e == E - 1;     // the cross-entropy feeds only the reported loss

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
      for (int j = 0; j < 4; ++j) zpt[w][rt][l16 * PP_ZS + 4 * (j ^ ((l16 >> 1) & 3)) + lg] = a[j];
    };
    // ---- the own slice's partials of one tile (wave order) ----
    auto own_sum = [&](int rt) {
      float4 p[NW];
#pragma unroll
      for (int i = 0; i < NW; ++i) p[i] = ld4(&zpt[i][rt][l16 * PP_ZS + 4 * (lg ^ ((l16 >> 1) & 3))]);
      floatx4 v = zero4;
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        v[0] += p[i].x; v[1] += p[i].y; v[2] += p[i].z; v[3] += p[i].w;
      }
      return v;
    };
    // (waves w and w + 4 publish the same component kk = w & 3: one unconditional store each)
    auto publish = [&](int rt, const floatx4& v) {
      const float x = kcol == 0 ? v[0] : (kcol == 1 ? v[1] : (kcol == 2 ? v[2] : v[3]));
      __hip_atomic_store(slot + (int64_t)g * PP_SZ + rt * 256 + kcol * 64 + lane, tag | __float_as_uint(x),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };

    // ================= row tile 0: forward, publish =================
    pp_wait<W_F0>();                                // this step's rt0 rows and labels landed
    PP_STAMP(1)
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) pp_own(lb[rt]);
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) pp_own(xf[i][0][q]);
    forward(0);
    PP_STAMP(2)
    lds_barrier();                                  // B1a: wave partials of rt0 (and the norms)
    if (PP_PRIO & 2) PP_SETPRIO(3);                 // the hand-off phases first
    PP_STAMP(3)
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
    PP_STAMP(4)
    if (PP_PRIO & 2) {
      if ((PP_PRIO & 1) && w >= 4) PP_SETPRIO(1);
      else PP_SETPRIO(0);
    }
    pp_wait<W_F1>();                                // this step's rt1 rows landed
    PP_STAMP(5)
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) pp_own(xf[i][1][q]);
    forward(1);
    PP_STAMP(6)
    lds_barrier();                                  // B1b
    if (PP_PRIO & 2) PP_SETPRIO(3);
    PP_STAMP(7)
    const floatx4 own1 = own_sum(1);
    publish(1, own1);
    pp_wait<W_IDX>();                               // the next step's row indices landed
    take_rows();
    // ---- this wave's column of the softmax: the partners' granules of (row tile hrt, kk) ----
    const bool nrm_w = NRM && w == 0;               // wave 0 also polls the norms
    auto poll = [&]() {
#pragma unroll
      for (int k = 0; k < G - 1; ++k) {
        const int h = k + (k >= g ? 1 : 0);
        pp_poll(pl[k], slot + (int64_t)h * PP_SZ + hrt * 256 + kcol * 64 + lane);
      }
      if (nrm_w)
#pragma unroll
        for (int k = 0; k < G - 1; ++k) {
          const int h = k + (k >= g ? 1 : 0);
          pp_poll(pnrm[k], slot + (int64_t)h * PP_SZ + 512 + (lane & 1));
        }
    };
    poll();
    PP_STAMP(8)
    // image of this wave's tiles for the backward (wave-private: no barrier), under the round trip
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          st4(xs_dyn + img_off(rt * 16 + l16, RS, w + NW * i, 4 * q + lg),
              make_float4(xf[i][rt][q][0], xf[i][rt][q][1], xf[i][rt][q][2], xf[i][rt][q][3]));
    PP_STAMP(9)
    pp_wait<0>();
#pragma unroll
    for (int k = 0; k < G - 1; ++k) pp_own(pl[k]);
    if (nrm_w)
#pragma unroll
      for (int k = 0; k < G - 1; ++k) pp_own(pnrm[k]);
    {
      if (X.spin_limit == 0 && gs == 0 && lane == 0)      // test knob: report an injected timeout
        __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned spins = 0;
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int k = 0; k < G - 1; ++k) ok &= (l16 >= C) | ((unsigned)(pl[k] >> 32) == tag32);
        if (nrm_w)
#pragma unroll
          for (int k = 0; k < G - 1; ++k) ok &= (unsigned)(pnrm[k] >> 32) == tag32;
        if (__all(ok)) break;
        if (dead || ++spins > X.spin_limit) {
          if (lane == 0) __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          dead = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        poll();
        pp_wait<0>();
#pragma unroll
        for (int k = 0; k < G - 1; ++k) pp_own(pl[k]);
        if (nrm_w)
#pragma unroll
          for (int k = 0; k < G - 1; ++k) pp_own(pnrm[k]);
      }
    }
    PP_STAMP(10)
    {
      // slice-order sum (own partial at position g): every partner gets the same bits
      const floatx4& own = hrt ? own1 : own0;
      const float ownv = kcol == 0 ? own[0] : (kcol == 1 ? own[1] : (kcol == 2 ? own[2] : own[3]));
      float z0 = 0.f;
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float pv = 0.f;
#pragma unroll
        for (int k = 0; k < G - 1; ++k)
          if (k + (k >= g ? 1 : 0) == h) pv = __uint_as_float((unsigned)pl[k]);
        z0 += (h == g) ? ownv : pv;
      }
      if (nrm_w) {
        // ||W||^2 at the start of this step: slice-order sum (lane 1; lane 0: ||W - W_a||^2)
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
        if (lane < 2) wn2sm[par][lane] = ns;
      }
      // the softmax of (row 16 hrt + 4 kcol + lg, class l16) -- the split form's arithmetic: its
      // xor butterflies 8, 4, 2, 1 over the class lanes with the same bits (the max is exact in
      // any order: four DPP rotations; in the sum, after the xor-8 level every lane's row_ror:4
      // partner holds the xor-4 partner's value)
      const int r = 16 * hrt + 4 * kcol + lg;
      const bool valid = r < bc && l16 < C;
      const float z = valid ? z0 : 0.f;
      const float m = row16_all<true>(valid ? z : -INFINITY);
      const float ex = valid ? __expf(z - m) : 0.f;
      float se = ex + dpp<0x128>(ex);                       // row_ror:8 = xor 8
      se = se + dpp<0x124>(se);                             // row_ror:4 (= the xor-4 value here)
      se = se + dpp<0x4E>(se);                              // quad xor 2
      se = se + dpp<0xB1>(se);                              // quad xor 1
      const int lab = __shfl(hrt ? lb[1] : lb[0], 4 * kcol + lg, 64);   // label of row r
      float gv = 0.f, ce = 0.f;
      if (valid) {
        const bool isy = l16 == lab;
        gv = (isy ? -invb_of(bc) : 0.f) + ex * __builtin_amdgcn_rcpf(se) * invb_of(bc);
        if (need_ce && isy) ce -= z - m - __logf(se);
      }
      gsm[par][hrt][lane][kcol] = gv;
      if (need_ce) {
        ce = wave_sum_dpp(ce, lane);              // the split form's wave (4 hrt + kcol) CE sum
        if (lane == 0) cesm[par][w] = ce;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the column (and wn2) before its flag
      if (lane == 0) gfl[par][hrt][kcol] = tag32;
    }
    // the next step's labels (the polls have all landed and this step's labels are read: nothing
    // of ours waits behind them); PROX: this step's anchor slice
    issue_labels();
    if (PROX) {
      int64_t b = (int64_t)min(l16, C - 1) * ld + 64 * t0 + 4 * lg + 64 * w;
      asm volatile("" : "+v"(b));
      const float* a = anc + b;
      pp_ld4<0>(av[0][0], a); pp_ld4<64>(av[0][1], a); pp_ld4<128>(av[0][2], a); pp_ld4<192>(av[0][3], a);
      pp_ld4<2048>(av[1][0], a); pp_ld4<2112>(av[1][1], a); pp_ld4<2176>(av[1][2], a); pp_ld4<2240>(av[1][3], a);
    }
    PP_STAMP(11)
    // ---- the g values of a row tile, once its four columns are flagged ----
    float gB[8];
    auto take_g = [&](int rt) {
      // (64-bit: 64 x a fs_tuning.spin_limit of 2^26 or more would wrap in 32 bits)
      unsigned long long sp = 0;
      for (;;) {
        typedef unsigned uintx4 __attribute__((ext_vector_type(4)));
        const uintx4 f = *reinterpret_cast<volatile const uintx4*>(&gfl[par][rt][0]);
        if ((f[0] == tag32) & (f[1] == tag32) & (f[2] == tag32) & (f[3] == tag32)) break;
        if (dead || ++sp > 64ull * X.spin_limit) {
          if (lane == 0) __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          dead = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      const floatx4 v = *reinterpret_cast<volatile const floatx4*>(&gsm[par][rt][lane][0]);
      gB[4 * rt + 0] = v[0]; gB[4 * rt + 1] = v[1]; gB[4 * rt + 2] = v[2]; gB[4 * rt + 3] = v[3];
    };

    // ================= backward: image rows 4 kk + lg, kk = 0..7 =================
    floatx4 ga[TPW][4];
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) ga[i][e4] = zero4;
    // (with the next step's 8 row loads of tile-row rt_ld, one per (tile, kk) iteration: the
    // stream spreads over the phase's MFMAs instead of a burst that fills the memory queue)
    auto bwd = [&](int kk0, int rt_ld) {
      const float* src = P.phi + (int64_t)pn[rt_ld] * ld + 64 * t0 + 4 * lg + 64 * w;
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
          const int f = 4 * i + (kk - kk0);          // row piece (tile f / 4, q = f % 4)
          switch (f) {
            case 0: pp_ld4<0>(xf[0][rt_ld][0], src); break;
            case 1: pp_ld4<64>(xf[0][rt_ld][1], src); break;
            case 2: pp_ld4<128>(xf[0][rt_ld][2], src); break;
            case 3: pp_ld4<192>(xf[0][rt_ld][3], src); break;
            case 4: pp_ld4<2048>(xf[1][rt_ld][0], src); break;
            case 5: pp_ld4<2112>(xf[1][rt_ld][1], src); break;
            case 6: pp_ld4<2176>(xf[1][rt_ld][2], src); break;
            default: pp_ld4<2240>(xf[1][rt_ld][3], src); break;
          }
        }
      }
    };
    if (PP_PRIO & 2) {
      if ((PP_PRIO & 1) && w >= 4) PP_SETPRIO(1);
      else PP_SETPRIO(0);
    }
    take_g(0);
    PP_STAMP(12)
    bwd(0, 0);                                      // K0 (beside the other half's round trip)
    PP_STAMP(13)
    take_g(1);
    float pn2 = 0.f, wn2 = 0.f;
    if (NRM) {
      pn2 = wn2sm[par][0];
      wn2 = wn2sm[par][1];
    }
    if (need_ce && w == 0) {
      // the loss as the split form sums it: the eight 4-row-group CE sums in row order
      float ce = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) ce += cesm[par][k];
      if (lane == 0) {
        float loss = ce / (float)bc;
        if (P.prox) loss = loss + P.mu * sqrtf(pn2);
        if (P.reg) loss = loss + P.lam * sqrtf(wn2);
        lsum += (double)loss * (double)bc;
      }
    }
    bwd(4, 1);                                      // K1
    // ---- update of the register-resident slice ----
    float npn = 0.f, nwn = 0.f;
    {
      const float sp = (P.prox && pn2 > 0.f) ? P.mu / sqrtf(pn2) : 0.f;
      const float sr = (P.reg && wn2 > 0.f) ? P.lam / sqrtf(wn2) : 0.f;
      const float lr = P.lr;
      if (PROX) {
        pp_wait<W_ANC>();                           // the anchor slice landed
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) pp_own(av[i][q]);
      }
      if (l16 < C) {
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) {
              const float ac = PROX ? av[i][q][e4] : 0.f;
              const float o = sgd_w(wr[i][q][e4], ga[i][e4][q], lr, PROX, ac, sp, P.reg, sr);
              wr[i][q][e4] = o;
              if (PROX) {                            // the split form's inline norms (its order)
                npn = sq_acc(npn, o - ac);
                nwn = sq_acc(nwn, o);
              }
            }
      }
    }
    if (PROX) {
      npn = wave_sum_dpp(npn, lane);
      nwn = wave_sum_dpp(nwn, lane);
      if (lane == 0) { wred[w][0] = npn; wred[w][1] = nwn; }
    } else if (NRM) {
      // ridge: ||W||^2 of the updated slice in the update's order (the split form's bits)
#pragma unroll
      for (int i = 0; i < TPW; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) nwn = sq_acc(nwn, wr[i][q][e4]);
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
    PP_STAMP(14)
  }
  pp_wait<0>();                                     // nothing of ours is in flight at the exit
#ifdef FS_STAMPS
  // (every wave: [grid][8 waves][16])
  if (lane == 0 && X.stamps) {
    for (int k = 0; k < 14; ++k) X.stamps[(blockIdx.x * 8 + w) * 16 + k] = stamp_acc[k];
    X.stamps[(blockIdx.x * 8 + w) * 16 + 15] = (unsigned long long)gs;
  }
#endif
}

bool pipe_fits(int C, int B, int NT, int G, int prox) {
  (void)prox;
  if (!(G == 2 || G == 4 || G == 8 || G == 16)) return false;
  return C >= 1 && C <= 16 && B > 16 && B <= 32 && NT == PP_NTS * G;
}

static int64_t pipe_xbuf_bytes(int ngroups, int G) { return (int64_t)ngroups * 2 * G * PP_SZ * 8; }

int pipe_groups(int N, int G, int chained, int cus) { return chained ? 1 : std::max(1, std::min(N, cus / G)); }

int64_t pipe_ws_bytes(int N, int G, int chained, int cus) {
  return pipe_xbuf_bytes(pipe_groups(N, G, chained, cus), G) + PP_ERR_BYTES;
}

template <int G, bool NRM, bool PROX>
static void launch_pipe_s(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&local_train_pipe_kernel<G, NRM, PROX>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((local_train_pipe_kernel<G, NRM, PROX>), dim3(grid), dim3(PP_THREADS), lds, st, P, X);
}

template <int G>
static void launch_pipe_g(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  if (P.prox) launch_pipe_s<G, true, true>(P, X, grid, lds, st);
  else if (P.reg) launch_pipe_s<G, true, false>(P, X, grid, lds, st);
  else launch_pipe_s<G, false, false>(P, X, grid, lds, st);
}

unsigned split_spin_bound();   // local_train_split.hip: fs_tuning.spin_limit / the test knob

int launch_local_train_pipe(const LTParams& P, int G, void* ws, int64_t ws_bytes, hipStream_t st) {
  const int NT = (int)(P.ld >> 6);
  if (!pipe_fits(P.C, P.B, NT, G, P.prox))
    return fail(FS_EUNSUPPORTED, "fs_local_train: the pipe form needs ld = 1024 G (G = 2, 4, 8 or 16), 16 < B <= 32 "
                                 "and C <= 16");
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
#ifdef FS_STAMPS
  X.stamps = reinterpret_cast<unsigned long long*>(base + xbytes);
#endif
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
    case 8: launch_pipe_g<8>(P, X, grid, lds, st); break;
    default: launch_pipe_g<16>(P, X, grid, lds, st); break;
  }
  return FS_OK;
}

}  // namespace fs
