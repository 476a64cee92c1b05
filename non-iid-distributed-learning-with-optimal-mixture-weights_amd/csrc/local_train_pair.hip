// Pair-client local training: a group of G workgroups (on G CUs) trains TWO clients at a
// time, interleaved, so that one client's cross-CU hand-off overlaps the other client's
// compute and the next step's row stream is in flight through every phase.
//
// Math: train_loop (/root/reference/functions/tools.py:177-215) for parallel clients (every
// client starts from the round's model, FedAvg / FedProx / FedAMW at tools.py:340-343,
// 367-370, 430-433 with clients='parallel').  Per step it is the split kernel's arithmetic
// (local_train_split.hip) in the same order -- forward over the workgroup's tiles, wave
// partials summed in wave order, the G slice partials folded in slice order, the same softmax,
// backward and update -- so at the same G both kernels give bitwise the same weights.
//
// Why a second kernel.  In the split kernel a step is forward -> hand-off -> softmax ->
// backward, and the next step's rows can only stream during the backward: the registers hold
// the current rows until the image write, and rows issued before a hand-off delay its polls
// (they queue behind them in the CU's memory pipe).  In-kernel stamps put the stream at about
// half of each step.  Here a group owns two client LANES; one half-step runs
// lane X's forward and lane Y's hand-off completion, softmax and backward:
//   [A] poll Y's partners (they published one half-step ago)
//   [B] forward X on its register-resident rows (issued two half-steps ago)          S1
//   [C] publish X's partial logits and norms; [D] LDS image of X's rows
//   [E] Y's hand-off: check the polls (re-poll while a partner is late)
//   [F] X's next rows: labels, 8 x 1 KiB row pieces per wave, the following step's indices
//   [G] sum Y's partials (slice order)  S2  softmax Y  S3  backward Y, update, norms
// X's rows stream during Y's softmax and backward and during the next half-step's forward and
// publish; Y's hand-off round trip overlaps X's forward.  Every load of a half-step is issued
// unconditionally (a lane with nothing to do loads row 0 and polls a dummy slot), so the
// compiler's vmcnt bookkeeping sees one straight-line pattern and each phase waits for exactly
// the loads it consumes; the client tables are read with scalar loads (split_common.h), so a
// client boundary never waits for the row stream.
// Layout: each workgroup owns 8 consecutive 64-column tiles (NT == 8 G), one per wave.  Per
// lane the weights (16 VGPRs) and one step's rows (32 VGPRs at B = 32) are register-resident,
// and so is the W_start slice -- every client's start and FedProx anchor.  LDS: one row image
// per lane (2 x 65 KB at B = 32).
// Hand-offs: 8-byte {tag, value} granules (cdna_hip_programming.md Guideline 16, R2 form), one
// slot per (lane, step parity, slice); every spin is bounded and a timeout sets the
// workspace's error word.
#include "common.h"
#include "eval_rows.h"
#include "lanes.h"
#include "split_common.h"

namespace fs {

constexpr int PR_WAVES = 8;
constexpr int PR_THREADS = PR_WAVES * 64;
constexpr int PR_TILES = PR_WAVES;            // 64-column tiles per workgroup and client (one per wave)
constexpr unsigned PR_SPIN_LIMIT = 1u << 22;
constexpr int PR_ERR_BYTES = 256;

// In-loop loads are inline asm, invisible to hipcc's vmcnt bookkeeping (which, across this
// loop's back-edge, drained the whole row stream before every row issue); their waits are
// counted by hand (PR_WAIT) from the fixed per-half-step issue pattern, and every destination
// is named "+v" by a statement after its wait (cdna_hip_programming.md 5.7 item 1, form ii).
// scripts/asm_audit.py checks the built code object: no instruction touches a destination
// between its load and that statement.
template <int OFF>
__device__ __forceinline__ void pr_ld4(floatx4& d, const float* p) {
  asm volatile("global_load_dwordx4 %0, %1, off offset:%2 ; pr-row" : "=v"(d) : "v"(p), "n"(OFF) : "memory");
}
__device__ __forceinline__ void pr_ld1(int& d, const int32_t* p) {
  asm volatile("global_load_dword %0, %1, off ; pr-idx" : "=v"(d) : "v"(p) : "memory");
}
__device__ __forceinline__ void pr_poll(unsigned long long& d, const unsigned long long* p) {
  asm volatile("global_load_dwordx2 %0, %1, off sc1 ; pr-poll" : "=v"(d) : "v"(p) : "memory");
}
// a re-poll: load and wait in one statement
__device__ __forceinline__ unsigned long long pr_poll_now(const unsigned long long* p) {
  unsigned long long d;
  asm volatile("global_load_dwordx2 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(d) : "v"(p) : "memory");
  return d;
}
template <int N>
__device__ __forceinline__ void pr_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" : : "n"(N) : "memory");
}
template <typename T>
__device__ __forceinline__ void pr_own(T& x) {
  asm volatile("; pr-own %0" : "+v"(x));
}

// Diagnostic build only (-DFS_STAMPS): per-phase cycle sums of wave 0 of every workgroup
// (never in the shipped library)
#ifdef FS_STAMPS
#define PR_STAMP(k)                                                                       \
  {                                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    unsigned long long t_;                                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    if (k > 0) stamp_acc[k > 0 ? k - 1 : 0] += t_ - stamp_prev;                           \
    stamp_prev = t_;                                                                      \
  }
#else
#define PR_STAMP(k)
#endif

template <int RT, int G, bool PROX>
__global__ __launch_bounds__(PR_THREADS, 1) void local_train_pair_kernel(LTParams P, SplitWS X) {
  constexpr int NW = PR_WAVES;
  constexpr int NC = 16;
  constexpr int NR = RT * 16;
  constexpr int RS = PR_TILES * 64 + 8;          // LDS row stride (floats)
  // wave partial logits in the MFMA accumulator's own layout, [rt][lg][class][i] = row
  // 16 rt + 4 lg + i: one conflict-free ds_write_b128 per row tile, and the (row, class)
  // reads of the publish stride 4 words across a 16-lane row (conflict-free too)
  __shared__ __attribute__((aligned(16))) float zpart[NW][NR * NC];
  __shared__ float gbuf[NR][NC];
  __shared__ int lab[2][NR];
  __shared__ float wred[2][NW][2];
  __shared__ float wce[NW];
  __shared__ float nrm[2];
  extern __shared__ __attribute__((aligned(16))) float xs_lds[];   // [2 lanes][NR][RS] row images

  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, lg = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t ld = P.ld;
  const int C = P.C, B = P.B, E = P.E;

  // fused evaluation blocks (the last fuse_E of the grid): round t-1's test evaluation of
  // W_start on the CUs the groups leave idle (as in the split kernel)
  const int nb = gridDim.x - P.fuse_E;
  if ((int)blockIdx.x >= nb) {
    eval_persistent<NW>(P.fuse_phi, P.ld, P.fuse_y, P.fuse_n, P.W_start, P.C, (int)blockIdx.x - nb, P.fuse_E, xs_lds,
                        P.fuse_part);
    return;
  }
  // consecutive linear ids on one XCD (round-robin placement), so a group's partners mostly
  // share an L2 -- speed only
  int lin = blockIdx.x;
  if (nb % 8 == 0) lin = (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8;
  const int ng = X.ngroups;
  const int grp = lin / G, g = lin % G;
  if (grp >= ng) return;
  const int nvg = 2 * ng;                        // lane L of group grp walks sequence 2 grp + L
  const int T = (P.N + nvg - 1) / nvg;
  const int t0 = PR_TILES * g;
  const float* start = P.W_start;
  unsigned long long* xb = X.xbuf + (int64_t)grp * 5 * G * X.SZ;   // [lane][parity][G][SZ], dummy [G][SZ]
  unsigned long long* dummy = xb + (int64_t)4 * G * X.SZ;
  const bool cl = l16 < C;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);

  // lane (l16, lg) of wave w holds W[c = l16][64 (t0 + w) + 16 q + 4 lg + e], q = 0..3
  const int64_t wbase = (int64_t)l16 * ld + 64 * (t0 + w) + 4 * lg;
  float4 ws[4];
  float s0 = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    ws[q] = cl ? ld4(start + wbase + 16 * q) : zero4;
    s0 = sq4_acc(s0, ws[q].x, ws[q].y, ws[q].z, ws[q].w);
  }
  const float nw0 = wave_sum_dpp(s0, lane);      // ||W_start||^2 partial of this wave
  float4 wr[2][4];
#pragma unroll
  for (int L = 0; L < 2; ++L)
#pragma unroll
    for (int q = 0; q < 4; ++q) wr[L][q] = ws[q];
  if (lane == 0)
#pragma unroll
    for (int L = 0; L < 2; ++L) { wred[L][w][0] = 0.f; wred[L][w][1] = nw0; }

  // per lane: compute cursor cc (the step being computed), load cursor lc (the next step
  // whose rows are to be issued), rows / labels / permutation indices in registers
  SpCur cc[2], lc[2];
  bool cok[2], lok[2], pend[2] = {false, false};
  unsigned gsl[2] = {0u, 0u};                    // steps completed per lane (hand-off tags / parity)
  double lsum[2] = {0.0, 0.0};
  float ownv[2] = {0.f, 0.f};                    // this thread's published value of the lane's pending step
  floatx4 xf[2][RT][4];
  int pr[2][RT], lb[2][RT];
  int64_t prow0[2];
  bool dead = false;

  // clients with no step (n_j = 0 or E = 0) between sequence positions [ka, kb) of lane L:
  // the result is W_start, the loss 0
  auto flush_empty = [&](int L, int ka, int kb) {
    for (int k = ka; k < kb; ++k) {
      const int j = sp_client<true>(P, 2 * grp + L, nvg, k);
      if (j < 0) continue;
      if (cl) {
        float* Wj = P.W_out + (int64_t)j * C * ld + wbase;
#pragma unroll
        for (int q = 0; q < 4; ++q) st4(Wj + 16 * q, ws[q]);
      }
      if (g == 0 && tid == 0) P.loss[j] = 0.0;
    }
  };

  // permutation indices of lane L's load cursor (row 0 of the phi block when it has none):
  // rows past the batch end take the batch's first row (their logits are ignored)
  auto fetch_perm = [&](auto Lc) {
    constexpr int L = decltype(Lc)::value;
    const int32_t* pp = P.perms;
    int bc = 1;
    int64_t r0 = 0;
    if (lok[L]) {
      const int e_ = lc[L].st / lc[L].nbat, s_ = lc[L].st - e_ * lc[L].nbat;
      const int b0_ = s_ * B;
      bc = min(B, lc[L].n - b0_);
      pp = P.perms + (int64_t)E * lc[L].row0 + (int64_t)e_ * lc[L].n + b0_;
      r0 = lc[L].row0;
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int r_ = rt * 16 + l16;
      pr_ld1(pr[L][rt], pp + (r_ < bc ? r_ : 0));
    }
    prow0[L] = lok[L] ? r0 : -1;
  };
  // labels (wave 0: it writes them to LDS) and the row bases of lane L's load cursor (row 0
  // when it has none): whatever the lane's state, wave 0 issues RT label loads
  auto row_src = [&](auto Lc, int rt) {
    constexpr int L = decltype(Lc)::value;
    const int64_t row = prow0[L] >= 0 ? prow0[L] + pr[L][rt] : 0;
    return P.phi + row * ld + 64 * (t0 + w) + 4 * lg;
  };
  auto issue_labels = [&](auto Lc) {
    constexpr int L = decltype(Lc)::value;
    if (w == 0)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) pr_ld1(lb[L][rt], P.labels + (prow0[L] >= 0 ? prow0[L] + pr[L][rt] : 0));
  };

#pragma unroll
  for (int L = 0; L < 2; ++L) {
    cok[L] = sp_seek<true>(cc[L], P, 2 * grp + L, nvg, T, 0);
    lc[L] = cc[L];
    lok[L] = cok[L];
    flush_empty(L, 0, cok[L] ? cc[L].k : T);
  }
  if (!(cok[0] || cok[1])) return;
  // prologue: each lane's first rows, then the indices of its second step; everything lands
  // before the loop (the loop's counted waits assume its own issue pattern)
  fetch_perm(std::integral_constant<int, 0>{});
  fetch_perm(std::integral_constant<int, 1>{});
  pr_wait<0>();
#pragma unroll
  for (int L = 0; L < 2; ++L)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) pr_own(pr[L][rt]);
  issue_labels(std::integral_constant<int, 0>{});
  issue_labels(std::integral_constant<int, 1>{});
  // lane 0's first rows whole; lane 1's but the last quarter, which half-step 0's forward issues
  // (as every forward issues the last quarter of the other lane's next rows)
  constexpr int NP = 4 * RT;                     // row pieces per step and wave
  const float* srcx[2][RT];                      // row bases of each lane's step being loaded
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    srcx[0][rt] = row_src(std::integral_constant<int, 0>{}, rt);
    srcx[1][rt] = row_src(std::integral_constant<int, 1>{}, rt);
  }
  auto piece = [&](auto Lc, int k) {             // row piece k = (rt, q) of lane L's step being loaded
    constexpr int L = decltype(Lc)::value;
    pr_ld4<0>(xf[L][k >> 2][k & 3], srcx[L][k >> 2] + 16 * (k & 3));
  };
#pragma unroll
  for (int k = 0; k < NP; ++k) piece(std::integral_constant<int, 0>{}, k);
#pragma unroll
  for (int k = 0; k < 3 * NP / 4; ++k) piece(std::integral_constant<int, 1>{}, k);
#pragma unroll
  for (int L = 0; L < 2; ++L)
    if (lok[L]) lok[L] = sp_advance<true>(lc[L], P, 2 * grp + L, nvg, T);
  fetch_perm(std::integral_constant<int, 0>{});
  fetch_perm(std::integral_constant<int, 1>{});
  pr_wait<0>();
  unsigned long long pl[G - 1];                  // polls of the lane published last half-step (partners)
#pragma unroll
  for (int h = 0; h < G - 1; ++h) pl[h] = 0ull;
  lds_barrier();

  // Per half-step every wave issues, in this order and whatever the lanes' states (a lane
  // with nothing to publish stores to the dummy slot, one with no next step loads row 0):
  //   P4: the last NP/4 row pieces of lane Y's next step, one per MFMA group of lane X's
  //   forward;  [C] 1 publish store;  P1: NP/4 row pieces of lane X's next step;  [E] ...;
  //   P2: NP/4 more;  [F] G - 1 polls (the partners), LBW label loads (wave 0 only: LBW = RT, else 0), RT index
  //   loads;  P3: NP/4 more inside lane Y's backward     (NP = 4 RT pieces per step)
  // -- each lane's next rows spread over two half-steps at about the rate one CU's memory pipe
  // drains them, never a burst that stalls the issuing waves (and skews the next barrier).
  // Hence the counted waits: the last piece of lane X's rows (P4 one half-step ago) has
  // 1 + 3 NP/4 + (G - 1) + LBW + RT operations behind it at [B]; lane Y's polls ([F] one half-step
  // ago) have LBW + RT + 3 NP/4 + 1 at [E].  Extra operations (client-end stores, re-polls)
  // only make a wait stricter.
  constexpr int WAIT_B0 = 1 + 3 * NP / 4 + (G - 1) + RT + RT, WAIT_B = 1 + 3 * NP / 4 + (G - 1) + RT;
  constexpr int WAIT_E0 = RT + RT + 3 * NP / 4 + 1, WAIT_E = RT + 3 * NP / 4 + 1;
  static_assert(WAIT_B0 < 64, "vmcnt is 6 bits");

#ifdef FS_STAMPS
  unsigned long long stamp_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, stamp_prev = 0;
  unsigned nhalf = 0;
#endif
  auto half = [&](auto Xc, auto Yc) {
    constexpr int XL = decltype(Xc)::value, YL = decltype(Yc)::value;
#ifdef FS_STAMPS
    ++nhalf;
#endif
    PR_STAMP(0)
    // ---- [B] forward partial of lane X: z_g = X_slice W_slice^T ----
    if (w == 0) pr_wait<WAIT_B0>();              // lane X's labels, indices and rows have landed
    else pr_wait<WAIT_B>();
    PR_STAMP(1)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      pr_own(lb[XL][rt]);
      pr_own(pr[XL][rt]);
#pragma unroll
      for (int q = 0; q < 4; ++q) pr_own(xf[XL][rt][q]);
    }
    {
      // (the MFMAs run whether or not X has a step: P4's loads sit in one code path; a lane
      // with nothing to publish publishes zeros)
      floatx4 acc[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[rt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma4(xf[XL][rt][q][e4], comp(wr[XL][q], e4), acc[rt]);
        if (RT == 1 ? q == 3 : (q & 1) != 0) piece(Yc, 3 * NP / 4 + (RT == 1 ? 0 : q >> 1));   // P4
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        st4(&zpart[w][rt * 256 + lg * 64 + l16 * 4], make_float4(acc[rt][0], acc[rt][1], acc[rt][2], acc[rt][3]));
    }
    // lane X's next step: row bases from its indices (fetched two half-steps ago)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) srcx[XL][rt] = row_src(Xc, rt);
    PR_STAMP(2)
    lds_barrier();  // S1: wave partials; lane X's norms of its previous update
    PR_STAMP(3)

    // ---- [C] publish lane X's partials: thread t owns (row, class) = (t / 16, t % 16) -- the
    // logits at class < C, ||W - W_a||^2 and ||W||^2 at row 0, classes 14 and 15 (C <= 14);
    // every thread stores one granule ----
    {
      float v = 0.f;
      if (cok[XL]) {
        const int r = tid >> 4, c = tid & 15;
        if (r < NR && c < C) {
#pragma unroll
          for (int i = 0; i < NW; ++i) v += zpart[i][zp_off(r, c)];
        } else if (r == 0 && c >= NC - 2) {
#pragma unroll
          for (int i = 0; i < NW; ++i) v += wred[XL][i][c - (NC - 2)];
        }
      }
      ownv[XL] = v;
      const unsigned tagX = cok[XL] ? X.tag_base + gsl[XL] + 1u : 0u;
      unsigned long long* slotX =
          cok[XL] ? xb + (int64_t)((2 * XL + (gsl[XL] & 1)) * G + g) * X.SZ : dummy + (int64_t)g * X.SZ;
      __hip_atomic_store(slotX + tid, ((unsigned long long)tagX << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    // ---- [D] lane X's rows into its LDS image (read by its backward next half-step) ----
    if (cok[XL]) {
      float* img = xs_lds + XL * NR * RS;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const floatx4 v = xf[XL][rt][q];
          st4(img + img_off(rt * 16 + l16, RS, w, 4 * q + lg), make_float4(v[0], v[1], v[2], v[3]));
        }
      if (w == 0 && lg == 0)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) lab[XL][rt * 16 + l16] = lb[XL][rt];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the image has read xf[X] before P1 refills it
#pragma unroll
    for (int k = 0; k < NP / 4; ++k) piece(Xc, k);         // P1
    PR_STAMP(4)

    // ---- [E] lane Y's hand-off: every partner's granule must carry this step's tag ----
    if (w == 0) pr_wait<WAIT_E0>();              // lane Y's polls (and everything before them) landed
    else pr_wait<WAIT_E>();
    PR_STAMP(5)
#pragma unroll
    for (int h = 0; h < G - 1; ++h) pr_own(pl[h]);
    const unsigned tagY = X.tag_base + gsl[YL] + 1u;
    unsigned long long* slotY = xb + (int64_t)((2 * YL + (gsl[YL] & 1)) * G) * X.SZ;
    if (pend[YL]) {
      if (X.spin_limit == 0 && gsl[YL] == 0) dead = true;    // test knob: an injected timeout
      bool ok = true;
#pragma unroll
      for (int h = 0; h < G - 1; ++h) ok &= (unsigned)(pl[h] >> 32) == tagY;
      if (!__all(ok)) {
        unsigned spins = 0;
        for (;;) {
          if (dead || ++spins > X.spin_limit) {
            dead = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          ok = true;
#pragma unroll
          for (int h = 0; h < G - 1; ++h) {
            pl[h] = pr_poll_now(slotY + (int64_t)(h < g ? h : h + 1) * X.SZ + tid);
            ok &= (unsigned)(pl[h] >> 32) == tagY;
          }
          if (__all(ok)) break;
        }
      }
      PR_STAMP(6)
    }
#pragma unroll
    for (int k = NP / 4; k < NP / 2; ++k) piece(Xc, k);    // P2
    // ---- [G] complete lane Y's step: sum the slices in order, then -- every value sits at
    // (row, class) = (tid / 16, tid % 16), a row on one 16-lane DPP row -- the softmax straight
    // from the registers (no LDS round trip, no barrier) ----
    // (a lane with nothing pending may have an exhausted cursor: its fields are not used)
    const int st = pend[YL] ? cc[YL].st : 0, nbat = pend[YL] ? cc[YL].nbat : 1, n = pend[YL] ? cc[YL].n : 1;
    const int e = st / nbat, sb = st - e * nbat;
    const int bc = max(1, min(B, n - sb * B));
    const float invb = 1.0f / (float)bc;
    if (pend[YL]) {
      float z = 0.f;
#pragma unroll
      for (int h = 0; h < G; ++h) {                // slice order, the own partial at position g
        // (partner slice h sits at pl[h] below g and at pl[h - 1] above it: static indices)
        const float lo = h < G - 1 ? __uint_as_float((unsigned)pl[h < G - 1 ? h : 0]) : 0.f;
        const float hi = h > 0 ? __uint_as_float((unsigned)pl[h > 0 ? h - 1 : 0]) : 0.f;
        z += (h == g) ? ownv[YL] : (h < g ? lo : hi);
      }
      const int r = tid >> 4, c = tid & 15;
      if (r == 0 && c >= NC - 2) nrm[c - (NC - 2)] = z;   // ||W - W_a||^2, ||W||^2 at the step's start
      const bool valid = r < bc && c < C;
      float m = valid ? z : -INFINITY;
#pragma unroll
      for (int off = NC / 2; off > 0; off >>= 1) m = fmaxf(m, xor_get(m, off, lane));
      // softmax on v_exp_f32 / v_rcp_f32 / v_log_f32 (one exponential per entry, e / sum e for
      // the gradient): within the fp32 tolerance of torch's log_softmax (tests/fixtures.py)
      const float ex = valid ? __expf(z - m) : 0.f;
      float se = ex;
#pragma unroll
      for (int off = NC / 2; off > 0; off >>= 1) se += xor_get(se, off, lane);
      float gv = 0.f, cep = 0.f;
      if (valid) {
        const bool isy = c == lab[YL][r];
        gv = (isy ? -invb : 0.f) + ex * __builtin_amdgcn_rcpf(se) * invb;
        if (isy) cep = -(z - m - __logf(se));
      }
      if (r < NR) gbuf[r][c] = gv;
      cep = wave_sum_dpp(cep, lane);
      if (lane == 0) wce[w] = cep;
    }
    PR_STAMP(7)
    lds_barrier();  // S3: g, CE partials
    PR_STAMP(8)

    // ---- [F] lane X's polls (its partials went out at [C]), labels and the indices of the step
    // after the one being loaded (a lane with nothing published polls the dummy slot) ----
    {
      unsigned long long* slotP =
          cok[XL] ? xb + (int64_t)((2 * XL + (gsl[XL] & 1)) * G) * X.SZ : dummy;
#pragma unroll
      for (int h = 0; h < G - 1; ++h) pr_poll(pl[h], slotP + (int64_t)(h < g ? h : h + 1) * X.SZ + tid);
    }
    issue_labels(Xc);
    if (lok[XL]) lok[XL] = sp_advance<true>(lc[XL], P, 2 * grp + XL, nvg, T);
    fetch_perm(Xc);
    PR_STAMP(9)

    // ---- [G] lane Y: loss, backward (+ P3 of lane X's next rows), update.  The backward's MFMAs
    // run whether or not Y has a step pending (their result is then dropped), so the row
    // loads sit in ONE code path: their destinations never meet a control-flow merge while
    // in flight (scripts/asm_audit.py) ----
    float npn = 0.f, nwn = 0.f;
    const float pn2 = nrm[0], wn2 = nrm[1];
    if (pend[YL] && g == 0 && tid == 0 && e == E - 1) {
      float ce = 0.f;
      for (int i = 0; i < NW; ++i) ce += wce[i];
      float loss = ce / (float)bc;
      if (P.prox) loss = loss + P.mu * sqrtf(pn2);
      if (P.reg) loss = loss + P.lam * sqrtf(wn2);
      lsum[YL] += (double)loss * (double)bc;
    }
    // A operand lane (l16, lg) = image row 4 kk + lg, block 4 (l16 & 3) + (l16 >> 2), so
    // output register q of lane (c, lg) is the gradient of d = 16 q + 4 lg + e (the lane's W)
    float gB[4 * RT];
#pragma unroll
    for (int kk = 0; kk < 4 * RT; ++kk) gB[kk] = gbuf[4 * kk + lg][l16];
    const int rblk = 4 * (l16 & 3) + (l16 >> 2);
    const float* img = xs_lds + YL * NR * RS;
    floatx4 ga[4];
#pragma unroll
    for (int e4 = 0; e4 < 4; ++e4) ga[e4] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4 * RT; ++kk) {
      const float4 x = ld4(img + img_off(4 * kk + lg, RS, w, rblk));
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) ga[e4] = mfma4(comp(x, e4), gB[kk], ga[e4]);
      if ((kk & 3) == 3) piece(Xc, NP / 2 + (kk >> 2));    // P3
    }
    if (pend[YL]) {
      const float sp = (P.prox && pn2 > 0.f) ? P.mu / sqrtf(pn2) : 0.f;
      const float sr = (P.reg && wn2 > 0.f) ? P.lam / sqrtf(wn2) : 0.f;
      const float lr = P.lr;
      if (cl) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float o[4];
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) {
            const float wc = comp(wr[YL][q], e4);
            const float ac = PROX ? comp(ws[q], e4) : 0.f;
            o[e4] = sgd_w(wc, ga[e4][q], lr, PROX, ac, sp, P.reg, sr);
            if (PROX) {                            // (without a prox term: below, if ridge)
              const float dp = o[e4] - ac;
              npn = sq_acc(npn, dp);
              nwn = sq_acc(nwn, o[e4]);
            }
          }
          wr[YL][q] = make_float4(o[0], o[1], o[2], o[3]);
        }
      }
      // the norms feed only the prox / ridge terms; ridge alone sums ||W||^2 here in the
      // update's own order (q, e4: the split form's bits; padding lanes hold zeros)
      if (!PROX && P.reg) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) nwn = sq_acc(nwn, comp(wr[YL][q], e4));
      }
      if (PROX || P.reg) {
        npn = PROX ? wave_sum_dpp(npn, lane) : 0.f;
        nwn = wave_sum_dpp(nwn, lane);
        if (lane == 0) { wred[YL][w][0] = npn; wred[YL][w][1] = nwn; }
      }
      if (st == cc[YL].steps - 1) {               // client end
        if (cl) {
          float* Wj = P.W_out + (int64_t)cc[YL].j * C * ld + wbase;
#pragma unroll
          for (int q = 0; q < 4; ++q) st4(Wj + 16 * q, wr[YL][q]);
        }
        if (g == 0 && tid == 0) P.loss[cc[YL].j] = lsum[YL] / (double)n;
      }
      const int kprev = cc[YL].k;
      cok[YL] = sp_advance<true>(cc[YL], P, 2 * grp + YL, nvg, T);
      flush_empty(YL, kprev + 1, cok[YL] ? cc[YL].k : T);
      if (cok[YL] && cc[YL].st == 0) {            // next client of the lane: restart from W_start
#pragma unroll
        for (int q = 0; q < 4; ++q) wr[YL][q] = ws[q];
        lsum[YL] = 0.0;
        if (lane == 0) { wred[YL][w][0] = 0.f; wred[YL][w][1] = nw0; }
      }
      pend[YL] = false;
      ++gsl[YL];
    }
    pend[XL] = cok[XL];                           // lane X's forward is published: complete it next
    PR_STAMP(10)
  };

  while (cok[0] || cok[1] || pend[0] || pend[1]) {
    half(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
    half(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
  }
  pr_wait<0>();                                   // nothing of ours is in flight at the exit
#ifdef FS_STAMPS
  if (tid == 0 && X.stamps) {
    for (int k = 0; k < 10; ++k) X.stamps[blockIdx.x * 16 + k] = stamp_acc[k];
    X.stamps[blockIdx.x * 16 + 15] = (unsigned long long)nhalf;
  }
#endif
  if (dead && tid == 0) __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static int pair_rt(int B) { return B <= 16 ? 1 : 2; }

static size_t pair_dyn_lds(int RT) { return sizeof(float) * 2 * (size_t)(RT * 16) * (size_t)(PR_TILES * 64 + 8); }

static size_t pair_static_lds(int RT) {
  const int NR = RT * 16;
  return (size_t)PR_WAVES * NR * 16 * 4 + (size_t)NR * 16 * 4 + 2 * NR * 4 + 2 * PR_WAVES * 2 * 4 +
         PR_WAVES * 4 + 8 + 64;
}

// can the pair kernel run this shape with groups of G workgroups?
bool pair_fits(int C, int B, int NT, int G) {
  if (!(G == 2 || G == 4 || G == 8 || G == 16)) return false;
  // C <= 14: the two norms travel at classes 14 and 15 of row 0 of the (row, class) hand-off
  if (C > 14 || B > 32 || NT != PR_TILES * G) return false;
  const int RT = pair_rt(B);
  return pair_dyn_lds(RT) + pair_static_lds(RT) <= 160 * 1024;
}

static int pair_sz(int RT) { return RT * 16 * 16 + 4 >= PR_THREADS ? RT * 16 * 16 + 4 : PR_THREADS; }

// groups in flight: one per G CUs, two clients each
int pair_groups(int N, int G, int cus) { return std::max(1, std::min((N + 1) / 2, cus / G)); }

int64_t pair_ws_bytes(int N, int G, int B, int cus) {
  return (int64_t)pair_groups(N, G, cus) * 5 * G * pair_sz(pair_rt(B)) * 8 + PR_ERR_BYTES;
}

template <int RT, int G, bool PROX>
static void launch_pair_s(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&local_train_pair_kernel<RT, G, PROX>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((local_train_pair_kernel<RT, G, PROX>), dim3(grid), dim3(PR_THREADS), lds, st, P, X);
}

template <int RT, int G>
static void launch_pair_g(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  if (P.prox) launch_pair_s<RT, G, true>(P, X, grid, lds, st);
  else launch_pair_s<RT, G, false>(P, X, grid, lds, st);
}

int launch_local_train_pair(const LTParams& P, int G, void* ws, int64_t ws_bytes, hipStream_t st) {
  const int RT = pair_rt(P.B);
  const int NT = (int)(P.ld >> 6);
  if (P.chained) return fail(FS_EINVAL, "fs_local_train: the pair form needs parallel clients");
  if (!pair_fits(P.C, P.B, NT, G))
    return fail(FS_EUNSUPPORTED, "fs_local_train: the pair form needs C <= 14, B <= 32 and ld == 512 G");
  const int cus = device_cus();
  if (cus <= 0) return fail(FS_EHIP, "fs_local_train: no device");
  if (G > cus) return fail(FS_EUNSUPPORTED, "fs_local_train: G exceeds the CU count");
  const int ng = pair_groups(P.N, G, cus);
  const int SZ = pair_sz(RT);
  const int64_t xbytes = (int64_t)ng * 5 * G * SZ * 8;
  if (!ws || ws_bytes < xbytes + PR_ERR_BYTES) return fail(FS_EINVAL, "fs_local_train: workspace too small");
  char* base = reinterpret_cast<char*>(ws);
  SplitWS X;
  X.xbuf = reinterpret_cast<unsigned long long*>(base);
  X.err = reinterpret_cast<unsigned*>(base + ws_bytes - PR_ERR_BYTES);
  X.SZ = SZ;
  X.ngroups = ng;
  {
    const fs_tuning t = tuning();
    X.spin_limit = t.inject_timeout ? 0u : (t.spin_limit ? t.spin_limit : PR_SPIN_LIMIT);
  }
  X.poll_delay = 0;                    // (the pair form polls half a step after publishing)
  X.stamps = nullptr;
#ifdef FS_STAMPS
  X.stamps = reinterpret_cast<unsigned long long*>(base + xbytes);
#endif
  // lanes walk ceil(N / 2 ng) clients each
  const int64_t lane_clients = (P.N + 2 * ng - 1) / (2 * ng);
  const bool long_launch = P.max_client_steps <= 0 || P.max_client_steps * lane_clients >= (1 << 20) - 1;
  const unsigned gen = exchange_generation(ws, long_launch);
  X.tag_base = gen << 20;
  if (gen <= 1) {
    hipError_t e = hipMemsetAsync(base, 0, (size_t)xbytes, st);
    if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_local_train: ") + hipGetErrorString(e));
  }
  const size_t lds = pair_dyn_lds(RT);
  if (P.fuse_E > 0 && ng * G + P.fuse_E > cus) return fail(FS_EINVAL, "fs_local_train: no room for the fused evaluation");
  const int grid = ng * G + P.fuse_E;
#define FS_PAIR_CASE(rt, g) \
  if (RT == rt && G == g) { launch_pair_g<rt, g>(P, X, grid, lds, st); return FS_OK; }
  FS_PAIR_CASE(2, 2) FS_PAIR_CASE(2, 4) FS_PAIR_CASE(2, 8) FS_PAIR_CASE(2, 16)
  FS_PAIR_CASE(1, 2) FS_PAIR_CASE(1, 4) FS_PAIR_CASE(1, 8) FS_PAIR_CASE(1, 16)
#undef FS_PAIR_CASE
  return fail(FS_EUNSUPPORTED, "fs_local_train: no pair kernel for this shape");
}

}  // namespace fs
