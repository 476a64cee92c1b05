// Double-buffered split-client local training (round 6): the split
// form of local_train_split.hip -- a group of G workgroups trains one client at a time, each owning
// a slice of the feature tiles, the G partial logits exchanged per step as {tag, value} granules --
// with the batch rows streamed ahead of the hand-off: each wave's last tile two steps ahead into a
// second register buffer, its other tiles one step ahead.
//
// Same math as train_loop (/root/reference/functions/tools.py:177-215), and the same arithmetic in
// the same order as the split form (the forward's MFMA chain tile by tile, the hand-off's sums in
// slice order, the softmax, the backward and the update through split_common.h's fma helpers), so
// its weights and losses are BITWISE the split form's (tests/test_gpu_dbuf.py).
//
// Why: in the split form a step's next-step rows can only be issued after its
// hand-off polls return (a poll issued behind row loads returns only after them: one in-order
// vector-memory path per CU) and must have landed by the next forward -- about 9 k cycles for
// 128 KB per CU at config 2's width, below the ~12 k the per-CU stream needs, so the forward and
// the S1 barrier waited ~6 k cycles per step for rows.  Here the rows of step s + 2 go out after
// step s's polls into the register buffer step s has just written to its LDS image, so they have
// from one poll return to the next (a whole step) to land; the forward finds its rows in
// registers.  The poll wait of step s + 1 retires them (in-order), so a step never waits for a
// row load by itself.
//
// Every in-loop global load is inline asm tagged as the pair / pipe forms' (`; pr-row`,
// `; pr-idx`, `; pr-poll`), invisible to hipcc's vmcnt bookkeeping, and retired by hand-counted
// waits; each destination is named `; pr-own` after the wait that retires it, and
// scripts/asm_audit.py checks the built code object for any touch of a destination in between.
// The client tables are read with scalar loads (lgkmcnt): the cursor never waits for the row
// stream.  Per step a wave issues, in this order:
//   [client start of a parallel client: 4 TPW weight loads, drained at once]
//   M publish stores                         (compiler stores: only make a wait stricter)
//   M * G polls                              [wait 0: the polls AND everything older -- the rows,
//                                             labels and indices of the steps ahead -- landed]
//   [PROX: 4 TPW anchor loads]  RT index loads (step s + 3)  RT label loads (step s + 2)
//   E1 row loads (step s + 2)   NLD - E1 row loads, one per backward iteration
// so the anchor of tile i is retired by vmcnt(2 RT + E1 + the row loads of tiles 0..i).
// Shapes: full slices (NTS = WAVES * TPW tiles per workgroup), 16 < B <= 32 (two row tiles),
// C <= 16; WAVES x TPW = 8 x 2 (the split form's parallel widths) or 4 x 1 (the narrow chained
// instance of exp.py's config 1).
#include <type_traits>

#include "common.h"
#include "eval_rows.h"
#include "lanes.h"
#include "split_common.h"

namespace fs {

template <int OFF>
__device__ __forceinline__ void db_ld4(floatx4& d, const float* p) {
  asm volatile("global_load_dwordx4 %0, %1, off offset:%2 ; pr-row" : "=v"(d) : "v"(p), "n"(OFF) : "memory");
}
__device__ __forceinline__ void db_ld1(int& d, const int32_t* p) {
  asm volatile("global_load_dword %0, %1, off ; pr-idx" : "=v"(d) : "v"(p) : "memory");
}
// a poll: the partner's slot base in SGPRs (wave-uniform), the granule's byte offset in one VGPR
// shared by every partner (no 64-bit address per partner held in VGPRs).  The s_nop 4 is the
// 5 wait states a VMEM read of an SGPR needs after a VALU write of it: hipcc restores spilled
// SGPRs with v_readlane right before their use and does not pad inline-asm VMEM for it (without
// the pad the load read a stale base: an illegal address, round 6)
__device__ __forceinline__ void db_poll(unsigned long long& d, const unsigned long long* base, unsigned voff) {
  asm volatile("s_nop 4\n\tglobal_load_dwordx2 %0, %1, %2 sc1 ; pr-poll" : "=v"(d) : "v"(voff), "s"(base) : "memory");
}
template <int N>
__device__ __forceinline__ void db_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" : : "n"(N) : "memory");
}
template <typename T>
__device__ __forceinline__ void db_own(T& x) {
  asm volatile("; pr-own %0" : "+v"(x));
}

// Diagnostic build only (-DFS_STAMPS): per-phase cycle sums of wave 0 of every workgroup
#ifdef FS_STAMPS
#define DB_STAMP(k)                                                                       \
  {                                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    unsigned long long t_;                                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    if (k > 0) stamp_acc[k > 0 ? k - 1 : 0] += t_ - stamp_prev;                           \
    stamp_prev = t_;                                                                      \
  }
#else
#define DB_STAMP(k)
#endif

// Diagnostic build only (-DDB_CHECK, scripts/build_variant.sh): every global address of the step is
// checked against its buffer's bounds first; a bad one is replaced by a safe address and reported
// through the workspace error word (bits above the timeout's 1: 0x100 rows, 0x200 labels, 0x400
// indices, 0x800 polls, 0x1000 publish, 0x2000 client results)
#ifdef DB_CHECK
#define DB_CHK(ok, bit, fix)                                                              \
  if (!(ok)) {                                                                            \
    __hip_atomic_fetch_or(X.err, (unsigned)(bit), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
    fix;                                                                                  \
  }
#else
#define DB_CHK(ok, bit, fix)
#endif

// row loads issued right after the hand-off (the rest one per backward iteration).  Measured
// (profiles/r06/dbuf_early_depth.txt, launch us, config 2 / config 5): 0 293-297 / 5,140-5,152;
// 2 283-287 / 4,939-4,940; 4 282.6-282.7 / 4,755-4,762; 6 287-291 / 4,769-4,782 (a burst of
// 6 + 2 + 2 loads per wave right after the polls takes ~1.4 k cycles to issue: 80 KB of requests
// at the CU's vector-memory issue rate); the split form 283.8-285.9 / 4,763-4,776
#ifndef DB_E1
#define DB_E1 4
#endif

// f(integral_constant<int, 0>), ..., f(integral_constant<int, N - 1>): compile-time indices for
// the unrolled issue pattern (C++17: no template lambdas)
template <typename F, int... I>
__device__ __forceinline__ void db_seq_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void db_seq(F&& f) {
  db_seq_impl(f, std::make_integer_sequence<int, N>{});
}

template <int RT, int G, bool PROX, int WAVES, int TPW>
__global__ __launch_bounds__(WAVES * 64, 1) void local_train_dbuf_kernel(LTParams P, SplitWS X) {
  static_assert(RT == 2, "two 16-row tiles (16 < B <= 32)");
  static_assert((WAVES == 8 && TPW == 2) || (WAVES == 4 && TPW == 1), "shapes");
  constexpr int NW = WAVES, NTH = NW * 64, NC = 16, NR = RT * 16, NZ = NR * NC;
  constexpr int NTS = NW * TPW;                   // full slices only
  constexpr int RS = NTS * 64 + 8;                // LDS image row stride (floats)
  constexpr int XT = NTH;
  constexpr int M = ((G >= 8 ? 512 : NZ + 2) + XT - 1) / XT;
  constexpr int HC = G;
  constexpr int NLD = TPW * 4 * RT;               // row loads per wave and step
  constexpr int E1 = DB_E1 < NLD ? DB_E1 : NLD;
  // tile stride of a wave's tiles (w, w + NW): NW * 64 floats -- in bytes, as load offsets
  constexpr int TSTR = NW * 64 * 4;
  __shared__ __attribute__((aligned(16))) float zpart[NW][NR * NC];
  __shared__ float gbuf[NR][NC];
  __shared__ float zsum[NR][NC];
  __shared__ int lab[2][NR];
  __shared__ float wred[NW][2];
  __shared__ float wce[NW];
  __shared__ float nrm[2];
  extern __shared__ __attribute__((aligned(16))) float xs_dyn[];   // [NR][RS] batch slice image

  const int tid = (int)threadIdx.x, lane = tid & 63, l16 = lane & 15, lg = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t ld = P.ld;
  const int NT = (int)(ld >> 6);
  const int C = P.C, B = P.B, E = P.E;
  const int NV = NR * C + 2;

  // block -> (group, slice) and the fused evaluation blocks: as the split form
  const int nb = gridDim.x - P.fuse_E;
  if ((int)blockIdx.x >= nb) {
    if constexpr (WAVES == 8)
      eval_persistent<8>(P.fuse_phi, P.ld, P.fuse_y, P.fuse_n, P.W_start, P.C, (int)blockIdx.x - nb, P.fuse_E, xs_dyn,
                         P.fuse_part);
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
  const int t0 = tile_lo(g, G, NT);               // the host guarantees t1 - t0 == NTS
  const float* start = P.W_start;
  unsigned long long* xb = X.xbuf + (int64_t)grp * 2 * G * X.SZ;
  const floatx4 zero4 = floatx4{0.f, 0.f, 0.f, 0.f};
#ifdef DB_CHECK
  const int64_t chk_rows = tab_i64(P.row_off, P.N);
  const int64_t chk_xb = (int64_t)ng * 2 * G * X.SZ;
#endif

  // ---- weights of this slice in registers: lane (c, lg) holds W[c][64 T + 16 q + 4 lg + e] ----
  floatx4 wr[TPW][4];
  // (the weight addresses are rebuilt behind an empty asm at every use: client boundaries only)
  auto wbase = [&]() {
    int64_t b = (int64_t)l16 * ld + 64 * t0 + 4 * lg + 64 * w;
    asm volatile("" : "+v"(b));
    return b;
  };
  // the round-start model as counted loads (lanes of padding classes read class C - 1's row --
  // every load unconditional -- and are zeroed), drained at once: client starts only
  auto load_start = [&]() {
    int64_t b = (int64_t)min(l16, C - 1) * ld + 64 * t0 + 4 * lg + 64 * w;
    asm volatile("" : "+v"(b));
    const float* src = start + b;
    db_ld4<0>(wr[0][0], src); db_ld4<64>(wr[0][1], src); db_ld4<128>(wr[0][2], src); db_ld4<192>(wr[0][3], src);
    if constexpr (TPW > 1) {
      db_ld4<TSTR>(wr[1][0], src); db_ld4<TSTR + 64>(wr[1][1], src); db_ld4<TSTR + 128>(wr[1][2], src);
      db_ld4<TSTR + 192>(wr[1][3], src);
    }
    db_wait<0>();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        db_own(wr[i][q]);
        if (l16 >= C) wr[i][q] = zero4;
        s = sq4_acc(s, wr[i][q][0], wr[i][q][1], wr[i][q][2], wr[i][q][3]);
      }
    return wave_sum_dpp(s, lane);
  };
  auto store_w = [&](float* Wj) {
    const int64_t base = wbase();
    if (l16 < C)
#pragma unroll
      for (int i = 0; i < TPW; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) st4(Wj + base + 64 * NW * i + 16 * q, make_float4(wr[i][q][0], wr[i][q][1], wr[i][q][2], wr[i][q][3]));
  };
  const float nw0 = load_start();
  if (lane == 0) { wred[w][0] = 0.f; wred[w][1] = nw0; }

  // ---- rows: lane (l16, lg) holds row 16 rt + l16, columns 64 T + 16 q + 4 lg .. +3 of each of its
  // tiles.  The LAST tile of a wave (i = TPW - 1) is double-buffered by step parity (xd[Q]) and
  // streamed two steps ahead; the others (i < TPW - 1, xs) one step ahead -- issued first after the
  // polls, so they land (64 KB per CU at config 2's width) well before the next forward, and the
  // second buffer costs TPW = 2's register budget 32 VGPRs instead of 64 ----
  constexpr int NS = TPW - 1;                     // single-buffered tiles per wave
  constexpr int NLS = NS * 4 * RT;                // their row loads per step (issued first)
  floatx4 xs[NS > 0 ? NS : 1][RT][4];
  floatx4 xd[2][RT][4];
  int lbv[2][RT];                                 // labels of the step two ahead (by its parity)
  int pnA[RT], pnB[RT], raw[RT];                  // row indices of steps s + 1 and s + 2; raw in flight
  int64_t rbase = 0;                              // raw's client first row
  bool rvalid = false;                            // raw addresses a real step
  SpCur lc;                                       // the step raw was (is next) fetched for
  bool lc_ok = sp_seek<true>(lc, P, grp, ng, T, 0);
  // RT index loads of cursor lc's step (unconditional: a dummy valid address past the sequence)
  auto fetch_raw = [&]() {
    const int e_ = lc_ok ? lc.st / lc.nbat : 0, s_ = lc_ok ? lc.st - e_ * lc.nbat : 0;
    const int b0_ = s_ * B, bc_ = lc_ok ? min(B, lc.n - b0_) : 1;
    const int32_t* pp_ = lc_ok ? P.perms + (int64_t)E * lc.row0 + (int64_t)e_ * lc.n + b0_ : P.perms;
    rbase = lc_ok ? lc.row0 : 0;
    rvalid = lc_ok;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int32_t* a_ = pp_ + (rt * 16 + l16 < bc_ ? rt * 16 + l16 : 0);
      DB_CHK(a_ >= P.perms && a_ < P.perms + (int64_t)E * chk_rows, 0x400, a_ = P.perms)
      db_ld1(raw[rt], a_);
    }
  };
  // (after the wait that retires raw) pnA <- pnB, pnB <- raw's step's row indices -- or, past the
  // sequence, pnB kept (valid rows of this launch)
  auto take_raw = [&]() {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      db_own(raw[rt]);
      pnA[rt] = pnB[rt];
      pnB[rt] = rvalid ? (int)(rbase + raw[rt]) : pnB[rt];
    }
  };
  auto issue_labels = [&](auto PB) {
    constexpr int Q = decltype(PB)::value;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      int r_ = pnB[rt];
      DB_CHK(r_ >= 0 && r_ < chk_rows, 0x200, r_ = 0)
      db_ld1(lbv[Q][rt], P.labels + r_);
    }
  };
  // the register of (tile i, row tile rt, q): the single buffer, or the last tile's buffer Q
  auto xr = [&](auto PB, auto IC, int rt, int q) -> floatx4& {
    constexpr int Q = decltype(PB)::value, i = decltype(IC)::value;
    if constexpr (i == TPW - 1) return xd[Q][rt][q];
    else return xs[i][rt][q];
  };
  // row load f (0 .. NLD-1) after step s's polls: f < NLS the single tiles of step s + 1 (pnA),
  // then the last tile of step s + 2 (pnB) into buffer Q
  auto issue_row = [&](auto PB, auto F) {
    constexpr int f = decltype(F)::value;
    constexpr int i = f / (4 * RT), kk = f % (4 * RT), rt = kk >> 2, q = kk & 3;
    int r_ = i == TPW - 1 ? pnB[rt] : pnA[rt];
    DB_CHK(r_ >= 0 && r_ < chk_rows, 0x100, r_ = 0)
    const float* src = P.phi + (int64_t)r_ * ld + 64 * t0 + 4 * lg + 64 * w;
    db_ld4<i * TSTR + 64 * q>(xr(PB, std::integral_constant<int, i>{}, rt, q), src);
  };
  auto own_last = [&](auto PB) {
    constexpr int Q = decltype(PB)::value;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      db_own(lbv[Q][rt]);
#pragma unroll
      for (int q = 0; q < 4; ++q) db_own(xd[Q][rt][q]);
    }
  };
  auto own_single = [&]() {
#pragma unroll
    for (int i = 0; i < NS; ++i)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int q = 0; q < 4; ++q) db_own(xs[i][rt][q]);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // prologue: step 0's labels and rows (all tiles), step 1's labels and last tile, step 2's
  // indices in flight (step 1's single tiles go out after step 0's polls, as in every step)
  for (int rt = 0; rt < RT; ++rt) pnB[rt] = 0;
  fetch_raw();
  db_wait<0>();
  take_raw();                                     // pnB = step 0
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) pnA[rt] = pnB[rt];
  issue_labels(I0{});
  db_seq<NLD>([&](auto F) { issue_row(I0{}, F); });
  if (lc_ok) lc_ok = sp_advance<true>(lc, P, grp, ng, T);
  fetch_raw();
  db_wait<0>();
  take_raw();                                     // pnB = step 1
  own_last(I0{});
  own_single();
  issue_labels(I1{});
  db_seq<4 * RT>([&](auto F) { issue_row(I1{}, std::integral_constant<int, NLS + decltype(F)::value>{}); });
  if (lc_ok) lc_ok = sp_advance<true>(lc, P, grp, ng, T);
  fetch_raw();
  lds_barrier();

  // clients with no step (n_j = 0 or E = 0): the result is the client's start (as the split form)
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
              const int64_t off = base + 64 * NW * i + 16 * q;
              st4(Wj + off, ld4(start + off));
            }
      }
      if (g == 0 && tid == 0) P.loss[j] = 0.0;
    }
  };

  SpCur cc;
  bool cc_ok = sp_seek<true>(cc, P, grp, ng, T, 0);
  flush_empty(0, cc_ok ? cc.k : T);
  unsigned gs = 0;
  bool dead = false;
  double lsum = 0.0;
  const float* anc = P.W_start;                   // PROX: the anchor of the current client
  const int rblk = 4 * (l16 & 3) + (l16 >> 2);
#ifdef FS_STAMPS
  unsigned long long stamp_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, stamp_prev = 0;
#endif

  // one step of the group's sequence on buffer Q (= the step's parity)
  auto step = [&](auto PB) {
    constexpr int Q = decltype(PB)::value;
    DB_STAMP(0)
    const int st = cc.st, n = cc.n, nbat = cc.nbat;
    if (st == 0) {
      // client start: parallel clients restart from W_start (the first one is loaded); chained
      // ones keep the registers.  The prox anchor is the start (tools.py:180).
      if (!P.chained && gs > 0) {
        (void)load_start();
        if (lane == 0) { wred[w][0] = 0.f; wred[w][1] = nw0; }
      } else if (lane == 0) {
        wred[w][0] = 0.f;                         // ||W - W_a|| = 0 at the new anchor
      }
      if (PROX) anc = (P.chained && cc.j > 0) ? P.W_out + (int64_t)(cc.j - 1) * C * ld : start;
      lsum = 0.0;
    }
    const int e = st / nbat, s = st - e * nbat;
    const int bc = min(B, n - s * B);
    const int par = gs & 1;
    const unsigned tag32 = X.tag_base + gs + 1u;
    // this step's last tile and labels landed at the previous step's poll wait (retire()); named
    // again here for scripts/asm_audit.py, which cannot rule out the path from this step's own
    // issue through the loop's exit test back to this point (the exit test always leaves there)
    own_last(PB);
    if (w == 0 && lg == 0)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) lab[par][rt * 16 + l16] = lbv[Q][rt];

    // ---------------- forward partial: z_g = X_slice W_slice^T (rows in registers) ----------------
    // the single tiles of this step went out after the previous step's polls, the last tile's rows
    // were retired by them: behind the single tiles' loads only the last tile's of step s + 1
    if constexpr (NS > 0) {
      db_wait<4 * RT>();
      own_single();
    }
    floatx4 acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = floatx4{0.f, 0.f, 0.f, 0.f};
    db_seq<TPW>([&](auto IC) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        floatx4 xa[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) xa[rt] = xr(PB, IC, rt, q);
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma4(xa[rt][e4], wr[decltype(IC)::value][q][e4], acc[rt]);
      }
    });
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      st4(&zpart[w][rt * 256 + lg * 64 + l16 * 4], make_float4(acc[rt][0], acc[rt][1], acc[rt][2], acc[rt][3]));
    DB_STAMP(1)
    lds_barrier();  // S1: wave partials, norm partials of the previous update; the image is free
    DB_STAMP(2)

    {
      // ---- hand-off: the split form's, polls as counted loads ----
      unsigned long long* slot = xb + ((int64_t)par * G) * X.SZ;
      const unsigned long long tag = (unsigned long long)tag32 << 32;
      float own[M], sum[M];
      unsigned long long pl[M][HC];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int idx = tid + XT * m;
        float v = 0.f;
        if (idx < NV - 2) {
          const int r = idx / C, c = idx - r * C;
#pragma unroll
          for (int i = 0; i < NW; ++i) v += zpart[i][zp_off(r, c)];
        } else if (idx < NV) {
#pragma unroll
          for (int i = 0; i < NW; ++i) v += wred[i][idx - (NV - 2)];
        }
        own[m] = v;
        sum[m] = 0.f;
        DB_CHK(idx >= NV || (slot - X.xbuf) + (int64_t)g * X.SZ + idx < chk_xb, 0x1000, continue)
        if (idx < NV)
          __hip_atomic_store(slot + (int64_t)g * X.SZ + idx, tag | __float_as_uint(v), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      DB_STAMP(3)
      if (X.spin_limit == 0 && gs == 0 && lane == 0)      // test knob: report an injected timeout
        __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      auto poll = [&]() {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const int idx = tid + XT * m;
          unsigned voff = 8u * (unsigned)(idx < NV ? idx : 0);
#pragma unroll
          for (int h = 0; h < HC; ++h) {
            DB_CHK((slot - X.xbuf) + (int64_t)h * X.SZ + voff / 8 < chk_xb && slot >= X.xbuf, 0x800, voff = 0)
            db_poll(pl[m][h], slot + (int64_t)h * X.SZ, voff);
          }
        }
      };
      for (int d_ = 0; d_ < X.poll_delay; ++d_) __builtin_amdgcn_s_sleep(1);
      poll();
      // image write (this buffer's rows; each wave only ever touches the image of its own tiles)
      db_seq<TPW>([&](auto IC) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const floatx4 v = xr(PB, IC, rt, q);
            st4(xs_dyn + img_off(rt * 16 + l16, RS, w + NW * decltype(IC)::value, 4 * q + lg),
                make_float4(v[0], v[1], v[2], v[3]));
          }
      });
      // (each poll's wait follows it in the same block: a re-poll's results are named before the
      // loop's back edge, so no copy the compiler places there can read a register in flight)
      auto retire = [&]() {
        db_wait<0>();                               // the polls -- and every older load -- landed
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
          for (int h = 0; h < HC; ++h) db_own(pl[m][h]);
      };
      retire();
      unsigned spins = 0;
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
          for (int h = 0; h < HC; ++h)
            ok &= (h == g) | (tid + XT * m >= NV) | ((unsigned)(pl[m][h] >> 32) == tag32);
        if (__all(ok)) break;
        if (dead || ++spins > X.spin_limit) {
          if (lane == 0) __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          dead = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        poll();
        retire();
      }
      // the last tile and labels of step s + 1 and the indices of step s + 2 landed with the polls
      own_last(std::integral_constant<int, Q ^ 1>{});
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int h = 0; h < HC; ++h) sum[m] += (h == g) ? own[m] : __uint_as_float((unsigned)pl[m][h]);
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int idx = tid + XT * m;
        if (idx < NV) {
          if (idx < NV - 2) {
            const int r = idx / C, c = idx - r * C;
            zsum[r][c] = sum[m];
          } else {
            nrm[idx - (NV - 2)] = sum[m];         // ||W - W_a||^2, ||W||^2 at the start of this step
          }
        }
      }
      DB_STAMP(4)
    }
    // ---- after the hand-off: the anchor (PROX), the indices of step s + 3, the labels and the
    // first E1 rows of step s + 2 (this buffer, free since the image write) ----
    floatx4 av[PROX ? TPW : 1][4];
    if constexpr (PROX) {
      int64_t b = (int64_t)min(l16, C - 1) * ld + 64 * t0 + 4 * lg + 64 * w;
      asm volatile("" : "+v"(b));
      const float* ap = anc + b;
      db_ld4<0>(av[0][0], ap); db_ld4<64>(av[0][1], ap); db_ld4<128>(av[0][2], ap); db_ld4<192>(av[0][3], ap);
      if constexpr (TPW > 1) {
        db_ld4<TSTR>(av[1][0], ap); db_ld4<TSTR + 64>(av[1][1], ap); db_ld4<TSTR + 128>(av[1][2], ap);
        db_ld4<TSTR + 192>(av[1][3], ap);
      }
    }
    take_raw();                                   // pnA = step s + 1, pnB = step s + 2 (landed with the polls)
    if (lc_ok) lc_ok = sp_advance<true>(lc, P, grp, ng, T);
    fetch_raw();                                  // step s + 3's indices
    issue_labels(PB);                             // step s + 2's labels
    db_seq<E1>([&](auto F) { issue_row(PB, F); });
    DB_STAMP(5)
    lds_barrier();  // S2: summed logits and norms, the image
    DB_STAMP(6)
    const float invb = 1.0f / (float)bc;
    float cep = 0.f;
    for (int idx = tid; idx < NZ; idx += NTH) {
      const int r = idx / NC, c = idx - r * NC;
      const bool valid = r < bc && c < C;
      const float z = valid ? zsum[r][c] : 0.f;
      float mx = valid ? z : -INFINITY;
#pragma unroll
      for (int off = NC / 2; off > 0; off >>= 1) mx = fmaxf(mx, xor_get(mx, off, lane));
      const float ex = valid ? __expf(z - mx) : 0.f;
      float se = ex;
#pragma unroll
      for (int off = NC / 2; off > 0; off >>= 1) se += xor_get(se, off, lane);
      float gv = 0.f;
      if (valid) {
        const bool isy = c == lab[par][r];
        gv = (isy ? -invb : 0.f) + ex * __builtin_amdgcn_rcpf(se) * invb;
        if (isy) cep -= z - mx - __logf(se);
      }
      gbuf[r][c] = gv;
    }
    cep = wave_sum_dpp(cep, lane);
    if (lane == 0) wce[w] = cep;
    lds_barrier();  // S3: g, CE partials
    DB_STAMP(7)
    const float pn2 = nrm[0], wn2 = nrm[1];
    if (g == 0 && tid == 0 && e == E - 1) {
      float ce = 0.f;
      for (int i = 0; i < NW; ++i) ce += wce[i];
      float loss = ce / (float)bc;
      if (P.prox) loss = loss + P.mu * sqrtf(pn2);
      if (P.reg) loss = loss + P.lam * sqrtf(wn2);
      lsum += (double)loss * (double)bc;
    }

    // ---------------- backward + update of the register-resident slice ----------------
    float gB[4 * RT];
#pragma unroll
    for (int kk = 0; kk < 4 * RT; ++kk) gB[kk] = gbuf[4 * kk + lg][l16];
    const float sp = (P.prox && pn2 > 0.f) ? P.mu / sqrtf(pn2) : 0.f;
    const float sr = (P.reg && wn2 > 0.f) ? P.lam / sqrtf(wn2) : 0.f;
    const float lr = P.lr;
    float npn = 0.f, nwn = 0.f;
    db_seq<TPW>([&](auto IC) {
            constexpr int i = decltype(IC)::value;
            floatx4 ga[4];
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) ga[e4] = floatx4{0.f, 0.f, 0.f, 0.f};
            const int Tl = w + NW * i;
            const float* ib0 = xs_dyn + lg * RS + 64 * Tl + 4 * (rblk ^ lg);
            const float* ib1 = xs_dyn + lg * RS + 64 * Tl + 4 * (rblk ^ (lg + 4));
            float4 xpre[TPW == 1 ? 4 * RT : 1];
            if constexpr (TPW == 1) {
#pragma unroll
              for (int kk = 0; kk < 4 * RT; ++kk) xpre[kk] = ld4(((kk & 1) ? ib1 : ib0) + 4 * kk * RS);
              __builtin_amdgcn_sched_barrier(0);
            }
            db_seq<4 * RT>([&](auto KC) {
                    constexpr int kk = decltype(KC)::value;
                    const float4 x = TPW == 1 ? xpre[kk] : ld4(((kk & 1) ? ib1 : ib0) + 4 * kk * RS);
#pragma unroll
                    for (int e4 = 0; e4 < 4; ++e4) ga[e4] = mfma4(comp(x, e4), gB[kk], ga[e4]);
                    // iteration it of the wave's backward issues row load it + E1
                    constexpr int f = i * 4 * RT + kk + E1;
                    if constexpr (f < NLD) issue_row(PB, std::integral_constant<int, f>{});
            });
            if constexpr (PROX) {
              // the anchor of tile i: behind it the indices, labels, E1 rows and the rows of tiles 0..i
              constexpr int after = 2 * RT + E1 + ((i + 1) * 4 * RT < NLD - E1 ? (i + 1) * 4 * RT : NLD - E1);
              db_wait<after>();
#pragma unroll
              for (int q = 0; q < 4; ++q) db_own(av[i][q]);
            }
            if (l16 < C) {
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                float o[4];
#pragma unroll
                for (int e4 = 0; e4 < 4; ++e4) {
                  const float wc = wr[i][q][e4];
                  const float ac = PROX ? av[PROX ? i : 0][q][e4] : 0.f;
                  o[e4] = sgd_w(wc, ga[e4][q], lr, PROX, ac, sp, P.reg, sr);
                  if (PROX) {
                    const float dp = o[e4] - ac;
                    npn = sq_acc(npn, dp);
                    nwn = sq_acc(nwn, o[e4]);
                  }
                }
                wr[i][q] = floatx4{o[0], o[1], o[2], o[3]};
              }
            }
    });
    if (!PROX && P.reg) {
#pragma unroll
      for (int i = 0; i < TPW; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) nwn = sq_acc(nwn, wr[i][q][e4]);
    }
    if (PROX || P.reg) {
      npn = PROX ? wave_sum_dpp(npn, lane) : 0.f;
      nwn = wave_sum_dpp(nwn, lane);
      if (lane == 0) { wred[w][0] = npn; wred[w][1] = nwn; }
    }
    DB_STAMP(8)
    if (st == cc.steps - 1) {                     // client end
      DB_CHK(cc.j >= 0 && cc.j < P.N, 0x2000, cc.j = 0)
      store_w(P.W_out + (int64_t)cc.j * C * ld);
      if (g == 0 && tid == 0) P.loss[cc.j] = lsum / (double)n;
    }
    const int kprev = cc.k;
    cc_ok = sp_advance<true>(cc, P, grp, ng, T);
    flush_empty(kprev + 1, cc_ok ? cc.k : T);
    ++gs;
  };
  while (cc_ok) {
    step(I0{});
    if (!cc_ok) break;
    step(I1{});
  }
  db_wait<0>();                                   // nothing of ours is in flight at the exit
#ifdef FS_STAMPS
  if (threadIdx.x == 0 && X.stamps) {
    for (int k = 0; k < 8; ++k) X.stamps[blockIdx.x * 16 + k] = stamp_acc[k];
    X.stamps[blockIdx.x * 16 + 15] = (unsigned long long)gs;
  }
#endif
}

// ---------------------------------------------------------------------------------------------
// host side: called by local_train_split.hip's launcher for the shapes this form covers
// ---------------------------------------------------------------------------------------------
template <int G, bool PROX, int WAVES, int TPW>
static void launch_dbuf_s(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  auto k = &local_train_dbuf_kernel<2, G, PROX, WAVES, TPW>;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(grid), dim3(WAVES * 64), lds, st, P, X);
}

// Does the double-buffered form cover this launch (full slices of 8 x 2 or, chained, 4 x 1 tiles;
// 16 < B <= 32)?  waves_out: its workgroup size in waves.
// (the 8-wave instance with a prox term would spill: its anchor slice is 32 more VGPRs)
bool dbuf_covers(int C, int B, int64_t ld, int G, int chained, int prox, int* waves_out) {
  if (!(G == 2 || G == 4 || G == 8 || G == 16) || C > 16 || B <= 16 || B > 32) return false;
  const int64_t NT = ld >> 6;
  if (NT == (int64_t)G * 16 && !prox) {
    if (waves_out) *waves_out = 8;
    return true;
  }
  if (chained && G >= 4 && NT == (int64_t)G * 4) {
    if (waves_out) *waves_out = 4;
    return true;
  }
  return false;
}

// LDS of one workgroup: the image (dynamic) + the static arrays, checked by the caller's fit test
int launch_local_train_dbuf(const LTParams& P, int G, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  int waves = 0;
  if (!dbuf_covers(P.C, P.B, P.ld, G, P.chained, P.prox, &waves)) return FS_EUNSUPPORTED;
  if (waves == 4) {
    // a 4-wave workgroup asks for 96 KB of LDS so that no two share a CU (as the split form's narrow instances)
    const size_t l4 = std::max(lds, (size_t)96 * 1024);
#define FS_DB4(g)                                                                            \
  if (G == g) {                                                                              \
    if (P.prox) launch_dbuf_s<g, true, 4, 1>(P, X, grid, l4, st);                           \
    else launch_dbuf_s<g, false, 4, 1>(P, X, grid, l4, st);                                 \
    return FS_OK;                                                                            \
  }
    FS_DB4(4) FS_DB4(8) FS_DB4(16)
#undef FS_DB4
    return FS_EUNSUPPORTED;
  }
#define FS_DB8(g)                                                                            \
  if (G == g) {                                                                              \
    launch_dbuf_s<g, false, 8, 2>(P, X, grid, lds, st);                                     \
    return FS_OK;                                                                            \
  }
  FS_DB8(2) FS_DB8(4) FS_DB8(8) FS_DB8(16)
#undef FS_DB8
  return FS_EUNSUPPORTED;
}

}  // namespace fs
