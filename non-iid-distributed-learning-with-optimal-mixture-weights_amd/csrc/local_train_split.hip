// Split-client local training: a GROUP of G workgroups (on G CUs) trains one client at a
// time, each workgroup owning a slice of the feature dimension.
//
// Same math as local_train.hip (train_loop, /root/reference/functions/tools.py:177-215).
// Workgroup g of a group owns a contiguous range of 64-column feature tiles (its "slice");
// wave w owns tiles w, w + 8:
//   * its slice of the client's weights lives in REGISTERS for the whole local training
//     (lane (c, k-slot) holds W[c][64T + 16 q + 4 k + e]), the prox anchor likewise;
//   * each step's gathered batch rows of the slice arrive in REGISTERS in the forward's
//     operand layout (64 contiguous bytes of 16 rows per load), so the forward
//     z_g = X_b,g W_g^T (v_mfma_f32_16x16x4_f32) reads no LDS; the same registers are then
//     written once into a bank-conflict-free LDS image that the backward
//     grad_g^T = X_b,g^T G reads, and are refilled with the NEXT step's rows -- which may
//     belong to the next client of the group's sequence, so the stream never drains at a
//     client boundary;
//   * per step the G partial logits (the B x C real ones only) plus the partial squared
//     norms of W - W_a and W are exchanged through a small global buffer as 8-byte
//     {tag, value} granules -- the write-through (sc1) store / sc1 load hand-off of
//     cdna_hip_programming.md Guideline 16, R2 form (no fences, no flags); every workgroup
//     sums the G partials in the same fixed order, so all of them compute bitwise-identical
//     softmax gradients.
// Work assignment:
//   parallel clients  ngroups = min(N, CUs / G) groups walk the (LPT-ordered) clients in a
//                     snake order, every client starting from W_start -- so any N runs
//                     split, as persistent groups, not just N * G <= CUs;
//   chained clients   ONE group walks clients 0..N-1 in order (reference semantics,
//                     SURVEY Q1): the weights stay in the registers from one client to the
//                     next and only the prox anchor is re-taken, so the strictly sequential
//                     chain runs on G CUs instead of one.
// Co-residency: the G partners spin on each other, so the grid never exceeds the CU count;
// every spin is bounded and a timeout is reported through the workspace error word.
// Hand-off tags are the group's step counter + 1 (32 bits): the exchange buffer is zeroed by
// the launcher before every launch.
#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "common.h"
#include "eval_rows.h"
#include "lanes.h"
#include "split_common.h"

namespace fs {

constexpr int SP_WAVES = 8;
constexpr int SP_TPW = 2;                 // max 64-column tiles per wave (register budget)
constexpr unsigned SP_SPIN_LIMIT = 1u << 22;
constexpr int SP_ERR_BYTES = 256;         // error block at the END of the workspace (never memset)
// next-step row loads per wave issued ahead of the backward: SP_E1 right after the hand-off,
// SP_E2 after the S2 barrier, SP_E3 after S3 (the rest inside the backward)
#ifndef SP_E1
#define SP_E1 6
#endif
#ifndef SP_E2
#define SP_E2 0
#endif
#ifndef SP_E3
#define SP_E3 0
#endif
constexpr int SP_EARLY = SP_E1 + SP_E2 + SP_E3;
// mb instances: the backward's image and g words read one row block ahead (SP_MB_BWD_PF; without
// it the reads waited just in time: config 2 313 -> 288 us per launch, config 5 5.99 -> 5.58 ms,
// profiles/r06/mb_ab.txt), and the next step's tile-0 forward at the step's end (SP_MB_PRE, where
// it fits: PRE_OK in the kernel)
#ifndef SP_MB_RSP
#define SP_MB_RSP 4   // (the mb image's row stride mod 32, RSP in the kernel; 8 = round 6's first form, for A/B)
#endif
#ifndef SP_MB_BWD_PF
#define SP_MB_BWD_PF 1
#endif
#ifndef SP_MB_PRE
#define SP_MB_PRE 1
#endif

// Diagnostic build only (-DFS_STAMPS): per-phase cycle sums of wave 0 of every workgroup,
// written to a side buffer that nothing else reads (never in the shipped library).
#ifdef FS_STAMPS
#define SP_STAMP(k)                                                                       \
  {                                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    unsigned long long t_;                                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    if (k > 0) stamp_acc[k > 0 ? k - 1 : 0] += t_ - stamp_prev;                           \
    stamp_prev = t_;                                                                      \
  }
#else
#define SP_STAMP(k)
#endif

// ---- the mb instances' MFMA pieces (v_mfma_f32_4x4x1_16b_f32; layouts at the kernel) ----
template <int CBSZ, int ABID, int BLGP>
__device__ __forceinline__ floatx4 mfma4x4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, CBSZ, ABID, BLGP);
}
// forward of one 16-column group q of a tile: 4 components x RT row tiles x CB class blocks
template <int Q, int RT, int CB>
__device__ __forceinline__ void mb_fwd_q(floatx4 (&acc)[RT][CB], const float4 (&xt)[RT][4], const float4 (&wt)[CB]) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) acc[rt][cb] = mfma4x4<2, Q, 0>(comp(wt[cb], e), comp(xt[rt][Q], e), acc[rt][cb]);
}
// backward of one batch row: the CB class blocks' gradients of one tile
template <int CB>
__device__ __forceinline__ void mb_bwd_row(floatx4 (&ga)[CB], float a, float g) {
  ga[0] = mfma4x4<0, 0, 4>(a, g, ga[0]);
  if constexpr (CB > 1) ga[1] = mfma4x4<0, 0, 5>(a, g, ga[1]);
  if constexpr (CB > 2) ga[2] = mfma4x4<0, 0, 6>(a, g, ga[2]);
  if constexpr (CB > 3) ga[3] = mfma4x4<0, 0, 7>(a, g, ga[3]);
}
__device__ __forceinline__ void mb_swap32(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void mb_swap16(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
// the four k-group partials of a forward accumulator summed: lane 16 lg + l16 of the result holds
// register mb_perm(lg) of acc (row l16) summed over lg = 0..3, as (k0 + k2) + (k1 + k3)
__device__ __forceinline__ float mb_kgroup_sum(floatx4 a) {
  float r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3];
  mb_swap32(r0, r1);
  mb_swap32(r2, r3);
  float s01 = r0 + r1, s23 = r2 + r3;
  mb_swap16(s01, s23);
  return s01 + s23;
}
__device__ __forceinline__ int mb_perm(int lg) { return ((lg & 1) << 1) | (lg >> 1); }
// offset of (row, class) in a wave's mb partial-logit block [rt][class block][j][l16 ^ 4 cb]: the
// rows of a 16-word segment XOR-swizzled by the class block, so the hand-off's (row, class) reads
// (classes c, c + 4, c + 8 of one row: the same j) fall in different banks; the writes (one
// segment per 16-lane group) stay a permutation of the block's 64 words
template <int CB>
__device__ __forceinline__ int zp_off_mb(int r, int c) {
  return ((r >> 4) * CB + (c >> 2)) * 64 + (c & 3) * 16 + ((r & 15) ^ ((c >> 2) << 2));
}

// Per-lane d mapping inside a 64-column tile (forward operand, weights, gradient):
// lane (l16, lg), register q, component e  <->  d = 16 q + 4 lg + e.  One load instruction
// (fixed q) then reads 64 contiguous bytes of each of 16 rows.
// Schedule: every wave runs the hand-off; no wave issues its next rows in a burst: each issues
// one row load per backward iteration (16 per wave per step), so the issue stalls of a full
// memory queue land between the backward's MFMAs instead of ahead of them.  Measured and
// dropped (round 2, r02f / r02q / r02w): two 4-wave workgroups per CU (two client chains per
// CU); half the waves streaming their next rows during the hand-off while the other half runs
// it; every wave issuing its rows in a burst after the hand-off or after the softmax; a prefix
// of 4 or 8 row loads issued right after the image write -- each slower at every BASELINE shape.
// Round 3: odd groups started half a step late (so half the CUs stream while the other half
// hand off) changed nothing (configs 2 / 4 / 5 within 0.5 %): the row stream is bound per CU,
// not by the chip's HBM.
// TEAMS = 2 (round 4, the "team" form, G | FS_G_TEAMS): the workgroup's 8 waves are two teams
// of 4 (one wave of each per SIMD), each training its own client lane with its own slice
// image, hand-off slots and team-local barriers (an LDS arrival counter, not s_barrier), so
// the two waves of a SIMD are in different phases: one team's hand-off, softmax and barriers
// run beside the other team's MFMAs.  Per wave the work is the split form's at 4 waves per
// slice (TPW = 2 tiles), so a team form at width G holds the registers of the split form at
// width G / 2.
// WAVES / TPWK (round 5): waves per workgroup and tiles per wave.  The shipped forms are 8 waves
// of up to 2 tiles; the NARROW chained instances (exp.py's config 1: D = 2000 -> 32 tiles) give
// every wave exactly one tile -- 4 waves at G = 8 (4 tiles per slice), 8 waves at G = 4 -- so the
// slice is full and the step runs the early row issue with no per-tile guard.  (The 8-wave form
// at 4 tiles per slice left waves 4-7 without a tile and guarded tile 1 of every wave: the
// compiler then waited vmcnt(0) for the whole next-step row stream at that guard's join, inside
// the backward -- 5.4 k of config 1's 12.1 k cycles per step, profiles/r05b/stamps_c1.txt.)
// MBK (round 6, the "mb" instances): 0 = the classes on v_mfma_f32_16x16x4_f32 (padded to 16);
// 1..4 = on v_mfma_f32_4x4x1_16b_f32 in MBK blocks of 4 classes (C = 10 pads to 12, C = 2 to 4).
// The 16-block instruction runs at the f32 MFMA rate, 8 cycles per SIMD with the kernel's operand
// pattern (scripts/probe/mb_fwd_rate.hip, profiles/r06/mb_fwd_rate_probe.txt: one wave's forward
// 1,576 vs 2,048 cycles at C = 10; a probe reusing one register pair issued faster and misled),
// so per step the MFMA cycles scale with ceil(C / 4) / 4: 3/4 at C = 10, 1/2 at C <= 8, 1/4 at C <= 4.
// Operand layouts (checked on one wave against a CPU product, scripts/probe/mb_layout.hip):
//   rows      xf[i][rt][q] as in the 16x16x4 form: lane (l16, lg), component e = X[16 rt + l16][16 q + 4 lg + e]
//   weights   wr[i][cb], lane 16 lg + 4 q + j, component e = W[4 cb + j][16 q + 4 lg + e] (the tile's columns)
//   forward   acc[rt][cb] += mfma(A = wr[i][cb].e broadcast from block q of each 16-lane group
//             (cbsz 2, abid q), B = xf[i][rt][q].e): lane 16 lg + l16, register j = the partial
//             logit (row 16 rt + l16, class 4 cb + j) over k-group lg; the four k-groups are summed
//             with v_permlane32_swap / v_permlane16_swap (mb_kgroup_sum)
//   backward  ga[i][cb] += mfma(A = image row r, lane 16 lg + 4 q + e at column 16 q + 4 lg + e,
//             B = g row r, lane 16 s + 4 x + j = g[r][4 s + j], broadcast from 16-lane group cb (blgp 4 + cb)):
//             lane 16 lg + 4 q + j, register e = grad[4 cb + j][16 q + 4 lg + e] -- wr's own layout
// Same steps, hand-off, softmax and schedule as the 16x16x4 instances; the products are summed in
// another order (within the fp32 tolerance of the oracle, not bitwise the other forms).
template <int RT, int G, bool PROX, int EARLY, int TEAMS, int WAVES = SP_WAVES, int TPWK = SP_TPW, int MBK = 0>
__global__ __launch_bounds__(WAVES * 64, 1) void local_train_split_kernel(LTParams P, SplitWS X) {
  static_assert(TEAMS == 1 || TEAMS == 2, "teams");
  static_assert(WAVES == SP_WAVES || (WAVES == 4 && TEAMS == 1), "waves");
  static_assert(MBK >= 0 && MBK <= 4 && (MBK == 0 || TEAMS == 1), "mb");
  constexpr bool MB = MBK > 0;
  constexpr int NQ = MB ? MBK : 4;                 // weight registers per tile: q (16x16x4) or class block (mb)
  constexpr int NCS = !MB || MBK > 2 ? 16 : 4 * MBK; // softmax lanes per row (a power of 2 >= the padded classes)
  constexpr int NW = WAVES / TEAMS;                // waves per client lane
  constexpr int NTH = NW * 64;
  constexpr int NC = 16;
  constexpr int NR = RT * 16;
  constexpr int NZ = NR * NC;
  constexpr int NZS = NR * NCS;
  constexpr int TPW = TPWK;
  constexpr int XT = NTH;                         // threads running the hand-off
  // exchanged values per hand-off thread: NR*C logits + 2 norms (G >= 8: NR*C + 2 <= 512)
  constexpr int M = ((G >= 8 ? 512 : NZ + 2) + XT - 1) / XT;
  constexpr int HC = G;                             // partners polled per round trip
  // wave partial logits in the MFMA accumulator's own layout, [rt][lg][class][i] = row
  // 16 rt + 4 lg + i: one conflict-free ds_write_b128 per row tile, and the (row, class)
  // reads of the publish stride 4 words across a 16-lane row (conflict-free too)
  __shared__ __attribute__((aligned(16))) float zpart_t[TEAMS][NW][NR * NC];
  __shared__ float gbuf_t[TEAMS][NR][NC];
  __shared__ float zsum_t[TEAMS][NR][NC];
  __shared__ int lab_t[TEAMS][2][NR];
  __shared__ float wred_t[TEAMS][NW][2];
  __shared__ float wce_t[TEAMS][NW];
  __shared__ float nrm_t[TEAMS][2];
  __shared__ unsigned tbar[TEAMS];                 // team barrier arrival counters
  extern __shared__ __attribute__((aligned(16))) float xs_dyn[];   // TEAMS x [NR][RS] batch slice images

  // team-local thread and wave ids (the whole workgroup when TEAMS == 1)
  // (a compile-time 0 for TEAMS == 1: the split form's addressing stays exactly round 3's)
  const int team = TEAMS > 1 ? __builtin_amdgcn_readfirstlane((int)threadIdx.x / NTH) : 0;
  const int tid = (int)threadIdx.x - team * NTH, lane = tid & 63, l16 = lane & 15, lg = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform for the compiler
  const int mq = (lane >> 2) & 3, mi = lane & 3;            // mb weight lanes: 16 lg + 4 mq + mi
  auto& zpart = zpart_t[team];
  auto& gbuf = gbuf_t[team];
  auto& zsum = zsum_t[team];
  auto& lab = lab_t[team];
  auto& wred = wred_t[team];
  auto& wce = wce_t[team];
  auto& nrm = nrm_t[team];
  const int64_t ld = P.ld;
  const int NT = (int)(ld >> 6);
  const int C = P.C, B = P.B, E = P.E;
  const int NV = NR * C + 2;
  static_assert(NZS % 64 == 0, "the softmax loop must stay wave-uniform");

  // block -> (group, slice).  Chained: 8*G blocks are launched and those with
  // blockIdx % 8 == 0 take part (one XCD under round-robin placement).  Parallel: consecutive
  // linear ids on one XCD, so a group's partners mostly share an L2.  Speed only.
  // fused evaluation blocks (the last fuse_E blocks of a parallel launch): the test-set
  // evaluation of W_start -- the previous round's global model -- on the CUs the groups leave
  // idle, LDS from the (unused) image
  const int nb = gridDim.x - P.fuse_E;
  if ((int)blockIdx.x >= nb) {
    if constexpr (WAVES == SP_WAVES)
      eval_persistent<SP_WAVES>(P.fuse_phi, P.ld, P.fuse_y, P.fuse_n, P.W_start, P.C, (int)blockIdx.x - nb, P.fuse_E,
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
  const int ngp = X.ngroups;                     // groups of G workgroups
  const int grpp = lin / G, g = lin % G;
  if (grpp >= ngp) return;
  // client lanes: TEAMS per group, each with its own client sequence and hand-off slots
  const int ng = ngp * TEAMS, grp = grpp * TEAMS + team;
  const int T = P.chained ? P.N : (P.N + ng - 1) / ng;     // client sequence length
  const int t0 = tile_lo(g, G, NT), t1 = tile_lo(g + 1, G, NT);
  const int NTS = t1 - t0;                       // tiles of this slice
  // LDS row stride (floats): 8 mod 64 for the 16x16x4 image (its swizzle assumes it); 4 mod 32 for
  // the mb image, whose ds_write_b128 of 8 consecutive rows (one 8-lane group) then covers the 32
  // banks once -- at 8 mod 32 rows r and r + 4 shared banks: 2-way, and 29-30 % of the mb
  // instances' LDS-array cycles were bank conflicts (profiles/r06/pmc_c3.txt, pmc_c5.txt)
  constexpr int RSP = MB ? SP_MB_RSP : 8;
  const int RS = NTS * 64 + RSP;
  // this lane's slice image; an expression, not a pointer variable: through a local pointer
  // hipcc lost the image's distinctness from the static LDS arrays and waited lgkmcnt(0) in
  // three places of the step (config 5: 5.28 -> 6.09 ms per launch, profiles/r04/teams_split_regression.txt);
  // so the split form (TEAMS == 1) compiles to exactly round 3's code
  const int xs_off = TEAMS > 1 ? team * (NR * RS) : 0;
#define xs_lds (xs_dyn + xs_off)
  const float* start = P.W_start;
  unsigned long long* xb = X.xbuf + (int64_t)grp * 2 * G * X.SZ;
  // barrier of this lane's waves: s_barrier for the whole workgroup, or (TEAMS == 2) an LDS
  // arrival counter -- waits for this wave's LDS operations only (never for its row stream)
  // (bounded like every spin: a timeout sets the error word and stops waiting)
  unsigned tb_target = 0;
  bool tb_dead = false;
  if (TEAMS > 1 && tid == 0) tbar[team] = 0u;
  auto team_sync = [&]() {
    if constexpr (TEAMS == 1) {
      lds_barrier();
    } else {
      tb_target += NW;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(&tbar[team], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      for (unsigned sp = 0; !tb_dead &&
                            __hip_atomic_load(&tbar[team], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < tb_target;) {
        if (++sp > 64u * SP_SPIN_LIMIT) {
          if (lane == 0) __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          tb_dead = true;
        }
        __builtin_amdgcn_s_sleep(1);               // yield the SIMD to the other team's wave
      }
      asm volatile("" ::: "memory");
    }
  };
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);

  // ---- weights (and prox anchor) of this slice into registers: the round-start model ----
  float4 wr[TPW][NQ];
  // the prox anchor (the client's start) is not kept in registers -- 32 more VGPRs per lane
  // spilled every prox variant -- but re-read in the update: W_start (parallel clients: one
  // [C][ld] model shared by every group, L2-resident) or the previous chained client's result,
  // which this workgroup itself stored at that client's end
  const float* anc = P.W_start;
  // (the weight addresses are rebuilt behind an empty asm at every use: they are used only at
  // client boundaries and must not be hoisted into registers that live across the step loop)
  // register q of tile Tl: W + wbase() + woff(Tl, q) (16x16x4: class l16, columns 16 q + 4 lg;
  // mb: class 4 q + mi, columns 16 mq + 4 lg), live where wok(Tl, q)
  auto wbase = [&]() {
    int64_t b = MB ? (int64_t)mi * ld + 64 * t0 + 16 * mq + 4 * lg : (int64_t)l16 * ld + 64 * t0 + 4 * lg;
    asm volatile("" : "+v"(b));
    return b;
  };
  auto woff = [&](int Tl, int q) -> int64_t { return MB ? 4 * q * ld + 64 * Tl : 64 * Tl + 16 * q; };
  auto wok = [&](int Tl, int q) { return Tl < NTS && (MB ? 4 * q + mi < C : l16 < C); };
  auto load_start = [&]() {
    const int64_t base = wbase();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int Tl = w + NW * i;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        wr[i][q] = wok(Tl, q) ? ld4(start + base + woff(Tl, q)) : zero4;
        s = sq4_acc(s, wr[i][q].x, wr[i][q].y, wr[i][q].z, wr[i][q].w);
      }
    }
    return wave_sum_dpp(s, lane);
  };
  auto store_w = [&](float* Wj) {
    const int64_t base = wbase();
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int Tl = w + NW * i;
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        if (wok(Tl, q)) st4(Wj + base + woff(Tl, q), wr[i][q]);
    }
  };
  const float nw0 = load_start();                // ||W_start||^2 partial of this wave
  if (lane == 0) { wred[w][0] = 0.f; wred[w][1] = nw0; }

  // ---- the batch slice lives in registers in the forward's operand layout: lane (l16, lg)
  // holds rows rt*16 + l16, columns 16 q + 4 lg .. +3 of each of its tiles.  Rows past the
  // batch end load a valid row (their logits are ignored, their softmax gradient is 0).
  // `lc` is the step whose rows pn[] address (global row indices, fetched one step before
  // the features); it runs one step ahead of the compute loop, across client boundaries.
  float4 xf[TPW][RT][4];
  int pn[RT], lb[RT];
  SpCur lc;
  bool lc_ok = sp_seek(lc, P, grp, ng, T, 0);
  // the step's local row indices (raw) and its client's first row (base): pn = base + raw.
  // (The add is left to the caller, so that issuing the loads does not wait for them.)
  auto fetch_raw = [&](int* raw, int64_t& base) {
    const int e_ = lc.st / lc.nbat, s_ = lc.st - e_ * lc.nbat;
    const int b0_ = s_ * B, bc_ = min(B, lc.n - b0_);
    const int32_t* pp_ = P.perms + (int64_t)E * lc.row0 + (int64_t)e_ * lc.n + b0_;
    base = lc.row0;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int r_ = rt * 16 + l16;
      raw[rt] = pp_[r_ < bc_ ? r_ : 0];
    }
  };
  auto fetch_rows = [&]() {
    int raw[RT];
    int64_t base;
    fetch_raw(raw, base);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) pn[rt] = (int)(base + raw[rt]);
  };
#define SP_XLOAD()                                                                   \
  {                                                                                  \
    _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {                              \
      const int64_t r_ = pn[rt];                                                     \
      if (w == 0 && lg == 0) lb[rt] = P.labels[r_];                                  \
      const float* src_ = P.phi + r_ * ld + 64 * t0 + 4 * lg;                        \
      _Pragma("unroll") for (int i = 0; i < TPW; ++i)                                \
        if (w + NW * i < NTS)                                                        \
          _Pragma("unroll") for (int q = 0; q < 4; ++q)                              \
            xf[i][rt][q] = ld4(src_ + 64 * (w + NW * i) + 16 * q);                   \
    }                                                                                \
  }
  if (lc_ok) {
    fetch_rows();
    SP_XLOAD();
    lc_ok = sp_advance(lc, P, grp, ng, T);
    if (lc_ok) fetch_rows();
  }
  if constexpr (NCS < NC)                         // the classes the mb softmax never writes
    for (int i = tid; i < NR * NC; i += NTH) gbuf[i / NC][i % NC] = 0.f;
  __syncthreads();

  // clients with no step (n_j = 0 or E = 0): the result is the client's start -- the
  // current weights in a chain, W_start for parallel clients; their loss is 0
  auto flush_empty = [&](int ka, int kb) {
    for (int k = ka; k < kb; ++k) {
      const int j = sp_client(P, grp, ng, k);
      if (j < 0) continue;
      float* Wj = P.W_out + (int64_t)j * C * ld;
      if (P.chained) {
        store_w(Wj);
      } else {
        const int64_t base = wbase();
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
          const int Tl = w + NW * i;
#pragma unroll
          for (int q = 0; q < NQ; ++q)
            if (wok(Tl, q)) {
              const int64_t off = base + woff(Tl, q);
              st4(Wj + off, ld4(start + off));
            }
        }
      }
      if (g == 0 && tid == 0) P.loss[j] = 0.0;
    }
  };

  // the compute loop walks the group's steps with its own cursor `cc` (one flat loop: the
  // client boundaries are branches inside it)
  SpCur cc;
  bool cc_ok = sp_seek(cc, P, grp, ng, T, 0);
  flush_empty(0, cc_ok ? cc.k : T);
  unsigned gs = 0;                                // steps run by this group in this launch
  bool dead = false;                              // a hand-off timed out: stop waiting
  double lsum = 0.0;
#ifdef FS_STAMPS
  unsigned long long stamp_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, stamp_prev = 0;
#endif
  // the forward partial z_g = X_slice W_slice^T, tile by tile, into acc (RT row tiles)
  floatx4 acc[RT];
  floatx4 accm[RT][MB ? MBK : 1];                  // (mb) per row tile and class block
  auto fwd_tile = [&](int i) {
    if (w + NW * i < NTS) {
      if constexpr (MB) {
        mb_fwd_q<0>(accm, xf[i], wr[i]);
        mb_fwd_q<1>(accm, xf[i], wr[i]);
        mb_fwd_q<2>(accm, xf[i], wr[i]);
        mb_fwd_q<3>(accm, xf[i], wr[i]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float4 xa[RT];
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) xa[rt] = xf[i][rt][q];
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma4(comp(xa[rt], e4), comp(wr[i][q], e4), acc[rt]);
        }
      }
    }
  };
  auto fwd_tile0 = [&]() {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      acc[rt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int cb = 0; cb < (MB ? MBK : 1); ++cb) accm[rt][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    fwd_tile(0);
  };
  // pre: the step's tile-0 forward ran at the end of the previous step (round 5, session 2).  A
  // step ends by waiting for its whole next-step row stream (hipcc drains vmcnt at the loop's
  // back-edge); tile 0's rows are the stream's first half, so its MFMAs run there, in the
  // stream's tail, instead of after it.  Same MFMAs in the same order: the same bits.
  bool pre = false;
  for (; cc_ok; ++gs) {
    const int st = cc.st, n = cc.n, nbat = cc.nbat;
    if (st == 0) {
      // client start: parallel clients restart from W_start (the first one is loaded);
      // chained ones keep the registers.  The prox anchor is the start (tools.py:180).
      if (!P.chained && gs > 0) {
        (void)load_start();
        if (lane == 0) { wred[w][0] = 0.f; wred[w][1] = nw0; }
      } else if (lane == 0) {
        wred[w][0] = 0.f;                         // ||W - W_a|| = 0 at the new anchor
      }
      if (PROX) anc = (P.chained && cc.j > 0) ? P.W_out + (int64_t)(cc.j - 1) * C * ld : start;
      lsum = 0.0;
    }
    {
      SP_STAMP(0)
      const int e = st / nbat, s = st - e * nbat;
      const int b0 = s * B, bc = min(B, n - b0);
      const int par = gs & 1;
      const unsigned tag32 = X.tag_base + gs + 1u;
      if (w == 0 && lg == 0)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) lab[par][rt * 16 + l16] = lb[rt];
      // (round 5, session 2) the next step's labels and the row indices of the step after it
      // are loaded here, ahead of this step's row stream: loaded after it (as before), the
      // index arithmetic at the step's end waited vmcnt(0) for the whole next-step stream, so
      // no part of the next forward could start on rows that had already landed
      const bool ilv = lc_ok;
      int lbn[RT], pnr[RT];
      int64_t pnb = 0;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) { lbn[rt] = lb[rt]; pnr[rt] = 0; }
      bool lcn_ok = false;
      // (the narrow chained instances keep the fetch at the step's end: their step is the hand-off
      // chain, and these loads ahead of its polls cost more than the stream's tail -- config 1
      // 7.0 vs 7.6 ms per launch, profiles/r05b/prefwd_forms.txt)
#ifndef SP_NARROW_TOP
#define SP_NARROW_TOP 0
#endif
      constexpr bool TOP_FETCH = TPW > 1 || SP_NARROW_TOP;
      auto fetch_next = [&]() {
        if (ilv) {
          if (w == 0 && lg == 0)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) lbn[rt] = P.labels[pn[rt]];
          lcn_ok = sp_advance(lc, P, grp, ng, T);
          if (lcn_ok) fetch_raw(pnr, pnb);
        }
      };
      if constexpr (TOP_FETCH) fetch_next();

      // image write: the backward of this step reads the slice from LDS (each wave only ever
      // touches the image of its own tiles)
#define SP_IMG_WRITE()                                                               \
  {                                                                                  \
    _Pragma("unroll") for (int i = 0; i < TPW; ++i)                                  \
      if (w + NW * i < NTS)                                                          \
        _Pragma("unroll") for (int rt = 0; rt < RT; ++rt)                            \
          _Pragma("unroll") for (int q = 0; q < 4; ++q)                              \
            st4(xs_lds + (MB ? (rt * 16 + l16) * RS + 64 * (w + NW * i) + 16 * lg + 4 * q \
                             : img_off(rt * 16 + l16, RS, w + NW * i, 4 * q + lg)),   \
                xf[i][rt][q]);                                                       \
  }

      // ---------------- forward partial: z_g = X_slice W_slice^T ----------------
      // (tile 0's part may already have run at the end of the previous step: `pre`)
      if (!pre) fwd_tile0();
#pragma unroll
      for (int i = 1; i < TPW; ++i) fwd_tile(i);
      if constexpr (MB) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int cb = 0; cb < MBK; ++cb)
            zpart[w][((rt * MBK + cb) * 4 + mb_perm(lg)) * 16 + (l16 ^ (cb << 2))] = mb_kgroup_sum(accm[rt][cb]);
      } else {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
          st4(&zpart[w][rt * 256 + lg * 64 + l16 * 4], make_float4(acc[rt][0], acc[rt][1], acc[rt][2], acc[rt][3]));
      }
      SP_STAMP(1)
      team_sync();  // S1: wave partials, norm partials of the previous update; the image is free
      SP_STAMP(2)

      {
        // ---- hand-off, spread over the hand-off threads: thread t owns the values t + XT m
        // (the B x C real logits row-major, then the two norms).  Guideline 16, R2 form:
        // every value travels as one 8-byte {tag, value} granule written by ONE relaxed
        // agent-scope (sc1) store -- the data is its own flag; the partners' granules are
        // re-read with sc1 loads until every tag equals this step's tag.  The polls are
        // issued before the image write and the next slice's loads are issued after the
        // check, so the round trip neither queues behind nor waits for them.
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
            const int zo = MB ? zp_off_mb<MB ? MBK : 1>(r, c) : zp_off(r, c);
#pragma unroll
            for (int i = 0; i < NW; ++i) v += zpart[i][zo];
          } else if (idx < NV) {
#pragma unroll
            for (int i = 0; i < NW; ++i) v += wred[i][idx - (NV - 2)];
          }
          own[m] = v;
          sum[m] = 0.f;
          if (idx < NV)
            __hip_atomic_store(slot + (int64_t)g * X.SZ + idx, tag | __float_as_uint(v), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        SP_STAMP(3)
        if (X.spin_limit == 0 && gs == 0 && lane == 0)      // test knob: report an injected timeout
          __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        // partners in chunks of HC (one round trip each); the sum runs in slice order
        // 0..G-1 with the own partial at position g: identical bits in every partner
#pragma unroll
        for (int h0 = 0; h0 < G; h0 += HC) {
          // (measured and dropped, round 6: waves holding no exchanged value at slot m skipping
          // their dummy polls -- config 5 4.76 -> 4.99 ms per launch, config 2 285 -> 288 us;
          // profiles/r06/poll_skip_ab.txt.  The dummy round trips act as the first-poll sleep does.)
          auto poll = [&]() {
#pragma unroll
            for (int m = 0; m < M; ++m) {
              const int idx = tid + XT * m;
#pragma unroll
              for (int h = 0; h < HC; ++h)
                pl[m][h] = __hip_atomic_load(slot + (int64_t)(h0 + h) * X.SZ + (idx < NV ? idx : 0),
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          };
          // (wait before the first poll: partners publish about then, and early round trips of
          // every wave on the same lines only clog the L2 -- as in the qmc p-solver)
          if (h0 == 0)
            for (int d_ = 0; d_ < X.poll_delay; ++d_) __builtin_amdgcn_s_sleep(1);
          poll();
          if (h0 == 0) SP_IMG_WRITE();
          for (;;) {
            bool ok = true;
#pragma unroll
            for (int m = 0; m < M; ++m)
#pragma unroll
              for (int h = 0; h < HC; ++h)
                ok &= (h0 + h == g) | (tid + XT * m >= NV) | ((unsigned)(pl[m][h] >> 32) == tag32);
            if (__all(ok)) break;
            if (dead || ++spins > X.spin_limit) {
              if (lane == 0) __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              dead = true;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
            poll();
          }
#pragma unroll
          for (int m = 0; m < M; ++m)
#pragma unroll
            for (int h = 0; h < HC; ++h)
              sum[m] += (h0 + h == g) ? own[m] : __uint_as_float((unsigned)pl[m][h]);
        }
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const int idx = tid + XT * m;
          if (idx < NV) {
            if (idx < NV - 2) {
              const int r = idx / C, c = idx - r * C;
              zsum[r][c] = sum[m];
            } else {
              nrm[idx - (NV - 2)] = sum[m];       // ||W - W_a||^2, ||W||^2 at the start of this step
            }
          }
        }
        SP_STAMP(4)
      }
      // the first SP_EARLY of this wave's next-step row loads go out here, behind the hand-off's
      // polls (which have all returned): they stream through S2, the softmax and S3 instead of
      // waiting for the backward (FedAvg / FedAMW on full slices; the prox anchor's loads would
      // queue behind them)
      constexpr int NLD = TPW * 4 * RT;           // row loads per wave and step
      constexpr int NE = EARLY < NLD ? EARLY : NLD;
      auto issue_row = [&](int f) {                 // (f is a constant after unrolling)
        const int i = f / (4 * RT), kk = f % (4 * RT);
        xf[i][kk >> 2][kk & 3] =
            ld4(P.phi + (int64_t)pn[kk >> 2] * ld + 64 * t0 + 4 * lg + 64 * (w + NW * i) + 16 * (kk & 3));
      };
      // (EARLY instances run only on full slices and issue every load unconditionally -- pn
      // always holds valid rows -- so the step is one straight path with one register
      // assignment for xf)
      // (one tile per wave, the narrow chained instances: the whole step's rows go out at once)
      constexpr int E1 = TPW == 1 ? NE : SP_E1;
      constexpr int NE1 = E1 < NE ? E1 : NE, NE2 = E1 + SP_E2 < NE ? E1 + SP_E2 : NE;
      // with a prox term (round 5) the anchor's whole slice goes out first, ahead of the early rows,
      // so the update waits only for it (the late form re-reads it per tile inside the backward,
      // behind that tile's predecessors' row loads); lanes of padding classes read class C - 1's
      // row -- every load unconditional, as the rows
      float4 avall[PROX && NE > 0 ? TPW : 1][NQ];
      if constexpr (PROX && NE > 0) {
        if constexpr (MB) {
          const float* ap = anc + 64 * t0 + 16 * mq + 4 * lg;
#pragma unroll
          for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int q = 0; q < NQ; ++q) avall[i][q] = ld4(ap + (int64_t)min(4 * q + mi, C - 1) * ld + 64 * (w + NW * i));
        } else {
          const float* ap = anc + (int64_t)min(l16, C - 1) * ld + 64 * t0 + 4 * lg;
#pragma unroll
          for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) avall[i][q] = ld4(ap + 64 * (w + NW * i) + 16 * q);
        }
      }
      if constexpr (NE > 0)
#pragma unroll
        for (int f = 0; f < NE1; ++f) issue_row(f);
      SP_STAMP(5)
      team_sync();  // S2: summed logits and norms, the image
      if constexpr (NE > 0)
#pragma unroll
        for (int f = NE1; f < NE2; ++f) issue_row(f);
      SP_STAMP(6)
      const float invb = 1.0f / (float)bc;
      float cep = 0.f;
      // (mb: NCS lanes per row, the class blocks' width rounded to a power of 2 -- 4 at C <= 4, 8 at
      // C <= 8; the classes past it stay the zeros written at the kernel's start.  The same sums:
      // the 16-lane trees only added exact zeros from lanes past NCS)
      for (int idx = tid; idx < NZS; idx += NTH) {         // NCS lanes of one wave hold one row
        const int r = idx / NCS, c = idx - r * NCS;
        const bool valid = r < bc && c < C;
        const float z = valid ? zsum[r][c] : 0.f;
        // (the loop is wave-uniform -- NZS is a multiple of 64 -- so the DPP exchanges run with
        // every lane active)
        float m = valid ? z : -INFINITY;
#pragma unroll
        for (int off = NCS / 2; off > 0; off >>= 1) m = fmaxf(m, xor_get(m, off, lane));
        // softmax on v_exp_f32 / v_rcp_f32 / v_log_f32 (one exponential per entry, e / sum e
        // for the gradient): within the fp32 tolerance of torch's log_softmax (tests/fixtures.py)
        const float ex = valid ? __expf(z - m) : 0.f;
        float se = ex;
#pragma unroll
        for (int off = NCS / 2; off > 0; off >>= 1) se += xor_get(se, off, lane);
        float gv = 0.f;
        if (valid) {
          const bool isy = c == lab[par][r];
          gv = (isy ? -invb : 0.f) + ex * __builtin_amdgcn_rcpf(se) * invb;
          if (isy) cep -= z - m - __logf(se);
        }
        gbuf[r][c] = gv;
      }
      cep = wave_sum_dpp(cep, lane);
      if (lane == 0) wce[w] = cep;
      team_sync();  // S3: g, CE partials
      if constexpr (NE > 0)
#pragma unroll
        for (int f = NE2; f < NE; ++f) issue_row(f);
      SP_STAMP(7)
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
      // A operand lane (l16, lg): image row 4 kk + lg, block 4 (l16 & 3) + (l16 >> 2), so the
      // output register q of lane (c, lg) is the gradient of d = 16 q + 4 lg + e (the lane's W).
      float gB[MB ? 1 : 4 * RT];
      if constexpr (!MB)
#pragma unroll
        for (int kk = 0; kk < 4 * RT; ++kk) gB[kk] = gbuf[4 * kk + lg][l16];
      const float sp = (P.prox && pn2 > 0.f) ? P.mu / sqrtf(pn2) : 0.f;
      const float sr = (P.reg && wn2 > 0.f) ? P.lam / sqrtf(wn2) : 0.f;
      const float lr = P.lr;
      const int rblk = 4 * (l16 & 3) + (l16 >> 2);
      float npn = 0.f, nwn = 0.f;
      // this wave's next rows go out one load per backward iteration
      // (two instances, so the interleaved loads are straight-line code: a branch around each
      // load would make the compiler wait for it at the join)
      // FULL: every wave owns TPW tiles (NTS = NW * TPW, every BASELINE shape but chained config
      // 1), so no tile guard splits the block either
      auto bwd = [&](auto LD, auto FULL, auto EA) {
        constexpr int EAN = decltype(EA)::value;   // row loads already issued (early)
      if constexpr (MB) {
        // (mb) rows outer, tiles inner: one g register per batch row serves every tile and
        // class block (lane 16 s + 4 x + j = g[r][4 s + j], broadcast from group cb by blgp);
        // one image read per (row, tile).  The mb image is in lane order (word 16 lg + 4 q + e of
        // a row's tile = column 16 q + 4 lg + e: the write's float4 of (row, q) lands at 16 lg + 4 q),
        // so the read is the lane's own word of the row -- one address register, the row and tile
        // as immediate offsets; both conflict-free (row stride = 4 mod 32 words, RSP)
        constexpr int RS_FULL = NW * TPW * 64 + RSP;
        const int RSx = decltype(FULL)::value ? RS_FULL : RS;
        float4 av[TPW][NQ];                         // prox anchor (late form: read per tile here)
        if constexpr (PROX && EAN > 0) {
#pragma unroll
          for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int q = 0; q < NQ; ++q) av[i][q] = avall[i][q];
        } else if constexpr (PROX) {
#pragma unroll
          for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
              const int Tl = w + NW * i;
              av[i][q] = wok(Tl, q) ? ld4(anc + wbase() + woff(Tl, q)) : zero4;
            }
        }
        floatx4 gm[TPW][NQ];
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
          for (int q = 0; q < NQ; ++q) gm[i][q] = floatx4{0.f, 0.f, 0.f, 0.f};
        if constexpr (decltype(FULL)::value && SP_MB_BWD_PF > 0) {
          // every row block's image and g words read one block ahead, in registers
          float xa[2][4][TPW], gq[2][4];
          auto rd = [&](int kk, int b) {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
#ifdef SP_MB_DIAG_NOGREAD   // diagnostic builds only (wrong results): which LDS reads the backward waits for
              gq[b][rr] = gbuf[0][4 * lg + mi] + (float)(kk + rr);
#else
              gq[b][rr] = gbuf[4 * kk + rr][4 * lg + mi];
#endif
#pragma unroll
              for (int i = 0; i < TPW; ++i)
#ifdef SP_MB_DIAG_NOXREAD
                xa[b][rr][i] = (float)(kk * 4 + rr + i) * gq[b][rr];
#else
                xa[b][rr][i] = xs_lds[(4 * kk + rr) * RSx + 64 * (w + NW * i) + lane];
#endif
            }
          };
          rd(0, 0);
#pragma unroll
          for (int kk = 0; kk < 4 * RT; ++kk) {
            if (kk + 1 < 4 * RT) rd(kk + 1, (kk + 1) & 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
#pragma unroll
              for (int i = 0; i < TPW; ++i) mb_bwd_row<MBK>(gm[i], xa[kk & 1][rr][i], gq[kk & 1][rr]);
            if constexpr (decltype(LD)::value) {
#pragma unroll
              for (int i = 0; i < TPW; ++i) {
                const int f = kk * TPW + i + EAN;
                if (f < NLD) issue_row(f);
              }
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        } else
#pragma unroll
        for (int kk = 0; kk < 4 * RT; ++kk) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int r = 4 * kk + rr;
            const float gv = gbuf[r][4 * lg + mi];
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
              const int Tl = w + NW * i;
              if (decltype(FULL)::value || Tl < NTS)
                mb_bwd_row<MBK>(gm[i], xs_lds[r * RSx + 64 * Tl + lane], gv);
            }
          }
          if constexpr (decltype(LD)::value) {
            // iteration (kk, i) issues load kk * TPW + i + EAN (as the 16x16x4 form: one per iteration)
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
              const int f = kk * TPW + i + EAN;
              if (f < NLD && (decltype(FULL)::value || w + NW * (f / (4 * RT)) < NTS)) issue_row(f);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
          const int Tl = w + NW * i;
#pragma unroll
          for (int q = 0; q < NQ; ++q)
            if ((decltype(FULL)::value || Tl < NTS) && 4 * q + mi < C) {
              float o[4];
#pragma unroll
              for (int e4 = 0; e4 < 4; ++e4) {
                const float wc = comp(wr[i][q], e4);
                const float ac = PROX ? comp(av[i][q], e4) : 0.f;
                o[e4] = sgd_w(wc, gm[i][q][e4], lr, PROX, ac, sp, P.reg, sr);
                if (PROX) {
                  const float dp = o[e4] - ac;
                  npn = sq_acc(npn, dp);
                  nwn = sq_acc(nwn, o[e4]);
                }
              }
              wr[i][q] = make_float4(o[0], o[1], o[2], o[3]);
            }
        }
      } else {
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        const int Tl = w + NW * i;
        if (decltype(FULL)::value || Tl < NTS) {
          float4 av[4];                            // prox anchor of this tile (issued first: the
          if constexpr (PROX && EAN > 0) {         // update waits only for these, not the rows)
#pragma unroll
            for (int q = 0; q < 4; ++q) av[q] = avall[i][q];
          } else if (PROX && l16 < C) {
            const float* ap = anc + wbase() + 64 * Tl;
#pragma unroll
            for (int q = 0; q < 4; ++q) av[q] = ld4(ap + 16 * q);
          }
          floatx4 ga[4];
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) ga[e4] = floatx4{0.f, 0.f, 0.f, 0.f};
          // image row 4 kk + lg, block rblk ^ (4 (kk & 1) + lg): two per-lane bases (kk even / odd)
          // and, in the FULL instance (compile-time row stride), the rows as immediate offsets --
          // 16 hoisted addresses per tile spilled at G = 16 and each reload waited vmcnt(0) for
          // the whole row stream inside this loop
          constexpr int RS_FULL = NW * TPW * 64 + 8;
          const int RSx = decltype(FULL)::value ? RS_FULL : RS;
          const float* ib0 = xs_lds + lg * RSx + 64 * Tl + 4 * (rblk ^ lg);
          const float* ib1 = xs_lds + lg * RSx + 64 * Tl + 4 * (rblk ^ (lg + 4));
          // one tile per wave (narrow, one wave per SIMD at 4 waves): nothing hides an image
          // read's latency behind another wave's MFMAs, so the tile's reads all go out first
          float4 xpre[TPW == 1 ? 4 * RT : 1];
          if constexpr (TPW == 1) {
#pragma unroll
            for (int kk = 0; kk < 4 * RT; ++kk) xpre[kk] = ld4(((kk & 1) ? ib1 : ib0) + 4 * kk * RSx);
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int kk = 0; kk < 4 * RT; ++kk) {
            const float4 x = TPW == 1 ? xpre[kk] : ld4(((kk & 1) ? ib1 : ib0) + 4 * kk * RSx);
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) ga[e4] = mfma4(comp(x, e4), gB[kk], ga[e4]);
            if constexpr (decltype(LD)::value) {
              if constexpr (EAN == 0) {
                xf[i][kk >> 2][kk & 3] = ld4(P.phi + (int64_t)pn[kk >> 2] * ld + 64 * t0 + 4 * lg + 64 * Tl + 16 * (kk & 3));
              } else {
                // iteration it of the wave's backward issues load it + EAN (the rest of the
                // stream goes out in the first NLD - EAN iterations)
                if (i * 4 * RT + kk + EAN < NLD) issue_row(i * 4 * RT + kk + EAN);
              }
            }
          }
          if (l16 < C) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              float o[4];
#pragma unroll
              for (int e4 = 0; e4 < 4; ++e4) {
                const float wc = comp(wr[i][q], e4);
                const float ac = PROX ? comp(av[q], e4) : 0.f;
                o[e4] = sgd_w(wc, ga[e4][q], lr, PROX, ac, sp, P.reg, sr);
                if (PROX) {                        // (without a prox term: after the loop, if ridge)
                  const float dp = o[e4] - ac;
                  npn = sq_acc(npn, dp);
                  nwn = sq_acc(nwn, o[e4]);
                }
              }
              wr[i][q] = make_float4(o[0], o[1], o[2], o[3]);
            }
          }
        }
      }
      }
      };
      using E0 = std::integral_constant<int, 0>;
      if constexpr (NE > 0) {
        bwd(std::true_type{}, std::true_type{}, std::integral_constant<int, NE>{});
      } else if (ilv) {
        if (NTS == NW * TPW)
          bwd(std::true_type{}, std::true_type{}, E0{});
        else
          bwd(std::true_type{}, std::false_type{}, E0{});
      } else {
        bwd(std::false_type{}, std::false_type{}, E0{});
      }
      if constexpr (!TOP_FETCH) fetch_next();
      if (ilv) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          lb[rt] = lbn[rt];
          if (lcn_ok) pn[rt] = (int)(pnb + pnr[rt]);
        }
        lc_ok = lcn_ok;
      }
      // the norms of the updated slice feed only the prox / ridge terms (loss and gradient): without
      // either nothing reads them; ridge alone sums ||W||^2 here in the update's own order (i, q,
      // e4: the same bits as summing it inline; padding lanes and tiles hold zeros)
      if (!PROX && P.reg) {
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
          for (int q = 0; q < NQ; ++q)
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) nwn = sq_acc(nwn, comp(wr[i][q], e4));
      }
      if (PROX || P.reg) {
        npn = PROX ? wave_sum_dpp(npn, lane) : 0.f;
        nwn = wave_sum_dpp(nwn, lane);
        if (lane == 0) { wred[w][0] = npn; wred[w][1] = nwn; }
      }
      // the next step's tile-0 forward, where the next step continues this client (the weights
      // stay; a new parallel client restarts from W_start at the step's top)
      // (mb: where the next step's forward accumulators fit beside the step's registers -- with more
      // class blocks or partners they spilled, and a spill reload waits vmcnt(0) for the row stream:
      // config 5 5.99 ms per launch with it, 4.70 without, profiles/r06/mb_ab.txt)
      constexpr bool PRE_OK = !MB || (SP_MB_PRE && ((MBK <= 2 && G <= 8) || (MBK == 3 && G == 2 && !PROX)));
      pre = TEAMS == 1 && TPW > 1 && PRE_OK && st + 1 < cc.steps;
      if (pre) fwd_tile0();
      SP_STAMP(8)
    }
    if (st == cc.steps - 1) {                     // client end
      store_w(P.W_out + (int64_t)cc.j * C * ld);
      if (g == 0 && tid == 0) P.loss[cc.j] = lsum / (double)n;
    }
    const int kprev = cc.k;
    cc_ok = sp_advance(cc, P, grp, ng, T);
    flush_empty(kprev + 1, cc_ok ? cc.k : T);
  }
#undef SP_XLOAD
#undef SP_IMG_WRITE
#undef xs_lds
#ifdef FS_STAMPS
  if (threadIdx.x == 0 && X.stamps) {
    for (int k = 0; k < 8; ++k) X.stamps[blockIdx.x * 16 + k] = stamp_acc[k];
    X.stamps[blockIdx.x * 16 + 15] = (unsigned long long)gs;
  }
#endif
}

#ifndef FS_SPLIT_KERNEL_ONLY   // (scripts/split_asm.sh: one instance's code, without the launchers)
unsigned exchange_generation(const void* ws, bool long_launch) {
  static std::mutex gm;
  static std::unordered_map<const void*, unsigned> gens;
  std::lock_guard<std::mutex> lk(gm);
  auto it = gens.find(ws);
  const unsigned prev = it == gens.end() ? 0u : it->second;
  const unsigned gen = (long_launch || prev >= 4095u) ? 0u : prev + 1u;
  gens[ws] = gen;
  return gen;
}

static int g_cus = 0;

int device_cus() {
  if (g_cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) g_cus = 0;
  }
  return g_cus;
}

static size_t split_dyn_lds(int RT, int NT, int G, int teams = 1) {
  const int tiles = (NT + G - 1) / G;
  return sizeof(float) * (size_t)teams * (size_t)(RT * 16) * (size_t)(tiles * 64 + 8);
}

static size_t split_static_lds(int RT, int NW, int teams = 1) {
  const int NR = RT * 16;
  return (size_t)teams * ((size_t)NW * NR * 16 * 4 + 2 * (size_t)NR * 16 * 4 + 2 * NR * 4 + NW * 3 * 4 + 8) + 64 +
         4 * teams;
}

static int split_rt(int B) { return B <= 16 ? 1 : 2; }

// can G workgroups split one client of this shape (teams = 2: two client lanes of 4 waves per
// workgroup, parallel clients only)?
static bool split_fits(int C, int B, int NT, int G, int teams = 1) {
  if (!(G == 2 || G == 4 || G == 8 || G == 16)) return false;
  if (C > 16 || B > 32 || NT < G) return false;
  const int RT = split_rt(B);
  const int nw = SP_WAVES / teams;
  const int tiles = (NT + G - 1) / G;
  if ((tiles + nw - 1) / nw > SP_TPW) return false;
  if (G >= 8 && RT * 16 * C + 2 > 512) return false;   // exchanged values: at most 512
  return split_dyn_lds(RT, NT, G, teams) + split_static_lds(RT, nw, teams) <= 160 * 1024;
}

static int split_sz(int RT) { return RT * 16 * 16 + 4; }

// groups in flight: one per G workgroups, one workgroup per CU (each with `teams` client lanes)
static int split_groups(int N, int G, int chained, int cus, int teams = 1) {
  return chained ? 1 : std::max(1, std::min((N + teams - 1) / teams, cus / G));
}

static int64_t split_xbuf_bytes(int ngroups, int G, int RT, int teams = 1) {
  return (int64_t)ngroups * teams * 2 * G * split_sz(RT) * 8;
}

static int64_t split_ws_bytes(int N, int G, int B, int chained, int cus, int teams = 1) {
  const int RT = split_rt(B);
  return split_xbuf_bytes(split_groups(N, G, chained, cus, teams), G, RT, teams) + SP_ERR_BYTES;
}

// s_sleep(1) units before a step's first poll (fs_tuning.split_poll_delay: 0 = by width, -1 =
// none, n > 0 = n).  By width (profiles/r04/split_poll_delay_*.txt, launch ms): G = 16 (config 5)
// 5.35-5.37 without, 5.21-5.23 at 16, 5.29-5.31 at 24, 5.45-5.49 at 48; G = 2 (config 2) no gain
constexpr int SPLIT_PD_WIDE = 16, SPLIT_PD_NARROW = 0;
static int split_poll_delay(int G, bool chained) {
  const int t = tuning().split_poll_delay;
  if (t < 0) return 0;
  if (t > 0) return t;
  if (chained) return 0;                 // one group: no other group's polls to yield to
  return G >= 8 ? SPLIT_PD_WIDE : SPLIT_PD_NARROW;
}

// the hand-off spin bound (fs_tuning.spin_limit); 0 = the injected-timeout test knob
static unsigned split_spin_limit() {
  const fs_tuning t = tuning();
  if (t.inject_timeout) return 0u;
  return t.spin_limit ? t.spin_limit : SP_SPIN_LIMIT;
}
unsigned split_spin_bound() { return split_spin_limit(); }

template <int RT, int G, bool PROX, int EARLY, int TEAMS, int WAVES = SP_WAVES, int TPWK = SP_TPW, int MBK = 0>
static void launch_split_k(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(
        reinterpret_cast<const void*>(&local_train_split_kernel<RT, G, PROX, EARLY, TEAMS, WAVES, TPWK, MBK>),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((local_train_split_kernel<RT, G, PROX, EARLY, TEAMS, WAVES, TPWK, MBK>), dim3(grid),
                     dim3(WAVES * 64), lds, st, P, X);
}

// class blocks of the mb instances for this launch (0: the 16x16x4 instances).  fs_tuning.split_mb:
// 1 = wherever they fit (16 < B <= 32, one team), 0 = by shape, -1 = never.  By shape: C <= 8 (at
// most 2 class blocks: half the 16x16x4 MFMA cycles or less) -- config 3 (C = 7, FedProx, G = 4)
// 4.57 -> 4.07-4.08 ms per launch, config 1 (C = 2, narrow chained) 7.07 -> 6.09-6.11 ms -- and
// 3 blocks at G = 16 (config 5: 4.66-4.68 -> 4.51-4.55 ms); at G = 2 (config 2) 283-285 vs 288-290 us:
// that step waits for its row stream, not for its MFMAs (without the backward's LDS reads the mb
// launch measured the same, profiles/r06/mb_ab.txt), so the 16x16x4 instances stay there
static int split_mbk(const LTParams& P, int G, int teams) {
  const int t = tuning().split_mb;
  if (t < 0 || teams != 1 || split_rt(P.B) != 2) return 0;
  const int cb = (P.C + 3) / 4;
  if (t == 0 && cb > 2 && !(cb == 3 && G >= 16)) return 0;
  return cb;
}

// the split form's instance for this launch: the 16x16x4 one, or the mb one with ceil(C / 4)
// class blocks (recorded for fs_local_train_last_kernel)
template <int RT, int G, bool PROX, int EARLY, int TEAMS, int WAVES = SP_WAVES, int TPWK = SP_TPW>
static void launch_split_s(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  if constexpr (RT == 2 && TEAMS == 1) {
    switch (split_mbk(P, G, TEAMS)) {
      case 1: set_last_lt_kernel(FS_LT_MB); launch_split_k<RT, G, PROX, EARLY, TEAMS, WAVES, TPWK, 1>(P, X, grid, lds, st); return;
      case 2: set_last_lt_kernel(FS_LT_MB); launch_split_k<RT, G, PROX, EARLY, TEAMS, WAVES, TPWK, 2>(P, X, grid, lds, st); return;
      case 3: set_last_lt_kernel(FS_LT_MB); launch_split_k<RT, G, PROX, EARLY, TEAMS, WAVES, TPWK, 3>(P, X, grid, lds, st); return;
      case 4: set_last_lt_kernel(FS_LT_MB); launch_split_k<RT, G, PROX, EARLY, TEAMS, WAVES, TPWK, 4>(P, X, grid, lds, st); return;
      default: break;
    }
  }
  launch_split_k<RT, G, PROX, EARLY, TEAMS, WAVES, TPWK, 0>(P, X, grid, lds, st);
}

// the narrow chained instances (one tile per wave, full slices, every row load early): NT = 4 G
// on 4-wave workgroups, NT = 8 G on 8-wave ones.  A 4-wave workgroup asks for 96 KB of LDS so
// that no two share a CU.  (fs_tuning.split_early = -1 turns them off with the early issue: the
// chain then runs the late 8-wave form, bitwise the same weights.)
constexpr int SPLIT_NARROW_EARLY = 8;
template <int RT, int G>
static bool launch_split_narrow(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  if constexpr (RT != 2 || G < 4) {
    return false;
  } else {
    const int64_t NT = P.ld >> 6;
    if (!P.chained || P.fuse_E > 0 || tuning().split_early < 0) return false;
    if (NT == 4 * G) {
      const size_t l4 = std::max(lds, (size_t)96 * 1024);
      if (P.prox) launch_split_s<RT, G, true, SPLIT_NARROW_EARLY, 1, 4, 1>(P, X, grid, l4, st);
      else launch_split_s<RT, G, false, SPLIT_NARROW_EARLY, 1, 4, 1>(P, X, grid, l4, st);
      return true;
    }
    if (NT == 8 * G) {
      if (P.prox) launch_split_s<RT, G, true, SPLIT_NARROW_EARLY, 1, SP_WAVES, 1>(P, X, grid, lds, st);
      else launch_split_s<RT, G, false, SPLIT_NARROW_EARLY, 1, SP_WAVES, 1>(P, X, grid, lds, st);
      return true;
    }
    return false;
  }
}

// the team form (G | FS_G_TEAMS): parallel clients, G = 4 or 8 (config 2 / 3 / 4 widths)
template <int RT, int G>
static void launch_split_teams(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  constexpr int EARLY_G = SP_EARLY;
  const bool full = (P.ld >> 6) == (int64_t)G * (SP_WAVES / 2) * SP_TPW;
  if (P.prox) launch_split_s<RT, G, true, 0, 2>(P, X, grid, lds, st);
  else if (full && EARLY_G > 0 && tuning().split_early >= 0) launch_split_s<RT, G, false, EARLY_G, 2>(P, X, grid, lds, st);
  else launch_split_s<RT, G, false, 0, 2>(P, X, grid, lds, st);
}

// the double-buffered instance (local_train_dbuf.hip, round 6): where it covers the launch and
// fs_tuning.split_dbuf asks for it (1 = wherever it covers; 0 = by shape: not chosen -- measured a
// tie at configs 2 and 5 and slower at config 1; -1 = never); bitwise the same
bool dbuf_covers(int C, int B, int64_t ld, int G, int chained, int prox, int* waves_out);
int launch_local_train_dbuf(const LTParams& P, int G, const SplitWS& X, int grid, size_t lds, hipStream_t st);
static bool dbuf_by_shape(const LTParams& P, int G) {
  if (tuning().split_dbuf <= 0 || tuning().split_early < 0) return false;
  return dbuf_covers(P.C, P.B, P.ld, G, P.chained, P.prox, nullptr);
}

template <int RT, int G>
static void launch_split_g(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  if (RT == 2 && dbuf_by_shape(P, G) && launch_local_train_dbuf(P, G, X, grid, lds, st) == FS_OK) {
    set_last_lt_kernel(FS_LT_DBUF);
    return;
  }
  // early row issue where every workgroup's slice is full (NT = G * 16 tiles)
  // (fs_tuning.split_early: 0 = by shape, -1 = never)
  // Depth per width (profiles/r03/split_early_ab2.txt, launch ms): at G = 2 (128 KB of rows per
  // CU per step) 4 early loads are fastest (config 2: 0.300-0.302 vs 0.304-0.307 with 6), at
  // G = 16 6 (config 5: 5.34-5.36 vs 5.58 with 4)
  // With a prox term (round 5) the anchor's slice (8 loads per wave) goes out ahead of the early
  // rows, and 2 early rows measured fastest (config 3, G = 4, launch us, profiles/r05/prox_early_depth.txt:
  // late 5,102-5,107; early 1: 4,678-4,691, 2: 4,488-4,530, 3: 4,605-4,622, 4: 4,539-4,544, 6: 4,699-4,715,
  // 8: 4,713-4,720)
  constexpr int EARLY_G = (G == 2 && SP_EARLY > 4) ? 4 : SP_EARLY;
#ifndef SP_EP
#define SP_EP 2
#endif
  constexpr int EARLY_PROX = SP_EARLY < SP_EP ? SP_EARLY : SP_EP;
  const bool full = (P.ld >> 6) == (int64_t)G * SP_WAVES * SP_TPW;
  const bool early = full && EARLY_G > 0 && tuning().split_early >= 0;
  if (launch_split_narrow<RT, G>(P, X, grid, lds, st)) return;
  if (P.prox && early) launch_split_s<RT, G, true, EARLY_PROX, 1>(P, X, grid, lds, st);
  else if (P.prox) launch_split_s<RT, G, true, 0, 1>(P, X, grid, lds, st);
  else if (early) launch_split_s<RT, G, false, EARLY_G, 1>(P, X, grid, lds, st);
  else launch_split_s<RT, G, false, 0, 1>(P, X, grid, lds, st);
}

int launch_local_train_split(const LTParams& P, int Gf, void* ws, int64_t ws_bytes, hipStream_t st) {
  const int teams = (Gf & FS_G_TEAMS) ? 2 : 1;
  const int G = Gf & (FS_G_PAIR - 1);
  if (teams > 1 && (P.chained || !(G == 4 || G == 8)))
    return fail(FS_EUNSUPPORTED, "fs_local_train: the team form runs parallel clients at G = 4 or 8");
  const int RT = split_rt(P.B);
  const int NT = (int)(P.ld >> 6);
  if (!(G == 2 || G == 4 || G == 8 || G == 16)) return fail(FS_EINVAL, "fs_local_train: G must be 1, 2, 4, 8 or 16");
  if (P.C > 16 || P.B > 32) return fail(FS_EUNSUPPORTED, "fs_local_train: split clients need C <= 16, B <= 32");
  if (NT < G) return fail(FS_EUNSUPPORTED, "fs_local_train: fewer feature tiles than workgroups per client");
  if (!split_fits(P.C, P.B, NT, G, teams)) return fail(FS_EUNSUPPORTED, "fs_local_train: slice too wide for one workgroup");
  const int cus = device_cus();
  if (cus <= 0) return fail(FS_EHIP, "fs_local_train: no device");
  if (G > cus) return fail(FS_EUNSUPPORTED, "fs_local_train: G exceeds the CU count");
  const int ng = split_groups(P.N, G, P.chained, cus, teams);
  const int64_t xbytes = split_xbuf_bytes(ng, G, RT, teams);
  if (!ws || ws_bytes < xbytes + SP_ERR_BYTES) return fail(FS_EINVAL, "fs_local_train: workspace too small");
  char* base = reinterpret_cast<char*>(ws);
  SplitWS X;
  X.xbuf = reinterpret_cast<unsigned long long*>(base);
  X.err = reinterpret_cast<unsigned*>(base + ws_bytes - SP_ERR_BYTES);   // last block: sticky
  X.SZ = split_sz(RT);
  X.ngroups = ng;
  X.spin_limit = split_spin_limit();
  X.poll_delay = split_poll_delay(G, P.chained != 0);
  X.stamps = nullptr;
#ifdef FS_STAMPS
  X.stamps = reinterpret_cast<unsigned long long*>(base + xbytes);
#endif
  // Hand-off tags: (launch generation << 20) + group step + 1, the generation counted per
  // workspace on the host, so a granule left by an earlier launch never carries a tag this
  // launch waits for and the exchange buffer needs no clearing per launch.  It is cleared
  // when a workspace is first seen, every 4095 launches (the generation wraps) and for a
  // launch whose groups may run 2^20 - 1 steps or more (then the generation is 0: tags are
  // the step + 1 alone, as after any clearing).
  // (groups walk clients in snake order: at most ceil(N / ng) each; chained: all N)
  const int64_t groups_clients = P.chained ? P.N : (P.N + ng * teams - 1) / (ng * teams);
  const bool long_launch = P.max_client_steps <= 0 || P.max_client_steps * groups_clients >= (1 << 20) - 1;
  const unsigned gen = exchange_generation(ws, long_launch);
  X.tag_base = gen << 20;
  if (gen <= 1) {                      // first use, wrap or long launch: clear the granules
    hipError_t e = hipMemsetAsync(base, 0, (size_t)xbytes, st);
    if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_local_train: ") + hipGetErrorString(e));
  }
  const size_t lds = split_dyn_lds(RT, NT, G, teams);
  if (P.fuse_E > 0 && (P.chained || ng * G + P.fuse_E > cus || lds < sizeof(float) * SP_WAVES * 16 * 17))
    return fail(FS_EINVAL, "fs_local_train: no room for the fused evaluation");
  const int grid = P.chained ? 8 * G : ng * G + P.fuse_E;
  if (teams > 1) {
    if (RT == 2 && G == 4) { launch_split_teams<2, 4>(P, X, grid, lds, st); return FS_OK; }
    if (RT == 2 && G == 8) { launch_split_teams<2, 8>(P, X, grid, lds, st); return FS_OK; }
    if (RT == 1 && G == 4) { launch_split_teams<1, 4>(P, X, grid, lds, st); return FS_OK; }
    if (RT == 1 && G == 8) { launch_split_teams<1, 8>(P, X, grid, lds, st); return FS_OK; }
    return fail(FS_EUNSUPPORTED, "fs_local_train: no team kernel for this shape");
  }
#define FS_SPLIT_CASE(rt, g) \
  if (RT == rt && G == g) { launch_split_g<rt, g>(P, X, grid, lds, st); return FS_OK; }
  FS_SPLIT_CASE(2, 2) FS_SPLIT_CASE(2, 4) FS_SPLIT_CASE(2, 8) FS_SPLIT_CASE(2, 16)
  FS_SPLIT_CASE(1, 2) FS_SPLIT_CASE(1, 4) FS_SPLIT_CASE(1, 8) FS_SPLIT_CASE(1, 16)
#undef FS_SPLIT_CASE
  return fail(FS_EUNSUPPORTED, "fs_local_train: no split kernel for this shape");
}

int split_idle_cus(int N, int C, int B, int64_t ld, int G, int chained) {
  const int NT = (int)(ld >> 6);
  if (G & FS_G_PIPE) {
    const int g = G & (FS_G_PAIR - 1);
    const int cus = device_cus();
    if (chained || cus <= 0 || !pipe_fits(C, B, NT, g, 0)) return 0;
    return std::max(0, cus - pipe_groups(N, g, 0, cus) * g);
  }
  if (G & FS_G_PAIR) {
    const int g = G & (FS_G_PAIR - 1);
    const int cus = device_cus();
    if (chained || cus <= 0 || !pair_fits(C, B, NT, g)) return 0;
    return std::max(0, cus - pair_groups(N, g, cus) * g);
  }
  const int teams = (G & FS_G_TEAMS) ? 2 : 1;
  G &= FS_G_PAIR - 1;
  if (chained || G < 2 || C > 16 || B > 32 || !split_fits(C, B, NT, G, teams)) return 0;
  const int cus = device_cus();
  if (cus <= 0) return 0;
  return std::max(0, cus - split_groups(N, G, 0, cus, teams) * G);
}

}  // namespace fs

using namespace fs;

// Plan the launch: G = workgroups per client (1 = one workgroup walks each client; 2..16 =
// a group of G workgroups splits the feature dimension of one client at a time) and the
// workspace bytes it needs.  On entry *G_out is a request: 0 = let the planner choose,
// 1 = one workgroup per client, 2..16 = that group width if the shape allows it (else the
// planner's choice).
// prox: the FedProx term is on (kept in the ABI; every split variant covers it).
// max_en = max_j E * n_j.
extern "C" int fs_local_train_plan(int N, int C, int B, int E, int64_t ld, int64_t max_en, int chained, int prox,
                                   int* G_out, int64_t* ws_bytes_out) {
  FS_REQUIRE(G_out && ws_bytes_out, "null pointer");
  FS_REQUIRE(N >= 1 && B >= 1 && ld >= 64 && ld % 64 == 0, "bad sizes");
  const int want = *G_out;
  *G_out = 1;
  *ws_bytes_out = 0;
  const int cus = device_cus();
  if (want == 1 || C > 16 || B > 32 || cus <= 0) return FS_OK;
  const int NT = (int)(ld >> 6);
  // an explicit pipe request
  if (want & FS_G_PIPE) {
    const int g = want & (FS_G_PAIR - 1);
    if (pipe_fits(C, B, NT, g, prox) && g <= cus) {
      *G_out = g | FS_G_PIPE;
      *ws_bytes_out = pipe_ws_bytes(N, g, chained, cus);
      return FS_OK;
    }
  }
  // the pipe form (fs_tuning.split_pipe = 1: wherever it fits; -1 = never; 0 = by shape: parallel
  // clients at G <= 4 where its groups walk several clients each -- config 4, 1,250 clients of 64
  // rows on 128 groups of 2: 395-409 vs 419-448 us per launch for the pair form (G = 4) and
  // 285-302 vs 300-310 us at config 2's 100 clients, where the split form stays
  // (profiles/r05/pipe_vs_forms.txt); config 5's G = 16: 6.5 vs 4.9 ms, not chosen)
  // (entered for an automatic choice or a pipe request only: an explicit split, pair or team
  // request is answered by its own form, never by the pipe form under split_pipe = 1)
  if ((want == 0 || (want & FS_G_PIPE)) && NT % 16 == 0 && tuning().split_pipe >= 0) {
    const int g = NT / 16;
    const bool by_shape = tuning().split_pipe == 0 && want == 0 && tuning().train_form == 0 && !chained &&
                          !prox && g <= 4 && N > pipe_groups(N, g, 0, cus);
    if ((tuning().split_pipe > 0 || by_shape) && pipe_fits(C, B, NT, g, prox) && g <= cus) {
      *G_out = g | FS_G_PIPE;
      *ws_bytes_out = pipe_ws_bytes(N, g, chained, cus);
      return FS_OK;
    }
  }
  // an explicit team request
  if (want & FS_G_TEAMS) {
    const int g = want & (FS_G_PAIR - 1);
    if (!chained && (g == 4 || g == 8) && split_fits(C, B, NT, g, 2) && g <= cus) {
      *G_out = g | FS_G_TEAMS;
      *ws_bytes_out = split_ws_bytes(N, g, B, 0, cus, 2);
      return FS_OK;
    }
  }
  // an explicit pair request
  if (want & FS_G_PAIR) {
    const int g = want & (FS_G_PAIR - 1);
    if (!chained && pair_fits(C, B, NT, g) && g <= cus) {
      *G_out = g | FS_G_PAIR;
      *ws_bytes_out = pair_ws_bytes(N, g, B, cus);
      return FS_OK;
    }
  }
  int G = (want > 1 && want < FS_G_PAIR && split_fits(C, B, NT, want) && want <= cus) ? want : 0;
  // the team form by tuning (fs_tuning.split_teams = 1: wherever it fits, at the narrowest
  // width; 0 = by shape: not yet chosen automatically; -1 never)
  if (G == 0 && !chained && tuning().split_teams > 0)
    for (int cand : {4, 8})
      if (split_fits(C, B, NT, cand, 2) && cand <= cus) {
        *G_out = cand | FS_G_TEAMS;
        *ws_bytes_out = split_ws_bytes(N, cand, B, 0, cus, 2);
        return FS_OK;
      }
  if (G == 0) {
    if (chained) {
      // one group walks the chain: slice one step's batch (B x ld floats) to ~32 KB per CU
      const int64_t bytes = (int64_t)B * ld * 4;
      for (int cand : {2, 4, 8, 16})
        if (split_fits(C, B, NT, cand) && cand <= cus) {
          G = cand;
          if (bytes / cand <= 32 * 1024) break;
        }
    } else {
      // parallel clients: the narrowest split group that fits (most clients in flight, fewest
      // partners) -- FedProx too since its anchor is re-read, not register-resident (r02t, prox,
      // us per launch, G = 1 vs split: config 2 741 / 362, config 3 5955 / 5263, config 4
      // 580 / 508, config 5 11237 / 7003)
      for (int cand : {2, 4, 8, 16})
        if (split_fits(C, B, NT, cand) && cand <= cus) { G = cand; break; }
      // ... unless the pair form fits and its groups would walk several clients each (where it
      // measured faster: config 4 0.434 vs 0.457 ms; with one client per group, config 2, the
      // split form: 0.343 vs 0.366 ms -- profiles/r03/pair_ab.txt) and there is no prox term
      // (round 5, config 3: split G = 4 5.09-5.11 ms vs pair G = 8 5.24-5.26 and pipe G = 4
      // 5.25-5.27, profiles/r05/forms_config3_4.txt; round 3 had measured the pair form ahead,
      // 5.16 vs 5.26), or fs_tuning.train_form asks for it (1: never, 2: wherever it fits)
      const int form = tuning().train_form;
      if (form != 1)
        for (int cand : {2, 4, 8, 16})
          if (pair_fits(C, B, NT, cand) && cand <= cus &&
              (form == 2 || G == 0 || (!prox && (int64_t)N > (int64_t)split_groups(N, G, 0, cus)))) {
            *G_out = cand | FS_G_PAIR;
            *ws_bytes_out = pair_ws_bytes(N, cand, B, cus);
            return FS_OK;
          }
    }
  }
  (void)max_en;
  (void)E;
  if (G == 0) return FS_OK;
  *G_out = G;
  *ws_bytes_out = split_ws_bytes(N, G, B, chained, cus);
  return FS_OK;
}
#else
}  // namespace fs
#endif
