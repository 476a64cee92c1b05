// Stream form of split-client local training (round 4): the split form's arithmetic
// (local_train_split.hip; train_loop, /root/reference/functions/tools.py:177-215) on FOUR
// waves per workgroup -- one per SIMD, so each wave may hold 512 registers -- with the batch
// rows DOUBLE-BUFFERED in registers.
//
// Why: in the split form (8 waves, 2 per SIMD, ~200 VGPRs each) a step's rows live in the one
// register set that the forward reads, so the next step's rows can only be issued once the
// image write has freed it: from the hand-off to the end of the backward.  The stamps put the
// CU's row stream at ~11 B/clk inside that window and idle through the forward, S1 and the
// publish (~6 k of ~19.8 k cycles per step at config 2), and the next forward waits for the
// loads issued last.  Here the rows sit in three register banks of two tiles' rows each
// (64 VGPRs): a step's rows in banks (X, Y), the first half of the next step's -- the tiles
// the next forward reads first -- go into the free bank Z from the first forward MFMA on, the
// second half into X once the image write has freed it; the banks rotate (X, Y, Z) -> (Z, X, Y)
// -> (Y, Z, X), so the stream runs through the forward and the hand-off as well.
//
// Scope: parallel clients, no prox anchor (FedAvg, FedAMW's local training; ridge allowed),
// full slices of 16 tiles per workgroup (ld = 1024 G: configs 2 and 5), B in (16, 32].
// Bitwise the split form: real wave w runs the split form's waves w and w + 4 ("virtual"
// waves: tiles w, w + 8 and w + 4, w + 12) with their partial sums -- forward logits, norms,
// cross-entropy -- kept apart and folded in the split form's wave order; the exchange, softmax,
// backward and update are the same per element (tests/test_gpu_stream.py).
#include "common.h"
#include "eval_rows.h"
#include "lanes.h"
#include "split_common.h"

namespace fs {

constexpr int ST_WAVES = 4;                // real waves
constexpr int ST_VW = 8;                   // the split form's waves
constexpr int ST_THREADS = ST_WAVES * 64;
constexpr int ST_TW = 4;                   // tiles per real wave: slot j -> virtual wave w + 4 (j >> 1), tile i = j & 1

#ifdef FS_STAMPS
#define ST_STAMP(k)                                                                       \
  {                                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    unsigned long long t_;                                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    if (k > 0) stamp_acc[k > 0 ? k - 1 : 0] += t_ - stamp_prev;                           \
    stamp_prev = t_;                                                                      \
  }
#else
#define ST_STAMP(k)
#endif

// LF: row loads of the next step a wave issues during the forward (one per forward iteration,
// from the first); LH: right after the hand-off's polls go out; the rest one per backward
// iteration (LF + LH <= 16: the loads before the image write go to the free bank).  Loads
// issued before the polls delay them (one in-order vector-memory counter per wave): LF stops
// early enough for its loads to have landed by then.
template <int G, int LF, int LH>
__global__ __launch_bounds__(ST_THREADS, 1) void local_train_stream_kernel(LTParams P, SplitWS X) {
  constexpr int RT = 2;
  constexpr int NTH = ST_THREADS;
  constexpr int NC = 16;
  constexpr int NR = RT * 16;
  constexpr int NZ = NR * NC;
  constexpr int NTS = ST_VW * 2;                  // tiles of the slice (full slices only)
  constexpr int RS = NTS * 64 + 8;                // LDS image row stride
  constexpr int M = ((G >= 8 ? 512 : NZ + 2) + NTH - 1) / NTH;   // exchanged values per thread
  constexpr int HC = G;
  constexpr int NLD = ST_TW * 4 * RT;             // row loads per wave and step (32)
  static_assert(LF + LH <= NLD / 2, "load schedule: the early loads fill the free bank");
  __shared__ __attribute__((aligned(16))) float zpart[ST_VW][NR * NC];
  __shared__ float gbuf[NR][NC];
  __shared__ float zsum[NR][NC];
  __shared__ int lab[2][NR];
  __shared__ float wred[ST_VW][2];
  __shared__ float wce[ST_VW];
  __shared__ float nrm[2];
  extern __shared__ __attribute__((aligned(16))) float xs_lds[];   // [NR][RS] batch slice image

  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, lg = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t ld = P.ld;
  const int C = P.C, B = P.B, E = P.E;
  const int NV = NR * C + 2;

  const int nb = gridDim.x - P.fuse_E;
  if ((int)blockIdx.x >= nb) {                    // the fused evaluation (8 virtual waves)
    eval_persistent<ST_VW, 2>(P.fuse_phi, P.ld, P.fuse_y, P.fuse_n, P.W_start, P.C, (int)blockIdx.x - nb, P.fuse_E,
                              xs_lds, P.fuse_part);
    return;
  }
  int lin = blockIdx.x;
  if (nb % 8 == 0) lin = (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8;
  const int ng = X.ngroups;
  const int grp = lin / G, g = lin % G;
  if (grp >= ng) return;
  const int T = (P.N + ng - 1) / ng;              // client sequence length
  const int t0 = tile_lo(g, G, G * NTS);
  const float* start = P.W_start;
  unsigned long long* xb = X.xbuf + (int64_t)grp * 2 * G * X.SZ;
  // tile of slot j: virtual wave vw(j) = w + 4 (j >> 1), its tile (j & 1): vw + 8 (j & 1)
  auto tile_of = [&](int j) { return w + 4 * (j >> 1) + ST_VW * (j & 1); };

  // ---- weights of this slice in registers (slot j = tile_of(j)); per virtual wave ||W||^2 ----
  float4 wr[ST_TW][4];
  auto wbase = [&]() {
    int64_t b = (int64_t)l16 * ld + 64 * t0 + 4 * lg;
    asm volatile("" : "+v"(b));
    return b;
  };
  auto load_start = [&](float& s0, float& s1) {
    const int64_t base = wbase();
    s0 = 0.f;
    s1 = 0.f;
#pragma unroll
    for (int j = 0; j < ST_TW; ++j) {
      const bool ok = l16 < C;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        wr[j][q] = ok ? ld4(start + base + 64 * tile_of(j) + 16 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float sq = wr[j][q].x * wr[j][q].x + wr[j][q].y * wr[j][q].y + wr[j][q].z * wr[j][q].z +
                         wr[j][q].w * wr[j][q].w;
        if (j < 2) s0 += sq;
        else s1 += sq;
      }
    }
    s0 = wave_sum_dpp(s0, lane);
    s1 = wave_sum_dpp(s1, lane);
  };
  auto store_w = [&](float* Wj) {
    const int64_t base = wbase();
#pragma unroll
    for (int j = 0; j < ST_TW; ++j)
      if (l16 < C)
#pragma unroll
        for (int q = 0; q < 4; ++q) st4(Wj + base + 64 * tile_of(j) + 16 * q, wr[j][q]);
  };
  float nw0a, nw0b;
  load_start(nw0a, nw0b);
  if (lane == 0) {
    wred[w][0] = 0.f; wred[w][1] = nw0a;
    wred[w + 4][0] = 0.f; wred[w + 4][1] = nw0b;
  }

  // ---- rows: three banks of two slots; pn = the row indices of the step the cursor lc points at ----
  typedef float4 Bank[2][RT][4];
  Bank ba, bb, bc3;
  int pn[RT], lb[RT];
  SpCur lc;
  bool lc_ok = sp_seek(lc, P, grp, ng, T, 0);
  auto fetch_rows = [&]() {
    const int e_ = lc.st / lc.nbat, s_ = lc.st - e_ * lc.nbat;
    const int b0_ = s_ * B, bc_ = min(B, lc.n - b0_);
    const int32_t* pp_ = P.perms + (int64_t)E * lc.row0 + (int64_t)e_ * lc.n + b0_;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int r_ = rt * 16 + l16;
      pn[rt] = (int)(lc.row0 + pp_[r_ < bc_ ? r_ : 0]);
    }
  };
  // load f of a wave's step: slot f / 8, row tile (f / 4) & 1, q = f & 3 (every load is issued
  // unconditionally: pn always holds valid rows).  One base address per row tile (the lane's
  // row, this wave's first tile), rebuilt behind an empty asm once per step; every load is
  // that base + a compile-time offset (< 4 KB: the instruction's immediate)
  const float* rbase[RT];
  auto row_bases = [&]() {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      int64_t o = (int64_t)pn[rt] * ld + 64 * t0 + 4 * lg + 64 * w;
      asm volatile("" : "+v"(o));
      rbase[rt] = P.phi + o;
    }
  };
  // loads f < 16 (slots 0, 1) into bank z, the rest (slots 2, 3) into bank x
  auto issue = [&](Bank& z, Bank& x, int f) {
    const int j = f >> 3, rt = (f >> 2) & 1, q = f & 3;
    float4 v = ld4(rbase[rt] + 64 * (4 * (j >> 1) + ST_VW * (j & 1)) + 16 * q);
    if (j < 2) z[j][rt][q] = v;
    else x[j - 2][rt][q] = v;
  };
  if (lc_ok) {
    fetch_rows();
    row_bases();
#pragma unroll
    for (int f = 0; f < NLD; ++f) issue(ba, bb, f);      // step 0's rows: slots 0, 1 in ba, 2, 3 in bb
    if (w == 0 && lg == 0)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) lb[rt] = P.labels[pn[rt]];
    lc_ok = sp_advance(lc, P, grp, ng, T);
    if (lc_ok) fetch_rows();
  }
  __syncthreads();

  auto flush_empty = [&](int ka, int kb) {
    for (int k = ka; k < kb; ++k) {
      const int j = sp_client(P, grp, ng, k);
      if (j < 0) continue;
      float* Wj = P.W_out + (int64_t)j * C * ld;
      const int64_t base = wbase();
#pragma unroll
      for (int jj = 0; jj < ST_TW; ++jj)
        if (l16 < C)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int64_t off = base + 64 * tile_of(jj) + 16 * q;
            st4(Wj + off, ld4(start + off));
          }
      if (g == 0 && tid == 0) P.loss[j] = 0.0;
    }
  };

  SpCur cc;
  bool cc_ok = sp_seek(cc, P, grp, ng, T, 0);
  flush_empty(0, cc_ok ? cc.k : T);
  unsigned gs = 0;
  bool dead = false;
  double lsum = 0.0;
#ifdef FS_STAMPS
  unsigned long long stamp_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, stamp_prev = 0;
#endif

  // one step on the rows in banks (x: slots 0, 1; y: slots 2, 3), issuing the next step's into
  // (z, x): z is free, x once the image write has read it
  auto step = [&](Bank& x, Bank& y, Bank& z) {
    auto row = [&](int j, int rt, int q) -> const float4& { return j < 2 ? x[j][rt][q] : y[j - 2][rt][q]; };
    const int st = cc.st, n = cc.n, nbat = cc.nbat;
    if (st == 0) {                                // client start: W_start, the anchor norms reset
      if (gs > 0) {
        float s0, s1;
        load_start(s0, s1);
        if (lane == 0) {
          wred[w][0] = 0.f; wred[w][1] = nw0a;
          wred[w + 4][0] = 0.f; wred[w + 4][1] = nw0b;
        }
      }
      lsum = 0.0;
    }
    ST_STAMP(0)
    const int e = st / nbat, s = st - e * nbat;
    const int b0 = s * B, bc = min(B, n - b0);
    const int par = gs & 1;
    const unsigned tag32 = X.tag_base + gs + 1u;
    if (w == 0 && lg == 0)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) lab[par][rt * 16 + l16] = lb[rt];
    row_bases();                                  // the next step's rows (pn)

    // ---------------- forward partials of the two virtual waves ----------------
    floatx4 acc[2][RT];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[u][rt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int it = 0; it < ST_TW * 4; ++it) {      // slot j = it / 4, q = it % 4: the split order per virtual wave
      const int j = it >> 2, q = it & 3, u = j >> 1;
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[u][rt] = mfma4(comp(row(j, rt, q), e4), comp(wr[j][q], e4), acc[u][rt]);
      if (it < LF) issue(z, x, it);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        st4(&zpart[w + 4 * u][rt * 256 + lg * 64 + l16 * 4],
            make_float4(acc[u][rt][0], acc[u][rt][1], acc[u][rt][2], acc[u][rt][3]));
    ST_STAMP(1)
    lds_barrier();  // S1
    ST_STAMP(2)
    {
      unsigned long long* slot = xb + ((int64_t)par * G) * X.SZ;
      const unsigned long long tag = (unsigned long long)tag32 << 32;
      float own[M], sum[M];
      unsigned long long pl[M][HC];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int idx = tid + NTH * m;
        float v = 0.f;
        if (idx < NV - 2) {
          const int r = idx / C, c = idx - r * C;
#pragma unroll
          for (int i = 0; i < ST_VW; ++i) v += zpart[i][zp_off(r, c)];
        } else if (idx < NV) {
#pragma unroll
          for (int i = 0; i < ST_VW; ++i) v += wred[i][idx - (NV - 2)];
        }
        own[m] = v;
        sum[m] = 0.f;
        if (idx < NV)
          __hip_atomic_store(slot + (int64_t)g * X.SZ + idx, tag | __float_as_uint(v), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      ST_STAMP(3)
      if (X.spin_limit == 0 && gs == 0 && lane == 0)
        __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned spins = 0;
      auto poll = [&]() {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const int idx = tid + NTH * m;
#pragma unroll
          for (int h = 0; h < HC; ++h)
            pl[m][h] = __hip_atomic_load(slot + (int64_t)h * X.SZ + (idx < NV ? idx : 0), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        }
      };
      poll();
      // the polls are out: loads issued from here on are younger and never delay them
#pragma unroll
      for (int f = LF; f < LF + LH; ++f) issue(z, x, f);
      // image write (the backward reads this step's rows from LDS)
#pragma unroll
      for (int j = 0; j < ST_TW; ++j)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int q = 0; q < 4; ++q) st4(xs_lds + img_off(rt * 16 + l16, RS, tile_of(j), 4 * q + lg), row(j, rt, q));
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
          for (int h = 0; h < HC; ++h)
            ok &= (h == g) | (tid + NTH * m >= NV) | ((unsigned)(pl[m][h] >> 32) == tag32);
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
        for (int h = 0; h < HC; ++h) sum[m] += (h == g) ? own[m] : __uint_as_float((unsigned)pl[m][h]);
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int idx = tid + NTH * m;
        if (idx < NV) {
          if (idx < NV - 2) {
            const int r = idx / C, c = idx - r * C;
            zsum[r][c] = sum[m];
          } else {
            nrm[idx - (NV - 2)] = sum[m];
          }
        }
      }
      ST_STAMP(4)
    }
    lds_barrier();  // S2: summed logits and norms, the image
    ST_STAMP(5)
    const float invb = 1.0f / (float)bc;
    float cep[2] = {0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {                 // idx = tid + 256 u: the split form's wave w + 4 u
      const int idx = tid + NTH * u;
      const int r = idx / NC, c = idx - r * NC;
      const bool valid = r < bc && c < C;
      const float z = valid ? zsum[r][c] : 0.f;
      float m = valid ? z : -INFINITY;
#pragma unroll
      for (int off = NC / 2; off > 0; off >>= 1) m = fmaxf(m, xor_get(m, off, lane));
      const float ex = valid ? __expf(z - m) : 0.f;
      float se = ex;
#pragma unroll
      for (int off = NC / 2; off > 0; off >>= 1) se += xor_get(se, off, lane);
      float gv = 0.f;
      if (valid) {
        const bool isy = c == lab[par][r];
        gv = (isy ? -invb : 0.f) + ex * __builtin_amdgcn_rcpf(se) * invb;
        if (isy) cep[u] -= z - m - __logf(se);
      }
      gbuf[r][c] = gv;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      cep[u] = wave_sum_dpp(cep[u], lane);
      if (lane == 0) wce[w + 4 * u] = cep[u];
    }
    lds_barrier();  // S3: g, CE partials
    ST_STAMP(6)
    const float wn2 = nrm[1];
    if (g == 0 && tid == 0 && e == E - 1) {
      float ce = 0.f;
      for (int i = 0; i < ST_VW; ++i) ce += wce[i];
      float loss = ce / (float)bc;
      if (P.reg) loss = loss + P.lam * sqrtf(wn2);
      lsum += (double)loss * (double)bc;
    }

    // ---------------- backward + update of the register-resident slice ----------------
    float gB[4 * RT];
#pragma unroll
    for (int kk = 0; kk < 4 * RT; ++kk) gB[kk] = gbuf[4 * kk + lg][l16];
    const float sr = (P.reg && wn2 > 0.f) ? P.lam / sqrtf(wn2) : 0.f;
    const float lr = P.lr;
    const int rblk = 4 * (l16 & 3) + (l16 >> 2);
#pragma unroll
    for (int j = 0; j < ST_TW; ++j) {
      const int Tl = tile_of(j);
      floatx4 ga[4];
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) ga[e4] = floatx4{0.f, 0.f, 0.f, 0.f};
      const float* ib0 = xs_lds + lg * RS + 64 * Tl + 4 * (rblk ^ lg);
      const float* ib1 = xs_lds + lg * RS + 64 * Tl + 4 * (rblk ^ (lg + 4));
#pragma unroll
      for (int kk = 0; kk < 4 * RT; ++kk) {
        const float4 xv = ld4(((kk & 1) ? ib1 : ib0) + 4 * kk * RS);
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) ga[e4] = mfma4(comp(xv, e4), gB[kk], ga[e4]);
        const int f = LF + LH + j * 4 * RT + kk;   // the rest of the stream, one per iteration
        if (f < NLD) issue(z, x, f);
      }
      if (l16 < C) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float o[4];
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) {
            const float wc = comp(wr[j][q], e4);
            float gr = ga[e4][q];
            if (P.reg) gr = gr + wc * sr;
            o[e4] = wc - lr * gr;
          }
          wr[j][q] = make_float4(o[0], o[1], o[2], o[3]);
        }
      }
    }
    if (lc_ok) {
      if (w == 0 && lg == 0)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) lb[rt] = P.labels[pn[rt]];
      lc_ok = sp_advance(lc, P, grp, ng, T);
      if (lc_ok) fetch_rows();
    }
    // ridge: ||W||^2 of the updated slice per virtual wave, in the split form's (i, q, e4) order
    if (P.reg) {
      float nwn[2] = {0.f, 0.f};
#pragma unroll
      for (int j = 0; j < ST_TW; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) nwn[j >> 1] += comp(wr[j][q], e4) * comp(wr[j][q], e4);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        nwn[u] = wave_sum_dpp(nwn[u], lane);
        if (lane == 0) { wred[w + 4 * u][0] = 0.f; wred[w + 4 * u][1] = nwn[u]; }
      }
    }
    ST_STAMP(7)
    if (st == cc.steps - 1) {
      store_w(P.W_out + (int64_t)cc.j * C * ld);
      if (g == 0 && tid == 0) P.loss[cc.j] = lsum / (double)n;
    }
    const int kprev = cc.k;
    cc_ok = sp_advance(cc, P, grp, ng, T);
    flush_empty(kprev + 1, cc_ok ? cc.k : T);
    ++gs;
  };
  while (cc_ok) {
    step(ba, bb, bc3);
    if (!cc_ok) break;
    step(bc3, ba, bb);
    if (!cc_ok) break;
    step(bb, bc3, ba);
  }
#ifdef FS_STAMPS
  if (tid == 0 && X.stamps) {
    for (int k = 0; k < 8; ++k) X.stamps[blockIdx.x * 16 + k] = stamp_acc[k];
    X.stamps[blockIdx.x * 16 + 15] = (unsigned long long)gs;
  }
#endif
}

// ---- launch (called by the split launcher for the shapes this form covers) ----
bool stream_fits(const LTParams& P, int G) {
  return !P.prox && !P.chained && P.B > 16 && P.B <= 32 && P.C <= 16 && (G == 2 || G == 4 || G == 8 || G == 16) &&
         (P.ld >> 6) == (int64_t)G * 16;
}

// default load schedule (LF, LH): row loads per wave during the forward / right after the polls
#ifndef ST_LF
#define ST_LF 8
#endif
#ifndef ST_LH
#define ST_LH 8
#endif

template <int G>
static void launch_stream_g(const LTParams& P, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  const void* k = reinterpret_cast<const void*>(&local_train_stream_kernel<G, ST_LF, ST_LH>);
  if (lds > 64 * 1024) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((local_train_stream_kernel<G, ST_LF, ST_LH>), dim3(grid), dim3(ST_THREADS), lds, st, P, X);
}

int launch_local_train_stream(const LTParams& P, int G, const SplitWS& X, int grid, size_t lds, hipStream_t st) {
  switch (G) {
    case 2: launch_stream_g<2>(P, X, grid, lds, st); return FS_OK;
    case 4: launch_stream_g<4>(P, X, grid, lds, st); return FS_OK;
    case 8: launch_stream_g<8>(P, X, grid, lds, st); return FS_OK;
    case 16: launch_stream_g<16>(P, X, grid, lds, st); return FS_OK;
    default: return fail(FS_EUNSUPPORTED, "fs_local_train: no stream kernel for this width");
  }
}

}  // namespace fs
