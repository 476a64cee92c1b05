// Split-client local training: G workgroups (on G CUs) cooperate on ONE client.
//
// Same math as local_train.hip (train_loop, /root/reference/functions/tools.py:177-215),
// used when a round has fewer clients than the chip has CUs (e.g. BASELINE config 2:
// 100 clients on 256 CUs).  Workgroup g of a client owns a contiguous range of 64-column
// feature tiles (its "slice"):
//   * its slice of the client's weights lives in REGISTERS for the whole local training
//     (lane-owned: lane (c, k-slot) holds W[c][64T + 16 k + 4 q + e]), anchor likewise;
//   * each step's gathered batch rows of its slice are staged ONCE in LDS (one HBM read
//     per byte), and both the forward (z_g = X_b,g W_g^T) and the backward
//     (grad_g^T = X_b,g^T G) read that image with v_mfma_f32_16x16x4_f32;
//   * the next step's slice is loaded into registers while the partners exchange
//     partial logits and written to LDS after the backward (async-stage split);
//   * per step the G partial logit tiles (plus the partial squared norms of W - W_a and
//     W the prox / ridge terms need) are exchanged through a small global buffer with
//     the write-through (sc1) stores + drained flag / sc1 loads hand-off of
//     cdna_hip_programming.md Guideline 16 (no fences on the per-step critical path);
//     every workgroup sums the G partials in the same fixed order, so all of them
//     compute bitwise-identical softmax gradients.
// Co-residency: the G partners spin on each other, so the launcher uses this path only
// when N*G workgroups fit on the device at one per CU; every spin is bounded and a
// timeout is reported through the workspace error word instead of hanging the GPU.
#include "common.h"

namespace fs {

constexpr int SP_WAVES = 8;
constexpr int SP_THREADS = SP_WAVES * 64;
constexpr int SP_IDX = 1536;           // E * n_j batch positions staged per client (all epochs)
constexpr unsigned SP_SPIN_LIMIT = 1u << 22;
#ifndef SP_STAGGER_CYCLES
#define SP_STAGGER_CYCLES 0
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
    if (k > 0) stamp_acc[k - 1] += t_ - stamp_prev;                                       \
    stamp_prev = t_;                                                                      \
  }
#else
#define SP_STAMP(k)
#endif

struct SplitWS {
  unsigned* flags;                     // [N][G] epoch of the last published step
  unsigned* err;                       // [1] nonzero: a partner never arrived (spin bound hit)
  unsigned long long* xbuf;            // [N][2][G][SZ] published partials: {epoch, value} granules
  unsigned long long* stamps;          // [grid][16] diagnostic build only
  int G;
  int SZ;
};

// Workgroup barrier for LDS hand-offs only.  __syncthreads() carries a workgroup-scope
// release that drains vmcnt -- i.e. waits for the next slice's loads in flight; this waits
// for this wave's LDS operations (lgkmcnt) and nothing else.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int tile_lo(int g, int G, int NT) { return (int)(((int64_t)NT * g) / G); }

template <int RT, int G, int TPW, bool PROX>
__global__ __launch_bounds__(SP_THREADS) void local_train_split_kernel(LTParams P, SplitWS X) {
  constexpr int CT = 1;
  constexpr int NC = CT * 16;
  constexpr int NR = RT * 16;
  constexpr int NZ = NR * NC;
  __shared__ float zpart[SP_WAVES][NR][NC];
  __shared__ float zg[NR][NC];
  __shared__ float zsum[NR][NC];
  __shared__ int erow[SP_IDX];
  __shared__ unsigned char elab[SP_IDX];
  __shared__ float wred[SP_WAVES][2];
  __shared__ float wce[SP_WAVES];
  __shared__ float nrm[2];
  __shared__ float nrmg[2];
  extern __shared__ __attribute__((aligned(16))) float xs_lds[];   // [NR][RS] batch slice image

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l16 = lane & 15, lg = lane >> 4;
  const int64_t ld = P.ld;
  const int NT = (int)(ld >> 6);
  const int C = P.C, B = P.B, E = P.E;

  // block -> (client slot, slice), partners on one XCD when the grid allows it (speed only)
  const int nb = gridDim.x;
  int lin = blockIdx.x;
  if (nb % 8 == 0 && (nb / 8) % G == 0) lin = (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8;
  const int cs = lin / G, g = lin % G;
  const int j = P.order ? P.order[cs] : cs;
  const int t0 = tile_lo(g, G, NT), t1 = tile_lo(g + 1, G, NT);
  const int NTS = t1 - t0;                       // tiles of this slice
  const int DS = NTS * 64;                       // slice width (floats)
  const int RS = DS + 4;                         // LDS row stride (floats)
  const int64_t row0 = P.row_off[j];
  const int n = (int)(P.row_off[j + 1] - row0);
  const int nbat = (n + B - 1) / B;
  const int steps = E * nbat;
  const float* start = P.W_start;
  float* Wj = P.W_out + (int64_t)j * C * ld;
  unsigned long long* xb = X.xbuf + (int64_t)cs * 2 * G * X.SZ;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);

  // ---- weights (and prox anchor) of this slice into registers ----
  float4 wr[TPW][4], ar[TPW][4];
  float nw0 = 0.f;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int Tl = w + SP_WAVES * i;
    const bool ok = Tl < NTS && l16 < C;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t off = (int64_t)l16 * ld + 64 * (t0 + Tl) + 16 * lg + 4 * q;
      wr[i][q] = ok ? ld4(start + off) : zero4;
      if (PROX) ar[i][q] = wr[i][q];
      nw0 += wr[i][q].x * wr[i][q].x + wr[i][q].y * wr[i][q].y + wr[i][q].z * wr[i][q].z + wr[i][q].w * wr[i][q].w;
    }
  }
  if (steps == 0) {
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int Tl = w + SP_WAVES * i;
      if (Tl < NTS && l16 < C)
#pragma unroll
        for (int q = 0; q < 4; ++q) st4(Wj + (int64_t)l16 * ld + 64 * (t0 + Tl) + 16 * lg + 4 * q, wr[i][q]);
    }
    if (g == 0 && tid == 0) P.loss[j] = 0.0;
    return;
  }
  if (E * n > SP_IDX) {                          // caller broke the plan: report, no hand-off attempted
    if (tid == 0) __hip_atomic_store(X.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  nw0 = wave_sum(nw0);
  if (lane == 0) { wred[w][0] = 0.f; wred[w][1] = nw0; }

  // ---- all epochs' shuffled rows + labels of this client into LDS ----
  for (int i = tid; i < E * n; i += SP_THREADS) {
    const int li = P.perms[(int64_t)E * row0 + i];
    erow[i] = (int)(row0 + li);
    elab[i] = (unsigned char)P.labels[row0 + li];
  }
  __syncthreads();

  // staging of one step's slice: thread -> one batch row (tr) and NPT float4 of it,
  // 16 B apart by TPR threads (TPR consecutive lanes read TPR*16 contiguous bytes), so a
  // thread needs one row address and immediate offsets; the zero fill of rows past the
  // batch end happens at the LDS store, never right behind a load (that would force a wait).
  constexpr int TPR = SP_THREADS / NR;                       // threads per row
  constexpr int NPT = (8 * TPW * 64 / 4) / TPR;              // max float4 per thread
  const int tr = tid / TPR, tc = tid - tr * TPR;
  const int F4R = DS / 4;                                    // float4 per row of the slice
  float4 stg[NPT];
#define SP_STAGE_LOAD(ST_)                                                          \
  {                                                                                 \
    const int e_ = (ST_) / nbat, s_ = (ST_) - e_ * nbat;                            \
    const int b0_ = s_ * B, bc_ = min(B, n - b0_);                                  \
    const float* src_ = P.phi + (int64_t)erow[e_ * n + b0_ + (tr < bc_ ? tr : 0)] * ld + 64 * t0 + 4 * tc; \
    _Pragma("unroll") for (int i = 0; i < NPT; ++i)                                 \
      if (tc + TPR * i < F4R) stg[i] = ld4(src_ + 4 * TPR * i);                     \
  }
#define SP_STAGE_STORE(ST_)                                                         \
  {                                                                                 \
    const int e_ = (ST_) / nbat, s_ = (ST_) - e_ * nbat;                            \
    const bool ok_ = tr < min(B, n - s_ * B);                                       \
    float* dst_ = xs_lds + tr * RS + 4 * tc;                                        \
    _Pragma("unroll") for (int i = 0; i < NPT; ++i)                                 \
      if (tc + TPR * i < F4R) st4(dst_ + 4 * TPR * i, ok_ ? stg[i] : zero4);        \
    (void)e_;                                                                       \
  }
  SP_STAGE_LOAD(0);
  SP_STAGE_STORE(0);
  __syncthreads();

  // Stagger: every client runs the same load -> compute -> exchange cycle, so in lockstep
  // all CUs would burst their next-slice loads into HBM at the same moment and idle it
  // during compute.  Client slot cs starts (cs % 4) quarter-steps late (wall-clock delay;
  // speed only, results unaffected) so the chip's load bursts interleave.
  if (SP_STAGGER_CYCLES > 0 && (cs & 3)) {
    const unsigned long long t_end = __builtin_amdgcn_s_memtime() + (unsigned long long)(cs & 3) * SP_STAGGER_CYCLES;
    while (__builtin_amdgcn_s_memtime() < t_end) __builtin_amdgcn_s_sleep(8);
  }

  double lsum = 0.0;
#ifdef FS_STAMPS
  unsigned long long stamp_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, stamp_prev = 0;
#endif
  for (int st = 0; st < steps; ++st) {
    SP_STAMP(0)
    const int e = st / nbat, s = st - e * nbat;
    const int b0 = s * B, bc = min(B, n - b0);
    const int par = st & 1;
    const unsigned epoch = (unsigned)st + 1u;
    const bool more = st + 1 < steps;

    // ---------------- forward partial: z_g = X_slice W_slice^T ----------------
    floatx4 acc[RT][CT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int Tl = w + SP_WAVES * i;
      if (Tl < NTS) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float4 xv[RT];
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) xv[rt] = ld4(xs_lds + (rt * 16 + l16) * RS + 64 * Tl + 16 * lg + 4 * q);
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
              for (int ct = 0; ct < CT; ++ct)
                acc[rt][ct] = mfma4(comp(xv[rt], e4), comp(wr[i][q], e4), acc[rt][ct]);
        }
      }
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int i = 0; i < 4; ++i) zpart[w][rt * 16 + 4 * lg + i][ct * 16 + l16] = acc[rt][ct][i];
    SP_STAMP(1)
    lds_barrier();  // S1: wave partials (and the previous update's norm partials)
    SP_STAMP(2)

    // ---- this slice's partial logits, fixed wave order ----
    for (int idx = tid; idx < NZ; idx += SP_THREADS) {
      const int r = idx / NC, c = idx - r * NC;
      float z = 0.f;
#pragma unroll
      for (int i = 0; i < SP_WAVES; ++i) z += zpart[i][r][c];
      zg[r][c] = z;
    }
    if (tid < 2) {
      float v = 0.f;
      for (int i = 0; i < SP_WAVES; ++i) v += wred[i][tid];
      nrmg[tid] = v;
    }
    lds_barrier();  // S1b
    SP_STAMP(3)

    // ---- hand-off, wave 0 only (the other waves' loads are not in flight yet, and vmcnt is
    // in order, so wave 0's waits cover exactly the hand-off traffic).  Guideline 16, R2
    // form: every value travels as one 8-byte {epoch, value} granule written by ONE
    // relaxed agent-scope (sc1) store -- the data is its own flag; a partner re-reads its
    // granules with sc1 loads until every tag equals this step's epoch: one round trip
    // once the data is there, no separate flag, no fences.  Tags are epochs (step + 1) of
    // this launch; the launcher zeroes the buffer before every launch.
    unsigned long long* slot = xb + ((int64_t)par * G) * X.SZ;
    if (w == 0) {
      constexpr int PER = (NZ + 2 + 63) / 64;
      const float* zgf = &zg[0][0];
      const unsigned long long tag = (unsigned long long)epoch << 32;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int idx = lane + 64 * k;
        if (idx < NZ + 2) {
          const float v = idx < NZ ? zgf[idx] : nrmg[idx - NZ];
          __hip_atomic_store(slot + (int64_t)g * X.SZ + idx, tag | __float_as_uint(v), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      // sum in slice order 0..G-1 (identical logits in every partner); all of a partner's
      // granules are loaded before any is checked: one round trip per sweep
      float pv[G - 1][PER];
      for (int hh = 0; hh < G - 1; ++hh) {
        const int h = hh < g ? hh : hh + 1;
        const unsigned long long* src = slot + (int64_t)h * X.SZ;
        unsigned spins = 0;
        for (;;) {
          bool ok = true;
#pragma unroll
          for (int k = 0; k < PER; ++k) {
            const int idx = lane + 64 * k;
            unsigned long long x = tag;
            if (idx < NZ + 2) x = __hip_atomic_load(src + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pv[hh][k] = __uint_as_float((unsigned)x);
            ok &= (x >> 32) == (unsigned long long)epoch;
          }
          if (__all(ok)) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > SP_SPIN_LIMIT) {
            if (lane == 0) __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
      float* zf = &zsum[0][0];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int idx = lane + 64 * k;
        if (idx < NZ + 2) {
          const float own = idx < NZ ? zgf[idx] : nrmg[idx - NZ];
          float v = 0.f;
#pragma unroll
          for (int h = 0; h < G; ++h) v += (h == g) ? own : pv[h < g ? h : h - 1][k];
          if (idx < NZ) zf[idx] = v;
          else nrm[idx - NZ] = v;                // ||W - W_a||^2, ||W||^2 at the start of this step
        }
      }
    }
    SP_STAMP(4)
    lds_barrier();  // S2: summed logits and norms
    SP_STAMP(5)
    const float invb = 1.0f / (float)bc;
    float cep = 0.f;
    for (int idx = tid; idx < NZ; idx += SP_THREADS) {   // NC lanes of one wave hold one row
      const int r = idx / NC, c = idx - r * NC;
      const float z = zsum[r][c];
      const bool valid = r < bc && c < C;
      float m = valid ? z : -INFINITY;
#pragma unroll
      for (int off = NC / 2; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
      float se = valid ? expf(z - m) : 0.f;
#pragma unroll
      for (int off = NC / 2; off > 0; off >>= 1) se += __shfl_xor(se, off, 64);
      float gv = 0.f;
      if (valid) {
        const float lp = z - m - logf(se);
        const bool isy = c == (int)elab[e * n + b0 + r];
        gv = (isy ? -invb : 0.f) + expf(lp) * invb;
        if (isy) cep -= lp;
      }
      zpart[0][r][c] = gv;                     // g lives in zpart[0] for the backward
    }
    cep = wave_sum(cep);
    if (lane == 0) wce[w] = cep;
    lds_barrier();  // S3: g, CE partials
    // next step's slice, issued around the backward so it streams behind the backward MFMAs
    // and lands in LDS after S4 (issuing it during the hand-off slowed the hand-off's own
    // round trips, which queue behind it in the CU's memory pipe).  Issuing 16 KB per wave
    // stalls the issuing wave on the memory pipe, so the two waves of a SIMD are staggered:
    // waves 4-7 issue first and then compute, waves 0-3 compute first and then issue, and
    // each SIMD's MFMA pipe always has one wave feeding it.
    const bool load_first = w >= SP_WAVES / 2;
    if (more && load_first) SP_STAGE_LOAD(st + 1);
    SP_STAMP(6)
    const float pn2 = nrm[0], wn2 = nrm[1];
    if (g == 0 && tid == 0 && e == E - 1) {
      float ce = 0.f;
      for (int i = 0; i < SP_WAVES; ++i) ce += wce[i];
      float loss = ce / (float)bc;
      if (P.prox) loss = loss + P.mu * sqrtf(pn2);
      if (P.reg) loss = loss + P.lam * sqrtf(wn2);
      lsum += (double)loss * (double)bc;
    }

    // ---------------- backward + update of the register-resident slice ----------------
    float gB[4 * RT][CT];
#pragma unroll
    for (int kk = 0; kk < 4 * RT; ++kk)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) gB[kk][ct] = zpart[0][4 * kk + lg][ct * 16 + l16];
    const float sp = (P.prox && pn2 > 0.f) ? P.mu / sqrtf(pn2) : 0.f;
    const float sr = (P.reg && wn2 > 0.f) ? P.lam / sqrtf(wn2) : 0.f;
    const float lr = P.lr;
    float npn = 0.f, nwn = 0.f;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int Tl = w + SP_WAVES * i;
      if (Tl < NTS) {
        floatx4 ga[4];
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) ga[e4] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 4 * RT; ++kk) {
          const float4 x = ld4(xs_lds + (4 * kk + lg) * RS + 64 * Tl + 4 * l16);
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) ga[e4] = mfma4(comp(x, e4), gB[kk][0], ga[e4]);
        }
        if (l16 < C) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float o[4];
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) {
              const float wc = comp(wr[i][q], e4);
              const float ac = PROX ? comp(ar[i][q], e4) : 0.f;
              float gr = ga[e4][q];
              if (PROX) gr = gr + (wc - ac) * sp;
              if (P.reg) gr = gr + wc * sr;
              o[e4] = wc - lr * gr;
              const float dp = o[e4] - ac;
              npn += dp * dp;
              nwn += o[e4] * o[e4];
            }
            wr[i][q] = make_float4(o[0], o[1], o[2], o[3]);
          }
        }
      }
    }
    if (more && !load_first) SP_STAGE_LOAD(st + 1);
    npn = wave_sum(npn);
    nwn = wave_sum(nwn);
    if (lane == 0) { wred[w][0] = npn; wred[w][1] = nwn; }
    SP_STAMP(7)
    lds_barrier();  // S4: every wave is done reading the slice image
    SP_STAMP(8)
    if (more) SP_STAGE_STORE(st + 1);
    lds_barrier();  // S5: next slice image visible
    SP_STAMP(9)
  }
#ifdef FS_STAMPS
  if (tid == 0 && X.stamps) {
    for (int k = 0; k < 9; ++k) X.stamps[blockIdx.x * 16 + k] = stamp_acc[k];
    X.stamps[blockIdx.x * 16 + 15] = (unsigned long long)steps;
  }
#endif

#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int Tl = w + SP_WAVES * i;
    if (Tl < NTS && l16 < C)
#pragma unroll
      for (int q = 0; q < 4; ++q) st4(Wj + (int64_t)l16 * ld + 64 * (t0 + Tl) + 16 * lg + 4 * q, wr[i][q]);
  }
  if (g == 0 && tid == 0) P.loss[j] = lsum / (double)n;
}

static int g_cus = 0;

static int device_cus() {
  if (g_cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) g_cus = 0;
  }
  return g_cus;
}

static size_t split_lds_bytes(int RT, int NT, int G) {
  const int tiles = (NT + G - 1) / G;
  return sizeof(float) * (size_t)(RT * 16) * (size_t)(tiles * 64 + 4);
}

constexpr size_t SP_STATIC_LDS = 8 * 32 * 16 * 4 + 2 * 32 * 16 * 4 + SP_IDX * 5 + 8 * 3 * 4 + 32;

static int64_t split_ws_bytes(int N, int G, int RT) {
  const int SZ = RT * 16 * 16 + 4;
  return 256 + ((int64_t)N * G * 4 + 255) / 256 * 256 + (int64_t)N * 2 * G * SZ * 8;
}

template <int RT, int G, int TPW, bool PROX>
static void launch_split_p(const LTParams& P, const SplitWS& X, size_t lds, hipStream_t st) {
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&local_train_split_kernel<RT, G, TPW, PROX>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((local_train_split_kernel<RT, G, TPW, PROX>), dim3(P.N * G), dim3(SP_THREADS), lds, st, P, X);
}

template <int RT, int G, int TPW>
static void launch_split_t(const LTParams& P, const SplitWS& X, size_t lds, hipStream_t st) {
  if (P.prox) launch_split_p<RT, G, TPW, true>(P, X, lds, st);
  else launch_split_p<RT, G, TPW, false>(P, X, lds, st);
}

int launch_local_train_split(const LTParams& P, int G, void* ws, int64_t ws_bytes, hipStream_t st) {
  const int RT = P.B <= 16 ? 1 : 2;
  const int NT = (int)(P.ld >> 6);
  if (!(G == 2 || G == 4)) return fail(FS_EINVAL, "fs_local_train: G must be 1, 2 or 4");
  if (P.C > 16 || P.B > 32) return fail(FS_EUNSUPPORTED, "fs_local_train: split clients need C <= 16, B <= 32");
  if (!ws || ws_bytes < split_ws_bytes(P.N, G, RT)) return fail(FS_EINVAL, "fs_local_train: workspace too small");
  const int cus = device_cus();
  if (cus <= 0 || P.N * G > cus) return fail(FS_EUNSUPPORTED, "fs_local_train: N*G workgroups exceed the CU count");
  const size_t lds = split_lds_bytes(RT, NT, G);
  if (lds + SP_STATIC_LDS > 160 * 1024) return fail(FS_EUNSUPPORTED, "fs_local_train: slice too wide for LDS");
  const int tiles = (NT + G - 1) / G;
  const int tpw = (tiles + SP_WAVES - 1) / SP_WAVES;
  char* base = reinterpret_cast<char*>(ws);
  SplitWS X;
  X.err = reinterpret_cast<unsigned*>(base);
  X.flags = reinterpret_cast<unsigned*>(base + 256);
  X.xbuf = reinterpret_cast<unsigned long long*>(base + 256 + ((int64_t)P.N * G * 4 + 255) / 256 * 256);
  X.G = G;
  X.SZ = RT * 16 * 16 + 4;
  X.stamps = nullptr;
#ifdef FS_STAMPS
  X.stamps = reinterpret_cast<unsigned long long*>(base + ws_bytes - (int64_t)P.N * G * 16 * 8);
#endif
  // error word, flags and granule tags: zeroed on the stream before every launch (epochs
  // restart at 1, so no granule of an earlier launch can carry a matching tag)
  hipError_t e = hipMemsetAsync(base, 0, (size_t)split_ws_bytes(P.N, G, RT), st);
  if (e != hipSuccess) return fail(FS_EHIP, std::string("fs_local_train: ") + hipGetErrorString(e));
#define FS_SPLIT_CASE(rt, g, tp) \
  if (RT == rt && G == g && tpw <= tp) { launch_split_t<rt, g, tp>(P, X, lds, st); return FS_OK; }
  FS_SPLIT_CASE(2, 2, 1) FS_SPLIT_CASE(2, 2, 2) FS_SPLIT_CASE(2, 4, 1) FS_SPLIT_CASE(2, 4, 2)
  FS_SPLIT_CASE(1, 2, 1) FS_SPLIT_CASE(1, 2, 2) FS_SPLIT_CASE(1, 2, 4) FS_SPLIT_CASE(1, 4, 1)
  FS_SPLIT_CASE(1, 4, 2) FS_SPLIT_CASE(1, 4, 4)
#undef FS_SPLIT_CASE
  return fail(FS_EUNSUPPORTED, "fs_local_train: no split kernel for this shape");
}

}  // namespace fs

using namespace fs;

// Plan the launch: G = workgroups per client (1 = one workgroup walks the client; 2 or 4 =
// split clients) and the workspace bytes it needs.  max_en = max_j E * n_j.
extern "C" int fs_local_train_plan(int N, int C, int B, int E, int64_t ld, int64_t max_en, int chained,
                                   int* G_out, int64_t* ws_bytes_out) {
  FS_REQUIRE(G_out && ws_bytes_out, "null pointer");
  FS_REQUIRE(N >= 1 && ld >= 64 && ld % 64 == 0, "bad sizes");
  *G_out = 1;
  *ws_bytes_out = 0;
  const int cus = device_cus();
  if (chained || C > 16 || B > 32 || max_en > SP_IDX || cus <= 0) return FS_OK;
  const int RT = B <= 16 ? 1 : 2;
  const int NT = (int)(ld >> 6);
  for (int G : {4, 2}) {
    if (N * G > cus || NT < G) continue;
    if (split_lds_bytes(RT, NT, G) + SP_STATIC_LDS > 160 * 1024) continue;
    const int tiles = (NT + G - 1) / G;
    if ((tiles + SP_WAVES - 1) / SP_WAVES > (RT == 2 ? 2 : 4)) continue;
    *G_out = G;
    *ws_bytes_out = split_ws_bytes(N, G, RT) + 4096;
    return FS_OK;
  }
  return FS_OK;
}
