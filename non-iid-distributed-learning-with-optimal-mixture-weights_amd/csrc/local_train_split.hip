// Split-client local training: G workgroups (on G CUs) cooperate on ONE client.
//
// Same math as local_train.hip (train_loop, /root/reference/functions/tools.py:177-215),
// used when a round has fewer clients than the chip has CUs (e.g. BASELINE config 2:
// 100 clients on 256 CUs, G = 2).  Workgroup g of a client owns a contiguous range of
// 64-column feature tiles (its "slice"); wave w owns tiles w, w + 8, ...:
//   * its slice of the client's weights lives in REGISTERS for the whole local training
//     (lane (c, k-slot) holds W[c][64T + 16 q + 4 k + e]), the prox anchor likewise;
//   * each step's gathered batch rows of the slice arrive in REGISTERS in the forward's
//     operand layout (64 contiguous bytes of 16 rows per load), so the forward
//     z_g = X_b,g W_g^T (v_mfma_f32_16x16x4_f32) reads no LDS; the same registers are then
//     written once into a bank-conflict-free LDS image that the backward
//     grad_g^T = X_b,g^T G reads, and are refilled with the next step's rows (half of the
//     waves issue those loads right after the hand-off, half after the softmax, so one wave
//     of each SIMD computes while its partner is held up issuing loads);
//   * per step the G partial logit tiles (plus the partial squared norms of W - W_a and W
//     the prox / ridge terms need) are exchanged through a small global buffer as 8-byte
//     {tag, value} granules -- the write-through (sc1) store / sc1 load hand-off of
//     cdna_hip_programming.md Guideline 16, R2 form (no fences, no flags) -- spread over
//     all 8 waves; every workgroup sums the G partials in the same fixed order, so all of
//     them compute bitwise-identical softmax gradients.
// Co-residency: the G partners spin on each other, so the launcher uses this path only
// when N*G workgroups fit on the device at one per CU; every spin is bounded and a
// timeout is reported through the workspace error word instead of hanging the GPU.
#include <atomic>

#include "common.h"

namespace fs {

constexpr int SP_WAVES = 8;
constexpr int SP_THREADS = SP_WAVES * 64;
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
    if (k > 0) stamp_acc[k > 0 ? k - 1 : 0] += t_ - stamp_prev;                                     \
    stamp_prev = t_;                                                                      \
  }
#else
#define SP_STAMP(k)
#endif

struct SplitWS {
  unsigned* err;                       // [1] sticky; nonzero: a partner never arrived (spin bound hit)
  unsigned long long* xbuf;            // [N][2][G][SZ] published partials: {tag, value} granules
  unsigned long long* stamps;          // [grid][16] diagnostic build only
  unsigned gen;                        // launch generation (1..65535): high half of every tag
  int G;
  int SZ;
};

__device__ __forceinline__ int tile_lo(int g, int G, int NT) { return (int)(((int64_t)NT * g) / G); }

// LDS image of one step's batch slice: row-major, row stride RS = DS + 8 floats, and the
// sixteen float4 blocks of every 64-column tile permuted by block ^ (row & 7).  With this
// layout both the image write (lanes 0-7 = eight rows, same block) and the backward's read
// (lanes = 16 blocks of one row, 4 rows per instruction) are bank-conflict free.
__device__ __forceinline__ int img_off(int row, int RS, int tile, int blk) {
  return row * RS + 64 * tile + 4 * (blk ^ (row & 7));
}

// Per-lane d mapping inside a 64-column tile (forward operand, weights, gradient):
// lane (l16, lg), register q, component e  <->  d = 16 q + 4 lg + e.  One load instruction
// (fixed q) then reads 64 contiguous bytes of each of 16 rows.
template <int RT, int G, int TPW, bool PROX>
__global__ __launch_bounds__(SP_THREADS, 1) void local_train_split_kernel(LTParams P, SplitWS X) {
  constexpr int NW = SP_WAVES;
  constexpr int NC = 16;
  constexpr int NR = RT * 16;
  constexpr int NZ = NR * NC;
  __shared__ float zpart[NW][NR][NC];
  __shared__ float gbuf[NR][NC];
  __shared__ float zsum[NR][NC];
  __shared__ int lab[2][NR];
  __shared__ float wred[NW][2];
  __shared__ float wce[NW];
  __shared__ float nrm[2];
  extern __shared__ __attribute__((aligned(16))) float xs_lds[];   // [NR][RS] batch slice image

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l16 = lane & 15, lg = lane >> 4;
  const int64_t ld = P.ld;
  const int NT = (int)(ld >> 6);
  const int C = P.C, B = P.B, E = P.E;

  // block -> (client slot, slice): consecutive linear ids on one XCD under round-robin
  // placement, so a client's partners mostly share an L2 (speed only, results unaffected)
  const int nb = gridDim.x;
  int lin = blockIdx.x;
  if (nb % 8 == 0) lin = (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8;
  const int cs = lin / G, g = lin % G;
  const int j = P.order ? P.order[cs] : cs;
  const int t0 = tile_lo(g, G, NT), t1 = tile_lo(g + 1, G, NT);
  const int NTS = t1 - t0;                       // tiles of this slice
  const int RS = NTS * 64 + 8;                   // LDS row stride (floats)
  const int64_t row0 = P.row_off[j];
  const int n = (int)(P.row_off[j + 1] - row0);
  const int nbat = (n + B - 1) / B;
  const int steps = E * nbat;
  const float* start = P.W_start;
  float* Wj = P.W_out + (int64_t)j * C * ld;
  unsigned long long* xb = X.xbuf + (int64_t)cs * 2 * G * X.SZ;
  const int32_t* perm = P.perms + (int64_t)E * row0;
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);

  // ---- weights (and prox anchor) of this slice into registers ----
  float4 wr[TPW][4], ar[TPW][4];
  float nw0 = 0.f;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int Tl = w + NW * i;
    const bool ok = Tl < NTS && l16 < C;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t off = (int64_t)l16 * ld + 64 * (t0 + Tl) + 16 * q + 4 * lg;
      wr[i][q] = ok ? ld4(start + off) : zero4;
      if (PROX) ar[i][q] = wr[i][q];
      nw0 += wr[i][q].x * wr[i][q].x + wr[i][q].y * wr[i][q].y + wr[i][q].z * wr[i][q].z + wr[i][q].w * wr[i][q].w;
    }
  }
  if (steps == 0) {
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int Tl = w + NW * i;
      if (Tl < NTS && l16 < C)
#pragma unroll
        for (int q = 0; q < 4; ++q) st4(Wj + (int64_t)l16 * ld + 64 * (t0 + Tl) + 16 * q + 4 * lg, wr[i][q]);
    }
    if (g == 0 && tid == 0) P.loss[j] = 0.0;
    return;
  }
  nw0 = wave_sum(nw0);
  if (lane == 0) { wred[w][0] = 0.f; wred[w][1] = nw0; }

  // ---- the batch slice lives in registers in the forward's operand layout: lane (l16, lg)
  // holds rows rt*16 + l16, columns 16 q + 4 lg .. +3 of each of its tiles.  Rows past the
  // batch end load a valid row (their logits are ignored, their softmax gradient is 0).
  // The shuffle entry of a step's rows is fetched one step before its features.
  auto pos_of = [&](int st_, int r_) {
    const int e_ = st_ / nbat, s_ = st_ - e_ * nbat;
    const int b0_ = s_ * B, bc_ = min(B, n - b0_);
    return e_ * n + b0_ + (r_ < bc_ ? r_ : 0);
  };
  float4 xf[TPW][RT][4];
  int pn[RT], lb[RT];
#define SP_XLOAD()                                                                   \
  {                                                                                  \
    _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {                              \
      const int64_t r_ = row0 + pn[rt];                                              \
      if (w == 0 && lg == 0) lb[rt] = P.labels[r_];                                  \
      const float* src_ = P.phi + r_ * ld + 64 * t0 + 4 * lg;                        \
      _Pragma("unroll") for (int i = 0; i < TPW; ++i)                                \
        if (w + NW * i < NTS)                                                        \
          _Pragma("unroll") for (int q = 0; q < 4; ++q)                              \
            xf[i][rt][q] = ld4(src_ + 64 * (w + NW * i) + 16 * q);                   \
    }                                                                                \
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) pn[rt] = perm[pos_of(0, rt * 16 + l16)];
  SP_XLOAD();
  if (steps > 1)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) pn[rt] = perm[pos_of(1, rt * 16 + l16)];
  __syncthreads();

  double lsum = 0.0;
#ifdef FS_STAMPS
  unsigned long long stamp_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, stamp_prev = 0;
#endif
  for (int st = 0; st < steps; ++st) {
    SP_STAMP(0)
    const int e = st / nbat, s = st - e * nbat;
    const int b0 = s * B, bc = min(B, n - b0);
    const int par = st & 1;
    const unsigned tag32 = (X.gen << 16) | (unsigned)(st + 1);
    const bool more = st + 1 < steps;
    if (w == 0 && lg == 0)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) lab[par][rt * 16 + l16] = lb[rt];

    // ---------------- forward partial: z_g = X_slice W_slice^T (registers only) ----------------
    floatx4 acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TPW; ++i)
      if (w + NW * i < NTS)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) acc[rt] = mfma4(comp(xf[i][rt][q], e4), comp(wr[i][q], e4), acc[rt]);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) zpart[w][rt * 16 + 4 * lg + i][l16] = acc[rt][i];
    SP_STAMP(1)
    lds_barrier();  // S1: wave partials, norm partials of the previous update; the image is free
    SP_STAMP(2)

    // image write: the backward of this step reads the slice from LDS
#define SP_IMG_WRITE()                                                               \
  {                                                                                  \
    _Pragma("unroll") for (int i = 0; i < TPW; ++i)                                  \
      if (w + NW * i < NTS)                                                          \
        _Pragma("unroll") for (int rt = 0; rt < RT; ++rt)                            \
          _Pragma("unroll") for (int q = 0; q < 4; ++q)                              \
            st4(xs_lds + img_off(rt * 16 + l16, RS, w + NW * i, 4 * q + lg), xf[i][rt][q]); \
  }
    // next step's slice into the (now free) registers, then the entry after it
// which waves issue the next slice's loads right after the hand-off (the others issue
// them after the softmax, so one wave of each SIMD computes while its partner is held up
// issuing loads)
#ifndef SP_LOAD_EARLY
#define SP_LOAD_EARLY(w_) ((w_) < SP_WAVES / 2)
#endif
#ifdef FS_NOLOAD
#define SP_NEXT_COND false
#else
#define SP_NEXT_COND more
#endif
#define SP_NEXT()                                                                    \
  if (SP_NEXT_COND) {                                                                \
    SP_XLOAD();                                                                      \
    if (st + 2 < steps)                                                              \
      _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) pn[rt] = perm[pos_of(st + 2, rt * 16 + l16)]; \
  }

    {
      // ---- hand-off, spread over the waves: wave w owns the values 64 (w + NW m) + lane
      // (logits, then the two norms).  Guideline 16, R2 form: every value travels as one
      // 8-byte {tag, value} granule written by ONE relaxed agent-scope (sc1) store -- the
      // data is its own flag; the partner's granules are re-read with sc1 loads until every
      // tag equals this step's tag: one round trip once the data is there, no separate flag,
      // no fences.  Tag = launch generation (high half) | step + 1 (low half), so granules of
      // an earlier launch never match and the buffer needs no clearing between launches.
      // The polls are issued before the image write and the next slice's loads are issued
      // after the check, so the round trip neither queues behind nor waits for them.
      constexpr int M = (NZ + 2 + 64 * NW - 1) / (64 * NW);
      unsigned long long* slot = xb + ((int64_t)par * G) * X.SZ;
      const unsigned long long tag = (unsigned long long)tag32 << 32;
      float own[M];
      unsigned long long pl[M][G];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int idx = 64 * (w + NW * m) + lane;
        float v = 0.f;
        if (idx < NZ) {
          const int r = idx / NC, c = idx - r * NC;
#pragma unroll
          for (int i = 0; i < NW; ++i) v += zpart[i][r][c];
        } else if (idx < NZ + 2) {
#pragma unroll
          for (int i = 0; i < NW; ++i) v += wred[i][idx - NZ];
        }
        own[m] = v;
        if (idx < NZ + 2)
          __hip_atomic_store(slot + (int64_t)g * X.SZ + idx, tag | __float_as_uint(v), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      SP_STAMP(3)
      auto poll = [&]() {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const int idx = 64 * (w + NW * m) + lane;
#pragma unroll
          for (int h = 0; h < G; ++h)
            pl[m][h] = __hip_atomic_load(slot + (int64_t)h * X.SZ + (idx < NZ + 2 ? idx : 0), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        }
      };
      poll();
      SP_IMG_WRITE();
      unsigned spins = 0;
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
          for (int h = 0; h < G; ++h)
            ok &= (h == g) | (64 * (w + NW * m) + lane >= NZ + 2) | ((unsigned)(pl[m][h] >> 32) == tag32);
        if (__all(ok)) break;
        if (++spins > SP_SPIN_LIMIT) {
          if (lane == 0) __hip_atomic_store(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        poll();
      }
      // sum in slice order 0..G-1 (own partial at position g): identical bits in every partner
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int idx = 64 * (w + NW * m) + lane;
        if (idx < NZ + 2) {
          float v = 0.f;
#pragma unroll
          for (int h = 0; h < G; ++h) v += (h == g) ? own[m] : __uint_as_float((unsigned)pl[m][h]);
          if (idx < NZ) (&zsum[0][0])[idx] = v;
          else nrm[idx - NZ] = v;                // ||W - W_a||^2, ||W||^2 at the start of this step
        }
      }
      SP_STAMP(4)
      if (SP_LOAD_EARLY(w)) SP_NEXT();
    }
    SP_STAMP(5)
    lds_barrier();  // S2: summed logits and norms, the image
    SP_STAMP(6)
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
        const bool isy = c == lab[par][r];
        gv = (isy ? -invb : 0.f) + expf(lp) * invb;
        if (isy) cep -= lp;
      }
      gbuf[r][c] = gv;
    }
    cep = wave_sum(cep);
    if (lane == 0) wce[w] = cep;
    lds_barrier();  // S3: g, CE partials
    if (!SP_LOAD_EARLY(w)) SP_NEXT();
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
    float gB[4 * RT];
#pragma unroll
    for (int kk = 0; kk < 4 * RT; ++kk) gB[kk] = gbuf[4 * kk + lg][l16];
    const float sp = (P.prox && pn2 > 0.f) ? P.mu / sqrtf(pn2) : 0.f;
    const float sr = (P.reg && wn2 > 0.f) ? P.lam / sqrtf(wn2) : 0.f;
    const float lr = P.lr;
    const int rblk = 4 * (l16 & 3) + (l16 >> 2);
    float npn = 0.f, nwn = 0.f;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int Tl = w + NW * i;
      if (Tl < NTS) {
        floatx4 ga[4];
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) ga[e4] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 4 * RT; ++kk) {
          const float4 x = ld4(xs_lds + img_off(4 * kk + lg, RS, Tl, rblk));
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) ga[e4] = mfma4(comp(x, e4), gB[kk], ga[e4]);
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
    npn = wave_sum(npn);
    nwn = wave_sum(nwn);
    if (lane == 0) { wred[w][0] = npn; wred[w][1] = nwn; }
    SP_STAMP(8)
  }
#undef SP_XLOAD
#undef SP_IMG_WRITE
#undef SP_NEXT
#ifdef FS_STAMPS
  if (tid == 0 && X.stamps) {
    for (int k = 0; k < 8; ++k) X.stamps[blockIdx.x * 16 + k] = stamp_acc[k];
    X.stamps[blockIdx.x * 16 + 15] = (unsigned long long)steps;
  }
#endif

#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int Tl = w + NW * i;
    if (Tl < NTS && l16 < C)
#pragma unroll
      for (int q = 0; q < 4; ++q) st4(Wj + (int64_t)l16 * ld + 64 * (t0 + Tl) + 16 * q + 4 * lg, wr[i][q]);
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

static size_t split_dyn_lds(int RT, int NT, int G) {
  const int tiles = (NT + G - 1) / G;
  return sizeof(float) * (size_t)(RT * 16) * (size_t)(tiles * 64 + 8);
}

static size_t split_static_lds(int RT) {
  const int NR = RT * 16;
  return (size_t)SP_WAVES * NR * 16 * 4 + 2 * (size_t)NR * 16 * 4 + 2 * NR * 4 + SP_WAVES * 3 * 4 + 8 + 64;
}

// tiles per wave the register budget allows without spilling (slice + weights + anchor)
static int split_tpw_max(int RT, int G) { return (RT == 2 && G == 4) ? 1 : 2; }

static bool split_fits(int RT, int NT, int G) {
  const int tiles = (NT + G - 1) / G;
  return (tiles + SP_WAVES - 1) / SP_WAVES <= split_tpw_max(RT, G) &&
         split_dyn_lds(RT, NT, G) + split_static_lds(RT) <= 160 * 1024;
}

static int64_t split_ws_bytes(int N, int G, int RT) {
  const int SZ = RT * 16 * 16 + 4;
  return 256 + (int64_t)N * 2 * G * SZ * 8;
}

static unsigned next_generation() {
  static std::atomic<unsigned> counter{0};
  return 1u + counter.fetch_add(1u, std::memory_order_relaxed) % 65535u;
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
  if (NT < G) return fail(FS_EUNSUPPORTED, "fs_local_train: fewer feature tiles than workgroups per client");
  if (!ws || ws_bytes < split_ws_bytes(P.N, G, RT)) return fail(FS_EINVAL, "fs_local_train: workspace too small");
  const int cus = device_cus();
  if (cus <= 0) return fail(FS_EHIP, "fs_local_train: no device");
  if (!split_fits(RT, NT, G)) return fail(FS_EUNSUPPORTED, "fs_local_train: slice too wide for one workgroup");
  if (P.N * G > cus) return fail(FS_EUNSUPPORTED, "fs_local_train: N*G workgroups exceed the CU count");
  const size_t lds = split_dyn_lds(RT, NT, G);
  const int tiles = (NT + G - 1) / G;
  const int tpw = (tiles + SP_WAVES - 1) / SP_WAVES;
  char* base = reinterpret_cast<char*>(ws);
  SplitWS X;
  X.err = reinterpret_cast<unsigned*>(base);
  X.xbuf = reinterpret_cast<unsigned long long*>(base + 256);
  X.G = G;
  X.SZ = RT * 16 * 16 + 4;
  X.gen = next_generation();
  X.stamps = nullptr;
#ifdef FS_STAMPS
  X.stamps = reinterpret_cast<unsigned long long*>(base + ws_bytes - (int64_t)P.N * G * 16 * 8);
#endif
#define FS_SPLIT_CASE(rt, g, tp) \
  if (RT == rt && G == g && tpw <= tp) { launch_split_t<rt, g, tp>(P, X, lds, st); return FS_OK; }
  FS_SPLIT_CASE(2, 2, 1) FS_SPLIT_CASE(2, 2, 2) FS_SPLIT_CASE(2, 4, 1)
  FS_SPLIT_CASE(1, 2, 1) FS_SPLIT_CASE(1, 2, 2) FS_SPLIT_CASE(1, 4, 1) FS_SPLIT_CASE(1, 4, 2)
#undef FS_SPLIT_CASE
  return fail(FS_EUNSUPPORTED, "fs_local_train: no split kernel for this shape");
}

}  // namespace fs

using namespace fs;

// Plan the launch: G = workgroups per client (1 = one workgroup walks the client; 2 or 4 =
// split clients) and the workspace bytes it needs.  max_en = max_j E * n_j (unused since
// the shuffle indices are streamed; kept for the ABI).  The caller zeroes the workspace
// once at allocation; launches never clear it (hand-off tags carry a launch generation).
extern "C" int fs_local_train_plan(int N, int C, int B, int E, int64_t ld, int64_t max_en, int chained,
                                   int* G_out, int64_t* ws_bytes_out) {
  FS_REQUIRE(G_out && ws_bytes_out, "null pointer");
  FS_REQUIRE(N >= 1 && ld >= 64 && ld % 64 == 0, "bad sizes");
  (void)max_en;
  *G_out = 1;
  *ws_bytes_out = 0;
  const int cus = device_cus();
  if (chained || C > 16 || B > 32 || cus <= 0) return FS_OK;
  const int RT = B <= 16 ? 1 : 2;
  const int NT = (int)(ld >> 6);
  const int64_t max_steps = (int64_t)E * ((max_en / (E > 0 ? E : 1) + B - 1) / B);
  if (max_steps >= 65535) return FS_OK;          // hand-off tags hold the step in 16 bits
  for (int G : {4, 2}) {
    if (NT < G || N * G > cus || !split_fits(RT, NT, G)) continue;
    *G_out = G;
    *ws_bytes_out = split_ws_bytes(N, G, RT) + 4096;
    return FS_OK;
  }
  return FS_OK;
}
