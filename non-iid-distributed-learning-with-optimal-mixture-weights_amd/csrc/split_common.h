// Pieces shared by the split-client (local_train_split.hip) and pair-client
// (local_train_pair.hip) local-training kernels: the exchange workspace, the LDS image
// layout of one step's batch slice, and the walk of a group's client sequence.
#pragma once

#include "common.h"

namespace fs {

int device_cus();   // CUs of the current device (cached)

// Hand-off tags of an exchanging launch: (launch generation << 20) + step + 1, the generation
// counted per workspace on the host, so a granule left by an earlier launch never carries a
// tag this launch waits for and the exchange buffer needs no clearing per launch.  0 (the
// caller then clears the granules): a workspace's first use, every 4095 launches (the
// generation wraps), and a launch whose client sequences may run 2^20 - 1 steps or more.
unsigned exchange_generation(const void* ws, bool long_launch);

// the pair form (local_train_pair.hip)
bool pair_fits(int C, int B, int NT, int G);
// the pipe form (local_train_pipe.hip)
bool pipe_fits(int C, int B, int NT, int G, int prox);
int pipe_groups(int N, int G, int chained, int cus);
int64_t pipe_ws_bytes(int N, int G, int chained, int cus);
int pair_groups(int N, int G, int cus);
int64_t pair_ws_bytes(int N, int G, int B, int cus);

struct SplitWS {
  unsigned* err;                       // [1] sticky; nonzero: a partner never arrived (spin bound hit)
  unsigned long long* xbuf;            // [ngroups][2][G][SZ] published partials: {tag, value} granules
  unsigned long long* stamps;          // [grid][16] diagnostic build only
  int SZ;                              // granules per (group, parity, slice)
  unsigned tag_base;                   // launch generation << 20 (0: the buffer was zeroed for this launch)
  int ngroups;
  unsigned spin_limit;                 // 0: test knob -- report a timeout at the first hand-off
  int poll_delay;                      // s_sleep(1) units between a step's publish and first poll
};

__device__ __forceinline__ int tile_lo(int g, int G, int NT) { return (int)(((int64_t)NT * g) / G); }

// The weight update and the squared norms with every rounding spelled out (explicit fma, no
// contraction left to the compiler, which fused `a*a + b*b` as fma(b, b, a*a) in one kernel and
// fma(a, a, b*b) in another): the split, pair and pipe forms share these, so they agree
// bitwise by construction.  s + (x^2 + y^2 + z^2 + w^2), the four as one fma chain from x^2:
__device__ __forceinline__ float sq4_acc(float s, float x, float y, float z, float w) {
  float t = x * x;
  t = __builtin_fmaf(y, y, t);
  t = __builtin_fmaf(z, z, t);
  t = __builtin_fmaf(w, w, t);
  return s + t;
}
__device__ __forceinline__ float sq_acc(float s, float x) { return __builtin_fmaf(x, x, s); }
// w - lr * (g + [prox] (w - a) sp + [reg] w sr)
__device__ __forceinline__ float sgd_w(float wc, float g, float lr, bool prox, float ac, float sp, bool reg, float sr) {
  if (prox) g = __builtin_fmaf(wc - ac, sp, g);
  if (reg) g = __builtin_fmaf(wc, sr, g);
  return __builtin_fmaf(-lr, g, wc);
}

// LDS image of one step's batch slice: row-major, row stride RS = DS + 8 floats, and the
// sixteen float4 blocks of every 64-column tile permuted by block ^ (row & 7).  With this
// layout both the image write (lanes 0-7 = eight rows, same block) and the backward's read
// (lanes = 16 blocks of one row, 4 rows per instruction) are bank-conflict free.
__device__ __forceinline__ int img_off(int row, int RS, int tile, int blk) {
  return row * RS + 64 * tile + 4 * (blk ^ (row & 7));
}

// Reads of the read-only client tables (row_off, order).  SC = true: scalar loads
// (lgkmcnt), so that a client boundary never waits for the vector-memory queue -- where
// the pair kernel keeps a step's row stream in flight; false: ordinary loads.
__device__ __forceinline__ int tab_i32(const int32_t* base, int i) {
  const int32_t* p = base + __builtin_amdgcn_readfirstlane(i);
  int v;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
__device__ __forceinline__ int64_t tab_i64(const int64_t* base, int i) {
  const int64_t* p = base + __builtin_amdgcn_readfirstlane(i);
  int64_t v;
  asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}

// offset of (row, class) in a wave's partial-logit block [rt][lg][class][i] (row = 16 rt + 4 lg + i)
__device__ __forceinline__ int zp_off(int r, int c) { return (r >> 4) * 256 + ((r >> 2) & 3) * 64 + c * 4 + (r & 3); }

// Client k of a group's sequence (-1: none).  Parallel: tier k of the LPT-ordered clients,
// snake order (even tiers forward, odd tiers backward) so the groups' step totals balance.
template <bool SC = false>
__device__ __forceinline__ int sp_client(const LTParams& P, int grp, int ng, int k) {
  if (P.chained) return k < P.N ? k : -1;
  const int idx = k * ng + ((k & 1) ? ng - 1 - grp : grp);
  if (idx >= P.N) return -1;
  if (!P.order) return idx;
  return SC ? tab_i32(P.order, idx) : P.order[idx];
}

// A position in the group's step sequence: client (k, j), step st of its E * nbat steps.
struct SpCur {
  int k, j, n, nbat, steps, st;
  int64_t row0;
};

// first client with at least one step at sequence position >= k (false: sequence exhausted)
template <bool SC = false>
__device__ __forceinline__ bool sp_seek(SpCur& c, const LTParams& P, int grp, int ng, int T, int k) {
  for (; k < T; ++k) {
    const int j = sp_client<SC>(P, grp, ng, k);
    if (j < 0) continue;
    const int64_t r0 = SC ? tab_i64(P.row_off, j) : P.row_off[j];
    const int n = (int)((SC ? tab_i64(P.row_off, j + 1) : P.row_off[j + 1]) - r0);
    const int nbat = (n + P.B - 1) / P.B;
    if (nbat == 0 || P.E == 0) continue;
    c.k = k; c.j = j; c.n = n; c.nbat = nbat; c.steps = P.E * nbat; c.st = 0; c.row0 = r0;
    return true;
  }
  c.k = T;
  return false;
}

template <bool SC = false>
__device__ __forceinline__ bool sp_advance(SpCur& c, const LTParams& P, int grp, int ng, int T) {
  if (c.k >= T) return false;
  if (++c.st < c.steps) return true;
  return sp_seek<SC>(c, P, grp, ng, T, c.k + 1);
}

}  // namespace fs
