// fs_mix_z: the FedAMW validation-logit GEMM (/root/reference/functions/tools.py:448, with the
// stack of tools.py:435-440 fixed for the whole p-solve, so computed once per round):
//
//   Z[v][c*ldN + n] = X_val[v] . W_n[c]     (ldN = N rounded up to 4; padding columns = 0)
//
// M = n_val rows, N = C*ldN columns, K = ld (a multiple of 64).  Both operands are K-contiguous
// fp32 rows (X_val [n_val][ld], W_all [N][C][ld]), so the tile images are rows of 128 B per
// K-step.  MFMA-bound: 2*M*N*K flops at config 5 = 10.5 TFLOP on the 157 TFLOP/s fp32 matrix
// pipe (exact f32 v_mfma_f32_32x32x2_f32; no reduced-precision fp32 MFMA exists on gfx950).
//
// Design (round 4; replaces the 64x64 / BK 16 / two-barrier tile GEMM that ran 105 TFLOP/s
// with 50 % LDS bank-conflict cycles):
//  * 256-thread workgroup (one wave per SIMD), 256 x 128 output tile, each wave 128 x 64 =
//    4 x 2 blocks of 32 x 32 (128 accumulator registers); 128 x 128 tiles (wave 64 x 64) when
//    256-row tiles would not give every CU one;
//  * K-step 32 (one 128-B line per row): A image 256 rows x 128 B, B image 128 rows x 128 B,
//    filled by global_load_lds_dwordx4 (LDS-DMA, no VGPR staging) in pieces of 8 rows x
//    128 B -- 48 pieces per K-step, 12 per wave -- into two LDS buffers (2 x 48 KB): the next
//    K-step's pieces are in flight while the waves run this K-step's 128 MFMAs each; one
//    barrier per K-step;
//  * the 16-B slot of a row's K-chunk c is stored at c ^ ((row >> 1) & 7) (the swizzle is on
//    the per-lane global source address; the LDS image stays lane-linear): every
//    ds_read_b128 lane group of 16 (rows {0-3,12-15,20-27} / {4-11,16-19,28-31} of a 32-row
//    block) then covers the 64 banks exactly once -- conflict-free;
//  * K order: lane half h of MFMA (kq, j) takes k = 4 (2 kq + h) + j, so one ds_read_b128 per
//    32-row block feeds four MFMAs.  Z is a sum over k, fp32 with a different order than
//    torch's matmul either way (tolerance-checked against fp64, tests/test_gpu_parity.py);
//  * workgroup -> tile: blocks b and b + 8 share an XCD (round-robin dispatch, speed only), so
//    each XCD gets one contiguous run of tiles (a bijection for any tile count), ordered in
//    groups of 8 row tiles: the 32 workgroups an XCD runs at once share 8 A and 4 B tiles.
#include "common.h"

namespace fs {

typedef float floatx16 __attribute__((ext_vector_type(16)));

__host__ __device__ __forceinline__ int mixz_ldn(int N) { return (N + 3) & ~3; }

// BM = 256 (each wave 128 x 64: MB = 4 row blocks of 32) where the grid gives every CU a tile
// (config 2: 400 tiles on 256 CUs); BM = 128 (MB = 2) for smaller grids
constexpr int ZG_BN = 128, ZG_BK = 32;
constexpr int ZG_ROWB = ZG_BK * 4;                       // 128 B per row per K-step
constexpr int ZG_GROUP_M = 8;                            // row tiles per tile-order group
template <int BM> struct ZgShape {
  static constexpr int MB = BM / 64;                     // 32-row blocks per wave
  static constexpr int ABYTES = BM * ZG_ROWB;            // 32 / 16 KB
  static constexpr int BUFB = (BM + ZG_BN) * ZG_ROWB;    // 48 / 32 KB per buffer
  static constexpr int PPW = (BM + ZG_BN) / 8 / 4;       // pieces of 8 rows x 128 B per wave: 12 / 8
};

__device__ __forceinline__ void zg_glds(const float* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__device__ __forceinline__ floatx16 mfma32(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// one K-step from one buffer: per kq, 4 + 2 ds_read_b128 feed 4 x 8 MFMAs; the fragments of
// kq + 1 are read while the MFMAs of kq run (two register sets)
template <int MB>
__device__ __forceinline__ void zg_frags(const char* cur, int a_off, int b_off, int frag, float4 (&a)[MB],
                                         float4 (&bb)[2]) {
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) a[mb] = *reinterpret_cast<const float4*>(cur + a_off + mb * 32 * ZG_ROWB + frag);
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) bb[nb] = *reinterpret_cast<const float4*>(cur + b_off + nb * 32 * ZG_ROWB + frag);
}

template <int MB>
__device__ __forceinline__ void zg_mfmas(const float4 (&a)[MB], const float4 (&bb)[2], floatx16 (&acc)[MB][2]) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = mfma32(comp(a[mb], j), comp(bb[nb], j), acc[mb][nb]);
}

// the fragment reads of kq + 1 go out after the first 4 of kq's 32 MFMAs (pinned with
// sched_group_barrier: left alone, hipcc put the reads after the MFMAs and waited for them);
// by the next group's first MFMA they have long returned
#define ZG_PIN_READS_THEN_MFMAS()                                 \
  __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);            \
  __builtin_amdgcn_sched_group_barrier(0x100, MB + 2, 0);       \
  __builtin_amdgcn_sched_group_barrier(0x008, 8 * MB - 4, 0);   \
  __builtin_amdgcn_sched_barrier(0)

template <int MB>
__device__ __forceinline__ void zg_kstep(const char* cur, int a_off, int b_off, const int (&frag)[4],
                                         floatx16 (&acc)[MB][2]) {
  float4 a0[MB], b0[2], a1[MB], b1[2];
  zg_frags(cur, a_off, b_off, frag[0], a0, b0);
  __builtin_amdgcn_sched_barrier(0);
  zg_frags(cur, a_off, b_off, frag[1], a1, b1);
  zg_mfmas(a0, b0, acc);
  ZG_PIN_READS_THEN_MFMAS();
  zg_frags(cur, a_off, b_off, frag[2], a0, b0);
  zg_mfmas(a1, b1, acc);
  ZG_PIN_READS_THEN_MFMAS();
  zg_frags(cur, a_off, b_off, frag[3], a1, b1);
  zg_mfmas(a0, b0, acc);
  ZG_PIN_READS_THEN_MFMAS();
  zg_mfmas(a1, b1, acc);
}

template <int BM>
__global__ __launch_bounds__(256, 1) void mix_z_gemm_kernel(const float* __restrict__ W,
                                                            const float* __restrict__ X, int64_t ld, int N,
                                                            int C, int nv, float* __restrict__ Z, int tiles_m,
                                                            int tiles_n) {
  using S = ZgShape<BM>;
  constexpr int MB = S::MB, PPW = S::PPW;
  __shared__ __attribute__((aligned(1024))) char lds0[S::BUFB];
  __shared__ __attribute__((aligned(1024))) char lds1[S::BUFB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ldN = mixz_ldn(N);
  const int CN = C * ldN;

  // ---- tile of this workgroup: a contiguous run of tiles per XCD, grouped by 8 row tiles ----
  const int T = tiles_m * tiles_n;
  const int b = blockIdx.x, x = b & 7, idx = b >> 3;
  const int base = T >> 3, rem = T & 7;
  const int t = x * base + min(x, rem) + idx;
  const int gsz = ZG_GROUP_M * tiles_n;
  const int g = t / gsz, tin = t - g * gsz;
  const int gm = min(ZG_GROUP_M, tiles_m - g * ZG_GROUP_M);
  const int tm = g * ZG_GROUP_M + tin % gm, tn = tin / gm;
  const int v0 = tm * BM, c0 = tn * ZG_BN;

  // ---- this lane's source rows for the wave's PPW pieces (clamped: rows past n_val and
  //      columns past C*ldN / of padding clients load a valid row; the epilogue masks them) ----
  const float* src[PPW];
  {
    const int rin = lane >> 3, slot = lane & 7;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int P = w * PPW + i;
      if (P < BM / 8) {
        const int r = 8 * P + rin;
        const int chunk = slot ^ ((r >> 1) & 7);
        const int v = min(v0 + r, nv - 1);
        src[i] = X + (int64_t)v * ld + chunk * 4;
      } else {
        const int r = 8 * (P - BM / 8) + rin;
        const int chunk = slot ^ ((r >> 1) & 7);
        const int col = min(c0 + r, CN - 1);
        const int c = col / ldN;
        const int n = min(col - c * ldN, N - 1);
        src[i] = W + ((int64_t)n * C + c) * ld + chunk * 4;
      }
    }
  }
  // ---- fragment offsets: lane (row l&31 of a 32-row block, half h) reads chunk 2 kq + h ----
  const int wm = w >> 1, wn = w & 1;
  const int lr = lane & 31, h = lane >> 5;
  int frag[4];
#pragma unroll
  for (int kq = 0; kq < 4; ++kq) frag[kq] = lr * ZG_ROWB + (((2 * kq + h) ^ ((lr >> 1) & 7)) << 4);
  const int a_off = (wm * (BM / 2)) * ZG_ROWB;
  const int b_off = S::ABYTES + (wn * 64) * ZG_ROWB;

  floatx16 acc[MB][2];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mb][nb][r] = 0.f;

  const int nk = (int)(ld / ZG_BK);     // even: ld is a multiple of 64
  // prologue: K-step 0 into buffer 0
#pragma unroll
  for (int i = 0; i < PPW; ++i) zg_glds(src[i], lds0 + w * PPW * 1024 + i * 1024);

  // Two K-steps per iteration, one per buffer: each half reads one __shared__ array while the
  // other's pieces are in flight.  With both halves naming their arrays statically the
  // compiler can see that the fragment reads do not alias the LDS-DMA in flight and emits no
  // vmcnt wait before them (with one array and a runtime buffer index it waited vmcnt(0)
  // before the first ds_read of every K-step, serialising the prefetch).
  for (int kt = 0; kt < nk; kt += 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    {
      const int64_t koff = (int64_t)(kt + 1) * ZG_BK;
#pragma unroll
      for (int i = 0; i < PPW; ++i) zg_glds(src[i] + koff, lds1 + w * PPW * 1024 + i * 1024);
    }
    __builtin_amdgcn_sched_barrier(0);
    zg_kstep<MB>(lds0, a_off, b_off, frag, acc);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 2 < nk) {
      const int64_t koff = (int64_t)(kt + 2) * ZG_BK;
#pragma unroll
      for (int i = 0; i < PPW; ++i) zg_glds(src[i] + koff, lds0 + w * PPW * 1024 + i * 1024);
    }
    __builtin_amdgcn_sched_barrier(0);
    zg_kstep<MB>(lds1, a_off, b_off, frag, acc);
  }

  // ---- epilogue: D[i][j] of a 32x32 block, reg r: i = (r&3) + 8 (r>>2) + 4 h, j = lane&31 ----
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int col = c0 + wn * 64 + nb * 32 + lr;
    if (col >= CN) continue;
    const bool pad = (col % ldN) >= N;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int v = v0 + wm * (BM / 2) + mb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (v < nv) Z[(int64_t)v * CN + col] = pad ? 0.f : acc[mb][nb][r];
      }
  }
}

}  // namespace fs

using namespace fs;

extern "C" int fs_mix_z(const float* d_W_all, const float* d_X_val, int64_t ld, int N, int C, int n_val, float* d_Z,
                        void* stream) {
  FS_REQUIRE(N >= 1 && C >= 1 && n_val >= 1, "bad sizes");
  FS_REQUIRE(ld >= 64 && ld % 64 == 0, "ld must be a positive multiple of 64");
  FS_REQUIRE(d_W_all && d_X_val && d_Z, "null pointer");
  const int64_t CN = (int64_t)C * mixz_ldn(N);       // padded columns (zeros for n >= N)
  FS_REQUIRE(CN < (int64_t)1 << 30, "C * N too large");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int tiles_n = (int)((CN + ZG_BN - 1) / ZG_BN);
  const int64_t t256 = (int64_t)((n_val + 255) / 256) * tiles_n;
  FS_REQUIRE(t256 < ((int64_t)1 << 29), "Z too large");
  int cus = 0, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  if (t256 >= (int64_t)cus) {          // 256-row tiles fill the chip (config 2: 400 tiles; as 800
                                       // 128-row tiles 0.595 vs 0.55 ms, profiles/r04/z_gemm_time.txt)
    const int tiles_m = (n_val + 255) / 256;
    hipLaunchKernelGGL(mix_z_gemm_kernel<256>, dim3(tiles_m * tiles_n), dim3(256), 0, st, d_W_all, d_X_val, ld, N, C,
                       n_val, d_Z, tiles_m, tiles_n);
  } else {
    const int tiles_m = (n_val + 127) / 128;
    hipLaunchKernelGGL(mix_z_gemm_kernel<128>, dim3(tiles_m * tiles_n), dim3(256), 0, st, d_W_all, d_X_val, ld, N, C,
                       n_val, d_Z, tiles_m, tiles_n);
  }
  FS_LAUNCH_CHECK();
  return FS_OK;
}
