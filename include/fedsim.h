/*
 * fedsim.h -- C-ABI of the MI355X (gfx950) federated-round engine.
 *
 * The reference (Bojian-Wei/Non-IID-Distributed-Learning-with-Optimal-Mixture-Weights)
 * is pure Python/PyTorch and has no native interface; every entry point below
 * replaces one Python-level piece of its hot path, cited as
 * /root/reference/<file>:<line>.  The Python drop-ins in
 * non-iid-distributed-learning-with-optimal-mixture-weights_amd/functions/tools.py
 * (FedAvg / FedProx / FedAMW) are the callers; INTEGRATION.md shows the ctypes
 * binding a maintainer of the reference would add.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Pointers named d_* are DEVICE pointers
 *     (hipMalloc / torch caching allocator); h_* are host pointers.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  All
 *     device entry points are asynchronous on that stream, allocate nothing and
 *     never synchronise (safe under hipGraph capture).  Kernels that exchange data
 *     between workgroups take a caller-owned workspace: the launch zeroes its
 *     exchange part itself; its LAST 256 bytes are an error block whose first
 *     uint32 is set (sticky) when a bounded cross-workgroup wait timed out -- the
 *     caller zeroes the workspace once at allocation, reads that word after the
 *     work and clears it.  Test knob: fs_tuning.inject_timeout = 1 makes every
 *     such launch report a timeout (the error path without a real hang).
 *   - Feature rows are fp32, row-major, with a leading dimension `ld` that is a
 *     multiple of 64 floats (D is zero-padded to ld; padded columns stay exactly 0).
 *   - Return value: 0 on success, negative on error; fs_last_error() returns a
 *     thread-local message.  No C++ exception crosses the ABI.
 */
#ifndef FEDSIM_H
#define FEDSIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FS_OK 0
#define FS_EINVAL (-1)
#define FS_EHIP (-2)
#define FS_EUNSUPPORTED (-3)

#define FS_ABI_VERSION 16

/* ABI version and the last error message of the calling thread. */
int fs_abi_version(void);
const char* fs_last_error(void);

/* ------------------------------------------------------------------------- *
 * Tuning (ABI 9).  Every knob that changes HOW (never what) the kernels compute, as
 * explicit fields -- the library reads no environment variable.  All-zero = the defaults
 * (what the planners pick by shape); fs_tuning_size() is for binding-layout checks.
 * Threading contract (ABI 12): a launch reads the tuning in effect for the HOST THREAD
 * that enqueues it, at the moment it is enqueued (fs_local_train*, fs_plan_*, fs_mix_solve,
 * fs_randperm_device ...; a launch already enqueued is never affected).  That is the
 * thread's own override if fs_set_thread_tuning(t) set one, else the process-wide value of
 * fs_set_tuning (mutex-protected; visible to every thread without an override).
 * fs_set_tuning(NULL) restores the process-wide defaults; fs_set_thread_tuning(NULL)
 * drops the calling thread's override; fs_get_tuning reports what the calling thread's
 * next launch would use.  Two host threads that drive two plans with different solver or
 * form choices therefore each set a thread override.
 *   mix_solver         0 = by shape, else force one p-solver (FS_SOLVER_*; a forced solver
 *                      that does not cover the shape falls through to the shape's choice)
 *   mix_prefetch       L2 prefetch helper workgroups beside the p-solve: 0 = by solver
 *                      (4 for the quarter-wave solver when Z outgrows the L2s, 24 for qmc),
 *                      -1 = none, n > 0 = n
 *   mix_prefetch_lead  steps the helpers run ahead (0 = by solver: 16 quad; qmc 8 at K >= 12
 *                      workgroups, else 6)
 *   mix_exact_softmax  quarter-wave solvers: 1 = torch's exp(o - m - log sum) form with libm
 *                      expf / logf (default: e * rcp(sum e) on v_exp_f32 / v_rcp_f32; both
 *                      within the fp32 tolerance of the reference)
 *   no_eval_fuse       fs_plan_create: 1 = never carry a deferred evaluation inside a
 *                      training launch (fs_plan_eval_blocks() is then 0)
 *   spin_limit         bound of every cross-workgroup spin, in polls (0 = the default)
 *   inject_timeout     test knob: 1 = every exchanging launch reports a timeout at its first
 *                      hand-off (the error path without a real hang)
 *   train_form         (ABI 10) fs_local_train_plan's choice for parallel clients: 0 = by shape
 *                      (the pair form where it fits, else the split form), 1 = never the pair
 *                      form, 2 = the pair form wherever it fits (else as 0)
 *   split_early        (ABI 11) split form without a prox anchor on full slices: 0 = issue the
 *                      first SP_E1 (local_train_split.hip: 4 at G = 2, 6 at G >= 4) of each
 *                      wave's 16 next-step row loads right after the hand-off (they stream
 *                      through the softmax), -1 = all of them inside the backward; since
 *                      round 5 it covers the prox term (anchor slice first, 2 early rows) and
 *                      the narrow chained instances (one tile per wave at 4 or 8 tiles per
 *                      slice: every row load early); -1 turns both off (bitwise the same W)
 *   mix_qmc_lane_clients (ABI 13) qmc p-solver: clients per lane, 0 = by shape (4 where
 *                      K = ceil(N / 64) <= 16 workgroups, else 8 for C <= 10), 4 = force 4,
 *                      8 = force 8 where C <= 10 (K = ceil(N / 128)); same p to fp32 rounding
 *                      of the K-partial sums (a different client-to-workgroup split)
 *   mix_quad_loaders   (ABI 13) quad p-solver at 64 < N <= 128, C <= 10 (config 2): 0 = with
 *                      4 loader waves that stream the late classes' Z rows into LDS (default),
 *                      -1 = without (each compute wave issues all of its loads); bitwise the
 *                      same p
 *   split_teams        (ABI 13) fs_local_train_plan's choice of the team form for parallel
 *                      clients: 0 = by shape (not chosen: measured slower), 1 = wherever it
 *                      fits, -1 = never
 *   mix_poll_delay     (ABI 13) qmc p-solver: s_sleep(1) units (~64 cycles each) between a
 *                      step's publish and its first poll: 0 = by shape (10 at K >= 12 with
 *                      C >= 8, else 8), -1 = none, n > 0 = n; bitwise the same p
 *   split_poll_delay   (ABI 13) split form: s_sleep(1) units between a step's publish and its
 *                      first poll: 0 = by width (16 at G >= 8 with parallel clients, else
 *                      none), -1 = none, n > 0 = n; bitwise the same results
 *   split_pipe         (ABI 14) fs_local_train_plan's choice of the pipe form (FS_G_PIPE):
 *                      0 = by shape, 1 = wherever it fits (G = ld / 1024), -1 = never
 *   split_dbuf         (ABI 15) split form on full slices (8 waves x 2 tiles, or the narrow
 *                      chained 4 x 1) with 16 < B <= 32: the double-buffered instance
 *                      (local_train_dbuf.hip: the rows streamed ahead of the hand-off);
 *                      1 = wherever it covers; 0 = by shape (not chosen: measured a tie at
 *                      configs 2 and 5, slower at config 1); -1 = never; bitwise the same results
 *   split_mb           (ABI 16) split form with 16 < B <= 32: the classes on the 16-block
 *                      v_mfma_f32_4x4x1_16b_f32 in ceil(C / 4) blocks of 4 (the "mb" instances,
 *                      local_train_split.hip) instead of v_mfma_f32_16x16x4_f32 padded to 16;
 *                      0 = by shape, 1 = wherever it fits, -1 = never.  Same steps and hand-off,
 *                      the products summed in another order (within the oracle's fp32 tolerance)
 * ------------------------------------------------------------------------- */
#define FS_SOLVER_AUTO 0
#define FS_SOLVER_REG 1
#define FS_SOLVER_MC 2
#define FS_SOLVER_STAGED 3
#define FS_SOLVER_GLOBAL 4
#define FS_SOLVER_REG2 5
#define FS_SOLVER_WAVE 6
#define FS_SOLVER_QUAD 8
#define FS_SOLVER_QMC 9
#define FS_SOLVER_BIN 10

typedef struct fs_tuning {
  int mix_solver;
  int mix_prefetch;
  int mix_prefetch_lead;
  int mix_exact_softmax;
  int no_eval_fuse;
  unsigned spin_limit;
  int inject_timeout;
  int train_form;
  int split_early;
  int mix_qmc_lane_clients;
  int mix_quad_loaders;
  int split_teams;
  int mix_poll_delay;
  int split_poll_delay;
  int split_pipe;
  int split_dbuf;
  int split_mb;
} fs_tuning;

int64_t fs_tuning_size(void);
int fs_set_tuning(const fs_tuning* t);
int fs_set_thread_tuning(const fs_tuning* t);
int fs_get_tuning(fs_tuning* t);
/* (ABI 14) the process-wide value alone (what fs_set_tuning last set), whatever the calling
 * thread's override; and the calling thread's override: returns 1 and fills *t if one is
 * set, 0 (and *t = all-zero) if not.  A binding that changes one field for a block of code
 * reads the value it will restore from the layer it writes (the ADVICE round-4 fix: a
 * process-wide set from a thread with an override neither copies that override into the
 * process value nor is shadowed silently). */
int fs_get_process_tuning(fs_tuning* t);
int fs_get_thread_tuning(fs_tuning* t);

/* ------------------------------------------------------------------------- *
 * Host: DataLoader shuffle replay.
 * Replaces the RandomSampler permutation of every shuffled pass
 * (torch.utils.data.DataLoader(shuffle=True) at tools.py:179, 220; exp.py:99):
 * for pass i, out[off[i] .. off[i]+n[i]) = torch.randperm(n[i], generator=g)
 * with g.manual_seed(seed[i]) -- MT19937 seeded with (uint32)seed, forward
 * Fisher-Yates with z = mt() % (n-k).  Bit-exact with torch 2.10 CPU.
 * nthreads <= 0 picks the hardware concurrency.
 * ------------------------------------------------------------------------- */
int fs_randperm_batch(const int64_t* h_seeds, const int64_t* h_n, const int64_t* h_off,
                      int64_t npasses, int32_t* h_out, int nthreads);

/* ------------------------------------------------------------------------- *
 * Host: LIBSVM / svmlight reader.  Replaces the parse of svmlight_data
 * (utils.py:36-38, sklearn load_svmlight_file) for the dense float32 rows
 * load_full_data feeds the feature map (utils.py:56): `label [qid:q] idx:val ...`
 * per line, `#` comments, blank lines skipped; values parsed as doubles and rounded
 * once to float32 (= csr.toarray().astype(float32)).  fs_libsvm_scan reports the
 * sample count and the smallest / largest feature index (-1: no features).
 * fs_libsvm_read fills X [n_rows][n_features] (zeroed first) and y [n_rows];
 * zero_based: 1 indices start at 0, 0 at 1, -1 auto (zero-based iff the smallest
 * index is 0, as sklearn's 'auto'); an index outside n_features is an error.
 * Parallel over line-aligned chunks (nthreads <= 0: min(16, hardware)).
 * ------------------------------------------------------------------------- */
int fs_libsvm_scan(const char* path, int64_t* n_rows, int64_t* min_index, int64_t* max_index);
int fs_libsvm_read(const char* path, int64_t n_rows, int64_t n_features, int zero_based, float* X, double* y,
                   int nthreads);

/* ------------------------------------------------------------------------- *
 * Device: the same shuffle replay as fs_randperm_batch, on the GPU; d_seeds/d_n/d_off
 * are device arrays of npasses int64.  max_n MUST bound every n[i] (the host chooses the
 * form from it before the device sees n): max_n <= 64 runs one pass per LANE (64 passes per
 * wave, the MT state and the shuffle in registers / the lane's LDS row); larger max_n runs
 * one wave per pass with an LDS-resident (max_n <= ~38K) or in-place global-memory
 * permutation.  Bit-identical to fs_randperm_batch.  Asynchronous on `stream`.
 * (ABI 14) d_err (device, may be NULL): a pass with n[i] > max_n -- a caller breaking the
 * contract -- is written as the identity permutation (memory-safe: no LDS row or buffer is
 * overrun) and sets *d_err to 1 (sticky; the caller zeroes it once, reads it after the work
 * and raises -- Shuffler.check_errors in engine.py).
 * ------------------------------------------------------------------------- */
int fs_randperm_device(const int64_t* d_seeds, const int64_t* d_n, const int64_t* d_off, int64_t npasses,
                       int64_t max_n, int32_t* d_out, uint32_t* d_err, void* stream);

/* ------------------------------------------------------------------------- *
 * Local training of N clients.  Replaces train_loop (tools.py:177-215) called
 * once per client by FedAvg/FedProx/FedAMW (tools.py:340-343, 367-370, 430-433).
 *
 *   d_phi      [rows][ld]      client features, client j = rows d_row_off[j] .. d_row_off[j+1]-1
 *   d_row_off  [N+1]  int64    CSR row offsets
 *   d_labels   [rows] int32    class index per row
 *   d_perms    [E*rows] int32  client j, epoch e: local indices at E*row_off[j] + e*n_j
 *   d_order    [N] int32       block -> client schedule (parallel mode; NULL = identity)
 *   d_W_start  [C][ld]         round-start weights (client 0's start when chained)
 *   d_W_out    [N][C][ld]      each client's trained weights (the clients x params buffer)
 *   d_loss     [N] double      last-epoch |b|-weighted mean loss (incl. prox/ridge terms)
 *   B, E       batch size (<= 64), local epochs
 *   lr, mu, lam, prox, reg     SGD lr; prox weight (used iff prox); ridge weight (iff reg)
 *   chained    1: client j starts from client j-1's result and its prox anchor is
 *              that start (reference semantics);  0: every client starts
 *              from d_W_start (parallel clients).
 *   G, d_ws    workgroups per client and their workspace, from fs_local_train_plan:
 *              G = 1: one workgroup walks each client (any shape, chained or not);
 *              G = 2/4/8/16: "split clients" -- a group of G co-resident workgroups
 *              shares one client's feature tiles and exchanges partial logits every
 *              step (C <= 16, B <= 32).  Parallel clients: min(N, CUs/G) groups walk
 *              the clients (LPT order, snake over the groups); chained clients: one
 *              group walks the chain with the weights kept in registers.  The error
 *              word (last 256 bytes of d_ws) is nonzero after the kernel if a partner
 *              never arrived (results invalid).
 *              G | FS_G_PAIR (ABI 10, parallel clients, ld == 512 G): the "pair" form --
 *              min(ceil(N/2), CUs/G) groups of G workgroups, each training TWO clients at a
 *              time interleaved, so one client's hand-off overlaps the other's compute and
 *              the feature rows stream through every phase; the same arithmetic as the split
 *              form at width G (bitwise the same results).
 *              G | FS_G_TEAMS (ABI 13, parallel clients, G = 4 or 8): the "team" form --
 *              min(ceil(N/2), CUs/G) groups of G workgroups, each workgroup's 8 waves two
 *              teams of 4 that train two clients at once with team-local barriers, so one
 *              team's hand-off and softmax run beside the other team's MFMAs (the split
 *              arithmetic with 4 waves per slice: within the fp32 tolerance of the split form).
 *              G | FS_G_PIPE (ABI 14, ld == 1024 G with G = 2, 4, 8 or 16, 16 < B <= 32, C <= 16;
 *              parallel or chained clients, ridge and prox terms): the "pipe" form -- the split form with
 *              each step's hand-off pipelined by 16-row tile (one tile's partner round trip under
 *              the other tile's forward or backward MFMAs, the softmax per wave in registers, two
 *              barriers per step); the same arithmetic in the same order as the split form at
 *              width G (bitwise the same results).
 *              fs_local_train_plan: *G_out on entry is a request (0 = planner's choice, 1 =
 *              one workgroup per client, 2..16 = that split width if the shape allows it,
 *              G | FS_G_PAIR = the pair form, G | FS_G_TEAMS = the team form at that width
 *              if the shape allows it); prox says whether the FedProx term is on.
 * Requires 1 <= C <= 32, B <= 64, ld % 64 == 0, D <= ld.
 * ------------------------------------------------------------------------- */
#define FS_G_PAIR 256
#define FS_G_TEAMS 512
#define FS_G_PIPE 1024
int fs_local_train_plan(int N, int C, int B, int E, int64_t ld, int64_t max_en, int chained, int prox,
                        int* G_out, int64_t* ws_bytes_out);
int fs_local_train(const float* d_phi, int64_t ld, const int64_t* d_row_off, const int32_t* d_labels,
                   const int32_t* d_perms, const int32_t* d_order, int N, int C, int B, int E,
                   float lr, float mu, int prox, float lam, int reg, int chained,
                   const float* d_W_start, float* d_W_out, double* d_loss, int G, void* d_ws,
                   int64_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------- *
 * Weighted aggregation: d_W_bar = p0*W0 + p1*W1 + ... + p_{N-1}*W_{N-1}, every
 * product and sum rounded separately in that left-to-right order
 * (tools.py:345-350, 372-377, 455-460).  W_j = d_W_all + j*stride, len floats.
 * chunks == 1 gives the reference's exact fold; chunks > 1 folds `chunks`
 * consecutive client ranges in parallel and then folds the partials in order
 * (needs d_ws of chunks*len floats).  chunks <= 0 picks a value from the shape.
 * ------------------------------------------------------------------------- */
int fs_aggregate(const float* d_W_all, int64_t stride, const float* d_p, int N, int64_t len,
                 float* d_W_bar, float* d_ws, int64_t ws_floats, int chunks, void* stream);

/* ------------------------------------------------------------------------- *
 * Test evaluation.  Replaces test_loop + comp_accuracy + Meter (tools.py:218-237,
 * 82-96, 99-148): d_out[0] = mean cross-entropy over n rows, d_out[1] = top-1
 * accuracy in percent.  Ties in the arg-max go to the lowest class index.
 * d_ws needs fs_eval_ws_doubles(n) doubles.
 * ------------------------------------------------------------------------- */
int64_t fs_eval_ws_doubles(int n);
int fs_eval(const float* d_phi, int64_t ld, const int32_t* d_labels, int n, const float* d_W, int C,
            double* d_out, double* d_ws, void* stream);

/* ------------------------------------------------------------------------- *
 * FedAMW mixture step 1: Z[v][c*ldN + n] = sum_d X_val[v][d] * W_n[c][d], where
 * ldN = (N + 3) & ~3 (d_Z holds n_val * C * ldN floats; padding columns are 0)
 * (the inner matmul of tools.py:448, hoisted out of the p-SGD loop because the
 * stacked W of tools.py:435-440 is fixed during it).  fp32 MFMA GEMM.
 * ------------------------------------------------------------------------- */
int fs_mix_z(const float* d_W_all, const float* d_X_val, int64_t ld, int N, int C, int n_val,
             float* d_Z, void* stream);

/* ------------------------------------------------------------------------- *
 * FedAMW mixture step 2: `epochs` passes of SGD(momentum) on p over the pooled
 * validation set (tools.py:441-453): per batch of <= Bv rows (order from d_perms,
 * [epochs][n_val]): out[b,c] = sum_n p_n Z[v_b][c*ldN+n]; CE mean; grad_p;
 * buf = first ? grad : momentum*buf + grad; p -= lr_p*buf.  d_p, d_buf [N] are
 * updated in place; *d_first (int) is read and cleared (the momentum buffer of
 * torch.optim.SGD starts empty, tools.py:423).  A single persistent workgroup
 * where a register-resident instance covers (N, C, Bv) -- for N <= 16 with C <= 2 one wave
 * ("bin", no LDS, no barrier); for N <= 128 the quarter-wave
 * solver (4 batch rows per wave), with 4 L2 prefetch helper workgroups on its XCD that
 * only load (fs_tuning.mix_prefetch sets their number, -1 = none; their progress word is
 * byte 128 of the error block); for N > 256 the multi-CU quarter-wave solver "qmc"
 * (K <= 16 workgroups of 128 clients on one XCD, one exchange hop per step, 16 helper
 * workgroups); otherwise (Bv <= 16, C <= 16, N <= 2048) K <= 32 workgroups that split the
 * clients and exchange partial logits every step (slices of S >= 16 clients: reduce-scatter
 * to owner workgroups, then an all-gather of the totals); otherwise one LDS-staged /
 * global workgroup.
 * d_ws: fs_mix_solve_ws_bytes(N, C, Bv) bytes, zeroed once at allocation (the multi-CU
 * exchange granules + the error block; a timed-out exchange also writes NaN into d_p).
 * Concurrent solves need separate workspaces.  fs_tuning.mix_solver (FS_SOLVER_*) forces a
 * solver (tests, diagnostics; one that does not cover the shape falls through).
 * ------------------------------------------------------------------------- */
int64_t fs_mix_solve_ws_bytes(int N, int C, int Bv);
int fs_mix_solve(const float* d_Z, const int32_t* d_labels, const int32_t* d_perms, int N, int C,
                 int n_val, int epochs, int Bv, float lr_p, float momentum, float* d_p, float* d_buf,
                 int* d_first, void* d_ws, int64_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------- *
 * (ABI 12) fs_mix_solve on the rank-blocked Z that one all-gather of the per-rank
 * Z blocks produces (the sharded FedAMW round, dist.py): d_Z is
 * [blocks][n_val][C][L], L = N / blocks (a multiple of 4), client n = block n / L,
 * column n % L -- no layout copy into [n_val][C][N] first.  Read by the qmc solver
 * only (N > 256, C <= 16, Bv <= 16; fs_tuning.mix_solver AUTO or QMC); any other
 * shape or forced solver returns FS_EUNSUPPORTED (use fs_mix_solve on the standard
 * layout).  Same arithmetic in the same order as fs_mix_solve on the standard layout:
 * bitwise the same p and momentum buffer.  Arguments otherwise as fs_mix_solve.
 * fs_mix_solve_blocked_covers tells, before the all-gather, which layout to assemble.
 * ------------------------------------------------------------------------- */
int fs_mix_solve_blocked(const float* d_Z, int blocks, const int32_t* d_labels, const int32_t* d_perms, int N,
                         int C, int n_val, int epochs, int Bv, float lr_p, float momentum, float* d_p, float* d_buf,
                         int* d_first, void* d_ws, int64_t ws_bytes, void* stream);
/* host-only: 1 if fs_mix_solve_blocked covers this shape under the calling thread's tuning */
int fs_mix_solve_blocked_covers(int N, int C, int n_val, int epochs, int Bv);

/* Diagnostic (host state only): the solver the calling thread's last fs_mix_solve
 * launched -- FS_SOLVER_REG (1, register-resident, one row per wave), _MC (2, multi-CU),
 * _STAGED (3), _GLOBAL (4), _REG2 (5, two rows per wave, Bv <= 16, C <= 10), _WAVE (6, one
 * wave: N <= 16, C <= 4, Bv <= 16), _QUAD (8, quarter-wave: N <= 64 with C <= 16, or N <= 128
 * with C <= 10; Bv <= 16), _QMC (9, multi-CU quarter-wave), _BIN (10, one wave, two classes:
 * N <= 16, C <= 2, Bv <= 16); 0 = none yet. */
int fs_mix_solve_last_mode(void);
/* (ABI 14) Diagnostic: the layout of the calling thread's last fs_mix_solve /
 * fs_mix_solve_blocked launch when it ran the qmc solver -- its workgroups K and clients per
 * lane (4 or 8; K = ceil(ldN / (16 * lane_clients))) -- else 0 and 0. */
int fs_mix_solve_last_layout(int* workgroups, int* lane_clients);
/* (ABI 15) Diagnostic (host state only): the kernel the calling thread's last fs_local_train
 * launched -- FS_LT_SINGLE (1, one workgroup per client), FS_LT_SPLIT (2), FS_LT_DBUF (3, the
 * split form's double-buffered instance: the rows streamed ahead of the hand-off),
 * FS_LT_PAIR (4), FS_LT_PIPE (5), FS_LT_TEAMS (6), FS_LT_MB (7, ABI 16: the split form's
 * 4x4x1 multi-block instances, fs_tuning.split_mb); 0 = none yet. */
#define FS_LT_SINGLE 1
#define FS_LT_SPLIT 2
#define FS_LT_DBUF 3
#define FS_LT_PAIR 4
#define FS_LT_PIPE 5
#define FS_LT_TEAMS 6
#define FS_LT_MB 7
int fs_local_train_last_kernel(void);

/* ------------------------------------------------------------------------- *
 * Random Fourier feature map.  Replaces RFF's use in feature_mapping
 * (tools.py:22-31: `1 / np.sqrt(D) * torch.cos(torch.matmul(X, W) + b)`, called at
 * exp.py:63 for the training and the test set with one draw of W, b):
 *   d_out[i][k] = scale * cos(sum_j d_X[i][j] * d_W[j][k] + d_b[k])   (k < D)
 *   d_out[i][k] = 0                                                   (D <= k < ldo)
 * d_X [n][ldx] raw features (d used), d_W [d][D] row-major, d_b [D]; scale = 1/sqrt(D).
 * The draw of W and b stays on the host generator (tools.py:15-19).  fp32 MFMA GEMM
 * with the +b / cos / scale epilogue fused; phi written once, in the engine's padded
 * layout when ldo > D.
 * ------------------------------------------------------------------------- */
int fs_feature_map(const float* d_X, int64_t ldx, const float* d_W, const float* d_b, int n, int d, int D,
                   float scale, float* d_out, int64_t ldo, void* stream);

/* ------------------------------------------------------------------------- *
 * Data heterogeneity of a partition (exp.py:67-74):
 *   fs_gram:   d_G[a][b] = sum_r phi[r][a] * phi[r][b] over rows [0, rows)   (D x D, row
 *              stride ldg; exactly symmetric).  `torch.matmul(X.T, X)` of exp.py:67
 *              before the division by len.
 *   fs_hetero: d_S[j] = sum_{a,b} (G[a][b] / n_total - G_j[a][b] / n_j)^2 with G_j the
 *              Gram of client j's rows [row_off[j], row_off[j+1]) (never materialised);
 *              the caller forms sum_j n_j / n_total * sqrt(d_S[j]) (exp.py:73).
 * phi [rows][ld] fp32 packed by client, ld % 64 == 0, columns >= D ignored.  MFMA SYRK.
 * ------------------------------------------------------------------------- */
int fs_gram(const float* d_phi, int64_t ld, int64_t rows, int D, float* d_G, int64_t ldg, void* stream);
int fs_hetero(const float* d_phi, int64_t ld, const int64_t* d_row_off, int N, int D, const float* d_G,
              int64_t ldg, int64_t n_total, double* d_S, void* stream);


/* ------------------------------------------------------------------------- *
 * Round plan: the native round driver.  One fs_plan_round call enqueues the
 * launches of one round of the reference's loop (tools.py:337-352 FedAvg,
 * 364-379 FedProx; the train / aggregate / evaluate phases of FedAMW, 427-462):
 *   FS_PHASE_TRAIN      fs_local_train over all N clients with the shuffles of
 *                       round t; losses to d_loss_hist[t*N .. t*N+N)
 *   FS_PHASE_AGGREGATE  fs_aggregate(W_out, p) -> d_W_g  (p = d_p, or the override)
 *   FS_PHASE_EVAL       fs_eval(d_W_g) -> d_eval_hist[2t], [2t+1]
 *   FS_PHASE_EVAL_DEFER (with FS_PHASE_EVAL) round t's evaluation may ride on the
 *                       next call's TRAIN launch, on the CUs its client groups
 *                       leave idle (parallel split launches, C <= 16; the same
 *                       per-row arithmetic as fs_eval).  d_eval_hist[2t..] is then
 *                       written by that call if it aggregates, else (round 5) by the
 *                       call after it: the fused evaluation's finaliser rides on the
 *                       next AGGREGATE launch, and any call that trains or does not
 *                       aggregate runs a pending one first -- make one more
 *                       fs_plan_round call (phases 0 will do) or, since ABI 15,
 *                       fs_plan_eval_flush before reading d_eval_hist after a
 *                       TRAIN-only call.  The pending evaluation reads d_W_g
 *                       as it is when that next call's launches run: the caller
 *                       must NOT write d_W_g (its own aggregate, an all-reduce into
 *                       it, a copy) between the deferring call and the next
 *                       fs_plan_round.  Which launch carries it: a next call whose
 *                       phases include TRAIN fuses it into the training launch, which
 *                       runs before that call's own AGGREGATE rewrites d_W_g; a next
 *                       call without TRAIN runs it as an fs_eval launch of its own
 *                       before anything else.  The fp64 sum of the per-block partials
 *                       then follows the launch's evaluation-block count (CUs left
 *                       idle), so deferred and standalone losses agree to ~1e-12
 *                       relative, not bitwise.  Do not defer the last round's
 *                       evaluation.
 * fs_plan_shuffle(plan, seeds, t) replays round t's N*E training shuffles
 * (DataLoader passes of tools.py:179, client-major / epoch-minor seeds) into slot
 * t % 2 on the plan's side stream -- on the GPU (fs_randperm_device, default) or on
 * the plan's host thread pool plus an async upload; call it for round t+1 after
 * enqueueing round t so it overlaps the GPU.
 * The plan owns its shuffle buffers, copy stream and events; every other pointer
 * is borrowed and must outlive the plan.
 * ------------------------------------------------------------------------- */
#define FS_PHASE_TRAIN 1
#define FS_PHASE_AGGREGATE 2
#define FS_PHASE_EVAL 4
#define FS_PHASE_EVAL_DEFER 8

typedef struct fs_plan fs_plan;

typedef struct fs_plan_desc {
  /* local training (see fs_local_train) */
  const float* d_phi;
  int64_t ld;
  const int64_t* d_row_off;
  const int32_t* d_labels;
  const int32_t* d_order;
  const int64_t* h_n;          /* [N] rows per client (host) */
  int N, C, B, E;
  int G;                       /* from fs_local_train_plan (1 when chained) */
  void* d_ws;
  int64_t ws_bytes;
  int chained, prox, reg;
  float mu, lam;
  float* d_W_g;                /* [C][ld] round-start model; the aggregate is written here */
  float* d_W_out;              /* [N][C][ld] */
  double* d_loss_hist;         /* [R][N] */
  /* aggregation (see fs_aggregate) */
  const float* d_p;            /* [N] default mixture weights (may be NULL) */
  float* d_agg_ws;
  int64_t agg_ws_floats;
  int agg_chunks;
  /* evaluation (see fs_eval; may be NULL when FS_PHASE_EVAL is never used) */
  const float* d_phi_t;
  const int32_t* d_labels_t;
  int n_t;
  double* d_eval_ws;
  double* d_eval_hist;         /* [R][2] */
  int shuffle_device;          /* 1: replay shuffles with fs_randperm_device on the plan's side
                                  stream; 0: on the plan's host thread pool + async upload */
  int host_threads;            /* host replay threads; <= 0: min(16, hardware) */
  int shuffle_after_train;     /* 1 (device replay): round t+1's shuffles also wait for round t's
                                  local training, so they run beside what follows it (FedAMW: the
                                  p-solve, which leaves most CUs idle) instead of holding CUs a
                                  group of the split kernel is waiting for */
} fs_plan_desc;

int64_t fs_plan_desc_size(void);   /* sizeof(fs_plan_desc), for binding-layout checks */
int fs_plan_create(const fs_plan_desc* desc, fs_plan** out);
int fs_plan_destroy(fs_plan* plan);
int fs_plan_shuffle(fs_plan* plan, const int64_t* h_seeds, int t);
int fs_plan_round(fs_plan* plan, int t, float lr, int phases, const float* d_p_override, void* stream);
/* ABI 15: complete on `stream` every evaluation the plan still holds (a deferred one not yet
 * carried by a TRAIN launch, a fused one whose finaliser waits for the next AGGREGATE), so
 * d_eval_hist is final once the stream reaches this point.  Replaces the "one more
 * fs_plan_round call with phases 0" of ABI 14 (which still works). */
int fs_plan_eval_flush(fs_plan* plan, void* stream);
/* ABI 7 (device replay only; call before the first fs_plan_shuffle): generate the shuffles of
 * `rounds` consecutive rounds (a chunk: rounds cK .. cK+K-1) with ONE fs_randperm_device launch
 * into one of two chunk slots.  fs_plan_shuffle then only collects round t's seeds and launches
 * when the chunk's last round arrives (a partly collected chunk is launched by the first
 * fs_plan_round that needs it); the local training waits for its slot, and releases it, once
 * per chunk instead of once per round -- no cross-stream wait between the rounds of a chunk.
 * Rounds must be prepared in order; prepare chunk c+1 while chunk c runs. */
int fs_plan_set_shuffle_chunk(fs_plan* plan, int rounds);
/* ABI 7: launch a partly collected chunk now (after preparing a run's last round). */
int fs_plan_shuffle_flush(fs_plan* plan);
/* ABI 8: evaluation workgroups a TRAIN launch of this plan carries for FS_PHASE_EVAL_DEFER
 * (0: the plan evaluates with launches of its own; fs_tuning.no_eval_fuse = 1 at creation
 * forces 0). */
int fs_plan_eval_blocks(const fs_plan* plan);

/* ABI 7, measurement: timing events recorded without a system-scope release (so timing a
 * launch inside a round does not stall the next one); elapsed_ms synchronises on `end`. */
int fs_timer_create(void** ev);
int fs_timer_record(void* ev, void* stream);
int fs_timer_elapsed_ms(void* start, void* end, float* ms);
int fs_timer_destroy(void* ev);

#ifdef __cplusplus
}
#endif

#endif /* FEDSIM_H */
