"""Client sharding across GPUs (one process per GPU, torch.distributed over RCCL).

The reference simulates clients serially in one process and has no collectives
(SURVEY.md section 2).  Here, with ``clients='parallel'``, clients are independent
inside a round, so they are sharded across ranks and the only exchange per round
is ONE all-reduce (sum, fp32) of the per-rank partial aggregates
sum_{j in rank} p_j W_j  (C x ld floats; 80 KB at C=10, D=2048) -- a latency-bound
collective over xGMI.  FedAMW additionally needs every client model applied to the pooled
validation set (Z, tools.py:448): each rank computes the Z columns of ITS clients (the
sharded Z-GEMM, fs_mix_z), the ranks all-gather Z once per round, and every rank runs the
identical, deterministic p-solve on it (no broadcast); the learned p then weights the same
partial aggregate + all-reduce as FedAvg.  The solver's client axis is rank-major
("solver order"): rank r's clients occupy columns r*L .. r*L + n_r - 1 of every class
segment, L = max_r n_r rounded up to 4, the rest are zero columns whose p stays 0.
``clients='sequential'`` (the reference's chained clients) cannot shard: every rank
runs a full replica.

Everything here is host logic (who owns which client, which RNG passes it
replays); it is exercised on CPU with the gloo backend in tests/test_dist.py.
"""
import numpy as np
import torch
import torch.distributed as tdist


def world():
    """(rank, world_size) of the default process group, (0, 1) without one."""
    if tdist.is_available() and tdist.is_initialized():
        return tdist.get_rank(), tdist.get_world_size()
    return 0, 1


def client_work(ns, E, B):
    """Dependent SGD steps per client: E * ceil(n_j / B) (the kernel's critical path)."""
    ns = np.asarray(ns, dtype=np.int64)
    return E * ((ns + B - 1) // B)


def shard_lpt(work, nranks):
    """Longest-processing-time-first assignment of clients to ranks.

    Returns a list (per rank) of client indices in ascending (global) order, so that
    each rank's partial fold visits its clients in the reference's order."""
    work = np.asarray(work, dtype=np.int64)
    order = np.argsort(-work, kind='stable')
    load = np.zeros(nranks, dtype=np.int64)
    owner = np.empty(len(work), dtype=np.int64)
    for j in order:
        r = int(np.argmin(load))
        owner[j] = r
        load[r] += work[j]
    return [np.nonzero(owner == r)[0] for r in range(nranks)]


def allreduce_sum_(t, group=None):
    """In-place sum across ranks (RCCL on GPU tensors, gloo on CPU)."""
    if world()[1] > 1:
        tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=group)
    return t


def allgather_rows(local, counts, group=None):
    """Concatenate every rank's ``local`` rows ([k_r, ...], k_r = counts[r]) in rank order."""
    rank, ws = world()
    if ws == 1:
        return local
    kmax = int(max(counts))
    pad = torch.zeros((kmax,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]].copy_(local)
    bufs = [torch.empty_like(pad) for _ in range(ws)]
    tdist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:int(c)] for b, c in zip(bufs, counts)], 0)


def solver_layout(shards):
    """Client axis of the sharded p-solve: returns (L, pos) with L the per-rank block width
    (max shard size rounded up to 4, so every rank's Z block has the same 16-byte aligned
    shape) and pos[j] = the solver column of global client j (rank-major)."""
    L = (max(len(s) for s in shards) + 3) // 4 * 4
    n = sum(len(s) for s in shards)
    pos = np.empty(n, dtype=np.int64)
    for r, s in enumerate(shards):
        pos[np.asarray(s, dtype=np.int64)] = r * L + np.arange(len(s))
    return L, pos


def allgather_z(Z_local, C, out, group=None, blocked=False):
    """Z_local [n_v, C*L] (this rank's clients, class-major: column c*L + i) -> out, R = world
    size.  ``blocked``: out's storage holds the rank blocks as the all-gather leaves them,
    [R][n_v][C*L] -- the layout fs_mix_solve_blocked reads (no copy); else out [n_v, C*R*L]
    in solver order (column c*(R*L) + r*L + i): one all-gather, then one layout copy."""
    nv, CL = Z_local.shape
    L = CL // C
    R = world()[1]
    if R == 1:
        out.copy_(Z_local)
        return out
    if blocked:
        tdist.all_gather_into_tensor(out.view(-1), Z_local.contiguous().view(-1), group=group)
        return out
    buf = torch.empty((R * nv, CL), dtype=Z_local.dtype, device=Z_local.device)    # rank blocks along dim 0
    tdist.all_gather_into_tensor(buf, Z_local.contiguous(), group=group)
    out.view(nv, C, R, L).copy_(buf.view(R, nv, C, L).permute(1, 2, 0, 3))
    return out
