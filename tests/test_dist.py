"""Multi-rank host logic on CPU (gloo, world size 2): LPT sharding, per-rank RNG pass
selection, and the partial-fold + all-reduce combination of the aggregate."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

import fedamw_amd
from fedamw_amd import dist


def test_shard_lpt_balances_and_covers():
    work = np.array([9, 1, 7, 3, 3, 8, 2, 2])
    shards = dist.shard_lpt(work, 3)
    allc = np.sort(np.concatenate(shards))
    np.testing.assert_array_equal(allc, np.arange(len(work)))
    loads = [work[s].sum() for s in shards]
    assert max(loads) - min(loads) <= work.max()
    for s in shards:
        assert list(s) == sorted(s)           # global order inside a shard


def test_client_work_counts_steps():
    np.testing.assert_array_equal(dist.client_work([32, 33, 1], 2, 32), [2, 4, 2])


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        rs = np.random.RandomState(0)
        N, C, D = 7, 3, 16
        Ws = rs.normal(size=(N, C, D)).astype(np.float32)
        ns = rs.randint(10, 100, size=N)
        p = (ns / ns.sum()).astype(np.float32)
        shards = dist.shard_lpt(dist.client_work(ns, 2, 32), world)
        mine = shards[rank]
        # rank-local ordered fold, then the single all-reduce of the round
        part = np.zeros((C, D), np.float32)
        for j in mine:
            part = (part + p[j] * Ws[j]).astype(np.float32)
        t = torch.from_numpy(part)
        dist.allreduce_sum_(t)
        # every rank draws the same seeds and keeps only its clients' passes
        torch.manual_seed(5)
        seeds = torch.empty(2 * N * 2, dtype=torch.int64).random_()[1::2].numpy().reshape(N, 2)
        g = dist.allgather_rows(torch.from_numpy(seeds[mine]), [len(s) for s in shards])
        inv = np.argsort(np.concatenate(shards), kind='stable')
        out[rank] = (t.numpy(), g.numpy()[inv], seeds)
    finally:
        tdist.destroy_process_group()


def test_two_rank_aggregate_and_seed_partition():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    rs = np.random.RandomState(0)
    N, C, D = 7, 3, 16
    Ws = rs.normal(size=(N, C, D)).astype(np.float32)
    ns = rs.randint(10, 100, size=N)
    p = (ns / ns.sum()).astype(np.float32)
    ref = np.zeros((C, D), np.float32)
    for j in range(N):
        ref = (ref + p[j] * Ws[j]).astype(np.float32)
    for r in range(world):
        agg, gathered, seeds = out[r]
        assert np.abs(agg - ref).max() <= 1e-6 * np.abs(ref).max()     # fp32 summation-order noise only
        np.testing.assert_array_equal(gathered, seeds)                 # shards reassemble the global order
    np.testing.assert_array_equal(out[0][0], out[1][0])               # identical global model on every rank


def _z_worker(rank, world, port, out):
    """Sharded FedAMW layout: each rank builds the Z block of ITS clients, all-gathers it into
    solver order; the solver-order matrix must equal the global Z with the columns permuted
    by solver_layout, and p mapped there and back must round-trip."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        rs = np.random.RandomState(3)
        N, C, nv = 11, 3, 5
        ns = rs.randint(10, 100, size=N)
        Zg = rs.normal(size=(nv, C, N)).astype(np.float32)          # global client order
        shards = dist.shard_lpt(dist.client_work(ns, 2, 32), world)
        L, pos = dist.solver_layout(shards)
        mine = shards[rank]
        Zl = np.zeros((nv, C, L), np.float32)
        Zl[:, :, :len(mine)] = Zg[:, :, mine]
        out_t = torch.empty(nv, C * world * L)
        dist.allgather_z(torch.from_numpy(Zl.reshape(nv, C * L)), C, out_t)
        out[rank] = (out_t.numpy(), L, pos)
    finally:
        tdist.destroy_process_group()


def test_two_rank_sharded_z_layout():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_z_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    rs = np.random.RandomState(3)
    N, C, nv = 11, 3, 5
    rs.randint(10, 100, size=N)
    Zg = rs.normal(size=(nv, C, N)).astype(np.float32)
    Z0, L, pos = out[0]
    np.testing.assert_array_equal(Z0, out[1][0])                     # every rank holds the same Z
    Zs = Z0.reshape(nv, C, world * L)
    np.testing.assert_array_equal(Zs[:, :, pos], Zg)                 # solver column pos[j] = client j
    pad = np.setdiff1d(np.arange(world * L), pos)
    assert (Zs[:, :, pad] == 0).all() and L % 4 == 0                  # padding clients are zero columns
    p = np.arange(N, dtype=np.float32) + 1
    ps = np.zeros(world * L, np.float32)
    ps[pos] = p
    np.testing.assert_array_equal(ps[pos], p)


def _zb_worker(rank, world, port, out):
    """Blocked all-gather (the sharded FedAMW path at every world size the driver runs):
    out's storage holds [R][n_v][C][L], rank r's block its clients in shard order."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        rs = np.random.RandomState(7)
        N, C, nv = 37, 4, 6
        ns = rs.randint(10, 100, size=N)
        Zg = rs.normal(size=(nv, C, N)).astype(np.float32)
        shards = dist.shard_lpt(dist.client_work(ns, 2, 32), world)
        L, pos = dist.solver_layout(shards)
        mine = shards[rank]
        Zl = np.zeros((nv, C, L), np.float32)
        Zl[:, :, :len(mine)] = Zg[:, :, mine]
        out_t = torch.empty(nv, C * world * L)
        dist.allgather_z(torch.from_numpy(Zl.reshape(nv, C * L)), C, out_t, blocked=True)
        out[rank] = (out_t.numpy(), L, pos)
    finally:
        tdist.destroy_process_group()


def test_four_rank_blocked_z_layout():
    """SURVEY 8(e), rehearsed at 4 ranks: the blocked all-gather leaves rank r's block at
    [r][n_v][C][L] (no layout copy), client j at block pos[j] // L, column pos[j] % L, padding
    columns zero -- the layout fs_mix_solve_blocked reads -- identically on every rank."""
    world = 4
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_zb_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    rs = np.random.RandomState(7)
    N, C, nv = 37, 4, 6
    rs.randint(10, 100, size=N)
    Zg = rs.normal(size=(nv, C, N)).astype(np.float32)
    Z0, L, pos = out[0]
    for r in range(1, world):
        np.testing.assert_array_equal(Z0, out[r][0])
    Zb = Z0.reshape(world, nv, C, L)
    for j in range(N):
        np.testing.assert_array_equal(Zb[pos[j] // L, :, :, pos[j] % L], Zg[:, :, j])
    used = np.zeros(world * L, bool)
    used[pos] = True
    assert (Zb.transpose(1, 2, 0, 3).reshape(nv, C, world * L)[:, :, ~used] == 0).all() and L % 4 == 0


def _rank_check_worker(rank, world, port, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import fedamw_amd  # noqa: F401
        from fedamw_amd.functions import tools
        X = [torch.zeros(5, 8)]
        y = [torch.zeros(5, dtype=torch.int64)]
        try:
            tools.FedAvg(X, y, X[0], y[0], 'classification', 2, 8, 0.1, 1, 32, False, 0.0, False, 0.0, 1,
                         clients='parallel', verbose=False)
            out[rank] = 'no error'
        except ValueError as e:
            out[rank] = str(e)
    finally:
        tdist.destroy_process_group()


def test_parallel_clients_need_one_per_rank():
    """N < world size with clients='parallel' is a clear ValueError on every rank (not a
    'bad sizes' failure deep in the planner)."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rank_check_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        assert 'at least one client per rank' in out[r], out[r]


def _label_shard_worker(rank, world, port, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import fedamw_amd  # noqa: F401
        from fedamw_amd import dist as fdist
        from fedamw_amd.functions import tools
        ns = np.array([5, 7, 6, 9])
        mine = fdist.shard_lpt(fdist.client_work(ns, 1, 32), world)[rank]
        res = []
        for bad_own in (False, True):
            # the other rank's clients carry garbage labels (bench.py passes placeholders there)
            y = [torch.full((int(n),), 999, dtype=torch.int64) for n in ns]
            for j in mine:
                y[j] = torch.zeros(int(ns[j]), dtype=torch.int64)
            if bad_own:
                y[mine[0]][0] = 5
            X = [torch.zeros(int(n), 8) for n in ns]
            try:
                tools.FedAvg(X, y, X[0], y[0][:1] * 0, 'classification', 2, 8, 0.1, 1, 32, False, 0.0, False, 0.0, 1,
                             clients='parallel', verbose=False)
                res.append('no error')
            except ValueError as e:
                res.append('ValueError: ' + str(e))
            except RuntimeError as e:          # no GPU here: past every input check
                res.append('RuntimeError')
        out[rank] = res
    finally:
        tdist.destroy_process_group()


def test_sharded_label_check_covers_own_clients_only():
    """clients='parallel' under torch.distributed: each rank validates the labels of ITS clients
    only -- the other ranks' entries need only have the right lengths (bench.py's placeholders)
    -- and an out-of-range label among its own clients is still a ValueError."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_label_shard_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        ok, bad = out[r]
        assert 'labels must lie' not in ok, ok
        assert bad.startswith('ValueError') and 'training labels' in bad, bad
