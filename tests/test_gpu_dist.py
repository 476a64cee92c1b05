"""Sharded (multi-rank) drop-in on the GPU box: 2 ranks share the one GPU through the
gloo backend (RCCL needs one GPU per rank; the 8-GPU RCCL run is the driver's), and the
sharded parallel-client FedAvg/FedProx/FedAMW must match the single-process run within
fp32 summation-order noise."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem():
    rs = np.random.RandomState(3)
    D, C, sizes = 192, 6, [40, 23, 64, 7, 90, 33, 51]
    Xs = [(np.cos(rs.normal(size=(n, D))) / np.sqrt(D)).astype(np.float32) for n in sizes]
    ys = [rs.randint(0, C, size=n).astype(np.int64) for n in sizes]
    Xt = (np.cos(rs.normal(size=(70, D))) / np.sqrt(D)).astype(np.float32)
    yt = rs.randint(0, C, size=70).astype(np.int64)
    Xv = (np.cos(rs.normal(size=(45, D))) / np.sqrt(D)).astype(np.float32)
    yv = rs.randint(0, C, size=45).astype(np.int64)
    return D, C, Xs, ys, Xt, yt, Xv, yv


def _run(algo):
    import fedamw_amd
    from fedamw_amd.functions import tools
    D, C, Xs, ys, Xt, yt, Xv, yv = _problem()
    T = torch.from_numpy
    args = ([T(x) for x in Xs], [T(y) for y in ys], T(Xt), T(yt))
    stats = {}
    torch.manual_seed(11)
    if algo == 'fedamw':
        vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(T(Xv), T(yv)), batch_size=16, shuffle=True)
        out = tools.FedAMW(*args, vl, 'classification', C, D, 0.5, 2, 32, False, 0.0, True, 1e-3, 3, 0.05,
                           clients='parallel', stats=stats, verbose=False)
    else:
        out = tools.FedProx(*args, 'classification', C, D, 0.5, 2, 32, algo == 'fedprox', 0.02, True, 1e-3, 3,
                            clients='parallel', stats=stats, verbose=False)
    return [o.numpy() for o in out], stats['W_global'].cpu().numpy()


def _worker(rank, world, port, algo, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group('gloo', rank=rank, world_size=world)
    try:
        out[rank] = _run(algo)
    finally:
        torch.distributed.destroy_process_group()


def _problem_wide():
    """300 clients: the sharded p-solve (solver N = 2 x 152) runs qmc on the all-gathered rank
    blocks in place (fs_mix_solve_blocked), the single-process one qmc on [n_v][C][300]."""
    rs = np.random.RandomState(5)
    D, C = 64, 6
    sizes = list(rs.randint(3, 14, size=300))
    Xs = [(np.cos(rs.normal(size=(n, D))) / np.sqrt(D)).astype(np.float32) for n in sizes]
    ys = [rs.randint(0, C, size=n).astype(np.int64) for n in sizes]
    Xt = (np.cos(rs.normal(size=(70, D))) / np.sqrt(D)).astype(np.float32)
    yt = rs.randint(0, C, size=70).astype(np.int64)
    Xv = (np.cos(rs.normal(size=(150, D))) / np.sqrt(D)).astype(np.float32)
    yv = rs.randint(0, C, size=150).astype(np.int64)
    return D, C, Xs, ys, Xt, yt, Xv, yv


def _run_wide():
    import fedamw_amd
    from fedamw_amd import _lib
    from fedamw_amd.functions import tools
    D, C, Xs, ys, Xt, yt, Xv, yv = _problem_wide()
    T = torch.from_numpy
    torch.manual_seed(12)
    vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(T(Xv), T(yv)), batch_size=16, shuffle=True)
    fed = tools.Federation('fedamw', [T(x) for x in Xs], [T(y) for y in ys], T(Xt), T(yt), vl, 'classification', C,
                           D, 0.5, 2, 32, False, 0.0, True, 1e-3, 2, 0.01, 'parallel', verbose=False)
    for _ in range(2):
        fed.round()
    out = fed.results()
    solver = _lib.SOLVER_NAMES[_lib.lib().fs_mix_solve_last_mode()]
    p = fed.mixture.p[fed.pos_dev].cpu().numpy() if fed.zshard else fed.mixture.p.cpu().numpy()
    return [o.numpy() for o in out], fed.W_g[:, :D].cpu().numpy(), p, solver, fed.mixture.blocks


def _worker_wide(rank, world, port, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group('gloo', rank=rank, world_size=world)
    try:
        out[rank] = _run_wide()
    finally:
        torch.distributed.destroy_process_group()


def test_sharded_fedamw_reads_rank_blocks():
    """SURVEY 8(e) sharded FedAMW at 300 clients on 2 ranks: the all-gathered Z stays in its
    rank blocks and the qmc solver reads them in place (no layout copy); the result matches the
    single-process run (qmc on the standard layout, a different client-to-workgroup split of
    the same sums) within the fp32 tolerances."""
    ref, Wref, pref, solver, blocks = _run_wide()
    assert solver == 'qmc' and blocks == 1
    mgr = mp.get_context('spawn').Manager()
    out = mgr.dict()
    mp.spawn(_worker_wide, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        res, W, p, solver, blocks = out[r]
        assert solver == 'qmc' and blocks == 2
        assert np.abs(p - pref).max() <= 1e-5 * np.abs(pref).max()
        assert np.abs(W - Wref).max() <= 1e-5 * np.abs(Wref).max()
        np.testing.assert_allclose(res[0], ref[0], atol=1e-5)
        np.testing.assert_allclose(res[1], ref[1], atol=1e-5)
    assert np.array_equal(out[0][2], out[1][2])            # the replicated solve: identical p


@pytest.mark.parametrize('algo', ['fedavg', 'fedprox', 'fedamw'])
def test_sharded_matches_single_process(algo):
    ref, Wref = _run(algo)
    mgr = mp.get_context('spawn').Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), algo, out), nprocs=2, join=True)
    for r in range(2):
        res, W = out[r]
        assert np.abs(W - Wref).max() <= 1e-5 * np.abs(Wref).max()
        np.testing.assert_allclose(res[0], ref[0], atol=1e-5)
        np.testing.assert_allclose(res[1], ref[1], atol=1e-5)
        assert np.abs(res[2] - ref[2]).max() <= 100.0 / 70 + 1e-4


def test_bench_two_ranks_launcher():
    """The launcher the driver's 8-GPU node runs: ``bench.py --gpus 2`` starts two workers of
    itself (no torchrun), here over gloo on the box's one GPU (FS_BENCH_BACKEND=gloo: the RCCL
    path needs a GPU per rank), and relays rank 0's line: n_gpus and the dist object come from
    the process group, the checked all-reduce of rank + 1 gives 3."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FS_BENCH_BACKEND='gloo', HSA_ENABLE_IPC_MODE_LEGACY='0')
    env.pop('WORLD_SIZE', None)
    r = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--config', '2', '--steps', '2',
                        '--warmup', '1', '--no-legs', '--no-cpu-baseline', '--no-fedamw-leg'],
                       cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line['n_gpus'] == 2
    assert line['dist']['world_size'] == 2 and line['dist']['backend'] == 'gloo'
    assert line['dist']['allreduce_check'] == 3.0
    assert line['value'] > 0 and line['config']['clients_total'] == 200


def _worker_rccl(rank, world, port, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      HSA_ENABLE_IPC_MODE_LEGACY='0')
    torch.cuda.set_device(rank)
    torch.distributed.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device('cuda', rank))
    try:
        dev = torch.device('cuda', rank)
        # the per-round all-reduce of the partial aggregate (C x ld at config 2) and the Z
        # all-gather into rank blocks, through RCCL with one rank
        g = torch.Generator(device='cpu').manual_seed(9)
        W = torch.randn(10, 2048, generator=g).to(dev)
        ref = W.clone()
        torch.distributed.all_reduce(W, op=torch.distributed.ReduceOp.SUM)
        Z = torch.randn(64, 40, generator=g).to(dev)
        Zo = torch.empty(64 * 40, device=dev)
        torch.distributed.all_gather_into_tensor(Zo, Z.contiguous().view(-1))
        torch.cuda.synchronize()
        out[rank] = (torch.equal(W, ref), torch.equal(Zo.view(64, 40), Z),
                     torch.distributed.get_backend())
    finally:
        torch.distributed.destroy_process_group()


def test_rccl_world_one_collectives():
    """The RCCL path itself on the box's one GPU: a one-rank ``nccl`` process group (RCCL on
    ROCm) runs the two collectives the sharded round issues -- the all-reduce of the partial
    aggregate (dist.allreduce_sum_) and the all-gather of Z into rank blocks
    (dist.allgather_z, blocked) -- and returns the input unchanged.  Two ranks need two GPUs
    (RCCL refuses a shared device); the 8-GPU run is the driver's."""
    mgr = mp.get_context('spawn').Manager()
    out = mgr.dict()
    mp.spawn(_worker_rccl, args=(1, _free_port(), out), nprocs=1, join=True)
    ok_ar, ok_ag, backend = out[0]
    assert backend == 'nccl'
    assert ok_ar and ok_ag
