#!/usr/bin/env python3
"""Benchmark: client-rounds/s of the federated round on MI355X (BASELINE.json config 2).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--algo fedavg|fedprox|fedamw]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

One step = one federated round with parallel clients (every client of the round
trains from the global model): per-client local SGD (fs_local_train), weighted
aggregation (fs_aggregate; + one RCCL all-reduce of the C x D partial aggregate
when N > 1), test evaluation (fs_eval), and the host's RNG replay of every shuffle.
Workload per GPU = config 2: 100 non-IID (label-skewed) a9a-shaped clients x 512
rows, random-feature dim 2048, 10 classes, E = 2, B = 32, 10,000 test rows.
Weak scaling: each rank owns 100 clients, so the job simulates 100 * N clients.
Inputs are resident in HBM before the timed region; `value` = all ranks' client
rounds / the max-over-ranks wall time of the K timed rounds.

Extra objects on the JSON line:
  roofline      fs_local_train (the dominant kernel): algorithmic HBM bytes per launch
                (4*E*sum(n_j)*D + 8*E*sum(n_j) + 8*N*C*D) / mean launch time
                from HIP events on the launch stream, against 8 TB/s; `traffic` = PMC HBM
                bytes per launch from profiles/traffic_local_train_<config>.json (rocprofv3
                FETCH_SIZE*2 + WRITE_SIZE), used only when its `source_rev` equals the
                revision of the kernel sources being run (_lib.source_revision()), else null.
  cpu_baseline  the CPU oracle (oracle/fedsim_oracle.py, numpy restatement of the
                reference round) timed on this host on whole rounds of the same workload.
  fedamw        (config 2, one GPU) the other half of config 2 -- "FedAvg vs optimal
                mixture weights": FedAMW rounds on the same clients plus 128 validation
                rows each (tools.py:413-463): ms per round, the p-solve's sequential steps/s
                and its bytes/s against 8 TB/s (4*R*N*C*n_v bytes of Z per round), the Z-GEMM's
                TFLOP/s against the fp32 MFMA peak (2*N*C*D*n_v flop per round).
Config 5 is BASELINE's 1000 clients over all GPUs (strong scaling: 1000/N clients per GPU);
the others keep their per-GPU share fixed (weak scaling).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as tdist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import fedamw_amd  # noqa: E402
from fedamw_amd import data as fdata  # noqa: E402
from fedamw_amd.functions import tools  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table (spec)
MFMA_F32_PEAK_TFS = 157.3   # dense fp32 MFMA (v_mfma_f32_16x16x4_f32), MI355X_MICROARCH.md

# BASELINE.json configs that fit one GPU, per-GPU shapes; config 4 is config 2's
# FedAvg shape at 1,250 clients x 64 rows per GPU (10,000 clients on 8 GPUs).
PRESETS = {
    2: dict(algo='fedavg', clients=100, rows=512, D=2048, C=10, test=10000, shape='a9a'),
    3: dict(algo='fedprox', clients=1000, rows=465, D=4096, C=7, test=50000, shape='covtype'),
    4: dict(algo='fedavg', clients=1250, rows=64, D=2048, C=10, test=10000, shape='a9a'),
    # config 5: FedAMW (mixture-weight solve every round) over 1000 clients in TOTAL x (128 train
    # + 32 validation rows), D = 16384 -- strong scaling: each of N GPUs trains 1000/N clients
    5: dict(algo='fedamw', clients=1000, rows=128, D=16384, C=10, test=10000, shape='a9a'),
}
STRONG = {5}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', type=int, default=2, choices=sorted(PRESETS),
                    help='BASELINE.json config preset (per-GPU shape); the flags below override it')
    ap.add_argument('--algo', choices=['fedavg', 'fedprox', 'fedamw'])
    ap.add_argument('--clients', type=int, help='clients per GPU')
    ap.add_argument('--rows', type=int, help='training rows per client')
    ap.add_argument('--D', type=int)
    ap.add_argument('--C', type=int)
    ap.add_argument('--test', type=int)
    ap.add_argument('--shape', choices=['a9a', 'covtype'])
    ap.add_argument('--rounds', type=int, help="the algorithm's `round` argument (LR schedule; FedAMW's inner "
                                                'p-SGD epochs per round); default 100 = the reference default')
    ap.add_argument('--cpu-seconds', type=float, default=10.0, help='budget of the CPU baseline sample')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--host-shuffle', action='store_true', help='replay shuffles on host threads, not the GPU')
    ap.add_argument('--no-fedamw-leg', action='store_true', help='skip the FedAMW object of the config-2 line')
    ap.add_argument('--fedamw-rounds', type=int, default=2, help='timed FedAMW rounds of the config-2 leg')
    a = ap.parse_args()
    for k, v in PRESETS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    a.custom = any(getattr(a, k) != v for k, v in PRESETS[a.config].items() if k != 'algo')
    if a.rounds is None:
        a.rounds = 100
    return a


def cpu_baseline(d, args, budget):
    """Whole FedAvg rounds of the same workload through the numpy oracle (rank 0 only)."""
    from oracle import fedsim_oracle as O
    from threadpoolctl import threadpool_info
    Xs = [x.cpu().numpy() for x in d['X_train']]
    ys = [y.cpu().numpy() for y in d['y_train']]
    Xt, yt = d['X_test'].cpu().numpy(), d['y_test'].cpu().numpy()
    p = O._weights(ys)
    W = O.mlp_init(args.D, args.C)
    state = torch.get_rng_state()
    torch.manual_seed(1234)
    rounds, clients_done = 0, 0
    t0 = time.perf_counter()
    while True:
        Ws = []
        for X, y in zip(Xs, ys):
            Wj, _ = O.train_client(X, y, W, 0.5, 2, 32, args.algo == 'fedprox', 5e-4, False, 0.0)
            Ws.append(Wj)
            clients_done += 1
        W = O.aggregate(Ws, p)
        O.test_eval(Xt, yt, W)
        rounds += 1
        el = time.perf_counter() - t0
        if el >= budget:
            break
    torch.set_rng_state(state)
    threads = max([i.get('num_threads', 1) for i in threadpool_info()] + [1])
    return {'value': clients_done / el, 'unit': 'client-rounds/s', 'cores': int(threads), 'kind': 'port',
            'sample': '%d whole round(s) (%d clients x %d rows, D=%d, C=%d, E=2, B=32, aggregate + %d-row test eval) '
                      'of the numpy oracle, %.1f s' % (rounds, len(Xs), args.rows, args.D, args.C, len(yt), el)}


def load_traffic(tag, kernel='local_train'):
    """PMC HBM bytes per launch measured for exactly this workload AND these kernel sources
    (profiles/traffic_<kernel>_<tag>.json with a matching source_rev), else None."""
    from fedamw_amd import _lib
    path = os.path.join(ROOT, 'profiles', 'traffic_%s_%s.json' % (kernel, tag))
    if not os.path.exists(path):
        return None, 'no PMC capture for this workload'
    with open(path) as f:
        rec = json.load(f)
    rev = _lib.source_revision(kernel)
    if rec.get('source_rev') != rev:
        return None, 'stale PMC capture (kernel sources %s, measured on %s)' % (rev, rec.get('source_rev'))
    return rec, 'PMC %s' % rec.get('source', '')


def pool_validation(d, ws, dev):
    """Every rank's clients contribute their validation rows; the pooled set (exp.py:92-99)
    is identical on every rank: one all-gather of the per-rank blocks (equal sizes)."""
    Xv, yv = d['X_val'], d['y_val']
    if ws == 1:
        return Xv, yv
    bx = torch.empty((ws * Xv.shape[0],) + tuple(Xv.shape[1:]), dtype=Xv.dtype, device=dev)
    by = torch.empty(ws * yv.shape[0], dtype=yv.dtype, device=dev)
    tdist.all_gather_into_tensor(bx, Xv.contiguous())
    tdist.all_gather_into_tensor(by, yv.contiguous())
    return bx, by


def phase_ms(events, name):
    v = [a.elapsed_time(b) for n, a, b in (events or []) if n == name]
    return float(np.mean(v)) if v else None


def fedamw_leg(d, args, dev, rounds, warmup=1):
    """The FedAMW half of config 2 on the same clients (one GPU)."""
    N, E, B, R = args.clients, 2, 32, args.rounds
    vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(d['X_val'], d['y_val']), batch_size=16,
                                     shuffle=True)
    torch.manual_seed(100)
    fed = tools.Federation('fedamw', d['X_train'], d['y_train'], d['X_test'], d['y_test'], vl, 'classification',
                           args.C, args.D, 0.5, E, B, False, 0.0, True, 1e-5, max(R, warmup + rounds), 1e-3,
                           'parallel', verbose=False)
    for _ in range(warmup):
        fed.round()
    torch.cuda.synchronize()
    fed.events = []
    t0 = time.perf_counter()
    for _ in range(rounds):
        fed.round()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    fed.results()
    nv = fed.mixture.nv
    steps = R * ((nv + 15) // 16)
    z_ms, solve_ms, train_ms = (phase_ms(fed.events, k) for k in ('z', 'solve', 'train'))
    z_flop = 2.0 * N * args.C * args.D * nv
    solve_bytes = 4.0 * R * N * args.C * nv
    return {'ms_per_round': 1e3 * el / rounds, 'client_rounds_per_s': N * rounds / el,
            'train_ms': train_ms, 'z_gemm_ms': z_ms, 'z_gemm_tflops': z_flop / (z_ms * 1e-3) / 1e12,
            'z_gemm_frac_mfma_f32': z_flop / (z_ms * 1e-3) / 1e12 / MFMA_F32_PEAK_TFS,
            'p_solve_ms': solve_ms, 'p_solve_steps': steps, 'p_solve_us_per_step': 1e3 * solve_ms / steps,
            'p_solve_steps_per_s': steps / (solve_ms * 1e-3), 'p_solve_gbs': solve_bytes / (solve_ms * 1e-3) / 1e9,
            'p_solve_frac_hbm': solve_bytes / (solve_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            'p_solver': fedamw_amd._lib.SOLVER_NAMES.get(fedamw_amd._lib.lib().fs_mix_solve_last_mode(), '?'),
            'n_val': nv, 'inner_epochs': R, 'rounds_timed': rounds}


def main():
    args = parse()
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    # (ranks wrap onto the visible devices and FS_BENCH_BACKEND=gloo swaps RCCL out: only to
    # rehearse the multi-rank path on a one-GPU box; the driver's runs are one rank per GPU)
    local = int(os.environ.get('LOCAL_RANK', '0')) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if ws > 1:
        backend = os.environ.get('FS_BENCH_BACKEND', 'nccl')
        if backend == 'nccl':
            tdist.init_process_group('nccl', device_id=dev)
        else:
            tdist.init_process_group(backend)
    strong = args.config in STRONG and not args.custom
    N_loc = args.clients // ws if strong else args.clients
    if N_loc < 1:
        raise SystemExit('bench: fewer clients than GPUs')
    E, B = 2, 32
    fedamw = args.algo == 'fedamw'
    leg = (args.config == 2 and not args.custom and not fedamw and ws == 1 and not args.no_fedamw_leg)
    n_val = 128 if leg else (args.rows // 4 if fedamw else 0)
    # every rank synthesises its own clients (seed 1000 + rank); the pooled validation set of
    # FedAMW is all-gathered so that every rank solves the same p
    d = fdata.federated(N_loc, args.rows, args.D, args.C, args.test, n_val=n_val, shape=args.shape,
                        seed=1000 + rank, device=dev)
    # the job's client list: Federation shards clients by LPT; this rank's synthetic clients are
    # placed at the positions it will own, the other ranks' rows are never touched here.
    from fedamw_amd import dist as fdist
    N_all = N_loc * ws
    shards = fdist.shard_lpt(fdist.client_work(np.full(N_all, args.rows), E, B), ws)
    Xs = [None] * N_all
    ys = [torch.zeros(args.rows, dtype=torch.int64)] * N_all      # other ranks' clients: lengths only
    for k, j in enumerate(shards[rank]):
        Xs[j], ys[j] = d['X_train'][k], d['y_train'][k]
    lr, mu = 0.5, (5e-4 if args.algo == 'fedprox' else 0.0)
    R = max(args.rounds, args.warmup + args.steps)
    vl = None
    if fedamw:
        Xv, yv = pool_validation(d, ws, dev)
        vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(Xv, yv), batch_size=16, shuffle=True)
    torch.manual_seed(100)
    fed = tools.Federation(args.algo, Xs, ys, d['X_test'], d['y_test'], vl, 'classification', args.C, args.D, lr,
                           E, B, args.algo == 'fedprox', mu, fedamw, 1e-5, R, 1e-3,
                           'parallel', verbose=False, shuffle_device=not args.host_shuffle)
    assert len(fed.mine) == N_loc
    for _ in range(args.warmup):
        fed.round()
    torch.cuda.synchronize()
    fed.events = None if os.environ.get('FS_BENCH_NO_EVENTS') == '1' else []   # (diagnostic A/B)
    if ws > 1:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_t = []
    for _ in range(args.steps):
        h0 = time.perf_counter()
        fed.round()
        host_t.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    if ws > 1:
        tdist.barrier()
    el = time.perf_counter() - t0
    if os.environ.get('FS_BENCH_HOST_TIMES') == '1':     # (diagnostic: host enqueue time per round)
        print('host us per round() call: mean %.1f min %.1f max %.1f; wall per round %.1f'
              % (1e6 * np.mean(host_t), 1e6 * np.min(host_t), 1e6 * np.max(host_t), 1e6 * el / args.steps),
              file=sys.stderr, flush=True)
    if ws > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        el = float(t.item())
    lt_ms = phase_ms(fed.events, 'train')
    tr, tl, ta = fed.results()
    n_rows = int(fed.feats.rows)
    alg_bytes = 4.0 * E * n_rows * args.D + 8.0 * E * n_rows + 8.0 * N_loc * args.C * args.D
    achieved = alg_bytes / (lt_ms * 1e-3) / 1e9 if lt_ms else float('nan')
    tag = 'c%d%s' % (args.config, '' if args.algo == PRESETS[args.config]['algo'] else '_' + args.algo)
    traffic, tnote = (None, 'custom workload') if args.custom else load_traffic(tag)
    total = N_loc * ws
    out = {
        'metric': 'client-rounds/sec (whole node)',
        'value': total * args.steps / el,
        'unit': 'client-rounds/s',
        'n_gpus': ws,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': 1e3 * el / args.steps,
        'higher_is_better': True,
        'scaling': 'strong' if strong else 'weak',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': 'synthetic (%s-shaped raw rows -> RFF, label-skewed Dirichlet(0.1) clients)' % args.shape,
        'config': {'workload': '%s: %s, %d clients%s x %d rows, RFF D=%d, C=%d, E=%d, B=%d, %d test rows, '
                               'round=%d, parallel clients'
                               % ('custom' if args.custom else 'config %d' % args.config, args.algo, total,
                                  '' if strong or ws == 1 else ' (%d/GPU)' % N_loc, args.rows, args.D, args.C, E, B,
                                  args.test, R),
                   'algo': args.algo, 'clients_total': total, 'clients_per_gpu': N_loc, 'rows_per_client': args.rows,
                   'D': args.D, 'C': args.C, 'epochs': E, 'batch': B, 'test_rows': args.test,
                   'parallelism': 'clients%d' % ws},
        'roofline': {'kernel': 'fs_local_train', 'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS,
                     'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS,
                     'traffic': (traffic or {}).get('bytes_per_launch'), 'traffic_note': tnote,
                     'launch_ms': lt_ms, 'alg_bytes_per_launch': alg_bytes, 'group_width': fed.trainer.G},
        'final_test_acc': float(ta[fed.t - 1]),
    }
    if fedamw:
        out['fedamw'] = {'z_gemm_ms': phase_ms(fed.events, 'z'), 'z_allgather_ms': phase_ms(fed.events, 'z_allgather'),
                         'p_solve_ms': phase_ms(fed.events, 'solve'), 'n_val': fed.mixture.nv}
    if leg:
        out['fedamw'] = fedamw_leg(d, args, dev, args.fedamw_rounds)
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(d, args, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if ws > 1:
        tdist.destroy_process_group()


if __name__ == '__main__':
    main()
