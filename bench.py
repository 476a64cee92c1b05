#!/usr/bin/env python3
"""Benchmark: client-rounds/s of the federated round on MI355X (BASELINE.json configs 2-5).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5] [...]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

Launch.  ``--gpus N`` with N > 1 and no WORLD_SIZE in the environment: this process
starts N worker processes of itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one per
GPU) before it makes any GPU call, relays rank 0's JSON line and exits non-zero if any
worker fails.  Under torchrun (WORLD_SIZE set) it is one of those workers.  A worker whose
LOCAL_RANK has no GPU fails; only the explicit FS_BENCH_BACKEND=gloo rehearsal (several
ranks sharing the visible GPUs, host-staged gloo collectives) wraps ranks onto devices.

One step = one federated round with parallel clients (every client of the round trains
from the global model): per-client local SGD (fs_local_train), weighted aggregation
(fs_aggregate; + one RCCL all-reduce of the C x D partial aggregate when N > 1), test
evaluation (fs_eval) and the device replay of every shuffle.  The headline workload
(``value``) is BASELINE config 2 per GPU: 100 non-IID (label-skewed) a9a-shaped clients x
512 rows, random-feature dim 2048, 10 classes, E = 2, B = 32, 10,000 test rows; weak
scaling: each rank owns 100 clients.  Inputs are resident in HBM before the timed region;
``value`` = all ranks' client-rounds / the max-over-ranks wall time of the K timed rounds.

Extra objects on the JSON line:
  dist          the process group as it ran: backend, world size, distinct devices, and one
                checked all-reduce (sum of rank+1 over the ranks).
  roofline      fs_local_train (the dominant kernel): algorithmic HBM bytes per launch
                (4*E*sum(n_j)*D + 8*E*sum(n_j) + 8*N*C*D) / mean launch time
                from HIP events on the launch stream, against 8 TB/s; ``traffic`` = PMC HBM
                bytes per launch and ``mfma_busy`` = the MFMA pipe's busy fraction, both from
                profiles/traffic_local_train_<config>.json, used only when its ``source_rev``
                equals the revision of the kernel sources being run (_lib.source_revision()).
  cpu_baseline  the CPU oracle (oracle/fedsim_oracle.py, numpy restatement of the reference
                round) timed on this host (rank 0, N = 1 only) on a bounded sample.
  fedamw        (config 2, one GPU) the other half of config 2 -- "FedAvg vs optimal mixture
                weights": FedAMW rounds on the same clients plus 128 validation rows each.
  config1       (default run, one GPU) exp.py's FedAMW on 10 chained a9a-shaped Dirichlet(0.01)
                clients, D = 2000, C = 2, R = 100: ms per round, the bin p-solve's us per step, and
                the numpy oracle's round on the host.
  config4 / config3 / config5
                (default run) the >= 1000-client BASELINE configs, each with its own rounds,
                ms_per_round, client-rounds/s, roofline and cpu_baseline; config 5 adds the
                p-solve's steps/s, bytes/s and PMC traffic.
Config 5 is BASELINE's 1000 clients over all GPUs (strong scaling: 1000/N clients per GPU);
the others keep their per-GPU share fixed (weak scaling).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

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
# the extra legs of the default run: (config, timed rounds, warmup rounds)
LEGS = ((4, 10, 10), (3, 5, 2), (5, 2, 1))     # (config, timed rounds, warm-up rounds)
# CPU-sample budget floors per leg: config 3's whole round (1,000 clients) fits in ~60 % of 6 s on
# the box's 16 host threads, so its baseline is a measured round instead of an extrapolation
# (VERDICT round 4, weak item 4); config 5's (~1 min of CPU per round) stays a stated sample
LEG_CPU_SECONDS = {3: 6.0}
# FedAMW legs whose CPU baseline is one whole oracle round timed end to end when the sample's
# estimate is at most this many seconds (config 5: ~90 s on 16 host cores)
CPU_WHOLE_ROUND_MAX_S = {5: 150.0}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None, help='GPUs (ranks); default WORLD_SIZE or 1')
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
    ap.add_argument('--cpu-seconds', type=float, default=10.0, help='budget of the headline CPU baseline sample')
    ap.add_argument('--leg-cpu-seconds', type=float, default=3.0, help='budget of each extra leg\'s CPU sample')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--host-shuffle', action='store_true', help='replay shuffles on host threads, not the GPU')
    ap.add_argument('--no-fedamw-leg', action='store_true', help='skip the FedAMW object of the config-2 line')
    ap.add_argument('--fedamw-rounds', type=int, default=2, help='timed FedAMW rounds of the config-2 leg')
    ap.add_argument('--no-legs', action='store_true', help='skip the config 3/4/5 objects of the default line')
    ap.add_argument('--train-form', choices=['auto', 'split', 'pair', 'teams', 'pipe'], default='auto',
                    help="fs_tuning.train_form / split_teams / split_pipe: the local-training kernel form for parallel "
                         "clients (A/B runs)")
    ap.add_argument('--launch-timeout', type=float, default=None,
                    help='--gpus N launcher: wall-clock bound on the whole run (seconds; default 1800 + 10 s per '
                         'timed or warm-up round + 60 s per FedAMW round, so a long but healthy run is not cut and a '
                         'launch whose every rank hangs still ends; 0 = none; exit code 124 when it trips)')
    ap.add_argument('--teardown-timeout', type=float, default=300.0,
                    help='--gpus N launcher: once a worker has exited 0, the seconds the others get to finish '
                         '(a rank hung in a collective or in teardown); exit code 124 when it trips (0 = none)')
    ap.add_argument('--no-eval-fuse', action='store_true',
                    help='fs_tuning.no_eval_fuse = 1: the deferred evaluation in launches of its own (PMC traffic split)')
    ap.add_argument('--split-early', choices=['auto', 'off'], default='auto',
                    help="fs_tuning.split_early: the split form's early row issue (A/B runs)")
    a = ap.parse_args(argv)
    for k, v in PRESETS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    a.custom = any(getattr(a, k) != v for k, v in PRESETS[a.config].items() if k != 'algo')
    if a.rounds is None:
        a.rounds = 100
    if a.launch_timeout is None:
        a.launch_timeout = default_launch_timeout(a)
    return a


def default_launch_timeout(a):
    """The launcher's default whole-run bound (with no bound, a launch whose
    every rank hangs in a collective before any finishes would wait forever): generous, and
    scaled to the work asked for."""
    return 1800.0 + 10.0 * (a.steps + a.warmup) + 60.0 * a.fedamw_rounds


# --------------------------------------------------------------------------------------------
# launcher (no GPU call in this process)
# --------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn(n, cmd=None, timeout=None, teardown=None):
    """Start n worker processes of this script (one per GPU; ``cmd`` overrides the command,
    for tests), relay rank 0's stdout, and return the exit code: 0 only if every worker
    exited 0.  A failed worker ends the others (they would wait forever in a collective).
    Two wall-clock bounds, each ending the workers (terminate, then kill) with exit code 124:
    ``teardown`` (default --teardown-timeout, 300 s) counts from the first worker that exits 0
    or from rank 0's result line, whichever comes first -- a rank hung in a collective or in
    teardown after the result is out must not hold the launcher forever -- and ``timeout``
    (default --launch-timeout: 1800 s + a per-round allowance) bounds the whole run."""
    if timeout is None or teardown is None:
        a = parse() if cmd is None else None
        if timeout is None:
            timeout = a.launch_timeout if a is not None else 0.0
        if teardown is None:
            teardown = a.teardown_timeout if a is not None else 300.0
    cmd = cmd or [sys.executable, '-u', os.path.abspath(__file__)] + sys.argv[1:]
    t_start = time.time()
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True))

    line_out = []                        # time rank 0's JSON result line was relayed

    def relay(pipe):
        for line in pipe:
            sys.stdout.write(line)
            sys.stdout.flush()
            if line.lstrip().startswith('{') and not line_out:
                line_out.append(time.time())

    th = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    th.start()
    def stop_all():
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + 20
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    rc = 0
    t_first_done = None
    while any(p.poll() is None for p in procs):
        bad = [p for p in procs if p.poll() not in (None, 0)]
        if bad:
            rc = bad[0].returncode
            print('bench: worker pid %d exited %d; stopping the others' % (bad[0].pid, rc), file=sys.stderr, flush=True)
            stop_all()
            break
        now = time.time()
        if t_first_done is None and (line_out or any(p.poll() == 0 for p in procs)):
            t_first_done = line_out[0] if line_out else now
        late = ('launch', timeout) if timeout and now - t_start > timeout else (
            ('teardown', teardown) if teardown and t_first_done is not None and now - t_first_done > teardown else None)
        if late:
            print('bench: workers still running after the %.0f s %s timeout; stopping them (exit 124)' % (late[1], late[0]),
                  file=sys.stderr, flush=True)
            stop_all()
            th.join(timeout=5)
            return 124
        time.sleep(0.2)
    th.join(timeout=5)
    for p in procs:
        if p.returncode not in (0, None) and rc == 0:
            rc = p.returncode
    return rc if rc >= 0 else 128 - rc


# --------------------------------------------------------------------------------------------
# worker
# --------------------------------------------------------------------------------------------
def setup_rank(args):
    """Device + process group of this worker.  Returns (ws, rank, dev, dist_info)."""
    import torch
    import torch.distributed as tdist
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    if args.gpus is not None and args.gpus != ws:
        raise SystemExit('bench: --gpus %d but WORLD_SIZE=%d' % (args.gpus, ws))
    backend = os.environ.get('FS_BENCH_BACKEND', 'nccl') if ws > 1 else None
    if backend not in (None, 'nccl', 'gloo'):
        raise SystemExit('bench: FS_BENCH_BACKEND must be nccl or gloo')
    local = int(os.environ.get('LOCAL_RANK', '0'))
    ndev = torch.cuda.device_count()
    if backend == 'gloo':
        local = local % max(1, ndev)          # rehearsal only: ranks may share the visible GPUs
    elif local >= ndev:
        raise SystemExit('bench: LOCAL_RANK %d has no GPU (%d visible)' % (local, ndev))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    info = {'backend': None, 'world_size': 1, 'devices': 1}
    if ws > 1:
        if backend == 'nccl':
            tdist.init_process_group('nccl', device_id=dev)
        else:
            tdist.init_process_group('gloo')
        t = torch.tensor([float(rank + 1)], device=dev if backend == 'nccl' else 'cpu')
        tdist.all_reduce(t, op=tdist.ReduceOp.SUM)
        want = ws * (ws + 1) / 2.0
        if float(t.item()) != want:
            raise SystemExit('bench: all-reduce sanity check gave %r, expected %r' % (float(t.item()), want))
        ids = [None] * ws
        props = torch.cuda.get_device_properties(dev)
        tdist.all_gather_object(ids, (socket.gethostname(), str(props.uuid) if hasattr(props, 'uuid') else local))
        info = {'backend': tdist.get_backend(), 'world_size': tdist.get_world_size(),
                'devices': len(set(str(i) for i in ids)), 'allreduce_check': float(t.item()),
                'rehearsal': backend == 'gloo'}
    return ws, rank, dev, info


def load_record(tag, kernel):
    """PMC record (HBM bytes, MFMA busy) measured for exactly this workload AND these kernel
    sources (profiles/traffic_<kernel>_<tag>.json with a matching source_rev), else None."""
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


def settle_clocks(dev, ms, work=None):
    """Hold the GPU busy for ``ms`` milliseconds before a measurement's warm-up rounds, so that a
    short timed region does not measure the device's clock ramp.  From idle the device takes tens
    of ms of sustained load to reach its steady clocks, and the steady state depends on the kind
    of load: config 2 at the driver's --warmup 5 ran 0.311-0.317 ms per round from idle,
    0.299-0.302 after 100 ms of fp32 GEMMs + 1 GiB copies, 0.292 / 0.290 after 50 / 200 warm-up
    rounds of the workload itself (profiles/r05/warmup_ab.txt).  So by default (``work`` given,
    FS_BENCH_SETTLE_KIND unset or 'workload') the settle repeats ``work`` -- launches of the
    workload's own local-training kernel into a scratch trainer on the same features, with
    shuffles from a private generator (the Federation's state and torch's global RNG are not
    touched; nothing the timed rounds read is produced here) -- and otherwise plain GEMMs / copies
    (FS_BENCH_SETTLE_KIND = gemm | copy | mixed).  Reported on the line as ``device_settle_ms``
    and ``device_settle_kind``; FS_BENCH_SETTLE_MS overrides the length (0 = off).
    Returns (ms, kind)."""
    ms = float(os.environ.get('FS_BENCH_SETTLE_MS', ms))
    if ms <= 0 or dev.type != 'cuda':
        return 0.0, None
    import torch
    kind = os.environ.get('FS_BENCH_SETTLE_KIND', 'workload' if work is not None else 'mixed')
    if kind == 'workload' and work is None:
        kind = 'mixed'
    if kind == 'workload':
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < ms:
            work()
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3, kind
    a = torch.randn(4096, 4096, device=dev)
    b = torch.randn(4096, 4096, device=dev)
    x = torch.empty(256 << 20, dtype=torch.float32, device=dev)      # 1 GiB streamed
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        if kind in ('gemm', 'mixed'):
            for _ in range(2):
                a = torch.mm(a, b) * 1e-3
        if kind in ('copy', 'mixed'):
            y.copy_(x)
            x.copy_(y)
        torch.cuda.synchronize()
    del x, y
    return (time.perf_counter() - t0) * 1e3, kind


def train_settle_work(fed, algo, lr):
    """The settle's unit of work for ``fed``: one launch of fed's local training (same features,
    group width and terms) into a scratch trainer, from a scratch copy of the global model, with
    shuffles drawn from a private numpy generator.  It runs the split form's LATE-issue instance
    (fs_tuning.split_early = -1; the pipe width as a plain split group): the same work and load as
    the timed launches under another kernel symbol, so that a kernel trace's statistics of the
    timed form hold only the timed rounds' launches (with their deferred evaluation) and agree
    with the line's launch time.  Returns (work, release)."""
    import torch
    from fedamw_amd import _lib, engine
    tr = engine.LocalTrainer(fed.feats, fed.C, fed.B, fed.E, split=fed.trainer.width, chained=False,
                             prox=algo == 'fedprox')
    seeds = np.random.default_rng(12345).integers(0, 2 ** 62, size=len(tr.pass_n), dtype=np.int64)
    tr.upload_perms(seeds)
    W0 = fed.W_g.detach().clone()
    prox, reg = algo == 'fedprox', algo == 'fedamw'

    def work():
        with _lib.tuning(split_early=-1):
            tr.run(W0, lr, prox, 5e-4 if prox else 0.0, reg, 1e-5, False)

    def release():
        nonlocal tr
        tr = None
        torch.cuda.synchronize()
    return work, release


def phase_ms(events, name):
    v = [a.elapsed_time(b) for n, a, b in (events or []) if n == name]
    return float(np.mean(v)) if v else None


def _np(x):
    return x.detach().cpu().numpy()


def cpu_fedamw_round(d, wl, rounds_R, lr_p=1e-3):
    """One WHOLE FedAMW round of the numpy oracle, timed end to end (config
    5's CPU baseline measured, not extrapolated): the local training of all N clients
    (tools.py:430-434), the Z GEMM of every client model on every validation row (448, hoisted), the
    R inner epochs of p-SGD over the pooled validation set (441-453), the aggregate with the learned
    p (455-460) and the test evaluation (461).  Returns (seconds, sample text)."""
    from oracle import fedsim_oracle as O
    N, D, C = len(d['X_train']), wl['D'], wl['C']
    W = O.mlp_init(D, C)
    Xv, yv = _np(d['X_val']).astype(np.float32), _np(d['y_val']).astype(np.int64)
    Xt, yt = _np(d['X_test']), _np(d['y_test'])
    t0 = time.perf_counter()
    Ws = [O.train_client(_np(d['X_train'][j]), _np(d['y_train'][j]), W, 0.5, 2, 32, False, 0.0, True, 1e-5)[0]
          for j in range(N)]
    t_train = time.perf_counter() - t0
    a = time.perf_counter()
    Z = np.einsum('ncd,vd->ncv', np.stack(Ws).astype(np.float32), Xv, optimize=True)
    t_z = time.perf_counter() - a
    a = time.perf_counter()
    p, _ = O.mixture_solve_z(Z, yv, np.full(N, 1.0 / N, np.float32), None, lr_p, rounds_R, 16)
    t_solve = time.perf_counter() - a
    del Z
    O.test_eval(Xt, yt, O.aggregate(Ws, p))
    el = time.perf_counter() - t0
    nv = len(yv)
    return el, ('1 whole FedAMW round of the numpy oracle timed end to end: %d client trainings (%d rows, D=%d, '
                'C=%d, E=2, B=32; %.1f s), the Z GEMM on all %d validation rows (%.1f s), all %d p-SGD steps '
                '(%d passes; %.1f s), aggregate + %d-row test eval; %.1f s'
                % (N, len(d['y_train'][0]), D, C, t_train, nv, t_z, rounds_R * ((nv + 15) // 16), rounds_R, t_solve,
                   len(yt), el))


def cpu_baseline(d, wl, budget, fedamw, rounds_R, z_rows=None, whole_max_s=0.0):
    """The numpy oracle on this host's cores, on a bounded sample of the same workload:
    local training of as many clients as fit ~60 % of ``budget`` (whole rounds when they all
    fit), the aggregate and the test evaluation; FedAMW adds the Z GEMM on a sample of the
    validation rows and 64 of the round's p-SGD steps on the round's own Z rows (``z_rows``:
    the GPU's Z of the first validation rows, all N clients; random logits only if absent).
    Extrapolated to client-rounds/s; ``extrapolation_factor`` = modelled round seconds /
    measured seconds, ``measured`` = whether whole rounds were timed (no extrapolation)."""
    import torch
    from oracle import fedsim_oracle as O
    from threadpoolctl import threadpool_info
    N, D, C = len(d['X_train']), wl['D'], wl['C']
    state = torch.get_rng_state()
    torch.manual_seed(1234)
    W = O.mlp_init(D, C)
    t0 = time.perf_counter()
    # local training of the clients, round after round, until about half the budget is spent
    # (at most 60 % inside a round): the per-client mean over every training done
    Ws, t_train, ntrain, rounds = [], 0.0, 0, 0
    while True:
        Ws = []
        for j in range(N):
            X, y = _np(d['X_train'][j]), _np(d['y_train'][j])
            a = time.perf_counter()
            Wj, _ = O.train_client(X, y, W, 0.5, 2, 32, wl['algo'] == 'fedprox', 5e-4, fedamw, 1e-5)
            t_train += time.perf_counter() - a
            ntrain += 1
            Ws.append(Wj)
            if time.perf_counter() - t0 > 0.6 * budget:
                break
        if len(Ws) == N:
            rounds += 1
        if len(Ws) < N or time.perf_counter() - t0 > 0.5 * budget:
            break
    k = len(Ws)
    p = np.full(k, 1.0 / N, dtype=np.float32)
    a = time.perf_counter()
    O.aggregate(Ws, p)
    t_agg = (time.perf_counter() - a) * N / k
    Xt, yt = _np(d['X_test']), _np(d['y_test'])
    a = time.perf_counter()
    O.test_eval(Xt, yt, Ws[-1])
    t_eval = time.perf_counter() - a
    t_round = t_train * N / ntrain + t_agg + t_eval
    sample = ('%d client trainings (%s; %d rows, D=%d, C=%d, E=2, B=32) + aggregate + %d-row test eval'
              % (ntrain, ('%d whole rounds of %d clients' % (rounds, N)) if rounds else ('%d of %d clients' % (k, N)),
                 len(d['y_train'][0]), D, C, len(yt)))
    if fedamw:
        nv = int(d['y_val'].numel()) if torch.is_tensor(d['y_val']) else len(d['y_val'])
        sv = min(nv, 512)
        Xv = _np(d['X_val'][:sv])
        a = time.perf_counter()
        np.einsum('ncd,vd->ncv', np.stack(Ws).astype(np.float32), Xv, optimize=True)
        t_z = (time.perf_counter() - a) * (N / k) * (nv / sv)
        steps = rounds_R * ((nv + 15) // 16)
        if z_rows is not None:             # [N, C, rows]: the round's own logits
            Zs = np.ascontiguousarray(z_rows)
            yv = _np(d['y_val'][:Zs.shape[2]]).astype(np.int64)
            zsrc = 'the round\'s Z on %d validation rows' % Zs.shape[2]
        else:
            Zs = np.random.RandomState(0).standard_normal((N, C, 16 * 64)).astype(np.float32) * 0.1
            yv = np.random.RandomState(1).randint(0, C, 16 * 64)
            zsrc = 'random logits'
        passes = max(1, 64 // ((Zs.shape[2] + 15) // 16))
        ps = passes * ((Zs.shape[2] + 15) // 16)
        a = time.perf_counter()
        O.mixture_solve_z(Zs, yv, np.full(N, 1.0 / N, np.float32), None, 1e-3, passes, 16)
        t_solve = (time.perf_counter() - a) / ps * steps
        t_round += t_z + t_solve
        sample += ('; FedAMW: Z GEMM on %d of %d validation rows, %d of the round\'s %d p-SGD steps on %s (N=%d)'
                   % (sv, nv, ps, steps, zsrc, N))
    el = time.perf_counter() - t0
    threads = max([i.get('num_threads', 1) for i in threadpool_info()] + [1])
    whole = bool(rounds) and not fedamw
    if fedamw and whole_max_s > 0 and t_round <= whole_max_s:
        # the sample's estimate fits: time one whole round instead (measured, factor 1)
        sec, text = cpu_fedamw_round(d, wl, rounds_R)
        torch.set_rng_state(state)
        return {'value': N / sec, 'unit': 'client-rounds/s', 'cores': int(threads), 'kind': 'port',
                'measured': True, 'extrapolation_factor': 1.0, 'sample': text,
                'sample_estimate': N / t_round}
    torch.set_rng_state(state)
    return {'value': N / t_round, 'unit': 'client-rounds/s', 'cores': int(threads), 'kind': 'port',
            'measured': whole, 'extrapolation_factor': 1.0 if whole else t_round / el,
            'sample': sample + ' of the numpy oracle, %.1f s, %s' % (
                el, 'whole rounds' if whole else 'extrapolated to whole rounds (x%.0f)' % (t_round / el))}


def pool_validation(d, ws, dev):
    """Every rank's clients contribute their validation rows; the pooled set (exp.py:92-99)
    is identical on every rank: one all-gather of the per-rank blocks (equal sizes)."""
    import torch
    import torch.distributed as tdist
    Xv, yv = d['X_val'], d['y_val']
    if ws == 1:
        return Xv, yv
    bx = torch.empty((ws * Xv.shape[0],) + tuple(Xv.shape[1:]), dtype=Xv.dtype, device=dev)
    by = torch.empty(ws * yv.shape[0], dtype=yv.dtype, device=dev)
    tdist.all_gather_into_tensor(bx, Xv.contiguous())
    tdist.all_gather_into_tensor(by, yv.contiguous())
    return bx, by


def fedamw_leg(d, wl, dev, R, rounds, warmup=1):
    """The FedAMW half of config 2 on the same clients (one GPU)."""
    import torch
    import fedamw_amd
    from fedamw_amd.functions import tools
    N, E, B = wl['clients'], 2, 32
    vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(d['X_val'], d['y_val']), batch_size=16,
                                     shuffle=True)
    torch.manual_seed(100)
    fed = tools.Federation('fedamw', d['X_train'], d['y_train'], d['X_test'], d['y_test'], vl, 'classification',
                           wl['C'], wl['D'], 0.5, E, B, False, 0.0, True, 1e-5, max(R, warmup + rounds), 1e-3,
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
    z_flop = 2.0 * N * wl['C'] * wl['D'] * nv
    solve_bytes = 4.0 * R * N * wl['C'] * nv
    rec, note = load_record('c2_fedamw', 'mix_solve')
    return {'ms_per_round': 1e3 * el / rounds, 'client_rounds_per_s': N * rounds / el,
            'train_ms': train_ms, 'z_gemm_ms': z_ms, 'z_gemm_tflops': z_flop / (z_ms * 1e-3) / 1e12,
            'z_gemm_frac_mfma_f32': z_flop / (z_ms * 1e-3) / 1e12 / MFMA_F32_PEAK_TFS,
            'p_solve_ms': solve_ms, 'p_solve_steps': steps, 'p_solve_us_per_step': 1e3 * solve_ms / steps,
            'p_solve_steps_per_s': steps / (solve_ms * 1e-3), 'p_solve_gbs': solve_bytes / (solve_ms * 1e-3) / 1e9,
            'p_solve_frac_hbm': solve_bytes / (solve_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            'p_solve_traffic': (rec or {}).get('bytes_per_launch'), 'p_solve_traffic_note': note,
            'p_solver': fedamw_amd._lib.SOLVER_NAMES.get(fedamw_amd._lib.lib().fs_mix_solve_last_mode(), '?'),
            'n_val': nv, 'inner_epochs': R, 'rounds_timed': rounds}


def config1_leg(dev, rounds=10, warmup=2, cpu_budget=3.0):
    """BASELINE config 1 -- exp.py's FedAMW on a9a split across 10 non-IID clients
    (/root/reference/exp.py:22-143 -> tools.py:413-463): exp.py's data prep (a9a-shaped synthetic
    rows -- no LIBSVM file travels -- Dirichlet(0.01) partition, full-batch pass, RFF map D = 2000,
    20/80 validation split) and FedAMW with exp.py's positional arguments and get_parameter('a9a')
    (default branch; lr_p = 1e-3, stated in experiment.py), CHAINED clients (the reference's
    semantics: one model walks the 10 clients), R = 100 (40,700 p-SGD steps per round with the
    `bin` p-solver).  Rounds ``warmup`` .. ``warmup + rounds`` of the 100 are timed (the LR
    schedule is the run's own); one GPU (a chain does not shard: replicas only).  CPU: the numpy
    oracle's whole round (the chained local training, the p-solve's R passes on the pooled
    validation set, the aggregate and the test evaluation), timed in full when it fits
    ``cpu_budget``, else with the p-SGD passes sampled and extrapolated (stated)."""
    import torch
    import fedamw_amd
    from fedamw_amd import experiment
    from fedamw_amd.functions import tools
    from fedamw_amd.functions.optimal_parameters import get_parameter
    P = get_parameter('a9a')
    D, N, R, E, B = 2000, 10, 100, 2, 32
    lr, lam, lr_p = P['lr'], P['lambda_reg'], P.get('lr_p', 1e-3)
    torch.manual_seed(100)
    np.random.seed(100)
    d = experiment.prepare('a9a', D, N, 0.01, P, '/nonexistent/', verbose=False)
    C = d['num_classes']
    fed = tools.Federation('fedamw', d['X_train'], d['y_train'], d['X_test'], d['y_test'], d['validloader'],
                           'classification', C, D, lr, E, B, False, 0.0, True, lam, R, lr_p, 'sequential',
                           verbose=False)
    settled, settle_kind = settle_clocks(dev, 100.0)
    for _ in range(warmup):
        fed.round()
    torch.cuda.synchronize()
    fed.events = []
    t0 = time.perf_counter()
    for _ in range(rounds):
        fed.round()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tr, tl, ta = fed.results()
    nv = fed.mixture.nv
    steps = R * ((nv + 15) // 16)
    solve_ms, train_ms, z_ms = (phase_ms(fed.events, k) for k in ('solve', 'train', 'z'))
    sizes = [int(len(y)) for y in d['y_train']]
    out = {'workload': 'config 1: exp.py FedAMW, a9a-shaped (synthetic), %d Dirichlet(0.01) clients (%d..%d rows, '
                       'sum %d), RFF D=%d, C=%d, E=%d, B=%d, round=%d, chained clients (reference semantics), '
                       '%d validation rows' % (N, min(sizes), max(sizes), sum(sizes), D, C, E, B, R, nv),
           'value': N * rounds / el, 'unit': 'client-rounds/s', 'ms_per_round': 1e3 * el / rounds,
           'rounds_timed': rounds, 'warmup': warmup, 'scaling': 'replicas only (a chain does not shard)',
           'train_ms': train_ms, 'z_gemm_ms': z_ms, 'p_solve_ms': solve_ms, 'p_solve_steps': steps,
           'p_solve_us_per_step': 1e3 * solve_ms / steps if solve_ms else None,
           'p_solver': fedamw_amd._lib.SOLVER_NAMES.get(fedamw_amd._lib.lib().fs_mix_solve_last_mode(), '?'),
           'local_train_group_width': fed.trainer.width, 'final_test_acc': float(ta[fed.t - 1]),
           'device_settle_ms': settled,
           'context': 'BASELINE.md: the reference CPU path runs this round in 20.0 s = 0.50 client-rounds/s on '
                      '8 Xeon cores (survey container; not a published number)'}
    if cpu_budget > 0:
        from oracle import fedsim_oracle as O
        from threadpoolctl import threadpool_info
        Xs = [_np(x) for x in d['X_train']]
        ys = [_np(y).astype(np.int64) for y in d['y_train']]
        Xv, yv = _np(d['X_val']).astype(np.float32), _np(d['y_val']).astype(np.int64)
        Xt, yt = _np(d['X_test']).astype(np.float32), _np(d['y_test']).astype(np.int64)
        state = torch.get_rng_state()
        torch.manual_seed(1234)
        W = O.mlp_init(D, C)
        a = time.perf_counter()
        Ws, _ = O._chain(Xs, ys, W, lr, E, B, False, 0.0, True, lam)
        t_train = time.perf_counter() - a
        a = time.perf_counter()
        Z = np.einsum('ncd,vd->ncv', np.stack(Ws).astype(np.float32), Xv, optimize=True)
        t_z = time.perf_counter() - a
        p = np.full(N, 1.0 / N, np.float32)
        spp = (nv + 15) // 16
        left = max(0.2, cpu_budget - t_train - t_z)
        a = time.perf_counter()
        p, buf = O.mixture_solve_z(Z, yv, p, None, lr_p, 1, 16)   # one pass: its cost decides the sample
        t_pass = time.perf_counter() - a
        passes = 1
        while passes < R and (passes + 1) * t_pass <= left:
            p, buf = O.mixture_solve_z(Z, yv, p, buf, lr_p, 1, 16)
            passes += 1
        t_solve = (time.perf_counter() - a) / passes * R
        a = time.perf_counter()
        O.aggregate(Ws, p)
        O.test_eval(Xt, yt, Ws[-1])
        t_rest = time.perf_counter() - a
        torch.set_rng_state(state)
        t_round = t_train + t_z + t_solve + t_rest
        threads = max([i.get('num_threads', 1) for i in threadpool_info()] + [1])
        whole = passes == R
        out['cpu_baseline'] = {
            'value': N / t_round, 'unit': 'client-rounds/s', 'cores': int(threads), 'kind': 'port',
            'measured': whole, 'extrapolation_factor': 1.0 if whole else R / passes,
            'sample': '1 round of the numpy oracle: the chained training of the %d clients (%.2f s), the Z GEMM '
                      '(%.2f s), %d of the %d p-SGD passes over the %d validation rows (%d steps each; %.2f s per '
                      'pass%s), aggregate + %d-row test eval' % (
                          N, t_train, t_z, passes, R, nv, spp, t_pass,
                          '' if whole else ', scaled to %d passes' % R, len(yt))}
    return out


def run_workload(wl, ws, rank, dev, steps, warmup, R_arg, cpu_seconds, host_shuffle=False, custom=False,
                 fedamw_leg_rounds=0):
    """One BASELINE workload: set up (untimed), ``warmup`` rounds, ``steps`` timed rounds
    bracketed by barrier + synchronize, max over ranks.  Returns the workload's line fields."""
    import torch
    import torch.distributed as tdist
    from fedamw_amd import data as fdata
    from fedamw_amd import dist as fdist
    from fedamw_amd.functions import tools
    cfg = wl['config']
    strong = cfg in STRONG and not custom
    N_loc = wl['clients'] // ws if strong else wl['clients']
    if N_loc < 1:
        raise SystemExit('bench: fewer clients than GPUs')
    E, B = 2, 32
    algo = wl['algo']
    fedamw = algo == 'fedamw'
    leg = fedamw_leg_rounds > 0
    n_val = 128 if leg else (wl['rows'] // 4 if fedamw else 0)
    # every rank synthesises its own clients (seed 1000 + rank); the pooled validation set of
    # FedAMW is all-gathered so that every rank solves the same p
    d = fdata.federated(N_loc, wl['rows'], wl['D'], wl['C'], wl['test'], n_val=n_val, shape=wl['shape'],
                        seed=1000 + rank, device=dev)
    # the job's client list: Federation shards clients by LPT; this rank's synthetic clients are
    # placed at the positions it will own, the other ranks' rows are never touched here.
    N_all = N_loc * ws
    shards = fdist.shard_lpt(fdist.client_work(np.full(N_all, wl['rows']), E, B), ws)
    Xs = [None] * N_all
    ys = [torch.zeros(wl['rows'], dtype=torch.int64)] * N_all      # other ranks' clients: lengths only
    for k, j in enumerate(shards[rank]):
        Xs[j], ys[j] = d['X_train'][k], d['y_train'][k]
    lr, mu = 0.5, (5e-4 if algo == 'fedprox' else 0.0)
    R = max(R_arg, warmup + steps)
    vl = None
    if fedamw:
        Xv, yv = pool_validation(d, ws, dev)
        vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(Xv, yv), batch_size=16, shuffle=True)
    torch.manual_seed(100)
    fed = tools.Federation(algo, Xs, ys, d['X_test'], d['y_test'], vl, 'classification', wl['C'], wl['D'], lr,
                           E, B, algo == 'fedprox', mu, fedamw, 1e-5, R, 1e-3,
                           'parallel', verbose=False, shuffle_device=not host_shuffle)
    assert len(fed.mine) == N_loc
    work, release = train_settle_work(fed, algo, lr)
    settled, settle_kind = settle_clocks(dev, 100.0, work)
    release()
    del work, release
    for _ in range(warmup):
        fed.round()
    torch.cuda.synchronize()
    # (FS_BENCH_NO_EVENTS=1: no per-launch timing events -- an A/B of their own cost; the line's
    # roofline then has no launch time)
    fed.events = None if os.environ.get('FS_BENCH_NO_EVENTS') == '1' else []
    if ws > 1:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fed.round()
    torch.cuda.synchronize()
    if ws > 1:
        tdist.barrier()
    el = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([el], device=dev if tdist.get_backend() == 'nccl' else 'cpu', dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        el = float(t.item())
    lt_ms = phase_ms(fed.events, 'train')
    tr, tl, ta = fed.results()
    agg = aggregate_timing(fed, wl)
    n_rows = int(fed.feats.rows)
    alg_bytes = 4.0 * E * n_rows * wl['D'] + 8.0 * E * n_rows + 8.0 * N_loc * wl['C'] * wl['D']
    achieved = alg_bytes / (lt_ms * 1e-3) / 1e9 if lt_ms else float('nan')
    tag = 'c%d%s' % (cfg, '' if algo == PRESETS[cfg]['algo'] else '_' + algo)
    rec, tnote = (None, 'custom workload') if custom else load_record(tag, 'local_train')
    # the same workload captured with fs_tuning.no_eval_fuse = 1: the training launch's own bytes,
    # without the deferred test-set evaluation the default plan carries inside it
    nrec, _ = (None, None) if custom else load_record(tag + '_nofuse', 'local_train')
    total = N_loc * ws
    out = {
        'value': total * steps / el,
        'ms_per_step': 1e3 * el / steps,
        'steps': steps,
        'scaling': 'strong' if strong else 'weak',
        'workload': '%s: %s, %d clients%s x %d rows, RFF D=%d, C=%d, E=%d, B=%d, %d test rows, round=%d, '
                    'parallel clients' % ('custom' if custom else 'config %d' % cfg, algo, total,
                                          '' if strong or ws == 1 else ' (%d/GPU)' % N_loc, wl['rows'], wl['D'],
                                          wl['C'], E, B, wl['test'], R),
        'config': {'algo': algo, 'clients_total': total, 'clients_per_gpu': N_loc, 'rows_per_client': wl['rows'],
                   'D': wl['D'], 'C': wl['C'], 'epochs': E, 'batch': B, 'test_rows': wl['test'],
                   'parallelism': 'clients%d' % ws},
        'roofline': {'kernel': 'fs_local_train', 'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS,
                     'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS,
                     'traffic': (rec or {}).get('bytes_per_launch'), 'traffic_note': tnote,
                     'traffic_no_eval_fuse': (nrec or {}).get('bytes_per_launch'),
                     'mfma_busy': (rec or {}).get('mfma_busy'),
                     'launch_ms': lt_ms, 'alg_bytes_per_launch': alg_bytes, 'group_width': fed.trainer.width,
                     'form': 'pair' if fed.trainer.pair else ('teams' if fed.trainer.teams else
                                                              ('pipe' if fed.trainer.pipe else
                                                               ('split' if fed.trainer.G > 1 else 'single')))},
        'aggregate': agg,
        'final_test_acc': float(ta[fed.t - 1]),
        'device_settle_ms': settled,
        'device_settle_kind': settle_kind,
    }
    if fedamw:
        nv = fed.mixture.nv
        p_steps = R * ((nv + 15) // 16)
        s_ms = phase_ms(fed.events, 'solve')
        z_ms = phase_ms(fed.events, 'z')
        sbytes = 4.0 * R * fed.mixture.N * wl['C'] * nv
        zflop = 2.0 * fed.mixture.N * wl['C'] * wl['D'] * nv / ws
        prec, pnote = (None, 'custom workload') if custom or ws > 1 else load_record(tag, 'mix_solve')
        out['fedamw'] = {'z_gemm_ms': z_ms, 'z_gemm_tflops': zflop / (z_ms * 1e-3) / 1e12 if z_ms else None,
                         'z_allgather_ms': phase_ms(fed.events, 'z_allgather'),
                         'p_solve_ms': s_ms, 'n_val': nv, 'p_solve_steps': p_steps,
                         'p_solve_us_per_step': 1e3 * s_ms / p_steps if s_ms else None,
                         'p_solve_steps_per_s': p_steps / (s_ms * 1e-3) if s_ms else None,
                         'p_solve_gbs': sbytes / (s_ms * 1e-3) / 1e9 if s_ms else None,
                         'p_solve_frac_hbm': sbytes / (s_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if s_ms else None,
                         'p_solve_alg_bytes': sbytes,
                         'p_solve_traffic': (prec or {}).get('bytes_per_launch'), 'p_solve_traffic_note': pnote,
                         'p_solver': _solver_name()}
    if leg:
        out['fedamw'] = fedamw_leg(d, wl, dev, R_arg, fedamw_leg_rounds)
    if rank == 0 and ws == 1 and cpu_seconds > 0:
        z_rows = None
        if fedamw:                      # the round's own Z rows (all clients) for the p-SGD sample
            mx = fed.mixture
            z_rows = _np(mx.Z[:512].view(-1, wl['C'], mx.ldN)[:, :, :mx.N].permute(2, 1, 0))
        out['cpu_baseline'] = cpu_baseline(d, wl, cpu_seconds, fedamw, R_arg, z_rows,
                                           whole_max_s=CPU_WHOLE_ROUND_MAX_S.get(cfg, 0.0) if not custom else 0.0)
    del fed, d, Xs, ys, vl
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def aggregate_timing(fed, wl, reps=20):
    """fs_aggregate -- the weighted aggregation kernel of the round (tools.py:345-350, 455-460) --
    timed with HIP events after the timed rounds: the round's own launch
    (FedAvg / FedProx: the plan's AGGREGATE phase; FedAMW: the Aggregator with the learned p) on
    the round's own clients x params buffer, ``reps`` launches back to back, the mean per launch.
    Algorithmic bytes per launch = 4 N C D (the clients' weights) + 4 C D (the aggregate) + 4 N (p)."""
    import torch
    from fedamw_amd import _lib
    N = len(fed.mine)
    nbytes = 4.0 * N * wl['C'] * wl['D'] + 4.0 * wl['C'] * wl['D'] + 4.0 * N
    t = max(fed.t - 1, 0)
    if fed.mixture is not None:
        p = fed.p_slice(fed.mixture.p) if fed.zshard else fed.mixture.p
        fn = lambda: fed.agg.run(fed.trainer.W_out, p, fed.W_g)     # noqa: E731
    else:
        fn = lambda: fed.plan.round(t, fed.lr, _lib.PHASE_AGGREGATE)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    # one event pair around the batch: the launches back to back as in a stream of rounds (an
    # event pair per launch measured dispatch gaps: 11.5 us per 8 MB launch at config 2)
    a, b = _lib.Timer(), _lib.Timer()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {'kernel': 'fs_aggregate', 'ms': ms, 'alg_bytes': nbytes, 'achieved': gbs, 'unit': 'GB/s',
            'peak': HBM_PEAK_GBS, 'frac': gbs / HBM_PEAK_GBS, 'clients': N, 'launches': reps,
            'note': 'HIP events around %d launches back to back after the timed rounds, the round\'s own inputs' % reps}


def _solver_name():
    from fedamw_amd import _lib
    return _lib.SOLVER_NAMES.get(_lib.lib().fs_mix_solve_last_mode(), '?')


def worker(args):
    # the JSON line is this process's only stdout: anything else -- gloo's / RCCL's connection
    # messages, library warnings -- goes to stderr (fd 1 is pointed at fd 2 for the whole run)
    sys.stdout.flush()
    line_out = os.fdopen(os.dup(1), 'w')
    os.dup2(2, 1)
    import torch
    import torch.distributed as tdist
    import fedamw_amd  # noqa: F401
    ws, rank, dev, dinfo = setup_rank(args)
    from fedamw_amd import _lib as flib
    flib.set_tuning(train_form={'auto': 0, 'split': 1, 'pair': 2, 'teams': 1, 'pipe': 1}[args.train_form],
                    split_teams={'auto': 0, 'split': -1, 'pair': -1, 'teams': 1, 'pipe': -1}[args.train_form],
                    split_pipe={'auto': 0, 'split': -1, 'pair': -1, 'teams': -1, 'pipe': 1}[args.train_form],
                    split_early={'auto': 0, 'off': -1}[args.split_early], no_eval_fuse=int(args.no_eval_fuse))
    wl = {k: getattr(args, k) for k in ('algo', 'clients', 'rows', 'D', 'C', 'test', 'shape')}
    wl['config'] = args.config
    headline = (args.config == 2 and not args.custom)
    leg_rounds = args.fedamw_rounds if (headline and args.algo == 'fedavg' and ws == 1
                                        and not args.no_fedamw_leg) else 0
    cpu_s = 0.0 if args.no_cpu_baseline else args.cpu_seconds
    main = run_workload(wl, ws, rank, dev, args.steps, args.warmup, args.rounds, cpu_s, args.host_shuffle,
                        args.custom, leg_rounds)
    out = {
        'metric': 'client-rounds/sec (whole node)',
        'value': main['value'],
        'unit': 'client-rounds/s',
        'n_gpus': dinfo['world_size'],
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': main['ms_per_step'],
        'higher_is_better': True,
        'scaling': main['scaling'],
        'vs_baseline': None,
        'dtype': 'f32',
        'data': 'synthetic (%s-shaped raw rows -> RFF, label-skewed Dirichlet(0.1) clients)' % args.shape,
        'config': dict(workload=main['workload'], **main['config']),
        'dist': dinfo,
        'roofline': main['roofline'],
        'aggregate': main['aggregate'],
        'final_test_acc': main['final_test_acc'],
        'device_settle_ms': main['device_settle_ms'],
        'device_settle_kind': main['device_settle_kind'],
    }
    for k in ('fedamw', 'cpu_baseline'):
        if k in main:
            out[k] = main[k]
    if headline and not args.no_legs:
        for cfg, k, w in LEGS:
            lw = dict(PRESETS[cfg], config=cfg)
            t0 = time.perf_counter()
            cpu_s = 0.0 if args.no_cpu_baseline else max(args.leg_cpu_seconds, LEG_CPU_SECONDS.get(cfg, 0.0))
            r = run_workload(lw, ws, rank, dev, k, w, 100, cpu_s)
            obj = {'workload': r['workload'], 'value': r['value'], 'unit': 'client-rounds/s',
                   'ms_per_round': r['ms_per_step'], 'rounds_timed': k, 'warmup': w, 'scaling': r['scaling'],
                   'roofline': r['roofline'], 'aggregate': r['aggregate'], 'final_test_acc': r['final_test_acc'],
                   'device_settle_ms': r['device_settle_ms'], 'device_settle_kind': r['device_settle_kind'],
                   'leg_wall_s': time.perf_counter() - t0}
            for key in ('fedamw', 'cpu_baseline'):
                if key in r:
                    obj[key] = r[key]
            out['config%d' % cfg] = obj
            if rank == 0:
                print('bench: config %d leg %.1f s, %.0f client-rounds/s' % (cfg, obj['leg_wall_s'], obj['value']),
                      file=sys.stderr, flush=True)
    if headline and not args.no_legs and ws == 1:
        t0 = time.perf_counter()
        obj = config1_leg(dev, cpu_budget=0.0 if args.no_cpu_baseline else args.leg_cpu_seconds)
        obj['leg_wall_s'] = time.perf_counter() - t0
        out['config1'] = obj
        print('bench: config 1 leg %.1f s, %.2f client-rounds/s (%.1f ms per round, p-solve %.3f us per step, %s)'
              % (obj['leg_wall_s'], obj['value'], obj['ms_per_round'], obj['p_solve_us_per_step'] or float('nan'),
                 obj['p_solver']), file=sys.stderr, flush=True)
    if rank == 0:
        print(json.dumps(out), file=line_out, flush=True)
    if ws > 1:
        tdist.barrier()
        tdist.destroy_process_group()


def main():
    args = parse()
    if (args.gpus or 1) > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(spawn(args.gpus))       # before any GPU call: this process only relays
    worker(args)


if __name__ == '__main__':
    main()
