"""HIP path vs the reference's golden vectors and the CPU oracle (run on the MI355X box).

Tolerances (fp32): see tests/fixtures.py -- global W per round within 1e-5 of max|W|,
losses within 1e-5, accuracy within one test sample; kernel-level checks state theirs.
"""
import json
import os
import re

import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.fixtures import (BENCH_CASES, HORIZON_CASES, LONG_CASES, LOSS_RTOL, P_RTOL, ROUND_CASES, TRAIN_UNITS,
                            W_RTOL, acc_tol, horizon_rtol, horizon_rtol_rounds, load, load_bench, load_horizon, load_long, positional,
                            split_clients)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def amd():
    import fedamw_amd
    from fedamw_amd import _lib, engine, rng
    from fedamw_amd.functions import tools
    _lib.lib()
    return type('amd', (), dict(lib=_lib, engine=engine, rng=rng, tools=tools))


def _dl(X, y, bs=16):
    return torch.utils.data.DataLoader(torch.utils.data.TensorDataset(torch.from_numpy(X), torch.from_numpy(y)),
                                       batch_size=bs, shuffle=True)


def run_dropin(amd, d, **kw):
    Xs, ys = split_clients(d)
    Xs = [torch.from_numpy(x) for x in Xs]
    ys = [torch.from_numpy(y) for y in ys]
    mode = 'parallel' if str(d['mode']) == 'par' else 'sequential'
    stats = {'trace': True}
    torch.manual_seed(int(d['torch_seed']))
    Xt, yt = torch.from_numpy(d['X_test']), torch.from_numpy(d['y_test'])
    if str(d['algo']) == 'fedamw':
        out = amd.tools.FedAMW(Xs, ys, Xt, yt, _dl(d['X_val'], d['y_val']), *positional(d), float(d['lr_p']),
                               clients=mode, stats=stats, verbose=False, **kw)
    else:
        fn = amd.tools.FedAvg if str(d['algo']) == 'fedavg' else amd.tools.FedProx
        out = fn(Xs, ys, Xt, yt, *positional(d), clients=mode, stats=stats, verbose=False, **kw)
    return out, stats


@pytest.mark.parametrize('name', ROUND_CASES)
def test_dropin_matches_reference_golden(amd, name):
    d = load(name)
    (tr, tl, ta), stats = run_dropin(amd, d)
    W, Wref = stats['W_rounds'], d['W']
    assert W.shape == Wref.shape
    for t in range(len(Wref)):
        err = np.abs(W[t] - Wref[t]).max()
        assert err <= W_RTOL * np.abs(Wref[t]).max(), (name, t, err)
    np.testing.assert_allclose(tr.numpy(), d['train_loss'], rtol=0,
                               atol=LOSS_RTOL * max(1, np.abs(d['train_loss']).max()))
    np.testing.assert_allclose(tl.numpy(), d['test_loss'], rtol=0,
                               atol=LOSS_RTOL * max(1, np.abs(d['test_loss']).max()))
    assert np.abs(ta.numpy() - d['test_acc']).max() <= acc_tol(d)
    if 'p' in d:
        p = stats['p'].cpu().numpy()
        assert np.abs(p - d['p'][-1]).max() <= P_RTOL * np.abs(d['p']).max()


@pytest.mark.parametrize('name', LONG_CASES)
def test_dropin_long_horizon_golden(amd, name):
    """20 rounds at D = 1024, C = 10 against the reference (FedProx / FedAMW, chained and
    parallel clients): fp32 drift over many rounds stays inside the stated tolerances."""
    d = load_long(name)
    (tr, tl, ta), stats = run_dropin(amd, d)
    W = stats['W_rounds'][d['snap']]
    for k in range(len(d['snap'])):
        err = np.abs(W[k] - d['W'][k]).max()
        assert err <= W_RTOL * np.abs(d['W'][k]).max(), (name, int(d['snap'][k]), err)
    np.testing.assert_allclose(tr.numpy(), d['train_loss'], rtol=0,
                               atol=LOSS_RTOL * max(1, np.abs(d['train_loss']).max()))
    np.testing.assert_allclose(tl.numpy(), d['test_loss'], rtol=0,
                               atol=LOSS_RTOL * max(1, np.abs(d['test_loss']).max()))
    assert np.abs(ta.numpy() - d['test_acc']).max() <= acc_tol(d)
    if 'p' in d:
        assert np.abs(stats['p'].cpu().numpy() - d['p'][-1]).max() <= P_RTOL * np.abs(d['p']).max()


@pytest.mark.parametrize('name', BENCH_CASES)
def test_dropin_benchmark_length_fedamw(amd, name):
    """The FedAMW drop-in at config 2's N = 100, C = 10 (the quarter-wave p-solver config 2's
    leg runs) with >= 5,000 dependent p-SGD steps per round over R = 34 rounds, chained and
    parallel clients, against the reference: global models at the snapshot rounds, the final
    mixture weights, losses and accuracy within the stated fp32 tolerances."""
    d = load_bench(name)
    (tr, tl, ta), stats = run_dropin(amd, d)
    assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == 'quad'
    W = stats['W_rounds'][d['snap']]
    for k in range(len(d['snap'])):
        err = np.abs(W[k] - d['W'][k]).max()
        assert err <= W_RTOL * np.abs(d['W'][k]).max(), (name, int(d['snap'][k]), err)
    p = stats['p'].cpu().numpy()
    assert np.abs(p - d['p'][-1]).max() <= P_RTOL * np.abs(d['p'][-1]).max()
    np.testing.assert_allclose(tr.numpy(), d['train_loss'], rtol=0,
                               atol=LOSS_RTOL * max(1, np.abs(d['train_loss']).max()))
    np.testing.assert_allclose(tl.numpy(), d['test_loss'], rtol=0,
                               atol=LOSS_RTOL * max(1, np.abs(d['test_loss']).max()))
    assert np.abs(ta.numpy() - d['test_acc']).max() <= acc_tol(d)
    np.testing.assert_array_equal(torch.empty(4, dtype=torch.int64).random_().numpy(), d['rng_after'])


def _record_margin(name, rec):
    """Append one case's measured distances and bounds to $FS_MARGINS_OUT (JSON lines; the GPU
    run's record of how far the GPU sits from the reference, scripts/horizon_margins.py
    tabulates it into profiles/<round>/horizon_margins.json)."""
    out = os.environ.get('FS_MARGINS_OUT')
    if out:
        os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
        with open(out, 'a') as f:
            f.write(json.dumps(dict(case=name, **rec)) + '\n')


@pytest.mark.parametrize('name', HORIZON_CASES)
def test_dropin_solver_horizon_fedamw(amd, name):
    """The FedAMW drop-in against the reference at the horizons of the two p-solvers configs 1
    and 5 run (tools.py:423 -- momentum persisting across rounds -- and 441-453): ``qmc``, the
    multi-CU solver of config 5 (N = 300 > 256, C = 10, R = 20 rounds of 1,740 dependent
    momentum steps; lr_p = 3e-4, at the configs' 1e-3 the reference itself diverges here, see
    make_golden.py HORIZON); ``qmc1000``, config 5's exact instance (N = 1000: K = 16 workgroups
    of 64 clients, the 16-partner hop; R = 10 rounds of 2,880 steps, lr_p = 1e-4 chained, 2e-5
    parallel); ``qmc1000s``, the same instance with parallel clients at lr_p = 1e-4 on
    label-skewed, better-conditioned inputs; and ``bin``, config 1's two-class solver (N = 10,
    C = 2, n_v = 6,509: 4,070 steps per round, R = 10, lr_p = 1e-3); chained and parallel
    clients.  Bounds (round 6): round t's global model and losses within max(1e-5, 2 x the
    fp32-vs-fp64 drift the restatement accumulates by round t) (tests/golden/horizon_drift.py,
    tests/fixtures.py horizon_rtol_rounds); the final p within the whole run's derived bound.
    Every round's global model, the final mixture weights, the losses, the accuracy and where
    the generator is left; the measured distances go to $FS_MARGINS_OUT."""
    d = load_horizon(name)
    (tr, tl, ta), stats = run_dropin(amd, d)
    solver = str(d['solver'])
    family = re.match(r'[a-z]+', solver).group(0)
    assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == family
    if solver.startswith('qmc1000'):
        # config 5's exact solver instance: K = 16 workgroups of 64 clients, 4 per lane
        assert amd.lib.last_mix_layout() == (16, 4)
    W = stats['W_rounds']
    assert W.shape == d['W'].shape
    bW, bl = horizon_rtol_rounds(name, 'W'), horizon_rtol_rounds(name, 'loss')
    tol_p = horizon_rtol(name, 'p')
    eW = [float(np.abs(W[t] - d['W'][t]).max() / np.abs(d['W'][t]).max()) for t in range(len(W))]
    p = stats['p'].cpu().numpy()
    ep = float(np.abs(p - d['p'][-1]).max() / np.abs(d['p'][-1]).max())
    ltr = float(max(1, np.abs(d['train_loss']).max()))
    lte = float(max(1, np.abs(d['test_loss']).max()))
    el = [float(max(abs(float(tr[t]) - float(d['train_loss'][t])) / ltr, abs(float(tl[t]) - float(d['test_loss'][t])) / lte))
          for t in range(len(W))]
    _record_margin(name, dict(W_rel_err=eW, W_bound=bW.tolist(), p_rel_err=ep, p_bound=tol_p, loss_err=el,
                              loss_bound=bl.tolist(), acc_abs_err=float(np.abs(ta.numpy() - d['test_acc']).max()),
                              acc_tol=float(acc_tol(d))))
    for t in range(len(W)):
        assert eW[t] <= bW[t], (name, t, eW[t], bW[t])
        assert el[t] <= bl[t], (name, t, el[t], bl[t])
    assert ep <= tol_p, (ep, tol_p)
    assert np.abs(ta.numpy() - d['test_acc']).max() <= acc_tol(d)
    np.testing.assert_array_equal(torch.empty(4, dtype=torch.int64).random_().numpy(), d['rng_after'])


def test_mix_solve_config5_horizon_vs_oracle(amd):
    """Config 5's p-solve shape (N = 1000, C = 10; the auto choice is qmc) over R = 100 inner
    epochs of n_val = 3,200 rows: 20,000 dependent momentum steps in one launch, lr_p = 1e-3
    (the configs' value), against the oracle's fp32 p-SGD on the GPU's own Z (tools.py:441-453);
    then a second call of 5,000 steps continuing p and the momentum buffer (tools.py:423)."""
    N, C, D, nv, R = 1000, 10, 64, 3200, 100
    rs = np.random.RandomState(17)
    dev = torch.device('cuda')
    Xv = (np.cos(rs.normal(size=(nv, D)) * 2.0) / np.sqrt(D)).astype(np.float32)
    yv = rs.randint(0, C, size=nv).astype(np.int64)
    # logits of std ~0.35: well-conditioned (the fp32 oracle against itself with fp64
    # accumulation of the logits and the gradient: 8e-7 of max|p| after 20,000 steps; at std 1.4
    # that summation-order sensitivity is 4.6e-6) while p still moves by 150x its start
    Wc = (rs.normal(size=(N, C, D)) * 0.5).astype(np.float32)
    p0 = np.full(N, 1.0 / N, np.float32)
    mix = amd.engine.Mixture(torch.from_numpy(Xv), torch.from_numpy(yv), D, C, N, 16, torch.from_numpy(p0), dev)
    Wd = torch.zeros(N, C, mix.f.ld, device=dev)
    Wd[:, :, :D] = torch.from_numpy(Wc)
    pr, br = p0, None
    for call, epochs in enumerate((R, R // 4)):
        torch.manual_seed(90 + call)
        mix.solve(Wd, amd.rng.draw_pass_seeds(epochs), 1e-3, z=(call == 0))
        torch.cuda.synchronize()
        assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == 'qmc'
        mix.check_errors()
        Zn = mix.Z.view(nv, C, mix.ldN)[:, :, :N].permute(2, 1, 0).contiguous().cpu().numpy()
        torch.manual_seed(90 + call)
        pr, br = O.mixture_solve_z(Zn, yv, pr, br, 1e-3, epochs, 16)
        p, b = mix.p.cpu().numpy(), mix.buf.cpu().numpy()
        assert np.abs(p - pr).max() <= P_RTOL * np.abs(pr).max(), (call, np.abs(p - pr).max(), np.abs(pr).max())
        assert np.abs(b - br).max() <= 1e-4 * np.abs(br).max(), call
        assert np.abs(pr - p0).max() > 10 * P_RTOL * np.abs(pr).max()      # p moved: not a vacuous check


@pytest.mark.parametrize('chunk', [1, 3, 7])
@pytest.mark.parametrize('name', [c for c in LONG_CASES if 'fedamw' not in c])
def test_dropin_shuffle_chunks(amd, name, chunk):
    """Shuffles generated K rounds per launch (options['shuffle_chunk']; the default is 8)
    give bitwise the same run as one launch per round, including a partial last chunk (R =
    20), and leave the generator where the reference leaves it."""
    d = load_long(name)
    (tr, tl, ta), st = run_dropin(amd, d, options={'shuffle_chunk': chunk})
    after = torch.empty(4, dtype=torch.int64).random_()
    (tr8, tl8, ta8), st8 = run_dropin(amd, d, options={'shuffle_chunk': 8})
    after8 = torch.empty(4, dtype=torch.int64).random_()
    assert np.array_equal(st['W_rounds'], st8['W_rounds'])
    assert torch.equal(tr, tr8) and torch.equal(tl, tl8) and torch.equal(ta, ta8) and torch.equal(after, after8)


def _federation(amd, d, **kw):
    Xs, ys = split_clients(d)
    Xs = [torch.from_numpy(x) for x in Xs]
    ys = [torch.from_numpy(y) for y in ys]
    algo = str(d['algo'])
    vl = _dl(d['X_val'], d['y_val']) if algo == 'fedamw' else None
    lr_p = float(d['lr_p']) if algo == 'fedamw' else 1e-3
    torch.manual_seed(int(d['torch_seed']))
    return amd.tools.Federation(algo, Xs, ys, torch.from_numpy(d['X_test']), torch.from_numpy(d['y_test']), vl,
                                *positional(d), lr_p, 'parallel' if str(d['mode']) == 'par' else 'sequential',
                                verbose=False, **kw)


@pytest.mark.parametrize('name', [c for c in LONG_CASES if 'seq' not in c])
def test_dropin_deferred_eval(amd, name):
    """A round's evaluation carried by the next round's training launch (FS_PHASE_EVAL_DEFER, on
    the CUs the client groups leave idle) gives the same test loss / accuracy as a launch of its
    own: the same per-row arithmetic (eval_rows.h, shared by both), only the double-precision
    sum order of the partials differs (rtol 1e-12); the training itself is bitwise unchanged."""
    d = load_long(name) if name in LONG_CASES else load(name)
    if _federation(amd, d).plan.eval_blocks() == 0:
        pytest.skip('the training launch of this shape carries no evaluation blocks')
    (tr0, tl0, ta0), st0 = run_dropin(amd, d, options={'defer_eval': False})
    (tr1, tl1, ta1), st1 = run_dropin(amd, d, options={'defer_eval': True})
    assert np.array_equal(st0['W_rounds'], st1['W_rounds']) and torch.equal(tr0, tr1)
    np.testing.assert_allclose(tl1.numpy(), tl0.numpy(), rtol=1e-12, atol=0)
    assert torch.equal(ta0, ta1)


def test_deferred_eval_uses_idle_cus(amd):
    """A parallel split plan with fewer client groups than CUs carries evaluation blocks (as
    many as the CUs the groups leave idle, at most one per 16 test rows), and a deferred
    evaluation lands in the history only once the next TRAIN (or any call without one) has
    run; fs_tuning.no_eval_fuse turns the fusion off."""
    d = load_long([c for c in LONG_CASES if 'seq' not in c and 'fedamw' not in c][0])
    Xs, ys = split_clients(d)
    Xs = [torch.from_numpy(x) for x in Xs]
    ys = [torch.from_numpy(y) for y in ys]
    torch.manual_seed(int(d['torch_seed']))
    fed = amd.tools.Federation('fedprox' if bool(d['prox']) else 'fedavg', Xs, ys, torch.from_numpy(d['X_test']),
                               torch.from_numpy(d['y_test']), None, *positional(d)[:7], float(d['mu']), False,
                               float(d['lam']), int(d['R']), 1e-3, 'parallel', verbose=False)
    if fed.trainer.G < 2:
        pytest.skip('not a split launch at this shape')
    E = fed.plan.eval_blocks()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    tr = fed.trainer
    assert E == min(cus - tr.groups(cus) * tr.width, (len(d['y_test']) + 15) // 16) and E > 0
    fed.eval_hist.fill_(-7.0)
    fed.round()                                    # evaluation of round 0 deferred
    torch.cuda.synchronize()
    assert float(fed.eval_hist[0, 0]) == -7.0
    fed.round()                                    # ... carried by round 1's training launch
    torch.cuda.synchronize()
    assert float(fed.eval_hist[0, 0]) != -7.0 and float(fed.eval_hist[1, 0]) == -7.0
    tr, tl, ta = fed.results()                     # results() runs the pending one
    assert np.isfinite(tl[:2].numpy()).all() and float(fed.eval_hist[1, 0]) != -7.0
    with amd.lib.tuning(no_eval_fuse=1):
        assert _federation(amd, d).plan.eval_blocks() == 0


def test_plan_eval_flush_after_train_only(amd):
    """ABI 15: after a TRAIN-only fs_plan_round that carried a deferred
    evaluation, d_eval_hist is not yet written (its finaliser waits for the next AGGREGATE);
    fs_plan_eval_flush completes it -- the same test loss / accuracy as the run that evaluates
    round 0 in a launch of its own (rtol 1e-12: only the fp64 sum order of the partials
    differs) -- and a second flush is a no-op."""
    d = load_long([c for c in LONG_CASES if 'seq' not in c and 'fedamw' not in c][0])
    # (each Federation re-seeds the global generator and its rounds draw from it: the reference
    # run goes first, so both runs train on the same shuffles)
    ref = _federation(amd, d, options={'defer_eval': False})
    ref.round()
    torch.cuda.synchronize()
    fed = _federation(amd, d)
    if fed.plan.eval_blocks() == 0:
        pytest.skip('the training launch of this shape carries no evaluation blocks')
    fed.eval_hist.fill_(-7.0)
    fed.round()                                    # round 0: its evaluation deferred
    fed.plan.round(1, fed.lr, amd.lib.PHASE_TRAIN)  # TRAIN only: carries it, the finaliser waits
    torch.cuda.synchronize()
    assert float(fed.eval_hist[0, 0]) == -7.0
    fed.plan.eval_flush()
    torch.cuda.synchronize()
    got, want = fed.eval_hist[0].cpu().numpy(), ref.eval_hist[0].cpu().numpy()
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=0)
    fed.plan.eval_flush()                          # nothing pending: no launch, no change
    torch.cuda.synchronize()
    assert np.array_equal(fed.eval_hist[0].cpu().numpy(), got) and float(fed.eval_hist[1, 0]) == -7.0
    fed.trainer.check_errors()


def test_dropin_consumes_rng_like_reference(amd):
    """After the call, the global generator must be where the reference left it."""
    d = load('fedprox_seq')
    run_dropin(amd, d)
    after_amd = torch.empty(4, dtype=torch.int64).random_()
    Xs, ys = split_clients(d)
    torch.manual_seed(int(d['torch_seed']))
    O.FedProx(Xs, ys, d['X_test'], d['y_test'], *positional(d))
    after_oracle = torch.empty(4, dtype=torch.int64).random_()
    assert torch.equal(after_amd, after_oracle)


# ----------------------------------------------------------------------------- kernels


def _train_via_abi(amd, Xs, ys, W0, lr, E, B, prox, mu, reg, lam, chained, ld=None, seed=0, split=None):
    """Run fs_local_train on clients Xs/ys; returns (W_out [N,C,D], loss [N])."""
    dev = torch.device('cuda')
    C, D = W0.shape
    feats = amd.engine.Features([torch.from_numpy(x) for x in Xs], [torch.from_numpy(y) for y in ys], D, dev, ld)
    tr = amd.engine.LocalTrainer(feats, C, B, E, split=split, chained=chained)
    torch.manual_seed(seed)
    seeds = amd.rng.draw_pass_seeds(len(Xs) * E)
    tr.upload_perms(seeds)
    Wg = torch.zeros(C, feats.ld, device=dev)
    Wg[:, :D] = torch.from_numpy(W0)
    W, loss = tr.run(Wg, lr, prox, mu, reg, lam, chained)
    torch.cuda.synchronize()
    tr.check_errors()
    _train_via_abi.last_G = tr.G
    Wn = W.cpu().numpy()
    assert np.all(Wn[:, :, D:] == 0), 'padded columns must stay exactly zero'
    return Wn[:, :, :D], loss.cpu().numpy()


@pytest.mark.parametrize('name', TRAIN_UNITS)
def test_local_train_unit_golden(amd, name):
    d = load(name)
    W, loss = _train_via_abi(amd, [d['X']], [d['y']], d['W0'], float(d['lr']), int(d['epoch']),
                             int(d['batch_size']), bool(d['prox']), float(d['mu']), bool(d['reg']), float(d['lam']),
                             chained=True, seed=int(d['seed']))
    assert np.abs(W[0] - d['W']).max() <= 2e-6 * np.abs(d['W']).max()
    assert abs(loss[0] - float(d['loss'])) <= 2e-6 * max(1.0, abs(float(d['loss'])))


def _rand_clients(rs, sizes, D, C):
    Xs = [(np.cos(rs.normal(size=(n, D))) / np.sqrt(D)).astype(np.float32) for n in sizes]
    ys = [rs.randint(0, C, size=n).astype(np.int64) for n in sizes]
    return Xs, ys


@pytest.mark.parametrize('D,C,B,sizes,prox,reg', [
    (200, 10, 32, [64, 33, 1, 7, 96], True, True),        # D not a multiple of 64, tail batches 1 and 7
    (130, 26, 32, [40, 65], False, True),                 # C > 16 (two class tiles), 'letter'-like
    (64, 3, 16, [50, 17], True, False),                   # B = 16 (one row tile)
    (96, 7, 64, [130, 64, 5], True, True),                # B = 64 (four row tiles)
    (2048, 10, 32, [512, 100], True, True),               # benchmark width (weights resident in LDS)
    (4000, 10, 32, [70, 33], True, True),                 # weights too large for LDS: global-memory path
])
@pytest.mark.parametrize('mode', ['chained-1wg', 'chained-auto', 'parallel-1wg', 'parallel-auto'])
def test_local_train_vs_oracle(amd, D, C, B, sizes, prox, reg, mode):
    """chained = reference semantics (client i starts from client i-1's result); *-1wg = one
    workgroup per client (chained: one workgroup walks the chain); *-auto = the planner's
    choice (a group of G workgroups splits each client's features and exchanges partial
    logits every step, whenever the shape allows; chained: one group walks the chain)."""
    rs = np.random.RandomState(D + C + B)
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    lr, mu, lam, E = 0.4, 0.03, 0.002, 2
    chained = mode.startswith('chained')
    W, loss = _train_via_abi(amd, Xs, ys, W0, lr, E, B, prox, mu, reg, lam, chained, seed=11,
                             split=1 if mode.endswith('1wg') else None)
    torch.manual_seed(11)   # the oracle draws the same passes (client-major, epoch-minor)
    start = W0
    for j, (X, y) in enumerate(zip(Xs, ys)):
        Wr, lref = O.train_client(X, y, start, lr, E, B, prox, mu, reg, lam)
        tol = 2e-5 * max(1.0, np.abs(Wr).max())
        assert np.abs(W[j] - Wr).max() <= tol, (j, np.abs(W[j] - Wr).max())
        assert abs(loss[j] - lref) <= 2e-5 * max(1.0, abs(lref))
        if chained:
            start = Wr


@pytest.mark.parametrize('G', [2, 4, 8, 16])
@pytest.mark.parametrize('chained', [True, False])
@pytest.mark.parametrize('prox', [True, False])
def test_local_train_split_widths(amd, G, chained, prox):
    """Every group width of the split-client kernel, chained (one group walks the chain) and
    parallel, against the oracle: D = 1000 (16 tiles, the last one ragged), C = 10, tail
    batches of 1 and 7 rows, and a client with no rows (its result is its start)."""
    rs = np.random.RandomState(G + 10 * chained + 100 * prox)
    D, C, B, E = 1000, 10, 32, 2
    sizes = [65, 33, 0, 7, 96, 40]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    lr, mu, lam = 0.4, 0.03, 0.002
    W, loss = _train_via_abi(amd, Xs, ys, W0, lr, E, B, prox, mu, True, lam, chained, seed=3, split=G)
    assert _train_via_abi.last_G == G
    torch.manual_seed(3)
    start = W0
    for j, (X, y) in enumerate(zip(Xs, ys)):
        Wr, lref = O.train_client(X, y, start, lr, E, B, prox, mu, True, lam)
        assert np.abs(W[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), (j, np.abs(W[j] - Wr).max())
        assert abs(loss[j] - lref) <= 2e-5 * max(1.0, abs(lref)), j
        if chained:
            start = Wr


@pytest.mark.parametrize('G,D', [(2, 2048), (4, 1000), (16, 4096)])
@pytest.mark.parametrize('chained', [False, True])
def test_local_train_split_slices(amd, G, D, chained):
    """The group kernel's row stream (each wave's next rows interleaved into its backward)
    against the oracle, with full slices (16 tiles per workgroup: the straight-line
    interleaved backward) and ragged ones (D = 1000), FedProx + ridge, chained and parallel."""
    sched = 2
    rs = np.random.RandomState(sched + 10 * G + chained)
    C, B, E = 7, 32, 2
    sizes = [70, 0, 33, 64, 9]
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    lr, mu, lam = 0.4, 0.03, 0.002
    W, loss = _train_via_abi(amd, Xs, ys, W0, lr, E, B, True, mu, True, lam, chained, seed=5, split=G)
    assert _train_via_abi.last_G == G
    torch.manual_seed(5)
    start = W0
    for j, (X, y) in enumerate(zip(Xs, ys)):
        Wr, lref = O.train_client(X, y, start, lr, E, B, True, mu, True, lam)
        assert np.abs(W[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), (j, np.abs(W[j] - Wr).max())
        assert abs(loss[j] - lref) <= 2e-5 * max(1.0, abs(lref)), j
        if chained:
            start = Wr


@pytest.mark.parametrize('N,G', [(300, 2), (700, 4)])
def test_local_train_persistent_groups(amd, N, G):
    """More clients than groups (N * G > CUs): every group walks several clients in the
    snake order over the LPT list, the next client's first rows streaming in during the
    previous client's last step.  All clients against the oracle."""
    rs = np.random.RandomState(N)
    D, C, B, E = 256, 6, 32, 2
    sizes = list(rs.randint(1, 90, size=N))
    Xs, ys = _rand_clients(rs, sizes, D, C)
    W0 = (rs.normal(size=(C, D)) * 0.1).astype(np.float32)
    W, loss = _train_via_abi(amd, Xs, ys, W0, 0.3, E, B, True, 0.02, True, 0.001, False, seed=9, split=G)
    torch.manual_seed(9)
    for j, (X, y) in enumerate(zip(Xs, ys)):
        Wr, lref = O.train_client(X, y, W0, 0.3, E, B, True, 0.02, True, 0.001)
        assert np.abs(W[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), j
        assert abs(loss[j] - lref) <= 2e-5 * max(1.0, abs(lref)), j


def test_split_handoff_timeout_raises(amd):
    """A timed-out partner hand-off is reported, not silently absorbed: fs_tuning.inject_timeout
    (the test knob) makes the launch set its workspace error word; check_errors raises and
    clears it, and the next launch is clean."""
    rs = np.random.RandomState(1)
    Xs, ys = _rand_clients(rs, [40, 70], 256, 4)
    W0 = (rs.normal(size=(4, 256)) * 0.1).astype(np.float32)
    with amd.lib.tuning(inject_timeout=1):
        with pytest.raises(amd.lib.FedsimError, match='timed out'):
            _train_via_abi(amd, Xs, ys, W0, 0.3, 2, 32, False, 0.0, False, 0.0, False, seed=1, split=2)
    _train_via_abi(amd, Xs, ys, W0, 0.3, 2, 32, False, 0.0, False, 0.0, False, seed=1, split=2)


def test_mix_solve_timeout_raises(amd):
    """Same for the multi-CU p-solve, through the FedAMW drop-in: results() raises
    FedsimError instead of returning NaN mixture weights."""
    rs = np.random.RandomState(2)
    N, D, C = 300, 64, 4
    Xs, ys = _rand_clients(rs, list(rs.randint(5, 20, size=N)), D, C)
    Xv = (np.cos(rs.normal(size=(64, D))) / np.sqrt(D)).astype(np.float32)
    yv = rs.randint(0, C, size=64).astype(np.int64)
    T = torch.from_numpy
    with amd.lib.tuning(inject_timeout=1), pytest.raises(amd.lib.FedsimError, match='fs_mix_solve'):
        amd.tools.FedAMW([T(x) for x in Xs], [T(y) for y in ys], T(Xv), T(yv), _dl(Xv, yv), 'classification', C,
                         D, 0.5, 1, 32, False, 0.0, True, 1e-3, 1, 0.01, clients='parallel', verbose=False)


def test_aggregate_bitexact_and_chunked(amd):
    rs = np.random.RandomState(0)
    N, C, D = 37, 10, 2048
    Ws = rs.normal(size=(N, C, D)).astype(np.float32)
    p = rs.dirichlet(np.ones(N)).astype(np.float32)
    ref = O.aggregate(list(Ws), p)
    dev = torch.device('cuda')
    Wd = torch.from_numpy(Ws).to(dev)
    pd = torch.from_numpy(p).to(dev)
    agg1 = amd.engine.Aggregator(N, C, D, dev, chunks=1)
    out = torch.empty(C, D, device=dev)
    agg1.run(Wd, pd, out)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)      # bitwise the reference's fold
    agg8 = amd.engine.Aggregator(N, C, D, dev, chunks=8)
    agg8.run(Wd, pd, out)
    assert np.abs(out.cpu().numpy() - ref).max() <= 1e-6 * np.abs(ref).max()


@pytest.mark.parametrize('N', [1, 9, 15, 16, 37, 100, 300, 512, 513, 1250])
def test_aggregate_auto_forms(amd, N):
    """fs_aggregate with the shape's own choice (chunks = 0): one launch with in-workgroup
    sub-range folds for 16 <= N <= 512 (round 5), the two-launch chunked fold above, and the
    reference's exact single fold below 16 clients -- bitwise there; elsewhere only the order of
    the N products' fp32 sum differs, so each element lies within the classical bound of two
    recursive summations of the same terms, 2 (N - 1) u sum_j |p_j W_j| (u = 2^-24), of the
    reference's fold."""
    rs = np.random.RandomState(N)
    C, D = 10, 2048
    Ws = rs.normal(size=(N, C, D)).astype(np.float32)
    p = rs.dirichlet(np.ones(N)).astype(np.float32)
    ref = O.aggregate(list(Ws), p)
    dev = torch.device('cuda')
    agg = amd.engine.Aggregator(N, C, D, dev, chunks=0)
    out = torch.full((C, D), float('nan'), device=dev)
    agg.run(torch.from_numpy(Ws).to(dev), torch.from_numpy(p).to(dev), out)
    got = out.cpu().numpy()
    if N < 16:
        np.testing.assert_array_equal(got, ref)
    else:
        S = np.abs(p.astype(np.float64)[:, None, None] * Ws).sum(0)
        bound = 2.0 * (N - 1) * 2.0 ** -24 * S
        assert (np.abs(got.astype(np.float64) - ref) <= bound).all(), np.max(np.abs(got - ref) / bound)


def test_eval_unit_golden(amd):
    d = load('unit_test')
    dev = torch.device('cuda')
    ev = amd.engine.Evaluator(torch.from_numpy(d['X']), torch.from_numpy(d['y']), d['X'].shape[1], d['W'].shape[0],
                              dev)
    W = torch.zeros(d['W'].shape[0], ev.f.ld, device=dev)
    W[:, :d['X'].shape[1]] = torch.from_numpy(d['W'])
    out = torch.empty(2, dtype=torch.float64, device=dev)
    ev.run(W, out)
    loss, acc = out.cpu().numpy()
    assert abs(loss - float(d['loss'])) <= 1e-5 * max(1, abs(float(d['loss'])))
    assert abs(acc - float(d['acc'])) <= 100.0 / len(d['y']) + 1e-4


@pytest.mark.parametrize('N,C,nv,Bv', [
    (10, 2, 203, 16),       # config 1 shape: the one-wave binary solver (C <= 2)
    (16, 4, 77, 16),        # one wave, every lane's class real, ragged last batch
    (5, 3, 40, 7),          # one wave, Bv < 16 (idle rows), N not a multiple of 4
    (1, 2, 33, 16),         # one client
    (100, 10, 517, 16),     # config 2 shape: NK=2, CP=16 (10 loaded classes)
    (200, 4, 301, 16),      # NK=4, CP=4 (at lr 0.1: lr 0.5 makes this p-SGD ill-conditioned, fp32 vs fp64 2e-4)
    (60, 8, 33, 9),         # CP=8, 9-row batches: the second row of every wave idles
    (64, 7, 130, 16),       # N exactly one lane per client
    (129, 3, 77, 8),        # NK=4, Bv < 16 (idle waves), ragged last batch
    (37, 20, 90, 16),       # C > 16: CP=32, 2-deep ring
    (23, 5, 211, 24),       # Bv > 16: LDS-staged solver
    (19, 24, 70, 20),       # Bv > 16 and C > 16: global-memory solver
    (300, 4, 60, 16),       # N > 256: multi-CU solver
])
def test_mix_solve_variants(amd, N, C, nv, Bv, lr=0.5):
    """fs_mix_solve (every solver variant it selects) vs the oracle's p-SGD, 2 rounds x 2 epochs.
    Every case is well-conditioned: the fp32 oracle is within 5e-6 of an fp64 run of it."""
    if (N, C, nv) == (200, 4, 301):
        lr = 0.1
    rs = np.random.RandomState(N + C + nv)
    D = 64
    Ws = (rs.normal(size=(N, C, D)) * 0.5).astype(np.float32)
    Xv = (np.cos(rs.normal(size=(nv, D))) / np.sqrt(D)).astype(np.float32)
    yv = rs.randint(0, C, size=nv).astype(np.int64)
    p0 = rs.dirichlet(np.ones(N)).astype(np.float32)
    dev = torch.device('cuda')
    mix = amd.engine.Mixture(torch.from_numpy(Xv), torch.from_numpy(yv), D, C, N, Bv, torch.from_numpy(p0), dev)
    Wd = torch.zeros(N, C, mix.f.ld, device=dev)
    Wd[:, :, :D] = torch.from_numpy(Ws)
    pr, br = p0, None
    for rnd in range(2):
        torch.manual_seed(70 + rnd)
        mix.solve(Wd, amd.rng.draw_pass_seeds(2), lr)
        torch.cuda.synchronize()
        mix.check_errors()
        torch.manual_seed(70 + rnd)
        pr, br = O.mixture_solve(list(Ws), Xv, yv, pr, br, lr, 2, batch_size=Bv)
        ep = float(np.abs(mix.p.cpu().numpy() - pr).max() / np.abs(pr).max())
        eb = float(np.abs(mix.buf.cpu().numpy() - br).max() / np.abs(br).max())
        assert ep <= 1e-5 and eb <= 1e-4, (rnd, ep, eb)


@pytest.mark.parametrize('N,C,Bv,solver', [(10, 2, 16, 'bin'), (16, 4, 16, 'wave'), (17, 4, 16, 'quad'),
                                           (16, 2, 16, 'bin'), (17, 2, 16, 'quad'), (16, 2, 17, 'staged'),
                                           (10, 5, 16, 'quad'), (100, 10, 16, 'quad'), (64, 16, 16, 'quad'),
                                           (37, 20, 16, 'reg'), (129, 3, 16, 'reg2'), (200, 4, 16, 'reg2'),
                                           (1000, 10, 16, 'qmc'), (300, 4, 16, 'qmc'), (1100, 16, 16, 'mc'),
                                           (23, 5, 24, 'staged')])
def test_mix_solve_auto_choice(amd, N, C, Bv, solver):
    """The solver fs_mix_solve picks by shape."""
    rs = np.random.RandomState(N)
    nv, D = 40, 64
    Xv = (np.cos(rs.normal(size=(nv, D))) / np.sqrt(D)).astype(np.float32)
    yv = rs.randint(0, C, size=nv).astype(np.int64)
    p0 = np.full(N, 1.0 / N, np.float32)
    dev = torch.device('cuda')
    mix = amd.engine.Mixture(torch.from_numpy(Xv), torch.from_numpy(yv), D, C, N, Bv, torch.from_numpy(p0), dev)
    Wd = torch.zeros(N, C, mix.f.ld, device=dev)
    torch.manual_seed(0)
    mix.solve(Wd, amd.rng.draw_pass_seeds(1), 0.1)
    torch.cuda.synchronize()
    mix.check_errors()
    assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == solver


@pytest.mark.parametrize('N,C,nv,Bv', [
    (100, 10, 517, 16),     # config 2 shape: S = 8, K = 13 workgroups, one hop
    (1000, 10, 97, 16),     # config 5 client count: S = 32, K = 32, two hops
    (300, 4, 60, 16),       # S = 16, ragged last slice
    (129, 3, 77, 8),        # Bv < 16: idle rows, ragged last batch (S = 16)
    (48, 16, 99, 16),       # C = 16: every class slot real
    (2000, 2, 45, 16),      # S = 64, K = 32
    (5, 2, 40, 16),         # one workgroup (K = 1)
    (1100, 16, 40, 16),     # S = 64, C = 16
])
def test_mix_solve_multi_cu(amd, N, C, nv, Bv):
    """fs_mix_solve's multi-CU solver (clients split over K workgroups of S, partial-logit
    exchange every step: one hop at S = 8, reduce-scatter + all-gather above) vs the oracle's
    p-SGD, 2 rounds x 2 epochs."""
    # (at N >= 1000, lr_p = 0.5 drives p to |p| ~ 10 within a few steps, where any two fp32
    # summation orders of the 10^4-term logits drift past 1e-5; the configs use lr_p ~ 1e-3)
    with amd.lib.tuning(mix_solver='mc'):
        test_mix_solve_variants(amd, N, C, nv, Bv, lr=0.05 if N >= 1000 else 0.5)
    mode = amd.lib.lib().fs_mix_solve_last_mode()
    assert mode == 2, mode             # the multi-CU solver ran (a timed-out spin raises in check_errors)


@pytest.mark.parametrize('h,lc', [(-1, 0), (16, 0), (16, 8), (16, 4)])
@pytest.mark.parametrize('N,C,nv,Bv', [
    (1000, 10, 97, 16),     # config 5 client count: K = 16 workgroups of 64 clients (lc = 8: 8 of 128)
    (300, 4, 60, 16),       # K = 3, ragged last slice
    (129, 3, 77, 8),        # K = 2, Bv < 16, ragged last batch
    (2000, 2, 45, 16),      # K = 16
    (1000, 16, 40, 16),     # C = 16: 64 clients per workgroup, K = 16
    (200, 10, 133, 16),     # K = 2
])
def test_mix_solve_qmc(amd, N, C, nv, Bv, h, lc):
    """fs_mix_solve's multi-CU quarter-wave solver (clients over K workgroups, one exchange of
    the partial logits per step; without / with L2 prefetch helpers; lc: the 4-clients-per-
    lane instance forced where the shape picks 8, 8 forced where it picks 4) vs the oracle's
    p-SGD."""
    if lc == 4 and (N + 3) // 4 * 4 > 16 * 64:
        pytest.skip('K = ceil(N / 64) > 16 workgroups: not a qmc shape at 4 clients per lane')
    if lc == 8 and C > 10:
        pytest.skip('8 clients per lane: C <= 10 only')
    with amd.lib.tuning(mix_solver='qmc', mix_prefetch=h, mix_qmc_lane_clients=lc):
        test_mix_solve_variants(amd, N, C, nv, Bv, lr=0.05 if N >= 1000 else 0.5)   # (see test_mix_solve_multi_cu)
    assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == 'qmc'


@pytest.mark.parametrize('N,C,nv', [(1000, 10, 97), (300, 4, 60)])
def test_mix_solve_qmc_poll_delay_bitwise(amd, N, C, nv):
    """The first-poll delay (fs_tuning.mix_poll_delay: none, by shape, a long one) changes only
    when the polls go out: p and the momentum buffer are bitwise the same."""
    rs = np.random.RandomState(N + 3)
    D = 64
    Xv = torch.from_numpy((np.cos(rs.normal(size=(nv, D))) / np.sqrt(D)).astype(np.float32))
    yv = torch.from_numpy(rs.randint(0, C, size=nv).astype(np.int64))
    p0 = torch.from_numpy(rs.dirichlet(np.ones(N)).astype(np.float32))
    Ws = torch.from_numpy((rs.normal(size=(N, C, D)) * 0.5).astype(np.float32))
    dev = torch.device('cuda')
    out = []
    for delay in (-1, 0, 40):
        with amd.lib.tuning(mix_solver='qmc', mix_poll_delay=delay):
            mix = amd.engine.Mixture(Xv, yv, D, C, N, 16, p0, dev)
            Wd = torch.zeros(N, C, mix.f.ld, device=dev)
            Wd[:, :, :D] = Ws
            for rnd in range(2):
                torch.manual_seed(30 + rnd)
                mix.solve(Wd, amd.rng.draw_pass_seeds(3), 0.05)
            torch.cuda.synchronize()
            mix.check_errors()
        assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == 'qmc'
        out.append((mix.p.cpu().clone(), mix.buf.cpu().clone()))
    for o in out[1:]:
        assert torch.equal(out[0][0], o[0]) and torch.equal(out[0][1], o[1])


def test_mix_solve_qmc_timeout_raises(amd):
    """A timed-out exchange of the multi-CU quarter-wave solver sets the error word; the next
    solve is clean."""
    with amd.lib.tuning(mix_solver='qmc'):
        with amd.lib.tuning(inject_timeout=1), pytest.raises(amd.lib.FedsimError):
            test_mix_solve_variants(amd, 300, 4, 60, 16)
        test_mix_solve_variants(amd, 300, 4, 60, 16)


@pytest.mark.parametrize('N,C,nv,Bv', [
    (100, 10, 517, 16),     # config 2 shape: NK = 8, CL = 10
    (10, 2, 203, 16),       # config 1 shape: NK = 4, CL = 2
    (16, 4, 77, 16),        # ragged last batch
    (5, 3, 40, 7),          # Bv = 7: idle row groups, N not a multiple of 4
    (1, 2, 33, 16),         # one client
    (60, 8, 33, 9),         # NK = 4, CL = 8, 9-row batches
    (64, 7, 130, 16),       # N = 64: every lane's clients real
    (37, 16, 90, 16),       # C = 16: every class slot real, 2-deep ring
    (128, 10, 77, 8),       # N = 128 (NK = 8 exactly), Bv = 8
    (65, 9, 211, 16),       # NK = 8, C = 9 < CL = 10 (class padding), ragged chunks
])
def test_mix_solve_quad(amd, N, C, nv, Bv):
    """fs_mix_solve's quarter-wave solver (4 batch rows per wave, 16 lanes per row; default
    issue split and L2 prefetch helpers) vs the oracle's p-SGD, 2 rounds x 2 epochs."""
    with amd.lib.tuning(mix_solver='quad'):
        test_mix_solve_variants(amd, N, C, nv, Bv)
    assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == 'quad'


@pytest.mark.parametrize('N,C,nv,Bv', [
    (10, 2, 203, 16),       # config 1 shape: 2 of each lane's 4 chunks past ldN = 12 read zeros
    (16, 2, 77, 16),        # every chunk real, ragged last batch
    (5, 2, 40, 7),          # Bv = 7: idle rows, N not a multiple of 4 (ldN = 8: half h = 1 all padding)
    (1, 2, 33, 16),         # one client
    (13, 2, 1000, 16),      # 63 steps per epoch: ring turns + a 7-step tail
    (8, 2, 16, 16),         # one batch per epoch (total = 2 steps: tail only)
])
@pytest.mark.parametrize('exact', [0, 1])
def test_mix_solve_bin(amd, N, C, nv, Bv, exact):
    """fs_mix_solve's one-wave binary solver (lane = row x class x client half; default
    v_exp / v_rcp softmax and torch's libm form) vs the oracle's p-SGD, 2 rounds x 2 epochs."""
    with amd.lib.tuning(mix_solver='bin', mix_exact_softmax=exact):
        test_mix_solve_variants(amd, N, C, nv, Bv)
    assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == 'bin'


@pytest.mark.parametrize('N,C,nv,Bv', [(100, 10, 517, 16), (60, 8, 33, 9), (37, 16, 90, 16)])
def test_mix_solve_quad_libm_softmax(amd, N, C, nv, Bv):
    """The quarter-wave solver with torch's softmax form on libm expf / logf
    (fs_tuning.mix_exact_softmax; the default is v_exp / v_rcp) vs the oracle."""
    with amd.lib.tuning(mix_solver='quad', mix_exact_softmax=1):
        test_mix_solve_variants(amd, N, C, nv, Bv)
    assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == 'quad'


@pytest.mark.parametrize('h,lead', [(1, 1), (3, 16), (7, 64)])
@pytest.mark.parametrize('N,C,nv,Bv', [
    (100, 10, 517, 16),     # config 2 shape
    (64, 7, 130, 16),       # NK = 1
    (129, 3, 77, 8),        # NK = 4, Bv < 16: idle waves in the helpers too, ragged last batch
])
@pytest.mark.parametrize('solver', ['reg', 'quad'])
def test_mix_solve_prefetch_helpers(amd, N, C, nv, Bv, h, lead, solver):
    """The single-CU solvers with L2 prefetch helper workgroups (fs_tuning.mix_prefetch): the
    helpers only load, so p and the momentum buffer are bitwise those of the solver alone, and
    match the oracle's p-SGD."""
    if solver == 'quad' and N > 128:
        pytest.skip('the quarter-wave solver covers N <= 128')
    rs = np.random.RandomState(N + nv)
    D = 64
    Xv = torch.from_numpy((np.cos(rs.normal(size=(nv, D))) / np.sqrt(D)).astype(np.float32))
    yv = torch.from_numpy(rs.randint(0, C, size=nv).astype(np.int64))
    p0 = torch.from_numpy(rs.dirichlet(np.ones(N)).astype(np.float32))
    Ws = torch.from_numpy((rs.normal(size=(N, C, D)) * 0.5).astype(np.float32))
    dev = torch.device('cuda')
    out = []
    for helpers in (-1, h):
        with amd.lib.tuning(mix_solver=solver, mix_prefetch=helpers, mix_prefetch_lead=lead):
            mix = amd.engine.Mixture(Xv, yv, D, C, N, Bv, p0, dev)
            Wd = torch.zeros(N, C, mix.f.ld, device=dev)
            Wd[:, :, :D] = Ws
            for rnd in range(2):
                torch.manual_seed(90 + rnd)
                mix.solve(Wd, amd.rng.draw_pass_seeds(3), 0.5)
            torch.cuda.synchronize()
            mix.check_errors()
        assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == solver
        out.append((mix.p.cpu().clone(), mix.buf.cpu().clone()))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    with amd.lib.tuning(mix_solver=solver, mix_prefetch=h):
        test_mix_solve_variants(amd, N, C, nv, Bv)


@pytest.mark.parametrize('h', [-1, 4])
@pytest.mark.parametrize('N,C,nv,Bv', [
    (100, 10, 517, 16),     # config 2 shape: ragged last batch, lanes past ldN (column-0 reads, p = 0)
    (128, 10, 77, 8),       # every lane's clients real, Bv = 8 (idle row groups)
    (65, 9, 211, 16),       # C = 9 < CL = 10 (class padding in the LDS ring)
    (97, 10, 16, 16),       # one batch per epoch: total = 3 steps (the loaders' tail)
])
def test_mix_solve_quad_loader_waves(amd, N, C, nv, Bv, h):
    """The quarter-wave solver with loader waves (fs_tuning.mix_quad_loaders, default at config
    2's instance: 4 waves stream the late classes' Z rows into a 2-slot LDS ring) is bitwise the
    quarter-wave solver without them, with and without L2 helpers, and matches the oracle."""
    rs = np.random.RandomState(N + nv + 7)
    D = 64
    Xv = torch.from_numpy((np.cos(rs.normal(size=(nv, D))) / np.sqrt(D)).astype(np.float32))
    yv = torch.from_numpy(rs.randint(0, C, size=nv).astype(np.int64))
    p0 = torch.from_numpy(rs.dirichlet(np.ones(N)).astype(np.float32))
    Ws = torch.from_numpy((rs.normal(size=(N, C, D)) * 0.5).astype(np.float32))
    dev = torch.device('cuda')
    out = []
    for loaders in (-1, 0):
        with amd.lib.tuning(mix_solver='quad', mix_prefetch=h, mix_quad_loaders=loaders):
            mix = amd.engine.Mixture(Xv, yv, D, C, N, Bv, p0, dev)
            Wd = torch.zeros(N, C, mix.f.ld, device=dev)
            Wd[:, :, :D] = Ws
            for rnd in range(2):
                torch.manual_seed(70 + rnd)
                mix.solve(Wd, amd.rng.draw_pass_seeds(3), 0.5)
            torch.cuda.synchronize()
            mix.check_errors()
        assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == 'quad'
        out.append((mix.p.cpu().clone(), mix.buf.cpu().clone()))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    with amd.lib.tuning(mix_solver='quad', mix_prefetch=h):
        test_mix_solve_variants(amd, N, C, nv, Bv)


@pytest.mark.parametrize('solver,N,C', [('global', 100, 10), ('global', 300, 4), ('staged', 100, 10),
                                        ('mc', 1000, 7), ('reg', 100, 10), ('reg', 10, 2), ('wave', 10, 2),
                                        ('quad', 10, 2), ('reg2', 100, 10)])
def test_mix_solve_forced_fallbacks(amd, solver, N, C):
    """The solvers the auto choice does not take at these shapes, forced through fs_tuning."""
    with amd.lib.tuning(mix_solver=solver):
        test_mix_solve_variants(amd, N, C, 133, 16, lr=0.05 if N >= 1000 else 0.5)   # (see test_mix_solve_multi_cu)
    assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == solver


@pytest.mark.parametrize('N,C,D,nv', [(1, 1, 64, 1), (3, 2, 64, 255), (23, 5, 192, 257), (100, 10, 2048, 700),
                                      (130, 7, 320, 513), (300, 4, 128, 1000), (998, 4, 64, 4097)])
def test_mix_z_shapes(amd, N, C, D, nv):
    """fs_mix_z (mix_z.hip: 128- or 256-row x 128 tiles, K-steps of 32, LDS-DMA images) against
    fp64 on ragged shapes: row tails (n_val mod 128 / 256), column tails (C * ldN mod 128),
    padding clients (N mod 4), the shortest K (ld = 64: one loop iteration); the last shape
    (544 tiles of 256 rows) takes the 256-row form, the others the 128-row form; padding columns
    exactly 0 and nothing written past Z (a guard row after it)."""
    rs = np.random.RandomState(N + nv)
    ld = (D + 63) // 64 * 64
    ldN = (N + 3) // 4 * 4
    dev = torch.device('cuda')
    X = torch.zeros(nv, ld, device=dev)
    X[:, :D] = torch.from_numpy((np.cos(rs.normal(size=(nv, D))) / np.sqrt(D)).astype(np.float32))
    W = torch.zeros(N, C, ld, device=dev)
    W[:, :, :D] = torch.from_numpy((rs.normal(size=(N, C, D)) * 0.3).astype(np.float32))
    Zb = torch.full((nv + 1, C * ldN), 7.0, device=dev)
    L = amd.lib
    L.check(L.lib().fs_mix_z(L.ptr(W), L.ptr(X), ld, N, C, nv, L.ptr(Zb), L.stream_ptr()), 'fs_mix_z')
    torch.cuda.synchronize()
    Z = Zb[:nv].view(nv, C, ldN).double().cpu().numpy()
    Xd, Wd = X[:, :D].double().cpu().numpy(), W[:, :, :D].double().cpu().numpy()
    ref = np.einsum('vd,ncd->vcn', Xd, Wd)
    scale = np.einsum('vd,ncd->vcn', np.abs(Xd), np.abs(Wd))
    assert (np.abs(Z[:, :, :N] - ref) <= 2e-6 * scale + 1e-30).all()
    assert (Z[:, :, N:] == 0).all()
    assert (Zb[nv] == 7.0).all()


@pytest.mark.parametrize('N,blocks,C', [(304, 2, 10), (384, 4, 10), (1024, 8, 10), (520, 2, 13)])
def test_mix_solve_blocked_layout_bitwise(amd, N, blocks, C):
    """fs_mix_solve_blocked on the rank-blocked Z an all-gather leaves ([blocks][n_val][C][L],
    dist.allgather_z(blocked=True)) == fs_mix_solve on the same Z in solver order, BITWISE in p
    and the momentum buffer (same solver, same arithmetic, only the addresses differ), over two
    calls; shapes the blocked form does not read are refused with FS_EUNSUPPORTED."""
    rs = np.random.RandomState(N + blocks)
    D, nv, ep = 64, 333, 3
    L = N // blocks
    dev = torch.device('cuda')
    Xv = torch.from_numpy((np.cos(rs.normal(size=(nv, D))) / np.sqrt(D)).astype(np.float32))
    yv = torch.from_numpy(rs.randint(0, C, size=nv).astype(np.int64))
    p0 = torch.from_numpy(rs.dirichlet(np.ones(N)).astype(np.float32))
    W = torch.from_numpy((rs.normal(size=(N, C, D)) * 0.5).astype(np.float32)).to(dev)
    std = amd.engine.Mixture(Xv, yv, D, C, N, 16, p0, dev)
    blk = amd.engine.Mixture(Xv, yv, D, C, N, 16, p0, dev)
    assert blk.blocked_covers(ep)
    blk.blocks = blocks
    Wd = torch.zeros(N, C, std.f.ld, device=dev)
    Wd[:, :, :D] = W
    L_ = amd.lib
    L_.check(L_.lib().fs_mix_z(L_.ptr(Wd), L_.ptr(std.f.phi), std.f.ld, N, C, nv, L_.ptr(std.Z), L_.stream_ptr()), 'z')
    # the blocked image: rank block r holds columns r*L .. r*L+L-1 of every class
    blk.Z.view(-1).copy_(std.Z.view(nv, C, blocks, L).permute(2, 0, 1, 3).reshape(-1))
    for call in range(2):
        torch.manual_seed(70 + call)
        seeds = amd.rng.draw_pass_seeds(ep)
        std.solve(None, seeds, 0.01, z=False)
        blk.solve(None, seeds, 0.01, z=False)
        torch.cuda.synchronize()
        assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] == 'qmc'
        assert torch.equal(std.p, blk.p) and torch.equal(std.buf, blk.buf), call
    assert bool(torch.isfinite(std.p).all()) and not torch.equal(std.p, p0.to(dev))
    small = amd.engine.Mixture(Xv, yv, D, C, 200, 16, torch.full((200,), 0.005), dev)
    assert not small.blocked_covers(ep)                 # N <= 256: not the qmc solver's shape
    small.blocks = 2
    with pytest.raises(amd.lib.FedsimError, match='qmc solver only'):
        small.solve(None, amd.rng.draw_pass_seeds(1), 0.01, z=False)


def test_mix_z_and_solve_vs_oracle(amd):
    rs = np.random.RandomState(3)
    N, C, D, nv = 23, 5, 192, 211
    Ws = (rs.normal(size=(N, C, D)) * 0.3).astype(np.float32)
    Xv = (np.cos(rs.normal(size=(nv, D))) / np.sqrt(D)).astype(np.float32)
    yv = rs.randint(0, C, size=nv).astype(np.int64)
    p0 = rs.dirichlet(np.ones(N)).astype(np.float32)
    dev = torch.device('cuda')
    mix = amd.engine.Mixture(torch.from_numpy(Xv), torch.from_numpy(yv), D, C, N, 16, torch.from_numpy(p0), dev)
    Wd = torch.zeros(N, C, mix.f.ld, device=dev)
    Wd[:, :, :D] = torch.from_numpy(Ws)
    for rnd in range(2):
        torch.manual_seed(40 + rnd)
        seeds = amd.rng.draw_pass_seeds(3)
        mix.solve(Wd, seeds, 0.05)
        torch.cuda.synchronize()
        Zref = np.einsum('ncd,vd->vcn', Ws, Xv).reshape(nv, C * N)
        Zgot = mix.Z.view(nv, C, mix.ldN).cpu().numpy()
        assert (Zgot[:, :, N:] == 0).all()                       # padding clients
        assert np.abs(Zgot[:, :, :N].reshape(nv, C * N) - Zref).max() <= 1e-5 * np.abs(Zref).max()
        torch.manual_seed(40 + rnd)
        if rnd == 0:
            pr, br = O.mixture_solve(list(Ws), Xv, yv, p0, None, 0.05, 3)
        else:
            pr, br = O.mixture_solve(list(Ws), Xv, yv, pr, br, 0.05, 3)
        ep = float(np.abs(mix.p.cpu().numpy() - pr).max() / np.abs(pr).max())
        eb = float(np.abs(mix.buf.cpu().numpy() - br).max() / np.abs(br).max())
        assert ep <= 1e-5 and eb <= 1e-4, (rnd, ep, eb)


# ----------------------------------------------------------------------------- full size


def test_fullsize_parallel_properties(amd):
    """Benchmark shape (config 2: 100 clients x 512 rows, D=2048, C=10): size-independent
    properties of the parallel round."""
    rs = np.random.RandomState(5)
    N, n, D, C, B, E = 100, 512, 2048, 10, 32, 2
    dev = torch.device('cuda')
    X = torch.randn(N * n, D, device=dev).cos_().mul_(D ** -0.5)
    y = torch.randint(0, C, (N * n,), device=dev)
    Xs = list(X.split(n))
    ys = [v.cpu() for v in y.split(n)]
    feats = amd.engine.Features(Xs, ys, D, dev)
    tr = amd.engine.LocalTrainer(feats, C, B, E)
    G = tr.G
    torch.manual_seed(1)
    seeds = amd.rng.draw_pass_seeds(N * E)
    tr.upload_perms(seeds)
    W0 = torch.zeros(C, D, device=dev)
    W0.normal_(0, 0.05)
    # (1) lr = 0 leaves every client at the start exactly
    W, _ = tr.run(W0, 0.0, True, 0.01, True, 0.001, False)
    assert torch.equal(W, W0.expand_as(W))
    # (2) clients are independent: one client alone == the same client inside the full batch (bitwise)
    W, loss = tr.run(W0, 0.3, True, 0.01, True, 0.001, False)
    Wfull = W.clone()
    j = 37
    f1 = amd.engine.Features([Xs[j]], [ys[j]], D, dev)
    t1 = amd.engine.LocalTrainer(f1, C, B, E, split=G)     # same slicing as in the full batch
    t1.upload_perms(seeds.reshape(N, E)[j])
    W1, l1 = t1.run(W0, 0.3, True, 0.01, True, 0.001, False)
    assert torch.equal(W1[0], Wfull[j]) and float(l1[0]) == float(loss[j])
    # (3) spot-check two clients against the oracle at full width
    torch.cuda.synchronize()
    for j in (0, 99):
        g_state = torch.get_rng_state()
        # replay this client's two passes through the oracle's RNG path
        torch.manual_seed(1)
        torch.empty(2 * E * j, dtype=torch.int64).random_()
        Wr, lr_ = O.train_client(Xs[j].cpu().numpy(), ys[j].numpy(), W0.cpu().numpy(), 0.3, E, B, True, 0.01, True,
                                 0.001)
        torch.set_rng_state(g_state)
        assert np.abs(Wfull[j].cpu().numpy() - Wr).max() <= 2e-5 * np.abs(Wr).max()
        assert abs(float(loss[j]) - lr_) <= 2e-5 * max(1.0, abs(lr_))
    # (4) aggregation with equal p over identical models returns the model (to rounding)
    agg = amd.engine.Aggregator(N, C, D, dev)
    out = torch.empty(C, D, device=dev)
    p = torch.full((N,), 1.0 / N, device=dev)
    agg.run(W0.expand(N, C, D).contiguous(), p, out)
    assert (out - W0).abs().max().item() <= 1e-6 * W0.abs().max().item()


@pytest.mark.parametrize('n', [1, 2, 33, 63, 64, 65, 511, 512, 12800, 50000])
def test_device_randperm_matches_host_and_torch(amd, n):
    """fs_randperm_device (one lane per pass up to n = 64, the one-wave LDS path, and the
    global-memory path at n=50000) == host replay == torch."""
    dev = torch.device('cuda')
    torch.manual_seed(n)
    P = 5
    seeds = amd.rng.draw_pass_seeds(P)
    ns = np.full(P, n, np.int64)
    offs = np.arange(P, dtype=np.int64) * n
    sh = amd.engine.Shuffler(ns, offs, P * n, dev)
    out = sh.run(seeds)
    host = np.empty(P * n, np.int32)
    amd.rng.randperms(seeds, ns, offs, host)
    np.testing.assert_array_equal(out.cpu().numpy(), host)
    g = torch.Generator()
    g.manual_seed(int(seeds[-1]))
    np.testing.assert_array_equal(host[-n:], torch.randperm(n, generator=g).numpy())


def test_device_randperm_short_passes_mixed(amd):
    """The one-lane-per-pass replay (every pass <= 64 rows) over 300 passes of mixed lengths
    0..64 (several waves, a partial last wave, empty passes) == host replay == torch."""
    dev = torch.device('cuda')
    rs = np.random.RandomState(64)
    torch.manual_seed(64)
    P = 300
    seeds = amd.rng.draw_pass_seeds(P)
    ns = rs.randint(0, 65, size=P).astype(np.int64)
    ns[:3] = [64, 0, 1]
    offs = np.concatenate([[0], np.cumsum(ns)[:-1]]).astype(np.int64)
    total = int(ns.sum())
    sh = amd.engine.Shuffler(ns, offs, total, dev)
    out = sh.run(seeds)
    host = np.empty(total, np.int32)
    amd.rng.randperms(seeds, ns, offs, host)
    np.testing.assert_array_equal(out.cpu().numpy(), host)
    for i in (0, 2, 150, P - 1):
        g = torch.Generator()
        g.manual_seed(int(seeds[i]))
        np.testing.assert_array_equal(host[offs[i]:offs[i] + ns[i]], torch.randperm(int(ns[i]), generator=g).numpy())


@pytest.mark.parametrize('max_n,long_n', [(64, 65), (40, 41), (512, 600), (512, 50000)])
def test_device_randperm_contract_violation_raises(amd, max_n, long_n):
    """a pass longer than the launch's max_n (a caller breaking the
    fs_randperm_device contract) is written as the identity permutation -- memory-safe, both
    forms (one lane per pass at max_n <= 64, one wave per pass above) -- and sets the error word,
    so check_errors raises FedsimError instead of training on a silently unshuffled pass.  The
    passes that keep the contract are still torch's draws."""
    dev = torch.device('cuda')
    torch.manual_seed(max_n)
    P = 7
    seeds = amd.rng.draw_pass_seeds(P)
    ns = np.full(P, min(max_n, 33), np.int64)
    ns[3] = long_n
    offs = np.concatenate([[0], np.cumsum(ns)[:-1]]).astype(np.int64)
    total = int(ns.sum())
    sh = amd.engine.Shuffler(ns, offs, total, dev, max_n=max_n)
    out = sh.run(seeds).cpu().numpy()
    np.testing.assert_array_equal(out[offs[3]:offs[3] + long_n], np.arange(long_n, dtype=np.int32))
    ok = np.ones(P, bool)
    ok[3] = False
    host = np.empty(total, np.int32)
    amd.rng.randperms(seeds, ns, offs, host)
    for i in np.flatnonzero(ok):
        np.testing.assert_array_equal(out[offs[i]:offs[i] + ns[i]], host[offs[i]:offs[i] + ns[i]])
    with pytest.raises(amd.lib.FedsimError, match='longer than max_n'):
        sh.check_errors()
    sh.check_errors()                                   # cleared: a second check passes
    ns[3] = min(max_n, 33)                              # a clean launch on the same shuffler
    sh2 = amd.engine.Shuffler(ns, offs, total, dev, max_n=max_n)
    sh2.run(seeds)
    sh2.check_errors()


@pytest.mark.parametrize('N', [300, 1000])
def test_fedamw_dropin_many_clients_vs_oracle(amd, N):
    """The FedAMW drop-in end to end with more clients than any single-workgroup p-solver
    covers (the multi-CU solver runs inside the round), parallel clients, vs the oracle."""
    rs = np.random.RandomState(N)
    D, C, R = 64, 4, 2
    sizes = list(rs.randint(5, 30, size=N))
    Xs, ys = _rand_clients(rs, sizes, D, C)
    Xt = (np.cos(rs.normal(size=(90, D))) / np.sqrt(D)).astype(np.float32)
    yt = rs.randint(0, C, size=90).astype(np.int64)
    Xv = (np.cos(rs.normal(size=(150, D))) / np.sqrt(D)).astype(np.float32)
    yv = rs.randint(0, C, size=150).astype(np.int64)
    # lr_p small enough that p stays O(1): with |p| >> 1 the aggregate sum_j p_j W_j of 1000
    # clients cancels, and any two fp32 p's within 1e-5 give W's further apart than 1e-5 max|W|
    lr_p = 0.05 if N <= 300 else 0.005
    T = torch.from_numpy
    stats = {'trace': True}
    torch.manual_seed(5)
    tr, tl, ta = amd.tools.FedAMW([T(x) for x in Xs], [T(y) for y in ys], T(Xt), T(yt), _dl(Xv, yv),
                                  'classification', C, D, 0.5, 2, 32, False, 0.0, True, 1e-3, R, lr_p,
                                  clients='parallel', stats=stats, verbose=False)
    assert amd.lib.SOLVER_NAMES[amd.lib.lib().fs_mix_solve_last_mode()] in ('mc', 'qmc')   # a multi-CU solver ran (results() checks its error word)
    torch.manual_seed(5)
    otr, otl, ota, trace = O.FedAMW(Xs, ys, Xt, yt, Xv, yv, 'classification', C, D, 0.5, 2, 32, False, 0.0, True,
                                    1e-3, R, lr_p, clients='parallel')
    print('max|p| %.3g, max|W| %.3g' % (np.abs(trace['p']).max(), np.abs(trace['W']).max()))
    W = stats['W_rounds']
    for t in range(R):
        assert np.abs(W[t] - trace['W'][t]).max() <= W_RTOL * np.abs(trace['W'][t]).max(), t
    p = stats['p'].cpu().numpy()
    assert np.abs(p - trace['p'][-1]).max() <= P_RTOL * np.abs(trace['p'][-1]).max()
    np.testing.assert_allclose(tr.numpy(), otr, rtol=0, atol=LOSS_RTOL * max(1, np.abs(otr).max()))
    np.testing.assert_allclose(tl.numpy(), otl, rtol=0, atol=LOSS_RTOL * max(1, np.abs(otl).max()))
    assert np.abs(ta.numpy() - ota).max() <= 100.0 / 90 + 1e-4
