"""Every BASELINE.json config exercised on the MI355X at its own workload shape, against the
CPU oracle (run on the GPU box; SURVEY.md 8(d) gives the shapes).

* config 1 -- exp.py's FedAMW on a9a (synthetic a9a-shaped LIBSVM data at full size: 32,561
  train / 16,281 test rows) split across 10 Dirichlet(0.01) clients, D = 2000, C = 2, chained
  clients (the reference's semantics; the chain runs on a group of CUs), 3 rounds.
* config 3 -- FedProx, 1000 covtype-shaped clients x 465 rows, D = 4096, C = 7, one round.
* config 4 -- FedAvg, 1250 clients x 64 rows (config 4's per-GPU share of 10,000), D = 2048.
* config 5 -- FedAMW, 1000 clients x 128 rows, D = 16384, C = 10, one round (validation set
  trimmed to 4 rows per client: 4,000 rows, 250 p-SGD steps).
Configs 3-5 check every client's result for finiteness, sampled clients' local training
against the oracle, the aggregate against the oracle's left fold over ALL clients, and the
test evaluation against the oracle.

Tolerances: per-client weights 2e-5 * max|W| (fp32 MFMA vs BLAS summation order, as in
test_gpu_parity.py); aggregate and global model 1e-5 * max|W| (tests/fixtures.py); losses
1e-5 relative; accuracy within one test sample; mixture weights 1e-5 * max|p|.  The config-1
run uses lr = 0.5 and lr_p = 0.05 (the a9a default branch's lr = 1e-3 barely moves the
model, which would make the comparison vacuous).
"""
import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.fixtures import LOSS_RTOL, P_RTOL, W_RTOL

pytestmark = pytest.mark.gpu

E, B = 2, 32


@pytest.fixture(scope='module')
def amd():
    import fedamw_amd
    from fedamw_amd import _lib, data, engine, experiment, rng
    from fedamw_amd.functions import tools
    _lib.lib()
    return type('amd', (), dict(lib=_lib, data=data, engine=engine, experiment=experiment, rng=rng, tools=tools))


def _np(t):
    return t.detach().cpu().numpy()


def test_config1_fedamw_chained_a9a(amd):
    params = {'kernel_par': 0.1, 'kernel_type': 'gaussian'}
    D, N, C, R, lr, lr_p, lam = 2000, 10, 2, 3, 0.5, 0.05, 1e-5
    torch.manual_seed(100)
    np.random.seed(100)
    d = amd.experiment.prepare('a9a', D, N, 0.01, params, '/nonexistent/', verbose=False)
    sizes = [len(y) for y in d['y_train']]
    assert len(sizes) == N and sum(sizes) > 20000 and min(sizes) >= 8      # exp.py's quantity skew
    stats = {'trace': True}
    torch.manual_seed(7)
    fed = amd.tools.Federation('fedamw', d['X_train'], d['y_train'], d['X_test'], d['y_test'], d['validloader'],
                               'classification', C, D, lr, E, B, False, 0.0, True, lam, R, lr_p, 'sequential',
                               stats=stats, verbose=False)
    assert fed.trainer.G > 1, 'the chain should run on a group of CUs'
    for _ in range(R):
        fed.round()
    tr, tl, ta = fed.results()
    Xs = [_np(x) for x in d['X_train']]
    ys = [_np(y) for y in d['y_train']]
    torch.manual_seed(7)
    otr, otl, ota, trace = O.FedAMW(Xs, ys, _np(d['X_test']), _np(d['y_test']), _np(d['X_val']), _np(d['y_val']),
                                    'classification', C, D, lr, E, B, False, 0.0, True, lam, R, lr_p)
    W = stats['W_rounds']
    for t in range(R):
        assert np.abs(W[t] - trace['W'][t]).max() <= W_RTOL * np.abs(trace['W'][t]).max(), t
    assert np.abs(_np(stats['p']) - trace['p'][-1]).max() <= P_RTOL * np.abs(trace['p'][-1]).max()
    np.testing.assert_allclose(tr.numpy(), otr, rtol=0, atol=LOSS_RTOL * max(1, np.abs(otr).max()))
    np.testing.assert_allclose(tl.numpy(), otl, rtol=0, atol=LOSS_RTOL * max(1, np.abs(otl).max()))
    assert np.abs(ta.numpy() - ota).max() <= 100.0 / len(d['y_test']) + 1e-4


def _one_round(amd, algo, N, n, D, C, nt, shape, prox, mu, n_val=0, sample=(0, 1), seed=11, lr=0.5, lr_p=1e-3):
    """One parallel-client round of `algo` through Federation on synthetic data of the config's
    shape; returns everything the checks need."""
    dev = torch.device('cuda')
    d = amd.data.federated(N, n, D, C, nt, n_val=n_val, shape=shape, seed=seed, device=dev)
    vl = None
    if n_val:
        vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(d['X_val'], d['y_val']), batch_size=16,
                                         shuffle=True)
    torch.manual_seed(seed)
    fed = amd.tools.Federation(algo, d['X_train'], d['y_train'], d['X_test'], d['y_test'], vl, 'classification', C,
                               D, lr, E, B, prox, mu, algo == 'fedamw', 1e-5, 1, lr_p, 'parallel', verbose=False)
    W0 = _np(fed.W_g[:, :D])
    fed.round()
    tr, tl, ta = fed.results()
    W_all = _np(fed.trainer.W_out[:, :, :D])
    assert np.isfinite(W_all).all()
    assert (_np(fed.trainer.W_out[:, :, D:]) == 0).all() if fed.ld > D else True
    loss = _np(fed.loss_hist[0])
    assert np.isfinite(loss).all()
    # sampled clients against the oracle: replay the round's RNG (init draw, then 2 draws per
    # training pass in client-major order); round = 1 puts t = 0 at the first decay
    # boundary int(R / 2) = 0 (tools.py:43-61), so round 0 trains at lr / 10
    lr0 = O.lr_schedule(0, lr, 1)
    for j in sample:
        torch.manual_seed(seed)
        O.mlp_init(D, C)
        torch.empty(2 * E * j, dtype=torch.int64).random_()
        Wr, lref = O.train_client(_np(d['X_train'][j]), _np(d['y_train'][j]), W0, lr0, E, B, prox, mu,
                                  algo == 'fedamw', 1e-5)
        assert np.abs(W_all[j] - Wr).max() <= 2e-5 * max(1.0, np.abs(Wr).max()), (j, np.abs(W_all[j] - Wr).max())
        assert abs(loss[j] - lref) <= 2e-5 * max(1.0, abs(lref)), j
    return dict(d=d, fed=fed, W_all=W_all, tr=tr, tl=tl, ta=ta, seed=seed)


def _check_aggregate_and_eval(r, p, D, n_val_passes=0):
    """The global model = the oracle's left fold of ALL clients' weights with `p`; the test
    metrics = the oracle's test_loop on it (same RNG pass)."""
    d, fed = r['d'], r['fed']
    W_ref = O.aggregate(list(r['W_all']), p)
    Wg = _np(fed.W_g[:, :D])
    assert np.abs(Wg - W_ref).max() <= W_RTOL * np.abs(W_ref).max()
    torch.manual_seed(r['seed'])
    O.mlp_init(D, fed.C)
    torch.empty(2 * (fed.N * E + n_val_passes), dtype=torch.int64).random_()
    tl, ta = O.test_eval(_np(d['X_test']), _np(d['y_test']), W_ref, B)
    assert abs(float(r['tl'][0]) - tl) <= LOSS_RTOL * max(1.0, abs(tl))
    assert abs(float(r['ta'][0]) - ta) <= 100.0 / len(d['y_test']) + 1e-4


@pytest.mark.parametrize('cfg', [3, 4])
def test_config3_config4_rounds(amd, cfg):
    if cfg == 3:      # FedProx, 1000 covtype-shaped clients x 465 rows, D = 4096, C = 7
        args = dict(algo='fedprox', N=1000, n=465, D=4096, C=7, nt=50000, shape='covtype', prox=True, mu=5e-4,
                    sample=(0, 517, 999))
    else:             # FedAvg, 1250 clients x 64 rows, D = 2048, C = 10 (config 4's per-GPU share)
        args = dict(algo='fedavg', N=1250, n=64, D=2048, C=10, nt=10000, shape='a9a', prox=False, mu=0.0,
                    sample=(3, 1249))
    r = _one_round(amd, **args)
    ns = np.array([len(y) for y in r['d']['y_train']])
    _check_aggregate_and_eval(r, (ns / ns.sum()).astype(np.float32), args['D'])


def test_config5_fedamw_wide(amd):
    N, n, D, C = 1000, 128, 16384, 10
    r = _one_round(amd, 'fedamw', N, n, D, C, 10000, 'a9a', False, 0.0, n_val=4, sample=(0, 999), lr_p=0.05)
    fed, d = r['fed'], r['d']
    mix = fed.mixture
    nv = mix.nv
    # Z = every client model applied to the validation rows (fs_mix_z, fp32 MFMA, K = 16384):
    # sampled rows against an fp64 product, within 2e-6 of sum_d |x_d w_d| per element
    Z = mix.Z.view(nv, C, mix.ldN)[:, :, :N]
    Wd = fed.trainer.W_out[:, :, :D].double()
    for v in (0, 1234, nv - 1):
        x = d['X_val'][v].double()
        ref = torch.einsum('ncd,d->cn', Wd, x)
        bound = torch.einsum('ncd,d->cn', Wd.abs(), x.abs())
        assert bool(((Z[v].double() - ref).abs() <= 2e-6 * bound + 1e-30).all()), v
    # the p-SGD on that Z against the oracle's (same RNG pass: after the training passes)
    torch.manual_seed(11)
    O.mlp_init(D, C)
    torch.empty(2 * N * E, dtype=torch.int64).random_()
    ns = np.array([len(y) for y in d['y_train']])
    p0 = (ns / ns.sum()).astype(np.float32)
    Zn = Z.permute(2, 1, 0).contiguous().cpu().numpy()        # [N, C, nv]
    p_ref, _ = O.mixture_solve_z(Zn, _np(d['y_val']), p0, None, 0.05, 1, 16)
    p = _np(mix.p)
    assert np.abs(p - p_ref).max() <= P_RTOL * np.abs(p_ref).max()
    _check_aggregate_and_eval(r, p, D, n_val_passes=1)
