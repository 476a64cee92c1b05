"""The experiment driver -- counterpart of the reference's ``exp.py`` (exp.py:22-143), on MI355X.

    python run_experiment.py --dataset a9a --D 2000 --clients 10 --rounds 100 ...

Reproduces exp.py's sequence exactly, consuming torch's and numpy's global generators in
the same order:
  1. seeds: torch.manual_seed(100), np.random.seed(100)                       exp.py:28-29
  2. load + Dirichlet partition (numpy reseeded to 2020)                        exp.py:60, utils.py:320
  3. the full-batch train pass (2 draws + randperm) and test pass (1 draw)     exp.py:61-62
     -- the partition's indices then address the SHUFFLED training rows, as in the
     reference
  4. the RFF draw and feature map (fs_feature_map)                              exp.py:63
  5. data heterogeneity (fs_gram + fs_hetero)                                   exp.py:66-74
  6. per-client 20/80 validation split with np.random.shuffle                  exp.py:78-99
  7. Centralized, Distributed, FedAMW_OneShot, FedAvg, FedProx, FedAMW with exp.py's
     positional arguments                                                       exp.py:102-130
and writes ``{result_dir}/exp1_{dataset}.pkl`` with the reference's keys (epochs,
train_loss, test_loss, test_acc of shape (6, Round, n_repeats), heterogeneity, name).

Stated choices where the reference is silent or broken: datasets missing from
``get_parameter`` (a9a, covtype) fall to its default branch, which lacks ``lr_p``,
``lr_p_os`` and ``lambda_reg_os``: they default to 1e-3, 1e-3 and ``lambda_reg``
(SURVEY.md 8(d) config 1); LIBSVM files that are absent are synthesised in their shape
(functions/utils.py).  ``clients='parallel'`` (not the reference's semantics) runs FedAvg,
FedProx and FedAMW with independent clients.
"""
import argparse
import os
import pickle
import time

import numpy as np
import torch

from .functions import tools, utils
from .functions.optimal_parameters import get_parameter
from . import engine

NAMES = ['CL', 'DL', 'FedAMW_OneShot', 'FedAvg', 'FedProx', 'FedAMW']


def prepare(dataset, D, num_partitions, alpha_Dirk, params, data_dir, synth=None, verbose=True):
    """exp.py:60-99 for one repeat.  Returns dict(X_train [list of N GPU tensors], y_train,
    X_test, y_test, X_val, y_val, validloader, heterogeneity, index_partitions)."""
    X, y, Xt, yt, parts, d, C = utils.load_full_data(dataset, num_partitions, alpha_Dirk, data_dir, synth=synth,
                                                     verbose=verbose)
    order = utils.full_batch_order(len(y), shuffle=True)                          # exp.py:61
    utils.full_batch_order(len(yt), shuffle=False)                                # exp.py:62
    X, y = X[order], torch.from_numpy(y[order]).long()
    yt = torch.from_numpy(yt).long()
    phi, phi_t = tools.feature_mapping(torch.from_numpy(X).reshape(1, X.shape[0], X.shape[1]), torch.from_numpy(Xt),
                                       params['kernel_par'], D, params['kernel_type'])
    phi = phi.reshape(-1, D)
    dev = phi.device
    Xc = [phi[torch.as_tensor(np.asarray(idx, dtype=np.int64), device=dev)] for idx in parts]
    yc = [y[np.asarray(idx, dtype=np.int64)] for idx in parts]
    hete, _ = engine.heterogeneity(engine.Features(Xc, yc, D, dev))               # exp.py:66-74
    Xv, yv, Xtr, ytr = [], [], [], []
    for Xi, yi in zip(Xc, yc):                                                    # exp.py:78-90
        ridx = np.arange(Xi.shape[0])
        np.random.shuffle(ridx)
        cut = int(Xi.shape[0] * 0.2)
        vi, ti = ridx[:cut], ridx[cut:]
        Xv.append(Xi[torch.from_numpy(vi).to(dev)])
        yv.append(yi[vi])
        Xtr.append(Xi[torch.from_numpy(ti).to(dev)])
        ytr.append(yi[ti])
    X_val, y_val = torch.cat(Xv, 0).cpu(), torch.cat(yv, 0)
    vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(X_val, y_val), batch_size=16, shuffle=True)
    return dict(X_train=Xtr, y_train=ytr, X_test=phi_t, y_test=yt, X_val=X_val, y_val=y_val, validloader=vl,
                heterogeneity=hete, index_partitions=parts, num_classes=C, d=d)


def run(dataset='a9a', D=2000, num_partitions=10, local_epoch=2, Round=100, batch_size=32, n_repeats=1,
        alpha_Dirk=0.01, data_dir='../FedAMW/datasets/', result_dir='./results', save=True, clients='sequential',
        algos=tuple(NAMES), synth=None, verbose=True):
    torch.manual_seed(100)
    np.random.seed(100)
    P = get_parameter(dataset)
    task, C, k_par = P['task_type'], P['num_classes'], P['kernel_par']
    lr, mu, lam = P['lr'], P['lambda_prox'], P['lambda_reg']
    lr_p, lr_p_os, lam_os = P.get('lr_p', 1e-3), P.get('lr_p_os', 1e-3), P.get('lambda_reg_os', P['lambda_reg'])
    train_mat = np.empty((6, Round, n_repeats))
    error_mat = np.empty((6, Round, n_repeats))
    acc_mat = np.empty((6, Round, n_repeats))
    hete_mat = np.empty(n_repeats)
    timing = {}
    for t in range(n_repeats):
        d = prepare(dataset, D, num_partitions, alpha_Dirk, P, data_dir, synth=synth, verbose=verbose)
        C = d['num_classes'] if task == 'classification' else C
        hete_mat[t] = d['heterogeneity']
        a = (d['X_train'], d['y_train'], d['X_test'], d['y_test'])
        kw = dict(verbose=verbose)
        par = dict(clients=clients, **kw)

        def timed(name, fn):
            t0 = time.perf_counter()
            out = fn()
            timing.setdefault(name, []).append(time.perf_counter() - t0)
            return out

        # exp.py:116-130, positional as the reference calls them; skipped algorithms leave NaN rows
        for k in range(6):
            train_mat[k, :, t] = error_mat[k, :, t] = acc_mat[k, :, t] = np.nan
        if 'CL' in algos:
            r = timed('CL', lambda: tools.Centralized(*a, task, C, D, lr, local_epoch * Round, batch_size, False, 0,
                                                      False, 0, **kw))
            train_mat[0, :, t], error_mat[0, :, t], acc_mat[0, :, t] = float(r[0]), r[1], r[2]
        if 'DL' in algos:
            r = timed('DL', lambda: tools.Distributed(*a, task, C, D, lr, local_epoch * Round, batch_size, False, 0,
                                                      False, 0, **kw))
            train_mat[1, :, t], error_mat[1, :, t], acc_mat[1, :, t] = float(r[0]), r[1], r[2]
        if 'FedAMW_OneShot' in algos:
            r = timed('FedAMW_OneShot', lambda: tools.FedAMW_OneShot(*a, d['validloader'], task, C, D, lr,
                                                                     local_epoch * Round, batch_size, False, 0, True,
                                                                     lam_os, Round, lr_p_os, **kw))
            train_mat[2, :, t], error_mat[2, :, t], acc_mat[2, :, t] = float(r[0]), r[1].numpy(), r[2].numpy()
        if 'FedAvg' in algos:
            r = timed('FedAvg', lambda: tools.FedAvg(*a, task, C, D, lr, local_epoch, batch_size, False, 0, False, 0,
                                                     Round, **par))
            train_mat[3, :, t], error_mat[3, :, t], acc_mat[3, :, t] = r[0].numpy(), r[1].numpy(), r[2].numpy()
        if 'FedProx' in algos:
            r = timed('FedProx', lambda: tools.FedProx(*a, task, C, D, lr, local_epoch, batch_size, True, mu, False,
                                                       0, Round, **par))
            train_mat[4, :, t], error_mat[4, :, t], acc_mat[4, :, t] = r[0].numpy(), r[1].numpy(), r[2].numpy()
        if 'FedAMW' in algos:
            r = timed('FedAMW', lambda: tools.FedAMW(*a, d['validloader'], task, C, D, lr, local_epoch, batch_size,
                                                     False, 0, True, lam, Round, lr_p, **par))
            train_mat[5, :, t], error_mat[5, :, t], acc_mat[5, :, t] = r[0].numpy(), r[1].numpy(), r[2].numpy()
    data_ = {'epochs': Round, 'train_loss': train_mat, 'test_loss': error_mat, 'test_acc': acc_mat,
             'heterogeneity': hete_mat, 'name': list(NAMES), 'seconds': {k: list(v) for k, v in timing.items()}}
    if save:
        os.makedirs(result_dir, exist_ok=True)
        with open(os.path.join(result_dir, 'exp1_{}.pkl'.format(dataset)), 'wb') as f:
            pickle.dump(data_, f)
    return data_


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split('\n')[0])
    ap.add_argument('--dataset', default='a9a')
    ap.add_argument('--D', type=int, default=2000)
    ap.add_argument('--clients', type=int, default=10, help='num_partitions')
    ap.add_argument('--local-epoch', type=int, default=2)
    ap.add_argument('--rounds', type=int, default=100)
    ap.add_argument('--batch-size', type=int, default=32)
    ap.add_argument('--repeats', type=int, default=1)
    ap.add_argument('--alpha', type=float, default=0.01, help='Dirichlet alpha (-1: uniform split)')
    ap.add_argument('--data-dir', default='../FedAMW/datasets/')
    ap.add_argument('--result-dir', default='./results')
    ap.add_argument('--mode', default='sequential', choices=['sequential', 'parallel'])
    ap.add_argument('--algos', default=','.join(NAMES))
    ap.add_argument('--quiet', action='store_true')
    a = ap.parse_args(argv)
    out = run(a.dataset, a.D, a.clients, a.local_epoch, a.rounds, a.batch_size, a.repeats, a.alpha, a.data_dir,
              a.result_dir, True, a.mode, tuple(a.algos.split(',')), verbose=not a.quiet)
    for k, name in enumerate(NAMES):
        print('%-15s final test acc %s' % (name, np.round(out['test_acc'][k, -1, :], 2)))
    print('heterogeneity', out['heterogeneity'], 'seconds', {k: np.round(v, 3) for k, v in out['seconds'].items()})
    return out
