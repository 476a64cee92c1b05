"""Helpers to load the golden fixtures written by tests/golden/make_golden.py."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')

ROUND_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, 'fed*.npz')))
TRAIN_UNITS = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, 'unit_train_*.npz')))
LONG_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, 'long_fed*.npz')))
BENCH_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, 'bench_fedamw_*.npz')))
HORIZON_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, 'horizon_*_*.npz'))
                       if not p.endswith('_data.npz'))


def load(name):
    z = np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False)
    return {k: z[k] for k in z.files}


def load_long(name):
    """A long-horizon case: the shared inputs (long_data.npz) merged with the case's
    hyper-parameters and reference outputs; ``W`` holds the global model at rounds ``snap``."""
    d = load('long_data')
    d.update(load(name))
    return d


def load_bench(name):
    """A benchmark-length FedAMW case (config 2's N = 100, C = 10; n_v >= 2,000, R = 34: >= 5,000
    p-SGD steps per round): bench_data.npz merged with the case; ``W`` at rounds ``snap``,
    ``p`` after every round."""
    d = load('bench_data')
    d.update(load(name))
    return d


def load_horizon(name):
    """A solver-horizon FedAMW case (make_golden.py run_horizon: 'qmc' = N 300, C 10, R 20;
    'bin' = N 10, C 2, n_v 6,509, R 10): horizon_<solver>_data.npz merged with the case; ``W``
    and ``p`` after every round, ``solver`` the p-solver the shape selects."""
    d = load('horizon_%s_data' % name.split('_')[1])
    d.update(load(name))
    return d


def split_clients(d):
    off = np.concatenate([[0], np.cumsum(d['sizes'])])
    Xs = [d['X_train'][off[i]:off[i + 1]] for i in range(len(d['sizes']))]
    ys = [d['y_train'][off[i]:off[i + 1]] for i in range(len(d['sizes']))]
    return Xs, ys


def positional(d):
    """The positional hyper-parameters, in the reference's order (tools.py:329)."""
    return ('classification', int(d['C']), int(d['D']), float(d['lr']), int(d['epoch']),
            int(d['batch_size']), bool(d['prox']), float(d['mu']), bool(d['reg']), float(d['lam']),
            int(d['R']))


# Tolerances (stated once, used by every parity test):
#   W (global model per round):  max|W - W_ref| <= W_RTOL * max|W_ref|
#   train/test loss:             |l - l_ref| <= LOSS_RTOL * max(1, |l_ref|)
#   test accuracy (percent):     within one test sample, 100/n_test points
W_RTOL = 1e-5
LOSS_RTOL = 1e-5
P_RTOL = 1e-5


# The solver-horizon cases (make_golden.py HORIZON) run up to 31,300 dependent p-SGD steps and
# up to 10,000 chained client trainings: there the fp32 arithmetic itself moves a result by more
# than 1e-5.  Their bounds are DERIVED, per case and quantity, by tests/golden/horizon_drift.py:
# the CPU restatement run in float32 and in float64 on the same inputs and RNG stream, delta =
# max over rounds of the relative distance of the two (how far any correct fp32 evaluation sits
# from the exact one at that horizon), bound = max(1e-5, 2 delta) -- two fp32 evaluations with
# different summation orders (the reference's torch kernels, the oracle's numpy, the GPU's
# MFMA) may each be delta away (horizon_drift.json: e.g. horizon_qmc_seq W 1.4e-4, p 3.6e-5;
# horizon_qmc1000_par W 3.7e-5).  W_RTOL / P_RTOL elsewhere.
with open(os.path.join(GOLDEN, 'horizon_drift.json')) as _f:
    HORIZON_DRIFT = json.load(_f)


def horizon_rtol(name, what='W'):
    """The derived bound of a horizon case for ``what`` in 'W', 'p', 'loss' (default bounds for
    any other case)."""
    rec = HORIZON_DRIFT.get(name)
    if rec is None:
        return {'W': W_RTOL, 'p': P_RTOL, 'loss': LOSS_RTOL}[what]
    return rec['rtol_' + what]


def horizon_rtol_rounds(name, what='W'):
    """Per-round bounds of a horizon case (round 6): round t is held to
    max(1e-5, 2 max_{s <= t} delta(s)) -- the fp32-vs-fp64 drift the restatement accumulates by
    round t -- instead of the whole run's worst round.  ``what`` in 'W', 'loss' (p is checked
    after the last round only: ``horizon_rtol(name, 'p')``)."""
    rec = HORIZON_DRIFT[name]
    d = np.maximum.accumulate(np.asarray(rec['delta_%s_per_round' % what], np.float64))
    return np.maximum(1e-5, 2.0 * d)


def acc_tol(d):
    return 100.0 / len(d['y_test']) + 1e-4
