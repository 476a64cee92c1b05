"""Helpers to load the golden fixtures written by tests/golden/make_golden.py."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')

ROUND_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, 'fed*.npz')))
TRAIN_UNITS = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, 'unit_train_*.npz')))
LONG_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, 'long_fed*.npz')))
BENCH_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, 'bench_fedamw_*.npz')))


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


def acc_tol(d):
    return 100.0 / len(d['y_test']) + 1e-4
