"""Data loading and partitioning for the experiment driver -- host-side setup, drop-ins for
the reference's ``functions/utils.py`` pieces that ``exp.py`` uses:

  * ``svmlight_labels``            -- label normalisation of ``svmlight_data``   utils.py:36-45
  * ``load_full_data``             -- LIBSVM train/test + Dirichlet partition  utils.py:124-167
  * ``get_Dirichlet_distribution`` -- label-skewed client partition            utils.py:314-349

Differences from the reference, all deliberate and stated:
  * the reference returns full-batch DataLoaders whose ``.next()`` exp.py:61-62 calls
    (gone in torch 2); ``load_full_data`` here returns the dense arrays and the driver
    replays the two loaders' RNG use itself (``full_batch_order``);
  * LIBSVM files are parsed by the native reader ``fs_libsvm_scan`` / ``fs_libsvm_read``
    (csrc/libsvm.cpp: multi-threaded, the rules of scikit-learn's ``load_svmlight_file``,
    which the reference calls at utils.py:38, and the same float32 values --
    tests/test_libsvm.py checks it against sklearn); the test file is read with the training
    file's width (a9a.t is one column narrower than a9a -- SURVEY Q14 -- which breaks the
    reference's matmul);
  * when the LIBSVM file is absent (no datasets ship with the reference or this image),
    ``load_full_data`` synthesises a dataset of the same shape from a private generator
    (``synthetic_libsvm``), so the global numpy / torch streams are consumed exactly as
    a file load consumes them (not at all).
The partitioner is a restatement of the reference's numpy algorithm (same calls, same
order, on the global numpy generator reseeded to 2020 as utils.py:320 does -- it stays on
numpy because its draws ARE numpy's legacy generator), pinned to the reference's own output:
tests/golden/make_golden.py imports the reference's utils.py behind an in-process
torchvision stub and records get_Dirichlet_distribution and the whole exp.py:60-99 data
path (tests/test_oracle_prep.py).
"""
import os

import numpy as np
import torch

from .. import rng

REGRESSION = ('abalone', 'cadata', 'cpusmall', 'space_ga')     # utils.py:32-34

# shapes of the LIBSVM datasets the benchmark configs name:
# name: (train rows, test rows, raw width, classes, kind)
SYNTH_SHAPES = {
    'a9a': (32561, 16281, 123, 2, 'a9a'),
    'covtype': (464810, 116202, 54, 7, 'covtype'),
}


def read_libsvm(path, n_features=None, zero_based=-1, nthreads=0):
    """A LIBSVM / svmlight file as dense float32 rows + float64 labels (the native reader,
    csrc/libsvm.cpp; the values of ``load_svmlight_file(path)[0].toarray().astype(float32)``).
    ``zero_based``: -1 auto (zero-based iff the smallest index is 0), 0 or 1.  Returns
    (X, y, zero_based_used, n_features)."""
    import ctypes
    from .. import _lib
    L = _lib.lib()
    bpath = os.fsencode(path)
    n, mn, mx = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    _lib.check(L.fs_libsvm_scan(bpath, ctypes.byref(n), ctypes.byref(mn), ctypes.byref(mx)), 'fs_libsvm_scan')
    zb = zero_based if zero_based in (0, 1) else (1 if mn.value == 0 else 0)
    d = int(n_features) if n_features is not None else max(0, mx.value + (1 if zb else 0))
    X = np.empty((n.value, d), np.float32)
    y = np.empty(n.value, np.float64)
    _lib.check(L.fs_libsvm_read(bpath, n.value, d, zb, X.ctypes.data, y.ctypes.data, int(nthreads)),
               'fs_libsvm_read')
    return X, y, zb, d


def svmlight_labels(y, dataset):
    """utils.py:39-45: regression targets scaled to [0, 100]; two classes mapped to {0, 1};
    more classes shifted to start at 0."""
    y = np.asarray(y, dtype=np.float64).copy()
    if dataset in REGRESSION:
        return 100 * (y - y.min()) / (y.max() - y.min())
    if len(set(y.tolist())) == 2:
        return (y - y.min()) / (y.max() - y.min())
    if len(set(y.tolist())) > 2:
        y -= y.min()
    return y


def synthetic_libsvm(name, n_train=None, n_test=None, seed=None):
    """A LIBSVM-shaped dataset from a private generator: a9a-like (123 binary columns, 14
    ones per row, P(y=1) ~ 0.24) or covtype-like (10 dense U[0,1] columns + one-hot groups of
    4 and 40, 7 classes); labels from a fixed random teacher on random cosine features, so
    the classes are learnable.  Returns (X_train, y_train, X_test, y_test) float32 / float64."""
    nt0, ne0, d, C, kind = SYNTH_SHAPES.get(name, SYNTH_SHAPES['a9a'])
    n_train, n_test = int(n_train or nt0), int(n_test or ne0)
    rs = np.random.RandomState(seed if seed is not None else (sum(map(ord, name)) + 7))
    n = n_train + n_test
    X = np.zeros((n, d), np.float32)
    if kind == 'a9a':
        cols = np.argsort(rs.rand(n, d), axis=1)[:, :14]
        np.put_along_axis(X, cols, 1.0, axis=1)
    else:
        X[:, :10] = rs.rand(n, 10)
        X[np.arange(n), 10 + rs.randint(0, 4, n)] = 1.0
        X[np.arange(n), 14 + rs.randint(0, 40, n)] = 1.0
    Wt = rs.normal(0, 0.6, size=(d, 64)).astype(np.float32)
    bt = rs.uniform(0, 2 * np.pi, size=64).astype(np.float32)
    score = np.cos(X @ Wt + bt) @ rs.normal(size=(64, C)).astype(np.float32)
    if C == 2:      # a9a's class balance: the top 24% of a margin score are positives
        m = score[:, 1] - score[:, 0]
        y = (m > np.quantile(m, 0.76)).astype(np.float64)
    else:
        y = np.argmax(score + 0.5 * rs.gumbel(size=score.shape), axis=1).astype(np.float64)
    return X[:n_train], y[:n_train], X[n_train:], y[n_train:]


def get_Dirichlet_distribution(labels, psizes=(0.7, 0.2, 0.1), alpha=0.1, verbose=True):
    """utils.py:314-349: label-skewed partition into len(psizes) clients.

    Reseeds the GLOBAL numpy generator to 2020 (utils.py:320) and redraws until every
    client holds >= 10 rows: per class k, its indices are shuffled, client proportions
    ~ Dirichlet(alpha), clients already holding >= N / n_clients rows get weight 0, every
    weight is lifted by 1/|class k|, and the class is cut at the cumulative proportions.
    Finally every client's index list is shuffled.  Returns (index lists, class counts)."""
    labels = np.asarray(labels)
    n_clients = len(psizes)
    n_classes = len(set(labels.tolist()))
    total = len(labels)
    np.random.seed(2020)
    smallest = 0
    while smallest < 10:
        parts = [[] for _ in range(n_clients)]
        for k in range(n_classes):
            members = np.where(labels == k)[0]
            np.random.shuffle(members)
            w = np.random.dirichlet(np.repeat(alpha, n_clients))
            open_ = np.array([len(p) < total / n_clients for p in parts])
            w = w * open_ + 1 / len(members)
            w = w / w.sum()
            cuts = (np.cumsum(w) * len(members)).astype(int)[:-1]
            for p, piece in zip(parts, np.split(members, cuts)):
                p.extend(piece.tolist())
            smallest = min(len(p) for p in parts)
    for p in parts:
        np.random.shuffle(p)
    counts = {}
    for j, p in enumerate(parts):
        u, c = np.unique(labels[p], return_counts=True)
        counts[j] = {u[i]: c[i] for i in range(len(u))}
    if verbose:
        print('Data statistics: %s' % str(counts))
    return parts, counts


def load_full_data(dataset_name, num_partitions=10, alpha=0.1, root_dir='../FedAMW/datasets/', synth=None,
                   verbose=True):
    """utils.py:124-167 for LIBSVM datasets: returns (X_train, y_train, X_test, y_test,
    index_partitions, feature_size, class_size) with dense float32 features and float64
    labels in the reference's normalisation.  ``alpha == -1`` partitions uniformly
    (a random permutation split into equal parts, global numpy generator).
    ``synth``: dict of synthetic_libsvm kwargs used when the file is absent (default: the
    dataset's full shape)."""
    path = os.path.join(root_dir, dataset_name)
    if os.path.exists(path):
        X, y, zb, d = read_libsvm(path)
        # each file picks its own index base, as the reference's two load_svmlight_file calls
        # do ('auto'); the test file keeps the training width
        Xt, yt, _, _ = read_libsvm(path + '.t', n_features=d, zero_based=-1)
        y, yt = svmlight_labels(y, dataset_name), svmlight_labels(yt, dataset_name)
    else:
        X, y, Xt, yt = synthetic_libsvm(dataset_name, **(synth or {}))
    psizes = [1.0 / num_partitions] * num_partitions
    if alpha != -1:
        parts, _ = get_Dirichlet_distribution(y, psizes, alpha, verbose=verbose)
    else:
        parts = np.array_split(np.random.permutation(len(y)), num_partitions)
    C = 1 if dataset_name in REGRESSION else len(set(y.tolist()))
    return X, y, Xt, yt, parts, X.shape[1], C


def full_batch_order(n, shuffle=True):
    """RNG use of ``next(iter(DataLoader(dataset, batch_size=len(dataset), shuffle)))``
    (exp.py:61-62): the worker base seed is drawn at iter(); a shuffling sampler draws its
    seed and runs randperm(n) (replayed bit-exactly by fs_randperm_batch).  Returns the row
    order of the single batch."""
    if not shuffle:
        torch.empty((), dtype=torch.int64).random_()
        return np.arange(n)
    seed = rng.draw_pass_seeds(1)
    out = np.empty(n, np.int32)
    rng.randperms(seed, [n], [0], out)
    return out.astype(np.int64)
