"""The native LIBSVM reader (csrc/libsvm.cpp, fs_libsvm_scan / fs_libsvm_read) against
scikit-learn's load_svmlight_file -- what the reference's svmlight_data calls
(/root/reference/functions/utils.py:36-38) -- on the dense float32 rows the reference feeds
its feature map (utils.py:56: `.A`, then float32).  Bit-exact: values and labels compared
with np.array_equal.  CPU only."""
import os

import numpy as np
import pytest
from sklearn.datasets import dump_svmlight_file, load_svmlight_file

import fedamw_amd  # noqa: F401
from fedamw_amd import _lib
from fedamw_amd.functions import utils


def _sk(path, **kw):
    X, y = load_svmlight_file(path, **kw)
    return X.toarray().astype(np.float32), y


def _check(path, **kw):
    Xs, ys = _sk(path, **kw)
    zb = {True: 1, False: 0, 'auto': -1}[kw.get('zero_based', 'auto')]
    X, y, _, d = utils.read_libsvm(path, n_features=kw.get('n_features'), zero_based=zb)
    assert X.shape == Xs.shape and d == Xs.shape[1]
    assert np.array_equal(X, Xs)
    assert np.array_equal(y, ys)
    return X, y


def test_a9a_shaped_binary(tmp_path):
    rs = np.random.RandomState(0)
    X = np.zeros((3000, 123), np.float32)
    cols = np.argsort(rs.rand(3000, 123), axis=1)[:, :14]
    np.put_along_axis(X, cols, 1.0, axis=1)
    y = np.where(rs.rand(3000) < 0.24, 1, -1)
    p = str(tmp_path / 'a9a')
    dump_svmlight_file(X, y, p, zero_based=False)
    _check(p)
    # the test file read at the training width (a9a.t is one column narrower)
    _check(p, n_features=130)


def test_covtype_shaped_dense_multichunk(tmp_path):
    """~20 MB of long decimal values: the parse runs over many line-aligned chunks."""
    rs = np.random.RandomState(1)
    n = 60000
    X = rs.uniform(-3000, 3000, size=(n, 54)) * rs.rand(n, 54) ** 3
    X[rs.rand(n, 54) < 0.4] = 0.0
    y = rs.randint(1, 8, size=n)
    p = str(tmp_path / 'covtype')
    dump_svmlight_file(X, y, p, zero_based=False)
    assert os.path.getsize(p) > 8 << 20
    _check(p)
    Xs, ys = _sk(p)
    for nt in (1, 3, 16):       # the result does not depend on the chunking
        X2, y2, _, _ = utils.read_libsvm(p, nthreads=nt)
        assert np.array_equal(X2, Xs) and np.array_equal(y2, ys)


def test_syntax_edges(tmp_path):
    text = ('# a comment line\n'
            '+1 1:0.5 3:1e-3 7:-2.25   \n'
            '\n'
            '-1\tqid:4 2:3.0000000000000004 5:1E+2 # trailing comment\n'
            '2 1:1 2:2 3:3\r\n'
            '   \n'
            '0 6:0.1 7:123456789.123456789\n')
    p = str(tmp_path / 'edges')
    with open(p, 'w') as f:
        f.write(text)
    X, y = _check(p)
    assert X.shape == (4, 7)
    _check(p, zero_based=False)
    _check(p, n_features=9)


def test_zero_based_auto(tmp_path):
    p = str(tmp_path / 'zb')
    with open(p, 'w') as f:
        f.write('1 0:1.5 4:2\n0 2:3\n')
    X, y = _check(p)
    assert X.shape == (2, 5) and X[0, 0] == 1.5
    _check(p, zero_based=True)


def test_errors(tmp_path):
    p = str(tmp_path / 'bad')
    with open(p, 'w') as f:
        f.write('1 1:1 9:2\n')
    with pytest.raises(_lib.FedsimError, match='outside'):
        utils.read_libsvm(p, n_features=5)
    with open(p, 'w') as f:
        f.write('1 1:1 x:2\n')
    with pytest.raises(_lib.FedsimError, match='line 1'):
        utils.read_libsvm(p)
    with pytest.raises(_lib.FedsimError, match='cannot read'):
        utils.read_libsvm(str(tmp_path / 'missing'))


def test_load_full_data_uses_the_file(tmp_path):
    """load_full_data on real LIBSVM files: the native reader's rows, the reference's label
    normalisation (utils.py:39-45), the test file at the training width."""
    rs = np.random.RandomState(3)
    X = (rs.rand(400, 20) < 0.3).astype(np.float64)
    y = rs.randint(1, 4, size=400)
    dump_svmlight_file(X[:300], y[:300], str(tmp_path / 'toy'), zero_based=False)
    dump_svmlight_file(X[300:, :19], y[300:], str(tmp_path / 'toy.t'), zero_based=False)
    Xtr, ytr, Xte, yte, parts, d, C = utils.load_full_data('toy', 4, 0.5, root_dir=str(tmp_path) + '/',
                                                           verbose=False)
    Xs, ys = _sk(str(tmp_path / 'toy'))
    Xts, yts = _sk(str(tmp_path / 'toy.t'), n_features=Xs.shape[1])
    assert np.array_equal(Xtr, Xs) and np.array_equal(Xte, Xts)
    assert np.array_equal(ytr, utils.svmlight_labels(ys, 'toy'))
    assert np.array_equal(yte, utils.svmlight_labels(yts, 'toy'))
    assert d == Xs.shape[1] and C == 3 and sum(len(p) for p in parts) == 300


def test_unsorted_or_duplicate_indices_rejected(tmp_path):
    """load_svmlight_file raises ValueError when a line's indices are not strictly increasing;
    the native reader refuses the same files (it used to keep the last value)."""
    for name, text in (('uns', '1 1:1 3:2 2:5\n'), ('dup', '0 2:1\n1 1:1 1:2\n')):
        p = str(tmp_path / name)
        with open(p, 'w') as f:
            f.write(text)
        with pytest.raises(ValueError, match='sorted and unique'):
            load_svmlight_file(p)
        with pytest.raises(_lib.FedsimError, match='sorted and unique'):
            utils.read_libsvm(p)


def test_load_full_data_index_base_per_file(tmp_path):
    """The reference calls load_svmlight_file once per file, each with zero_based='auto':
    a training file that uses feature 0 and a test file that does not are read with
    different bases (the test file at the training width)."""
    with open(tmp_path / 'mix', 'w') as f:
        f.write(''.join('%d 0:1 %d:2\n' % (i % 2, 1 + i % 5) for i in range(40)))
    with open(tmp_path / 'mix.t', 'w') as f:
        f.write(''.join('%d %d:3 6:1\n' % (i % 2, 1 + i % 4) for i in range(12)))
    Xtr, ytr, Xte, yte, parts, d, C = utils.load_full_data('mix', 2, 0.5, root_dir=str(tmp_path) + '/',
                                                           verbose=False)
    Xs, _ = _sk(str(tmp_path / 'mix'))
    Xts, _ = _sk(str(tmp_path / 'mix.t'), n_features=Xs.shape[1])
    assert d == Xs.shape[1] == 6
    assert np.array_equal(Xtr, Xs) and np.array_equal(Xte, Xts)
    assert Xte[0, 0] == 3.0 and Xte[0, 5] == 1.0      # one-based: index 1 -> column 0
