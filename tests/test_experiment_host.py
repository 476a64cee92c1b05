"""Host-side pieces of the experiment driver (no GPU): get_parameter against the reference's
table (tests/golden/params.json), the Dirichlet partitioner (utils.py:314-349) against the
oracle's restatement and its invariants, label normalisation, full-batch RNG replay."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import fedsim_oracle as O
from tests.fixtures import GOLDEN


@pytest.fixture(scope='module')
def host():
    import fedamw_amd  # noqa: F401
    from fedamw_amd.functions import optimal_parameters, utils
    return type('host', (), dict(utils=utils, params=optimal_parameters))


def test_get_parameter_matches_reference_table(host):
    with open(os.path.join(GOLDEN, 'params.json')) as f:
        ref = json.load(f)
    for name, d in ref.items():
        got = host.params.get_parameter(name)
        assert list(got.keys()) == list(d.keys()), name
        assert got == d, name


@pytest.mark.parametrize('n,clients,alpha,C', [(600, 5, 0.01, 2), (2000, 10, 0.1, 7), (900, 3, 1.0, 4)])
def test_dirichlet_partition(host, n, clients, alpha, C):
    rs = np.random.RandomState(n)
    y = rs.randint(0, C, n).astype(np.float64)
    np.random.seed(1)
    parts, counts = host.utils.get_Dirichlet_distribution(y, [1.0 / clients] * clients, alpha, verbose=False)
    after = np.random.get_state()[1].copy()
    np.random.seed(1)
    ref = O.dirichlet_partition(y, clients, alpha)
    assert [list(p) for p in parts] == [list(p) for p in ref]
    np.testing.assert_array_equal(after, np.random.get_state()[1])      # same numpy stream consumed
    allidx = np.concatenate([np.asarray(p, dtype=np.int64) for p in parts])
    assert np.array_equal(np.sort(allidx), np.arange(n))                 # every row exactly once
    assert min(len(p) for p in parts) >= 10
    assert sum(sum(c.values()) for c in counts.values()) == n


def test_svmlight_labels(host):
    u = host.utils
    np.testing.assert_array_equal(u.svmlight_labels(np.array([-1., 1, 1, -1]), 'a9a'), [0, 1, 1, 0])
    np.testing.assert_array_equal(u.svmlight_labels(np.array([1., 3, 2, 7]), 'covtype'), [0, 2, 1, 6])
    np.testing.assert_allclose(u.svmlight_labels(np.array([2., 4, 3]), 'abalone'), [0, 100, 50])


def test_full_batch_order_replays_dataloader(host):
    X = torch.arange(50, dtype=torch.float32).reshape(50, 1)
    torch.manual_seed(3)
    batch = next(iter(torch.utils.data.DataLoader(torch.utils.data.TensorDataset(X), batch_size=50, shuffle=True)))
    next(iter(torch.utils.data.DataLoader(torch.utils.data.TensorDataset(X), batch_size=50, shuffle=False)))
    after = torch.empty(3, dtype=torch.int64).random_()
    torch.manual_seed(3)
    order = host.utils.full_batch_order(50, True)
    host.utils.full_batch_order(50, False)
    np.testing.assert_array_equal(order, batch[0][:, 0].numpy().astype(np.int64))
    np.testing.assert_array_equal(torch.empty(3, dtype=torch.int64).random_().numpy(), after.numpy())


def test_synthetic_libsvm_shapes(host):
    X, y, Xt, yt = host.utils.synthetic_libsvm('a9a', 400, 100)
    assert X.shape == (400, 123) and Xt.shape == (100, 123)
    assert (X.sum(1) == 14).all() and set(np.unique(y)) <= {0.0, 1.0}
    X, y, Xt, yt = host.utils.synthetic_libsvm('covtype', 300, 50)
    assert X.shape == (300, 54) and len(set(y.tolist())) <= 7
