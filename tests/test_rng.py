"""Host-side RNG replay (C++ in libfedsim.so) vs torch's own generator -- CPU only."""
import numpy as np
import pytest
import torch

import fedamw_amd
from fedamw_amd import rng


@pytest.mark.parametrize('n', [1, 2, 20, 513, 70000])
def test_randperm_matches_torch(n):
    torch.manual_seed(n)
    seeds = rng.draw_pass_seeds(3)
    out = np.empty(3 * n, np.int32)
    rng.randperms(seeds, [n] * 3, [0, n, 2 * n], out, nthreads=2)
    for i, s in enumerate(seeds):
        g = torch.Generator()
        g.manual_seed(int(s))
        np.testing.assert_array_equal(out[i * n:(i + 1) * n], torch.randperm(n, generator=g).numpy())


def test_pass_seeds_are_dataloader_draws():
    """Two global draws per shuffled DataLoader pass; the second seeds the sampler."""
    X = torch.arange(50, dtype=torch.float32)[:, None]
    ds = torch.utils.data.TensorDataset(X, torch.zeros(50, dtype=torch.int64))
    torch.manual_seed(3)
    orders = [torch.cat([b[0][:, 0] for b in torch.utils.data.DataLoader(ds, 16, shuffle=True)]).long().numpy()
              for _ in range(4)]
    after = torch.empty(2, dtype=torch.int64).random_()
    torch.manual_seed(3)
    seeds = rng.draw_pass_seeds(4)
    out = np.empty(200, np.int32)
    rng.randperms(seeds, [50] * 4, [0, 50, 100, 150], out)
    for i in range(4):
        np.testing.assert_array_equal(out[50 * i:50 * (i + 1)], orders[i])
    assert torch.equal(torch.empty(2, dtype=torch.int64).random_(), after)


def test_randperm_threads_agree():
    torch.manual_seed(0)
    seeds = rng.draw_pass_seeds(64)
    ns = np.random.RandomState(0).randint(1, 3000, size=64)
    offs = np.concatenate([[0], np.cumsum(ns)[:-1]])
    a = np.empty(ns.sum(), np.int32)
    b = np.empty(ns.sum(), np.int32)
    rng.randperms(seeds, ns, offs, a, nthreads=1)
    rng.randperms(seeds, ns, offs, b, nthreads=7)
    np.testing.assert_array_equal(a, b)


def test_randperm_rejects_small_buffer():
    with pytest.raises(ValueError):
        rng.randperms([1], [10], [0], np.empty(5, np.int32))
