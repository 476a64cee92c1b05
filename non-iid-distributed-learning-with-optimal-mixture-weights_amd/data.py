"""Synthetic libsvm-shaped federated data (setup only, not on the timed path).

The reference reads LIBSVM files that do not ship with it (utils.py:36-65, exp.py:33)
and maps them through random Fourier features (tools.py:15-31):
phi(x) = D^-1/2 cos(x W + b), W ~ N(0, sigma^2)^{d x D}, b ~ U(0, 2 pi).
Here raw rows are synthesised in the shape of the datasets the benchmark configs
name:
  * a9a-shaped:     d = 123 binary features, 14 ones per row;
  * covtype-shaped: d = 54 = 10 dense U[0,1] columns + one-hot groups of 4 and 40.
Labels come from a fixed random teacher on the RFF features (so accuracy means
something), and clients are label-skewed: each client's class mix ~ Dirichlet(alpha).
"""
import math

import numpy as np
import torch


def raw_rows(n, shape, gen, device):
    if shape == 'a9a':
        d = 123
        keys = torch.rand(n, d, generator=gen, device=device)
        idx = keys.topk(14, dim=1).indices
        X = torch.zeros(n, d, device=device)
        X.scatter_(1, idx, 1.0)
        return X
    if shape == 'covtype':
        X = torch.zeros(n, 54, device=device)
        X[:, :10] = torch.rand(n, 10, generator=gen, device=device)
        X[torch.arange(n, device=device), 10 + torch.randint(0, 4, (n,), generator=gen, device=device)] = 1.0
        X[torch.arange(n, device=device), 14 + torch.randint(0, 40, (n,), generator=gen, device=device)] = 1.0
        return X
    raise ValueError(shape)


def rff(X, D, sigma, gen):
    """tools.py:15-31 (setup): phi = D^-1/2 cos(X W + b)."""
    d = X.shape[1]
    W = torch.randn(d, D, generator=gen, device=X.device) * sigma
    b = torch.rand(1, D, generator=gen, device=X.device) * (2 * math.pi)
    return torch.cos(X @ W + b) / math.sqrt(D)


def federated(n_clients, n_train, D, C, n_test, n_val=0, shape='a9a', sigma=0.1, alpha=0.1, seed=0,
              device='cuda', chunk=65536):
    """Returns dict(X_train=[N tensors n_train x D], y_train=[N int64], X_test, y_test, X_val, y_val).

    ``n_train`` / ``n_val`` are per-client row counts (int or length-N sequence)."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    ntr = np.broadcast_to(np.asarray(n_train, dtype=np.int64), (n_clients,)).copy()
    nva = np.broadcast_to(np.asarray(n_val, dtype=np.int64), (n_clients,)).copy()
    need = int(ntr.sum() + nva.sum())
    pool_n = int(need * 1.25) + n_test + C
    d = 123 if shape == 'a9a' else 54
    Wr = torch.randn(d, D, generator=gen, device=device) * sigma
    br = torch.rand(1, D, generator=gen, device=device) * (2 * math.pi)
    T = torch.randn(D, C, generator=gen, device=device)
    phi = torch.empty(pool_n, D, device=device)
    y = torch.empty(pool_n, dtype=torch.int64, device=device)
    for s in range(0, pool_n, chunk):
        e = min(pool_n, s + chunk)
        X = raw_rows(e - s, shape, gen, device)
        phi[s:e] = torch.cos(X @ Wr + br) * (1.0 / math.sqrt(D))
        logits = phi[s:e] @ T
        logits = (logits - logits.mean(0)) / (logits.std(0) + 1e-6)   # balance the teacher's classes
        y[s:e] = logits.argmax(1)
    test = torch.arange(pool_n - n_test, pool_n, device=device)
    yc = y[:pool_n - n_test].cpu().numpy()
    rs = np.random.RandomState(seed)
    buckets = [list(rs.permutation(np.nonzero(yc == c)[0])) for c in range(C)]
    fill = list(rs.permutation(len(yc)))
    out = {'X_train': [], 'y_train': [], 'X_val': [], 'y_val': []}
    for j in range(n_clients):
        mix = rs.dirichlet(np.full(C, alpha))
        cnt = rs.multinomial(int(ntr[j] + nva[j]), mix)
        idx = []
        for c in range(C):
            take = min(int(cnt[c]), len(buckets[c]))
            idx += [buckets[c].pop() for _ in range(take)]
        while len(idx) < ntr[j] + nva[j]:
            idx.append(fill.pop())
        idx = torch.as_tensor(np.array(idx[:int(ntr[j] + nva[j])]), device=device)
        idx = idx[torch.randperm(len(idx), generator=gen, device=device)]
        out['X_train'].append(phi[idx[:ntr[j]]])
        out['y_train'].append(y[idx[:ntr[j]]])
        if nva[j]:
            out['X_val'].append(phi[idx[ntr[j]:]])
            out['y_val'].append(y[idx[ntr[j]:]])
    out['X_test'] = phi[test]
    out['y_test'] = y[test]
    if out['X_val']:
        out['X_val'] = torch.cat(out['X_val'])
        out['y_val'] = torch.cat(out['y_val'])
    else:
        out['X_val'] = out['y_val'] = None
    return out
