"""CPU restatement of the reference's federated round -- TEST INFRASTRUCTURE ONLY.

This module is the *oracle* (checker) for the MI355X HIP path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker / the CPU baseline -- never as the product path.  The
product (``fedamw_amd``) has no CPU fallback and never imports this file.

What it restates (numpy float32, closed-form gradients, one client at a time):

  * ``lr_schedule``      -- ``update_learning_rate``        tools.py:43-61  (compounding)
  * ``mlp_init``         -- ``MLP.__init__``                tools.py:34-40  (Kaiming draw then Xavier, Q12)
  * ``pass_order``       -- one ``DataLoader(shuffle=True)`` pass's RNG use (Q11)
  * ``train_client``     -- ``train_loop``                  tools.py:177-215 (unsquared prox/ridge, Q2/Q5)
  * ``test_eval``        -- ``test_loop`` + ``comp_accuracy`` + ``Meter``  tools.py:218-237, 82-166 (Q13)
  * ``aggregate``        -- the inline left fold            tools.py:345-350
  * ``mixture_solve``    -- FedAMW's p-SGD                  tools.py:441-453 (Q6, Q7)
                            (``mixture_solve_z``: the same on precomputed validation logits)
  * ``FedAvg/FedProx/FedAMW`` -- round drivers              tools.py:329-380, 413-463

The RNG stream is torch's own CPU generator (the generator the reference draws
from), used through the same calls the reference's DataLoader makes, so seeds
line up draw-for-draw.  ``clients='sequential'`` is the reference semantics
(client i starts from client i-1's weights); ``clients='parallel'``
starts every client from the round's global model (the harness-level variant
the golden generator builds by calling the reference's own ``train_loop`` on a
deep copy per client).

Parity pinning: this oracle is checked against the golden fixtures in
``tests/golden/`` that ``tests/golden/make_golden.py`` produced by importing the
unmodified reference ``functions/tools.py`` in the build container
(``tests/test_oracle_golden.py``).
"""
from __future__ import annotations

import math

import numpy as np
import torch

F32 = np.float32


# --------------------------------------------------------------------------- #
# small pieces
# --------------------------------------------------------------------------- #
def lr_schedule(t: int, lr: float, R: int) -> float:
    """tools.py:43-61 -- returns the *new* lr; callers rebind it (tools.py:338)."""
    if t == int(R / 2):
        return lr / 10
    if t == int(R * 0.75):
        return lr / 100
    return lr


def mlp_init(D: int, C: int) -> np.ndarray:
    """tools.py:34-40: nn.Linear(D, C, bias=False) default init, then xavier_uniform_.

    Consumes the global torch RNG exactly like ``MLP(D, C)`` (C*D uniforms for the
    discarded Kaiming draw, then C*D for Xavier).
    """
    w = torch.empty(C, D)
    torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
    torch.nn.init.xavier_uniform_(w)
    return w.numpy().astype(F32)


def pass_order(n: int, shuffle: bool = True) -> np.ndarray:
    """RNG use of one pass over ``DataLoader(TensorDataset, batch_size, shuffle)``.

    iter() draws the worker base seed (1 int64); RandomSampler draws its seed
    (1 int64) and runs randperm(n) on a private generator.
    tools.py:178-179, 190 (train), 219-220, 229 (test), exp.py:99 (valid).
    """
    torch.empty((), dtype=torch.int64).random_()
    if not shuffle:
        return np.arange(n)
    seed = int(torch.empty((), dtype=torch.int64).random_().item())
    g = torch.Generator()
    g.manual_seed(seed)
    return torch.randperm(n, generator=g).numpy()


def _log_softmax(z: np.ndarray) -> np.ndarray:
    m = z.max(axis=1, keepdims=True)
    s = np.exp(z - m).sum(axis=1, keepdims=True, dtype=F32)
    return (z - m - np.log(s)).astype(F32)


# --------------------------------------------------------------------------- #
# train_loop / test_loop
# --------------------------------------------------------------------------- #
def train_client(X, y, W, lr, epoch, batch_size, prox, mu, reg, lam):
    """tools.py:177-215.  Returns (W_new, last-epoch mean loss).

    Per batch (size |b| <= batch_size, last one short):
      z = X_b W^T ; L = CE_mean(z, y) [+ mu*||W-W_a||_F] [+ lam*||W||_F]   (tools.py:194-209)
      grad = (softmax(z) - onehot)^T X_b / |b| [+ mu (W-W_a)/||W-W_a||] [+ lam W/||W||]
      (a zero norm contributes a zero gradient, as torch's norm backward does -- Q2)
      W -= lr * grad                                                         (tools.py:210-211)
    The reported loss is the |b|-weighted mean over the LAST epoch (Meter reset
    per epoch, tools.py:187-189, 212, 215).
    """
    X = np.asarray(X, dtype=F32)
    y = np.asarray(y, dtype=np.int64)
    W = np.array(W, dtype=F32, copy=True)
    Wa = W.copy()                                  # global_model = deepcopy(model)  tools.py:180
    lr32, mu32, lam32 = F32(lr), F32(mu), F32(lam)
    n = len(y)
    avg = 0.0
    for _ in range(epoch):
        order = pass_order(n)
        s, cnt = 0.0, 0
        for b0 in range(0, n, batch_size):
            idx = order[b0:b0 + batch_size]
            xb, yb = X[idx], y[idx]
            bsz = len(idx)
            z = xb @ W.T
            logp = _log_softmax(z)
            ce = F32(-logp[np.arange(bsz), yb].mean(dtype=F32))
            g = np.exp(logp).astype(F32)
            g[np.arange(bsz), yb] -= F32(1.0)
            g /= F32(bsz)
            grad = (g.T @ xb).astype(F32)
            loss = ce
            if prox:
                dw = W - Wa
                pn = F32(np.sqrt(np.sum(dw * dw, dtype=F32)))
                loss = F32(loss + mu32 * pn)
                if pn > 0:
                    grad = grad + mu32 * (dw / pn)
            if reg:
                wn = F32(np.sqrt(np.sum(W * W, dtype=F32)))
                loss = F32(loss + lam32 * wn)
                if wn > 0:
                    grad = grad + lam32 * (W / wn)
            W = (W - lr32 * grad.astype(F32)).astype(F32)
            s += float(loss) * bsz
            cnt += bsz
        avg = s / cnt if cnt else 0.0
    return W, avg


def test_eval(X, y, W, batch_size=32):
    """tools.py:218-237 (+ comp_accuracy tools.py:82-96, Meter tools.py:99-148).

    Shuffled batches of ``batch_size``; loss = sum_b CE_mean_b*|b| / n,
    acc = sum_b (100*correct_b/|b|)*|b| / n  (percent, Q13).
    """
    X = np.asarray(X, dtype=F32)
    y = np.asarray(y, dtype=np.int64)
    n = len(y)
    order = pass_order(n)
    ls, acs, cnt = 0.0, 0.0, 0
    for b0 in range(0, n, batch_size):
        idx = order[b0:b0 + batch_size]
        xb, yb = X[idx], y[idx]
        bsz = len(idx)
        z = xb @ W.T
        logp = _log_softmax(z)
        ce = F32(-logp[np.arange(bsz), yb].mean(dtype=F32))
        correct = F32((z.argmax(axis=1) == yb).sum())
        acc = F32(correct * F32(100.0 / bsz))
        ls += float(ce) * bsz
        acs += float(acc) * bsz
        cnt += bsz
    return ls / cnt, acs / cnt


def aggregate(Ws, p):
    """tools.py:345-350: global = p0*W0 + p1*W1 + ... as a float32 left fold,
    every product and every sum rounded separately."""
    p = np.asarray(p, dtype=F32)
    acc = (Ws[0] * p[0]).astype(F32)
    for j in range(1, len(Ws)):
        acc = (acc + (p[j] * Ws[j]).astype(F32)).astype(F32)
    return acc


def mixture_solve(Ws, Xv, yv, p, buf, lr_p, epochs, batch_size=16, momentum=0.9):
    """tools.py:441-453: ``epochs`` passes of SGD(momentum) on p over the pooled
    validation set.  out[b,c] = sum_n p_n Z[n,c,b], Z[n,c,b] = W_n[c,:].x_b (Q7);
    buf = grad on the very first step (buf is None), else 0.9*buf + grad;
    p -= lr_p*buf.  ``buf`` persists across rounds (optimizer built once, tools.py:423).
    Returns (p, buf).
    """
    Xv = np.asarray(Xv, dtype=F32)
    W3 = np.stack(Ws, axis=0).astype(F32)          # [N, C, D]
    Z = np.einsum('ncd,vd->ncv', W3, Xv, optimize=True).astype(F32)   # [N, C, n_v]
    return mixture_solve_z(Z, yv, p, buf, lr_p, epochs, batch_size, momentum)


def mixture_solve_z(Z, yv, p, buf, lr_p, epochs, batch_size=16, momentum=0.9):
    """The p-SGD of ``mixture_solve`` on precomputed validation logits Z [N, C, n_v]
    (tools.py:448 with the inner matmul hoisted, Q7) -- lets a check at large N x D feed the
    GPU's own Z (itself checked separately) instead of recomputing the D-wide GEMM here."""
    Zt = np.ascontiguousarray(np.asarray(Z, dtype=F32).transpose(2, 0, 1))   # [n_v, N, C]: batch rows gather whole
    yv = np.asarray(yv, dtype=np.int64)
    p = np.array(p, dtype=F32, copy=True)
    lr32, mom32 = F32(lr_p), F32(momentum)
    nv = len(yv)
    for _ in range(epochs):
        order = pass_order(nv)
        for b0 in range(0, nv, batch_size):
            idx = order[b0:b0 + batch_size]
            bsz = len(idx)
            zb = Zt[idx]                            # [b, N, C]
            out = np.einsum('bnc,n->bc', zb, p).astype(F32)
            logp = _log_softmax(out)
            g = np.exp(logp).astype(F32)
            g[np.arange(bsz), yv[idx]] -= F32(1.0)
            g /= F32(bsz)
            gp = np.einsum('bc,bnc->n', g, zb).astype(F32)
            buf = gp.copy() if buf is None else (mom32 * buf + gp).astype(F32)
            p = (p - lr32 * buf).astype(F32)
    return p, buf


# --------------------------------------------------------------------------- #
# round drivers
# --------------------------------------------------------------------------- #
def _as_np_list(xs, dtype):
    return [np.asarray(x.numpy() if isinstance(x, torch.Tensor) else x, dtype=dtype) for x in xs]


def _weights(ys):
    num = np.array([len(y) for y in ys])
    return (num / sum(num)).astype(F32)


def _local_round(Xs, ys, Wg, lr, epoch, batch_size, prox, mu, reg, lam, clients):
    Ws, losses = [], []
    W = Wg
    for X, y in zip(Xs, ys):
        start = Wg if clients == 'parallel' else W
        W, l = train_client(X, y, start, lr, epoch, batch_size, prox, mu, reg, lam)
        Ws.append(W)
        losses.append(l)
    return Ws, losses


def FedAvg(X_train, y_train, X_test, y_test, type='classification', num_classes=10, D=200,
           lr=0.01, epoch=2, batch_size=32, prox=False, mu=0.1, lambda_reg_if=False,
           lambda_reg=0.01, round=100, clients='sequential'):
    """tools.py:329-353 (FedProx = same with prox=True, tools.py:356-380).

    Returns (train_loss[R], test_loss[R], test_acc[R], trace) with
    trace = {'W': [R, C, D] global weights after each round}.
    """
    Xs = _as_np_list(X_train, F32)
    ys = _as_np_list(y_train, np.int64)
    Xt = np.asarray(X_test, dtype=F32)
    yt = np.asarray(y_test, dtype=np.int64)
    Wg = mlp_init(D, num_classes)
    p = _weights(ys)
    tr = np.zeros(round, F32)
    tl = np.zeros(round, F32)
    ta = np.zeros(round, F32)
    Wtr = []
    for t in range(round):
        lr = lr_schedule(t, lr, round)
        Ws, losses = _local_round(Xs, ys, Wg, lr, epoch, batch_size, prox, mu,
                                  lambda_reg_if, lambda_reg, clients)
        tr[t] = np.sum(p * np.asarray(losses, dtype=F32), dtype=F32)
        Wg = aggregate(Ws, p)
        Wtr.append(Wg.copy())
        tl[t], ta[t] = test_eval(Xt, yt, Wg, batch_size)
    return tr, tl, ta, {'W': np.stack(Wtr)}


def FedProx(X_train, y_train, X_test, y_test, type='classification', num_classes=10, D=200,
            lr=0.01, epoch=2, batch_size=32, prox=True, mu=0.1, lambda_reg_if=False,
            lambda_reg=0.01, round=100, clients='sequential'):
    """tools.py:356-380 -- FedAvg with prox defaulting to True."""
    return FedAvg(X_train, y_train, X_test, y_test, type, num_classes, D, lr, epoch, batch_size,
                  prox, mu, lambda_reg_if, lambda_reg, round, clients=clients)


def FedAMW(X_train, y_train, X_test, y_test, X_val, y_val, type='classification', num_classes=10,
           D=200, lr=0.01, epoch=2, batch_size=32, prox=False, mu=0.1, lambda_reg_if=True,
           lambda_reg=0.01, round=100, lr_p=5e-5, clients='sequential', val_batch_size=16):
    """tools.py:413-463.  The validation set is passed as arrays (the reference
    takes a DataLoader with batch 16 and shuffle=True, exp.py:98-99).

    Returns (train_loss, test_loss, test_acc, trace) with trace = {'W': [R,C,D], 'p': [R,N]}.
    """
    Xs = _as_np_list(X_train, F32)
    ys = _as_np_list(y_train, np.int64)
    Xt = np.asarray(X_test, dtype=F32)
    yt = np.asarray(y_test, dtype=np.int64)
    Xv = np.asarray(X_val, dtype=F32)
    yv = np.asarray(y_val, dtype=np.int64)
    Wg = mlp_init(D, num_classes)
    p = _weights(ys)
    buf = None
    tr = np.zeros(round, F32)
    tl = np.zeros(round, F32)
    ta = np.zeros(round, F32)
    Wtr, ptr = [], []
    for t in range(round):
        lr = lr_schedule(t, lr, round)
        Ws, losses = _local_round(Xs, ys, Wg, lr, epoch, batch_size, prox, mu,
                                  lambda_reg_if, lambda_reg, clients)
        tr[t] = np.sum(p * np.asarray(losses, dtype=F32), dtype=F32)     # tools.py:434 (old p)
        p, buf = mixture_solve(Ws, Xv, yv, p, buf, lr_p, round, val_batch_size)
        Wg = aggregate(Ws, p)
        Wtr.append(Wg.copy())
        ptr.append(p.copy())
        tl[t], ta[t] = test_eval(Xt, yt, Wg, batch_size)
    return tr, tl, ta, {'W': np.stack(Wtr), 'p': np.stack(ptr)}


# --------------------------------------------------------------------------- #
# single-shot algorithms -- tools.py:240-326
# --------------------------------------------------------------------------- #
def _chain(Xs, ys, W, lr, epoch, batch_size, prox, mu, reg, lam):
    """One shared ``model`` trained by every client in turn (tools.py:263-266, 284-287):
    client i starts from client i-1's weights, anchored (prox) to that start."""
    Ws, losses = [], []
    for X, y in zip(Xs, ys):
        W, l = train_client(X, y, W, lr, epoch, batch_size, prox, mu, reg, lam)
        Ws.append(W)
        losses.append(l)
    return Ws, losses


def Centralized(X_train, y_train, X_test, y_test, type='classification', num_classes=10, D=200, lr=0.01,
                epoch=200, batch_size=32, prox=False, mu=0.1, lambda_reg_if=False, lambda_reg=0.01):
    """tools.py:240-255: all clients' rows concatenated in client order, one train_loop of
    ``epoch`` epochs, one test_loop.  Returns (train_loss, test_loss, test_acc, trace)."""
    Xs = _as_np_list(X_train, F32)
    ys = _as_np_list(y_train, np.int64)
    W = mlp_init(D, num_classes)
    W, loss = train_client(np.concatenate(Xs), np.concatenate(ys), W, lr, epoch, batch_size, prox, mu,
                           lambda_reg_if, lambda_reg)
    tl, ta = test_eval(np.asarray(X_test, F32), np.asarray(y_test, np.int64), W, batch_size)
    return loss, tl, ta, {'W': W[None]}


def Distributed(X_train, y_train, X_test, y_test, type='classification', num_classes=10, D=200, lr=0.01,
                epoch=200, batch_size=32, prox=False, mu=0.1, lambda_reg_if=False, lambda_reg=0.01):
    """tools.py:258-276: chained local training of ``epoch`` epochs per client, one
    n_j-weighted aggregate (left fold), one test_loop."""
    Xs = _as_np_list(X_train, F32)
    ys = _as_np_list(y_train, np.int64)
    W = mlp_init(D, num_classes)
    p = _weights(ys)
    Ws, losses = _chain(Xs, ys, W, lr, epoch, batch_size, prox, mu, lambda_reg_if, lambda_reg)
    tr = np.sum(p * np.asarray(losses, dtype=F32), dtype=F32)                     # tools.py:268
    Wg = aggregate(Ws, p)
    tl, ta = test_eval(np.asarray(X_test, F32), np.asarray(y_test, np.int64), Wg, batch_size)
    return tr, tl, ta, {'W': Wg[None]}


def FedAMW_OneShot(X_train, y_train, X_test, y_test, X_val, y_val, type='classification', num_classes=10,
                   D=200, lr=0.01, epoch=200, batch_size=32, prox=False, mu=0.1, lambda_reg_if=True,
                   lambda_reg=0.01, round=100, lr_p=5e-5, val_batch_size=16):
    """tools.py:279-326: chained local training once; then ``round`` times: one pass of plain
    SGD (no momentum, tools.py:300) on p over the validation set, aggregate, test_loop.

    The aggregate compounds: ``global_weights = local_weights[0]`` aliases client
    0's state DICT (tools.py:317), ``*= p[0]`` scales its tensor in place and the fold rebinds the
    dict entry to the sum (tools.py:318-321), so from round 1 on the fold starts from the
    previous round's global model: W(t) = W(t-1) * p0(t) + sum_{j>0} p_j(t) W_j, with
    W(-1) = W_0.  The p-solve reads the stack taken before the loop (tools.py:293-297)."""
    Xs = _as_np_list(X_train, F32)
    ys = _as_np_list(y_train, np.int64)
    Xt = np.asarray(X_test, F32)
    yt = np.asarray(y_test, np.int64)
    W = mlp_init(D, num_classes)
    p = _weights(ys)
    Ws, losses = _chain(Xs, ys, W, lr, epoch, batch_size, prox, mu, lambda_reg_if, lambda_reg)
    tr = np.sum(p * np.asarray(losses, dtype=F32), dtype=F32)                     # tools.py:292 (initial p)
    S = Ws[0].copy()
    tl = np.zeros(round, F32)
    ta = np.zeros(round, F32)
    Wtr, ptr = [], []
    for t in range(round):
        p, _ = mixture_solve(Ws, X_val, y_val, p, None, lr_p, 1, val_batch_size, momentum=0.0)
        Wg = aggregate([(S * p[0]).astype(F32)] + Ws[1:], np.concatenate([[F32(1.0)], p[1:]]).astype(F32))
        S = Wg
        Wtr.append(Wg)
        ptr.append(p.copy())
        tl[t], ta[t] = test_eval(Xt, yt, Wg, batch_size)
    return tr, tl, ta, {'W': np.stack(Wtr), 'p': np.stack(ptr)}


# --------------------------------------------------------------------------- #
# random Fourier features -- tools.py:15-31
# --------------------------------------------------------------------------- #
def rff(d, sigma, D):
    """tools.py:15-19: W ~ N(0, sigma) (d x D) then b ~ U(0, 2pi) drawn as Uniform.sample((1, D))
    -> shape (1, D, 1) -> view(-1, D); Uniform.rsample is low + rand * (high - low)."""
    W = torch.normal(0, sigma, size=(d, D)).numpy()
    r = torch.rand(1, D, 1).numpy().reshape(1, D)
    b = (F32(0.0) + r * (F32(2 * torch.pi) - F32(0.0))).astype(F32)
    return W.astype(F32), b


def feature_map(X, W, b, D):
    """tools.py:27, 29: 1/sqrt(D) * cos(X W + b), in float32 (the float64 scale is a
    wrapped scalar: torch multiplies in the tensor's dtype)."""
    z = (np.asarray(X, F32) @ W + b).astype(F32)
    return (F32(1.0 / np.sqrt(D)) * np.cos(z)).astype(F32)


def feature_mapping(X_train, X_test, k_par=10, D=200, type='gaussian'):
    """tools.py:22-31: X_train is (P, n, d) (exp.py:63 passes P = 1); one RFF draw shared by
    train and test.  Non-gaussian types return the inputs unchanged."""
    if type != 'gaussian':
        return X_train, X_test
    X_train = np.asarray(X_train, F32)
    W, b = rff(X_train[0].shape[1], k_par, D)
    tr = np.stack([feature_map(x, W, b, D) for x in X_train])
    return tr, feature_map(X_test, W, b, D)


# --------------------------------------------------------------------------- #
# exp.py's data preparation -- exp.py:60-99,
# utils.py:314-349.  Restatements, pinned to the reference's own output: make_golden.py runs
# the reference's utils.py (with a torchvision stub) on synthetic LIBSVM files and records
# the partition, the full-batch order, the splits, feature heads and the heterogeneity
# (tests/golden/prep_*.npz, checked in tests/test_oracle_prep.py).
# --------------------------------------------------------------------------- #
def dirichlet_partition(labels, n_clients, alpha):
    """utils.py:314-349 (psizes = [1/n_clients] * n_clients, exp.py -> utils.py:125)."""
    labels = np.asarray(labels)
    K = len(set(labels.tolist()))
    N = len(labels)
    np.random.seed(2020)
    min_size = 0
    while min_size < 10:
        idx_batch = [[] for _ in range(n_clients)]
        for k in range(K):
            idx_k = np.where(labels == k)[0]
            np.random.shuffle(idx_k)
            prop = np.random.dirichlet(np.repeat(alpha, n_clients))
            prop = np.array([q * (len(b) < N / n_clients) for q, b in zip(prop, idx_batch)]) + 1 / len(idx_k)
            prop = prop / prop.sum()
            cut = (np.cumsum(prop) * len(idx_k)).astype(int)[:-1]
            idx_batch = [b + piece.tolist() for b, piece in zip(idx_batch, np.split(idx_k, cut))]
            min_size = min(len(b) for b in idx_batch)
    for b in idx_batch:
        np.random.shuffle(b)
    return idx_batch


def heterogeneity(phi_all, parts):
    """exp.py:66-74: sum_j n_j/n * ||Phi^T Phi / n - Phi_j^T Phi_j / n_j||_F (float32 matrices,
    float64 norms -- the checker's accumulation is more accurate than torch's)."""
    phi_all = np.asarray(phi_all, F32)
    n = len(phi_all)
    C = (phi_all.T @ phi_all).astype(F32) / F32(n)
    h = 0.0
    for idx in parts:
        X = phi_all[np.asarray(idx, dtype=np.int64)]
        Cj = (X.T @ X).astype(F32) / F32(len(X))
        h += len(X) / n * float(np.sqrt(np.sum(((C - Cj).astype(np.float64)) ** 2)))
    return h


def exp_prepare(X, y, Xt, yt, n_clients, alpha, k_par, D):
    """exp.py:60-99 on raw arrays (the loaded LIBSVM data): partition (numpy reseeded to
    2020), full-batch train pass (2 draws + randperm) and test pass (1 draw), RFF, per-client
    20/80 validation split (np.random.shuffle).  Call after torch.manual_seed(100) /
    np.random.seed(100).  Returns dict(parts, X_train, y_train, X_val, y_val, X_test, hete)."""
    parts = dirichlet_partition(y, n_clients, alpha)
    order = pass_order(len(y))                                          # exp.py:61
    pass_order(len(yt), shuffle=False)                                  # exp.py:62
    X, y = np.asarray(X, F32)[order], np.asarray(y)[order].astype(np.int64)
    tr, te = feature_mapping(X[None], Xt, k_par, D)
    phi = tr.reshape(-1, D)
    Xc = [phi[np.asarray(i, dtype=np.int64)] for i in parts]
    yc = [y[np.asarray(i, dtype=np.int64)] for i in parts]
    hete = heterogeneity(phi, parts)
    Xv, yv, Xs, ys = [], [], [], []
    for Xi, yi in zip(Xc, yc):
        r = np.arange(len(Xi))
        np.random.shuffle(r)
        cut = int(len(Xi) * 0.2)
        Xv.append(Xi[r[:cut]])
        yv.append(yi[r[:cut]])
        Xs.append(Xi[r[cut:]])
        ys.append(yi[r[cut:]])
    return dict(parts=parts, X_train=Xs, y_train=ys, X_val=np.concatenate(Xv), y_val=np.concatenate(yv),
                X_test=te, hete=hete, X_clients=Xc)
