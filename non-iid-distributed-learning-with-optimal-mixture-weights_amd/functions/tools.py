"""Drop-in FedAvg / FedProx / FedAMW on MI355X.

Same names, positional signatures, defaults and return values as the reference
(/root/reference/functions/tools.py:329, 356, 413):

    train_loss, test_loss, test_acc = FedAvg(X_train, y_train, X_test, y_test, type,
                                             num_classes, D, lr, epoch, batch_size, prox,
                                             mu, lambda_reg_if, lambda_reg, round)

* ``X_train`` / ``y_train``: per-client lists of feature matrices [n_j, D] (fp32) and
  integer labels, on CPU or GPU; ``X_test`` / ``y_test`` likewise; FedAMW takes the
  reference's ``validloader`` (a DataLoader over a TensorDataset, batch 16, shuffle).
* Returns three CPU float32 tensors of length ``round``; ``test_acc`` is in percent.
  One ``Test loss: ..., \\t Test Acc: ...`` line per round is printed (tools.py:236),
  after the last round (the run is not synchronised per round).
* The global torch CPU generator is consumed exactly as the reference consumes it
  (MLP init, every DataLoader pass), so seeds and shuffles line up draw for draw.

Keyword-only extensions (not in the reference):
* ``clients='sequential'`` (default) -- the reference's semantics: the clients of a
  round are chained (client i starts from client i-1's trained weights and its
  FedProx anchor is that start); runs as one workgroup walking the chain.
  ``clients='parallel'`` -- every client starts from the round's global model (and is
  anchored to it); clients train concurrently, one workgroup each, and shard across
  GPUs when a torch.distributed process group is initialised.
* ``stats`` -- a dict that receives the final global model (and, with
  ``stats={'trace': True}``, the global model after every round in ``'W_rounds'``).

All arithmetic of the round runs in the gfx950 kernels of libfedsim.so; there is no
CPU path.  ``type`` must be 'classification' (the reference's MSE branch,
tools.py:183-184, is not on the benchmarked path).
"""
import numpy as np
import torch

from .. import dist, engine, rng
from .. import _lib
from .._lib import FedsimError

__all__ = ['FedAvg', 'FedProx', 'FedAMW', 'Federation', 'update_learning_rate', 'init_weights']


def update_learning_rate(epoch, target_lr, T):
    """tools.py:43-61 (callers rebind lr, so the decay compounds: lr0, lr0/10, lr0/1000)."""
    if epoch == int(T / 2):
        return target_lr / 10
    if epoch == int(T * 0.75):
        return target_lr / 100
    return target_lr


def init_weights(D, C):
    """MLP(D, C) initialisation (tools.py:34-40): nn.Linear's Kaiming-uniform draw
    (discarded) then xavier_uniform_, on the global CPU generator -> [C, D] fp32."""
    w = torch.empty(C, D)
    torch.nn.init.kaiming_uniform_(w, a=5 ** 0.5)
    torch.nn.init.xavier_uniform_(w)
    return w


def _device():
    if not torch.cuda.is_available():
        raise FedsimError('fedamw_amd needs a ROCm GPU (MI355X); there is no CPU fallback')
    return torch.device('cuda', torch.cuda.current_device())


def _check_inputs(type, X_train, y_train, num_classes, batch_size, epoch, round):
    if type != 'classification':
        raise NotImplementedError("only type='classification' is implemented (tools.py:181-184 MSE branch "
                                  "is out of scope)")
    if len(X_train) != len(y_train) or len(y_train) == 0:
        raise ValueError('X_train and y_train must be equal-length non-empty lists')
    for y in y_train:
        if len(y) == 0:
            # torch.utils.data.RandomSampler rejects an empty dataset (raised inside train_loop)
            raise ValueError('num_samples should be a positive integer value, but got num_samples=0')
    if not (1 <= num_classes <= 32):
        raise NotImplementedError('num_classes must be in [1, 32]')
    if not (1 <= batch_size <= 64):
        raise NotImplementedError('batch_size must be in [1, 64]')
    if epoch < 1 or round < 0:
        raise ValueError('epoch must be >= 1 and round >= 0')


class Federation:
    """One algorithm call split into setup / rounds / results (bench.py drives the
    rounds one at a time through the same code path as the drop-ins)."""

    def __init__(self, algo, X_train, y_train, X_test, y_test, validloader, type, num_classes, D, lr, epoch,
                 batch_size, prox, mu, lambda_reg_if, lambda_reg, round, lr_p, clients, stats=None, verbose=True,
                 shuffle_device=True):
        _check_inputs(type, X_train, y_train, num_classes, batch_size, epoch, round)
        if clients not in ('sequential', 'parallel'):
            raise ValueError("clients must be 'sequential' or 'parallel'")
        dev = _device()
        self.algo, self.stats, self.verbose = algo, stats, verbose
        self.C, self.E, self.B, self.R, self.D = int(num_classes), int(epoch), int(batch_size), int(round), int(D)
        self.lr, self.lr_p, self.prox, self.mu, self.reg, self.lam = lr, lr_p, prox, mu, lambda_reg_if, lambda_reg
        C, E, B, R = self.C, self.E, self.B, self.R
        N = len(y_train)
        self.N = N
        ns = np.array([len(y) for y in y_train], dtype=np.int64)
        self.ns = ns
        self.chained = clients == 'sequential'
        self.rank, nranks = dist.world()
        self.sharded = (not self.chained) and nranks > 1
        self.shards = dist.shard_lpt(dist.client_work(ns, E, B), nranks) if self.sharded else [np.arange(N)]
        self.mine = self.shards[self.rank] if self.sharded else self.shards[0]
        mine = self.mine

        # model init + mixture weights exactly as the reference (tools.py:330-333, 414-417)
        W_init = init_weights(D, C)
        self.p_all = torch.tensor(ns / sum(ns), dtype=torch.float32)

        self.feats = engine.Features([torch.as_tensor(X_train[j]) for j in mine],
                                     [torch.as_tensor(y_train[j]) for j in mine], D, dev)
        ld = self.ld = self.feats.ld
        self.trainer = engine.LocalTrainer(self.feats, C, B, E, chained=self.chained)
        self.evaluator = engine.Evaluator(X_test, y_test, D, C, dev, ld)
        self.W_g = torch.zeros(C, ld, device=dev, dtype=torch.float32)
        self.W_g[:, :D].copy_(W_init)
        p_dev = self.p_all.to(dev)
        self.p_mine = p_dev[torch.from_numpy(mine).to(dev)] if self.sharded else p_dev
        self.mixture = None
        self.inv = (torch.from_numpy(np.argsort(np.concatenate(self.shards), kind='stable')).to(dev)
                    if self.sharded else None)
        if algo == 'fedamw':
            Xv, yv = validloader.dataset.tensors[:2]
            Bv = int(validloader.batch_size)
            if not isinstance(validloader.sampler, torch.utils.data.RandomSampler):
                raise NotImplementedError('validloader must shuffle (exp.py:99)')
            self.mixture = engine.Mixture(Xv, yv, D, C, N, Bv, self.p_all, dev, ld)
            self.agg = engine.Aggregator(N, C, ld, dev)
            self.p_hist = torch.empty(R, N, dtype=torch.float32, device=dev)
        else:
            self.agg = engine.Aggregator(len(mine), C, ld, dev)
        self.loss_hist = torch.empty(R, len(mine), dtype=torch.float64, device=dev)
        self.eval_hist = torch.empty(R, 2, dtype=torch.float64, device=dev)
        self.W_hist = torch.empty(R, C, ld, device=dev) if (stats is not None and stats.get('trace')) else None
        self.n_val_pass = R if algo == 'fedamw' else 0
        self.side = torch.cuda.Stream(device=dev)    # FedAMW validation shuffles of round t+1 run here
        # the native round driver (csrc/round.hip): one call per round phase, training shuffles
        # replayed into a double-buffered slot on its side stream
        self.plan = engine.RoundPlan(self.trainer, self.W_g, self.loss_hist, p=self.p_mine,
                                     aggregator=self.agg if self.mixture is None else None,
                                     evaluator=self.evaluator, eval_hist=self.eval_hist, prox=prox, mu=mu,
                                     reg=lambda_reg_if, lam=lambda_reg, chained=self.chained,
                                     shuffle_device=shuffle_device)
        self.t = 0
        self.on_local_train = None      # optional (before, after) hooks around the local-training launch

    def _prepare(self, t):
        """Draw round t's shuffle seeds (torch's global CPU generator, in the reference's
        order: train passes client-major, then validation passes, then the test pass), replay
        the training shuffles into the plan's slot t % 2 (on its side stream) and enqueue the validation shuffles (FedAMW) on the side stream."""
        N, E = self.N, self.E
        seeds = rng.draw_pass_seeds(N * E + self.n_val_pass + 1)
        self.plan.shuffle(seeds[:N * E].reshape(N, E)[self.mine].reshape(-1), t)
        if self.mixture is not None:
            self.mixture.prepare(seeds[N * E:N * E + self.n_val_pass], t % 2, self.side)

    def round(self):
        """Run round t (tools.py:337-352 / 364-379 / 427-462) -- all launches async.  Round
        t+1's seeds are drawn (and its shuffles replayed) after round t is
        enqueued, so the host work overlaps the GPU; the draw pattern is data-independent,
        so this leaves the generator exactly where the reference leaves it after each call."""
        t = self.t
        if t == 0:
            self._prepare(0)
        self.lr = update_learning_rate(t, self.lr, self.R)
        P = _lib.PHASE_TRAIN, _lib.PHASE_AGGREGATE, _lib.PHASE_EVAL
        if self.on_local_train:
            self.on_local_train[0]()
        self.plan.round(t, self.lr, P[0])
        if self.on_local_train:
            self.on_local_train[1]()
        if self.mixture is not None:
            self.p_hist[t].copy_(self.mixture.p)
            W_all = self.trainer.W_out
            if self.sharded:
                W_all = dist.allgather_rows(W_all, [len(s) for s in self.shards])[self.inv]
            p = self.mixture.solve(W_all, None, self.lr_p, slot=t % 2)
            self.agg.run(W_all, p, self.W_g)
            self.plan.round(t, self.lr, P[2])
        elif self.sharded:
            self.plan.round(t, self.lr, P[1])
            dist.allreduce_sum_(self.W_g)
            self.plan.round(t, self.lr, P[2])
        else:
            self.plan.round(t, self.lr, P[1] | P[2])
        if self.W_hist is not None:
            self.W_hist[t].copy_(self.W_g)
        self.t += 1
        if self.t < self.R:
            self._prepare(self.t)

    def results(self):
        """Single host sync: (train_loss, test_loss, test_acc) CPU float32 tensors."""
        R, D = self.t, self.D
        self.trainer.check_errors()
        loss_hist = self.loss_hist[:R]
        if self.sharded:
            loss_hist = dist.allgather_rows(loss_hist.t().contiguous(), [len(s) for s in self.shards]).t()
            loss_hist = loss_hist[:, self.inv]
        lh = loss_hist.cpu().numpy()
        ev = self.eval_hist[:R].cpu().numpy()
        ph = self.p_hist[:R].cpu() if self.mixture is not None else None
        train_loss, test_loss, test_acc = torch.zeros(self.R), torch.zeros(self.R), torch.zeros(self.R)
        for t in range(R):
            pt = ph[t] if ph is not None else self.p_all
            train_loss[t] = torch.sum(pt * torch.tensor([float(v) for v in lh[t]]))   # tools.py:344 / 434
            test_loss[t], test_acc[t] = float(ev[t, 0]), float(ev[t, 1])
            if self.verbose and self.rank == 0:
                print('Test loss: {}, \t Test Acc: {}'.format(float(ev[t, 0]), float(ev[t, 1])))
        if self.stats is not None:
            self.stats.update(W_global=self.W_g[:, :D].detach().clone(), N=self.N, local_clients=len(self.mine),
                              ld=self.ld)
            if self.W_hist is not None:
                self.stats['W_rounds'] = self.W_hist[:R, :, :D].cpu().numpy()
            if self.mixture is not None:
                self.stats['p'] = self.mixture.p.detach().clone()
        return train_loss, test_loss, test_acc


def _run(algo, *args, stats=None, verbose=True):
    fed = Federation(algo, *args, stats=stats, verbose=verbose)
    for _ in range(fed.R):
        fed.round()
    return fed.results()


def FedAvg(X_train, y_train, X_test, y_test, type='classification', num_classes=10, D=200, lr=0.01, epoch=2,
           batch_size=32, prox=False, mu=0.1, lambda_reg_if=False, lambda_reg=0.01, round=100, *,
           clients='sequential', stats=None, verbose=True):
    """tools.py:329-353."""
    return _run('fedavg', X_train, y_train, X_test, y_test, None, type, num_classes, D, lr, epoch, batch_size,
                prox, mu, lambda_reg_if, lambda_reg, round, None, clients, stats=stats, verbose=verbose)


def FedProx(X_train, y_train, X_test, y_test, type='classification', num_classes=10, D=200, lr=0.01, epoch=2,
            batch_size=32, prox=True, mu=0.1, lambda_reg_if=False, lambda_reg=0.01, round=100, *,
            clients='sequential', stats=None, verbose=True):
    """tools.py:356-380 (FedAvg with the proximal term on by default)."""
    return _run('fedprox', X_train, y_train, X_test, y_test, None, type, num_classes, D, lr, epoch, batch_size,
                prox, mu, lambda_reg_if, lambda_reg, round, None, clients, stats=stats, verbose=verbose)


def FedAMW(X_train, y_train, X_test, y_test, validloader, type='classification', num_classes=10, D=200, lr=0.01,
           epoch=2, batch_size=32, prox=False, mu=0.1, lambda_reg_if=True, lambda_reg=0.01, round=100, lr_p=5e-5,
           *, clients='sequential', stats=None, verbose=True):
    """tools.py:413-463: FedAvg-style round + learned mixture weights p (SGD momentum 0.9
    on the pooled validation set, ``round`` inner epochs per round), aggregate with p."""
    return _run('fedamw', X_train, y_train, X_test, y_test, validloader, type, num_classes, D, lr, epoch,
                batch_size, prox, mu, lambda_reg_if, lambda_reg, round, lr_p, clients, stats=stats, verbose=verbose)
