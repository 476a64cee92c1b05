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

__all__ = ['FedAvg', 'FedProx', 'FedAMW', 'Centralized', 'Distributed', 'FedAMW_OneShot', 'Federation', 'RFF',
           'feature_mapping', 'update_learning_rate', 'init_weights']


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


def _check_labels(ys, num_classes, what):
    """Every label in [0, num_classes): the kernels index class rows by label, and the
    reference's CrossEntropyLoss raises on an out-of-range target."""
    for y in ys:
        y = torch.as_tensor(y)
        if y.numel() and (int(y.min()) < 0 or int(y.max()) >= num_classes):
            raise ValueError('%s labels must lie in [0, %d), got [%d, %d]' % (what, num_classes, int(y.min()),
                                                                              int(y.max())))


def _check_inputs(type, X_train, y_train, num_classes, batch_size, epoch, round, y_test=None, y_val=None,
                  train_labels=True):
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
    if train_labels:
        _check_labels(y_train, num_classes, 'training')
    if y_test is not None:
        _check_labels([y_test], num_classes, 'test')
    if y_val is not None:
        _check_labels([y_val], num_classes, 'validation')


# scheduling options of a Federation (how the launches of the rounds are arranged; none of
# them changes a result bit):
#   shuffle_chunk   FedAvg / FedProx with device-replayed shuffles: the shuffles of this many
#                   rounds come from one launch, one chunk ahead (1 = per round)
#   defer_eval      round t's test evaluation rides on round t+1's training launch where that
#                   launch leaves CUs idle (FS_PHASE_EVAL_DEFER)
#   fedamw_shuffle  'early': FedAMW's round t+1 shuffles run beside the Z GEMM; 'late': after
#                   the round, beside the p-solve
OPTIONS = {'shuffle_chunk': 8, 'defer_eval': True, 'fedamw_shuffle': 'early'}


class Federation:
    """One algorithm call split into setup / rounds / results (bench.py drives the
    rounds one at a time through the same code path as the drop-ins)."""

    def __init__(self, algo, X_train, y_train, X_test, y_test, validloader, type, num_classes, D, lr, epoch,
                 batch_size, prox, mu, lambda_reg_if, lambda_reg, round, lr_p, clients, stats=None, verbose=True,
                 shuffle_device=True, options=None):
        opts = dict(OPTIONS)
        for k, v in (options or {}).items():
            if k not in opts:
                raise ValueError('unknown Federation option %r (known: %s)' % (k, ', '.join(sorted(OPTIONS))))
            opts[k] = v
        if opts['fedamw_shuffle'] not in ('early', 'late'):
            raise ValueError("fedamw_shuffle must be 'early' or 'late'")
        self.options = opts
        # (training labels: only this rank's clients, below -- in sharded mode the other ranks'
        # entries of X_train / y_train need only have the right lengths)
        _check_inputs(type, X_train, y_train, num_classes, batch_size, epoch, round, y_test,
                      validloader.dataset.tensors[1] if validloader is not None else None, train_labels=False)
        if clients not in ('sequential', 'parallel'):
            raise ValueError("clients must be 'sequential' or 'parallel'")
        self.chained = clients == 'sequential'
        self.rank, nranks = dist.world()
        self.sharded = (not self.chained) and nranks > 1
        if self.sharded and len(y_train) < nranks:
            raise ValueError("clients='parallel' over %d ranks needs at least one client per rank (got %d clients)"
                             % (nranks, len(y_train)))
        self.algo, self.stats, self.verbose = algo, stats, verbose
        self.C, self.E, self.B, self.R, self.D = int(num_classes), int(epoch), int(batch_size), int(round), int(D)
        self.lr, self.lr_p, self.prox, self.mu, self.reg, self.lam = lr, lr_p, prox, mu, lambda_reg_if, lambda_reg
        C, E, B, R = self.C, self.E, self.B, self.R
        N = len(y_train)
        self.N = N
        ns = np.array([len(y) for y in y_train], dtype=np.int64)
        self.ns = ns
        self.shards = dist.shard_lpt(dist.client_work(ns, E, B), nranks) if self.sharded else [np.arange(N)]
        self.mine = self.shards[self.rank] if self.sharded else self.shards[0]
        mine = self.mine
        _check_labels([y_train[j] for j in mine], num_classes, 'training')
        dev = _device()

        # model init + mixture weights exactly as the reference (tools.py:330-333, 414-417)
        W_init = init_weights(D, C)
        self.p_all = torch.tensor(ns / sum(ns), dtype=torch.float32)

        self.feats = engine.Features([torch.as_tensor(X_train[j]) for j in mine],
                                     [torch.as_tensor(y_train[j]) for j in mine], D, dev)
        ld = self.ld = self.feats.ld
        # sharded FedAMW: the p-solve's client axis is rank-major blocks of L columns (dist.py)
        self.zshard = algo == 'fedamw' and self.sharded
        if self.zshard:
            self.L, self.pos = dist.solver_layout(self.shards)
            self.pos_dev = torch.from_numpy(self.pos).to(dev)
        self.trainer = engine.LocalTrainer(self.feats, C, B, E, chained=self.chained,
                                           rows=self.L if self.zshard else None, prox=prox)
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
            if self.zshard:
                Ns = nranks * self.L
                p0 = torch.zeros(Ns, dtype=torch.float32)
                p0[torch.from_numpy(self.pos)] = self.p_all
                self.mixture = engine.Mixture(Xv, yv, D, C, Ns, Bv, p0, dev, ld)
                # the qmc solver reads the all-gathered rank blocks as they land (no layout copy);
                # which layout to gather is decided again every round, right before the
                # all-gather (round()), under the tuning the enqueueing thread has then
                self.nranks = nranks
                self.Z_local = torch.empty(self.mixture.nv, C * self.L, device=dev, dtype=torch.float32)
                lo = self.rank * self.L
                self.p_slice = lambda p: p[lo:lo + len(mine)]
                self.agg = engine.Aggregator(len(mine), C, ld, dev)
            else:
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
                                     shuffle_device=shuffle_device, shuffle_after_train=self.mixture is not None)
        # FedAMW: round t+1's shuffles (training and validation passes) are generated behind
        # round t's local training, beside its p-solve (one to 32 CUs busy), not beside the
        # training kernel, whose groups would wait for the CUs they hold
        # FedAvg / FedProx with device-replayed shuffles: generate them K rounds per launch
        # (options['shuffle_chunk'], default 8; 1 = per round), one chunk ahead of the rounds that
        # use them, so consecutive rounds run with no cross-stream wait between them.  FedAMW
        # keeps per-round shuffles (its validation shuffles are double-buffered per round).
        self.chunk = 1
        if self.mixture is None and shuffle_device:
            self.chunk = max(1, min(int(opts['shuffle_chunk']), R))
            if self.chunk > 1:
                self.plan.set_chunk(self.chunk)
        # round t's test-set evaluation is deferred into round t+1's training launch when that
        # launch leaves CUs idle (options['defer_eval'] = False: an evaluation launch per round)
        self.defer_eval = bool(opts['defer_eval'])
        self._prepared = 0              # next round whose shuffles are to be prepared
        self._train_done = None
        self.t = 0
        self.events = None              # a list: round() appends (phase, start, end) HIP timing events

    def _prepare(self, t):
        """Draw round t's shuffle seeds (torch's global CPU generator, in the reference's
        order: train passes client-major, then validation passes, then the test pass), replay
        the training shuffles into the plan's slot t % 2 (on its side stream) and enqueue the validation shuffles (FedAMW) on the side stream."""
        N, E = self.N, self.E
        seeds = rng.draw_pass_seeds(N * E + self.n_val_pass + 1)
        self.plan.shuffle(seeds[:N * E].reshape(N, E)[self.mine].reshape(-1), t)
        if self.mixture is not None:
            if self._train_done is not None:
                self.side.wait_event(self._train_done)
            self.mixture.prepare(seeds[N * E:N * E + self.n_val_pass], t % 2, self.side)

    def _prepare_upto(self, end):
        """Prepare the shuffles of every round before ``min(end, R)`` not prepared yet, in order."""
        while self._prepared < min(end, self.R):
            self._prepare(self._prepared)
            self._prepared += 1
            if self._prepared == self.R and self.chunk > 1:
                self.plan.flush()

    def round(self):
        """Run round t (tools.py:337-352 / 364-379 / 427-462) -- all launches async.  Round
        t+1's seeds are drawn (and its shuffles replayed) after round t is
        enqueued, so the host work overlaps the GPU; the draw pattern is data-independent,
        so this leaves the generator exactly where the reference leaves it after each call."""
        t = self.t
        if t == 0:
            self._prepare_upto(2 * self.chunk if self.chunk > 1 else 1)
        self.lr = update_learning_rate(t, self.lr, self.R)
        P = _lib.PHASE_TRAIN, _lib.PHASE_AGGREGATE, _lib.PHASE_EVAL
        if t + 1 < self.R and self.defer_eval:
            # this round's evaluation rides on round t+1's training launch where that launch
            # leaves CUs idle (fs_plan_round, FS_PHASE_EVAL_DEFER); same arithmetic per row
            P = P[0], P[1], P[2] | _lib.PHASE_EVAL_DEFER
        ev = self.events

        def timed(name, fn):
            if ev is None:
                return fn()
            a, b = _lib.Timer(), _lib.Timer()     # no system-scope release (fs_timer_*)
            a.record()
            out = fn()
            b.record()
            ev.append((name, a, b))
            return out

        timed('train', lambda: self.plan.round(t, self.lr, P[0]))
        early = False
        if self.mixture is not None:
            self._train_done = torch.cuda.Event()
            self._train_done.record()
            # FedAMW: round t+1's shuffles are enqueued now (nothing else draws from the global
            # generator in between, so the draw order is unchanged) and the p-solve waits for the
            # validation shuffles: they run beside the Z GEMM, not on the CUs of the p-solve's
            # workgroups (options['fedamw_shuffle'] = 'late': after the round, beside the p-solve)
            early = self.t + 1 < self.R and self.options['fedamw_shuffle'] != 'late'
            if early:
                self._prepare_upto(t + 2)
        if self.zshard:
            # tools.py:435-453 sharded: this rank's Z columns, one all-gather, the replicated
            # p-solve, then this rank's partial aggregate with its learned p and one all-reduce
            self.p_hist[t].copy_(self.mixture.p[self.pos_dev])
            # the blocked layout only where fs_mix_solve_blocked covers the shape under THIS
            # thread's tuning now (a tuning change between rounds, or a round
            # enqueued from another thread, must not leave a blocked Z for a solver that
            # cannot read it)
            self.mixture.blocks = (self.nranks if self.nranks > 1 and self.mixture.blocked_covers(self.R) else 1)
            timed('z', lambda: self.mixture.z_block(self.trainer.W_out, self.L, self.Z_local))
            timed('z_allgather', lambda: dist.allgather_z(self.Z_local, self.C, self.mixture.Z,
                                                          blocked=self.mixture.blocks > 1))
            if early:
                torch.cuda.current_stream().wait_stream(self.side)
            p = timed('solve', lambda: self.mixture.solve(None, None, self.lr_p, slot=t % 2, z=False))
            self.agg.run(self.trainer.W_out, self.p_slice(p), self.W_g)
            dist.allreduce_sum_(self.W_g)
            self.plan.round(t, self.lr, P[2])
        elif self.mixture is not None:
            self.p_hist[t].copy_(self.mixture.p)
            timed('z', lambda: self.mixture.z_block(self.trainer.W_out, self.N, self.mixture.Z))
            if early:
                torch.cuda.current_stream().wait_stream(self.side)
            p = timed('solve', lambda: self.mixture.solve(None, None, self.lr_p, slot=t % 2, z=False))
            self.agg.run(self.trainer.W_out, p, self.W_g)
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
        if self.chunk > 1:
            if t % self.chunk == 0 and t >= self.chunk:      # chunk c started: prepare chunk c + 1
                self._prepare_upto(t + 2 * self.chunk)
        elif self.t < self.R and not early:
            self._prepare_upto(self.t + 1)

    def results(self):
        """Single host sync: (train_loss, test_loss, test_acc) CPU float32 tensors."""
        R, D = self.t, self.D
        if 0 < R and self.defer_eval:
            self.plan.eval_flush()                       # completes a deferred evaluation, if any (ABI 15)
        self.trainer.check_errors()
        if self.mixture is not None:
            self.mixture.check_errors()
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
                p = self.mixture.p[self.pos_dev] if self.zshard else self.mixture.p
                self.stats['p'] = p.detach().clone()
        return train_loss, test_loss, test_acc


def _run(algo, *args, stats=None, verbose=True, options=None):
    fed = Federation(algo, *args, stats=stats, verbose=verbose, options=options)
    for _ in range(fed.R):
        fed.round()
    return fed.results()


def FedAvg(X_train, y_train, X_test, y_test, type='classification', num_classes=10, D=200, lr=0.01, epoch=2,
           batch_size=32, prox=False, mu=0.1, lambda_reg_if=False, lambda_reg=0.01, round=100, *,
           clients='sequential', stats=None, verbose=True, options=None):
    """tools.py:329-353.  ``options``: launch-scheduling options (``OPTIONS``)."""
    return _run('fedavg', X_train, y_train, X_test, y_test, None, type, num_classes, D, lr, epoch, batch_size,
                prox, mu, lambda_reg_if, lambda_reg, round, None, clients, stats=stats, verbose=verbose,
                options=options)


def FedProx(X_train, y_train, X_test, y_test, type='classification', num_classes=10, D=200, lr=0.01, epoch=2,
            batch_size=32, prox=True, mu=0.1, lambda_reg_if=False, lambda_reg=0.01, round=100, *,
            clients='sequential', stats=None, verbose=True, options=None):
    """tools.py:356-380 (FedAvg with the proximal term on by default)."""
    return _run('fedprox', X_train, y_train, X_test, y_test, None, type, num_classes, D, lr, epoch, batch_size,
                prox, mu, lambda_reg_if, lambda_reg, round, None, clients, stats=stats, verbose=verbose,
                options=options)


def FedAMW(X_train, y_train, X_test, y_test, validloader, type='classification', num_classes=10, D=200, lr=0.01,
           epoch=2, batch_size=32, prox=False, mu=0.1, lambda_reg_if=True, lambda_reg=0.01, round=100, lr_p=5e-5,
           *, clients='sequential', stats=None, verbose=True, options=None):
    """tools.py:413-463: FedAvg-style round + learned mixture weights p (SGD momentum 0.9
    on the pooled validation set, ``round`` inner epochs per round), aggregate with p."""
    return _run('fedamw', X_train, y_train, X_test, y_test, validloader, type, num_classes, D, lr, epoch,
                batch_size, prox, mu, lambda_reg_if, lambda_reg, round, lr_p, clients, stats=stats, verbose=verbose,
                options=options)


# --------------------------------------------------------------------------- #
# Random Fourier features (tools.py:15-31)
# --------------------------------------------------------------------------- #
def RFF(d, sigma, D):
    """tools.py:15-19: W ~ N(0, sigma) [d, D], b ~ U(0, 2 pi) [1, D], drawn on torch's global
    CPU generator exactly as the reference draws them (Uniform.sample((1, D)) -> (1, D, 1) ->
    view), then placed on the GPU.

    RNG stream: this reproduces the reference run on a CPU-only host (device = cpu,
    tools.py:12), which is what the golden fixtures pin.  On a CUDA/ROCm host the reference
    draws W and b from the GPU generator instead and leaves the CPU stream untouched, so its
    later MLP inits and DataLoader shuffles are shifted by these d*D + D draws relative to
    this drop-in; that GPU-host stream is not reproduced (parity unpinned for it)."""
    m = torch.distributions.Uniform(torch.tensor([0.0]), torch.tensor([2 * torch.pi]))
    W = torch.normal(0, sigma, size=(d, D))
    b = m.sample((1, D)).view(-1, D)
    dev = _device()
    return W.to(dev), b.to(dev)


def feature_mapping(X_train, X_test, k_par=10, D=200, type='gaussian'):
    """tools.py:22-31: one RFF draw, then ``1/sqrt(D) * cos(X W + b)`` for every slice of
    ``X_train`` ([P, n, d]; exp.py:63 passes P = 1) and for ``X_test`` -- each map one
    fs_feature_map launch (MFMA GEMM with the cos epilogue fused).  Returns GPU tensors
    [P, n, D] and [n_t, D]; other ``type`` values return the inputs unchanged."""
    if type != 'gaussian':
        return X_train, X_test
    X_train = torch.as_tensor(X_train)
    W, b = RFF(X_train[0].shape[1], k_par, D)
    out = torch.empty(X_train.shape[0], X_train.shape[1], D, device=W.device, dtype=torch.float32)
    for i in range(len(X_train)):
        engine.feature_map(X_train[i], W, b, D, out=out[i])
    return out, engine.feature_map(X_test, W, b, D)


# --------------------------------------------------------------------------- #
# Single-shot algorithms (tools.py:240-326)
# --------------------------------------------------------------------------- #
def _chain_train(X_train, y_train, W_init, D, C, lr, epoch, batch_size, prox, mu, reg, lam, dev):
    """One shared model trained by the clients in turn (tools.py:263-266 / 284-287: train_loop
    mutates the one ``model``), each for ``epoch`` epochs and anchored (prox) to its start --
    one fs_local_train launch in chained mode.  Consumes the generator like the reference
    (epoch passes per client, client-major).  Returns (feats, W_out [N, C, ld], loss [N])."""
    feats = engine.Features([torch.as_tensor(x) for x in X_train], [torch.as_tensor(y) for y in y_train], D, dev)
    trainer = engine.LocalTrainer(feats, C, batch_size, epoch, chained=True, prox=prox)
    trainer.upload_perms(rng.draw_pass_seeds(trainer.N * epoch))
    W0 = torch.zeros(C, feats.ld, device=dev, dtype=torch.float32)
    W0[:, :D].copy_(W_init)
    W_out, loss = trainer.run(W0, lr, prox, mu, reg, lam, chained=True)
    return feats, trainer, W_out, loss


def _test(evaluator, W, out2):
    rng.draw_pass_seeds(1)                  # test_loop's shuffled pass (tools.py:219-220)
    evaluator.run(W, out2)


def _print_tests(ev, verbose):
    if verbose and dist.world()[0] == 0:
        for tl, ta in ev:
            print('Test loss: {}, \t Test Acc: {}'.format(float(tl), float(ta)))


def Centralized(X_train, y_train, X_test, y_test, type='classification', num_classes=10, D=200, lr=0.01,
                epoch=200, batch_size=32, prox=False, mu=0.1, lambda_reg_if=False, lambda_reg=0.01, *,
                stats=None, verbose=True):
    """tools.py:240-255: every client's rows concatenated (client order), ONE train_loop of
    ``epoch`` epochs (exp.py:116 passes local_epoch * Round), one test_loop.  Returns
    (train_loss, test_loss, test_acc) as Python floats, like the reference's Meter averages."""
    _check_inputs(type, X_train, y_train, num_classes, batch_size, epoch, 0, y_test)
    dev = _device()
    C = int(num_classes)
    W_init = init_weights(D, C)
    Xc = torch.cat([torch.as_tensor(x).to(dev, torch.float32) for x in X_train], 0)
    yc = torch.cat([torch.as_tensor(y).reshape(-1).to('cpu', torch.int64) for y in y_train], 0)
    feats, trainer, W_out, loss = _chain_train([Xc], [yc], W_init, D, C, lr, epoch, batch_size, prox, mu,
                                               lambda_reg_if, lambda_reg, dev)
    ev = engine.Evaluator(X_test, y_test, D, C, dev, feats.ld)
    out2 = torch.empty(2, dtype=torch.float64, device=dev)
    _test(ev, W_out[0], out2)
    trainer.check_errors()
    res = out2.cpu().numpy()
    _print_tests([res], verbose)
    if stats is not None:
        stats.update(W_global=W_out[0, :, :D].detach().clone())
    return float(loss[0].item()), float(res[0]), float(res[1])


def Distributed(X_train, y_train, X_test, y_test, type='classification', num_classes=10, D=200, lr=0.01,
                epoch=200, batch_size=32, prox=False, mu=0.1, lambda_reg_if=False, lambda_reg=0.01, *,
                stats=None, verbose=True):
    """tools.py:258-276: chained local training of ``epoch`` epochs per client, one
    n_j-weighted aggregate (fs_aggregate, the reference's left fold), one test_loop.  Returns
    (train_loss 0-dim fp32 tensor, test_loss float, test_acc float)."""
    _check_inputs(type, X_train, y_train, num_classes, batch_size, epoch, 0, y_test)
    dev = _device()
    C = int(num_classes)
    W_init = init_weights(D, C)
    ns = np.array([len(y) for y in y_train])
    p = torch.tensor(ns / sum(ns), dtype=torch.float32)
    feats, trainer, W_out, loss = _chain_train(X_train, y_train, W_init, D, C, lr, epoch, batch_size, prox, mu,
                                               lambda_reg_if, lambda_reg, dev)
    ld = feats.ld
    agg = engine.Aggregator(len(ns), C, ld, dev, chunks=1)
    W_g = torch.empty(C, ld, device=dev, dtype=torch.float32)
    agg.run(W_out, p.to(dev), W_g)
    ev = engine.Evaluator(X_test, y_test, D, C, dev, ld)
    out2 = torch.empty(2, dtype=torch.float64, device=dev)
    _test(ev, W_g, out2)
    trainer.check_errors()
    res = out2.cpu().numpy()
    train_loss = torch.sum(p * torch.tensor([float(v) for v in loss.cpu().numpy()]))    # tools.py:268
    _print_tests([res], verbose)
    if stats is not None:
        stats.update(W_global=W_g[:, :D].detach().clone())
    return train_loss, float(res[0]), float(res[1])


def FedAMW_OneShot(X_train, y_train, X_test, y_test, validloader, type='classification', num_classes=10, D=200,
                   lr=0.01, epoch=200, batch_size=32, prox=False, mu=0.1, lambda_reg_if=True, lambda_reg=0.01,
                   round=100, lr_p=5e-5, *, stats=None, verbose=True):
    """tools.py:279-326: chained local training once (``epoch`` epochs per client), then
    ``round`` times: one pass of plain SGD (no momentum, tools.py:300) on the mixture weights
    over the validation loader, aggregate, test_loop.  Z = the stacked client models applied
    to the validation set is computed once (fs_mix_z; the stack is fixed, tools.py:293-297).

    The reference's aggregate compounds: ``global_weights = local_weights[0]``
    aliases client 0's state dict, so from round 1 on the fold starts from the previous
    global model: W(t) = W(t-1) * p0(t) + sum_{j>0} p_j(t) W_j (W(-1) = W_0).  Reproduced with
    two fs_aggregate launches per round (a 1-client fold scales W(t-1) by p0(t) into row 0 of
    a copy of the clients x params buffer; the N-client fold with weight 1 on that row adds
    the rest), bitwise the reference's sequence of roundings.
    Returns (train_loss 0-dim fp32 tensor, test_loss [round], test_acc [round])."""
    _check_inputs(type, X_train, y_train, num_classes, batch_size, epoch, round, y_test,
                  validloader.dataset.tensors[1])
    dev = _device()
    C, R = int(num_classes), int(round)
    W_init = init_weights(D, C)
    ns = np.array([len(y) for y in y_train])
    N = len(ns)
    p0 = torch.tensor(ns / np.sum(ns), dtype=torch.float32)
    feats, trainer, W_out, loss = _chain_train(X_train, y_train, W_init, D, C, lr, epoch, batch_size, prox, mu,
                                               lambda_reg_if, lambda_reg, dev)
    ld = feats.ld
    Xv, yv = validloader.dataset.tensors[:2]
    if not isinstance(validloader.sampler, torch.utils.data.RandomSampler):
        raise NotImplementedError('validloader must shuffle (exp.py:99)')
    mix = engine.Mixture(Xv, yv, D, C, N, int(validloader.batch_size), p0, dev, ld, momentum=0.0)
    ev = engine.Evaluator(X_test, y_test, D, C, dev, ld)
    agg1 = engine.Aggregator(1, C, ld, dev, chunks=1)
    aggN = engine.Aggregator(N, C, ld, dev, chunks=1)
    W_agg = W_out.clone()                       # row 0 rewritten every round, rows 1.. = W_j
    W_prev = W_out[0].clone()
    q = torch.ones(N, dtype=torch.float32, device=dev)
    W_g = torch.empty(C, ld, device=dev, dtype=torch.float32)
    eval_hist = torch.empty(max(R, 1), 2, dtype=torch.float64, device=dev)
    p_hist = torch.empty(max(R, 1), N, dtype=torch.float32, device=dev)
    W_hist = torch.empty(R, C, ld, device=dev) if (stats is not None and stats.get('trace')) else None
    for t in range(R):
        seeds = rng.draw_pass_seeds(2)          # the validation pass, then test_loop's pass
        mix.solve(W_out, seeds[:1], lr_p, z=(t == 0))
        agg1.run(W_prev, mix.p, W_agg[0])       # W(t-1) * p0(t), in place in the reference
        if N > 1:
            q[1:].copy_(mix.p[1:])
        aggN.run(W_agg, q, W_g)
        W_prev.copy_(W_g)
        p_hist[t].copy_(mix.p)
        if W_hist is not None:
            W_hist[t].copy_(W_g)
        ev.run(W_g, eval_hist[t])
    trainer.check_errors()
    mix.check_errors()
    train_loss = torch.sum(p0 * torch.tensor([float(v) for v in loss.cpu().numpy()]))   # tools.py:292
    evh = eval_hist[:R].cpu().numpy()
    _print_tests(evh, verbose)
    test_loss = torch.tensor(evh[:, 0], dtype=torch.float32) if R else torch.zeros(0)
    test_acc = torch.tensor(evh[:, 1], dtype=torch.float32) if R else torch.zeros(0)
    if stats is not None:
        stats.update(W_global=W_g[:, :D].detach().clone(), p=mix.p.detach().clone())
        if stats.get('trace'):
            stats['p_rounds'] = p_hist[:R].cpu().numpy()
            stats['W_rounds'] = W_hist[:, :, :D].cpu().numpy()
    return train_loss, test_loss, test_acc
