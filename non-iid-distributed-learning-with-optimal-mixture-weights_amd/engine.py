"""Device-resident round engine: HBM layout + the launches of one federated round.

HBM layout (one GPU; see DESIGN.md "Data layout"):
  phi      [rows, ld]   fp32  all local clients' features, CSR by client (row_off), D zero-padded to ld % 64 == 0
  labels   [rows]       int32
  row_off  [N+1]        int64
  perms    [E*rows]     int32 this round's shuffles, client j epoch e at E*row_off[j] + e*n_j
  W_out    [N, C, ld]   fp32  the clients x params buffer (each client's trained weights)
  W_g      [C, ld]      fp32  global model
  Z        [n_val, C*ldN] fp32 FedAMW validation logits per client (row v, column c*ldN+n,
                             ldN = N rounded up to 4, padding columns 0)
Everything stays resident across rounds.  Per round the host draws the shuffle
seeds from torch's global CPU generator (one vectorised call) and uploads them
(pinned, double-buffered, async on the compute stream); the permutations themselves
are replayed on the GPU by fs_randperm_device.
"""
import numpy as np
import torch

from . import _lib


def pad_ld(D):
    return max(64, (int(D) + 63) // 64 * 64)


def _to_device_f32(xs, device):
    if len(xs) == 1:
        return xs[0].to(device=device, dtype=torch.float32, non_blocking=True)
    if all(x.is_cuda for x in xs):
        return torch.cat([x.to(device=device, dtype=torch.float32) for x in xs], 0)
    return torch.cat([x.detach().to('cpu', torch.float32) for x in xs], 0).to(device, non_blocking=True)


class Features:
    """Rows of features packed CSR-style in HBM (``phi[rows, ld]``) plus int32 labels."""

    def __init__(self, X_list, y_list, D, device, ld=None):
        self.device = device
        self.D = int(D)
        self.ld = ld or pad_ld(D)
        self.ns = np.array([int(len(y)) for y in y_list], dtype=np.int64)
        self.row_off = np.concatenate([[0], np.cumsum(self.ns)]).astype(np.int64)
        rows = int(self.row_off[-1])
        self.rows = rows
        for X in X_list:
            if X.dim() != 2 or X.shape[1] != self.D:
                raise ValueError('feature matrix must be [n, D=%d], got %s' % (self.D, tuple(X.shape)))
        self.phi = torch.zeros(max(rows, 1), self.ld, device=device, dtype=torch.float32)
        if rows:
            self.phi[:rows, :self.D].copy_(_to_device_f32([torch.as_tensor(x) for x in X_list], device))
            y = torch.cat([torch.as_tensor(v).reshape(-1).to('cpu', torch.int64) for v in y_list])
            self.labels = y.to(torch.int32).to(device)
        else:
            self.labels = torch.zeros(1, dtype=torch.int32, device=device)
        self.row_off_dev = torch.from_numpy(self.row_off).to(device)


class Shuffler:
    """Shuffles of a fixed set of passes (sizes ns, output offsets offs), replayed on the
    GPU from host-drawn seeds (fs_randperm_device), on whatever stream is current.

    Two output slots let round t+1's shuffles be generated on a side stream while round t
    trains (``prepare``), ordered by events: a slot is rewritten only after the kernel
    that consumed it has finished (``consumed``), and read only after it is ready."""

    def __init__(self, ns, offs, size, device, max_n=None):
        self.P = int(len(ns))
        # the launch contract (include/fedsim.h): max_n bounds every pass; a caller may pass a
        # smaller value only to exercise the error path (check_errors then raises)
        self.max_n = int(max_n) if max_n is not None else (int(np.max(ns)) if self.P else 0)
        self.err = torch.zeros(_lib.ERR_BLOCK // 4, dtype=torch.int32, device=device)
        self.n_dev = torch.as_tensor(np.asarray(ns, dtype=np.int64)).to(device)
        self.off_dev = torch.as_tensor(np.asarray(offs, dtype=np.int64)).to(device)
        self.bufs = [torch.empty(max(1, int(size)), dtype=torch.int32, device=device) for _ in range(2)]
        self.seed_dev = [torch.empty(max(1, self.P), dtype=torch.int64, device=device) for _ in range(2)]
        self.seed_host = [torch.empty(max(1, self.P), dtype=torch.int64, pin_memory=True) for _ in range(2)]
        self.host_free = [None, None]
        self.ready = [None, None]
        self.consumed = [None, None]

    def prepare(self, seeds, slot, stream=None):
        """Enqueue the shuffles for one round into ``bufs[slot]`` on ``stream`` (default: current)."""
        stream = stream or torch.cuda.current_stream()
        seeds = np.asarray(seeds, dtype=np.int64)
        assert seeds.shape == (self.P,)
        if self.host_free[slot] is not None:
            self.host_free[slot].synchronize()
        self.seed_host[slot].numpy()[:] = seeds
        if self.consumed[slot] is not None:
            stream.wait_event(self.consumed[slot])
        with torch.cuda.stream(stream):
            self.seed_dev[slot].copy_(self.seed_host[slot], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
            self.host_free[slot] = ev
            if self.P:
                _lib.check(_lib.lib().fs_randperm_device(_lib.ptr(self.seed_dev[slot]), _lib.ptr(self.n_dev),
                                                         _lib.ptr(self.off_dev), self.P, self.max_n,
                                                         _lib.ptr(self.bufs[slot]), _lib.ptr(self.err),
                                                         _lib.stream_ptr(stream)),
                           'fs_randperm_device')
            ready = torch.cuda.Event()
            ready.record(stream)
        self.ready[slot] = ready

    def acquire(self, slot):
        """Make the current stream wait for ``bufs[slot]`` and return it."""
        torch.cuda.current_stream().wait_event(self.ready[slot])
        return self.bufs[slot]

    def release(self, slot):
        """Mark ``bufs[slot]`` consumed by the work enqueued so far on the current stream."""
        ev = torch.cuda.Event()
        ev.record()
        self.consumed[slot] = ev

    def run(self, seeds, slot=0):
        """Synchronous-order convenience: prepare on the current stream and return the buffer."""
        self.prepare(seeds, slot)
        return self.acquire(slot)

    def check_errors(self):
        """Raise if a pass broke the max_n contract (it was written unshuffled; synchronises)."""
        err = int(self.err[0].item())
        if err:
            self.err.zero_()
            raise _lib.FedsimError('fs_randperm_device: a pass is longer than max_n = %d; it was written as the '
                                   'identity permutation (code %d)' % (self.max_n, err))


def _check_ws_error(ws, what):
    """Read (synchronising) and clear the sticky error word at the start of the workspace's
    last 256-byte block (include/fedsim.h); raise if a bounded cross-workgroup wait timed out."""
    if ws is None:
        return
    blk = ws[ws.numel() - _lib.ERR_BLOCK:]
    err = int(blk[:4].view(torch.int32).item())
    if err:
        blk.zero_()
        raise _lib.FedsimError('%s: a cross-workgroup hand-off timed out (code %d); results are invalid' % (what, err))


class LocalTrainer:
    """fs_local_train for a fixed set of clients; owns the clients x params buffer.

    ``split``: workgroups per client.  None asks fs_local_train_plan (a group of G
    workgroups splits each client's feature dimension whenever the shape allows, in parallel
    mode as persistent groups over the clients -- two clients per group in the pair form
    (G | _lib.G_PAIR) where the shape allows it -- in chained mode as one group walking the
    chain); 1 forces one workgroup per client, G a split width, G | _lib.G_PAIR the pair form,
    G | _lib.G_TEAMS the team form, G | _lib.G_PIPE the pipelined split form."""

    def __init__(self, feats, C, B, E, split=None, chained=False, rows=None, prox=False):
        self.f = feats
        self.C, self.B, self.E = int(C), int(B), int(E)
        dev = feats.device
        N = len(feats.ns)
        self.N = N
        self.chained = bool(chained)
        # rows > N: zero padding clients after the real ones (the sharded FedAMW Z block)
        self.W_out = torch.zeros(max(N, int(rows or 0)), self.C, feats.ld, device=dev, dtype=torch.float32)
        self.loss = torch.zeros(N, device=dev, dtype=torch.float64)
        # pass p = j*E + e  ->  (n_j, offset)
        ns = feats.ns
        self.pass_n = np.repeat(ns, self.E)
        self.pass_off = (np.repeat(self.E * feats.row_off[:-1], self.E)
                         + np.tile(np.arange(self.E), N) * np.repeat(ns, self.E)).astype(np.int64)
        self._shuffler = None
        steps = self.E * ((ns + self.B - 1) // self.B)
        order = np.argsort(-steps, kind='stable').astype(np.int32)     # LPT: longest clients dispatched first
        self.order = torch.from_numpy(order).to(dev)
        import ctypes
        g, wsb = ctypes.c_int(0 if split is None else int(split)), ctypes.c_int64(0)
        max_en = int(self.E * ns.max()) if N else 0
        _lib.check(_lib.lib().fs_local_train_plan(N, self.C, self.B, self.E, feats.ld, max_en, int(self.chained),
                                                  int(bool(prox)), ctypes.byref(g), ctypes.byref(wsb)),
                   'fs_local_train_plan')
        if split is not None and int(split) != g.value:
            raise _lib.FedsimError('fs_local_train_plan: G=%d is not available for this shape (planner: %d)'
                                   % (int(split), g.value))
        self.G = int(g.value)                       # as the ABI takes it (G | G_PAIR: the pair form)
        self.pair = bool(self.G & _lib.G_PAIR)
        self.teams = bool(self.G & _lib.G_TEAMS)
        self.pipe = bool(self.G & _lib.G_PIPE)
        self.width = self.G & (_lib.G_PAIR - 1)     # workgroups per client group
        self.ws = (torch.zeros(max(2 * _lib.ERR_BLOCK, int(wsb.value)), dtype=torch.uint8, device=dev)
                   if self.G > 1 else None)

    def groups(self, cus):
        """Client groups a launch of this trainer runs on ``cus`` CUs (fs_local_train_plan's rule)."""
        if self.G <= 1:
            return 1 if self.chained else self.N
        if self.chained:
            return 1
        per = (self.N + 1) // 2 if (self.pair or self.teams) else self.N
        return max(1, min(per, cus // self.width))

    @property
    def shuffler(self):
        """GPU shuffle replay for direct ``run`` calls (the round plan owns its own slots)."""
        if self._shuffler is None:
            self._shuffler = Shuffler(self.pass_n, self.pass_off, self.E * self.f.rows, self.f.device)
        return self._shuffler

    def check_errors(self):
        """Raise if a split-client launch reported a broken hand-off, or a shuffle of this
        trainer's passes broke its length contract (synchronises)."""
        _check_ws_error(self.ws, 'fs_local_train')
        if self._shuffler is not None:
            self._shuffler.check_errors()

    def upload_perms(self, seeds, slot=0, stream=None):
        """seeds: [N*E] sampler seeds of one round's local training passes (client-major);
        the permutations are replayed on the GPU into shuffle slot ``slot``."""
        self.shuffler.prepare(seeds, slot, stream)

    def run(self, W_start, lr, prox, mu, reg, lam, chained, slot=0, loss_out=None):
        """Launch local training of every client; ``loss_out`` (float64 [N], default the
        trainer's own buffer) receives the last-epoch losses."""
        f = self.f
        L = _lib.lib()
        loss = self.loss if loss_out is None else loss_out
        perms = self.shuffler.acquire(slot)
        _lib.check(L.fs_local_train(_lib.ptr(f.phi), f.ld, _lib.ptr(f.row_off_dev), _lib.ptr(f.labels),
                                    _lib.ptr(perms), None if chained else _lib.ptr(self.order),
                                    self.N, self.C, self.B, self.E, float(lr), float(mu), int(bool(prox)),
                                    float(lam), int(bool(reg)), int(bool(chained)), _lib.ptr(W_start),
                                    _lib.ptr(self.W_out), _lib.ptr(loss), self.G, _lib.ptr(self.ws),
                                    0 if self.ws is None else self.ws.numel(), _lib.stream_ptr()),
                   'fs_local_train')
        self.shuffler.release(slot)
        return self.W_out, loss


class RoundPlan:
    """fs_plan: the native round driver (csrc/round.hip).  One ``round`` call enqueues a
    round's local training / aggregation / evaluation; ``shuffle`` replays a round's
    training shuffles into a slot on the plan's side stream (GPU replay by default,
    ``shuffle_device=False``: host thread pool + async upload).
    Borrows every device buffer from the objects passed in (they must outlive it)."""

    def __init__(self, trainer, W_g, loss_hist, p=None, aggregator=None, evaluator=None, eval_hist=None,
                 prox=False, mu=0.0, reg=False, lam=0.0, chained=False, shuffle_device=True, host_threads=0,
                 shuffle_after_train=False):
        import ctypes
        f = trainer.f
        self._keep = [trainer, W_g, loss_hist, p, aggregator, evaluator, eval_hist]
        self._h_n = np.ascontiguousarray(f.ns, dtype=np.int64)
        d = _lib.PlanDesc()
        d.d_phi, d.ld, d.d_row_off, d.d_labels = f.phi.data_ptr(), f.ld, f.row_off_dev.data_ptr(), f.labels.data_ptr()
        d.d_order = None if chained else trainer.order.data_ptr()
        d.h_n = self._h_n.ctypes.data
        d.N, d.C, d.B, d.E, d.G = trainer.N, trainer.C, trainer.B, trainer.E, trainer.G
        d.d_ws = None if trainer.ws is None else trainer.ws.data_ptr()
        d.ws_bytes = 0 if trainer.ws is None else trainer.ws.numel()
        d.chained, d.prox, d.reg = int(bool(chained)), int(bool(prox)), int(bool(reg))
        d.mu, d.lam = float(mu), float(lam)
        d.d_W_g, d.d_W_out, d.d_loss_hist = W_g.data_ptr(), trainer.W_out.data_ptr(), loss_hist.data_ptr()
        d.d_p = None if p is None else p.data_ptr()
        if aggregator is not None:
            d.d_agg_ws, d.agg_ws_floats, d.agg_chunks = aggregator.ws.data_ptr(), aggregator.ws.numel(), \
                int(aggregator.chunks)
        if evaluator is not None:
            d.d_phi_t, d.d_labels_t, d.n_t = evaluator.f.phi.data_ptr(), evaluator.f.labels.data_ptr(), evaluator.n
            d.d_eval_ws, d.d_eval_hist = evaluator.ws.data_ptr(), eval_hist.data_ptr()
        d.shuffle_device = int(bool(shuffle_device))
        d.host_threads = int(host_threads)
        d.shuffle_after_train = int(bool(shuffle_after_train))
        self._desc = d
        self._h = ctypes.c_void_p()
        _lib.check(_lib.lib().fs_plan_create(ctypes.byref(d), ctypes.byref(self._h)), 'fs_plan_create')
        self.npasses = int(trainer.N * trainer.E)

    def set_chunk(self, rounds):
        """Generate the shuffles of ``rounds`` consecutive rounds per launch (device replay;
        before the first ``shuffle``): no cross-stream wait between the rounds of a chunk."""
        _lib.check(_lib.lib().fs_plan_set_shuffle_chunk(self._h, int(rounds)), 'fs_plan_set_shuffle_chunk')

    def eval_blocks(self):
        """Evaluation workgroups a TRAIN launch carries for a deferred evaluation (0: none)."""
        n = _lib.lib().fs_plan_eval_blocks(self._h)
        if n < 0:
            _lib.check(n, 'fs_plan_eval_blocks')
        return n

    def flush(self):
        """Launch a partly collected chunk of shuffles (after a run's last round was prepared)."""
        _lib.check(_lib.lib().fs_plan_shuffle_flush(self._h), 'fs_plan_shuffle_flush')

    def shuffle(self, seeds, t):
        """seeds: [N*E] sampler seeds of round t's training passes (client-major)."""
        seeds = np.ascontiguousarray(seeds, dtype=np.int64)
        assert seeds.shape == (self.npasses,)
        _lib.check(_lib.lib().fs_plan_shuffle(self._h, seeds.ctypes.data, int(t)), 'fs_plan_shuffle')

    def eval_flush(self):
        """fs_plan_eval_flush (ABI 15): complete any evaluation still deferred, so the eval
        history is final on the current stream."""
        _lib.check(_lib.lib().fs_plan_eval_flush(self._h, _lib.stream_ptr()), 'fs_plan_eval_flush')

    def round(self, t, lr, phases, p_override=None):
        _lib.check(_lib.lib().fs_plan_round(self._h, int(t), float(lr), int(phases),
                                            None if p_override is None else _lib.ptr(p_override),
                                            _lib.stream_ptr()), 'fs_plan_round')

    def __del__(self):
        h = getattr(self, '_h', None)
        if h is not None and h.value and _lib._lib is not None:
            _lib._lib.fs_plan_destroy(h)
            self._h = None


class Aggregator:
    """fs_aggregate over a clients x params buffer."""

    def __init__(self, N, C, ld, device, chunks=0):
        self.N, self.len = int(N), int(C) * int(ld)
        self.chunks = chunks
        maxc = max(1, min(64, self.N))
        self.ws = torch.empty(maxc * self.len, dtype=torch.float32, device=device)

    def run(self, W_all, p, out):
        _lib.check(_lib.lib().fs_aggregate(_lib.ptr(W_all), self.len, _lib.ptr(p), self.N, self.len, _lib.ptr(out),
                                           _lib.ptr(self.ws), self.ws.numel(), int(self.chunks), _lib.stream_ptr()),
                   'fs_aggregate')
        return out


class Evaluator:
    """fs_eval on a resident test set."""

    def __init__(self, X_test, y_test, D, C, device, ld=None):
        self.f = Features([torch.as_tensor(X_test)], [torch.as_tensor(y_test)], D, device, ld)
        self.C = int(C)
        self.n = int(self.f.rows)
        if self.n < 1:
            raise ValueError('empty test set')
        self.ws = torch.empty(int(_lib.lib().fs_eval_ws_doubles(self.n)), dtype=torch.float64, device=device)

    def run(self, W, out2):
        _lib.check(_lib.lib().fs_eval(_lib.ptr(self.f.phi), self.f.ld, _lib.ptr(self.f.labels), self.n, _lib.ptr(W),
                                      self.C, _lib.ptr(out2), _lib.ptr(self.ws), _lib.stream_ptr()), 'fs_eval')
        return out2


class Mixture:
    """FedAMW's mixture-weight estimation: Z GEMM + persistent p-SGD (tools.py:435-453)."""

    def __init__(self, X_val, y_val, D, C, N, Bv, p0, device, ld=None, momentum=0.9):
        self.f = Features([torch.as_tensor(X_val)], [torch.as_tensor(y_val)], D, device, ld)
        self.C, self.N, self.Bv = int(C), int(N), int(Bv)
        self.nv = int(self.f.rows)
        if self.nv < 1:
            raise ValueError('empty validation set')
        self.momentum = float(momentum)
        self.ldN = (self.N + 3) // 4 * 4
        self.Z = torch.empty(self.nv, self.C * self.ldN, dtype=torch.float32, device=device)
        self.p = p0.to(device=device, dtype=torch.float32).clone()
        self.buf = torch.zeros(self.N, dtype=torch.float32, device=device)
        self.first = torch.ones(1, dtype=torch.int32, device=device)
        self.ws = torch.zeros(int(_lib.lib().fs_mix_solve_ws_bytes(self.N, self.C, self.Bv)), dtype=torch.uint8,
                              device=device)
        self.shuffler = None
        self.blocks = 1          # > 1: Z holds `blocks` rank blocks [blocks][n_val][C][N/blocks] (dist.py)

    def blocked_covers(self, epochs):
        """Whether fs_mix_solve_blocked reads this shape (the qmc solver; include/fedsim.h)."""
        return bool(_lib.lib().fs_mix_solve_blocked_covers(self.N, self.C, self.nv, int(epochs), self.Bv))

    def check_errors(self):
        """Raise if a multi-CU p-solve reported a timed-out exchange (synchronises)."""
        _check_ws_error(self.ws, 'fs_mix_solve')

    def z_block(self, W_all, n, out):
        """fs_mix_z of ``n`` client models (W_all [n, C, ld]) on the validation rows into
        ``out`` [n_val, C * ldN(n)] -- one rank's block of the sharded Z-GEMM."""
        _lib.check(_lib.lib().fs_mix_z(_lib.ptr(W_all), _lib.ptr(self.f.phi), self.f.ld, int(n), self.C, self.nv,
                                       _lib.ptr(out), _lib.stream_ptr()), 'fs_mix_z')
        return out

    def prepare(self, seeds, slot=0, stream=None):
        """Enqueue one round's validation-pass shuffles (one seed per inner epoch)."""
        ep = len(seeds)
        if self.shuffler is None or self.shuffler.P != ep:
            self.shuffler = Shuffler(np.full(ep, self.nv, np.int64), np.arange(ep, dtype=np.int64) * self.nv,
                                     ep * self.nv, self.Z.device)
        self.shuffler.prepare(seeds, slot, stream)

    def solve(self, W_all, seeds, lr_p, slot=None, z=True):
        """W_all: [N, C, ld] every client's weights; seeds: sampler seeds of the round's
        validation passes (one per inner epoch), or None when ``prepare`` already enqueued
        them into ``slot``.  ``z=False`` reuses Z from the previous call (W_all unchanged)."""
        L = _lib.lib()
        if z and self.blocks > 1:
            # fs_mix_z writes the standard [n_val][C][ldN] layout; fs_mix_solve_blocked would
            # read it as rank blocks
            raise ValueError('Mixture.solve(z=True) with blocks=%d: Z must come from the rank-block '
                             'all-gather (dist.allgather_z(blocked=True)), then solve(z=False)' % self.blocks)
        if z:
            _lib.check(L.fs_mix_z(_lib.ptr(W_all), _lib.ptr(self.f.phi), self.f.ld, self.N, self.C, self.nv,
                                  _lib.ptr(self.Z), _lib.stream_ptr()), 'fs_mix_z')
        if seeds is not None:
            slot = 0
            if len(seeds) == 0:
                return self.p
            self.prepare(seeds, slot)
        epochs = self.shuffler.P
        perms = self.shuffler.acquire(slot)
        tail = (_lib.ptr(self.f.labels), _lib.ptr(perms), self.N, self.C, self.nv, epochs, self.Bv, float(lr_p),
                self.momentum, _lib.ptr(self.p), _lib.ptr(self.buf), _lib.ptr(self.first), _lib.ptr(self.ws),
                self.ws.numel(), _lib.stream_ptr())
        if self.blocks > 1:
            _lib.check(L.fs_mix_solve_blocked(_lib.ptr(self.Z), self.blocks, *tail), 'fs_mix_solve_blocked')
        else:
            _lib.check(L.fs_mix_solve(_lib.ptr(self.Z), *tail), 'fs_mix_solve')
        self.shuffler.release(slot)
        return self.p


def feature_map(X, W, b, D, out=None, ldo=None):
    """fs_feature_map: ``scale * cos(X W + b)`` (tools.py:27, 29) on the current stream.
    X [n, d] (any device; copied to the GPU as fp32 if needed), W [d, D], b [D] -> out [n, ldo]
    (default ldo = D; columns D..ldo-1 are written as 0)."""
    dev = torch.device('cuda', torch.cuda.current_device())
    X = torch.as_tensor(X).to(device=dev, dtype=torch.float32).contiguous()
    W = torch.as_tensor(W).to(device=dev, dtype=torch.float32).reshape(-1, int(D)).contiguous()
    b = torch.as_tensor(b).to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
    n, d = X.shape
    if W.shape[0] != d or b.numel() != D:
        raise ValueError('feature_map: X [n, %d] needs W [%d, %d] and b [%d]' % (d, d, D, D))
    ldo = int(ldo or D)
    if out is None:
        out = torch.empty(n, ldo, device=dev, dtype=torch.float32)
    assert out.is_contiguous() and out.shape[1] == ldo and out.shape[0] >= n
    scale = float(np.float32(1.0 / np.sqrt(D)))      # the float64 scalar torch multiplies in fp32
    _lib.check(_lib.lib().fs_feature_map(_lib.ptr(X), d, _lib.ptr(W), _lib.ptr(b), n, d, int(D), scale,
                                         _lib.ptr(out), ldo, _lib.stream_ptr()), 'fs_feature_map')
    return out


def heterogeneity(feats):
    """exp.py:67-74 over a client-packed feature buffer (``Features``): fs_gram for
    G = Phi^T Phi, fs_hetero for S_j = ||G/n - G_j/n_j||_F^2 per client.  Returns
    (sum_j n_j/n * sqrt(S_j), S [N] numpy float64)."""
    dev = feats.phi.device
    D, N, n = feats.D, len(feats.ns), int(feats.rows)
    if n < 1:
        raise ValueError('heterogeneity of an empty partition')
    G = torch.empty(D, D, device=dev, dtype=torch.float32)
    S = torch.empty(N, device=dev, dtype=torch.float64)
    L = _lib.lib()
    _lib.check(L.fs_gram(_lib.ptr(feats.phi), feats.ld, n, D, _lib.ptr(G), D, _lib.stream_ptr()), 'fs_gram')
    _lib.check(L.fs_hetero(_lib.ptr(feats.phi), feats.ld, _lib.ptr(feats.row_off_dev), N, D, _lib.ptr(G), D, n,
                           _lib.ptr(S), _lib.stream_ptr()), 'fs_hetero')
    S = S.cpu().numpy()
    hete = np.float32(0.0)
    for nj, s in zip(feats.ns, S):      # data_hete += len_j / len * torch.norm(C - C_j), an fp32 tensor
        hete = np.float32(hete + np.float32(nj / n * np.float32(np.sqrt(s))))
    return float(hete), S
