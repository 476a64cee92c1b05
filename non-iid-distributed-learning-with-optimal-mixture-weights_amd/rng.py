"""Replay of the reference's RNG consumption (torch global CPU generator).

Every ``DataLoader(..., shuffle=True)`` pass in the reference (train: tools.py:179;
test: tools.py:220; validation: exp.py:99) draws two int64 values from torch's
global CPU generator -- the worker base seed at ``iter()`` and the RandomSampler
seed at the first ``next()`` -- then permutes with ``randperm(n)`` on a private
generator seeded with the second draw.  The draw
pattern is data-independent, so a whole round's seeds come from ONE vectorised
``random_()`` call on the very same generator (k vectorised draws == k scalar
draws), and the permutations are replayed bit-exactly in C++
(``fs_randperm_batch``), spread over host threads.
"""
import numpy as np
import torch

from . import _lib


def draw_pass_seeds(npasses):
    """Consume 2*npasses int64 draws from torch's global CPU generator and return
    the npasses sampler seeds (int64 numpy array)."""
    if npasses == 0:
        return np.zeros(0, np.int64)
    d = torch.empty(2 * npasses, dtype=torch.int64).random_()
    return d[1::2].numpy().copy()


def randperms(seeds, ns, offs, out, nthreads=0):
    """out[offs[i]:offs[i]+ns[i]] = torch.randperm(ns[i], generator=manual_seed(seeds[i])).

    ``out`` is an int32 numpy array or a pinned CPU int32 tensor."""
    seeds = np.ascontiguousarray(seeds, dtype=np.int64)
    ns = np.ascontiguousarray(ns, dtype=np.int64)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    if isinstance(out, torch.Tensor):
        assert out.dtype == torch.int32 and not out.is_cuda
        optr = out.data_ptr()
    else:
        assert out.dtype == np.int32 and out.flags['C_CONTIGUOUS']
        optr = out.ctypes.data
    assert len(seeds) == len(ns) == len(offs)
    if len(ns) and int((offs + ns).max()) > (out.numel() if isinstance(out, torch.Tensor) else out.size):
        raise ValueError('randperms: output buffer too small')
    _lib.check(_lib.lib().fs_randperm_batch(seeds.ctypes.data, ns.ctypes.data, offs.ctypes.data, len(ns), optr,
                                            int(nthreads)), 'fs_randperm_batch')
    return out
