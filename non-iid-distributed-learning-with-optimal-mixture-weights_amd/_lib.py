"""ctypes binding of libfedsim.so (C-ABI declared in include/fedsim.h).

``torch`` is imported first on purpose: its wheel ships ``libamdhip64.so`` with the
same SONAME (libamdhip64.so.7) as /opt/rocm's, so the loader reuses torch's HIP
runtime for our kernels and both share one device context, one set of streams and
one caching allocator.  A missing library raises -- there is no fallback path.
"""
import ctypes as C
import os

import torch  # noqa: F401  (must be loaded before libfedsim.so, see above)

from . import LIB_PATH

_c_f32p = C.POINTER(C.c_float)
_SIGS = {
    'fs_abi_version': (C.c_int, []),
    'fs_last_error': (C.c_char_p, []),
    'fs_tuning_size': (C.c_int64, []),
    'fs_set_tuning': (C.c_int, [C.c_void_p]),
    'fs_set_thread_tuning': (C.c_int, [C.c_void_p]),
    'fs_get_tuning': (C.c_int, [C.c_void_p]),
    'fs_get_process_tuning': (C.c_int, [C.c_void_p]),
    'fs_get_thread_tuning': (C.c_int, [C.c_void_p]),
    'fs_randperm_batch': (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int]),
    'fs_libsvm_scan': (C.c_int, [C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    'fs_libsvm_read': (C.c_int, [C.c_char_p, C.c_int64, C.c_int64, C.c_int, C.c_void_p, C.c_void_p, C.c_int]),
    'fs_randperm_device': (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p,
                                     C.c_void_p, C.c_void_p]),
    'fs_local_train_plan': (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int64, C.c_int,
                                      C.c_int, C.c_void_p, C.c_void_p]),
    'fs_local_train': (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float, C.c_int,
                                 C.c_float, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_int, C.c_void_p, C.c_int64, C.c_void_p]),
    'fs_aggregate': (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_int64, C.c_void_p,
                               C.c_void_p, C.c_int64, C.c_int, C.c_void_p]),
    'fs_eval_ws_doubles': (C.c_int64, [C.c_int]),
    'fs_eval': (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                          C.c_void_p, C.c_void_p]),
    'fs_mix_z': (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_void_p,
                           C.c_void_p]),
    'fs_mix_solve_ws_bytes': (C.c_int64, [C.c_int, C.c_int, C.c_int]),
    'fs_mix_solve': (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                               C.c_int, C.c_float, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p,
                               C.c_void_p, C.c_int64, C.c_void_p]),
    'fs_mix_solve_blocked': (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.c_int, C.c_float, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_int64, C.c_void_p]),
    'fs_mix_solve_blocked_covers': (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    'fs_mix_solve_last_mode': (C.c_int, []),
    'fs_mix_solve_last_layout': (C.c_int, [C.c_void_p, C.c_void_p]),
    'fs_feature_map': (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                 C.c_float, C.c_void_p, C.c_int64, C.c_void_p]),
    'fs_gram': (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_void_p, C.c_int64, C.c_void_p]),
    'fs_hetero': (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_int64,
                            C.c_void_p, C.c_void_p]),
    'fs_plan_desc_size': (C.c_int64, []),
    'fs_plan_create': (C.c_int, [C.c_void_p, C.c_void_p]),
    'fs_plan_destroy': (C.c_int, [C.c_void_p]),
    'fs_plan_shuffle': (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    'fs_plan_round': (C.c_int, [C.c_void_p, C.c_int, C.c_float, C.c_int, C.c_void_p, C.c_void_p]),
    'fs_plan_eval_flush': (C.c_int, [C.c_void_p, C.c_void_p]),
    'fs_local_train_last_kernel': (C.c_int, []),
    'fs_plan_set_shuffle_chunk': (C.c_int, [C.c_void_p, C.c_int]),
    'fs_plan_shuffle_flush': (C.c_int, [C.c_void_p]),
    'fs_plan_eval_blocks': (C.c_int, [C.c_void_p]),
    'fs_timer_create': (C.c_int, [C.c_void_p]),
    'fs_timer_record': (C.c_int, [C.c_void_p, C.c_void_p]),
    'fs_timer_elapsed_ms': (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    'fs_timer_destroy': (C.c_int, [C.c_void_p]),
}

EXPORTS = tuple(_SIGS)
ABI_VERSION = 16

PHASE_TRAIN, PHASE_AGGREGATE, PHASE_EVAL, PHASE_EVAL_DEFER = 1, 2, 4, 8
G_PAIR = 256             # fs_local_train_plan: G | G_PAIR = the pair-client form at width G (ABI 10)
G_TEAMS = 512            # fs_local_train_plan: G | G_TEAMS = the team form at width G (ABI 13)
LT_KERNELS = {1: 'single', 2: 'split', 3: 'dbuf', 4: 'pair', 5: 'pipe', 6: 'teams', 7: 'mb'}   # fs_local_train_last_kernel (ABI 15; mb: 16)
G_PIPE = 1024            # fs_local_train_plan: G | G_PIPE = the pipelined split form at width G (ABI 14)
ERR_BLOCK = 256          # the error block at the end of every exchange workspace (include/fedsim.h)
SOLVER_NAMES = {0: 'none', 1: 'reg', 2: 'mc', 3: 'staged', 4: 'global', 5: 'reg2', 6: 'wave', 8: 'quad', 9: 'qmc', 10: 'bin'}
SOLVERS = {v: k for k, v in SOLVER_NAMES.items() if k}


class Tuning(C.Structure):
    """fs_tuning (include/fedsim.h), field for field: how -- never what -- the kernels compute."""
    _fields_ = [('mix_solver', C.c_int), ('mix_prefetch', C.c_int), ('mix_prefetch_lead', C.c_int),
                ('mix_exact_softmax', C.c_int), ('no_eval_fuse', C.c_int), ('spin_limit', C.c_uint),
                ('inject_timeout', C.c_int), ('train_form', C.c_int),
                ('split_early', C.c_int), ('mix_qmc_lane_clients', C.c_int),
                ('mix_quad_loaders', C.c_int), ('split_teams', C.c_int),
                ('mix_poll_delay', C.c_int), ('split_poll_delay', C.c_int), ('split_pipe', C.c_int),
                ('split_dbuf', C.c_int),
                ('split_mb', C.c_int)]


class PlanDesc(C.Structure):
    """fs_plan_desc (include/fedsim.h), field for field."""
    _fields_ = [
        ('d_phi', C.c_void_p), ('ld', C.c_int64), ('d_row_off', C.c_void_p), ('d_labels', C.c_void_p),
        ('d_order', C.c_void_p), ('h_n', C.c_void_p),
        ('N', C.c_int), ('C', C.c_int), ('B', C.c_int), ('E', C.c_int), ('G', C.c_int),
        ('d_ws', C.c_void_p), ('ws_bytes', C.c_int64),
        ('chained', C.c_int), ('prox', C.c_int), ('reg', C.c_int), ('mu', C.c_float), ('lam', C.c_float),
        ('d_W_g', C.c_void_p), ('d_W_out', C.c_void_p), ('d_loss_hist', C.c_void_p),
        ('d_p', C.c_void_p), ('d_agg_ws', C.c_void_p), ('agg_ws_floats', C.c_int64), ('agg_chunks', C.c_int),
        ('d_phi_t', C.c_void_p), ('d_labels_t', C.c_void_p), ('n_t', C.c_int), ('d_eval_ws', C.c_void_p),
        ('d_eval_hist', C.c_void_p), ('shuffle_device', C.c_int), ('host_threads', C.c_int),
        ('shuffle_after_train', C.c_int),
    ]

_lib = None


class FedsimError(RuntimeError):
    pass


def lib():
    """Load (once) and return the ctypes handle; raises if the library is missing.
    FEDSIM_LIB overrides the path (diagnostic builds, e.g. the in-kernel stamp build)."""
    global _lib
    if _lib is None:
        path = os.environ.get('FEDSIM_LIB') or LIB_PATH
        if not os.path.exists(path):
            raise FedsimError(
                'libfedsim.so not found at %s -- build it with `python -c "import __graft_entry__ as g; g.build()"` '
                'or `make -C <pkg>/csrc`; there is no CPU fallback' % path)
        h = C.CDLL(path, mode=C.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            f = getattr(h, name)
            f.restype = res
            f.argtypes = args
        if h.fs_abi_version() != ABI_VERSION:
            raise FedsimError('libfedsim.so ABI %d != %d' % (h.fs_abi_version(), ABI_VERSION))
        if h.fs_tuning_size() != C.sizeof(Tuning):
            raise FedsimError('fs_tuning layout mismatch (%d != %d bytes)' % (h.fs_tuning_size(), C.sizeof(Tuning)))
        if h.fs_plan_desc_size() != C.sizeof(PlanDesc):
            raise FedsimError('fs_plan_desc layout mismatch (%d != %d bytes)' % (h.fs_plan_desc_size(),
                                                                                  C.sizeof(PlanDesc)))
        _lib = h
    return _lib


def get_tuning():
    """The fs_tuning the calling thread's next launch would use, as a dict (include/fedsim.h:
    the thread's own override, else the process-wide value)."""
    t = Tuning()
    check(lib().fs_get_tuning(C.byref(t)), 'fs_get_tuning')
    return {k: getattr(t, k) for k, _ in Tuning._fields_}


def last_mix_layout():
    """(workgroups, clients per lane) of the calling thread's last qmc p-solve, else (0, 0)."""
    k, nk = C.c_int(0), C.c_int(0)
    check(lib().fs_mix_solve_last_layout(C.byref(k), C.byref(nk)), 'fs_mix_solve_last_layout')
    return k.value, nk.value


def get_process_tuning():
    """The process-wide fs_tuning (fs_set_tuning's value), whatever the calling thread's override."""
    t = Tuning()
    check(lib().fs_get_process_tuning(C.byref(t)), 'fs_get_process_tuning')
    return {k: getattr(t, k) for k, _ in Tuning._fields_}


def get_thread_tuning():
    """The calling thread's override as a dict, or None when the thread has none."""
    t = Tuning()
    has = lib().fs_get_thread_tuning(C.byref(t))
    if has < 0:
        check(has, 'fs_get_thread_tuning')
    return {k: getattr(t, k) for k, _ in Tuning._fields_} if has else None


def _merged(base, fields):
    cur = dict(base)
    for k, v in fields.items():
        if k not in cur:
            raise KeyError('fs_tuning has no field %r' % k)
        if k == 'mix_solver' and isinstance(v, str):
            v = 0 if v == 'auto' else SOLVERS[v]
        cur[k] = int(v)
    return cur


def set_tuning(**fields):
    """Set process-wide fs_tuning fields (the others keep their current process-wide values,
    never a thread override's).  ``mix_solver`` may be a solver name ('quad', 'qmc', ...).
    Returns the previous process-wide settings (a dict).  A thread that holds an override
    keeps using it: ``tuning`` below changes the override instead on such a thread."""
    prev = get_process_tuning()
    check(lib().fs_set_tuning(C.byref(Tuning(**_merged(prev, fields)))), 'fs_set_tuning')
    return prev


def set_thread_tuning(fields=None):
    """fs_set_thread_tuning: an override for the launches the calling host thread enqueues
    (``fields``: a dict over the all-default tuning, solver names allowed), or None to drop
    the thread's override."""
    if fields is None:
        check(lib().fs_set_thread_tuning(None), 'fs_set_thread_tuning')
        return
    cur = _merged({k: 0 for k, _ in Tuning._fields_}, fields)
    check(lib().fs_set_thread_tuning(C.byref(Tuning(**cur))), 'fs_set_thread_tuning')


class tuning:
    """Context manager: ``with _lib.tuning(mix_solver='qmc', mix_prefetch=-1): ...`` sets
    fs_tuning fields for the block and restores the previous values after it.  On a thread
    without an override it changes the process-wide value (every thread without an override
    sees it); on a thread that holds an override it changes that override (the layer the
    thread's launches read) and restores it on exit -- the process-wide value is untouched."""

    def __init__(self, **fields):
        self.fields = fields

    def __enter__(self):
        own = get_thread_tuning()
        self.thread_prev = own
        if own is not None:
            set_thread_tuning(_merged(own, self.fields))
        else:
            self.prev = set_tuning(**self.fields)
        return self

    def __exit__(self, *exc):
        if self.thread_prev is not None:
            set_thread_tuning(self.thread_prev)
        else:
            check(lib().fs_set_tuning(C.byref(Tuning(**self.prev))), 'fs_set_tuning')
        return False


def check(status, what):
    if status != 0:
        msg = lib().fs_last_error()
        raise FedsimError('%s failed (%d): %s' % (what, status, msg.decode() if msg else ''))


def ptr(t):
    """Raw data pointer of a tensor (device or host) or None."""
    return None if t is None else C.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


# the device sources each measured kernel is compiled from (its own file + the headers it includes)
KERNEL_SOURCES = {
    'local_train': ('local_train.hip', 'local_train_split.hip', 'local_train_pair.hip', 'local_train_pipe.hip',
                    'local_train_dbuf.hip', 'split_common.h', 'common.h',
                    'eval_rows.h', 'lanes.h'),
    'mix_solve': ('mixture.hip', 'common.h', 'lanes.h'),
    'mix_z': ('mix_z.hip', 'common.h'),
}


def source_revision(kernel=None):
    """sha256 (16 hex digits) of the code (comments and whitespace runs dropped) of the device
    sources of libfedsim.so: all of them (csrc/*.hip,
    csrc/*.h; host-only .cpp files and the C-ABI header carry no device code), or only those
    ``kernel`` ('local_train', 'mix_solve') is compiled from.  Profiles under profiles/
    record it; bench.py uses a PMC traffic figure only when it was measured on the kernel's
    exact sources."""
    import hashlib
    import glob
    pkg = os.path.dirname(os.path.abspath(__file__))
    if kernel:
        files = sorted(os.path.join(pkg, 'csrc', f) for f in KERNEL_SOURCES[kernel])
    else:
        files = sorted(glob.glob(os.path.join(pkg, 'csrc', '*.hip')) + glob.glob(os.path.join(pkg, 'csrc', '*.h')))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, 'rb') as fh:
            h.update(_code_only(fh.read().decode()).encode())
    return h.hexdigest()[:16]


_TOKENS = None


def _code_only(src):
    """The source without comments and with whitespace runs collapsed (string and character
    literals kept verbatim): a comment edit does not change a kernel's revision."""
    global _TOKENS
    import re
    if _TOKENS is None:
        _TOKENS = re.compile(r'"(?:\\.|[^"\\])*"|\'(?:\\.|[^\'\\])*\'|//[^\n]*|/\*.*?\*/|\s+|[^"\'/\s]+|/',
                             re.S)
    out = []
    for m in _TOKENS.finditer(src):
        t = m.group(0)
        if t.startswith('//') or t.startswith('/*'):
            out.append(' ')
        elif t.isspace():
            out.append(' ')
        else:
            out.append(t)
    return re.sub(r' +', ' ', ''.join(out)).strip()


class Timer:
    """A timing event on the current stream without a system-scope release (fs_timer_*):
    ``record()`` now, ``elapsed_time(other)`` in ms, as torch.cuda.Event's."""

    def __init__(self):
        self._ev = C.c_void_p()
        check(lib().fs_timer_create(C.byref(self._ev)), 'fs_timer_create')

    def record(self):
        check(lib().fs_timer_record(self._ev, stream_ptr()), 'fs_timer_record')

    def elapsed_time(self, end):
        ms = C.c_float()
        check(lib().fs_timer_elapsed_ms(self._ev, end._ev, C.byref(ms)), 'fs_timer_elapsed_ms')
        return float(ms.value)

    def __del__(self):
        if getattr(self, '_ev', None) is not None and self._ev.value and _lib is not None:
            _lib.fs_timer_destroy(self._ev)
            self._ev = None
