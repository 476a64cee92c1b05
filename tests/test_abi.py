"""The C-ABI library loads and exports every symbol include/fedsim.h declares (CPU only;
no compute calls), and argument validation fails cleanly through fs_last_error."""
import ctypes
import os
import re

import pytest

import fedamw_amd
from fedamw_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, 'include', 'fedsim.h')).read()
    return sorted(set(re.findall(r'\b(fs_[a-z_]+)\s*\(', src)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_symbol():
    h = ctypes.CDLL(fedamw_amd.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(h, name), name


def test_abi_version():
    assert _lib.lib().fs_abi_version() == _lib.ABI_VERSION


@pytest.mark.parametrize('call,needle', [
    (lambda L: L.fs_local_train(None, 64, None, None, None, None, 1, 40, 32, 2, 0.1, 0.0, 0, 0.0, 0, 0,
                                None, None, None, 1, None, 0, None), 'num_classes'),
    (lambda L: L.fs_local_train(None, 100, None, None, None, None, 1, 10, 32, 2, 0.1, 0.0, 0, 0.0, 0, 0,
                                None, None, None, 1, None, 0, None), 'ld'),
    (lambda L: L.fs_local_train_plan(0, 10, 32, 2, 64, 64, 0, 0, None, None), 'null'),
    (lambda L: L.fs_aggregate(None, 64, None, 0, 64, None, None, 0, 1, None), 'N'),
    (lambda L: L.fs_eval(None, 64, None, 0, None, 10, None, None, None), 'n'),
    (lambda L: L.fs_mix_solve(None, None, None, 5, 3, 10, 1, 65, 0.1, 0.9, None, None, None, None, 0, None),
     'batch'),
    (lambda L: L.fs_plan_set_shuffle_chunk(None, 8), 'bad arguments'),
    (lambda L: L.fs_plan_shuffle_flush(None), 'bad arguments'),
    (lambda L: L.fs_plan_eval_blocks(None), 'bad arguments'),
    (lambda L: L.fs_plan_eval_flush(None, None), 'bad arguments'),
    (lambda L: L.fs_timer_create(None), 'null'),
    (lambda L: L.fs_timer_record(None, None), 'null'),
    (lambda L: L.fs_timer_elapsed_ms(None, None, None), 'null'),
])
def test_invalid_arguments_fail_without_touching_the_gpu(call, needle):
    L = _lib.lib()
    rc = call(L)
    assert rc == -1
    assert needle in L.fs_last_error().decode()


def test_workspace_sizes_are_host_only():
    """Workspace queries are pure host arithmetic (no GPU needed) and always leave room for
    the 256-byte error block at the end."""
    L = _lib.lib()
    assert L.fs_mix_solve_ws_bytes(100, 10, 16) >= _lib.ERR_BLOCK
    assert L.fs_mix_solve_ws_bytes(1000, 10, 16) > L.fs_mix_solve_ws_bytes(10, 2, 16)   # multi-CU granules
    assert L.fs_mix_solve_last_mode() in _lib.SOLVER_NAMES


def test_tuning_threading_contract():
    """include/fedsim.h (ABI 12): a launch reads the tuning of the host thread that enqueues it
    -- the thread's fs_set_thread_tuning override, else the process-wide fs_set_tuning value.
    Checked through fs_get_tuning (what the calling thread's next launch would use); host-only."""
    import threading
    prev = _lib.set_tuning(mix_solver='quad')
    try:
        seen = {}

        def worker(name, fields):
            if fields is not None:
                _lib.set_thread_tuning(fields)
            seen[name + '_own'] = _lib.get_tuning()['mix_solver']
            barrier.wait()                  # both threads hold their settings at once
            seen[name + '_after'] = _lib.get_tuning()['mix_solver']
            _lib.set_thread_tuning(None)
            seen[name + '_dropped'] = _lib.get_tuning()['mix_solver']

        barrier = threading.Barrier(2)
        ts = [threading.Thread(target=worker, args=('a', {'mix_solver': 'qmc'})),
              threading.Thread(target=worker, args=('b', None))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert seen['a_own'] == seen['a_after'] == _lib.SOLVERS['qmc']
        assert seen['b_own'] == seen['b_after'] == _lib.SOLVERS['quad']       # the process-wide value
        assert seen['a_dropped'] == seen['b_dropped'] == _lib.SOLVERS['quad']
        assert _lib.get_tuning()['mix_solver'] == _lib.SOLVERS['quad']       # this thread: untouched
        L = _lib.lib()
        bad = _lib.Tuning(train_form=7)
        assert L.fs_set_thread_tuning(ctypes.byref(bad)) == -1
        assert 'train_form' in L.fs_last_error().decode()
        bad = _lib.Tuning(mix_qmc_lane_clients=6)
        assert L.fs_set_thread_tuning(ctypes.byref(bad)) == -1
        assert 'mix_qmc_lane_clients' in L.fs_last_error().decode()
        bad = _lib.Tuning(mix_quad_loaders=1)
        assert L.fs_set_thread_tuning(ctypes.byref(bad)) == -1
        assert 'mix_quad_loaders' in L.fs_last_error().decode()
        bad = _lib.Tuning(split_teams=2)
        assert L.fs_set_thread_tuning(ctypes.byref(bad)) == -1
        assert 'split_teams' in L.fs_last_error().decode()
        bad = _lib.Tuning(mix_poll_delay=-2)
        assert L.fs_set_thread_tuning(ctypes.byref(bad)) == -1
        assert 'mix_poll_delay' in L.fs_last_error().decode()
    finally:
        _lib.set_tuning(**prev)


def test_tuning_context_on_a_thread_with_an_override():
    """``with _lib.tuning(...)`` on a thread that holds an override changes that
    override (the layer the thread's launches read) and restores it on exit; the process-wide
    value is neither overwritten with the override's fields nor changed.  set_tuning from such a
    thread changes only the process-wide value.  Host-only."""
    import threading
    prev = _lib.set_tuning(mix_solver='quad', mix_poll_delay=3)
    try:
        seen = {}

        def worker():
            _lib.set_thread_tuning({'mix_solver': 'qmc', 'split_poll_delay': 5})
            with _lib.tuning(mix_prefetch=-1):
                seen['inside'] = _lib.get_tuning()
                seen['inside_process'] = _lib.get_process_tuning()
            seen['after'] = _lib.get_tuning()
            seen['thread_after'] = _lib.get_thread_tuning()
            old = _lib.set_tuning(mix_poll_delay=7)          # process-wide only
            seen['set_prev'] = old
            seen['own_after_set'] = _lib.get_tuning()
            _lib.set_tuning(**old)
            _lib.set_thread_tuning(None)
            seen['dropped'] = _lib.get_thread_tuning()

        t = threading.Thread(target=worker)
        t.start()
        t.join()
        assert seen['inside']['mix_solver'] == _lib.SOLVERS['qmc'] and seen['inside']['mix_prefetch'] == -1
        assert seen['inside']['split_poll_delay'] == 5
        assert seen['inside_process']['mix_solver'] == _lib.SOLVERS['quad']
        assert seen['inside_process']['mix_prefetch'] == 0 and seen['inside_process']['split_poll_delay'] == 0
        assert seen['after']['mix_prefetch'] == 0 and seen['after']['mix_solver'] == _lib.SOLVERS['qmc']
        assert seen['thread_after'] == seen['after']
        assert seen['set_prev']['mix_solver'] == _lib.SOLVERS['quad'] and seen['set_prev']['mix_poll_delay'] == 3
        assert seen['own_after_set']['mix_poll_delay'] == 0                 # the override still wins
        assert seen['dropped'] is None
        proc = _lib.get_process_tuning()
        assert proc['mix_solver'] == _lib.SOLVERS['quad'] and proc['mix_poll_delay'] == 3
        assert _lib.get_thread_tuning() is None
        with _lib.tuning(mix_prefetch=-1):                  # no override here: process-wide
            assert _lib.get_process_tuning()['mix_prefetch'] == -1
        assert _lib.get_process_tuning()['mix_prefetch'] == 0
    finally:
        _lib.set_tuning(**prev)


def test_source_revision_ignores_comments():
    """bench.py keys a PMC capture to the code it measured (_lib.source_revision): a comment or
    whitespace edit keeps the key, a code edit changes it; literals are kept verbatim."""
    c = _lib._code_only
    base = 'int a = 1; // one\n/* two\n three */ float b = a / 2;\n'
    assert c(base) == c('int a = 1;\n\n  float b = a / 2; // changed comment\n')
    assert c(base) != c(base.replace('a / 2', 'a / 3'))
    assert c('const char* s = "x // y";') == 'const char* s = "x // y";'
    assert c("asm(\"s_waitcnt vmcnt(0) ; pr-own\"); char q = '/';") == "asm(\"s_waitcnt vmcnt(0) ; pr-own\"); char q = '/';"
    assert re.fullmatch(r'[0-9a-f]{16}', _lib.source_revision('local_train'))
