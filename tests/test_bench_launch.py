"""bench.py's multi-rank launcher on CPU: ``--gpus N`` starts N workers with the
torch.distributed environment, relays rank 0's line, and fails when a worker fails."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

WORKER = r'''
import json, os, sys
import torch, torch.distributed as tdist
r, ws = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
assert os.environ['MASTER_ADDR'] == '127.0.0.1' and os.environ['LOCAL_RANK'] == str(r)
tdist.init_process_group('gloo')
t = torch.tensor([float(r + 1)])
tdist.all_reduce(t)
if r == 0:
    print(json.dumps({'world_size': tdist.get_world_size(), 'sum': float(t.item())}), flush=True)
tdist.destroy_process_group()
sys.exit(int(os.environ.get('FAIL_RANK', '-1') == str(r)) * 3)
'''


def test_spawn_relays_rank0(tmp_path, capfd):
    w = tmp_path / 'w.py'
    w.write_text(WORKER)
    rc = bench.spawn(3, [sys.executable, str(w)])
    out = capfd.readouterr().out
    assert rc == 0
    line = json.loads(out.strip().splitlines()[-1])
    assert line == {'world_size': 3, 'sum': 6.0}


def test_spawn_fails_when_a_worker_fails(tmp_path, monkeypatch):
    w = tmp_path / 'w.py'
    w.write_text(WORKER)
    monkeypatch.setenv('FAIL_RANK', '1')
    assert bench.spawn(2, [sys.executable, str(w)]) == 3


def test_spawn_stops_the_others(tmp_path):
    w = tmp_path / 'w.py'
    w.write_text('import os, sys, time\nif os.environ["RANK"] == "1": sys.exit(5)\ntime.sleep(600)\n')
    assert bench.spawn(2, [sys.executable, str(w)]) == 5


def test_spawn_launch_timeout(tmp_path, capfd):
    """A rank that never exits (here: sleeps after a clean rank 0 has printed its line and
    exited 0) is stopped at the launcher's wall-clock bound, and the launch fails (124)."""
    w = tmp_path / 'w.py'
    w.write_text('import os, sys, time\nif os.environ["RANK"] == "0":\n    print("{}", flush=True)\n    sys.exit(0)\n'
                 'time.sleep(600)\n')
    import time
    t0 = time.time()
    assert bench.spawn(2, [sys.executable, str(w)], timeout=3.0) == 124
    assert time.time() - t0 < 60
    assert '{}' in capfd.readouterr().out


def test_spawn_teardown_timeout(tmp_path, capfd):
    """The teardown bound counts from the first worker that exits 0 (or rank 0's result line): a
    rank still running that long after rank 0 finished is stopped (124); a run whose ranks all
    finish inside it is not cut."""
    w = tmp_path / 'w.py'
    w.write_text('import os, sys, time\nif os.environ["RANK"] == "0":\n    print("{}", flush=True)\n    sys.exit(0)\n'
                 'time.sleep(600)\n')
    import time
    t0 = time.time()
    assert bench.spawn(2, [sys.executable, str(w)], teardown=2.0) == 124
    assert time.time() - t0 < 60
    assert '{}' in capfd.readouterr().out
    slow = tmp_path / 'slow.py'
    slow.write_text('import time\ntime.sleep(4)\nprint("{}", flush=True)\n')
    assert bench.spawn(2, [sys.executable, str(slow)], teardown=2.0) == 0
    # the default whole-run bound is finite and scaled to the rounds asked for
    a = bench.parse([])
    assert a.launch_timeout == bench.default_launch_timeout(a) >= 1800.0
    assert bench.parse(['--steps', '1000']).launch_timeout > a.launch_timeout
    assert bench.parse(['--launch-timeout', '0']).launch_timeout == 0.0


def test_spawn_teardown_counts_from_the_result_line(tmp_path, capfd):
    """Every rank hangs after rank 0 printed its result line (none exits): the teardown bound
    counts from that line, so the launch still ends (124) with the line relayed."""
    w = tmp_path / 'w.py'
    w.write_text('import os, time\nif os.environ["RANK"] == "0":\n    print("{\\"metric\\": 1}", flush=True)\n'
                 'time.sleep(600)\n')
    import time
    t0 = time.time()
    assert bench.spawn(2, [sys.executable, str(w)], teardown=2.0) == 124
    assert time.time() - t0 < 60
    assert '{"metric": 1}' in capfd.readouterr().out


def test_gpus_must_match_world_size(monkeypatch):
    monkeypatch.setenv('WORLD_SIZE', '2')
    args = bench.parse(['--gpus', '4'])
    with pytest.raises(SystemExit, match='WORLD_SIZE=2'):
        bench.setup_rank(args)


def test_defaults_are_config2():
    a = bench.parse([])
    assert (a.config, a.algo, a.clients, a.D, a.C, a.custom) == (2, 'fedavg', 100, 2048, 10, False)
    assert [c for c, _, _ in bench.LEGS] == [4, 3, 5]


def test_cpu_fedamw_round_is_one_whole_oracle_round():
    """bench.cpu_fedamw_round (config 5's measured CPU baseline, round 6): one whole FedAMW round of
    the oracle -- every client's training, the Z GEMM on every validation row, all R x ceil(n_v / 16)
    p-SGD steps -- on a tiny workload; the sample text states what was timed, and the global torch
    generator is left where it was (the bench's RNG use must not move the workload's)."""
    import numpy as np
    import torch
    rs = np.random.RandomState(3)
    N, n, D, C, nv = 4, 40, 64, 3, 37
    d = {'X_train': [torch.from_numpy(rs.rand(n, D).astype(np.float32)) for _ in range(N)],
         'y_train': [torch.from_numpy(rs.randint(0, C, n)) for _ in range(N)],
         'X_val': torch.from_numpy(rs.rand(nv, D).astype(np.float32)), 'y_val': torch.from_numpy(rs.randint(0, C, nv)),
         'X_test': torch.from_numpy(rs.rand(50, D).astype(np.float32)), 'y_test': torch.from_numpy(rs.randint(0, C, 50))}
    torch.manual_seed(7)
    before = torch.get_rng_state()
    out = bench.cpu_baseline(d, {'D': D, 'C': C, 'algo': 'fedamw'}, 1.0, True, 5, None, whole_max_s=60.0)
    assert out['measured'] is True and out['extrapolation_factor'] == 1.0 and out['value'] > 0
    assert ('%d client trainings' % N) in out['sample'] and ('all %d p-SGD steps' % (5 * ((nv + 15) // 16))) in out['sample']
    assert torch.equal(torch.get_rng_state(), before)
    # without the whole-round budget the FedAMW sample stays an extrapolation, labelled as one
    out = bench.cpu_baseline(d, {'D': D, 'C': C, 'algo': 'fedamw'}, 1.0, True, 5, None)
    assert out['measured'] is False and 'extrapolated' in out['sample']
