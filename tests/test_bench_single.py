"""bench.py --process-model single: the reference daemon's shape (one process
drives every GPU, src/lib.rs:36-59, blocks fanned out in parallel,
src/vfs/mod.rs:93-96), rehearsed on CPU -- the thread orchestration, timing
and error handling of shmr_amd.placement.fan_out, and the bench's wiring."""
import os
import sys
import threading
import time

import pytest

from shmr_amd import placement

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fan_out_runs_devices_concurrently():
    order = []
    lock = threading.Lock()

    def prep(i):
        def f():
            time.sleep(0.02 * (3 - i))        # uneven ramps: the barrier waits for the slowest
            with lock:
                order.append(("prep", i))
            return i * 10
        return f

    def timed(i):
        def f():
            with lock:
                order.append(("timed", i))
            time.sleep(0.2)
            return [float(i)] * 3
        return f

    res, wall = placement.fan_out([prep(i) for i in range(3)], [timed(i) for i in range(3)])
    assert res == [(0, [0.0] * 3), (10, [1.0] * 3), (20, [2.0] * 3)]
    # every prepare finished before any timed section started
    assert [x[0] for x in order[:3]] == ["prep"] * 3 and [x[0] for x in order[3:]] == ["timed"] * 3
    assert 0.19 < wall < 0.5, wall                  # concurrent: ~0.2 s, not 0.6 s


def test_fan_out_propagates_a_failing_device():
    def boom():
        raise RuntimeError("device 1 failed")

    started = []
    with pytest.raises(RuntimeError, match="device 1 failed"):
        placement.fan_out([lambda: 0, boom, lambda: 2],
                          [lambda: started.append(0), lambda: None, lambda: started.append(2)])
    assert started == []                             # nobody entered the timed section


def test_fan_out_failure_in_timed_section():
    def bad():
        raise ValueError("timed failure")

    with pytest.raises(ValueError):
        placement.fan_out([lambda: 0, lambda: 1], [lambda: 1, bad])


def test_fan_out_rejects_mismatched_lists():
    with pytest.raises(ValueError):
        placement.fan_out([lambda: 0], [])
    with pytest.raises(ValueError):
        placement.fan_out([], [])


def test_single_model_partition_is_round_robin():
    """Device d of N owns global blocks d + j * N: disjoint, complete."""
    n, B = 8, 512
    parts = [placement.weak_batch(B, d, n) for d in range(n)]
    assert placement.check_partition(parts, B * n)
    assert parts[3][:3] == [3, 11, 19]


def test_bench_single_model_is_wired():
    """--process-model single never goes through the launcher, refuses to run
    under one, and its line names the model (source check: no GPU here)."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    main = src[src.index("def main():"):src.index("def run(args):") if "def run(args):" in src[src.index("def main():"):] else None]
    assert main.index('args.process_model == "single"') < main.index("launch(")
    assert "def run_single(args):" in src and "placement.fan_out(" in src
    assert '"process_model": process_model' in src
    sys.path.insert(0, ROOT)
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--process-model", "single", "--gpus", "2"],
                       capture_output=True, text=True, env=env, timeout=120, cwd=ROOT)
    assert r.returncode != 0 and "one process" in r.stderr
