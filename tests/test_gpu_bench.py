"""bench.py's output contract, on small batches (the driver parses this line).

Each case runs bench.py once as a child process (one GPU process at a time)
and checks the JSON line: the task's keys, the roofline object, the CPU
baseline (encode and decode legs, each re-checking the GPU's bytes against the
CPU restatement), and the codec round trip.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


def run_bench(*args):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
           "--ramp-seconds", "0.05", "--cpu-seconds", "0.2", *args]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("config,blocks,extra", [("encode83", 16, ()), ("decode83", 16, ()), ("codec104", 4, ()),
                                                ("decode83", 16, ("--rebuild-out", "inplace")),
                                                ("codec104", 4, ("--rebuild-out", "inplace")),
                                                ("encode83", 16, ("--layout", "ptrs")),
                                                ("decode104", 4, ("--layout", "ptrs")),
                                                ("decode83", 16, ("--layout", "ptrs", "--ptrs-alloc", "torch"))])
def test_bench_line_contract(gpu, config, blocks, extra):
    d = run_bench("--config", config, "--blocks", str(blocks), *extra)
    assert KEYS <= set(d)
    assert d["value"] > 0 and d["unit"] == "GiB/s" and d["n_gpus"] == 1 and d["steps"] == 3
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "u8"
    assert d["config"]["workload"] and d["config"]["blocks_per_gpu"] == blocks
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert "traffic" in r               # null here: the PMC table is keyed by the bench batch size
    if "--layout" in extra:               # slab buffers: every timed call ran as a slot grid
        slab = "torch" not in extra
        assert d["config"]["ptr_table_grid_calls_timed"] == (3 if slab else 0)
    pr = d["per_rank"]
    assert len(pr) == 1 and pr[0]["rank"] == 0 and 0 < pr[0]["frac"] < 1
    hp = pr[0]["host_probe"]
    assert hp["parity_equals_device_resident"] is True and hp["zero_copy_blocks"] == hp["blocks"] > 0
    assert sum(hp["blocks_per_device"]) == hp["blocks"]
    c = d["cpu_baseline"]
    assert c["kind"] == "port" and c["cores"] >= 1 and c["value"] > 0 and c["sample"]
    if config == "encode83":
        assert c["gpu_parity_bit_exact_on_sample"] is True
    elif config in ("decode83", "decode104"):
        assert c["gpu_rebuilt_bit_exact_on_sample"] is True
    else:
        assert r["round_trip_bit_exact"] is True
        assert c["gpu_parity_bit_exact_on_sample"] is True and c["gpu_rebuilt_bit_exact_on_sample"] is True


@pytest.mark.gpu
def test_bench_contiguous_vram(gpu):
    d = run_bench("--blocks", "16", "--contig", "--no-cpu")
    assert d["value"] > 0 and "contiguous" in d["config"]["memory"] and d["cpu_baseline"] is None


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["encode83", "codec104"])
def test_bench_single_process_model(gpu, config):
    """--process-model single: one process, one thread + stream per GPU (here
    one GPU); the line names the model and carries the per-device figures."""
    d = run_bench("--config", config, "--blocks", "8", "--process-model", "single")
    assert KEYS <= set(d)
    assert d["process_model"] == "single" and d["launcher"] == "threads"
    assert d["n_gpus"] == 1 and d["ranks_seen"] == 1 and d["distinct_gpus"] == 1
    assert len(d["per_device"]) == 1 and 0 < d["per_device"][0]["frac"] < 1
    assert d["cpu_baseline"]["value"] > 0
    if config == "codec104":
        assert d["roofline"]["round_trip_bit_exact"] is True


@pytest.mark.gpu
def test_bench_single_process_model_eight_devices(gpu):
    """--process-model single --gpus 8, rehearsed on one card
    (SHMR_BENCH_SHARE_GPU=1: eight device slots, eight host threads and
    streams on the same GPU): one line, eight per-device figures, global
    batch 8 x B, the codec round trip exact on every device."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--ramp-seconds", "0.05",
           "--no-cpu", "--config", "codec104", "--blocks", "2", "--process-model", "single", "--gpus", "8"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=150,
                         env=dict(os.environ, SHMR_BENCH_SHARE_GPU="1"))
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["process_model"] == "single" and d["n_gpus"] == 8 and d["distinct_gpus"] == 1
    assert len(d["per_device"]) == 8 and all(0 < x["frac"] < 1 for x in d["per_device"])
    assert d["config"]["global_batch_blocks"] == 16 and d["value"] > 0
    assert d["roofline"]["round_trip_bit_exact"] is True and d["cpu_baseline"] is None
