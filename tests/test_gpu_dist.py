"""Multi-process GPU runs, rehearsed on one GPU (ranks share the card,
SHMR_BENCH_SHARE_GPU=1): the library under torch.distributed with whole
blocks round-robin, checked against the CPU oracle, and bench.py's own
multi-rank launch.  The 8-GPU node runs the same code with one GPU per rank.
"""
import hashlib
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import c_oracle
from shmr_amd import placement

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gpu_dist_worker as W  # noqa: E402


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    return dict(os.environ, SHMR_BENCH_SHARE_GPU="1", MASTER_ADDR="127.0.0.1")


@pytest.mark.parametrize("world", [2, 3, 8])
def test_library_round_robin_ranks(gpu, world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tests", "gpu_dist_worker.py")]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=150, env=_env())
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["world"] == world and len(res["ranks"]) == world
    seen = {}
    for r, part in enumerate(res["ranks"]):
        assert part["rebuilt_ok"], f"rank {r} rebuilt shards differ"
        for b, rec in part["blocks"].items():
            b = int(b)
            assert rec["rank"] == r == placement.owner(b, world)
            seen[b] = rec["parity_sha256"]
    assert sorted(seen) == list(range(W.NBLOCKS))
    for b in range(W.NBLOCKS):
        d = W.block_data(b)
        sh = [d[i].copy() for i in range(W.K)] + [np.zeros(W.S, np.uint8) for _ in range(W.P)]
        c_oracle.encode(W.K, W.P, sh)
        assert seen[b] == hashlib.sha256(np.stack(sh[W.K:]).tobytes()).hexdigest(), b


@pytest.mark.parametrize("config", ["encode83", "decode83"])
def test_bench_self_launch_two_ranks(gpu, config):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", config, "--blocks", "16",
           "--steps", "3", "--warmup", "1", "--ramp-seconds", "0.05", "--no-cpu"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=150, env=_env())
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    b = json.loads(lines[0])
    assert b["n_gpus"] == 2 and b["ranks_seen"] == 2 and b["launcher"] == "spawn"
    assert b["config"]["global_batch_blocks"] == 32 and b["value"] > 0 and b["cpu_baseline"] is None
    assert [d["rank"] for d in b["devices"]] == [0, 1]


def test_bench_self_launch_eight_ranks(gpu, tmp_path):
    """bench.py --gpus 8 as the driver's 8-GPU run starts it, on one GPU
    (SHMR_BENCH_SHARE_GPU=1): eight ranks join, the line counts them and
    reports the one physical GPU honestly (distinct_gpus 1), the global batch
    is 8 x B blocks round-robin, and every rank's coded blocks equal the
    oracle's (each rank dumps its first blocks after the timed region)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--blocks", "4", "--steps", "3",
           "--warmup", "1", "--ramp-seconds", "0.05", "--no-cpu", "--dump-dir", str(tmp_path), "--dump-blocks", "2"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=_env())
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout[-2000:]    # nothing else on stdout
    b = json.loads(lines[0])
    assert b["n_gpus"] == 8 and b["ranks_seen"] == 8 and b["launcher"] == "spawn"
    assert [d["rank"] for d in b["devices"]] == list(range(8))
    assert b["distinct_gpus"] == 1                 # one physical GPU shared by the eight ranks
    assert b["config"]["global_batch_blocks"] == 32 and b["scaling"] == "weak" and b["value"] > 0
    assert [r["rank"] for r in b["per_rank"]] == list(range(8))
    for r in b["per_rank"]:      # every rank's host-path probe: zero-copy, same parity as device-resident
        hp = r["host_probe"]
        assert hp["parity_equals_device_resident"] is True and hp["zero_copy_blocks"] == hp["blocks"], r
    seen = []
    for r in range(8):
        z = np.load(os.path.join(str(tmp_path), f"rank{r}.npz"))
        data, parity, blocks = z["data"], z["parity"], z["blocks"]
        assert list(blocks) == placement.weak_batch(4, r, 8)[:2]
        assert all(placement.owner(int(g), 8) == r for g in blocks)
        seen.extend(int(g) for g in blocks)
        n, k, S = data.shape
        want = np.zeros((n, parity.shape[1], S), np.uint8)
        c_oracle.encode_batch(k, parity.shape[1], np.ascontiguousarray(data), want, n, S, 8)
        assert np.array_equal(parity, want), f"rank {r}"
    assert len(set(seen)) == 16
