"""bench.py's multi-GPU launch, rehearsed on CPU (gloo, no GPU).

`bench.py --gpus N` must produce one JSON line whether the driver starts it
under torch.distributed.run or directly: started directly, the parent spawns
N worker processes (rank r -> GPU r) before touching the GPU and relays their
exit status.  --launch-check runs the launcher and the process group without
the GPU work.  Reference fan-out being mirrored: src/vfs/mod.rs:91-103.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(cmd, env=None, timeout=180):
    e = dict(os.environ, MASTER_ADDR="127.0.0.1")
    e.pop("WORLD_SIZE", None)
    e.pop("RANK", None)
    e.pop("MASTER_PORT", None)
    e.update(env or {})
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e, cwd=ROOT)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _json_lines(out):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def test_direct_launch_spawns_ranks():
    r = _run([sys.executable, BENCH, "--gpus", "3", "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout            # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == 3 and line["ranks_seen"] == 3
    assert [x["rank"] for x in line["ranks"]] == [0, 1, 2]
    assert [x["local_rank"] for x in line["ranks"]] == [0, 1, 2]
    assert len({x["pid"] for x in line["ranks"]}) == 3
    assert {x["launcher"] for x in line["ranks"]} == {"spawn"}


def test_torchrun_launch_still_works():
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), BENCH, "--gpus", "2", "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1 and lines[0]["ranks_seen"] == 2
    assert {x["launcher"] for x in lines[0]["ranks"]} == {"torchrun"}


def test_a_failing_rank_fails_the_launch():
    """A rank that dies before joining leaves the others waiting in the
    rendezvous: the parent stops them and exits with the failing status."""
    r = _run([sys.executable, BENCH, "--gpus", "2", "--launch-check"],
             env={"SHMR_BENCH_LAUNCH_FAIL_RANK": "1"}, timeout=120)
    assert r.returncode == 3
    assert not _json_lines(r.stdout)


def test_single_rank_needs_no_launcher():
    r = _run([sys.executable, BENCH, "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = _json_lines(r.stdout)[0]
    assert line["ranks_seen"] == 1 and line["n_gpus"] == 1


def test_parent_never_touches_the_gpu():
    """The launcher path runs before torch / the HIP library are imported."""
    src = open(BENCH).read()
    head = src[:src.index("def run(args):")]
    assert "\nimport torch" not in head and "\nimport shmr_amd" not in head
    main = src[src.index("def main():"):src.index("def run(args):")]
    assert main.index("launch(") < main.index("run(args)")


def test_traffic_is_reported_only_for_the_profiled_build(tmp_path, monkeypatch):
    """roofline.traffic comes from profiles/pmc_traffic.json only when the
    record names the running kernel build, variant and batch size."""
    sys.path.insert(0, ROOT)
    import bench
    (tmp_path / "profiles").mkdir()
    rec = {"encode83": {"build_id": "abc123abc123", "variant": "v1", "blocks": 512, "hbm_bytes_per_launch": 42}}
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "HERE", str(tmp_path))
    t, src = bench.load_traffic("encode83", 512, "abc123abc123", "v1")
    assert t == 42 and src["status"] == "match" and src["file"] == "profiles/pmc_traffic.json"
    for args in (("encode83", 512, "000000000000", "v1"), ("encode83", 512, "abc123abc123", "v2"),
                 ("encode83", 256, "abc123abc123", "v1")):
        t, src = bench.load_traffic(*args)
        assert t is None and src["status"].startswith("stale")
    t, src = bench.load_traffic("decode83", 512, "abc123abc123", "v1")
    assert t is None and src["status"] == "no record for this config"


def test_cpu_threads_default_is_available_parallelism(monkeypatch):
    """rayon's default pool = std::thread::available_parallelism(): the
    affinity set capped by the cgroup v2 quota (rounded up)."""
    sys.path.insert(0, ROOT)
    import bench
    aff = len(os.sched_getaffinity(0))
    monkeypatch.setattr(bench, "cpu_quota", lambda: None)
    assert bench.cpu_threads(0) == aff
    monkeypatch.setattr(bench, "cpu_quota", lambda: 1.5)
    assert bench.cpu_threads(0) == min(aff, 2)
    monkeypatch.setattr(bench, "affinity_cores", lambda: 256)
    monkeypatch.setattr(bench, "cpu_quota", lambda: 16.0)
    assert bench.cpu_threads(0) == 16
    assert bench.cpu_threads(5) == 5


def test_direct_launch_eight_ranks():
    """The driver's N = 8 launch shape (bench.py started directly): eight
    ranks, one line, ranks 0..7 with their own processes -- and nothing else
    on stdout (Gloo's connection messages go to stderr)."""
    r = _run([sys.executable, BENCH, "--gpus", "8", "--launch-check"], timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(r.stdout.strip().splitlines()) == 1, r.stdout[:2000]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1 and lines[0]["ranks_seen"] == 8 and lines[0]["n_gpus"] == 8
    assert [x["rank"] for x in lines[0]["ranks"]] == list(range(8))
    assert len({x["pid"] for x in lines[0]["ranks"]}) == 8


def test_torchrun_launch_eight_ranks():
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), BENCH, "--gpus", "8", "--launch-check"],
             timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(r.stdout.strip().splitlines()) == 1, r.stdout[:2000]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1 and lines[0]["ranks_seen"] == 8
    assert [x["local_rank"] for x in lines[0]["ranks"]] == list(range(8))
