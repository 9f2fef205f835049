"""A 10-second slice of tools/soak.py inside the GPU suite: 8 threads mixing
every entry point -- per-block and started calls, host batches (pageable and
mapped), device batches, pointer tables, and pointer-table encodes captured
into graphs -- each result checked against the CPU oracle.  Guards the
cross-thread capture rules (relaxed capture mode at every entry,
mirrored readiness events), whose faults only show under this concurrency."""
import importlib.util
import os
import threading
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_soak_slice(gpu):
    spec = importlib.util.spec_from_file_location("soak", os.path.join(ROOT, "tools", "soak.py"))
    soak = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(soak)
    threads = 8
    deadline = time.time() + 10
    errors, counts = [], [0] * threads
    th = [threading.Thread(target=soak.worker, args=(t, deadline, errors, counts)) for t in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join(90)
    assert not any(t.is_alive() for t in th), "a soak thread did not finish"
    for e in errors[:5]:
        print(*e, sep="\n", flush=True)
    assert errors == [], errors[:5]
    assert sum(counts) > 100, counts
