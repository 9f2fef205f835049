"""Concurrency: the reference calls ReedSolomon::encode / reconstruct from
rayon workers at once (src/vfs/mod.rs:93-96); the C ABI is documented
reentrant.  16 threads issue mixed calls -- per-block encode and reconstruct
on pageable and mapped buffers, host batches, several (k, p) codecs sharing
the per-codec plan caches and the per-device staging pools -- and every result
is checked against the oracle."""
import threading

import numpy as np
import pytest

import shmr_amd
from oracle import c_oracle

pytestmark = pytest.mark.gpu

SHAPES = [(8, 3, 524288), (4, 2, 65536 + 16), (10, 4, 100003), (6, 6, 4096), (3, 1, 17)]


def _worker(tid, errors, pinned_pool):
    rng = np.random.default_rng([tid, 99])
    try:
        for it in range(12):
            k, p, L = SHAPES[int(rng.integers(0, len(SHAPES)))]
            rs = shmr_amd.ReedSolomon(k, p)
            mapped = bool(rng.integers(0, 2))
            if mapped:
                buf = pinned_pool[tid]
                arr = buf.array[:(k + p) * L].reshape(k + p, L)
                shards = [arr[i] for i in range(k + p)]
            else:
                shards = [np.zeros(L, np.uint8) for _ in range(k + p)]
            for i in range(k):
                shards[i][:] = rng.integers(0, 256, L, dtype=np.uint8)
            rs.encode(shards)
            want = [s.copy() for s in shards[:k]] + [np.zeros(L, np.uint8) for _ in range(p)]
            c_oracle.encode(k, p, want)
            for r in range(p):
                if not np.array_equal(shards[k + r], want[k + r]):
                    errors.append((tid, it, "encode", k, p, L, mapped))
            lost = rng.choice(k + p, size=int(rng.integers(1, p + 1)), replace=False)
            got = [None if i in lost else shards[i].copy() for i in range(k + p)]
            rs.reconstruct(got)
            for i in range(k + p):
                if not np.array_equal(got[i], want[i]):
                    errors.append((tid, it, "reconstruct", k, p, L, i))
            if it % 4 == 3:   # a small host batch now and then
                blocks = [[rng.integers(0, 256, L, dtype=np.uint8) if i < k else np.zeros(L, np.uint8)
                           for i in range(k + p)] for _ in range(3)]
                rs.encode_blocks_host(blocks)
                for blk in blocks:
                    w = [x.copy() for x in blk[:k]] + [np.zeros(L, np.uint8) for _ in range(p)]
                    c_oracle.encode(k, p, w)
                    if not all(np.array_equal(blk[k + r], w[k + r]) for r in range(p)):
                        errors.append((tid, it, "blocks_host", k, p, L))
    except Exception as e:   # surfaced by the main thread
        errors.append((tid, "exception", repr(e)))


def test_concurrent_mixed_calls(gpu):
    n = 16
    pool = [shmr_amd.PinnedBuffer(16 * 524288) for _ in range(n)]
    errors = []
    th = [threading.Thread(target=_worker, args=(t, errors, pool)) for t in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in th), "a worker hung"
    assert not errors, errors[:5]
