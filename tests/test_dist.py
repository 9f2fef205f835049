"""World-size-2 gloo tests (CPU) of the multi-GPU path: whole StorageBlocks
round-robin over ranks, no data-path collective, max-over-ranks timing.

The per-rank compute here is the CPU oracle standing in for each rank's GPU
(this file runs without a GPU); the GPU box exercises the same placement
through bench.py.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from shmr_amd import placement


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, nblocks, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import c_oracle
        from oracle import rs_oracle as O
        k, p, S = 4, 2, 4096
        mine = placement.blocks_for_rank(nblocks, rank, world)
        digests = {}
        for b in mine:
            data = O.seeded_block(O.BENCH_SEED, b, k * S)
            sh = [data[i * S:(i + 1) * S].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
            c_oracle.encode(k, p, sh)
            digests[b] = hashlib.sha256(b"".join(x.tobytes() for x in sh[k:])).hexdigest()
        gathered = [None] * world
        dist.all_gather_object(gathered, digests)       # test-side check only
        elapsed = placement.max_over_ranks(1.0 + rank)
        out_q.put((rank, mine, gathered, elapsed))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nblocks", [(2, 11), (8, 29)])
def test_round_robin_partition(world, nblocks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nblocks, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    results.sort()
    parts = [r[1] for r in results]
    assert placement.check_partition(parts, nblocks)
    if world == 2:
        assert parts[0] == [0, 2, 4, 6, 8, 10] and parts[1] == [1, 3, 5, 7, 9]
    for r, part in enumerate(parts):
        assert part == list(range(r, nblocks, world))
    assert all(r[3] == float(world) for r in results)      # max over ranks (rank r reports 1 + r)
    # every rank's parity equals a single-process encode of the same block
    from oracle import c_oracle
    from oracle import rs_oracle as O
    merged = {}
    for d in results[0][2]:
        merged.update(d)
    assert sorted(merged) == list(range(nblocks))
    k, p, S = 4, 2, 4096
    for b in range(nblocks):
        data = O.seeded_block(O.BENCH_SEED, b, k * S)
        sh = [data[i * S:(i + 1) * S].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
        c_oracle.encode(k, p, sh)
        assert merged[b] == hashlib.sha256(b"".join(x.tobytes() for x in sh[k:])).hexdigest()


def test_weak_batch_indices():
    for world in (1, 2, 4, 8):
        parts = [placement.weak_batch(5, r, world) for r in range(world)]
        assert placement.check_partition(parts, 5 * world)
        for r in range(world):
            assert all(placement.owner(b, world) == r for b in parts[r])


def test_bad_rank():
    with pytest.raises(ValueError):
        placement.blocks_for_rank(4, 2, 2)
