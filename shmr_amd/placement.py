"""Multi-GPU placement of StorageBlocks: whole blocks round-robin, no collectives.

StorageBlocks are independent (the reference flushes them in parallel with
rayon, src/vfs/mod.rs:93-96), so N GPUs split a batch by block index:
global block b is handled by rank ``b % N`` (one process per GPU).  The data
path exchanges nothing; the only collectives are the benchmark's timing
barrier and the max-over-ranks of the elapsed time.
"""
from __future__ import annotations

import threading
import time
from typing import Callable, List, Sequence, Tuple


def owner(block: int, world: int) -> int:
    """Rank that encodes/decodes global block ``block``."""
    return block % world


def blocks_for_rank(nblocks: int, rank: int, world: int) -> List[int]:
    """Global block indices owned by ``rank`` (ascending)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError((rank, world))
    return list(range(rank, nblocks, world))


def global_index(local: int, rank: int, world: int) -> int:
    """The global block index of a rank's ``local``-th block."""
    return local * world + rank


def weak_batch(blocks_per_rank: int, rank: int, world: int) -> List[int]:
    """Weak scaling: every rank owns ``blocks_per_rank`` blocks of a global
    batch of ``blocks_per_rank * world`` blocks."""
    return [global_index(j, rank, world) for j in range(blocks_per_rank)]


def max_over_ranks(value: float, device=None) -> float:
    """Max of ``value`` over all ranks (identity without torch.distributed)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def check_partition(parts: Sequence[Sequence[int]], nblocks: int) -> bool:
    """True when the rank partitions are disjoint and cover 0..nblocks-1."""
    seen = sorted(b for part in parts for b in part)
    return seen == list(range(nblocks))


def fan_out(prepare: Sequence[Callable[[], object]], timed: Sequence[Callable[[], object]]
            ) -> Tuple[List[Tuple[object, object]], float]:
    """The single-process multi-GPU shape of the reference daemon (one process,
    src/lib.rs:36-59; blocks fanned out in parallel, src/vfs/mod.rs:93-96):
    one host thread per device.  Thread i runs ``prepare[i]()`` (untimed: clock
    ramp, warmup), all threads meet at a barrier, then each runs ``timed[i]()``.
    The wall clock starts once every device is prepared and stops when the last
    thread returns.  Returns ``([(prepare result, timed result)], wall seconds)``
    in device order.  An exception in any thread breaks the barrier for the
    others and is re-raised here after every thread has exited."""
    n = len(prepare)
    if n != len(timed) or n == 0:
        raise ValueError("one prepare and one timed callable per device")
    barrier = threading.Barrier(n + 1)
    results: List[object] = [None] * n
    errors: List[BaseException] = []

    def body(i):
        try:
            pr = prepare[i]()
            barrier.wait()          # every device ramped and warmed up
            barrier.wait()          # the main thread took t0
            results[i] = (pr, timed[i]())
        except threading.BrokenBarrierError:
            pass
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            errors.append(e)
            barrier.abort()

    threads = [threading.Thread(target=body, args=(i,), name=f"shmr-dev{i}", daemon=True) for i in range(n)]
    for t in threads:
        t.start()
    t0 = None
    try:
        barrier.wait()
        t0 = time.perf_counter()
        barrier.wait()
    except threading.BrokenBarrierError:
        pass
    for t in threads:
        t.join()
    wall = time.perf_counter() - t0 if t0 is not None else 0.0
    if errors:
        raise errors[0]
    return results, wall
