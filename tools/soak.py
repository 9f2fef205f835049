#!/usr/bin/env python3
"""Randomised multi-threaded soak of the C ABI on one GPU, every result checked
against the CPU oracle: per-block encode / reconstruct on pageable and mapped
buffers (zero-copy, bounce, staged DMA), host batches on pageable arrays
(pinned mirror) and mapped slabs, device-resident batches on per-thread
torch streams, per-shard device buffers through pointer tables (reused, so
the device's table cache hits), started per-block calls (shmr_ec_*_start) and
pointer-table encodes captured into graphs and destroyed again (the capture
reserve), device Block Cache slots after churn (shmr_ec_pool_*) through the
submission queue's merged per-block calls and through pointer-table batches --
several (k, p) codecs and shard lengths (aligned, tail,
byte-granular) at once.  Not part of the test suite (minutes of GPU time).

    python tools/soak.py [--seconds 120] [--threads 12]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import shmr_amd  # noqa: E402
from oracle import c_oracle  # noqa: E402

SHAPES = [(8, 3, 524288), (8, 3, 4096), (4, 2, 65536 + 16), (10, 4, 100003), (6, 6, 777), (3, 1, 17), (17, 7, 8192)]


def oracle_encode(k, p, data):
    L = len(data[0])
    sh = [np.ascontiguousarray(d).copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(p)]
    c_oracle.encode(k, p, sh)
    return sh


class CaptureGate:
    """Graph captures (op 6) against the legacy default stream: torch work on the
    null stream (op 4's default-stream branch, the .cpu() reads and allocations
    outside a stream context in ops 3-4, 7-9) synchronises implicitly with every
    stream and would join -- and invalidate -- another thread's capture (a
    HIP / CUDA rule, not the library's).  Captures run exclusively against ops
    3-4 and 7-9; the host-buffer ops (0-2, 5), which use only the library's own
    non-blocking streams, run alongside them."""

    def __init__(self):
        self.cv = threading.Condition()
        self.readers = 0
        self.writer = False

    def shared(self):
        gate = self

        class _S:
            def __enter__(self):
                with gate.cv:
                    gate.cv.wait_for(lambda: not gate.writer)
                    gate.readers += 1

            def __exit__(self, *exc):
                with gate.cv:
                    gate.readers -= 1
                    gate.cv.notify_all()
        return _S()

    def exclusive(self):
        gate = self

        class _X:
            def __enter__(self):
                with gate.cv:
                    gate.cv.wait_for(lambda: not gate.writer and gate.readers == 0)
                    gate.writer = True

            def __exit__(self, *exc):
                with gate.cv:
                    gate.writer = False
                    gate.cv.notify_all()
        return _X()


GATE = CaptureGate()


class _Nothing:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


def worker(tid, deadline, errors, counts, ops=tuple(range(10)), shapes=tuple(range(len(SHAPES)))):
    rng = np.random.default_rng([tid, 2024])
    stream = torch.cuda.Stream()
    slab = shmr_amd.PinnedBuffer(4 * 24 * 524288)
    kept = {}   # (shape, set) -> per-shard device buffers reused across calls (pointer-table cache hits)
    while time.time() < deadline and not errors:
        k, p, L = SHAPES[shapes[int(rng.integers(0, len(shapes)))]]
        rs = shmr_amd.ReedSolomon(k, p)
        op = ops[int(rng.integers(0, len(ops)))]
        gate = GATE.exclusive() if op == 6 else GATE.shared() if op in (3, 4, 7, 8, 9) else _Nothing()
        try:
            with gate:
                if op == 0:        # per-block calls, pageable or mapped
                    mapped = bool(rng.integers(0, 2))
                    if mapped:
                        arr = slab.array[:(k + p) * L].reshape(k + p, L)
                        shards = [arr[i] for i in range(k + p)]
                    else:
                        shards = [np.zeros(L, np.uint8) for _ in range(k + p)]
                    for i in range(k):
                        shards[i][:] = rng.integers(0, 256, L, dtype=np.uint8)
                    rs.encode(shards)
                    want = oracle_encode(k, p, shards[:k])
                    if not all(np.array_equal(shards[i], want[i]) for i in range(k, k + p)):
                        errors.append((tid, "encode", k, p, L, mapped))
                    lost = rng.choice(k + p, size=int(rng.integers(1, p + 1)), replace=False)
                    got = [None if i in lost else shards[i].copy() for i in range(k + p)]
                    rs.reconstruct(got)
                    if not all(np.array_equal(got[i], want[i]) for i in range(k + p)):
                        errors.append((tid, "reconstruct", k, p, L, mapped))
                elif op == 1:      # host batch on a pageable [B, t, L] array (pinned mirror)
                    B = int(rng.integers(1, 6))
                    blk = np.zeros((B, k + p, L), np.uint8)
                    blk[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
                    rs.encode_blocks_host(blk)
                    full = blk.copy()
                    for b in range(B):
                        want = oracle_encode(k, p, list(blk[b, :k]))
                        if not all(np.array_equal(blk[b, i], want[i]) for i in range(k, k + p)):
                            errors.append((tid, "blocks_host encode", k, p, L, B))
                    present = np.ones((B, k + p), np.uint8)
                    for b in range(B):
                        present[b, rng.choice(k + p, size=int(rng.integers(1, p + 1)), replace=False)] = 0
                    blk[present == 0] = 0
                    rs.reconstruct_blocks_host(blk, present)
                    if not np.array_equal(blk, full):
                        errors.append((tid, "blocks_host reconstruct", k, p, L, B))
                elif op == 2:      # host batch on the mapped slab (zero-copy)
                    B = int(min(4, (slab.nbytes // ((k + p) * L))))
                    if B == 0:
                        continue
                    blk = slab.array[:B * (k + p) * L].reshape(B, k + p, L)
                    blk[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
                    rs.encode_blocks_host(blk)
                    for b in range(B):
                        want = oracle_encode(k, p, list(blk[b, :k]))
                        if not all(np.array_equal(blk[b, i], want[i]) for i in range(k, k + p)):
                            errors.append((tid, "mapped batch encode", k, p, L, B))
                elif op == 5:      # started per-block calls (shmr_ec_*_start + shmr_ec_op_wait), mapped or pageable
                    import ctypes
                    from shmr_amd.reed_solomon import _ptr, _u8p
                    mapped = bool(rng.integers(0, 2))
                    if mapped:
                        arr = slab.array[:(k + p) * L].reshape(k + p, L)
                        shards = [arr[i] for i in range(k + p)]
                    else:
                        shards = [np.zeros(L, np.uint8) for _ in range(k + p)]
                    for i in range(k):
                        shards[i][:] = rng.integers(0, 256, L, dtype=np.uint8)
                    tab = (_u8p * (k + p))(*[_ptr(x) for x in shards])
                    lens = (ctypes.c_size_t * (k + p))(*([L] * (k + p)))
                    h = ctypes.c_void_p()
                    assert rs._L.shmr_ec_encode_start(rs._h, tab, lens, k + p, ctypes.byref(h)) == 0
                    assert rs._L.shmr_ec_op_wait(h) == 0
                    want = oracle_encode(k, p, shards[:k])
                    if not all(np.array_equal(shards[i], want[i]) for i in range(k, k + p)):
                        errors.append((tid, "encode_start", k, p, L, mapped))
                    present = np.ones(k + p, np.uint8)
                    present[rng.choice(k + p, size=int(rng.integers(1, p + 1)), replace=False)] = 0
                    for i in np.flatnonzero(present == 0):
                        shards[i][:] = 0xEE
                        lens[i] = 0
                    assert rs._L.shmr_ec_reconstruct_start(rs._h, tab, lens, _ptr(present), k + p, 0, ctypes.byref(h)) == 0
                    assert rs._L.shmr_ec_op_wait(h) == 0
                    if not all(np.array_equal(shards[i], want[i]) for i in range(k + p)):
                        errors.append((tid, "reconstruct_start", k, p, L, mapped))
                elif op == 6:      # a pointer-table encode captured into a graph (capture reserve), replayed, destroyed
                    B = int(rng.integers(1, 5))
                    host = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
                    # allocated and filled on this thread's stream (a fill on the legacy
                    # stream would race the non-blocking stream's copies)
                    with torch.cuda.stream(stream):
                        blocks = [[torch.empty(L, dtype=torch.uint8, device="cuda") for _ in range(k + p)]
                                  for _ in range(B)]
                        for b in range(B):
                            for i in range(k):
                                blocks[b][i].copy_(torch.from_numpy(host[b, i]).cuda())
                    stream.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
                        rs.encode_ptrs_dev(blocks)
                    g.replay()
                    stream.synchronize()
                    for b in range(B):
                        want = oracle_encode(k, p, list(host[b]))
                        if not all(np.array_equal(blocks[b][i].cpu().numpy(), want[i]) for i in range(k, k + p)):
                            errors.append((tid, "captured ptrs encode", k, p, L, B))
                            break
                    del g
                elif op == 4:      # per-shard device buffers (pointer tables), on this thread's stream or the default one
                    key = (k, p, L, int(rng.integers(0, 3)))
                    if key not in kept:
                        B = int(rng.integers(1, 6))
                        kept[key] = [[torch.empty(L, dtype=torch.uint8, device="cuda") for _ in range(k + p)]
                                     for _ in range(B)]
                    blocks = kept[key]
                    B = len(blocks)
                    host = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
                    st = stream if rng.integers(0, 4) else torch.cuda.current_stream()
                    with torch.cuda.stream(st):
                        for b in range(B):
                            for i in range(k):
                                blocks[b][i].copy_(torch.from_numpy(host[b, i]).cuda(), non_blocking=False)
                        rs.encode_ptrs_dev(blocks)
                        lost = [sorted(rng.choice(k + p, size=int(rng.integers(1, p + 1)), replace=False).tolist())
                                for _ in range(B)]
                        partial = [[None if i in lost[b] else blocks[b][i] for i in range(k + p)] for b in range(B)]
                        rs.reconstruct_ptrs_dev(partial)
                    st.synchronize()
                    for b in range(B):
                        want = oracle_encode(k, p, list(host[b]))
                        if not all(np.array_equal(blocks[b][i].cpu().numpy(), want[i]) for i in range(k, k + p)):
                            errors.append((tid, "ptrs encode", k, p, L, B))
                            break
                        if not all(np.array_equal(partial[b][i].cpu().numpy(), want[i]) for i in lost[b]):
                            errors.append((tid, "ptrs reconstruct", k, p, L, B))
                            break
                elif op == 7:      # slab buffers (shmr_ec_device_alloc_shards): grid pointer tables, strided kernels
                    import ctypes
                    from shmr_amd.reed_solomon import _u8p
                    key = ("slab", k, p, L)
                    if key not in kept:
                        B = int(rng.integers(1, 6))
                        kept[key] = (shmr_amd.ShardSlab(B, k, L), shmr_amd.ShardSlab(B, p, L),
                                     shmr_amd.ShardSlab(B, k + p, L), shmr_amd.ShardSlab(B, p, L))
                    ds, ps, js, outs = kept[key]
                    B = ds.nblocks
                    host = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
                    sp = ctypes.c_void_p(stream.cuda_stream)
                    tab = np.ascontiguousarray(np.concatenate([ds.ptrs.reshape(B, k), ps.ptrs.reshape(B, p)], axis=1))
                    present = np.ones((B, k + p), np.uint8)
                    for b in range(B):
                        present[b, rng.choice(k + p, size=int(rng.integers(1, p + 1)), replace=False)] = 0
                    fresh = js.ptrs.reshape(B, k + p).copy()   # rebuilt shard j of block b -> outs slot (b, j)
                    for b in range(B):
                        for j, i in enumerate(np.flatnonzero(present[b] == 0)):
                            fresh[b, i] = outs.ptrs[b * p + j]
                    fresh = np.ascontiguousarray(fresh)
                    with torch.cuda.stream(stream):
                        ds.tensor()[:, :, :L] = torch.from_numpy(host).cuda()
                        assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab.ctypes.data_as(ctypes.POINTER(_u8p)), B, L, 0,
                                                             sp) == 0
                        jv = js.tensor()
                        jv[:, :k, :L] = ds.tensor()[:, :, :L]
                        jv[:, k:, :L] = ps.tensor()[:, :, :L]
                        full = jv[:, :, :L].clone()
                        jv[:, :, :L][torch.from_numpy(present == 0).cuda()] = 0xEE
                        assert rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, fresh.ctypes.data_as(ctypes.POINTER(_u8p)),
                                                                  present.ctypes.data_as(_u8p), B, L, 0, 0, sp) == 0
                        rebuilt = outs.tensor()[:, :, :L].clone()
                        assert rs._L.shmr_ec_reconstruct_ptrs_dev(
                            rs._h, js.ptrs.ctypes.data_as(ctypes.POINTER(_u8p)), present.ctypes.data_as(_u8p), B, L,
                            0, 0, sp) == 0
                    stream.synchronize()
                    h, hr = full.cpu().numpy(), rebuilt.cpu().numpy()
                    if not np.array_equal(js.tensor()[:, :, :L].cpu().numpy(), h):
                        errors.append((tid, "slab rebuild in place", k, p, L, B))
                    for b in range(B):
                        want = oracle_encode(k, p, list(host[b]))
                        if not all(np.array_equal(h[b, i], want[i]) for i in range(k, k + p)):
                            errors.append((tid, "slab encode", k, p, L, B))
                            break
                        if not all(np.array_equal(hr[b, j], h[b, i])
                                   for j, i in enumerate(np.flatnonzero(present[b] == 0))):
                            errors.append((tid, "slab rebuild fresh", k, p, L, B))
                            break
                elif op in (8, 9):  # device Block Cache slots (shmr_ec_pool_*) after churn, blocks in shuffled
                    #                 order: per-block calls through the submission queue (8: plain or
                    #                 started, merged with other threads' calls) or one pointer-table
                    #                 batch on this thread's stream (9: the slot lattice or the table path)
                    import ctypes
                    from shmr_amd.reed_solomon import _ptr, _u8p
                    key = ("pool", k, p, L)
                    if key not in kept:
                        kept[key] = (shmr_amd.ShardPool(k + p, L, 8), [])
                    pool, live = kept[key]
                    for _ in range(int(rng.integers(0, 6))):    # churn (past 8 live blocks: a second slab)
                        if live and rng.integers(0, 2):
                            pool.free(live.pop(int(rng.integers(0, len(live)))))
                        elif len(live) < 12:
                            live.append(pool.alloc())
                    if not live:
                        live.append(pool.alloc())
                    order = [live[int(j)] for j in rng.permutation(len(live))]
                    B = len(order)
                    host = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
                    with torch.cuda.stream(stream):
                        hd = torch.from_numpy(host).cuda()
                        for b in range(B):
                            for i in range(k):
                                pool.shard(order[b], i).copy_(hd[b, i])
                    stream.synchronize()                        # queue inputs complete before the call
                    present = np.ones((B, k + p), np.uint8)
                    for b in range(B):
                        present[b, rng.choice(k + p, size=int(rng.integers(1, p + 1)), replace=False)] = 0
                    data_only = op == 8 and bool(rng.integers(0, 4) == 0)
                    start = bool(rng.integers(0, 2))
                    tab = np.ascontiguousarray(np.stack(order))
                    sp = ctypes.c_void_p(stream.cuda_stream)
                    if op == 8:
                        pend = [rs.encode_dev([(int(a), L) for a in blk], start=start) for blk in order]
                        for o in pend:
                            if o is not None:
                                o.wait()
                    else:
                        assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab.ctypes.data_as(ctypes.POINTER(_u8p)), B, L, 0,
                                                             sp) == 0
                    with torch.cuda.stream(stream):
                        enc = torch.stack([torch.stack([pool.shard(blk, i) for i in range(k + p)]) for blk in order])
                        full = enc.cpu().numpy()
                        for b in range(B):
                            for i in np.flatnonzero(present[b] == 0):
                                pool.shard(order[b], int(i)).fill_(0xEE)
                    stream.synchronize()
                    bad = False
                    for b in range(B):
                        want = oracle_encode(k, p, list(host[b]))
                        if not all(np.array_equal(full[b, i], want[i]) for i in range(k, k + p)):
                            errors.append((tid, "pool encode", op, k, p, L, B))
                            bad = True
                            break
                    if bad:
                        continue
                    if op == 8:
                        pend = []
                        for b, blk in enumerate(order):
                            row = [None if (data_only and i >= k and not present[b, i]) else (int(blk[i]), L)
                                   for i in range(k + p)]
                            pend.append(rs.reconstruct_dev(row, present[b], data_only=data_only, start=start))
                        for o in pend:
                            if o is not None:
                                o.wait()
                    else:
                        assert rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab.ctypes.data_as(ctypes.POINTER(_u8p)),
                                                                  _ptr(present), B, L, 0, 0, sp) == 0
                    with torch.cuda.stream(stream):
                        got = torch.stack([torch.stack([pool.shard(blk, i) for i in range(k + p)])
                                           for blk in order]).cpu().numpy()
                    for b in range(B):
                        rows = range(k) if data_only else range(k + p)
                        if not all(np.array_equal(got[b, i], full[b, i]) for i in rows):
                            errors.append((tid, "pool reconstruct", op, k, p, L, B, data_only))
                            break
                else:              # device-resident batch on this thread's stream: encode, in-place and compact rebuild
                    B = int(rng.integers(1, 9))
                    P = (L + 255) // 256 * 256
                    with torch.cuda.stream(stream):
                        d = torch.zeros((B, k + p, P), dtype=torch.uint8, device="cuda")
                        host = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
                        d[:, :k, :L] = torch.from_numpy(host).cuda()
                        rs.encode_batch_dev(d[:, :k], d[:, k:], shard_len=L)
                        present = np.ones((B, k + p), np.uint8)
                        for b in range(B):
                            present[b, rng.choice(k + p, size=int(rng.integers(1, p + 1)), replace=False)] = 0
                        full = d.clone()
                        erased = torch.from_numpy(present == 0).cuda()
                        d[erased] = 0
                        rs.reconstruct_batch_dev(d, present, shard_len=L)
                        ok = torch.equal(d[:, :, :L], full[:, :, :L])
                        # compact rebuild (the crate's fresh-buffer semantics) from a copy
                        # whose erased slots are poisoned: they must not be read
                        src = full.clone()
                        src[erased] = 0xEE
                        out = torch.zeros((B, int((present == 0).sum(axis=1).max()), P), dtype=torch.uint8, device="cuda")
                        rs.reconstruct_batch_dev_out(src, present, out, shard_len=L)
                    stream.synchronize()
                    h = full.cpu().numpy()
                    ho = out.cpu().numpy()
                    for b in range(B):
                        for j, i in enumerate(np.flatnonzero(present[b] == 0)):
                            if not np.array_equal(ho[b, j, :L], h[b, i, :L]):
                                errors.append((tid, "batch_dev compact", k, p, L, B))
                                break
                    for b in range(B):
                        want = oracle_encode(k, p, list(host[b]))
                        if not all(np.array_equal(h[b, i, :L], want[i]) for i in range(k, k + p)):
                            errors.append((tid, "batch_dev encode", k, p, L, B))
                    if not ok:
                        errors.append((tid, "batch_dev reconstruct", k, p, L, B))
                counts[tid] += 1
        except Exception as e:   # surfaced by the main thread
            import traceback
            errors.append((tid, "exception", op, k, p, L, repr(e), traceback.format_exc(limit=4)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--threads", type=int, default=12)
    ap.add_argument("--ops", default="0,1,2,3,4,5,6,7,8,9", help="subset of the operations (comma list)")
    ap.add_argument("--shapes", default=",".join(str(i) for i in range(len(SHAPES))),
                    help="subset of SHAPES (indices)")
    a = ap.parse_args()
    ops = tuple(int(x) for x in a.ops.split(","))
    shapes = tuple(int(x) for x in a.shapes.split(","))
    deadline = time.time() + a.seconds
    errors, counts = [], [0] * a.threads
    th = [threading.Thread(target=worker, args=(t, deadline, errors, counts, ops, shapes)) for t in range(a.threads)]
    for t in th:
        t.start()
    last = time.time()
    while any(t.is_alive() for t in th):
        time.sleep(1)
        if time.time() - last > 30:
            print(json.dumps({"progress_ops": sum(counts), "errors": len(errors)}), flush=True)
            last = time.time()
    zc, st = shmr_amd.path_stats()
    print(json.dumps({"ops": sum(counts), "threads": a.threads, "seconds": a.seconds, "errors": errors[:5],
                      "zero_copy_blocks": zc, "staged_blocks": st,
                      "ptr_table_hits": shmr_amd.device_stats(0)["ptr_table_hits"],
                      "capture_tables": shmr_amd.device_stats(0)["capture_tables"],
                      "capture_released": shmr_amd.device_stats(0)["capture_released"],
                      "ptr_table_grids": shmr_amd.device_stats(0)["ptr_table_grids"]}), flush=True)
    sys.exit(1 if errors else 0)


if __name__ == "__main__":
    main()
