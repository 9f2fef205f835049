"""The submission queue (include/shmr_ec.h shmr_ec_encode_dev /
shmr_ec_reconstruct_dev and their *_start forms; the host-buffer calls on
mapped memory under knob "coalesce") vs the CPU oracle, bit-exact.

The reference codes ONE block per call, from rayon workers
(src/vfs/mod.rs:91-97 -> block.rs:427 encode, :560 reconstruct).  Concurrent
calls on one device merge into batch launches (submit.hpp): these tests check
that every caller gets exactly its own block's bytes and its own status, for
mixed codecs, shard lengths, erasure patterns, memory kinds and device IDs,
and that merging happened (queue counters)."""
import ctypes
import threading

import numpy as np
import pytest

import shmr_amd
from shmr_amd import _native
from oracle import c_oracle

pytestmark = pytest.mark.gpu

GUARD = 0x5A


def _parity(k, p, data):
    """data [k][S] -> parity [p][S] (oracle)."""
    S = data.shape[1]
    par = np.zeros((1, p, S), np.uint8)
    c_oracle.encode_batch(k, p, np.ascontiguousarray(data[None]), par, 1, S, 1)
    return par[0]


def _rebuilt(k, p, full, present, data_only):
    """The oracle's reconstruct of a codeword-or-not block (absent rows ignored)."""
    S = full.shape[1]
    shards = [full[i].copy() if present[i] else None for i in range(k + p)]
    out = c_oracle.reconstruct(k, p, shards, S, data_only)
    return np.stack(out)


class Arena:
    """One guarded device allocation; blocks get shard views at `slot` pitch."""

    def __init__(self, gpu, nbytes):
        import torch
        self.t = torch.full((nbytes,), GUARD, dtype=torch.uint8, device=gpu)
        self.used = []

    def view(self, off, n):
        self.used.append((off, n))
        return self.t[off:off + n]

    def guards_intact(self):
        import torch
        mask = torch.ones(self.t.numel(), dtype=torch.bool, device=self.t.device)
        for off, n in self.used:
            mask[off:off + n] = False
        return bool((self.t[mask] == GUARD).all())


def _random_pattern(rng, k, p):
    t = k + p
    pr = np.ones(t, np.uint8)
    lost = rng.choice(t, size=int(rng.integers(1, p + 1)), replace=False)
    pr[lost] = 0
    return pr


@pytest.mark.parametrize("k,p,S", [(8, 3, 512 * 1024), (10, 4, 1677722), (4, 2, 4096 * 3 + 100), (1, 1, 17),
                                   (5, 5, 65536)])
def test_encode_dev_one_block(gpu, k, p, S):
    import torch
    rng = np.random.default_rng(k * 100 + p)
    t = k + p
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    shards = [torch.from_numpy(data[i]).to(gpu) for i in range(k)] + \
             [torch.full((S,), 0xEE, dtype=torch.uint8, device=gpu) for _ in range(p)]
    torch.cuda.synchronize()
    q0 = shmr_amd.queue_stats(0)
    shmr_amd.ReedSolomon(k, p).encode_dev(shards)
    q1 = shmr_amd.queue_stats(0)
    assert q1["requests"] == q0["requests"] + 1 and q1["batches"] >= q0["batches"] + 1
    want = _parity(k, p, data)
    for r in range(p):
        assert np.array_equal(shards[k + r].cpu().numpy(), want[r]), r
    assert t == len(shards)


@pytest.mark.parametrize("data_only", [False, True])
def test_reconstruct_dev_patterns(gpu, data_only):
    """Every 1- and 2-erasure pattern of RS(6,3) at an odd length, one block
    per call, rebuilt into buffers of their own (the crate's fresh Vec per
    None): the oracle's bytes, nothing else written (guards)."""
    import itertools
    import torch
    k, p, S = 6, 3, 40000 + 3
    t = k + p
    rng = np.random.default_rng(7)
    rs = shmr_amd.ReedSolomon(k, p)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    full = np.concatenate([data, _parity(k, p, data)])
    pats = [c for n in (1, 2) for c in itertools.combinations(range(t), n)]
    arena = Arena(gpu, len(pats) * t * (S + 64) + 256)
    jobs = []
    for q, lost in enumerate(pats):
        pr = np.ones(t, np.uint8)
        pr[list(lost)] = 0
        row = []
        for i in range(t):
            v = arena.view((q * t + i) * (S + 64) + 32 + (i % 3), S)
            if pr[i]:
                v.copy_(torch.from_numpy(full[i]).to(gpu))
            row.append(None if (not pr[i] and data_only and i >= k) else v)
        jobs.append((pr, row))
    torch.cuda.synchronize()
    for pr, row in jobs:
        rs.reconstruct_dev(row, pr, data_only=data_only)
    for pr, row in jobs:
        for i in range(t):
            if row[i] is None:
                continue
            assert np.array_equal(row[i].cpu().numpy(), full[i]), (pr, i)
    assert arena.guards_intact()


def test_concurrent_callers_merge_bit_exact(gpu):
    """16 threads, each a stream of per-block calls (encode and reconstruct,
    RS(8,3) / RS(10,4) / RS(4,2), two lengths, random erasure patterns, one
    op in four started and waited later) on blocks of their own in one
    arena: every block equals the oracle's, guards intact, and the queue
    merged calls (fewer launches than requests, a batch of several)."""
    import torch
    T, OPS = 16, 24
    codecs = [(8, 3, 65536), (10, 4, 12345 * 4), (4, 2, 4096 * 5 + 8), (8, 3, 4096)]
    slot = max(S for _, _, S in codecs) + 4096
    tmax = max(k + p for k, p, _ in codecs)
    arena = Arena(gpu, T * OPS * tmax * slot + 4096)
    rng = np.random.default_rng(11)
    plans = []   # per thread: list of (kind, k, p, S, views, present, want)
    for th in range(T):
        ops = []
        for o in range(OPS):
            k, p, S = codecs[int(rng.integers(0, len(codecs)))]
            t = k + p
            base = ((th * OPS + o) * tmax) * slot
            views = [arena.view(base + i * slot, S) for i in range(t)]
            data = rng.integers(0, 256, (k, S), dtype=np.uint8)
            full = np.concatenate([data, _parity(k, p, data)])
            if rng.integers(0, 2):
                for i in range(k):
                    views[i].copy_(torch.from_numpy(full[i]).to(gpu))
                ops.append(("enc", k, p, S, views, None, full, bool(rng.integers(0, 4) == 0)))
            else:
                pr = _random_pattern(rng, k, p)
                for i in range(t):
                    if pr[i]:
                        views[i].copy_(torch.from_numpy(full[i]).to(gpu))
                ops.append(("rec", k, p, S, views, pr, full, bool(rng.integers(0, 4) == 0)))
        plans.append(ops)
    torch.cuda.synchronize()
    codec_objs = {(k, p): shmr_amd.ReedSolomon(k, p) for k, p, _ in codecs}
    errors = []
    barrier = threading.Barrier(T)

    def worker(ops):
        try:
            barrier.wait()
            pending = []
            for kind, k, p, S, views, pr, _, started in ops:
                rs = codec_objs[(k, p)]
                if kind == "enc":
                    op = rs.encode_dev(views, start=started)
                else:
                    op = rs.reconstruct_dev(views, pr, start=started)
                if op is not None:
                    pending.append(op)
            for op in pending:
                op.wait()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    q0 = shmr_amd.queue_stats(0)
    # Python threads submit slower than the GPU codes a block, so the queue
    # would launch almost every call at once; a 3 ms window (knob coalesce_us:
    # an idle queue's launch waits for company) makes the merging certain
    shmr_amd.set_tuning(coalesce_us=3000)
    try:
        ths = [threading.Thread(target=worker, args=(plans[i],)) for i in range(T)]
        for x in ths:
            x.start()
        for x in ths:
            x.join()
    finally:
        shmr_amd.set_tuning(coalesce_us=-2)
    assert not errors, errors[:3]
    q1 = shmr_amd.queue_stats(0)
    nreq = q1["requests"] - q0["requests"]
    assert nreq == T * OPS
    assert q1["batches"] - q0["batches"] < nreq, "no call was merged"
    assert q1["max_batch"] > 1
    for ops in plans:
        for kind, k, p, S, views, pr, full, _ in ops:
            t = k + p
            for i in range(t):
                assert np.array_equal(views[i].cpu().numpy(), full[i]), (kind, k, p, S, i)
    assert arena.guards_intact()


def test_started_calls_batch_and_wait_out_of_order(gpu):
    """64 started encodes of blocks in the slots of one slab (a lattice: the
    launches run the strided kernels) and 64 started 1-erasure rebuilds,
    waited in random order: exact."""
    import torch
    k, p, S, B = 8, 3, 65536, 64
    t = k + p
    slab = shmr_amd.ShardSlab(B, t, S)
    rs = shmr_amd.ReedSolomon(k, p)
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    view = slab.tensor()
    view[:, :k, :S] = torch.from_numpy(data).to(gpu)
    torch.cuda.synchronize()
    q0 = shmr_amd.queue_stats(0)
    g0 = shmr_amd.device_stats(0)["ptr_table_grids"]
    order = rng.permutation(B)
    ops = [rs.encode_dev([slab.shard(int(b), i) for i in range(t)], start=True) for b in order]
    for j in rng.permutation(B):
        ops[int(j)].wait()
    q1 = shmr_amd.queue_stats(0)
    # (one Python thread submits slower than the GPU codes a block: whether
    # calls merge here depends on timing -- merging is asserted with threads
    # above and measured by tools/perblock_dev.cpp)
    assert q1["requests"] - q0["requests"] == B and 0 < q1["batches"] - q0["batches"] <= B
    assert shmr_amd.device_stats(0)["ptr_table_grids"] > g0
    want = np.stack([_parity(k, p, data[b]) for b in range(B)])
    got = view[:, :, :S].cpu().numpy()
    assert np.array_equal(got[:, k:], want)
    # rebuild one lost shard per block in place (shard b mod t), started
    lost = [int(b) % t for b in range(B)]
    for b in range(B):
        view[b, lost[b], :S] = 0xEE
    torch.cuda.synchronize()
    ops = []
    for b in order:
        pr = np.ones(t, np.uint8)
        pr[lost[int(b)]] = 0
        ops.append(rs.reconstruct_dev([slab.shard(int(b), i) for i in range(t)], pr, start=True))
    for j in rng.permutation(B):
        ops[int(j)].wait()
    assert np.array_equal(view[:, :, :S].cpu().numpy(), got)


@pytest.mark.parametrize("lead_us", [0, 1000000])
def test_early_launch_knob(gpu, lead_us):
    """coalesce_lead_us: 0 launches held-back calls only when the running batch
    completes (no early launches counted); a lead longer than any batch makes
    the watcher launch every call that arrives while one batch runs at once,
    behind it on the stream.  Both exact (8 threads of started encodes of 16
    MiB shards, waited in random order)."""
    import torch
    k, p, S, T, per = 4, 2, 1 << 24, 8, 3
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    slab = shmr_amd.ShardSlab(T * per, t, S)
    rng = np.random.default_rng(lead_us % 97)
    data = rng.integers(0, 256, (T * per, k, 4096), dtype=np.uint8)
    view = slab.tensor()
    view[:, :k, :S] = torch.from_numpy(data).to(gpu).repeat(1, 1, S // 4096)
    view[:, k:, :S] = 0xEE
    torch.cuda.synchronize()
    errors = []
    barrier = threading.Barrier(T)

    def worker(th):
        try:
            barrier.wait()
            ops = [rs.encode_dev([slab.shard(th * per + j, i) for i in range(t)], start=True) for j in range(per)]
            for j in np.random.default_rng(th).permutation(per):
                ops[int(j)].wait()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    shmr_amd.set_tuning(coalesce_lead_us=lead_us)
    try:
        assert shmr_amd.get_tuning("coalesce_lead_us") == lead_us
        q0 = shmr_amd.queue_stats(0)
        ths = [threading.Thread(target=worker, args=(i,)) for i in range(T)]
        for x in ths:
            x.start()
        for x in ths:
            x.join()
        q1 = shmr_amd.queue_stats(0)
    finally:
        shmr_amd.set_tuning(coalesce_lead_us=-2)
    assert shmr_amd.get_tuning("coalesce_lead_us") == 30
    assert not errors, errors[:3]
    assert q1["requests"] - q0["requests"] == T * per
    if lead_us == 0:
        assert q1["early"] == q0["early"]
    got = view[:, k:, :4096].cpu().numpy()
    for b in range(T * per):
        assert np.array_equal(got[b], _parity(k, p, data[b])), b
    # every column of a shard repeats the same 4 KiB: the whole parity row too
    assert bool((view[:, k:, :S].reshape(T * per, p, S // 4096, 4096) == view[:, k:, None, :4096]).all())


def test_validation_in_crate_order(gpu):
    import torch
    k, p, S = 4, 2, 4096
    rs = shmr_amd.ReedSolomon(k, p)
    sh = [torch.zeros(S, dtype=torch.uint8, device=gpu) for _ in range(k + p)]
    q0 = shmr_amd.queue_stats(0)
    for bad, code in ((sh[:5], -1), (sh + sh[:1], -2)):
        with pytest.raises(shmr_amd.Error) as e:
            rs.encode_dev(bad)
        assert e.value.code == code
    with pytest.raises(shmr_amd.Error) as e:          # unequal lengths
        rs.encode_dev(sh[:5] + [torch.zeros(S + 1, dtype=torch.uint8, device=gpu)])
    assert e.value.code == -9
    with pytest.raises(shmr_amd.Error) as e:          # empty shard
        rs.encode_dev([(sh[0].data_ptr(), 0)] + sh[1:])
    assert e.value.code == -11
    with pytest.raises(shmr_amd.Error) as e:          # NULL shard (a length of S: the size checks pass)
        rs.encode_dev([(0, S)] + sh[1:])
    assert e.value.code == -100
    with pytest.raises(shmr_amd.Error) as e:          # device ID out of range
        rs.encode_dev(sh, device=shmr_amd.device_count() + 5)
    assert e.value.code == -100
    pr = np.array([1, 0, 0, 0, 1, 1], np.uint8)       # 3 present < 4
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct_dev(sh, pr)
    assert e.value.code == -10
    rs.reconstruct_dev(sh, np.ones(k + p, np.uint8))  # all present: Ok, nothing queued
    assert shmr_amd.queue_stats(0)["requests"] == q0["requests"]


def test_mapped_host_calls_coalesced(gpu):
    """The drop-in shmr_ec_encode / shmr_ec_reconstruct on mapped Block-Cache
    buffers (shmr_ec_host_alloc) from 8 threads go through the queue under knob
    "coalesce" = 1 (default 0: measured no faster, tools/perblock_host.cpp):
    the oracle's bytes, counted zero-copy; with the knob off the same calls
    take one zero-copy launch each and give the same bytes."""
    k, p, S, B = 8, 3, 131072, 32
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    rng = np.random.default_rng(21)
    data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    want = np.stack([_parity(k, p, data[b]) for b in range(B)])
    for knob in (1, 0):
        shmr_amd.set_tuning(coalesce=knob)
        try:
            buf = shmr_amd.PinnedBuffer(B * t * S)
            arr = buf.array.reshape(B, t, S)
            arr[:, :k] = data
            arr[:, k:] = 0xEE
            q0 = shmr_amd.queue_stats(0)
            z0, _ = shmr_amd.path_stats()
            errors = []

            def worker(th):
                try:
                    for b in range(th, B, 8):
                        rs.encode([arr[b, i] for i in range(t)])
                        pr = np.ones(t, np.uint8)
                        pr[b % t] = 0
                        shards = [arr[b, i] if pr[i] else None for i in range(t)]
                        rs.reconstruct(shards)
                        assert np.array_equal(shards[b % t], arr[b, b % t])
                except Exception as e:  # noqa: BLE001
                    errors.append(e)
            ths = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
            for x in ths:
                x.start()
            for x in ths:
                x.join()
            assert not errors, errors[:3]
            assert np.array_equal(arr[:, k:], want)
            q1 = shmr_amd.queue_stats(0)
            z1, _ = shmr_amd.path_stats()
            assert z1 - z0 == B   # the encodes (the reconstructs' fresh buffers are pageable: staged)
            assert (q1["requests"] - q0["requests"] == B) == bool(knob)
            del arr
            buf = None
        finally:
            shmr_amd.set_tuning(coalesce=-2)


def test_mapped_rebuild_in_place_coalesced(gpu):
    """Reconstructs whose absent shards are mapped too (the Block Cache slot
    itself): every shard zero-copy, merged through the queue, exact."""
    k, p, S, B = 10, 4, 65536 + 48, 24
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    rng = np.random.default_rng(22)
    data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    full = np.stack([np.concatenate([data[b], _parity(k, p, data[b])]) for b in range(B)])
    buf = shmr_amd.PinnedBuffer(B * t * S)
    arr = buf.array.reshape(B, t, S)
    arr[:] = full
    pats = [_random_pattern(rng, k, p) for _ in range(B)]
    for b in range(B):
        arr[b, pats[b] == 0] = 0xEE
    L = rs._L
    q0 = shmr_amd.queue_stats(0)
    shmr_amd.set_tuning(coalesce=1)

    def worker(th):
        for b in range(th, B, 6):
            ptrs = (ctypes.POINTER(ctypes.c_uint8) * t)(*[arr[b, i].ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
                                                         for i in range(t)])
            lens = (ctypes.c_size_t * t)(*[S if pats[b][i] else 0 for i in range(t)])
            pr = pats[b].copy()
            assert L.shmr_ec_reconstruct(rs._h, ptrs, lens, pr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), t,
                                         0) == 0
    try:
        ths = [threading.Thread(target=worker, args=(i,)) for i in range(6)]
        for x in ths:
            x.start()
        for x in ths:
            x.join()
    finally:
        shmr_amd.set_tuning(coalesce=-2)
    assert np.array_equal(arr, full)
    assert shmr_amd.queue_stats(0)["requests"] - q0["requests"] == B


def test_alias_devices_have_queues_of_their_own(gpu):
    """Tools build, alias device IDs on the one GPU: concurrent per-block
    calls spread over four IDs are merged per ID (each ID's queue counts its
    own requests) and every block is exact."""
    import torch
    with _native.tools():
        n = shmr_amd.device_count()
        shmr_amd.set_tuning(alias_devices=7)
        try:
            # (IDs past n + 3: test_gpu_capture needs alias ID n untouched)
            ids = [0, n + 4, n + 5, n + 6]
            k, p, S, per = 8, 3, 32768, 12
            t = k + p
            rs = shmr_amd.ReedSolomon(k, p)
            arena = Arena(gpu, len(ids) * per * t * (S + 4096) + 4096)
            rng = np.random.default_rng(3)
            jobs = {d: [] for d in ids}
            for j, d in enumerate(ids):
                for b in range(per):
                    base = ((j * per) + b) * t * (S + 4096)
                    views = [arena.view(base + i * (S + 4096), S) for i in range(t)]
                    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
                    for i in range(k):
                        views[i].copy_(torch.from_numpy(data[i]).to(gpu))
                    jobs[d].append((views, _parity(k, p, data)))
            torch.cuda.synchronize()
            before = {d: shmr_amd.queue_stats(d)["requests"] for d in ids}

            def worker(d):
                ops = [rs.encode_dev(v, device=d, start=True) for v, _ in jobs[d]]
                for op in ops:
                    op.wait()
            ths = [threading.Thread(target=worker, args=(d,)) for d in ids]
            for x in ths:
                x.start()
            for x in ths:
                x.join()
            for d in ids:
                assert shmr_amd.queue_stats(d)["requests"] - before[d] == per
                for views, want in jobs[d]:
                    for r in range(p):
                        assert np.array_equal(views[k + r].cpu().numpy(), want[r])
            assert arena.guards_intact()
        finally:
            shmr_amd.set_tuning(alias_devices=0)
