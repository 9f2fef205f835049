"""Stream-ordered device entry points: after the device's one-time init, the
device-resident calls make no blocking HIP call, so they can be captured into
a HIP graph (torch.cuda.graph) -- including a reconstruct with an erasure
pattern the device has never seen (its plan upload becomes a graph node that
re-copies the same bytes from a permanent pinned slot on every replay).

Reference shape: the daemon's concurrent per-block callers
(src/vfs/mod.rs:93-96) issue encodes / reconstructs while other work is in
flight; none of them may stall the host behind queued kernels.
"""
import numpy as np
import pytest

import shmr_amd
from shmr_amd import _native
from oracle import c_oracle

pytestmark = pytest.mark.gpu

POISON = 0xEE


def _blocking(dev=0):
    return shmr_amd.device_stats(dev)["blocking_calls"]


def _oracle_parity(k, p, data):
    B, _, S = data.shape
    par = np.zeros((B, p, S), np.uint8)
    c_oracle.encode_batch(k, p, np.ascontiguousarray(data), par, B, S, 8)
    return par


def test_graph_capture_encode_and_unseen_patterns(gpu):
    import torch
    # a codec no other test uses: its encode plan and every erasure pattern
    # below are first uploaded inside the capture
    k, p = 9, 5
    t = k + p
    S = 8192 * 3 + 2458                    # full 8 KiB tiles + a partial one (fused tails)
    pitch = (S + 4095) // 4096 * 4096
    B = 12
    rs = shmr_amd.ReedSolomon(k, p)
    shmr_amd.device_init(0)
    base = _blocking()

    g = torch.Generator(device=gpu).manual_seed(9)
    data = torch.randint(0, 256, (B, k, pitch), dtype=torch.uint8, device=gpu, generator=g)
    parity = torch.zeros((B, p, pitch), dtype=torch.uint8, device=gpu)
    # codewords for the rebuilds (computed on the CPU oracle)
    rng = np.random.default_rng(5)
    host = np.zeros((B, t, pitch), np.uint8)
    host[:, :k, :S] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    host[:, k:, :S] = _oracle_parity(k, p, host[:, :k, :S])
    present = np.ones((B, t), np.uint8)
    for b in range(B):                     # 12 blocks, 4 patterns (segment launch)
        present[b, [[0, 13], [2, 7, 12], [4], [1, 3, 8, 10]][b % 4]] = 0
    many = 40                              # > 32 runs of one row count: the table launch
    hmany = np.zeros((many, t, pitch), np.uint8)
    hmany[:, :k, :S] = rng.integers(0, 256, (many, k, S), dtype=np.uint8)
    hmany[:, k:, :S] = _oracle_parity(k, p, hmany[:, :k, :S])
    pmany = np.ones((many, t), np.uint8)
    for b in range(many):
        pmany[b, rng.choice(t, size=2, replace=False)] = 0
    shards = torch.from_numpy(host).to(gpu)
    shards_many = torch.from_numpy(hmany).to(gpu)
    out = torch.zeros((B, 4, pitch), dtype=torch.uint8, device=gpu)
    poison = torch.from_numpy(present == 0).to(gpu)
    poison_many = torch.from_numpy(pmany == 0).to(gpu)
    torch.cuda.synchronize()

    graph = torch.cuda.CUDAGraph()
    stream = torch.cuda.Stream()
    with torch.cuda.graph(graph, stream=stream):
        rs.encode_batch_dev(data, parity, shard_len=S)
        rs.reconstruct_batch_dev(shards, present, shard_len=S)
        rs.reconstruct_batch_dev_out(shards, present, out, shard_len=S)
        rs.reconstruct_batch_dev(shards_many, pmany, shard_len=S)
    assert _blocking() == base, "a blocking HIP call inside the capture"

    for rep in range(2):
        data.copy_(torch.randint(0, 256, (B, k, pitch), dtype=torch.uint8, device=gpu, generator=g))
        parity.fill_(0)
        shards[poison] = POISON
        shards_many[poison_many] = POISON
        out.fill_(0)
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        hd = data.cpu().numpy()
        want = _oracle_parity(k, p, hd[:, :, :S])
        assert np.array_equal(parity.cpu().numpy()[:, :, :S], want), rep
        # the in-place rebuild ran first, so the compact rebuild read a full
        # codeword: both equal the original shards
        assert np.array_equal(shards.cpu().numpy()[:, :, :S], host[:, :, :S]), rep
        assert np.array_equal(shards_many.cpu().numpy()[:, :, :S], hmany[:, :, :S]), rep
        got = out.cpu().numpy()
        for b in range(B):
            for j, i in enumerate(np.flatnonzero(present[b] == 0)):
                assert np.array_equal(got[b, j, :S], host[b, i, :S]), (rep, b, i)
    # eager calls after the capture (the captured-only plan uploads are redone
    # on the caller's stream) stay exact and non-blocking
    shards[poison] = POISON
    rs.reconstruct_batch_dev(shards, present, shard_len=S)
    torch.cuda.synchronize()
    assert np.array_equal(shards.cpu().numpy()[:, :, :S], host[:, :, :S])
    assert _blocking() == base


def test_unseen_pattern_on_second_stream_waits_for_upload(gpu):
    """A plan uploaded on stream A and used at once on stream B: B waits for the
    upload on the device (an event), the host never blocks."""
    import torch
    k, p, S, B = 7, 6, 65536, 8
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    shmr_amd.device_init(0)
    rng = np.random.default_rng(13)
    host = np.zeros((B, t, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    host[:, k:] = _oracle_parity(k, p, host[:, :k])
    present = np.ones((B, t), np.uint8)
    present[:, [1, 9]] = 0
    a_shards = torch.from_numpy(host).to(gpu)
    b_shards = torch.from_numpy(host).to(gpu)
    mask = torch.from_numpy(present == 0).to(gpu)
    a_shards[mask] = POISON
    b_shards[mask] = POISON
    torch.cuda.synchronize()
    base = _blocking()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(sa):
        torch.cuda._sleep(20_000_000)          # keep stream A busy: its upload lands late
        rs.reconstruct_batch_dev(a_shards, present, shard_len=S)
    with torch.cuda.stream(sb):
        rs.reconstruct_batch_dev(b_shards, present, shard_len=S)
    torch.cuda.synchronize()
    assert _blocking() == base
    assert np.array_equal(a_shards.cpu().numpy(), host)
    assert np.array_equal(b_shards.cpu().numpy(), host)


def test_init_refused_inside_capture(gpu):
    """A device whose state does not exist yet cannot be initialised inside a
    capture (it allocates and synchronises): InvalidArgument, nothing enqueued,
    and the capture stays usable.  Tools build: alias device ID 1 of GPU 0."""
    import torch
    with _native.tools():
        shmr_amd.set_tuning(alias_devices=1)
        try:
            rs = shmr_amd.ReedSolomon(4, 2)
            S = 4096 * 4
            data = torch.randint(0, 256, (2, 4, S), dtype=torch.uint8, device=gpu)
            parity = torch.zeros((2, 2, S), dtype=torch.uint8, device=gpu)
            shmr_amd.device_init(0)
            assert shmr_amd.device_stats(1)["blocking_calls"] == 0
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=torch.cuda.Stream()):
                with pytest.raises(shmr_amd.Error) as e:
                    rs.encode_batch_dev(data, parity, device=1)
                rs.encode_batch_dev(data, parity, device=0)
            assert e.value.name == "InvalidArgument"
            assert shmr_amd.device_stats(1)["blocking_calls"] == 0
            graph.replay()
            torch.cuda.synchronize()
            want = _oracle_parity(4, 2, data.cpu().numpy())
            assert np.array_equal(parity.cpu().numpy(), want)
        finally:
            shmr_amd.set_tuning(alias_devices=0)


def _ptr_table(base, B, t, S):
    """ctypes table of B x t device pointers into one buffer (shard i of block
    b at base + (b * t + i) * S)."""
    import ctypes
    from shmr_amd.reed_solomon import _u8p
    addrs = (np.uint64(base) + np.arange(B * t, dtype=np.uint64) * np.uint64(S)).astype(np.uint64)
    return addrs, addrs.ctypes.data_as(ctypes.POINTER(_u8p))


def _wait_released(dev, want, timeout=10.0):
    import time
    t0 = time.time()
    while shmr_amd.device_stats(dev)["capture_released"] < want and time.time() - t0 < timeout:
        time.sleep(0.01)
    return shmr_amd.device_stats(dev)["capture_released"]


def test_capture_reserve_reused_across_graphs_and_large_capture(gpu, table_kernels):
    """Captured calls take their tables from the capture reserve and give them
    back when the graph is destroyed: 120 capture / replay / destroy cycles of a
    48 KiB pointer table run in the 4 MiB reserve (without the release they
    would exhaust it after ~85).  A capture larger than the reserve fails with
    OUT_OF_MEMORY and nothing enqueued; after shmr_ec_capture_reserve it
    succeeds and replays bit-exact."""
    import ctypes
    import gc
    import torch
    shmr_amd.device_init(0)
    stream = torch.cuda.Stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    # repeated captures (RS(4,2), 1000 blocks of 256-byte shards)
    k, p, S, B = 4, 2, 256, 1000
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    buf = torch.randint(0, 256, (B * t * S,), dtype=torch.uint8, device=gpu)
    addrs, tab = _ptr_table(buf.data_ptr(), B, t, S)
    # two live graphs (torch destroys the captured hipGraph_t right after instantiating it, so the
    # executable graph alone must keep its table): each replays its own table, not the other's
    buf2 = torch.randint(0, 256, (B * t * S,), dtype=torch.uint8, device=gpu)
    _, tab2 = _ptr_table(buf2.data_ptr(), B, t, S)
    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(ga, stream=stream):
        assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, sp) == 0
    with torch.cuda.graph(gb, stream=stream):
        assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab2, B, S, 0, sp) == 0
    for g, mine, other in ((ga, buf, buf2), (gb, buf2, buf)):
        mine.view(B, t, S)[:, k:] = 0
        other.view(B, t, S)[:, k:] = 0
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        h = mine.view(B, t, S).cpu().numpy()
        assert np.array_equal(h[:, k:], _oracle_parity(k, p, h[:, :k]))
        assert not other.view(B, t, S)[:, k:].any().item(), "a graph ran another graph's table"
    del ga, gb
    gc.collect()
    torch.cuda.synchronize()
    st0 = shmr_amd.device_stats(0)
    for cycle in range(120):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            rc = rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, sp)
        assert rc == 0, (cycle, shmr_amd.Error(rc).name)
        if cycle % 40 == 0:
            buf.view(B, t, S)[:, k:] = 0
            g.replay()
            torch.cuda.synchronize()
            h = buf.view(B, t, S).cpu().numpy()
            assert np.array_equal(h[:, k:], _oracle_parity(k, p, h[:, :k])), cycle
        del g
        gc.collect()
        torch.cuda.synchronize()
    st1 = shmr_amd.device_stats(0)
    assert st1["capture_tables"] - st0["capture_tables"] == 120
    assert _wait_released(0, st0["capture_released"] + 110) >= st0["capture_released"] + 110
    # a capture larger than the reserve: RS(10,4), 40,000 blocks = 4.48 MB of pointers
    k, p, S, B = 10, 4, 256, 40000
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    big = torch.randint(0, 256, (B * t * S,), dtype=torch.uint8, device=gpu)
    addrs, tab = _ptr_table(big.data_ptr(), B, t, S)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        rc = rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, sp)
    assert shmr_amd.Error(rc).name == "OutOfMemory"
    del g
    shmr_amd.capture_reserve(B * t * 8, 0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        rc = rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, sp)
    assert rc == 0, shmr_amd.Error(rc).name
    big.view(B, t, S)[:, k:] = 0
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    h = big.view(B, t, S).cpu().numpy()
    assert np.array_equal(h[:, k:], _oracle_parity(k, p, h[:, :k]))
    del g
    gc.collect()


def test_capture_block_not_reused_while_a_replay_is_queued(gpu, table_kernels):
    """A captured call's table block goes back to the capture reserve when its
    graph is destroyed.  Destroying the graph (and its executable) while a
    replay is still queued -- behind a long kernel on the replay's stream --
    must not let a new capture take that block: the new capture writes its own
    table into it at once, and the queued replay's H2D node and kernel would
    then read the other call's shard pointers.  The first replay
    must hit only its own buffers."""
    import ctypes
    import gc
    import torch
    shmr_amd.device_init(0)
    k, p, S, B = 4, 2, 4096 * 4, 64
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    buf1 = torch.randint(0, 256, (B * t * S,), dtype=torch.uint8, device=gpu)
    buf2 = torch.randint(0, 256, (B * t * S,), dtype=torch.uint8, device=gpu)
    _, tab1 = _ptr_table(buf1.data_ptr(), B, t, S)
    _, tab2 = _ptr_table(buf2.data_ptr(), B, t, S)
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, stream=s1):
        assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab1, B, S, 0, ctypes.c_void_p(s1.cuda_stream)) == 0
    buf1.view(B, t, S)[:, k:] = 0
    buf2.view(B, t, S)[:, k:] = 0
    torch.cuda.synchronize()
    st0 = shmr_amd.device_stats(0)
    done1 = torch.cuda.Event()
    with torch.cuda.stream(s1):
        torch.cuda._sleep(400_000_000)       # ~0.2 s: the replay below waits behind it
        g1.replay()
        done1.record(s1)
    import time
    t0 = time.perf_counter()
    del g1
    gc.collect()
    destroy_s = time.perf_counter() - t0
    replay_done_at_release = done1.query()
    released = shmr_amd.device_stats(0)["capture_released"] - st0["capture_released"]
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=s2):
        assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab2, B, S, 0, ctypes.c_void_p(s2.cuda_stream)) == 0
    g2.replay()                              # on s2, while g1's replay may still wait on s1
    torch.cuda.synchronize()
    print(f"graph destroy took {destroy_s * 1e3:.1f} ms; blocks released by then: {released}; "
          f"queued replay already done then: {replay_done_at_release}")
    h1 = buf1.view(B, t, S).cpu().numpy()
    h2 = buf2.view(B, t, S).cpu().numpy()
    assert np.array_equal(h2[:, k:], _oracle_parity(k, p, h2[:, :k])), "the new capture's replay"
    assert np.array_equal(h1[:, k:], _oracle_parity(k, p, h1[:, :k])), "the queued replay lost its own table"
    del g2
    gc.collect()


@pytest.mark.parametrize("mode", ["global", "thread_local"])
def test_library_allocations_while_another_thread_captures(gpu, mode):
    """One thread holds a graph capture open while another makes calls that
    allocate (device / mapped buffers, host registration, a fresh codec's
    pageable per-block and batch calls that grow the staging buffers).  Under
    the default capture mode HIP refuses such calls while any thread captures
    and invalidates that capture; the library makes its own allocations under
    the relaxed mode, so both sides succeed: every call exact, the capture
    replays bit-exact (soak finding: tools/soak.py, profiles/r04/s6)."""
    import threading
    import torch
    shmr_amd.device_init(0)
    k, p, S, B = 8, 3, 65536, 4
    rs = shmr_amd.ReedSolomon(k, p)
    data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=gpu)
    parity = torch.zeros((B, p, S), dtype=torch.uint8, device=gpu)
    torch.cuda.synchronize()
    in_capture, done = threading.Event(), threading.Event()
    results = {}

    def other():
        try:
            assert in_capture.wait(60)
            dev = shmr_amd.DeviceBuffer(48 << 20)
            pin = shmr_amd.PinnedBuffer(24 << 20)
            arr = np.zeros(8 << 20, np.uint8)
            shmr_amd.host_register(arr)
            shmr_amd.host_unregister(arr)
            del dev, pin
            # a codec and sizes no other test uses: fresh staging and plans
            k2, p2, L2 = 13, 6, (3 << 20) + 4096
            rs2 = shmr_amd.ReedSolomon(k2, p2)
            rng = np.random.default_rng(31)
            blk = np.zeros((3, k2 + p2, L2), np.uint8)
            blk[:, :k2] = rng.integers(0, 256, (3, k2, L2), dtype=np.uint8)
            rs2.encode_blocks_host(blk)
            want = np.zeros((3, p2, L2), np.uint8)
            c_oracle.encode_batch(k2, p2, np.ascontiguousarray(blk[:, :k2]), want, 3, L2, 8)
            results["batch"] = np.array_equal(blk[:, k2:], want)
            shards = [np.ascontiguousarray(blk[0, i]) for i in range(k2 + p2)]
            for i in range(k2, k2 + p2):
                shards[i][:] = 0
            rs2.encode(shards)
            results["block"] = all(np.array_equal(shards[k2 + r], want[0, r]) for r in range(p2))
        except BaseException as e:   # reported by the capturing thread
            results["error"] = repr(e)
        finally:
            done.set()

    th = threading.Thread(target=other)
    th.start()
    graph = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(graph, stream=torch.cuda.Stream(), capture_error_mode=mode):
            rs.encode_batch_dev(data, parity)
            in_capture.set()
            assert done.wait(120), "the other thread did not finish"
    finally:
        in_capture.set()
        th.join(120)
    assert "error" not in results, results
    assert results == {"batch": True, "block": True}, results
    graph.replay()
    torch.cuda.synchronize()
    assert np.array_equal(parity.cpu().numpy(), _oracle_parity(k, p, data.cpu().numpy()))


def test_events_recorded_before_a_capture_on_that_stream(gpu, table_kernels):
    """The library's readiness events (a plan upload, an upload-ring slot, a
    pointer-table cache entry) recorded by eager calls on stream S stay usable
    by other threads after S begins a graph capture: every query or wait goes
    to a mirror recorded on the device's private stream, never to the event on
    S -- HIP fails a query of an event whose stream is capturing
    (hipErrorCapturedEvent) and invalidates the capture (soak finding,
    profiles/r04/s8)."""
    import ctypes
    import threading
    import torch
    from shmr_amd.reed_solomon import _ptr, _u8p
    shmr_amd.device_init(0)
    k, p, S, B = 11, 5, 4096, 40          # a codec no other test uses: fresh plans
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    L = rs._L
    rng = np.random.default_rng(77)
    host = np.zeros((B, t, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    host[:, k:] = _oracle_parity(k, p, host[:, :k])
    present = np.ones((B, t), np.uint8)
    for b in range(B):                     # 40 runs of 2-row rebuilds: the upload-ring table launch
        present[b, [[0, 1], [2, 3]][b % 2]] = 0
    s_cap, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    # every buffer exists before the capture: the other thread makes no torch call
    cw0, cw2 = torch.from_numpy(host).to(gpu), torch.from_numpy(host).to(gpu)
    data = torch.from_numpy(np.ascontiguousarray(host[:, :k])).to(gpu)
    par0, par_cap, par_other = (torch.zeros((B, p, S), dtype=torch.uint8, device=gpu) for _ in range(3))
    pbuf = torch.zeros((9, t, S), dtype=torch.uint8, device=gpu)
    pbuf[:, :k] = torch.from_numpy(host[:9, :k]).to(gpu)
    tabs = [np.array([pbuf[j, i].data_ptr() for i in range(t)], dtype=np.uint64) for j in range(9)]
    torch.cuda.synchronize()
    # eager calls on s_cap: plan uploads, a ring slot and 8 table-cache entries recorded there
    with torch.cuda.stream(s_cap):
        rs.encode_batch_dev(data, par0)
        rs.reconstruct_batch_dev(cw0, present)
        for j in range(8):
            assert L.shmr_ec_encode_ptrs_dev(rs._h, tabs[j].ctypes.data_as(ctypes.POINTER(_u8p)), 1, S, 0,
                                             ctypes.c_void_p(s_cap.cuda_stream)) == 0
    in_capture, done = threading.Event(), threading.Event()
    rcs = []

    def other():                            # C-ABI calls only, on s2, while s_cap captures
        try:
            assert in_capture.wait(60)
            sp = ctypes.c_void_p(s2.cuda_stream)
            rcs.append(L.shmr_ec_encode_batch_dev(rs._h, ctypes.c_void_p(data.data_ptr()), S, k * S,
                                                  ctypes.c_void_p(par_other.data_ptr()), S, p * S, B, S, 0, sp))
            for _ in range(33):             # around the 32-slot ring: reuses the slot s_cap armed
                rcs.append(L.shmr_ec_reconstruct_batch_dev(rs._h, ctypes.c_void_p(cw2.data_ptr()), S, t * S,
                                                           _ptr(present), B, S, 0, 0, sp))
            # a ninth table: the cache's victim search looks at the 8 entries s_cap filled
            rcs.append(L.shmr_ec_encode_ptrs_dev(rs._h, tabs[8].ctypes.data_as(ctypes.POINTER(_u8p)), 1, S, 0, sp))
        except BaseException as e:   # reported by the capturing thread
            rcs.append(repr(e))
        finally:
            done.set()

    th = threading.Thread(target=other)
    th.start()
    graph = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(graph, stream=s_cap):
            rs.encode_batch_dev(data, par_cap)
            in_capture.set()
            assert done.wait(120), "the other thread did not finish"
    finally:
        in_capture.set()
        th.join(120)
    assert rcs == [0] * 35, [shmr_amd.Error(r).name if isinstance(r, int) and r else r for r in rcs]
    graph.replay()
    torch.cuda.synchronize()
    want = host[:, k:]
    for name, par in (("eager", par0), ("captured", par_cap), ("other thread", par_other)):
        assert np.array_equal(par.cpu().numpy(), want), name
    assert np.array_equal(cw0.cpu().numpy(), host) and np.array_equal(cw2.cpu().numpy(), host)
    got = pbuf.cpu().numpy()
    for j in range(9):
        assert np.array_equal(got[j, k:], want[j]), j


def test_host_buffer_calls_inside_own_capture(gpu):
    """A host-buffer call (synchronous, on the library's own streams) made by
    the thread that is capturing a graph in the default global mode: it runs
    eagerly and exactly, and the capture -- which it does not touch -- stays
    valid and replays its own work."""
    import torch
    k, p, S = 6, 3, 70001
    rs = shmr_amd.ReedSolomon(k, p)
    shmr_amd.device_init(0)
    rng = np.random.default_rng(41)
    shards = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    x = torch.zeros(1024, device=gpu)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=torch.cuda.Stream()):
        x.add_(1)
        rs.encode(shards)                                  # eager, not part of the graph
        blocks = np.zeros((2, k + p, 4096), np.uint8)
        blocks[:, :k] = rng.integers(0, 256, (2, k, 4096), dtype=np.uint8)
        rs.encode_blocks_host(blocks)
    want = [np.zeros(S, np.uint8) for _ in range(p)]
    c_oracle.encode(k, p, [s.copy() for s in shards[:k]] + want)
    for r in range(p):
        assert np.array_equal(shards[k + r], want[r]), r
    par = _oracle_parity(k, p, blocks[:, :k])
    assert np.array_equal(blocks[:, k:], par)
    graph.replay()
    graph.replay()
    torch.cuda.synchronize()
    assert float(x[0].item()) == 2.0


def test_null_stream_call_while_another_thread_captures_a_blocking_stream(gpu):
    """A device call on the legacy null stream while another thread captures a
    BLOCKING stream in global mode: work on the null stream would join that
    capture, so the library refuses the call (INVALID_ARGUMENT, nothing
    enqueued) and the other capture stays valid (HIP runtime driven through
    ctypes: torch's streams are non-blocking)."""
    import ctypes
    import threading
    import torch
    H = ctypes.CDLL("libamdhip64.so.7")   # the runtime torch (and the library) already loaded
    vp = ctypes.c_void_p
    k, p, S, B = 4, 2, 8192, 2
    rs = shmr_amd.ReedSolomon(k, p)
    shmr_amd.device_init(0)
    data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=gpu)
    parity = torch.zeros((B, p, S), dtype=torch.uint8, device=gpu)
    scratch = torch.zeros(4096, dtype=torch.uint8, device=gpu)
    torch.cuda.synchronize()
    blocking = vp()
    assert H.hipStreamCreate(ctypes.byref(blocking)) == 0
    in_capture, done = threading.Event(), threading.Event()
    out = {}

    def other():
        assert in_capture.wait(60)
        out["rc"] = rs._L.shmr_ec_encode_batch_dev(rs._h, vp(data.data_ptr()), S, k * S, vp(parity.data_ptr()),
                                                  S, p * S, B, S, 0, vp(0))
        done.set()

    th = threading.Thread(target=other)
    th.start()
    assert H.hipStreamBeginCapture(blocking, ctypes.c_int(0)) == 0          # global mode
    assert H.hipMemsetAsync(vp(scratch.data_ptr()), ctypes.c_int(7), ctypes.c_size_t(4096), blocking) == 0
    in_capture.set()
    assert done.wait(60)
    th.join(60)
    g = vp()
    end = H.hipStreamEndCapture(blocking, ctypes.byref(g))
    H.hipGetLastError()
    if end == 0 and g.value:
        H.hipGraphDestroy(g)
    H.hipStreamDestroy(blocking)
    assert end == 0, f"the other thread's capture was broken ({end})"
    assert shmr_amd.Error(out["rc"]).name == "InvalidArgument", out
    torch.cuda.synchronize()
    assert not parity.any().item(), "a refused call enqueued work"


def test_entry_points_restore_the_thread_capture_mode(gpu):
    """Every entry point runs under the relaxed capture mode and gives the
    calling thread its own mode back (global, thread-local or relaxed), on
    success and on a refused call alike."""
    import ctypes
    import torch
    H = ctypes.CDLL("libamdhip64.so.7")
    k, p, S = 5, 2, 4096
    rs = shmr_amd.ReedSolomon(k, p)
    data = torch.randint(0, 256, (2, k, S), dtype=torch.uint8, device=gpu)
    parity = torch.zeros((2, p, S), dtype=torch.uint8, device=gpu)
    shards = [np.zeros(S, np.uint8) for _ in range(k + p)]

    def mode_now():
        m = ctypes.c_int(2)
        assert H.hipThreadExchangeStreamCaptureMode(ctypes.byref(m)) == 0
        back = ctypes.c_int(m.value)
        assert H.hipThreadExchangeStreamCaptureMode(ctypes.byref(back)) == 0
        return m.value

    try:
        for mode in (0, 1, 2):   # global, thread-local, relaxed
            m = ctypes.c_int(mode)
            assert H.hipThreadExchangeStreamCaptureMode(ctypes.byref(m)) == 0
            rs.encode_batch_dev(data, parity)
            rs.encode(shards)
            with pytest.raises(shmr_amd.Error):
                rs.reconstruct([None] * (k + p))          # refused: too few shards
            assert mode_now() == mode
    finally:
        m = ctypes.c_int(0)
        H.hipThreadExchangeStreamCaptureMode(ctypes.byref(m))
    torch.cuda.synchronize()
    assert np.array_equal(parity.cpu().numpy(), _oracle_parity(k, p, data.cpu().numpy()))
