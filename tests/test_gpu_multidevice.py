"""Multi-device bookkeeping of the host-buffer and device-batch entry points,
rehearsed on one GPU.

The reference fans blocks out per block (rayon, src/vfs/mod.rs:93-96); this
library spreads whole blocks round-robin over a device list (block b ->
devices[b % ndev]) and keeps every per-device object -- plan images, upload
rings, staging streams -- per device ID.  One MI355X cannot show N distinct
GPUs, so the tools build's alias IDs (tuning "alias_devices" = a: IDs n ..
n+a-1 run on physical GPU id mod n with their own per-device state) stand in
for them; shmr_ec_device_stats shows per ID what ran there and which objects
were created for it.  Results are checked bit for bit against the CPU oracle.
"""
import numpy as np
import pytest

import shmr_amd
from shmr_amd import _native
from oracle import rs_oracle as O

pytestmark = pytest.mark.gpu

INVALID = -100


def _blocks(k, p, S, B, seed):
    rng = np.random.default_rng(seed)
    blk = rng.integers(0, 256, (B, k + p, S), dtype=np.uint8)
    blk[:, k:] = 0
    return blk


def _expect(k, p, blk):
    want = blk.copy()
    for b in range(blk.shape[0]):
        sh = [want[b, i].copy() for i in range(k + p)]
        O.ReedSolomon(k, p).encode(sh)
        want[b] = np.stack(sh)
    return want


@pytest.fixture
def aliases(gpu):
    """Tools build with 3 alias IDs on top of the physical GPUs."""
    with _native.tools():
        n = shmr_amd.device_count()
        shmr_amd.set_tuning(alias_devices=3)
        try:
            yield n
        finally:
            shmr_amd.set_tuning(alias_devices=0)


def _delta(before, after):
    return {k: after[k] - before[k] for k in after}


def test_device_list_validated_before_any_work(gpu):
    """Out-of-range / negative device IDs: INVALID_ARGUMENT before any buffer is
    touched (encode and reconstruct, product library)."""
    k, p, S, B = 8, 3, 4096, 4
    n = shmr_amd.device_count()
    rs = shmr_amd.ReedSolomon(k, p)
    blk = _blocks(k, p, S, B, 1)
    blk[:, k:] = 0x5A
    for devs in ([0, n], [n + 7], [-1], [0, 0, -3]):
        with pytest.raises(shmr_amd.Error) as e:
            rs.encode_blocks_host(blk, devices=devs)
        assert e.value.code == INVALID
        assert (blk[:, k:] == 0x5A).all()
    want = _expect(k, p, _blocks(k, p, S, B, 1))
    present = np.ones((B, k + p), np.uint8)
    present[:, 2] = 0
    work = want.copy()
    work[:, 2] = 0xA5
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct_blocks_host(work, present, devices=[0, n])
    assert e.value.code == INVALID and (work[:, 2] == 0xA5).all()
    with pytest.raises(shmr_amd.Error):
        rs.set_device(-1)
    rs.set_device(n)                      # accepted here, checked at the call
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode([want[0, i].copy() for i in range(k + p)])
    assert e.value.code == INVALID


def test_product_library_has_no_alias_ids(gpu):
    assert _native.lib().shmr_ec_set_tuning(b"alias_devices", 2) == INVALID
    assert _native.lib().shmr_ec_set_tuning(b"alias_devices", 0) == 0


def test_host_batches_keep_per_device_state(aliases):
    """Pageable and mapped host batches over 4 device IDs: blocks round-robin,
    each ID gets its own plan image, staging streams / upload ring, and the
    parity / rebuilt shards are bit-exact."""
    n = aliases
    k, p, S, B = 8, 3, 65536 + 48, 12
    ids = list(range(n + 3))[-4:] if n >= 1 else [0]
    ids = [0, n, n + 1, n + 2]
    rs = shmr_amd.ReedSolomon(k, p)
    before = {d: shmr_amd.device_stats(d) for d in ids}
    # pageable: gathered into each device's pinned mirror (its own pipe streams)
    blk = _blocks(k, p, S, B, 2)
    want = _expect(k, p, blk)
    rs.encode_blocks_host(blk, devices=ids)
    assert np.array_equal(blk, want)
    mid = {d: shmr_amd.device_stats(d) for d in ids}
    for d in ids:
        dd = _delta(before[d], mid[d])
        assert dd["blocks_encoded"] == B // len(ids), (d, dd)
        assert dd["launches"] >= 1
    for d in ids[1:]:                      # alias IDs were never used before this test
        assert mid[d]["plan_images"] >= 1 and mid[d]["staging_streams"] >= 3, (d, mid[d])
    # mapped Block Cache slab: zero-copy, per-device upload rings of pointer tables
    slab = shmr_amd.PinnedBuffer(B * (k + p) * S)
    arr = slab.array.reshape(B, k + p, S)
    arr[:] = _blocks(k, p, S, B, 3)
    want2 = _expect(k, p, arr.copy())
    z0, _ = shmr_amd.path_stats()
    rs.encode_blocks_host(arr, devices=ids[::-1])
    assert np.array_equal(arr, want2)
    assert shmr_amd.path_stats()[0] - z0 == B
    after = {d: shmr_amd.device_stats(d) for d in ids}
    for d in ids:
        assert after[d]["blocks_encoded"] - mid[d]["blocks_encoded"] == B // len(ids)
        assert after[d]["upload_rings"] >= 1, (d, after[d])
    # reconstruct, a different erasure pattern per block, over the same IDs
    present = np.ones((B, k + p), np.uint8)
    for b in range(B):
        present[b, [b % k, k + b % p]] = 0
    arr[present == 0] = 0
    rs.reconstruct_blocks_host(arr, present, devices=ids)
    assert np.array_equal(arr, want2)
    final = {d: shmr_amd.device_stats(d) for d in ids}
    for d in ids:
        assert final[d]["blocks_reconstructed"] - after[d]["blocks_reconstructed"] == B // len(ids)
    del slab


def test_device_batch_on_alias_id(aliases):
    """A device-resident batch submitted under an alias ID runs on the physical
    GPU behind it and is counted under that ID only."""
    import torch
    n = aliases
    k, p, S, B = 10, 4, 1677722, 3
    pitch = (S + 255) // 256 * 256
    rs = shmr_amd.ReedSolomon(k, p)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(5)
    data = torch.randint(0, 256, (B, k, pitch), dtype=torch.uint8, device="cuda:0", generator=g)
    parity = torch.zeros((B, p, pitch), dtype=torch.uint8, device="cuda:0")
    b0, bn = shmr_amd.device_stats(0), shmr_amd.device_stats(n + 1)
    rs.encode_batch_dev(data, parity, shard_len=S, device=n + 1)
    torch.cuda.synchronize()
    assert shmr_amd.device_stats(n + 1)["blocks_encoded"] - bn["blocks_encoded"] == B
    assert shmr_amd.device_stats(0)["blocks_encoded"] == b0["blocks_encoded"]
    hd, hp = data.cpu().numpy(), parity.cpu().numpy()
    for b in range(B):
        sh = [hd[b, i, :S].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
        O.ReedSolomon(k, p).encode(sh)
        for r in range(p):
            assert np.array_equal(hp[b, r, :S], sh[k + r]), (b, r)
    with pytest.raises(shmr_amd.Error) as e:       # one past the last alias
        rs.encode_batch_dev(data, parity, shard_len=S, device=n + 3)
    assert e.value.code == INVALID


def test_eight_device_ids_single_process(gpu):
    """The daemon's single-process shape at N = 8, rehearsed with alias IDs
    (tools build; alias_devices = 8 - n): per-device state created by eight
    threads at once, then pageable and mapped host batches (encode and a
    reconstruct of two erasures per block, a pattern per block) round-robin
    over eight IDs.  Every ID shows its own counter set (blocks, plan images,
    staging streams, upload rings) and every byte equals the oracle's."""
    import threading
    with _native.tools():
        n = shmr_amd.device_count()
        extra = max(0, 8 - n)
        shmr_amd.set_tuning(alias_devices=max(extra, 1))
        try:
            ids = list(range(8))
            errs = []

            def init(d):
                try:
                    shmr_amd.device_init(d)
                except Exception as e:   # reported below
                    errs.append((d, repr(e)))
            th = [threading.Thread(target=init, args=(d,)) for d in ids]
            for t in th:
                t.start()
            for t in th:
                t.join(60)
            assert not errs, errs
            k, p, S, B = 8, 3, 65536 + 48, 24
            rs = shmr_amd.ReedSolomon(k, p)
            before = {d: shmr_amd.device_stats(d) for d in ids}
            blk = _blocks(k, p, S, B, 11)
            want = _expect(k, p, blk)
            rs.encode_blocks_host(blk, devices=ids)                  # pageable: per-device pinned mirrors
            assert np.array_equal(blk, want)
            slab = shmr_amd.PinnedBuffer(B * (k + p) * S)             # mapped: zero-copy per device
            arr = slab.array.reshape(B, k + p, S)
            arr[:] = _blocks(k, p, S, B, 12)
            want2 = _expect(k, p, arr.copy())
            rs.encode_blocks_host(arr, devices=ids)
            assert np.array_equal(arr, want2)
            present = np.ones((B, k + p), np.uint8)
            for b in range(B):
                present[b, [b % (k + p), (b + 4) % (k + p)]] = 0
            arr[present == 0] = 0
            rs.reconstruct_blocks_host(arr, present, devices=ids)
            assert np.array_equal(arr, want2)
            work = want.copy()
            work[present == 0] = 0xEE
            rs.reconstruct_blocks_host(work, present, devices=ids)
            assert np.array_equal(work, want)
            after = {d: shmr_amd.device_stats(d) for d in ids}
            for d in ids:
                dd = _delta(before[d], after[d])
                assert dd["blocks_encoded"] == 2 * B // 8, (d, dd)
                assert dd["blocks_reconstructed"] == 2 * B // 8, (d, dd)
                assert after[d]["plan_images"] >= 1 and after[d]["staging_streams"] >= 1, (d, after[d])
                assert after[d]["upload_rings"] >= 1, (d, after[d])
            del slab
        finally:
            shmr_amd.set_tuning(alias_devices=0)
