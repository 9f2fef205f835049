"""GPU parity tests: the HIP path through the C ABI vs the CPU oracle, bit-exact.

Reference call sites under test: ReedSolomon::encode (src/vfs/block.rs:427)
and ReedSolomon::reconstruct (src/vfs/block.rs:560), with shard sizes from
calculate_shard_size (src/vfs/mod.rs:16-18).
"""
import itertools

import numpy as np
import pytest

import shmr_amd
from shmr_amd import _native
from oracle import c_oracle
from oracle import rs_oracle as O

pytestmark = pytest.mark.gpu


def rand_shards(rng, n, L):
    return [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(n)]


def oracle_parity(k, p, data):
    L = len(data[0])
    sh = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(p)]
    c_oracle.encode(k, p, sh)
    return sh[k:]


# ---------------------------------------------------------------- host-buffer API
@pytest.mark.parametrize("k,p,L", [(4, 2, 262144), (8, 3, 524288), (10, 4, 1677722), (5, 5, 2),
                                   (1, 1, 1), (3, 2, 17), (8, 3, 4095), (8, 3, 4097), (8, 3, 8192 + 5),
                                   (17, 3, 100003), (2, 7, 33)])
def test_encode_host_matches_oracle(gpu, k, p, L):
    rng = np.random.default_rng([k, p, L])
    data = rand_shards(rng, k, L)
    shards = [d.copy() for d in data] + [np.full(L, 0xAA, np.uint8) for _ in range(p)]
    shmr_amd.ReedSolomon(k, p).encode(shards)
    for a, b in zip(shards[k:], oracle_parity(k, p, data)):
        assert np.array_equal(a, b)
    for a, b in zip(shards[:k], data):
        assert np.array_equal(a, b)   # inputs untouched


def test_encode_kat_5_5(gpu):
    """Upstream known-answer vector (JavaReedSolomon / crate test_encoding)."""
    data = [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]]
    shards = [np.array(d, np.uint8) for d in data] + [np.zeros(2, np.uint8) for _ in range(5)]
    shmr_amd.ReedSolomon(5, 5).encode(shards)
    assert [s.tolist() for s in shards[5:]] == [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]


@pytest.mark.parametrize("fill", [0x00, 0xFF])
def test_encode_constant_blocks(gpu, fill):
    k, p, L = 8, 3, 524288
    data = [np.full(L, fill, np.uint8) for _ in range(k)]
    shards = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(p)]
    shmr_amd.ReedSolomon(k, p).encode(shards)
    for a, b in zip(shards[k:], oracle_parity(k, p, data)):
        assert np.array_equal(a, b)


def test_every_coefficient_and_byte(gpu):
    """Exhaustive multiply check: 256 data values x every coefficient that a
    (255, 1) code and a (1, 255) code use."""
    for k, p in [(255, 1), (1, 255), (128, 128)]:
        L = 256 * 3 + 7
        rng = np.random.default_rng(k)
        data = [np.resize(np.roll(np.arange(256, dtype=np.uint8), i), L) for i in range(k)]
        data[0] = rng.integers(0, 256, L, dtype=np.uint8)
        shards = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(p)]
        shmr_amd.ReedSolomon(k, p).encode(shards)
        for a, b in zip(shards[k:], oracle_parity(k, p, data)):
            assert np.array_equal(a, b), (k, p)


PATTERNS_83 = [
    [0], [7], [8], [10], [0, 8], [3, 4], [1, 9, 10], [0, 1, 2], [5, 6, 7], [2, 8, 9],
]


@pytest.mark.parametrize("missing", PATTERNS_83)
@pytest.mark.parametrize("data_only", [False, True])
def test_reconstruct_host_matches_oracle(gpu, missing, data_only):
    k, p, L = 8, 3, 524288 + 13
    rng = np.random.default_rng(sum(missing) + 100 * data_only)
    full = rand_shards(rng, k, L)
    full += oracle_parity(k, p, full)
    got = [None if i in missing else full[i].copy() for i in range(k + p)]
    rs = shmr_amd.ReedSolomon(k, p)
    (rs.reconstruct_data if data_only else rs.reconstruct)(got)
    ref = [None if i in missing else full[i].copy() for i in range(k + p)]
    (O.ReedSolomon(k, p).reconstruct_data if data_only else O.ReedSolomon(k, p).reconstruct)(ref)
    for i in range(k + p):
        if data_only and i >= k and i in missing:
            assert got[i] is None
            continue
        assert np.array_equal(got[i], ref[i]), i
        assert np.array_equal(got[i], full[i]), i


def test_reconstruct_inconsistent_shards_follow_crate(gpu):
    """Inputs that are not a codeword: the crate uses the first k present
    shards and then re-encodes missing parity from the rebuilt data."""
    k, p, L = 4, 3, 4099
    rng = np.random.default_rng(7)
    shards = rand_shards(rng, k + p, L)      # random: not a codeword
    for missing in itertools.combinations(range(k + p), 2):
        got = [None if i in missing else shards[i].copy() for i in range(k + p)]
        ref = [None if i in missing else shards[i].copy() for i in range(k + p)]
        shmr_amd.ReedSolomon(k, p).reconstruct(got)
        O.ReedSolomon(k, p).reconstruct(ref)
        for i in range(k + p):
            assert np.array_equal(got[i], ref[i]), (missing, i)


def test_reconstruct_all_patterns_10_4(gpu):
    k, p, L = 10, 4, 3000
    rng = np.random.default_rng(11)
    full = rand_shards(rng, k, L)
    full += oracle_parity(k, p, full)
    rs = shmr_amd.ReedSolomon(k, p)
    for n in (1, 2, 3, 4):
        for missing in itertools.combinations(range(k + p), n):
            got = [None if i in missing else full[i].copy() for i in range(k + p)]
            rs.reconstruct(got)
            for i in missing:
                assert np.array_equal(got[i], full[i]), (missing, i)


# --------------------------------------------------------------- device batch API
KNOBS = ("chunks", "nt_load", "nt_store", "occ8", "grid", "threads", "depth", "wgs_per_cu", "occ", "early", "spre",
         "fuse_tail", "glds", "serial", "peel", "wave_run")


def _dev_encode_check(gpu, k, p, L, B, pitch=None, **knobs):
    """Encode on the device and compare with the oracle.  With knobs: the
    measurement variant from the tools build (libshmr_ec_tools.so)."""
    if knobs:
        with _native.tools():
            return _dev_encode_check_in(gpu, k, p, L, B, pitch, knobs)
    return _dev_encode_check_in(gpu, k, p, L, B, pitch, knobs)


def _dev_encode_check_in(gpu, k, p, L, B, pitch, knobs):
    import torch
    saved = {f"encode.{kk}": shmr_amd.get_tuning(f"encode.{kk}") for kk in KNOBS}
    shmr_amd.set_tuning(**{f"encode.{kk}": v for kk, v in knobs.items()})
    try:
        pitch = pitch or L
        g = torch.Generator(device=gpu)
        g.manual_seed(k * 1000 + p * 10 + B)
        data = torch.randint(0, 256, (B, k, pitch), dtype=torch.uint8, device=gpu, generator=g)
        parity = torch.full((B, p, pitch), 0x5A, dtype=torch.uint8, device=gpu)
        shmr_amd.ReedSolomon(k, p).encode_batch_dev(data, parity, shard_len=L)
        torch.cuda.synchronize()
        hd, hp = data.cpu().numpy(), parity.cpu().numpy()
        for b in range(B):
            ref = oracle_parity(k, p, [hd[b, i, :L].copy() for i in range(k)])
            for r in range(p):
                assert np.array_equal(hp[b, r, :L], ref[r]), (b, r)
                assert (hp[b, r, L:] == 0x5A).all(), "wrote past shard_len"
    finally:
        shmr_amd.set_tuning(**saved)


@pytest.mark.parametrize("k,p,L,B", [(8, 3, 524288, 16), (4, 2, 262144, 8), (10, 4, 1677722, 3),
                                     (6, 3, 8192 * 3 + 16, 5), (3, 5, 16, 7),
                                     # 4-row encodes (early + serial policy): tile-multiple length,
                                     # and 6 rows = a 4-row and a 2-row launch with partial tiles
                                     (10, 4, 8192 * 40, 3), (5, 6, 8192 * 5 + 7, 4)])
def test_encode_batch_dev(gpu, k, p, L, B):
    _dev_encode_check(gpu, k, p, L, B, pitch=(L + 255) // 256 * 256)


BASE = dict(chunks=1, nt_load=0, nt_store=0, occ8=0, grid=-1, threads=256, depth=3, wgs_per_cu=0, occ=0, early=0, spre=0,
            fuse_tail=0, glds=0, serial=0, peel=0, wave_run=0)
VARIANTS = [dict(BASE, **v) for v in (
    {}, dict(nt_load=1), dict(nt_store=1), dict(nt_load=1, nt_store=1),
    dict(occ8=1, nt_load=1, nt_store=1),
    dict(chunks=2), dict(chunks=2, nt_load=1, nt_store=1), dict(chunks=4, nt_load=1, nt_store=1),
    dict(grid=0), dict(chunks=2, grid=0), dict(chunks=4, grid=7, nt_load=1, nt_store=1),
    dict(nt_load=1, nt_store=1, threads=128), dict(nt_load=1, nt_store=1, threads=512),
    dict(nt_store=1, threads=512), dict(chunks=2, nt_load=1, nt_store=1, threads=128),
    dict(nt_load=1, nt_store=1, depth=5), dict(nt_load=1, nt_store=1, depth=9),
    dict(nt_load=1, depth=5), dict(nt_load=1, depth=9), dict(nt_load=1, nt_store=1, depth=2),
    dict(nt_load=1, nt_store=1, depth=2, wgs_per_cu=3), dict(nt_load=1, nt_store=1, depth=2, occ=7),
    dict(nt_load=1, nt_store=1, occ=6), dict(nt_load=1, nt_store=1, depth=2, early=1),
    dict(chunks=2, nt_load=1, nt_store=1, depth=2, early=1), dict(nt_load=1, nt_store=1, early=1),
    dict(nt_load=1, nt_store=1, depth=2, early=1, grid=0), dict(nt_load=1, nt_store=1, depth=2, spre=1),
    dict(chunks=2, nt_load=1, nt_store=1, depth=2, spre=1), dict(nt_load=1, nt_store=1, spre=1),
    dict(nt_load=1, nt_store=1, depth=2, spre=1, grid=0), dict(chunks=4, nt_load=1, nt_store=1, grid=7),
    dict(nt_load=1, nt_store=1, depth=2, fuse_tail=1), dict(nt_load=1, nt_store=1, depth=2, early=1, fuse_tail=1),
    dict(chunks=2, nt_load=1, nt_store=1, depth=2, fuse_tail=1), dict(nt_load=1, nt_store=1, depth=2, fuse_tail=1, grid=0),
    dict(nt_store=1, depth=2, fuse_tail=1), dict(chunks=2, nt_load=1, nt_store=1, depth=2, early=1, fuse_tail=1),
    # LDS-DMA input ring (global_load_lds_dwordx4)
    dict(nt_load=1, nt_store=1, glds=1), dict(nt_load=1, nt_store=1, glds=1, depth=5),
    dict(nt_load=1, nt_store=1, glds=1, depth=9), dict(chunks=2, nt_load=1, nt_store=1, glds=1),
    dict(chunks=2, nt_load=1, nt_store=1, glds=1, depth=5), dict(nt_load=1, nt_store=1, glds=1, fuse_tail=1),
    dict(nt_load=1, nt_store=1, glds=1, depth=5, fuse_tail=1), dict(chunks=2, nt_load=1, nt_store=1, glds=1, fuse_tail=1),
    dict(nt_load=1, nt_store=1, glds=1, depth=5, grid=0),
    # GF math ordered one dword at a time (fewer live registers)
    dict(nt_load=1, nt_store=1, depth=2, serial=1), dict(chunks=2, nt_load=1, nt_store=1, depth=2, serial=1),
    dict(nt_load=1, nt_store=1, depth=2, fuse_tail=1, serial=1),
    dict(chunks=2, nt_load=1, nt_store=1, depth=2, fuse_tail=1, serial=1), dict(nt_load=1, nt_store=1, serial=1),
    dict(nt_load=1, nt_store=1, depth=2, early=1, serial=1), dict(nt_load=1, nt_store=1, depth=5, serial=1),
    dict(nt_load=1, nt_store=1, depth=2, early=1, fuse_tail=1, serial=1),
    dict(chunks=2, nt_load=1, nt_store=1, depth=2, early=1, serial=1),
    dict(chunks=2, nt_load=1, nt_store=1, depth=2, early=1, fuse_tail=1, serial=1),
    # scalar-loaded tables with fused tails (tools/ab_spre.sh)
    dict(chunks=2, nt_load=1, nt_store=1, depth=2, spre=1, fuse_tail=1),
    dict(chunks=2, nt_load=1, nt_store=1, depth=2, spre=1, fuse_tail=1, serial=1),
    dict(nt_load=1, nt_store=1, depth=2, spre=1, fuse_tail=1),
    dict(nt_load=1, nt_store=1, depth=2, spre=1, fuse_tail=1, serial=1, wgs_per_cu=6),
    # depth-2 ring with the tail peeled (k = 5 and 7 end it on an odd shard)
    dict(nt_load=1, nt_store=1, depth=2, peel=1), dict(nt_load=1, nt_store=1, depth=2, early=1, peel=1),
    dict(nt_load=1, nt_store=1, depth=2, early=1, fuse_tail=1, peel=1),
    dict(nt_load=1, nt_store=1, depth=2, fuse_tail=1, peel=1),
    dict(chunks=2, nt_load=1, nt_store=1, depth=2, early=1, serial=1, peel=1),
    dict(chunks=2, nt_load=1, nt_store=1, depth=2, early=1, fuse_tail=1, serial=1, peel=1),
    # U = 2 slots in wave-contiguous runs
    dict(chunks=2, nt_load=1, nt_store=1, depth=2, early=1, fuse_tail=1, serial=1, wave_run=1),
    dict(chunks=2, nt_load=1, nt_store=1, depth=2, fuse_tail=1, wave_run=1))]


@pytest.mark.parametrize("knobs", VARIANTS, ids=lambda d: ",".join(f"{k}={v}" for k, v in d.items() if BASE[k] != v) or "base")
@pytest.mark.parametrize("k,p", [(8, 3), (5, 1), (10, 4), (7, 6)])
def test_encode_batch_dev_tuning_variants(gpu, knobs, k, p):
    _dev_encode_check(gpu, k, p, 524288 + 4096 + 48, 3, pitch=524288 + 8192, **knobs)


def test_reconstruct_variants_match(gpu):
    """Every decode variant (tools build) produces identical bytes."""
    with _native.tools():
        _reconstruct_variants_match(gpu)


def _reconstruct_variants_match(gpu):
    import torch
    k, p, S, B = 8, 3, 65536 * 3 + 4096 + 32, 6
    pitch = (S + 255) // 256 * 256
    rng = np.random.default_rng(4)
    host = rng.integers(0, 256, (B, k + p, pitch), dtype=np.uint8)
    for b in range(B):
        par = oracle_parity(k, p, [host[b, i, :S].copy() for i in range(k)])
        for r in range(p):
            host[b, k + r, :S] = par[r]
    present = np.ones((B, k + p), np.uint8)
    for b in range(B):
        present[b, [b % k, k + b % p]] = 0
    rs = shmr_amd.ReedSolomon(k, p)
    saved = {f"decode.{kk}": shmr_amd.get_tuning(f"decode.{kk}") for kk in KNOBS}
    try:
        for knobs in VARIANTS:
            shmr_amd.set_tuning(**{f"decode.{kk}": v for kk, v in knobs.items()})
            dev = torch.from_numpy(host.copy()).to(gpu)
            for b in range(B):
                for i in range(k + p):
                    if not present[b, i]:
                        dev[b, i, :S] = 0
            rs.reconstruct_batch_dev(dev, present, shard_len=S)
            torch.cuda.synchronize()
            assert np.array_equal(dev.cpu().numpy()[:, :, :S], host[:, :, :S]), knobs
    finally:
        shmr_amd.set_tuning(**saved)


def test_uncompiled_variant_is_reported(gpu):
    with _native.tools():
        _uncompiled_variant_is_reported(gpu)


def _uncompiled_variant_is_reported(gpu):
    import torch
    saved = {f"encode.{kk}": shmr_amd.get_tuning(f"encode.{kk}") for kk in KNOBS}
    try:
        shmr_amd.set_tuning(**{"encode.chunks": 4, "encode.nt_load": 0, "encode.nt_store": 1, "encode.occ8": 1})
        data = torch.zeros((1, 2, 65536), dtype=torch.uint8, device=gpu)
        parity = torch.zeros((1, 1, 65536), dtype=torch.uint8, device=gpu)
        with pytest.raises(shmr_amd.Error) as ei:
            shmr_amd.ReedSolomon(2, 1).encode_batch_dev(data, parity)
        assert ei.value.name == "InvalidArgument"
    finally:
        shmr_amd.set_tuning(**saved)


def test_encode_batch_dev_unaligned_reference_layout(gpu):
    """The reference buffer layout with S = 1,677,722 (S % 4 == 2): shard i at
    i*S, so odd shards are misaligned -> byte-granular path, same bytes."""
    import torch
    k, p = 10, 4
    S = shmr_amd.calculate_shard_size(16 << 20, k)
    assert S == 1677722
    g = torch.Generator(device=gpu)
    g.manual_seed(3)
    B = 2
    data = torch.randint(0, 256, (B, k * S), dtype=torch.uint8, device=gpu, generator=g)
    parity = torch.empty((B, p * S), dtype=torch.uint8, device=gpu)
    shmr_amd.ReedSolomon(k, p).encode_batch_dev(data, parity, shard_len=S, data_shard_pitch=S,
                                                parity_shard_pitch=S)
    torch.cuda.synchronize()
    hd, hp = data.cpu().numpy(), parity.cpu().numpy()
    for b in range(B):
        ref = oracle_parity(k, p, [hd[b, i * S:(i + 1) * S].copy() for i in range(k)])
        for r in range(p):
            assert np.array_equal(hp[b, r * S:(r + 1) * S], ref[r])


@pytest.mark.parametrize("k,p,erasures,B", [(8, 3, 1, 24), (10, 4, 2, 24), (8, 3, 3, 24),
                                             (10, 4, 2, 90)])   # > 32 runs: uploaded block/plan tables
def test_reconstruct_batch_dev_mixed_patterns(gpu, k, p, erasures, B):
    """Mixed erasure patterns in one batch: few runs travel in the kernel
    arguments (segment launch), many take the uploaded-table launch."""
    import torch
    S = 65536 + 12
    pitch = (S + 255) // 256 * 256
    rng = np.random.default_rng(k + erasures)
    host = rng.integers(0, 256, (B, k + p, pitch), dtype=np.uint8)
    for b in range(B):
        par = oracle_parity(k, p, [host[b, i, :S].copy() for i in range(k)])
        for r in range(p):
            host[b, k + r, :S] = par[r]
    present = np.ones((B, k + p), np.uint8)
    for b in range(B):
        miss = rng.choice(k + p, size=erasures, replace=False)
        present[b, miss] = 0
    present[5] = 1                 # an all-present block is a no-op
    dev = torch.from_numpy(host.copy()).to(gpu)
    # poison the erased shards on the device
    for b in range(B):
        for i in range(k + p):
            if not present[b, i]:
                dev[b, i, :S] = 0xEE
    rs = shmr_amd.ReedSolomon(k, p)
    rs.reconstruct_batch_dev(dev, present, shard_len=S)
    torch.cuda.synchronize()
    out = dev.cpu().numpy()
    assert np.array_equal(out[:, :, :S], host[:, :, :S])


def test_roundtrip_full_size_83(gpu):
    """Size-independent property at the benchmark size: encode -> erase every
    single data shard in turn -> reconstruct == original (512 blocks would be
    the bench batch; 64 keeps the test quick)."""
    import torch
    k, p, S, B = 8, 3, 524288, 64
    g = torch.Generator(device=gpu)
    g.manual_seed(99)
    shards = torch.empty((B, k + p, S), dtype=torch.uint8, device=gpu)
    shards[:, :k] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=gpu, generator=g)
    rs = shmr_amd.ReedSolomon(k, p)
    rs.encode_batch_dev(shards[:, :k], shards[:, k:], shard_len=S, data_shard_pitch=S, parity_shard_pitch=S)
    ref = shards.clone()
    present = np.ones((B, k + p), np.uint8)
    present[np.arange(B), np.arange(B) % k] = 0
    present[np.arange(B), k + np.arange(B) % p] = 0
    shards[torch.arange(B), torch.arange(B) % k] = 0
    shards[torch.arange(B), k + torch.arange(B) % p] = 0
    rs.reconstruct_batch_dev(shards, present, shard_len=S)
    torch.cuda.synchronize()
    assert torch.equal(shards, ref)
    # checksum of checksums: parity of the batch vs a CPU oracle sample
    hd = ref[:2].cpu().numpy()
    for b in range(2):
        par = oracle_parity(k, p, [hd[b, i].copy() for i in range(k)])
        for r in range(p):
            assert np.array_equal(hd[b, k + r], par[r])


def test_encode_blocks_host_round_robin(gpu):
    k, p, S, B = 8, 3, 100000, 5
    rng = np.random.default_rng(5)
    blocks = [[rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
              for _ in range(B)]
    shmr_amd.ReedSolomon(k, p).encode_blocks_host(blocks, devices=[0])
    for blk in blocks:
        ref = oracle_parity(k, p, blk[:k])
        for r in range(p):
            assert np.array_equal(blk[k + r], ref[r])


def test_sync_data_erasure_via_gpu(gpu):
    """VirtualBlock::sync_data Erasure arm (block.rs:404-440) on a partial
    buffer (700,001 B of a 1 MiB RS(4,2) block -> 3 data chunks + 1 zero
    shard), arithmetic on the GPU, layout from the oracle's glue."""
    size, k, p = 1 << 20, 4, 2
    rng = np.random.default_rng(0)
    buf = rng.integers(0, 256, 700001, dtype=np.uint8)
    S = shmr_amd.calculate_shard_size(size, k)
    shards = []
    for off in range(0, len(buf), S):
        c = np.zeros(S, np.uint8)
        c[:len(buf[off:off + S])] = buf[off:off + S]
        shards.append(c)
    shards += [np.zeros(S, np.uint8) for _ in range(p + k - len(shards))]
    shmr_amd.ReedSolomon(k, p).encode(shards)
    ref = O.sync_data_erasure(buf.tobytes(), size, k, p)
    for a, b in zip(shards, ref):
        assert np.array_equal(a, b)


# ------------------------------------------------------- maximum shard counts
@pytest.mark.parametrize("k,p", [(255, 1), (1, 255), (128, 128), (200, 56)])
def test_max_shard_counts_encode_reconstruct(gpu, k, p):
    """k + p = 256, the crate's limit (ReedSolomon::new, block.rs:405): encode
    on the GPU vs the oracle, then lose p shards (the most the code allows)
    and rebuild them, bit-exact.  p > 4 output rows run as several launches."""
    L = 4096 + 24
    rng = np.random.default_rng([k, p])
    data = rand_shards(rng, k, L)
    shards = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(p)]
    rs = shmr_amd.ReedSolomon(k, p)
    rs.encode(shards)
    want = oracle_parity(k, p, data)
    for a, b in zip(shards[k:], want):
        assert np.array_equal(a, b)
    full = [s.copy() for s in shards]
    lost = rng.choice(k + p, size=p, replace=False)
    got = [None if i in lost else full[i].copy() for i in range(k + p)]
    rs.reconstruct(got)
    for i in range(k + p):
        assert np.array_equal(got[i], full[i]), i


def test_too_many_erasures_on_gpu_path(gpu):
    """p + 1 absent shards -> TooFewShardsPresent before any device work, and
    the present buffers are untouched (the reference would panic on unwrap)."""
    k, p, L = 8, 3, 1000
    rng = np.random.default_rng(1)
    shards = rand_shards(rng, k + p, L)
    keep = [s.copy() for s in shards]
    for i in (0, 3, 9, 10):
        shards[i] = None
    with pytest.raises(shmr_amd.Error) as e:
        shmr_amd.ReedSolomon(k, p).reconstruct(shards)
    assert e.value.name == "TooFewShardsPresent"
    for i in range(k + p):
        if shards[i] is not None:
            assert np.array_equal(shards[i], keep[i])


@pytest.mark.parametrize("mapped", [False, True])
def test_blocks_host_device_list_round_robin(gpu, mapped):
    """devices=[0, 0, 0]: the multi-device worker fan-out (block b ->
    devices[b % 3], one worker per entry) on the one GPU of the box, staged
    and zero-copy."""
    k, p, S, B = 8, 3, 65536 + 48, 10
    rng = np.random.default_rng(17)
    keep = None
    if mapped:
        keep = shmr_amd.PinnedBuffer(B * (k + p) * S)
        arr = keep.array.reshape(B, k + p, S)
        blocks = [[arr[b, i] for i in range(k + p)] for b in range(B)]
    else:
        blocks = [[np.zeros(S, np.uint8) for _ in range(k + p)] for _ in range(B)]
    for blk in blocks:
        for i in range(k):
            blk[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
    rs = shmr_amd.ReedSolomon(k, p)
    z0, s0 = shmr_amd.path_stats()
    rs.encode_blocks_host(blocks, devices=[0, 0, 0])
    z1, s1 = shmr_amd.path_stats()
    assert (z1 - z0, s1 - s0) == ((B, 0) if mapped else (0, B))
    for blk in blocks:
        for got, want in zip(blk[k:], oracle_parity(k, p, blk[:k])):
            assert np.array_equal(got, want)
    full = [[x.copy() for x in blk] for blk in blocks]
    present = np.ones((B, k + p), np.uint8)
    for b in range(B):
        present[b, [(b % k), k + (b % p)]] = 0
        blocks[b][b % k][:] = 0
        blocks[b][k + b % p][:] = 0
    rs.reconstruct_blocks_host(blocks, present, devices=[0, 0, 0])
    for b in range(B):
        for i in range(k + p):
            assert np.array_equal(blocks[b][i], full[b][i]), (b, i)


def test_reconstruct_segments_irregular_runs(gpu):
    """Two patterns whose blocks are not one arithmetic progression each (some
    blocks lose nothing): split into several runs, still one segment launch."""
    import torch
    k, p, S, B = 8, 3, 8192 + 16, 40
    pitch = S + 240
    rng = np.random.default_rng(23)
    host = rng.integers(0, 256, (B, k + p, pitch), dtype=np.uint8)
    for b in range(B):
        par = oracle_parity(k, p, [host[b, i, :S].copy() for i in range(k)])
        for r in range(p):
            host[b, k + r, :S] = par[r]
    present = np.ones((B, k + p), np.uint8)
    for b in range(B):
        if b % 7 == 3:
            continue                       # untouched blocks break the progressions
        present[b, 2 if b % 2 else 9] = 0
    dev = torch.from_numpy(host.copy()).to(gpu)
    for b in range(B):
        for i in range(k + p):
            if not present[b, i]:
                dev[b, i, :S] = 0xEE
    shmr_amd.ReedSolomon(k, p).reconstruct_batch_dev(dev, present, shard_len=S)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy()[:, :, :S], host[:, :, :S])


def test_roundtrip_full_size_104(gpu):
    """BASELINE config 4 at its full per-GPU size (64 x 16 MiB RS(10,4) blocks,
    S = 1,677,722, pitched): encode -> erase {b mod 10, (b+3) mod 10} (the bench
    pattern) plus every parity shard of every 7th block (4 erasures, the most the
    code allows) -> reconstruct == original; one block's parity vs the oracle."""
    import torch
    k, p, B = 10, 4, 64
    S = shmr_amd.calculate_shard_size(16 << 20, k)
    pitch = (S + 255) // 256 * 256
    g = torch.Generator(device=gpu)
    g.manual_seed(104)
    shards = torch.zeros((B, k + p, pitch), dtype=torch.uint8, device=gpu)
    shards[:, :k, :S] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=gpu, generator=g)
    rs = shmr_amd.ReedSolomon(k, p)
    rs.encode_batch_dev(shards[:, :k], shards[:, k:], shard_len=S, data_shard_pitch=pitch, parity_shard_pitch=pitch)
    ref = shards.clone()
    present = np.ones((B, k + p), np.uint8)
    b = np.arange(B)
    present[b, b % 10] = 0
    present[b, (b + 3) % 10] = 0
    present[::7] = 1
    present[::7, k:] = 0
    for i in range(B):
        for s in range(k + p):
            if not present[i, s]:
                shards[i, s, :S] = 0xEE
    rs.reconstruct_batch_dev(shards, present, shard_len=S)
    torch.cuda.synchronize()
    assert torch.equal(shards[:, :, :S], ref[:, :, :S])
    hd = ref[5].cpu().numpy()
    par = oracle_parity(k, p, [hd[i, :S].copy() for i in range(k)])
    for r in range(p):
        assert np.array_equal(hd[k + r, :S], par[r])


@pytest.mark.parametrize("bounce_kib", [0, 65536])
def test_single_block_pageable_paths(gpu, bounce_kib):
    """Pageable drop-in calls through the mapped bounce buffer (one launch) and
    through per-shard staged DMA give identical, oracle-exact results."""
    saved = shmr_amd.get_tuning("bounce_kib")
    shmr_amd.set_tuning(bounce_kib=bounce_kib)
    try:
        for k, p, L in [(8, 3, 524288), (4, 2, 4099), (10, 4, 100000)]:
            rng = np.random.default_rng([k, p, L, bounce_kib])
            data = rand_shards(rng, k, L)
            shards = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(p)]
            rs = shmr_amd.ReedSolomon(k, p)
            z0, s0 = shmr_amd.path_stats()
            rs.encode(shards)
            z1, s1 = shmr_amd.path_stats()
            assert (z1 - z0, s1 - s0) == (0, 1)       # user buffers are never touched by a kernel
            want = oracle_parity(k, p, data)
            for a, b in zip(shards[k:], want):
                assert np.array_equal(a, b)
            got = [None if i in (1, k) else shards[i].copy() for i in range(k + p)]
            rs.reconstruct(got)
            for i in range(k + p):
                assert np.array_equal(got[i], shards[i])
    finally:
        shmr_amd.set_tuning(bounce_kib=saved)


@pytest.mark.parametrize("contiguous", [False, True])
def test_encode_reconstruct_in_device_buffer(gpu, contiguous):
    """Batches in shmr_ec_device_alloc memory (plain and physically contiguous
    VRAM) viewed as torch tensors: encode + 1-erasure rebuild, bit-exact."""
    import torch
    k, p, L, B = 8, 3, 65536, 6
    buf = shmr_amd.DeviceBuffer(B * (k + p) * L, contiguous=contiguous)
    shards = buf.tensor((B, k + p, L))
    assert shards.is_cuda and shards.data_ptr() == buf._p.value
    g = torch.Generator(device=gpu).manual_seed(7)
    shards[:, :k] = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=gpu, generator=g)
    rs = shmr_amd.ReedSolomon(k, p)
    rs.encode_batch_dev(shards[:, :k], shards[:, k:], shard_len=L, data_shard_pitch=L, parity_shard_pitch=L)
    torch.cuda.synchronize()
    host = shards.cpu().numpy()
    for b in range(B):
        want = oracle_parity(k, p, [host[b, i] for i in range(k)])
        for r in range(p):
            assert np.array_equal(host[b, k + r], want[r])
    present = np.ones((B, k + p), np.uint8)
    for b in range(B):
        present[b, b % k] = 0
        shards[b, b % k] = 0
    rs.reconstruct_batch_dev(shards, present, shard_len=L)
    torch.cuda.synchronize()
    assert np.array_equal(shards.cpu().numpy(), host)
    del shards
    del buf


def test_device_buffer_view_keeps_buffer_alive(gpu):
    """A tensor view holds its DeviceBuffer: dropping the buffer object first
    does not free the VRAM under the tensor (checked without touching it)."""
    import gc
    import weakref
    buf = shmr_amd.DeviceBuffer(1 << 20, contiguous=False)
    t = buf.tensor((4, 1 << 18))
    assert t.shape == (4, 1 << 18) and t.is_cuda
    ref = weakref.ref(buf)
    del buf
    gc.collect()
    assert ref() is not None
    del t
    gc.collect()
    assert ref() is None
    with pytest.raises(ValueError):
        shmr_amd.DeviceBuffer(1024, contiguous=False).tensor((2, 1024))


# ------------------------------------------------ misaligned (contiguous) layouts
@pytest.mark.gpu
@pytest.mark.parametrize("path", ["auto", "realign", "vector", "dpp", "st_align"])
@pytest.mark.parametrize("k,p,L,B,off", [
    (10, 4, 1677722, 3, 0),      # RS(10,4) 16 MiB: the reference's block buffer, shard i at i * S
    (8, 3, 524288 + 4096 + 5, 4, 3),   # odd pitch and a misaligned base
    (5, 2, 4096 * 3 + 1, 5, 7),  # 3 full tiles + a 1-byte tail per shard
    (4, 4, 4096 * 2, 2, 9),      # tile-multiple shards, every base misaligned
    (10, 4, 8192 * 3 + 2458, 2, 1),   # 4-row encode policy (8 KiB tiles, fused tails) off alignment
])
def test_contiguous_layout_realigned(gpu, path, k, p, L, B, off):
    """Shards packed at i * L inside each [k+p] * L block buffer (and the batch
    shifted by `off` bytes) are not 16-byte aligned.  "auto": the product
    policy (the vector kernels on a device that passed the unaligned-access
    probe); tools build "realign" (knob uvec=0): the realigning kernel for full
    4 KiB tiles, the remainder byte-granular; "vector" (uvec=1): the vector
    kernels unconditionally; "dpp" (uvec=1, realign=1): aligned loads realigned
    across lanes with a DPP wavefront shift; "st_align" (uvec=1, st_align=1):
    aligned stores realigned across lanes, partial chunks at the runs' ends.  Encode into the buffer's parity slots, then
    rebuild two erased shards per block in place, all against the oracle;
    bytes outside the shards stay untouched."""
    if path == "auto":
        return _contiguous_layout_check(gpu, k, p, L, B, off)
    with _native.tools():
        shmr_amd.set_tuning(uvec=0 if path == "realign" else 1)
        if path == "dpp":
            shmr_amd.set_tuning(realign=1)
        if path == "st_align":
            shmr_amd.set_tuning(st_align=1)
        try:
            _contiguous_layout_check(gpu, k, p, L, B, off)
        finally:
            shmr_amd.set_tuning(uvec=-2, realign=-2, st_align=-2)


def _contiguous_layout_check(gpu, k, p, L, B, off):
    import torch
    t = k + p
    rng = np.random.default_rng(L + B + off)
    host = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    flat = torch.full((off + B * t * L + 64,), 0x5A, dtype=torch.uint8, device=gpu)
    for b in range(B):
        for i in range(k):
            s0 = off + (b * t + i) * L
            flat[s0:s0 + L] = torch.from_numpy(host[b, i]).to(gpu)
    blocks = flat[off:off + B * t * L].view(B, t, L)
    rs = shmr_amd.ReedSolomon(k, p)
    rs.encode_batch_dev(blocks[:, :k], blocks[:, k:], shard_len=L, data_shard_pitch=L, parity_shard_pitch=L)
    torch.cuda.synchronize()
    got = blocks.cpu().numpy()
    for b in range(B):
        ref = oracle_parity(k, p, [host[b, i].copy() for i in range(k)])
        for r in range(p):
            assert np.array_equal(got[b, k + r], ref[r]), ("encode", b, r)
    full = got.copy()
    present = np.ones((B, t), np.uint8)
    for b in range(B):
        for e in ((b % t), ((b + 3) % t)):
            present[b, e] = 0
            blocks[b, e] = 0
    rs.reconstruct_batch_dev(blocks, present, shard_len=L)
    torch.cuda.synchronize()
    assert np.array_equal(blocks.cpu().numpy(), full)
    edge = flat.cpu().numpy()
    assert (edge[:off] == 0x5A).all() and (edge[off + B * t * L:] == 0x5A).all(), "wrote outside the batch"
