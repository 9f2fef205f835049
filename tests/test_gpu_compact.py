"""Reconstruct into a compact output (shmr_ec_reconstruct_batch_dev_out) vs the
CPU oracle, bit-exact.

The crate rebuilds every absent shard into a buffer of its own
(``None -> Some(vec![0; len])``, called at reference src/vfs/block.rs:556-565),
and ``load_block`` then concatenates the shards (block.rs:567-576).  The device
entry point reads the present shards in place and writes block b's rebuilt
shards, in ascending shard index, to ``out[b, j]``.  Absent slots of the input
are neither read nor written (poisoned here and checked), bytes of the output
past the rebuilt rows / shard length stay untouched (guards).
"""
import numpy as np
import pytest

import shmr_amd
from shmr_amd import _native
from oracle import c_oracle
from oracle import rs_oracle as O

pytestmark = pytest.mark.gpu

POISON, GUARD = 0xEE, 0x5A


def _codewords(k, p, S, B, pitch, seed, codeword=True):
    rng = np.random.default_rng(seed)
    host = rng.integers(0, 256, (B, k + p, pitch), dtype=np.uint8)
    if codeword:
        par = np.zeros((B, p, S), np.uint8)
        data = np.ascontiguousarray(host[:, :k, :S])
        c_oracle.encode_batch(k, p, data, par, B, S, 8)
        host[:, k:, :S] = par
    return host


def _expected(k, p, host, present, S, data_only):
    """Oracle rebuild of every block, then the compact rows in index order."""
    B, t = present.shape
    work = np.ascontiguousarray(host[:, :, :S]).copy()
    work[present == 0] = 0
    c_oracle.reconstruct_batch(k, p, work, present, S, 8, data_only=data_only)
    rows = []
    for b in range(B):
        absent = [i for i in range(t) if not present[b, i] and (i < k or not data_only)]
        if present[b].all():
            absent = []
        rows.append([work[b, i] for i in absent])
    return rows


def _run(gpu, k, p, S, B, present, data_only=False, codeword=True, pitch=None, out_pitch=None, out_rows=None,
         seed=0):
    import torch
    pitch = pitch or (S + 255) // 256 * 256
    out_pitch = out_pitch or pitch + 64
    host = _codewords(k, p, S, B, pitch, seed, codeword)
    dev = torch.from_numpy(host.copy()).to(gpu)
    mask = torch.from_numpy(present == 0).to(gpu)
    dev[mask] = POISON                      # absent slots: never read, never written
    n = out_rows if out_rows is not None else max(1, int((present == 0).sum(axis=1).max()))
    out = torch.full((B, n, out_pitch), GUARD, dtype=torch.uint8, device=gpu)
    rs = shmr_amd.ReedSolomon(k, p)
    rs.reconstruct_batch_dev_out(dev, present, out, shard_len=S, data_only=data_only)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    want = _expected(k, p, host, present, S, data_only)
    for b in range(B):
        for j, row in enumerate(want[b]):
            assert np.array_equal(got[b, j, :S], row), (b, j)
        assert (got[b, len(want[b]):] == GUARD).all(), ("rows past the rebuilt ones written", b)
        assert (got[b, :, S:] == GUARD).all(), ("bytes past the shard written", b)
    after = dev.cpu().numpy()
    assert (after[present == 0] == POISON).all(), "an absent slot was written"
    assert np.array_equal(after[present == 1], host[present == 1]), "a present shard was modified"
    return got


@pytest.mark.parametrize("k,p,erasures,B", [(8, 3, 1, 24), (8, 3, 3, 24), (10, 4, 2, 24), (10, 4, 4, 16),
                                             (10, 4, 2, 90)])   # > 32 runs: uploaded block/plan tables
@pytest.mark.parametrize("data_only", [False, True])
def test_compact_mixed_patterns(gpu, k, p, erasures, B, data_only):
    S = 65536 + 12
    rng = np.random.default_rng([k, erasures, B, data_only])
    present = np.ones((B, k + p), np.uint8)
    for b in range(B):
        present[b, rng.choice(k + p, size=erasures, replace=False)] = 0
    present[3] = 1                           # an all-present block writes nothing
    _run(gpu, k, p, S, B, present, data_only=data_only, seed=k + erasures)


def test_compact_bench_patterns_full_size(gpu):
    """BASELINE configs 3 and 4 on the compact output at full shard size: RS(8,3)
    4 MiB blocks with data shard b mod 8 lost, RS(10,4) 16 MiB blocks with
    {b mod 10, (b+3) mod 10} lost (S = 1,677,722: partial tiles fused)."""
    for k, p, size, B, pat in ((8, 3, 4 << 20, 24, lambda b: [b % 8]),
                               (10, 4, 16 << 20, 6, lambda b: [b % 10, (b + 3) % 10])):
        S = shmr_amd.calculate_shard_size(size, k)
        present = np.ones((B, k + p), np.uint8)
        for b in range(B):
            present[b, pat(b)] = 0
        _run(gpu, k, p, S, B, present, pitch=(S + 4095) // 4096 * 4096 + (4096 if S % 65536 == 0 else 0),
             out_pitch=(S + 4095) // 4096 * 4096, seed=size)


def test_compact_inconsistent_shards_follow_crate(gpu):
    """Inputs that are not a codeword: the crate decodes from the first k present
    shards and re-encodes missing parity from the rebuilt data -- the compact
    rows equal the crate's rebuilt shards (python oracle, every 2-erasure
    pattern of RS(4,3))."""
    import itertools
    import torch
    k, p, S = 4, 3, 4099
    pats = list(itertools.combinations(range(k + p), 2))
    B = len(pats)
    present = np.ones((B, k + p), np.uint8)
    for b, m in enumerate(pats):
        present[b, list(m)] = 0
    got = _run(gpu, k, p, S, B, present, codeword=False, seed=7)
    host = _codewords(k, p, S, B, (S + 255) // 256 * 256, 7, codeword=False)
    for b, m in enumerate(pats):
        ref = [None if i in m else host[b, i, :S].copy() for i in range(k + p)]
        O.ReedSolomon(k, p).reconstruct(ref)
        for j, i in enumerate(sorted(m)):
            assert np.array_equal(got[b, j, :S], ref[i]), (m, i)
    del torch


@pytest.mark.parametrize("off", [3, 0])
@pytest.mark.parametrize("path", ["auto", "realign", "dpp", "st_align"])
def test_compact_packed_layout(gpu, path, off):
    """The reference's packed block buffer (shard i at i * S, RS(10,4) 16 MiB:
    off 16-byte alignment) read in place, rebuilt shards to a compact output
    whose rows are misaligned too (off = 3) or start aligned (off = 0: sc1
    stores allowed).  "realign": the tools build's realigning kernel (knob
    uvec=0) instead of the unaligned vector path; "dpp": aligned loads
    realigned across lanes (uvec=1, realign=1); "st_align": aligned stores
    realigned across lanes (uvec=1, st_align=1)."""
    import torch

    def check():
        k, p, B = 10, 4, 3
        S = shmr_amd.calculate_shard_size(16 << 20, k)
        t = k + p
        rng = np.random.default_rng(41)
        blocks = np.zeros((B, t, S), np.uint8)
        blocks[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
        par = np.zeros((B, p, S), np.uint8)
        c_oracle.encode_batch(k, p, np.ascontiguousarray(blocks[:, :k]), par, B, S, 8)
        blocks[:, k:] = par
        present = np.ones((B, t), np.uint8)
        for b in range(B):
            present[b, [(b * 3) % t, (b * 3 + 5) % t]] = 0
        dev = torch.from_numpy(blocks.copy()).to(gpu)
        dev[torch.from_numpy(present == 0).to(gpu)] = POISON
        flat = torch.full((off + B * 2 * S + 64,), GUARD, dtype=torch.uint8, device=gpu)
        out = flat[off:off + B * 2 * S].view(B, 2, S)
        shmr_amd.ReedSolomon(k, p).reconstruct_batch_dev_out(dev, present, out, shard_len=S)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for b in range(B):
            for j, i in enumerate(np.flatnonzero(present[b] == 0)):
                assert np.array_equal(got[b, j], blocks[b, i]), (b, i)
        edge = flat.cpu().numpy()
        assert (edge[:off] == GUARD).all() and (edge[off + B * 2 * S:] == GUARD).all()

    if path == "auto":
        return check()
    with _native.tools():
        knobs = {"realign": dict(uvec=0), "dpp": dict(uvec=1, realign=1), "st_align": dict(uvec=1, st_align=1)}[path]
        shmr_amd.set_tuning(**knobs)
        try:
            check()
        finally:
            shmr_amd.set_tuning(uvec=-2, realign=-2, st_align=-2)


@pytest.mark.parametrize("k", [8, 7])
def test_compact_store_policies_match(gpu, k):
    """sc1 (the policy), nontemporal and plain stores into the compact output
    give identical bytes, and so does the peeled shard ring (tools build
    knobs; k = 7 ends the ring on an odd shard)."""
    with _native.tools():
        p, S, B = 3, 65536 * 2 + 4096, 16
        present = np.ones((B, k + p), np.uint8)
        present[np.arange(B), np.arange(B) % k] = 0
        outs = []
        for knobs in ({}, {"decode.sc1_store": 0, "decode.nt_store": 1}, {"decode.sc1_store": 0, "decode.nt_store": 0},
                      {"decode.peel": 1}):
            shmr_amd.set_tuning(**knobs)
            try:
                outs.append(_run(gpu, k, p, S, B, present, seed=5))
            finally:
                shmr_amd.set_tuning(**{"decode.sc1_store": -2, "decode.nt_store": -2, "decode.peel": -2})
        assert all(np.array_equal(outs[0], o) for o in outs[1:])


def test_compact_validation(gpu):
    """The shim checks the output tensor before the raw-pointer call; the
    library validates the presence flags before any launch."""
    import torch
    rs = shmr_amd.ReedSolomon(4, 2)
    shards = torch.zeros((3, 6, 1024), dtype=torch.uint8, device=gpu)
    present = np.ones((3, 6), np.uint8)
    present[:, [0, 5]] = 0
    with pytest.raises(shmr_amd.Error) as e:                   # one row, two rebuilt shards per block
        rs.reconstruct_batch_dev_out(shards, present, torch.zeros((3, 1, 1024), dtype=torch.uint8, device=gpu))
    assert e.value.name == "TooFewShards"
    with pytest.raises(TypeError):
        rs.reconstruct_batch_dev_out(shards, present, torch.zeros((2, 2, 1024), dtype=torch.uint8, device=gpu))
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct_batch_dev_out(shards, present, torch.zeros((3, 2, 1000), dtype=torch.uint8, device=gpu))
    assert e.value.name == "IncorrectShardSize"
    present[1, :3] = 0                                          # 5 absent of 6: too few present
    out = torch.full((3, 5, 1024), GUARD, dtype=torch.uint8, device=gpu)
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct_batch_dev_out(shards, present, out)
    assert e.value.name == "TooFewShardsPresent"
    torch.cuda.synchronize()
    assert (out.cpu().numpy() == GUARD).all()                  # nothing launched
    # data_only: only the absent data shard is rebuilt (one row suffices)
    present = np.ones((3, 6), np.uint8)
    present[:, [1, 4]] = 0
    rs.reconstruct_batch_dev_out(shards, present, torch.zeros((3, 1, 1024), dtype=torch.uint8, device=gpu),
                                 data_only=True)
