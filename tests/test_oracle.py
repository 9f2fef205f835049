"""CPU tests of the oracle itself: pinned to the crate's published KATs, the
numpy and C restatements agree, and the committed fixtures reproduce.

The reference (volfco/shmr) holds no erasure test vectors (its only
"erasure" test, src/vfs/block.rs:799-817, builds a Single block), so the
pins are the upstream crate's published known answers (tests/golden/kat.json
"published") plus this repo's own regression vectors.
"""
import hashlib
import itertools
import json
import os

import numpy as np
import pytest

from oracle import c_oracle
from oracle import rs_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
KAT = json.load(open(os.path.join(GOLDEN, "kat.json")))
SMALL = np.load(os.path.join(GOLDEN, "small_vectors.npz"))   # allow_pickle=False (default)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ---------------------------------------------------------------- published KATs
@pytest.mark.parametrize("a,b,c", KAT["published"]["gal_mul"])
def test_gal_mul_kat(a, b, c):
    assert O.gal_mul(a, b) == c
    assert c_oracle.lib().oracle_gal_mul(a, b) == c


@pytest.mark.parametrize("a,n,c", KAT["published"]["gal_exp"])
def test_gal_exp_kat(a, n, c):
    assert O.gal_exp(a, n) == c
    assert c_oracle.lib().oracle_gal_exp(a, n) == c


def test_encode_kat():
    for case in KAT["published"]["encode"]:
        k, p = case["data_shards"], case["parity_shards"]
        sh = [np.array(d, np.uint8) for d in case["data"]] + [np.zeros(2, np.uint8) for _ in range(p)]
        O.ReedSolomon(k, p).encode(sh)
        assert [s.tolist() for s in sh[k:]] == case["parity"]
        sh2 = [np.array(d, np.uint8) for d in case["data"]] + [np.zeros(2, np.uint8) for _ in range(p)]
        c_oracle.encode(k, p, sh2, variant=0)
        assert [s.tolist() for s in sh2[k:]] == case["parity"]


@pytest.mark.parametrize("c,inp,want", KAT["published"]["mul_slice"])
def test_mul_slice_kat(c, inp, want):
    x = np.array(inp, np.uint8)
    out = np.zeros_like(x)
    O.mul_slice(c, x, out)
    assert out.tolist() == want
    acc = np.array(want, np.uint8)          # mul_slice_xor onto its own product -> zeros
    O.mul_slice_xor(c, x, acc)
    assert not acc.any()
    for variant in (0, 1):                  # scalar table loop and the AVX2 nibble loop (+ byte tail)
        assert c_oracle.apply(np.array([[c]], np.uint8), [x], len(x), variant=variant)[0].tolist() == want


@pytest.mark.parametrize("c,inp,want", KAT["published"]["mul_slice_full"])
def test_mul_slice_full_upstream_vector(c, inp, want):
    """All 34 inputs of the upstream mul_slice(25) vector, each byte checked
    on its own (so a failure names the input)."""
    for x, y in zip(inp, want):
        assert O.gal_mul(c, x) == y, (c, x)
    got = np.zeros(len(inp), np.uint8)
    O.mul_slice(c, np.array(inp, np.uint8), got)
    assert list(got) == want


def test_published_kats_name_their_source():
    pub = KAT["published"]
    for key in ("gal_mul", "gal_exp", "mul_slice", "mul_slice_full", "encode", "mat_mul", "mat_invert"):
        assert key in pub and pub["sources"][key], key


@pytest.mark.parametrize("a,b,want", KAT["published"]["mat_mul"])
def test_mat_mul_kat(a, b, want):
    assert O.mat_mul(np.array(a, np.uint8), np.array(b, np.uint8)).tolist() == want


@pytest.mark.parametrize("m,want", KAT["published"]["mat_invert"])
def test_mat_invert_kat(m, want):
    m = np.array(m, np.uint8)
    assert O.mat_invert(m).tolist() == want
    assert c_oracle.invert(m).tolist() == want


# ---------------------------------------------------------------- field properties
def test_field_axioms():
    m = O.MUL_TABLE.astype(np.int64)
    assert (m[1] == np.arange(256)).all()
    assert (m == m.T).all()                                 # commutative
    for a in range(1, 256):                                 # every non-zero has an inverse
        assert O.gal_mul(a, O.gal_div(1, a)) == 1
    rng = np.random.default_rng(0)
    for a, b, c in rng.integers(0, 256, (200, 3)):          # distributive over XOR
        assert O.gal_mul(a, b ^ c) == O.gal_mul(a, b) ^ O.gal_mul(a, c)
    assert len(set(O.EXP_TABLE[:255].tolist())) == 255      # 2 generates GF(2^8)*


def test_tables_pinned():
    t = KAT["build_pins"]["tables"]
    assert sha(O.LOG_TABLE) == t["log_sha256"]
    assert sha(O.EXP_TABLE) == t["exp_sha256"]
    assert sha(O.MUL_TABLE) == t["mul_sha256"]


def test_nibble_tables_match_full_table():
    for c in range(256):
        for x in range(256):
            assert O.MUL_TABLE_LOW[c][x & 15] ^ O.MUL_TABLE_HIGH[c][x >> 4] == O.MUL_TABLE[c][x]


def test_three_table_split_matches_full_table():
    """The kernel's v_perm decomposition: c(x)b = T0[b&7] ^ T1[(b>>3)&7] ^ T2[b>>6]."""
    for c in range(256):
        t0 = [O.gal_mul(c, x) for x in range(8)]
        t1 = [O.gal_mul(c, x << 3) for x in range(8)]
        t2 = [O.gal_mul(c, x << 6) for x in range(4)]
        for b in range(256):
            assert t0[b & 7] ^ t1[(b >> 3) & 7] ^ t2[b >> 6] == O.gal_mul(c, b)


# ---------------------------------------------------------------- matrices
@pytest.mark.parametrize("k,p", [(1, 1), (2, 1), (4, 2), (8, 3), (10, 4), (5, 5), (17, 3), (100, 100), (255, 1), (1, 255)])
def test_matrix_numpy_equals_c(k, p):
    assert (O.build_matrix(k, k + p) == c_oracle.build_matrix(k, p)).all()


@pytest.mark.parametrize("kp", list(KAT["build_pins"]["parity_rows"]))
def test_parity_rows_pinned(kp):
    k, p = map(int, kp.split(","))
    assert O.ReedSolomon(k, p).parity_rows().tolist() == KAT["build_pins"]["parity_rows"][kp]


@pytest.mark.parametrize("k,p", [(4, 2), (8, 3), (10, 4), (5, 5)])
def test_matrix_systematic_and_mds(k, p):
    m = O.build_matrix(k, k + p)
    assert (m[:k] == np.eye(k, dtype=np.uint8)).all()
    for rows in itertools.combinations(range(k + p), k):   # every k rows invertible (MDS)
        inv = O.mat_invert(m[list(rows)])
        assert (O.mat_mul(inv, m[list(rows)]) == np.eye(k, dtype=np.uint8)).all()


def test_new_errors():
    for (k, p), name in [((0, 1), "TooFewDataShards"), ((1, 0), "TooFewParityShards"),
                         ((200, 57), "TooManyShards"), ((0, 0), "TooFewDataShards")]:
        with pytest.raises(O.RSError) as e:
            O.ReedSolomon(k, p)
        assert e.value.name == name
    assert c_oracle.lib().oracle_build_matrix(0, 1, c_oracle._ptr(np.zeros(1, np.uint8))) == -3


def test_encode_errors():
    r = O.ReedSolomon(3, 2)
    with pytest.raises(O.RSError) as e:
        r.encode([np.zeros(4, np.uint8)] * 4)
    assert e.value.name == "TooFewShards"
    with pytest.raises(O.RSError) as e:
        r.encode([np.zeros(4, np.uint8)] * 6)
    assert e.value.name == "TooManyShards"
    with pytest.raises(O.RSError) as e:
        r.encode([np.zeros(0, np.uint8)] * 5)
    assert e.value.name == "EmptyShard"
    with pytest.raises(O.RSError) as e:
        r.encode([np.zeros(4, np.uint8)] * 4 + [np.zeros(5, np.uint8)])
    assert e.value.name == "IncorrectShardSize"


def test_reconstruct_errors_and_noop():
    r = O.ReedSolomon(3, 2)
    full = [np.arange(4, dtype=np.uint8) + i for i in range(5)]
    same = [x.copy() for x in full]
    r.reconstruct(same)                                   # all present: no-op
    assert all((a == b).all() for a, b in zip(same, full))
    with pytest.raises(O.RSError) as e:
        r.reconstruct([full[0], None, None, None, full[4]])
    assert e.value.name == "TooFewShardsPresent"
    with pytest.raises(O.RSError) as e:
        r.reconstruct([full[0], np.zeros(3, np.uint8), None, full[3], full[4]])
    assert e.value.name == "IncorrectShardSize"
    with pytest.raises(O.RSError) as e:
        r.reconstruct([np.zeros(0, np.uint8), None, full[2], full[3], full[4]])
    assert e.value.name == "EmptyShard"


def test_decode_matrix_lru():
    r = O.ReedSolomon(4, 2)
    full = [np.arange(16, dtype=np.uint8) * (i + 1) for i in range(4)] + [np.zeros(16, np.uint8)] * 2
    full = [x.copy() for x in full]
    r.encode(full)
    for _ in range(3):
        got = [None] + [x.copy() for x in full[1:]]
        r.reconstruct(got)
        assert (got[0] == full[0]).all()
    assert len(r._cache) == 1


# ---------------------------------------------------------------- numpy vs C oracle
@pytest.mark.parametrize("k,p,L", [(8, 3, 1000), (10, 4, 4099), (4, 2, 7), (1, 1, 33), (20, 5, 65)])
@pytest.mark.parametrize("variant", [0, 1])
def test_encode_numpy_equals_c(k, p, L, variant):
    rng = np.random.default_rng([k, p, L])
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    a = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(p)]
    b = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(p)]
    O.ReedSolomon(k, p).encode(a)
    c_oracle.encode(k, p, b, variant=variant)
    assert all((x == y).all() for x, y in zip(a, b))


def test_reconstruct_numpy_equals_c_all_patterns():
    k, p, L = 4, 3, 33
    rng = np.random.default_rng(3)
    shards = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k + p)]   # not a codeword
    for n in (1, 2, 3):
        for miss in itertools.combinations(range(k + p), n):
            for data_only in (False, True):
                a = [None if i in miss else shards[i].copy() for i in range(k + p)]
                (O.ReedSolomon(k, p).reconstruct_data if data_only else O.ReedSolomon(k, p).reconstruct)(a)
                b = c_oracle.reconstruct(k, p, [None if i in miss else shards[i].copy() for i in range(k + p)],
                                         L, data_only=data_only)
                for i in range(k + p):
                    if a[i] is not None:
                        assert (a[i] == b[i]).all(), (miss, data_only, i)


# ---------------------------------------------------------------- committed vectors
def test_small_vectors_reproduce():
    for key in SMALL.files:
        if not key.startswith("enc_") or not key.endswith("_data"):
            continue
        _, k, p, L, _ = key.split("_")
        k, p = int(k), int(p)
        data = SMALL[key]
        sh = [d.copy() for d in data] + [np.zeros(int(L), np.uint8) for _ in range(p)]
        O.ReedSolomon(k, p).encode(sh)
        assert (np.stack(sh[k:]) == SMALL[key.replace("_data", "_parity")]).all()


def test_reconstruct_vectors_reproduce():
    shards = SMALL["rec_4_3_shards"]
    for miss, want in zip(SMALL["rec_4_3_missing"], SMALL["rec_4_3_result"]):
        miss = [int(i) for i in miss if i >= 0]
        got = [None if i in miss else shards[i].copy() for i in range(7)]
        O.ReedSolomon(4, 3).reconstruct(got)
        assert (np.stack(got) == want).all()


@pytest.mark.parametrize("case", [c for c in KAT["large"] if c.get("case") is None][:2])
def test_large_vectors_reproduce(case):
    buf = O.seeded_block(*case["seed"], case["block_bytes"])
    shards = O.sync_data_erasure(buf.tobytes(), case["block_bytes"], case["k"], case["p"])
    assert [sha(s) for s in shards] == case["shard_sha256"]


def test_edge_blocks_reproduce():
    for case in KAT["large"]:
        if case.get("case") is None:
            continue
        if case["case"] == "zeros":
            buf = np.zeros(case["buffer_len"], np.uint8)
        elif case["case"] == "ones":
            buf = np.full(case["buffer_len"], 0xFF, np.uint8)
        else:
            buf = O.seeded_block(*case["seed"], case["buffer_len"])
        shards = O.sync_data_erasure(buf.tobytes(), case["block_bytes"], case["k"], case["p"])
        assert [sha(s) for s in shards] == case["shard_sha256"], case["case"]


# ---------------------------------------------------------------- shmr glue
@pytest.mark.parametrize("length,k,want", KAT["build_pins"]["shard_size"])
def test_calculate_shard_size_pins(length, k, want):
    assert O.calculate_shard_size(length, k) == want


def test_f32_hazard_documented():
    """src/vfs/mod.rs:16-18 uses f32: for sizes past 2^24 the shard size can be
    one short, so buffer.chunks(S) yields k + 1 chunks."""
    assert O.calculate_shard_size(16777217, 8) * 8 < 16777217
    buf = np.zeros(16777217, np.uint8).tobytes()
    with pytest.raises(O.RSError) as e:                     # the mirror's default
        O.sync_data_erasure(buf, 16777217, 8, 3, mode="refuse")
    assert e.value.name == "TooManyDataShards"
    with pytest.raises(O.ReferencePanic):                   # debug build: overflow check
        O.sync_data_erasure(buf, 16777217, 8, 3, mode="debug")
    with pytest.raises(ValueError):
        O.sync_data_erasure(buf, 16777217, 8, 3, mode="fast")


def test_f32_hazard_release_semantics():
    """block.rs:421 in the reference's release build (Cargo.toml:10-13, no
    overflow checks): 9 chunks of S = 2,097,152 for a 16,777,217 B buffer at
    Erasure(1,8,3); `3 + (8 - 9 as u8)` wraps to 2 zero shards, so encode sees
    k+p = 11 shards and succeeds, overwriting chunk 8 (the buffer's last byte)
    with parity row 0.  A later load_block returns that parity byte as the
    block's last byte (concat of all k+p shards, [..size], block.rs:567-576)."""
    size, k, p = 16777217, 8, 3
    S = O.calculate_shard_size(size, k)
    buf = O.seeded_block(O.BENCH_SEED, 9, size)
    shards = O.sync_data_erasure(buf.tobytes(), size, k, p)           # release is the default
    assert len(shards) == k + p and all(len(s) == S for s in shards)
    for i in range(k):
        assert np.array_equal(shards[i], buf[i * S:(i + 1) * S])
    assert O.ReedSolomon(k, p).verify(shards)
    case = KAT["f32_hazard_release"]
    assert case["block_bytes"] == size and case["shard_bytes"] == S
    assert [sha(s) for s in shards] == case["shard_sha256"]
    loaded = O.load_block_erasure([s.tobytes() for s in shards], size, k, p)
    assert len(loaded) == size and np.array_equal(loaded[:k * S], buf[:k * S])
    assert loaded[k * S] == shards[k][0]                               # parity, not buf[k*S]
    assert sha(loaded) == case["load_block_sha256"]


def test_sync_data_partial_buffer_layout():
    """block.rs:408-423: a 700,001 B buffer in a 1 MiB RS(4,2) block gives 3 data
    chunks (the last zero-padded), one all-zero data shard and 2 parity."""
    buf = O.seeded_block(O.BENCH_SEED, 7, 700001)
    shards = O.sync_data_erasure(buf.tobytes(), 1 << 20, 4, 2)
    S = 262144
    assert len(shards) == 6 and all(len(s) == S for s in shards)
    assert (shards[0] == buf[:S]).all() and (shards[2][:700001 - 2 * S] == buf[2 * S:]).all()
    assert not shards[2][700001 - 2 * S:].any() and not shards[3].any()
    assert O.sync_data_erasure(b"", 1 << 20, 4, 2) == []       # block.rs:389-391


def test_load_block_quirks():
    case = KAT["load_block"]
    k, p, size = 4, 2, 4096
    buf = O.seeded_block(O.BENCH_SEED, 42, size)
    shards = O.sync_data_erasure(buf.tobytes(), size, k, p)
    s1 = [bytes(x) for x in shards]
    s1[1] = None
    assert sha(O.load_block_erasure(s1, size, k, p)) == case["read_error_data1"] == case["original"]
    s2 = [bytes(x) for x in shards]
    s2[2] = s2[2][:100]
    got = O.load_block_erasure(s2, size, k, p)
    assert sha(got) == case["truncated_data2"] != case["original"]   # zero padding survives (block.rs:548-551)


def test_reconstruct_batch_matches_single_block():
    """Threaded AVX2 batch reconstruct (the decode CPU baseline) == the
    single-block oracle (scalar), mixed patterns incl. data_only."""
    k, p, S, B = 8, 3, 4096 + 7, 9
    rng = np.random.default_rng(77)
    data = rng.integers(0, 256, (B, k + p, S), dtype=np.uint8)
    for b in range(B):
        sh = [data[b, i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
        c_oracle.encode(k, p, sh)
        data[b, k:] = np.stack(sh[k:])
    full = data.copy()
    present = np.ones((B, k + p), np.uint8)
    for b in range(B):
        present[b, rng.choice(k + p, size=int(rng.integers(0, p + 1)), replace=False)] = 0
    for data_only in (False, True):
        work = full.copy()
        work[present == 0] = 0
        assert c_oracle.reconstruct_batch(k, p, work, present, S, 4, data_only=data_only) >= 0
        for b in range(B):
            for i in range(k + p):
                if data_only and i >= k and not present[b, i]:
                    assert not work[b, i].any()
                else:
                    assert np.array_equal(work[b, i], full[b, i]), (b, i, data_only)


@pytest.mark.parametrize("size", [1 << 20, 700_001, 8 * 4096 - 100])
def test_sync_data_batch_matches_restatement(size):
    """Threaded sync_data-minus-disk baseline (block.rs:406-430) == the
    numpy restatement of the Erasure arm, parity for parity."""
    k, p, B = 4, 2, 5
    S = O.calculate_shard_size(1 << 20, k) if size == 700_001 else O.calculate_shard_size(size, k)
    rng = np.random.default_rng(size)
    src = rng.integers(0, 256, B * size, dtype=np.uint8)
    par = np.zeros(B * p * S, np.uint8)
    c_oracle.sync_data_batch(k, p, src, size, S, par, B, 3)
    block = 1 << 20 if size == 700_001 else size
    for b in range(B):
        want = O.sync_data_erasure(src[b * size:(b + 1) * size].tobytes(), block, k, p)
        for r in range(p):
            assert np.array_equal(par[(b * p + r) * S:(b * p + r + 1) * S], want[k + r])
