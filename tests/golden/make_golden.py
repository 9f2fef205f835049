#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/.

Two kinds of data, kept apart on purpose:

* kat.json "published" -- known-answer values of the crate the reference calls
  (reed-solomon-erasure 6.0.0, itself a port of Backblaze JavaReedSolomon):
  galois multiply/exp/slice-multiply KATs, the matrix multiply/invert tests
  and the RS(5,5) encode vector.  These pin the
  oracle to the upstream algorithm; they are data, not code.
* everything else -- produced by this repo's CPU oracle (oracle/rs_oracle.py)
  from seeded inputs: parity rows of the BASELINE configs, small blocks in full
  bytes, benchmark-sized blocks as SHA-256 per shard, shmr glue cases
  (calculate_shard_size f32 edges, sync_data partial buffers, load_block
  quirks).  These are the build's own pins (regression vectors).

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import rs_oracle as O  # noqa: E402

SEED = O.BENCH_SEED


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


_SLICE_IN = [0, 1, 2, 3, 4, 5, 6, 10, 50, 100, 150, 174, 201, 255, 99, 32, 67, 85]


def published_kats():
    return {
        "source": "reed-solomon-erasure 6.0.0 galois_8 tests / Backblaze JavaReedSolomon (published KATs)",
        "gal_mul": [[3, 4, 12], [7, 7, 21], [23, 45, 41]],
        "gal_exp": [[2, 2, 4], [5, 20, 235], [13, 7, 43]],
        "encode": [{"data_shards": 5, "parity_shards": 5,
                    "data": [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]],
                    "parity": [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]}],
        # galois slice multiply (upstream test_slice_mul / galMulSlice): [c, in, expected]
        "mul_slice": [
            [25, _SLICE_IN, [0x00, 0x19, 0x32, 0x2b, 0x64, 0x7d, 0x56, 0xfa, 0xb8, 0x6d, 0xc7, 0x85, 0xc3,
                             0x1f, 0x22, 0x07, 0x25, 0xfe]],
            [177, _SLICE_IN, [0x00, 0xb1, 0x7f, 0xce, 0xfe, 0x4f, 0x81, 0x9e, 0x03, 0x06, 0xe8, 0x75, 0xbd,
                              0x40, 0x36, 0xa3, 0x95, 0xcb]],
        ],
        # matrix tests (upstream MatrixTest / matrix.rs tests): [a, b, a*b] and [m, inv(m)]
        "mat_mul": [[[[1, 2], [3, 4]], [[5, 6], [7, 8]], [[11, 22], [19, 42]]]],
        "mat_invert": [
            [[[56, 23, 98], [3, 100, 200], [45, 201, 123]], [[175, 133, 33], [130, 13, 245], [112, 35, 126]]],
            [[[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [0, 0, 0, 1, 0], [0, 0, 0, 0, 1], [7, 7, 6, 6, 1]],
             [[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [123, 123, 1, 122, 122], [0, 0, 1, 0, 0], [0, 0, 0, 1, 0]]],
        ],
    }


def build_pins():
    pins = {"parity_rows": {}, "shard_size": [], "tables": {}}
    for k, p in [(4, 2), (8, 3), (10, 4), (5, 5), (1, 1), (2, 1), (17, 3), (200, 56)]:
        pins["parity_rows"][f"{k},{p}"] = O.ReedSolomon(k, p).parity_rows().tolist()
    for length, k in [(1 << 20, 4), (4 << 20, 8), (16 << 20, 10), (7000, 4), (16777217, 8), (16777221, 10),
                      (16777216, 3), (1, 7), (0, 3), (33554433, 16), (100, 3)]:
        pins["shard_size"].append([length, k, O.calculate_shard_size(length, k)])
    pins["tables"] = {"log_sha256": sha(O.LOG_TABLE), "exp_sha256": sha(O.EXP_TABLE),
                      "mul_sha256": sha(O.MUL_TABLE)}
    return pins


def small_vectors():
    """Full-byte vectors, small enough to commit as .npz."""
    out = {}
    cases = [(4, 2, 1024), (8, 3, 777), (10, 4, 1000), (3, 3, 17), (1, 1, 5), (6, 2, 4096 + 3)]
    for ci, (k, p, L) in enumerate(cases):
        rng = np.random.default_rng([SEED, 1000 + ci])
        data = rng.integers(0, 256, (k, L), dtype=np.uint8)
        sh = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(p)]
        O.ReedSolomon(k, p).encode(sh)
        out[f"enc_{k}_{p}_{L}_data"] = data
        out[f"enc_{k}_{p}_{L}_parity"] = np.stack(sh[k:])
    # reconstruct vectors: inconsistent (random) shards exercise the crate's
    # "first k present + re-encode parity" rule
    k, p, L = 4, 3, 64
    rng = np.random.default_rng([SEED, 2000])
    shards = rng.integers(0, 256, (k + p, L), dtype=np.uint8)
    out["rec_4_3_shards"] = shards
    pats = [[0], [6], [0, 4], [1, 2, 3], [3, 5, 6], [0, 1, 2]]
    results = []
    for miss in pats:
        got = [None if i in miss else shards[i].copy() for i in range(k + p)]
        O.ReedSolomon(k, p).reconstruct(got)
        results.append(np.stack(got))
    out["rec_4_3_missing"] = np.array([m + [-1] * (3 - len(m)) for m in pats], dtype=np.int16)
    out["rec_4_3_result"] = np.stack(results)
    return out


def large_vectors():
    """Benchmark-sized blocks as SHA-256 per shard (inputs regenerated from seed)."""
    out = []
    for k, p, size, idx in [(4, 2, 1 << 20, 0), (8, 3, 4 << 20, 0), (8, 3, 4 << 20, 1), (10, 4, 16 << 20, 0)]:
        S = O.calculate_shard_size(size, k)
        buf = O.seeded_block(SEED, idx, size)
        shards = O.sync_data_erasure(buf.tobytes(), size, k, p)
        out.append({"k": k, "p": p, "block_bytes": size, "seed": [SEED, idx], "shard_bytes": S,
                    "generator": "numpy.random.default_rng([seed, idx]).integers(0, 256, block_bytes, uint8)",
                    "shard_sha256": [sha(s) for s in shards]})
    # edge blocks: all-0x00, all-0xFF, partial buffer 700,001 B
    for name, buf in [("zeros", np.zeros(1 << 20, np.uint8)), ("ones", np.full(1 << 20, 0xFF, np.uint8)),
                      ("partial_700001", O.seeded_block(SEED, 7, 700001))]:
        shards = O.sync_data_erasure(buf.tobytes(), 1 << 20, 4, 2)
        out.append({"k": 4, "p": 2, "block_bytes": 1 << 20, "case": name, "buffer_len": int(buf.size),
                    "seed": [SEED, 7] if name.startswith("partial") else None,
                    "shard_sha256": [sha(s) for s in shards]})
    return out


def f32_hazard_release():
    """block.rs:421's u8 wrap in the reference's release build: a full
    16,777,217 B Erasure(1,8,3) buffer (9 chunks of S = 2,097,152) encodes
    into k+p shards with chunk 8 overwritten by parity row 0
    (oracle sync_data_erasure, mode="release")."""
    size, k, p = 16777217, 8, 3
    buf = O.seeded_block(SEED, 9, size)
    shards = O.sync_data_erasure(buf.tobytes(), size, k, p, mode="release")
    loaded = O.load_block_erasure([s.tobytes() for s in shards], size, k, p)
    return {"k": k, "p": p, "block_bytes": size, "buffer_len": size, "seed": [SEED, 9],
            "shard_bytes": O.calculate_shard_size(size, k),
            "generator": "numpy.random.default_rng([seed, idx]).integers(0, 256, block_bytes, uint8)",
            "shard_sha256": [sha(s) for s in shards], "load_block_sha256": sha(loaded),
            "lost_byte_offset": k * O.calculate_shard_size(size, k), "lost_byte": int(buf[-1]),
            "loaded_last_byte": int(loaded[-1])}


def glue_cases():
    """load_block quirks (src/vfs/block.rs:529-579)."""
    k, p, size = 4, 2, 4096
    buf = O.seeded_block(SEED, 42, size)
    shards = O.sync_data_erasure(buf.tobytes(), size, k, p)
    cases = {}
    # a read error on data shard 1 -> None -> reconstructed
    s1 = [bytes(x) for x in shards]
    s1[1] = None
    cases["read_error_data1"] = sha(O.load_block_erasure(s1, size, k, p))
    # a truncated shard is zero-padded and stays "present" -> reconstruct is a
    # no-op when every shard is Some, so the zero padding survives
    s2 = [bytes(x) for x in shards]
    s2[2] = s2[2][:100]
    cases["truncated_data2"] = sha(O.load_block_erasure(s2, size, k, p))
    cases["intact"] = sha(O.load_block_erasure([bytes(x) for x in shards], size, k, p))
    cases["original"] = sha(buf)
    return cases


def main():
    kat = {"published": published_kats(), "build_pins": build_pins(), "large": large_vectors(),
           "load_block": glue_cases(), "f32_hazard_release": f32_hazard_release()}
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "small_vectors.npz"), **small_vectors())
    print("wrote", os.path.join(HERE, "kat.json"), "and small_vectors.npz")


if __name__ == "__main__":
    main()
