"""The Rust binding written out in INTEGRATION.md §1 against include/shmr_ec.h.

There is no Rust toolchain in this image, so the binding a shmr maintainer
would add (replacing `reed_solomon_erasure::galois_8::ReedSolomon`,
reference `src/vfs/block.rs:10`) cannot be compiled here.  These CPU tests
keep it from drifting away from the C ABI it binds: every `extern "C"`
function it declares exists in the header with the same number and kind of
parameters and the same return kind, and its status-code mapping is the
header's enum (1:1 with the crate's `Error` variants, `config.rs:158,170-174`).
"""
from __future__ import annotations

import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _read(rel):
    with open(os.path.join(ROOT, rel)) as f:
        return f.read()


def _rust_blocks():
    doc = _read("INTEGRATION.md")
    return re.findall(r"```rust\n(.*?)```", doc, re.S)


def _rust_externs():
    """name -> (param types, return type) for every fn in an extern "C" block."""
    out = {}
    for block in _rust_blocks():
        for body in re.findall(r'extern "C" \{(.*?)\n?\}', block, re.S):
            for m in re.finditer(r"fn\s+(\w+)\s*\((.*?)\)\s*(?:->\s*([\w:*\s]+?))?\s*;", body, re.S):
                name, params, ret = m.group(1), m.group(2), (m.group(3) or "").strip()
                types = [p.split(":", 1)[1].strip() for p in params.split(",") if p.strip()]
                out[name] = (types, ret)
    return out


def _header_decls():
    """name -> (param types, return type) for every function the header declares."""
    hdr = _read("include/shmr_ec.h")
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    out = {}
    for m in re.finditer(r"^([\w\s\*]+?)\b(shmr_ec_\w+)\s*\(([^;]*?)\)\s*;", hdr, re.S | re.M):
        ret, name, params = m.group(1).strip(), m.group(2), m.group(3).strip()
        types = [] if params in ("", "void") else [" ".join(p.split()[:-1]) + ("*" * p.split()[-1].count("*"))
                                                  for p in (q.strip() for q in params.split(","))]
        out[name] = (types, ret)
    return out


def _kind_c(t):
    t = t.replace(" ", "")
    if "*" in t:
        return "ptr"
    return {"uint32_t": "u32", "int": "i32", "size_t": "usize", "uint64_t": "u64", "void": "", "constchar": "ptr"}[t]


def _kind_rust(t):
    t = t.replace(" ", "")
    if t.startswith("*"):
        return "ptr"
    return {"u32": "u32", "c_int": "i32", "usize": "usize", "u64": "u64", "": ""}[t]


def test_rust_binding_present():
    ext = _rust_externs()
    for name in ("shmr_ec_new", "shmr_ec_free", "shmr_ec_encode", "shmr_ec_reconstruct",
                 "shmr_ec_data_shard_count"):
        assert name in ext, name


def test_rust_externs_match_header():
    ext, hdr = _rust_externs(), _header_decls()
    assert len(hdr) > 20            # the parser saw the whole header
    for name, (rtypes, rret) in ext.items():
        assert name in hdr, f"{name} bound in INTEGRATION.md but not declared in include/shmr_ec.h"
        ctypes_, cret = hdr[name]
        assert [_kind_rust(t) for t in rtypes] == [_kind_c(t) for t in ctypes_], name
        assert _kind_rust(rret) == _kind_c(cret), name


def test_rust_status_mapping_matches_header_enum():
    hdr = _read("include/shmr_ec.h")
    enum = {name: int(v) for name, v in re.findall(r"SHMR_EC_(\w+)\s*=\s*(-?\d+)", hdr)}
    code = "\n".join(_rust_blocks())
    arms = dict((int(c), v) for c, v in re.findall(r"(-\d+)\s*=>\s*(\w+)", code))
    crate = {k: v for k, v in enum.items() if -13 <= v <= -1}
    assert len(crate) == 13
    for name, v in crate.items():
        # SHMR_EC_TOO_FEW_DATA_SHARDS <-> TooFewDataShards
        camel = "".join(w.capitalize() for w in name.lower().split("_"))
        assert arms.get(v) == camel, (v, name, arms.get(v))
    # device / host conditions (< -13) fall through to Device(code)
    assert re.search(r"other\s*=>\s*Device\(other\)", code)
