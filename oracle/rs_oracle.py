"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.

This module is the *checker* for the MI355X erasure path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``shmr_amd``) never calls it and has no CPU fallback.

What it restates
----------------
The reference (volfco/shmr @ 2024-08-07) delegates all erasure arithmetic to
the third-party Rust crate ``reed-solomon-erasure`` **6.0.0**
(``Cargo.toml:16`` with ``features=["simd-accel"]``; ``Cargo.lock:1577-1589``,
checksum 7263373d500d4d4f505d43a2a662d475a894aa94503a1ee28e9188b5f3960d4f).
The crate is not vendored and cannot be built here (no cargo/rustc, no
network), so this file restates its published algorithm:

* GF(2^8) with generating polynomial 29 (x^8+x^4+x^3+x^2+1, i.e. 0x11D) and
  generator 2: crate ``build.rs`` log/exp/mul tables, ``galois_8::{mul, div,
  exp}``.
* ``ReedSolomon::new(k, p)``: encoding matrix M = V * inv(V[0..k]) where
  V[r][c] = exp(r, c) (so 0^0 = 1), (k+p) x k, systematic.
  Errors: k == 0 -> TooFewDataShards, p == 0 -> TooFewParityShards,
  k + p > 256 -> TooManyShards.
* ``encode``: parity[r] = XOR_i M[k+r][i] (x) data[i]; loop order outer over
  input shards, inner over parity rows (``mul_slice`` at i == 0 then
  ``mul_slice_xor``).  Checks: shard count == k+p, equal non-zero lengths.
* ``reconstruct`` / ``reconstruct_data``: first k present shards in index order
  form the sub-matrix; its inverse (LRU-cached, keyed by the absent indices)
  rebuilds absent data shards; absent parity shards are then re-encoded from
  the full data unless ``data_only``.

and the shmr glue that calls it:

* ``calculate_shard_size`` -- ``src/vfs/mod.rs:16-18`` (f32 ceil).
* ``VirtualBlock::sync_data`` Erasure arm -- ``src/vfs/block.rs:404-440``
  (chunks(S), zero pad, zero shards appended, encode).
* ``VirtualBlock::load_block`` Erasure arm -- ``src/vfs/block.rs:529-579``
  (read flags, reconstruct trigger, concat, ``[..size]``).

Parity pinning: the reference's own tests never exercise encode/reconstruct
(SURVEY.md section 4/8c), so this oracle is pinned against the crate's published
known-answer tests (``tests/golden/kat.json``), see tests/test_oracle.py.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Optional, Sequence

import numpy as np

FIELD_SIZE = 256
GENERATING_POLYNOMIAL = 29          # crate build.rs constant (0x11D without x^8)
DATA_DECODE_MATRIX_CACHE_CAPACITY = 254


# ----------------------------------------------------------------------------
# Errors: 1:1 with reed_solomon_erasure::Error (the variants shmr can hit,
# mapped into ShmrError::EcError at src/config.rs:158,170-174).
# ----------------------------------------------------------------------------
class RSError(Exception):
    def __init__(self, name: str):
        super().__init__(name)
        self.name = name


def _err(name):
    raise RSError(name)


# ----------------------------------------------------------------------------
# Field tables (crate build.rs: gen_log_table / gen_exp_table / gen_mul_table)
# ----------------------------------------------------------------------------
def _gen_log_table(poly: int) -> np.ndarray:
    log = np.zeros(FIELD_SIZE, dtype=np.uint8)
    b = 1
    for lg in range(FIELD_SIZE - 1):
        log[b] = lg
        b <<= 1
        if b >= FIELD_SIZE:
            b = (b - FIELD_SIZE) ^ poly
    return log


def _gen_exp_table(log: np.ndarray) -> np.ndarray:
    exp = np.zeros(FIELD_SIZE * 2 - 2, dtype=np.uint8)
    for i in range(1, FIELD_SIZE):
        lg = int(log[i])
        exp[lg] = i
        exp[lg + FIELD_SIZE - 1] = i
    return exp


LOG_TABLE = _gen_log_table(GENERATING_POLYNOMIAL)
EXP_TABLE = _gen_exp_table(LOG_TABLE)


def _gen_mul_table() -> np.ndarray:
    a = np.arange(256)[:, None]
    b = np.arange(256)[None, :]
    s = LOG_TABLE[a].astype(np.int64) + LOG_TABLE[b].astype(np.int64)
    t = EXP_TABLE[s]
    t[(a == 0) | (b == 0)] = 0
    return t.astype(np.uint8)


MUL_TABLE = _gen_mul_table()                       # [256][256]
MUL_TABLE_LOW = MUL_TABLE[:, :16].copy()           # c (x) n        (pshufb table)
MUL_TABLE_HIGH = MUL_TABLE[:, ::16].copy()         # c (x) (n << 4) (pshufb table)


def gal_add(a: int, b: int) -> int:
    return a ^ b


def gal_mul(a: int, b: int) -> int:
    return int(MUL_TABLE[a, b])


def gal_div(a: int, b: int) -> int:
    if a == 0:
        return 0
    if b == 0:
        raise ZeroDivisionError("Divisor is 0")
    lr = int(LOG_TABLE[a]) - int(LOG_TABLE[b])
    if lr < 0:
        lr += 255
    return int(EXP_TABLE[lr])


def gal_exp(a: int, n: int) -> int:
    if n == 0:
        return 1
    if a == 0:
        return 0
    lr = int(LOG_TABLE[a]) * n
    while lr >= 255:
        lr -= 255
    return int(EXP_TABLE[lr])


# ----------------------------------------------------------------------------
# Matrices over GF(2^8) (crate matrix.rs semantics; inverse is unique, so the
# elimination order does not affect results).
# ----------------------------------------------------------------------------
def mat_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    rows, inner = a.shape
    inner2, cols = b.shape
    assert inner == inner2
    out = np.zeros((rows, cols), dtype=np.uint8)
    for r in range(rows):
        acc = np.zeros(cols, dtype=np.uint8)
        for i in range(inner):
            acc ^= MUL_TABLE[a[r, i], b[i, :]]
        out[r] = acc
    return out


class SingularMatrix(Exception):
    pass


def mat_invert(m: np.ndarray) -> np.ndarray:
    n = m.shape[0]
    assert m.shape == (n, n)
    work = np.concatenate([m.astype(np.uint8), np.eye(n, dtype=np.uint8)], axis=1)
    for r in range(n):
        if work[r, r] == 0:
            for below in range(r + 1, n):
                if work[below, r] != 0:
                    work[[r, below]] = work[[below, r]]
                    break
        if work[r, r] == 0:
            raise SingularMatrix()
        if work[r, r] != 1:
            scale = gal_div(1, int(work[r, r]))
            work[r] = MUL_TABLE[scale, work[r]]
        for other in range(n):
            if other != r and work[other, r] != 0:
                work[other] ^= MUL_TABLE[int(work[other, r]), work[r]]
    return work[:, n:].copy()


def vandermonde(rows: int, cols: int) -> np.ndarray:
    v = np.zeros((rows, cols), dtype=np.uint8)
    for r in range(rows):
        for c in range(cols):
            v[r, c] = gal_exp(r, c)
    return v


def build_matrix(data_shards: int, total_shards: int) -> np.ndarray:
    v = vandermonde(total_shards, data_shards)
    top = v[:data_shards, :data_shards]
    return mat_mul(v, mat_invert(top))


# ----------------------------------------------------------------------------
# Slice kernels (galois_8::mul_slice / mul_slice_xor)
# ----------------------------------------------------------------------------
def mul_slice(c: int, inp: np.ndarray, out: np.ndarray) -> None:
    out[:] = MUL_TABLE[c][inp]


def mul_slice_xor(c: int, inp: np.ndarray, out: np.ndarray) -> None:
    out ^= MUL_TABLE[c][inp]


def _as_u8(x) -> np.ndarray:
    if isinstance(x, np.ndarray):
        assert x.dtype == np.uint8
        return x
    return np.frombuffer(memoryview(x), dtype=np.uint8)


class ReedSolomon:
    """Restatement of ``reed_solomon_erasure::galois_8::ReedSolomon``."""

    def __init__(self, data_shards: int, parity_shards: int):
        if data_shards == 0:
            _err("TooFewDataShards")
        if parity_shards == 0:
            _err("TooFewParityShards")
        if data_shards + parity_shards > FIELD_SIZE:
            _err("TooManyShards")
        self.data_shard_count = data_shards
        self.parity_shard_count = parity_shards
        self.total_shard_count = data_shards + parity_shards
        self.matrix = build_matrix(data_shards, self.total_shard_count)
        self._cache: "OrderedDict[tuple, np.ndarray]" = OrderedDict()

    # -- helpers -------------------------------------------------------------
    def parity_rows(self) -> np.ndarray:
        return self.matrix[self.data_shard_count:]

    def _check_count(self, n: int):
        if n < self.total_shard_count:
            _err("TooFewShards")
        if n > self.total_shard_count:
            _err("TooManyShards")

    @staticmethod
    def _check_slices(slices: Sequence[np.ndarray]):
        size = len(slices[0])
        if size == 0:
            _err("EmptyShard")
        for s in slices:
            if len(s) != size:
                _err("IncorrectShardSize")

    def _code_some_slices(self, rows: Sequence[np.ndarray], inputs, outputs):
        # outer over input shards, inner over output rows (crate order)
        for i_input in range(self.data_shard_count):
            for i_row, out in enumerate(outputs):
                c = int(rows[i_row][i_input])
                if i_input == 0:
                    mul_slice(c, inputs[i_input], out)
                else:
                    mul_slice_xor(c, inputs[i_input], out)

    # -- encode ----------------------------------------------------------------
    def encode(self, shards: List) -> None:
        self._check_count(len(shards))
        sl = [_as_u8(s) for s in shards]
        self._check_slices(sl)
        k = self.data_shard_count
        self._code_some_slices(list(self.parity_rows()), sl[:k], sl[k:])

    def encode_sep(self, data: Sequence, parity: List) -> None:
        if len(data) < self.data_shard_count:
            _err("TooFewDataShards")
        if len(data) > self.data_shard_count:
            _err("TooManyDataShards")
        if len(parity) < self.parity_shard_count:
            _err("TooFewParityShards")
        if len(parity) > self.parity_shard_count:
            _err("TooManyParityShards")
        d = [_as_u8(s) for s in data]
        p = [_as_u8(s) for s in parity]
        self._check_slices(d + p)
        self._code_some_slices(list(self.parity_rows()), d, p)

    def verify(self, shards: Sequence) -> bool:
        self._check_count(len(shards))
        sl = [_as_u8(s) for s in shards]
        self._check_slices(sl)
        k = self.data_shard_count
        tmp = [np.zeros_like(sl[0]) for _ in range(self.parity_shard_count)]
        self._code_some_slices(list(self.parity_rows()), sl[:k], tmp)
        return all(np.array_equal(a, b) for a, b in zip(tmp, sl[k:]))

    # -- reconstruct -----------------------------------------------------------
    def get_data_decode_matrix(self, valid_indices, invalid_indices) -> np.ndarray:
        key = tuple(invalid_indices)
        if key in self._cache:
            self._cache.move_to_end(key)
            return self._cache[key]
        sub = self.matrix[list(valid_indices), :]
        dec = mat_invert(sub)
        self._cache[key] = dec
        if len(self._cache) > DATA_DECODE_MATRIX_CACHE_CAPACITY:
            self._cache.popitem(last=False)
        return dec

    def reconstruct(self, shards: List[Optional[np.ndarray]]) -> None:
        self._reconstruct_internal(shards, data_only=False)

    def reconstruct_data(self, shards: List[Optional[np.ndarray]]) -> None:
        self._reconstruct_internal(shards, data_only=True)

    def _reconstruct_internal(self, shards, data_only: bool) -> None:
        self._check_count(len(shards))
        k = self.data_shard_count
        number_present = 0
        shard_len = None
        for s in shards:
            if s is not None:
                n = len(s)
                if n == 0:
                    _err("EmptyShard")
                number_present += 1
                if shard_len is not None and n != shard_len:
                    _err("IncorrectShardSize")
                shard_len = n
        if number_present == self.total_shard_count:
            return
        if number_present < k:
            _err("TooFewShardsPresent")

        sub_shards, valid, invalid = [], [], []
        missing_data, missing_parity = [], []
        for row, s in enumerate(shards):
            if s is None:
                if row >= k and data_only:
                    invalid.append(row)
                    continue
                buf = np.zeros(shard_len, dtype=np.uint8)
                shards[row] = buf
                (missing_data if row < k else missing_parity).append(buf)
                invalid.append(row)
            else:
                if len(sub_shards) < k:
                    sub_shards.append(_as_u8(s))
                    valid.append(row)

        dec = self.get_data_decode_matrix(valid, invalid)
        rows = [dec[i] for i in invalid if i < k]
        self._code_some_slices(rows, sub_shards, missing_data)
        if data_only:
            return
        prow = self.parity_rows()
        rows = [prow[i - k] for i in invalid if i >= k]
        # all data shards: old ones (front of sub_shards) interleaved with new
        all_data, i_old, i_new = [], 0, 0
        missing_set = [i for i in invalid if i < k]
        for d in range(k):
            if d in missing_set:
                all_data.append(missing_data[i_new])
                i_new += 1
            else:
                all_data.append(sub_shards[i_old])
                i_old += 1
        self._code_some_slices(rows, all_data, missing_parity)


# ----------------------------------------------------------------------------
# shmr glue
# ----------------------------------------------------------------------------
def calculate_shard_size(length: int, data_shards: int) -> int:
    """src/vfs/mod.rs:16-18: ``(length as f32 / data_shards as f32).ceil() as usize``."""
    q = np.float32(length) / np.float32(data_shards)
    return int(np.ceil(np.float32(q)))


class ReferencePanic(Exception):
    """Where the reference binary would panic (debug-build integer overflow
    check, or an ``.unwrap()`` on a crate error).  ``.cause`` names it."""

    def __init__(self, cause: str):
        super().__init__(cause)
        self.cause = cause


SYNC_MODES = ("release", "debug", "refuse")


def sync_data_erasure(buffer: bytes, size: int, data: int, parity: int,
                      mode: str = "release") -> List[np.ndarray]:
    """src/vfs/block.rs:404-440 -- shards that the Erasure arm writes.

    Returns [] for an empty buffer (block.rs:389-391 writes nothing).

    ``block.rs:421`` appends ``parity + (data - nchunks as u8)`` zero shards,
    computed in u8.  ``nchunks`` exceeds ``data`` only past the f32 shard-size
    hazard (``calculate_shard_size``; first at 16,777,217 B for k = 8).  What
    happens then depends on the build (``mode``):

    * ``"release"`` (default; the reference's shipped profile,
      ``Cargo.toml:10-13``, has no overflow checks): both u8 operations wrap,
      so with nchunks = k + e it appends ``(p - e) mod 256`` zero shards.  For
      e <= p that is exactly k + p shards: encode SUCCEEDS and the trailing
      data chunks k..k+e-1 are overwritten by parity rows (their bytes are
      lost from the shard files).  (e > p would leave 256 extra shards, the
      crate's encode would return TooManyShards and the ``.unwrap()`` at
      ``block.rs:427`` panic; unreachable, since the f32 error keeps k*S
      within k bytes of ``size``, so e <= 1 <= p.)
    * ``"debug"``: the subtraction's overflow check panics at block.rs:421.
    * ``"refuse"``: the MI355X mirror's default -- ``TooManyDataShards``
      before any shard is written (a documented deviation: it refuses the
      silent data loss).  Raises RSError("TooManyDataShards").
    """
    if mode not in SYNC_MODES:
        raise ValueError(f"mode must be one of {SYNC_MODES}")
    buf = _as_u8(buffer)
    if len(buf) == 0:
        return []
    r = ReedSolomon(data, parity)                       # block.rs:405
    s = calculate_shard_size(size, data)                # block.rs:406
    shards = []
    for off in range(0, len(buf), s):                   # block.rs:408-419
        c = np.zeros(s, dtype=np.uint8)
        chunk = buf[off:off + s]
        c[:len(chunk)] = chunk
        shards.append(c)
    nchunks = len(shards)
    if nchunks > data:
        if mode == "refuse":
            raise RSError("TooManyDataShards")
        if mode == "debug":
            raise ReferencePanic("attempt to subtract with overflow (block.rs:421)")
    extra = (parity + ((data - nchunks) & 0xFF)) & 0xFF   # block.rs:421, u8 arithmetic
    for _ in range(extra):                              # block.rs:421-423
        shards.append(np.zeros(s, dtype=np.uint8))
    try:
        r.encode(shards)                                # block.rs:427
    except RSError as e:
        raise ReferencePanic(f"called `Result::unwrap()` on an `Err` value: {e.name} (block.rs:427)") from e
    return shards


def load_block_erasure(shards: List[Optional[bytes]], size: int, data: int, parity: int) -> np.ndarray:
    """src/vfs/block.rs:529-579 (version 1).

    ``shards[i]`` is what ``read_to_end`` returned (None == read error).
    Short/long shards are resized to S and *stay present* (block.rs:548-551).
    """
    r = ReedSolomon(data, parity)
    s = calculate_shard_size(size, data)
    missing = False
    ec: List[Optional[np.ndarray]] = []
    for raw in shards:
        if raw is None:
            missing = True
            ec.append(None)
            continue
        b = _as_u8(raw)
        if len(b) != s:
            missing = True
            c = np.zeros(s, dtype=np.uint8)
            c[:min(s, len(b))] = b[:s]
            b = c
        else:
            b = b.copy()
        ec.append(b)
    if missing:
        r.reconstruct(ec)                               # block.rs:560 (unwrap)
    out = np.concatenate(ec)
    return out[:size].copy()


def seeded_block(seed: int, index: int, nbytes: int) -> np.ndarray:
    """SURVEY 8(d) input generator: default_rng([seed, index]) uniform 0..255."""
    rng = np.random.default_rng([seed, index])
    return rng.integers(0, 256, size=nbytes, dtype=np.uint8)


BENCH_SEED = 0x53484D52   # "SHMR"
