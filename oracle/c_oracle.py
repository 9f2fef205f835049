"""ctypes binding for the C oracle (oracle/rs_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / CPU baseline.  Never imported by shmr_amd.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "librs_oracle.so")
_lib = None

_u8p = ctypes.POINTER(ctypes.c_uint8)


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_gal_mul.restype = ctypes.c_uint8
        L.oracle_gal_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.oracle_gal_exp.restype = ctypes.c_uint8
        L.oracle_gal_exp.argtypes = [ctypes.c_uint8, ctypes.c_uint32]
        L.oracle_build_matrix.restype = ctypes.c_int
        L.oracle_build_matrix.argtypes = [ctypes.c_uint32, ctypes.c_uint32, _u8p]
        L.oracle_invert.restype = ctypes.c_int
        L.oracle_invert.argtypes = [_u8p, ctypes.c_uint32, _u8p]
        L.oracle_apply.restype = None
        L.oracle_apply.argtypes = [ctypes.c_int, _u8p, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.POINTER(_u8p), ctypes.POINTER(_u8p), ctypes.c_size_t]
        L.oracle_encode.restype = ctypes.c_int
        L.oracle_encode.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.POINTER(_u8p), ctypes.c_size_t]
        L.oracle_reconstruct.restype = ctypes.c_int
        L.oracle_reconstruct.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(_u8p),
                                         _u8p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_encode_batch.restype = ctypes.c_double
        L.oracle_encode_batch.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                          ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                          ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]
        L.oracle_reconstruct_batch.restype = ctypes.c_double
        L.oracle_reconstruct_batch.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                               ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                               ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        L.oracle_sync_data_batch.restype = ctypes.c_double
        L.oracle_sync_data_batch.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                             ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.c_int]
        L.oracle_has_avx2.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_u8p)


def build_matrix(k: int, p: int) -> np.ndarray:
    out = np.zeros((k + p) * k, dtype=np.uint8)
    rc = lib().oracle_build_matrix(k, p, _ptr(out))
    if rc != 0:
        raise ValueError(rc)
    return out.reshape(k + p, k)


def invert(m: np.ndarray) -> np.ndarray:
    m = np.ascontiguousarray(m, dtype=np.uint8)
    out = np.zeros_like(m)
    if lib().oracle_invert(_ptr(m), m.shape[0], _ptr(out)) != 0:
        raise ValueError("singular")
    return out


def apply(rows: np.ndarray, inputs: Sequence[np.ndarray], length: int, variant: int = 1) -> List[np.ndarray]:
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    nr, k = rows.shape
    assert len(inputs) == k
    outs = [np.zeros(length, dtype=np.uint8) for _ in range(nr)]
    ins = (_u8p * k)(*[_ptr(np.ascontiguousarray(x)) for x in inputs])
    os_ = (_u8p * max(nr, 1))(*[_ptr(o) for o in outs])
    lib().oracle_apply(variant, _ptr(rows), nr, k, ins, os_, length)
    return outs


def encode(k: int, p: int, shards: List[np.ndarray], variant: int = 1) -> None:
    arr = (_u8p * (k + p))(*[_ptr(s) for s in shards])
    rc = lib().oracle_encode(variant, k, p, arr, len(shards[0]))
    if rc != 0:
        raise ValueError(rc)


def reconstruct(k: int, p: int, shards: List[Optional[np.ndarray]], length: int,
                data_only: bool = False) -> List[np.ndarray]:
    present = np.array([s is not None for s in shards], dtype=np.uint8)
    full = [s if s is not None else np.zeros(length, dtype=np.uint8) for s in shards]
    arr = (_u8p * (k + p))(*[_ptr(s) for s in full])
    rc = lib().oracle_reconstruct(k, p, arr, _ptr(present), length, int(data_only))
    if rc != 0:
        raise ValueError(rc)
    return full


def encode_batch(k: int, p: int, data: np.ndarray, parity: np.ndarray, nblocks: int, length: int,
                 nthreads: int, variant: int = 1) -> float:
    """data: [nblocks][k][length] contiguous; parity: [nblocks][p][length]."""
    assert data.size >= nblocks * k * length and parity.size >= nblocks * p * length
    return lib().oracle_encode_batch(variant, k, p, data.ctypes.data, length, k * length,
                                     parity.ctypes.data, length, p * length, nblocks, length, nthreads)


def reconstruct_batch(k: int, p: int, shards: np.ndarray, present: np.ndarray, length: int, nthreads: int,
                      variant: int = 1, data_only: bool = False) -> float:
    """shards: uint8 [nblocks][k+p][pitch] (absent shards overwritten in place);
    present: [nblocks][k+p].  Returns seconds (one block per thread task)."""
    assert shards.ndim == 3 and shards.dtype == np.uint8 and shards.flags["C_CONTIGUOUS"]
    pr = np.ascontiguousarray(present, dtype=np.uint8)
    B = shards.shape[0]
    secs = lib().oracle_reconstruct_batch(variant, k, p, shards.ctypes.data, shards.strides[1], shards.strides[0],
                                          pr.ctypes.data, B, length, int(data_only), nthreads)
    if secs < 0:
        raise ValueError("reconstruct failed")
    return secs


def sync_data_batch(k: int, p: int, src: np.ndarray, size: int, shard: int, parity: np.ndarray, nblocks: int,
                    nthreads: int, variant: int = 1) -> float:
    """VirtualBlock::sync_data minus disk (block.rs:406-430) for nblocks
    size-byte buffers at src + b * size: chunk to_vec copies, zero pad, zero
    shards, encode.  parity: [nblocks][p][shard] out.  Returns seconds."""
    assert src.size >= nblocks * size and parity.size >= nblocks * p * shard
    secs = lib().oracle_sync_data_batch(variant, k, p, src.ctypes.data, size, shard, parity.ctypes.data, nblocks,
                                        nthreads)
    if secs < 0:
        raise ValueError("sync_data batch failed")
    return secs
