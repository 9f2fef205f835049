"""Loader for the in-tree native library ``shmr_amd/_lib/libshmr_ec.so``.

There is no fallback: if the library is missing or fails to load, importing
the compute API raises.  ``tools()`` switches the calling code to the tools
build ``libshmr_ec_tools.so`` (same sources plus the measurement-only kernel
variants and knobs) for the duration of a ``with`` block; the
environment variable ``SHMR_EC_FLAVOUR=tools`` makes it the default (tools/
scripts).  Objects (``ReedSolomon``, buffers) keep the library they were
created with.  ``torch`` is imported first when available so that
the library binds to the same HIP runtime instance as PyTorch (both carry the
SONAME ``libamdhip64.so.7``; loading ours first would map a second runtime).
"""
from __future__ import annotations

import contextlib
import ctypes
import os

try:  # share torch's HIP runtime (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libshmr_ec.so")
TOOLS_LIB_PATH = os.path.join(_HERE, "_lib", "libshmr_ec_tools.so")
_PATHS = {"product": LIB_PATH, "tools": TOOLS_LIB_PATH}

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u8pp = ctypes.POINTER(_u8p)
_sz = ctypes.c_size_t

# (name, restype, argtypes) for every symbol declared in include/shmr_ec.h
SIGNATURES = [
    ("shmr_ec_status_name", ctypes.c_char_p, [ctypes.c_int]),
    ("shmr_ec_version", ctypes.c_char_p, []),
    ("shmr_ec_build_id", ctypes.c_char_p, []),
    ("shmr_ec_is_tools_build", ctypes.c_int, []),
    ("shmr_ec_shard_size", _sz, [ctypes.c_uint64, ctypes.c_uint32]),
    ("shmr_ec_new", ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    ("shmr_ec_free", None, [ctypes.c_void_p]),
    ("shmr_ec_data_shard_count", ctypes.c_uint32, [ctypes.c_void_p]),
    ("shmr_ec_parity_shard_count", ctypes.c_uint32, [ctypes.c_void_p]),
    ("shmr_ec_total_shard_count", ctypes.c_uint32, [ctypes.c_void_p]),
    ("shmr_ec_matrix", ctypes.c_int, [ctypes.c_void_p, _u8p, _sz]),
    ("shmr_ec_reconstruct_plan", ctypes.c_int,
     [ctypes.c_void_p, _u8p, _sz, ctypes.c_int, ctypes.POINTER(ctypes.c_uint16),
      ctypes.POINTER(ctypes.c_uint16), _u8p, _sz, ctypes.POINTER(ctypes.c_uint32)]),
    ("shmr_ec_encode", ctypes.c_int, [ctypes.c_void_p, _u8pp, ctypes.POINTER(_sz), _sz]),
    ("shmr_ec_reconstruct", ctypes.c_int,
     [ctypes.c_void_p, _u8pp, ctypes.POINTER(_sz), _u8p, _sz, ctypes.c_int]),
    ("shmr_ec_encode_batch_dev", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, _sz, _sz, ctypes.c_void_p, _sz, _sz, _sz, _sz,
      ctypes.c_int, ctypes.c_void_p]),
    ("shmr_ec_reconstruct_batch_dev", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, _sz, _sz, _u8p, _sz, _sz, ctypes.c_int, ctypes.c_int,
      ctypes.c_void_p]),
    ("shmr_ec_reconstruct_batch_dev_out", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, _sz, _sz, _u8p, _sz, _sz, ctypes.c_int, ctypes.c_void_p, _sz, _sz,
      ctypes.c_int, ctypes.c_void_p]),
    ("shmr_ec_device_init", ctypes.c_int, [ctypes.c_int]),
    ("shmr_ec_capture_reserve", ctypes.c_int, [ctypes.c_int, _sz]),
    ("shmr_ec_encode_ptrs_dev", ctypes.c_int, [ctypes.c_void_p, _u8pp, _sz, _sz, ctypes.c_int, ctypes.c_void_p]),
    ("shmr_ec_reconstruct_ptrs_dev", ctypes.c_int,
     [ctypes.c_void_p, _u8pp, _u8p, _sz, _sz, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("shmr_ec_encode_blocks_host", ctypes.c_int,
     [ctypes.c_void_p, _u8pp, _sz, _sz, ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    ("shmr_ec_reconstruct_blocks_host", ctypes.c_int,
     [ctypes.c_void_p, _u8pp, _u8p, _sz, _sz, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    ("shmr_ec_device_alloc", ctypes.c_int, [ctypes.c_int, _sz, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("shmr_ec_device_free", ctypes.c_int, [ctypes.c_int, ctypes.c_void_p]),
    ("shmr_ec_device_alloc_shards", ctypes.c_int, [ctypes.c_int, _sz, _sz, _sz, _u8pp]),
    ("shmr_ec_device_free_shards", ctypes.c_int, [ctypes.c_int, _u8p]),
    ("shmr_ec_host_alloc", ctypes.c_int, [_sz, ctypes.POINTER(ctypes.c_void_p)]),
    ("shmr_ec_host_free", None, [ctypes.c_void_p]),
    ("shmr_ec_host_register", ctypes.c_int, [ctypes.c_void_p, _sz]),
    ("shmr_ec_host_unregister", ctypes.c_int, [ctypes.c_void_p]),
    ("shmr_ec_path_stats", ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    ("shmr_ec_set_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("shmr_ec_set_tuning", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    ("shmr_ec_get_tuning", ctypes.c_int, [ctypes.c_char_p]),
    ("shmr_ec_describe_variant", ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p, _sz]),
    ("shmr_ec_cache_stats", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    ("shmr_ec_device_count", ctypes.c_int, []),
    ("shmr_ec_device_stats", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), _sz]),
    ("shmr_ec_kernel_inventory", _sz, [ctypes.c_void_p, _sz]),
    ("shmr_ec_encode_start", ctypes.c_int,
     [ctypes.c_void_p, _u8pp, ctypes.POINTER(_sz), _sz, ctypes.POINTER(ctypes.c_void_p)]),
    ("shmr_ec_reconstruct_start", ctypes.c_int,
     [ctypes.c_void_p, _u8pp, ctypes.POINTER(_sz), _u8p, _sz, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("shmr_ec_op_wait", ctypes.c_int, [ctypes.c_void_p]),
    ("shmr_ec_encode_dev", ctypes.c_int, [ctypes.c_void_p, _u8pp, ctypes.POINTER(_sz), _sz, ctypes.c_int]),
    ("shmr_ec_reconstruct_dev", ctypes.c_int,
     [ctypes.c_void_p, _u8pp, ctypes.POINTER(_sz), _u8p, _sz, ctypes.c_int, ctypes.c_int]),
    ("shmr_ec_encode_dev_start", ctypes.c_int,
     [ctypes.c_void_p, _u8pp, ctypes.POINTER(_sz), _sz, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("shmr_ec_reconstruct_dev_start", ctypes.c_int,
     [ctypes.c_void_p, _u8pp, ctypes.POINTER(_sz), _u8p, _sz, ctypes.c_int, ctypes.c_int,
      ctypes.POINTER(ctypes.c_void_p)]),
    ("shmr_ec_queue_stats", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), _sz]),
    ("shmr_ec_pool_new", ctypes.c_int, [ctypes.c_int, _sz, _sz, _sz, ctypes.POINTER(ctypes.c_void_p)]),
    ("shmr_ec_pool_alloc", ctypes.c_int, [ctypes.c_void_p, _u8pp]),
    ("shmr_ec_pool_free", ctypes.c_int, [ctypes.c_void_p, _u8p]),
    ("shmr_ec_pool_destroy", ctypes.c_int, [ctypes.c_void_p]),
    ("shmr_ec_pool_stats", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
      ctypes.POINTER(ctypes.c_uint64)]),
]


class KernelInfo(ctypes.Structure):
    """shmr_ec_kernel_info (include/shmr_ec.h)."""
    _fields_ = [("rows", ctypes.c_uint32), ("chunks", ctypes.c_uint32), ("mode", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("launches", ctypes.c_uint64)]

_libs = {}
_flavour = "tools" if os.environ.get("SHMR_EC_FLAVOUR") == "tools" else "product"


class NativeLibraryMissing(RuntimeError):
    pass


def _load(flavour: str):
    L = _libs.get(flavour)
    if L is None:
        path = _PATHS[flavour]
        if not os.path.exists(path):
            raise NativeLibraryMissing(
                f"{path} is missing: build it with `make -C shmr_amd/csrc` or "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        L = ctypes.CDLL(path)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _libs[flavour] = L
    return L


def lib():
    """Returns the active native library (product unless inside ``tools()``);
    raises if it is not built."""
    return _load(_flavour)


def flavour() -> str:
    return _flavour


@contextlib.contextmanager
def tools():
    """Within the block, new objects and the module-level calls use the tools
    build.  Not thread-safe: for tests and tools/ scripts."""
    global _flavour
    prev = _flavour
    _load("tools")
    _flavour = "tools"
    try:
        yield _libs["tools"]
    finally:
        _flavour = prev
