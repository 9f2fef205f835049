"""Host-side mirror of ``reed_solomon_erasure::galois_8::ReedSolomon``.

The reference binds the crate at ``src/vfs/block.rs:10`` and calls
``ReedSolomon::new`` (block.rs:405, :531), ``encode`` (block.rs:427) and
``reconstruct`` (block.rs:560).  This class keeps those names, argument
meanings and error behaviour (``Error.name`` is the crate variant name), and
runs every byte of arithmetic on the MI355X through ``include/shmr_ec.h``.

Device-resident batch entry points (``encode_batch_dev`` /
``reconstruct_batch_dev``) take torch CUDA(HIP) tensors and enqueue on the
current torch stream.
"""
from __future__ import annotations

import ctypes
from typing import List, MutableSequence, Optional, Sequence

import numpy as np

from . import _native
from ._native import _u8p, lib

__all__ = ["Error", "ReedSolomon", "calculate_shard_size", "device_count", "set_tuning", "get_tuning", "describe_variant",
           "PinnedBuffer", "ShardSlab", "host_register", "host_unregister", "path_stats", "device_init", "kernel_inventory", "capture_reserve"]


class Error(Exception):
    """A non-zero status from the native library (crate variant names)."""

    def __init__(self, code: int):
        self.code = code
        self.name = lib().shmr_ec_status_name(code).decode()
        super().__init__(f"{self.name} ({code})")


def _check(rc: int) -> None:
    if rc != 0:
        raise Error(rc)


def calculate_shard_size(length: int, data_shards: int) -> int:
    """``calculate_shard_size`` (reference src/vfs/mod.rs:16-18), f32 ceil."""
    return int(lib().shmr_ec_shard_size(length, data_shards))


def device_count() -> int:
    return int(lib().shmr_ec_device_count())


def set_tuning(**knobs) -> None:
    """Kernel knobs, e.g. set_tuning(chunks=1, grid=-1) or set_tuning(**{"decode.nt_load": 1})."""
    for key, value in knobs.items():
        _check(lib().shmr_ec_set_tuning(key.encode(), int(value)))


def get_tuning(key: str) -> int:
    return int(lib().shmr_ec_get_tuning(key.encode()))


def describe_variant(decode, data_shards: int, rows: int) -> str:
    """The kernel variant a launch of this shape uses (after the auto policy).
    decode: 0/False encode, 1/True reconstruct in place, 2 reconstruct into a
    compact output (reconstruct_batch_dev_out); 3 / 4 encode / reconstruct
    over device shard-pointer tables (encode_ptrs_dev / reconstruct_ptrs_dev)."""
    buf = ctypes.create_string_buffer(256)
    _check(lib().shmr_ec_describe_variant(int(decode), data_shards, rows, buf, 256))
    return buf.value.decode()


def kernel_inventory(flavour: Optional[str] = None) -> list:
    """Every gf_apply kernel instantiation compiled into the library, with the
    launches each has served in this process (shmr_ec_kernel_inventory): dicts
    with rows, chunks, mode (0 full tiles, 1 partial tail, 2 byte-granular,
    3 realigning) and flags (the kernel's template flags)."""
    L = _native._load(flavour) if flavour else lib()
    n = L.shmr_ec_kernel_inventory(None, 0)
    arr = (_native.KernelInfo * n)()
    L.shmr_ec_kernel_inventory(ctypes.cast(arr, ctypes.c_void_p), n)
    return [{"rows": e.rows, "chunks": e.chunks, "mode": e.mode, "flags": e.flags, "launches": e.launches}
            for e in arr]


def _writable_u8(buf) -> np.ndarray:
    """A uint8 view over a writable buffer (bytearray, numpy array, memoryview)."""
    if isinstance(buf, np.ndarray):
        if buf.dtype != np.uint8 or not buf.flags["C_CONTIGUOUS"]:
            raise TypeError("shards must be C-contiguous uint8 arrays")
        return buf
    arr = np.frombuffer(buf, dtype=np.uint8)
    if not arr.flags["WRITEABLE"]:
        raise TypeError("shard buffers must be writable (bytearray / numpy)")
    return arr


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_u8p) if a.size else ctypes.cast(ctypes.c_void_p(1), _u8p)


class ReedSolomon:
    """``ReedSolomon::new(data_shards, parity_shards)`` -- raises ``Error``."""

    def __init__(self, data_shards: int, parity_shards: int, device: int = 0):
        self._L = lib()   # the library this codec lives in (product unless _native.tools())
        h = ctypes.c_void_p()
        _check(self._L.shmr_ec_new(data_shards, parity_shards, ctypes.byref(h)))
        self._h = h
        self.device = int(device)
        if device:
            _check(self._L.shmr_ec_set_device(self._h, device))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.shmr_ec_free(h)
            self._h = None

    # -- crate accessors -------------------------------------------------------
    def data_shard_count(self) -> int:
        return int(self._L.shmr_ec_data_shard_count(self._h))

    def parity_shard_count(self) -> int:
        return int(self._L.shmr_ec_parity_shard_count(self._h))

    def total_shard_count(self) -> int:
        return int(self._L.shmr_ec_total_shard_count(self._h))

    def matrix(self) -> np.ndarray:
        t, k = self.total_shard_count(), self.data_shard_count()
        out = np.zeros(t * k, dtype=np.uint8)
        _check(self._L.shmr_ec_matrix(self._h, _ptr(out), out.size))
        return out.reshape(t, k)

    def set_device(self, device: int) -> None:
        self.device = int(device)
        _check(self._L.shmr_ec_set_device(self._h, device))

    def cache_stats(self):
        h, m = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self._L.shmr_ec_cache_stats(self._h, ctypes.byref(h), ctypes.byref(m)))
        return int(h.value), int(m.value)

    def reconstruct_plan(self, present: Sequence[bool], data_only: bool = False):
        """(in_idx, out_idx, rows) of the plan the GPU runs for this pattern."""
        t, k = self.total_shard_count(), self.data_shard_count()
        pr = np.array([1 if x else 0 for x in present], dtype=np.uint8)
        in_idx = (ctypes.c_uint16 * k)()
        out_idx = (ctypes.c_uint16 * t)()
        rows = np.zeros(t * k, dtype=np.uint8)
        n = ctypes.c_uint32()
        _check(self._L.shmr_ec_reconstruct_plan(self._h, _ptr(pr), len(pr), int(data_only), in_idx, out_idx,
                                              _ptr(rows), rows.size, ctypes.byref(n)))
        m = n.value
        return list(in_idx), list(out_idx)[:m], rows[:m * k].reshape(m, k).copy()

    # -- crate calls ---------------------------------------------------------------
    def encode(self, shards: MutableSequence) -> None:
        """``ReedSolomon::encode``: shards[k:] are overwritten with parity."""
        arrs = [_writable_u8(s) for s in shards]
        n = len(arrs)
        ptrs = (_u8p * max(n, 1))(*[_ptr(a) for a in arrs])
        lens = (ctypes.c_size_t * max(n, 1))(*[a.size for a in arrs])
        _check(self._L.shmr_ec_encode(self._h, ptrs, lens, n))

    def _reconstruct(self, shards: MutableSequence[Optional[object]], data_only: bool) -> None:
        n = len(shards)
        k = self.data_shard_count()
        present = np.array([s is not None for s in shards], dtype=np.uint8)
        arrs: List[Optional[np.ndarray]] = [None if s is None else _writable_u8(s) for s in shards]
        shard_len = next((a.size for a in arrs if a is not None), 0)
        # The crate allocates absent shards (get_or_initialize); mirror that,
        # but only once the crate's own checks would pass.
        fill = [False] * n
        if n == self.total_shard_count() and 0 < present.sum() < n and present.sum() >= k:
            for i, a in enumerate(arrs):
                if a is None and (i < k or not data_only):
                    arrs[i] = np.zeros(shard_len, dtype=np.uint8)
                    fill[i] = True
        ptrs = (_u8p * max(n, 1))(*[(_ptr(a) if a is not None else _u8p()) for a in arrs])
        lens = (ctypes.c_size_t * max(n, 1))(*[(a.size if a is not None else 0) for a in arrs])
        _check(self._L.shmr_ec_reconstruct(self._h, ptrs, lens, _ptr(present), n, int(data_only)))
        for i in range(n):
            if fill[i]:
                shards[i] = arrs[i]

    def reconstruct(self, shards: MutableSequence[Optional[object]]) -> None:
        """``ReedSolomon::reconstruct``: None entries become rebuilt shards."""
        self._reconstruct(shards, data_only=False)

    def reconstruct_data(self, shards: MutableSequence[Optional[object]]) -> None:
        """``ReedSolomon::reconstruct_data``: only absent data shards are rebuilt."""
        self._reconstruct(shards, data_only=True)

    def verify(self, shards: Sequence) -> bool:
        """``ReedSolomon::verify``: recompute parity on the GPU and compare."""
        k = self.data_shard_count()
        arrs = [_writable_u8(s) if not isinstance(s, (bytes,)) else np.frombuffer(s, np.uint8) for s in shards]
        tmp = [a.copy() for a in arrs[:k]] + [np.zeros_like(a) for a in arrs[k:]]
        self.encode(tmp)
        return all(np.array_equal(a, b) for a, b in zip(tmp[k:], arrs[k:]))

    # -- device-resident batches (torch tensors on the GPU) ------------------------
    @staticmethod
    def _check_batch_tensor(t, rows: int, shard_pitch: int, shard_len: int) -> None:
        """Bounds of one [B, rows, pitch] / [B, rows*pitch] batch tensor, checked
        before the launch: the C ABI takes raw pointers and pitches and cannot
        see the allocation, so a short tensor would be an out-of-bounds kernel
        access.  Order: dtype, shard count, shard size, then memory kind."""
        import torch
        if not isinstance(t, torch.Tensor) or t.dtype != torch.uint8:
            raise TypeError("batch tensors must be torch.uint8")
        if t.dim() == 3:
            if t.shape[1] != rows:
                raise Error(-1 if t.shape[1] < rows else -2)     # TooFewShards / TooManyShards
            if t.stride(2) != 1:
                raise TypeError("shard bytes must be contiguous (stride 1 in the last dimension)")
            extent = (t.shape[1] - 1) * t.stride(1) + t.shape[2]
        elif t.dim() == 2:
            if t.stride(1) != 1:
                raise TypeError("block bytes must be contiguous (stride 1 in the last dimension)")
            extent = t.shape[1]
        else:
            raise TypeError("batch tensors are [blocks, shards, bytes] or [blocks, shards * bytes]")
        if shard_len <= 0 and t.shape[0] > 0:
            raise Error(-11)                                     # EmptyShard
        if shard_pitch < 0 or (rows - 1) * shard_pitch + shard_len > extent:
            raise Error(-9)                                      # IncorrectShardSize

    @staticmethod
    def _check_addressable(*tensors) -> None:
        """After the shape checks of every operand: the GPU must be able to
        address them (device memory, or pinned host memory for zero-copy)."""
        for t in tensors:
            if not (t.is_cuda or t.is_pinned()):
                raise TypeError("batch tensors must be on the GPU or in pinned host memory")

    @staticmethod
    def _stream_and_device(t):
        import torch
        dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
        return dev, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def encode_batch_dev(self, data, parity, shard_len: Optional[int] = None,
                         data_shard_pitch: Optional[int] = None, parity_shard_pitch: Optional[int] = None,
                         device: Optional[int] = None) -> None:
        """data: uint8 [B, k, pitch] (or [B, k*pitch]); parity: uint8 [B, p, pitch'].

        Enqueued on torch's current stream of the tensors' device.  ``device``:
        the device ID passed to the library (default: the tensors' device; the
        tools build's alias IDs run on the same GPU, shmr_ec.h)."""
        B = data.shape[0]
        dbp = data.stride(0)
        pbp = parity.stride(0)
        dsp = data_shard_pitch if data_shard_pitch is not None else (data.stride(1) if data.dim() == 3 else dbp // self.data_shard_count())
        psp = parity_shard_pitch if parity_shard_pitch is not None else (parity.stride(1) if parity.dim() == 3 else pbp // self.parity_shard_count())
        L = shard_len if shard_len is not None else dsp
        if parity.shape[0] != B:
            raise ValueError(f"data has {B} blocks, parity {parity.shape[0]}")
        self._check_batch_tensor(data, self.data_shard_count(), dsp, L)
        self._check_batch_tensor(parity, self.parity_shard_count(), psp, L)
        self._check_addressable(data, parity)
        dev, stream = self._stream_and_device(data)
        dev = dev if device is None else int(device)
        _check(self._L.shmr_ec_encode_batch_dev(self._h, ctypes.c_void_p(data.data_ptr()), dsp, dbp,
                                              ctypes.c_void_p(parity.data_ptr()), psp, pbp, B, L, dev, stream))

    def reconstruct_batch_dev(self, shards, present: np.ndarray, shard_len: Optional[int] = None,
                              data_only: bool = False, device: Optional[int] = None) -> None:
        """shards: uint8 [B, total, pitch] on the GPU; present: host bool/uint8 [B, total]."""
        if shards.dim() != 3:
            raise TypeError("shards must be a [blocks, total, bytes] tensor")
        B, t = shards.shape[0], self.total_shard_count()
        L = shard_len if shard_len is not None else shards.stride(1)
        self._check_batch_tensor(shards, t, shards.stride(1), L)
        pr = np.ascontiguousarray(present, dtype=np.uint8)
        if pr.size != B * t:
            raise ValueError(f"present must hold {B} x {t} flags")
        pr = pr.reshape(B, t)
        self._check_addressable(shards)
        dev, stream = self._stream_and_device(shards)
        dev = dev if device is None else int(device)
        _check(self._L.shmr_ec_reconstruct_batch_dev(self._h, ctypes.c_void_p(shards.data_ptr()), shards.stride(1),
                                                   shards.stride(0), _ptr(pr), B, L, int(data_only), dev, stream))

    def reconstruct_batch_dev_out(self, shards, present: np.ndarray, out, shard_len: Optional[int] = None,
                                  data_only: bool = False, device: Optional[int] = None) -> None:
        """Rebuild the absent shards of every block into a separate compact
        output -- the crate's semantics, where each ``None`` shard becomes a
        fresh buffer (reference src/vfs/block.rs:556-565).

        shards: uint8 [B, total, pitch] on the GPU (present shards are read in
        place; absent slots are neither read nor written); present: host
        [B, total] flags; out: uint8 [B, n_out, pitch'] on the GPU, where
        out[b, j] receives block b's j-th rebuilt shard in ascending shard
        index (absent data shards only with ``data_only``)."""
        if shards.dim() != 3:
            raise TypeError("shards must be a [blocks, total, bytes] tensor")
        B, t, k = shards.shape[0], self.total_shard_count(), self.data_shard_count()
        L = shard_len if shard_len is not None else shards.stride(1)
        self._check_batch_tensor(shards, t, shards.stride(1), L)
        pr = np.ascontiguousarray(present, dtype=np.uint8)
        if pr.size != B * t:
            raise ValueError(f"present must hold {B} x {t} flags")
        pr = pr.reshape(B, t)
        absent = pr == 0
        if data_only:
            absent[:, k:] = False
        rebuilt = np.where(pr.all(axis=1), 0, absent.sum(axis=1)) if B else np.zeros(0, np.int64)
        need = int(rebuilt.max()) if B else 0
        if out.dim() != 3 or out.shape[0] != B:
            raise TypeError("out must be a [blocks, rebuilt shards, bytes] tensor with one row per block")
        if need:
            self._check_batch_tensor(out[:, :need] if out.shape[1] >= need else out, need, out.stride(1), L)
        self._check_addressable(shards, out)
        dev, stream = self._stream_and_device(shards)
        dev = dev if device is None else int(device)
        _check(self._L.shmr_ec_reconstruct_batch_dev_out(
            self._h, ctypes.c_void_p(shards.data_ptr()), shards.stride(1), shards.stride(0), _ptr(pr), B, L,
            int(data_only), ctypes.c_void_p(out.data_ptr()), out.stride(1), out.stride(0), dev, stream))

    # -- device-resident shards anywhere (shard-pointer tables) ----------------------
    def _dev_table(self, blocks, need_buffer):
        """Per-block lists of 1-D contiguous uint8 GPU tensors (None allowed
        where ``need_buffer(b, i)`` is false) -> (tensors kept alive, shard
        length, device index, ctypes pointer table).  Crate check order per
        shard list: shard count, EmptyShard, IncorrectShardSize."""
        import torch
        t = self.total_shard_count()
        for blk in blocks:
            if len(blk) != t:
                raise Error(-1 if len(blk) < t else -2)          # TooFewShards / TooManyShards
        L, dev = 0, None
        for blk in blocks:
            for s in blk:
                if s is None:
                    continue
                if not isinstance(s, torch.Tensor) or s.dtype != torch.uint8 or not s.is_cuda:
                    raise TypeError("shards must be torch.uint8 tensors on the GPU (or None)")
                if not s.is_contiguous():
                    raise TypeError("shard bytes must be contiguous")
                if dev is None:
                    L, dev = s.numel(), s.device.index
                elif s.device.index != dev:
                    raise ValueError("every shard of a call must be on one GPU")
        if blocks and L == 0:
            raise Error(-11)                                     # EmptyShard
        flat = []
        for b, blk in enumerate(blocks):
            for i, s in enumerate(blk):
                if s is None:
                    if need_buffer(b, i):
                        raise ValueError(f"block {b} shard {i} needs a buffer")
                    flat.append(None)
                elif s.numel() != L:
                    raise Error(-9)                              # IncorrectShardSize
                else:
                    flat.append(s)
        ptrs = (_u8p * max(len(flat), 1))(*[(_u8p() if s is None else ctypes.cast(s.data_ptr(), _u8p)) for s in flat])
        return flat, L, (dev if dev is not None else torch.cuda.current_device()), ptrs

    def encode_ptrs_dev(self, blocks, device: Optional[int] = None) -> None:
        """``ReedSolomon::encode`` (reference src/vfs/block.rs:427) for many blocks whose
        shards are separate GPU buffers -- the crate's shape, where every shard is its
        own ``Vec<u8>`` (block.rs:408-419).  blocks: per-block lists of ``total``
        1-D uint8 tensors of one length (data in, parity overwritten).  Enqueued on
        torch's current stream of their device."""
        keep, L, dev, ptrs = self._dev_table(blocks, lambda b, i: True)
        import torch
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _check(self._L.shmr_ec_encode_ptrs_dev(self._h, ptrs, len(blocks), L,
                                               dev if device is None else int(device), stream))
        del keep

    def reconstruct_ptrs_dev(self, blocks, data_only: bool = False, device: Optional[int] = None) -> None:
        """``ReedSolomon::reconstruct`` / ``reconstruct_data`` (block.rs:560) for many
        blocks of separate GPU shard buffers, with the crate's semantics: every
        ``None`` entry becomes a fresh buffer holding the rebuilt shard
        (block.rs:556-565); absent parity stays ``None`` with ``data_only``.  Blocks
        with every shard present are left alone; a block with fewer than
        ``data`` present shards fails the whole call before any launch."""
        import torch
        t, k = self.total_shard_count(), self.data_shard_count()
        for blk in blocks:
            if len(blk) != t:
                raise Error(-1 if len(blk) < t else -2)
        present = np.array([[s is not None for s in blk] for blk in blocks], dtype=np.uint8).reshape(len(blocks), t)
        for row in present:
            if row.sum() != t and row.sum() < k:
                raise Error(-10)                                 # TooFewShardsPresent
        live = [s for blk in blocks for s in blk if s is not None]
        if not live:
            return
        L, dev0 = live[0].numel(), live[0].device
        # the crate allocates each None shard (vec![0; len]); here: a fresh GPU buffer
        fresh = [list(blk) for blk in blocks]
        for b, blk in enumerate(fresh):
            if present[b].all():
                continue
            for i in range(t):
                if blk[i] is None and not (data_only and i >= k):
                    blk[i] = torch.zeros(L, dtype=torch.uint8, device=dev0)
        keep, L, dev, ptrs = self._dev_table(fresh, lambda b, i: not (data_only and i >= k))
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _check(self._L.shmr_ec_reconstruct_ptrs_dev(self._h, ptrs, _ptr(present), len(blocks), L, int(data_only),
                                                    dev if device is None else int(device), stream))
        for b, blk in enumerate(blocks):
            for i in range(t):
                if blk[i] is None and fresh[b][i] is not None:
                    blk[i] = fresh[b][i]
        del keep

    # -- one block per call on device buffers: the submission queue ------------------
    def _one_block(self, shards, present=None):
        """One block's shards -> (ctypes pointer array, lengths, device).  Entries
        are uint8 CUDA tensors or raw device addresses (ints, with ``shard_len``
        given through ``present``-free calls); None = a NULL pointer."""
        import torch
        t = len(shards)
        ptrs = (_u8p * max(t, 1))()
        lens = (ctypes.c_size_t * max(t, 1))()
        dev = None
        for i, s in enumerate(shards):
            if s is None:
                continue
            if isinstance(s, torch.Tensor):
                if s.dtype != torch.uint8 or not s.is_cuda or not s.is_contiguous():
                    raise TypeError("shards must be contiguous torch.uint8 GPU tensors")
                ptrs[i] = ctypes.cast(s.data_ptr(), _u8p)
                lens[i] = s.numel()
                dev = s.device.index if dev is None else dev
            else:
                addr, n = s
                ptrs[i] = ctypes.cast(int(addr), _u8p)
                lens[i] = int(n)
        return ptrs, lens, dev

    def encode_dev(self, shards, device: Optional[int] = None, start: bool = False):
        """``ReedSolomon::encode`` (reference src/vfs/block.rs:427) of ONE block whose
        shards are GPU buffers (tensors, or (address, length) pairs), through the
        device's submission queue (shmr_ec_encode_dev): concurrent calls merge into
        batch launches.  Inputs must be complete (synchronised) before the call.
        start=True returns an ``Op`` (shmr_ec_encode_dev_start)."""
        ptrs, lens, dev = self._one_block(shards)
        dev = int(device) if device is not None else (dev if dev is not None else self.device)
        if start:
            op = ctypes.c_void_p()
            _check(self._L.shmr_ec_encode_dev_start(self._h, ptrs, lens, len(shards), dev, ctypes.byref(op)))
            return Op(self._L, op, (ptrs, lens, shards))
        _check(self._L.shmr_ec_encode_dev(self._h, ptrs, lens, len(shards), dev))
        return None

    def reconstruct_dev(self, shards, present, data_only: bool = False, device: Optional[int] = None,
                        start: bool = False):
        """``ReedSolomon::reconstruct{,_data}`` (block.rs:560) of ONE block of GPU
        buffers through the submission queue (shmr_ec_reconstruct_dev): ``present``
        flags per shard; absent shards name the buffers that receive the rebuilt
        bytes (absent parity may be None with data_only)."""
        ptrs, lens, dev = self._one_block(shards)
        pr = np.ascontiguousarray(np.asarray(present, dtype=np.uint8))
        for i in range(len(shards)):
            if not pr[i]:
                lens[i] = 0
        dev = int(device) if device is not None else (dev if dev is not None else self.device)
        if start:
            op = ctypes.c_void_p()
            _check(self._L.shmr_ec_reconstruct_dev_start(self._h, ptrs, lens, _ptr(pr), len(shards), int(data_only),
                                                          dev, ctypes.byref(op)))
            return Op(self._L, op, (ptrs, lens, pr, shards))
        _check(self._L.shmr_ec_reconstruct_dev(self._h, ptrs, lens, _ptr(pr), len(shards), int(data_only), dev))
        return None

    def _host_ptrs(self, blocks):
        t = self.total_shard_count()
        if isinstance(blocks, np.ndarray):
            # [B, total, S] array (e.g. a Block Cache slab): shard pointers computed
            # in one vectorised step instead of B * total Python views
            if blocks.ndim != 3 or blocks.dtype != np.uint8 or blocks.strides[2] != 1:
                raise TypeError("blocks array must be uint8 [nblocks, total, shard_len], shard bytes contiguous")
            if not blocks.flags["WRITEABLE"]:
                raise TypeError("blocks array must be writable")
            if blocks.shape[1] != t:
                raise Error(-1 if blocks.shape[1] < t else -2)
            B, _, L = blocks.shape
            base = blocks.ctypes.data
            ptrs = (np.uint64(base) + np.arange(B, dtype=np.uint64)[:, None] * np.uint64(blocks.strides[0])
                    + np.arange(t, dtype=np.uint64)[None, :] * np.uint64(blocks.strides[1])).reshape(-1)
            ptrs = np.ascontiguousarray(ptrs)
            return (blocks, ptrs), L, ptrs.ctypes.data_as(ctypes.POINTER(_u8p))
        arrs = [[(None if s is None else _writable_u8(s)) for s in blk] for blk in blocks]
        for blk in arrs:
            if len(blk) != t:
                raise Error(-1 if len(blk) < t else -2)
        L = next((a.size for blk in arrs for a in blk if a is not None), 0)
        # The C ABI takes one shard_len for every pointer, so every shard must
        # hold exactly that many bytes (a shorter buffer would be read or
        # written past its end).  Crate check order: EmptyShard, then
        # IncorrectShardSize.
        if arrs and L == 0:
            raise Error(-11)                                     # EmptyShard
        if any(a is not None and a.size != L for blk in arrs for a in blk):
            raise Error(-9)                                      # IncorrectShardSize
        flat = [a for blk in arrs for a in blk]
        ptrs = (_u8p * max(len(flat), 1))(*[(_ptr(a) if a is not None else _u8p()) for a in flat])
        return arrs, L, ptrs

    def encode_blocks_host(self, blocks, devices: Sequence[int] = (0,)) -> None:
        """Encode many host-resident blocks, whole blocks round-robin over
        devices.  blocks: a list of per-block shard lists, or one uint8 array
        [nblocks, total, shard_len] (parity rows overwritten)."""
        keep, L, ptrs = self._host_ptrs(blocks)
        n = len(blocks)
        devs = (ctypes.c_int * len(devices))(*devices)
        _check(self._L.shmr_ec_encode_blocks_host(self._h, ptrs, n, L, devs, len(devices)))
        del keep

    def reconstruct_blocks_host(self, blocks, present, data_only: bool = False,
                                devices: Sequence[int] = (0,)) -> None:
        """Rebuild absent shards of many host-resident blocks in place (blocks as
        for encode_blocks_host).  present: [nblocks][total] flags; absent shards
        need (writable) buffers."""
        keep, L, ptrs = self._host_ptrs(blocks)
        n = len(blocks)
        pr = np.ascontiguousarray(present, dtype=np.uint8).reshape(n, self.total_shard_count())
        devs = (ctypes.c_int * len(devices))(*devices)
        _check(self._L.shmr_ec_reconstruct_blocks_host(self._h, ptrs, _ptr(pr), n, L, int(data_only), devs,
                                                     len(devices)))
        del keep


class Op:
    """A started call (shmr_ec_*_start): ``wait()`` completes it and raises on
    its status; the arguments are kept alive until then."""

    def __init__(self, L, op, keep):
        self._L, self._op, self._keep = L, op, keep

    def wait(self) -> None:
        op, self._op = self._op, None
        if op:
            rc = self._L.shmr_ec_op_wait(op)
            self._keep = None
            _check(rc)

    def __del__(self):
        op = getattr(self, "_op", None)
        if op:
            self._L.shmr_ec_op_wait(op)


class PinnedBuffer:
    """Page-locked host memory from shmr_ec_host_alloc (Block Cache buffers):
    host-buffer entry points DMA it without a staging copy."""

    def __init__(self, nbytes: int):
        self._L = lib()
        p = ctypes.c_void_p()
        _check(self._L.shmr_ec_host_alloc(nbytes, ctypes.byref(p)))
        self._p = p
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(nbytes,))

    def __del__(self):
        p = getattr(self, "_p", None)
        if p:
            self.array = None
            self._L.shmr_ec_host_free(p)
            self._p = None


class _DeviceView:
    """One ``__cuda_array_interface__`` view of a DeviceBuffer; the tensor made
    from it holds this object, which holds the buffer."""

    def __init__(self, buf, shape):
        self.buf = buf
        self.__cuda_array_interface__ = {"shape": shape, "typestr": "|u1", "data": (int(buf._p.value), False),
                                         "version": 2, "strides": None}


class DeviceBuffer:
    """VRAM for block batches from shmr_ec_device_alloc; ``contiguous=True``
    asks for physically contiguous memory (large page fragments: fewer
    translation misses on multi-GiB batches).  ``tensor(shape)`` views it as
    a torch.uint8 CUDA tensor (``__cuda_array_interface__``) for the
    ``*_batch_dev`` entry points; the view keeps the buffer alive."""

    def __init__(self, nbytes: int, device: int = 0, contiguous: bool = True):
        self._L = lib()
        p = ctypes.c_void_p()
        _check(self._L.shmr_ec_device_alloc(device, nbytes, int(bool(contiguous)), ctypes.byref(p)))
        self._p = p
        self.nbytes = nbytes
        self.device = device
        self.contiguous = bool(contiguous)

    def tensor(self, shape=None):
        import torch
        shape = tuple(int(n) for n in shape) if shape is not None else (self.nbytes,)
        if int(np.prod(shape)) > self.nbytes:
            raise ValueError(f"view of {shape} exceeds the {self.nbytes}-byte buffer")
        return torch.as_tensor(_DeviceView(self, shape), device=torch.device("cuda", self.device))

    def __del__(self):
        p = getattr(self, "_p", None)
        if p:
            self._L.shmr_ec_device_free(self.device, p)
            self._p = None


def _slot_pitch(shard_len: int) -> int:
    """The allocator's slot pitch: shard_len rounded up
    to 4 KiB, one page more when that is a multiple of 64 KiB."""
    p = (shard_len + 4095) // 4096 * 4096
    return p + 4096 if p % 65536 == 0 else p


class ShardSlab:
    """Shard buffers from shmr_ec_device_alloc_shards: ``nblocks`` x
    ``shards_per_block`` buffers of ``shard_len`` bytes at the slot pitch of the
    device-resident batches (4 KiB-aligned slots, one page more for a
    power-of-two stride), carved from one device slab -- a device Block Cache
    for the crate's buffer-per-shard shape (reference src/vfs/block.rs:408-419).
    ``ptrs`` is the uint64 address table [nblocks * shards_per_block];
    ``shard(b, i)`` a 1-D uint8 tensor view of one shard; ``tensor()`` the
    whole slab as [nblocks, shards_per_block, pitch]."""

    def __init__(self, nblocks: int, shards_per_block: int, shard_len: int, device: int = 0):
        self._L = lib()
        n = nblocks * shards_per_block
        arr = (_u8p * max(n, 1))()
        _check(self._L.shmr_ec_device_alloc_shards(int(device), int(nblocks), int(shards_per_block), int(shard_len),
                                                    arr))
        self.ptrs = np.array([ctypes.cast(arr[j], ctypes.c_void_p).value for j in range(n)], dtype=np.uint64)
        self._first = arr[0]
        self.nblocks, self.shards_per_block, self.shard_len, self.device = nblocks, shards_per_block, shard_len, device
        self.pitch = int(self.ptrs[1] - self.ptrs[0]) if n > 1 else _slot_pitch(shard_len)
        self._views = []

    def tensor(self):
        import torch
        view = _RawView(self, int(self.ptrs[0]), (self.nblocks, self.shards_per_block, self.pitch))
        return torch.as_tensor(view, device=torch.device("cuda", self.device))

    def shard(self, b: int, i: int):
        import torch
        view = _RawView(self, int(self.ptrs[b * self.shards_per_block + i]), (self.shard_len,))
        return torch.as_tensor(view, device=torch.device("cuda", self.device))

    def table(self):
        """ctypes pointer table over ``ptrs`` (valid while the slab lives)."""
        return self.ptrs.ctypes.data_as(ctypes.POINTER(_u8p))

    def __del__(self):
        f = getattr(self, "_first", None)
        if f:
            self._L.shmr_ec_device_free_shards(self.device, f)
            self._first = None


class ShardPool:
    """A device Block Cache of per-block slots (shmr_ec_pool_*): ``alloc()``
    hands out one block's ``shards_per_block`` shard buffers (the lowest free
    slot of a slab of ``slots_per_slab``), ``free(block)`` takes them back.
    A block is a numpy uint64 address array; ``shard(block, i)`` a 1-D uint8
    tensor view.  Tables over pool blocks in any order run the strided kernels
    (the slab's slot lattice)."""

    def __init__(self, shards_per_block: int, shard_len: int, slots_per_slab: int, device: int = 0):
        self._L = lib()
        h = ctypes.c_void_p()
        _check(self._L.shmr_ec_pool_new(int(device), int(shards_per_block), int(shard_len), int(slots_per_slab),
                                        ctypes.byref(h)))
        self._h = h
        self.shards_per_block, self.shard_len, self.device = shards_per_block, shard_len, device

    def alloc(self) -> np.ndarray:
        arr = (_u8p * self.shards_per_block)()
        _check(self._L.shmr_ec_pool_alloc(self._h, arr))
        return np.array([ctypes.cast(arr[i], ctypes.c_void_p).value for i in range(self.shards_per_block)],
                        dtype=np.uint64)

    def free(self, block: np.ndarray) -> None:
        _check(self._L.shmr_ec_pool_free(self._h, ctypes.cast(int(block[0]), _u8p)))

    def shard(self, block: np.ndarray, i: int):
        import torch
        view = _RawView(self, int(block[i]), (self.shard_len,))
        return torch.as_tensor(view, device=torch.device("cuda", self.device))

    def stats(self) -> dict:
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(self._L.shmr_ec_pool_stats(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return {"slabs": int(a.value), "slots": int(b.value), "in_use": int(c.value)}

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.shmr_ec_pool_destroy(h)
            self._h = None


class _RawView:
    """``__cuda_array_interface__`` over part of a ShardSlab (keeps it alive)."""

    def __init__(self, owner, addr, shape):
        self.owner = owner
        self.__cuda_array_interface__ = {"shape": shape, "typestr": "|u1", "data": (addr, False), "version": 2,
                                         "strides": None}


def host_register(arr: np.ndarray) -> None:
    """Page-lock and map an existing C-contiguous host array for zero-copy
    use by the host-buffer entry points (shmr_ec_host_register)."""
    # Register the array's own memory: a reshape of a non-contiguous array would
    # be a temporary copy, whose registration would outlive it.
    if not isinstance(arr, np.ndarray) or not arr.flags["C_CONTIGUOUS"] or not arr.flags["WRITEABLE"]:
        raise TypeError("host_register needs a writable C-contiguous numpy array")
    if arr.nbytes == 0:
        raise ValueError("host_register needs a non-empty array")
    _check(lib().shmr_ec_host_register(ctypes.c_void_p(arr.ctypes.data), arr.nbytes))


def host_unregister(arr: np.ndarray) -> None:
    _check(lib().shmr_ec_host_unregister(ctypes.c_void_p(arr.ctypes.data)))


def path_stats():
    """(zero_copy_blocks, staged_blocks) served by the host-buffer entry points."""
    z, st = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().shmr_ec_path_stats(ctypes.byref(z), ctypes.byref(st)))
    return int(z.value), int(st.value)


DEVICE_COUNTERS = ("blocks_encoded", "blocks_reconstructed", "launches", "plan_images", "upload_rings",
                   "staging_streams", "blocking_calls", "ptr_table_hits", "capture_tables", "capture_released",
                   "ptr_table_grids")


def device_init(device: int = 0) -> None:
    """One-time per-device initialisation (shmr_ec_device_init): after it the
    device-resident entry points make no blocking HIP call and can be
    captured into a graph."""
    _check(lib().shmr_ec_device_init(int(device)))


def capture_reserve(bytes_: int, device: int = 0) -> None:
    """shmr_ec_capture_reserve: make sure one free range of ``bytes_`` exists in
    the device's capture reserve (the tables of captured calls; a capture never
    grows it).  Blocking; call it before the capture."""
    _check(lib().shmr_ec_capture_reserve(int(device), int(bytes_)))


QUEUE_COUNTERS = ("requests", "batches", "max_batch", "sleeps", "early")


def queue_stats(device: int = 0) -> dict:
    """Submission-queue counters of a device ID (include/shmr_ec.h SHMR_EC_Q_*)."""
    out = (ctypes.c_uint64 * len(QUEUE_COUNTERS))()
    _check(lib().shmr_ec_queue_stats(int(device), out, len(QUEUE_COUNTERS)))
    return {name: int(out[i]) for i, name in enumerate(QUEUE_COUNTERS)}


def device_stats(device: int) -> dict:
    """Per-device counters of the current library (include/shmr_ec.h
    SHMR_EC_DEV_*): work done on that device ID and the per-device objects
    (plan images, upload rings, staging streams) created for it."""
    out = (ctypes.c_uint64 * len(DEVICE_COUNTERS))()
    _check(lib().shmr_ec_device_stats(int(device), out, len(DEVICE_COUNTERS)))
    return {name: int(out[i]) for i, name in enumerate(DEVICE_COUNTERS)}
