"""CPU tests of the C ABI (include/shmr_ec.h): the library loads, exports every
declared symbol, and its host-side logic (no GPU compute) matches the oracle
and the crate's error behaviour.  No kernel is launched here.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import shmr_amd
from shmr_amd import _native
from oracle import rs_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "shmr_ec.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(shmr_ec_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for required in ("shmr_ec_new", "shmr_ec_free", "shmr_ec_encode", "shmr_ec_reconstruct",
                     "shmr_ec_shard_size", "shmr_ec_encode_batch_dev", "shmr_ec_reconstruct_batch_dev"):
        assert required in fns


@pytest.mark.parametrize("flavour", ["product", "tools"])
def test_library_exports_every_declared_symbol(flavour):
    lib = _native._load(flavour)
    for fn in declared_functions():
        assert hasattr(lib, fn), fn
    out = subprocess.run(["nm", "-D", "--defined-only", _native._PATHS[flavour]], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (shmr_ec_\w+)", out))
    assert set(declared_functions()) <= exported


def test_python_signatures_cover_header():
    assert {name for name, _, _ in _native.SIGNATURES} == set(declared_functions())


def test_library_is_gfx950_code_object():
    """The fat binary carries a gfx950 (MI355X) device code object and no other target."""
    data = open(_native.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", data))
    assert targets == {b"gfx950"}


def test_header_compiles_as_c():
    src = '#include "shmr_ec.h"\nint main(void){shmr_ec_t* r=0; return shmr_ec_new(8,3,&r) == 0 ? 0 : 1;}\n'
    path = "/tmp/shmr_abi_check.c"
    with open(path, "w") as f:
        f.write(src)
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-c", "-I", os.path.join(ROOT, "include"), path,
                        "-o", "/tmp/shmr_abi_check.o"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_status_names_match_crate_variants():
    lib = _native.lib()
    names = {c: lib.shmr_ec_status_name(c).decode() for c in range(-13, 1)}
    assert names[-1] == "TooFewShards" and names[-2] == "TooManyShards"
    assert names[-3] == "TooFewDataShards" and names[-5] == "TooFewParityShards"
    assert names[-9] == "IncorrectShardSize" and names[-10] == "TooFewShardsPresent"
    assert names[-11] == "EmptyShard" and names[0] == "Ok"


@pytest.mark.parametrize("length,k", [(1 << 20, 4), (4 << 20, 8), (16 << 20, 10), (7000, 4), (16777217, 8),
                                      (16777221, 10), (1, 7), (0, 3), (2 ** 40 + 3, 13), (123456789, 5)])
def test_shard_size_matches_oracle(length, k):
    assert shmr_amd.calculate_shard_size(length, k) == O.calculate_shard_size(length, k)


def test_shard_size_random_sweep():
    rng = np.random.default_rng(0)
    for length, k in zip(rng.integers(1, 1 << 34, 2000), rng.integers(1, 256, 2000)):
        assert shmr_amd.calculate_shard_size(int(length), int(k)) == O.calculate_shard_size(int(length), int(k))


def test_new_errors_match_crate():
    for (k, p), name in [((0, 1), "TooFewDataShards"), ((1, 0), "TooFewParityShards"),
                         ((200, 57), "TooManyShards"), ((255, 2), "TooManyShards")]:
        with pytest.raises(shmr_amd.Error) as e:
            shmr_amd.ReedSolomon(k, p)
        assert e.value.name == name
    r = shmr_amd.ReedSolomon(255, 1)
    assert (r.data_shard_count(), r.parity_shard_count(), r.total_shard_count()) == (255, 1, 256)


@pytest.mark.parametrize("k,p", [(4, 2), (8, 3), (10, 4), (5, 5), (1, 1), (17, 3), (128, 128)])
def test_matrix_matches_oracle(k, p):
    assert (shmr_amd.ReedSolomon(k, p).matrix() == O.build_matrix(k, k + p)).all()


@pytest.mark.parametrize("k,p", [(8, 3), (10, 4), (4, 3)])
def test_reconstruct_plan_rows_match_oracle(k, p):
    """The GPU runs one fused matrix per erasure pattern: rows of the inverted
    sub-matrix for absent data, and M[parity] * Dec for absent parity -- the
    same bytes the crate gets by rebuilding data then re-encoding parity."""
    import itertools
    rs = shmr_amd.ReedSolomon(k, p)
    m = O.build_matrix(k, k + p)
    for n in range(1, p + 1):
        for miss in list(itertools.combinations(range(k + p), n))[:40]:
            present = [i not in miss for i in range(k + p)]
            for data_only in (False, True):
                in_idx, out_idx, rows = rs.reconstruct_plan(present, data_only)
                valid = [i for i in range(k + p) if present[i]][:k]
                assert in_idx == valid
                dec = O.mat_invert(m[valid])
                want_idx = [i for i in miss if i < k] + ([] if data_only else [i for i in miss if i >= k])
                assert out_idx == want_idx
                for r, j in enumerate(out_idx):
                    want = dec[j] if j < k else O.mat_mul(m[j:j + 1], dec)[0]
                    assert (rows[r] == want).all(), (miss, j)


def test_reconstruct_plan_checks():
    rs = shmr_amd.ReedSolomon(4, 2)
    assert rs.reconstruct_plan([1] * 6)[1] == []                  # all present: nothing to do
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct_plan([1, 1, 1, 0, 0, 0])
    assert e.value.name == "TooFewShardsPresent"
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct_plan([1] * 5)
    assert e.value.name == "TooFewShards"


def test_encode_validation_precedes_device_use():
    """The crate's checks (count, then empty, then equal lengths) run before any
    device is touched, in the crate's order."""
    rs = shmr_amd.ReedSolomon(3, 2)
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode([np.zeros(4, np.uint8)] * 4)
    assert e.value.name == "TooFewShards"
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode([np.zeros(4, np.uint8)] * 6)
    assert e.value.name == "TooManyShards"
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode([np.zeros(0, np.uint8) for _ in range(5)])
    assert e.value.name == "EmptyShard"
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode([np.zeros(4, np.uint8) for _ in range(4)] + [np.zeros(5, np.uint8)])
    assert e.value.name == "IncorrectShardSize"


def test_reconstruct_validation_precedes_device_use():
    rs = shmr_amd.ReedSolomon(3, 2)
    full = [np.arange(4, dtype=np.uint8) for _ in range(5)]
    same = [x.copy() for x in full]
    rs.reconstruct(same)                                          # all present: no-op, no device
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct([full[0], None, None, None, full[4]])
    assert e.value.name == "TooFewShardsPresent"
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct([full[0], np.zeros(3, np.uint8), None, full[3], full[4]])
    assert e.value.name == "IncorrectShardSize"
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct([np.zeros(0, np.uint8), None, full[2], full[3], full[4]])
    assert e.value.name == "EmptyShard"


def test_ptrs_dev_validation_precedes_device_use():
    """The pointer-table entry points check their arguments before any device
    work (no GPU needed): NULL table / presence flags, empty shards, NULL shards
    a call would touch, too few present shards; a well-formed call without a
    GPU reports NoDevice (no CPU fallback).  Fake device addresses are never
    dereferenced on the host."""
    import ctypes
    L = _native.lib()
    rs = shmr_amd.ReedSolomon(4, 2)
    h = rs._h
    u8p = _native._u8p
    fake = [ctypes.cast(ctypes.c_void_p(0x100000 + 0x1000 * i), u8p) for i in range(6)]
    tab = (u8p * 6)(*fake)
    pr = np.array([1, 1, 1, 1, 1, 0], np.uint8)
    prp = pr.ctypes.data_as(u8p)
    assert L.shmr_ec_encode_ptrs_dev(None, tab, 1, 64, 0, None) == -100
    assert L.shmr_ec_encode_ptrs_dev(h, None, 1, 64, 0, None) == -100
    assert L.shmr_ec_encode_ptrs_dev(h, tab, 0, 64, 0, None) == 0           # nothing to do
    assert L.shmr_ec_encode_ptrs_dev(h, tab, 1, 0, 0, None) == -11          # EmptyShard
    nulls = (u8p * 6)(*(fake[:5] + [u8p()]))
    assert L.shmr_ec_encode_ptrs_dev(h, nulls, 1, 64, 0, None) == -100
    assert L.shmr_ec_reconstruct_ptrs_dev(h, tab, None, 1, 64, 0, 0, None) == -100
    few = np.array([1, 1, 1, 0, 0, 0], np.uint8)
    assert L.shmr_ec_reconstruct_ptrs_dev(h, tab, few.ctypes.data_as(u8p), 1, 64, 0, 0, None) == -10
    # data_only: the absent parity shard may be NULL
    ok = L.shmr_ec_reconstruct_ptrs_dev(h, nulls, prp, 1, 64, 1, 0, None)
    assert ok in (0, -101)                  # all data present: nothing to rebuild, no device needed
    assert L.shmr_ec_reconstruct_ptrs_dev(h, nulls, prp, 1, 64, 0, 0, None) == -100
    import torch
    if not torch.cuda.is_available():
        assert L.shmr_ec_encode_ptrs_dev(h, tab, 1, 64, 0, None) == -101   # NoDevice
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode_ptrs_dev([[None] * 5])
    assert e.value.name == "TooFewShards"
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct_ptrs_dev([[None] * 7])
    assert e.value.name == "TooManyShards"
    with pytest.raises(TypeError):
        rs.encode_ptrs_dev([[torch.zeros(64, dtype=torch.uint8) for _ in range(6)]])   # host tensors


def test_alloc_shards_argument_checks():
    """shmr_ec_device_alloc_shards / _free_shards: bad arguments are refused
    before any device work; without a GPU a well-formed allocation reports
    NoDevice; only a slab base the library handed out can be freed (a NULL
    first pointer is a no-op)."""
    import ctypes
    import torch
    L = _native.lib()
    u8p = _native._u8p
    arr = (u8p * 8)()
    assert L.shmr_ec_device_alloc_shards(0, 0, 4, 64, arr) == -100
    assert L.shmr_ec_device_alloc_shards(0, 2, 0, 64, arr) == -100
    assert L.shmr_ec_device_alloc_shards(0, 2, 4, 0, arr) == -100
    assert L.shmr_ec_device_alloc_shards(0, 2, 4, 64, None) == -100
    assert L.shmr_ec_device_alloc_shards(0, 1 << 40, 1 << 30, 64, arr) == -100   # count overflows
    if not torch.cuda.is_available():
        assert L.shmr_ec_device_alloc_shards(0, 2, 4, 64, arr) == -101           # NoDevice
    assert L.shmr_ec_device_free_shards(0, None) == 0
    assert L.shmr_ec_device_free_shards(0, ctypes.cast(ctypes.c_void_p(0x7000), u8p)) == -100


def test_compute_without_gpu_fails_loudly():
    """No CPU fallback: on a machine without a GPU the compute entry points
    report NoDevice instead of computing anything."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    rs = shmr_amd.ReedSolomon(3, 2)
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode([np.zeros(4, np.uint8) for _ in range(5)])
    assert e.value.name == "NoDevice"
    assert shmr_amd.device_count() == 0
    for contiguous in (False, True):
        with pytest.raises(shmr_amd.Error) as e:
            shmr_amd.DeviceBuffer(1 << 20, contiguous=contiguous)
        assert e.value.name == "NoDevice"


def test_tuning_api():
    # product library: kernel knobs are the measured policy; a knob can only be
    # "set" to its default (the restore pattern of callers), nothing else
    assert _native.lib().shmr_ec_is_tools_build() == 0
    assert b"product" in _native.lib().shmr_ec_version()
    for key, default in (("encode.chunks", -2), ("chunks", -2), ("grid", -1), ("threads", 256), ("diag", 0),
                         ("decode.depth", -2), ("occ8", 0), ("uvec", -2)):
        shmr_amd.set_tuning(**{key: default})
    for key, value in (("encode.chunks", 2), ("diag", 1), ("decode.diag", 1), ("depth", 3), ("grid", 0),
                       ("threads", 512), ("spre", 1), ("occ8", 1), ("uvec", 1)):
        with pytest.raises(shmr_amd.Error) as e:
            shmr_amd.set_tuning(**{key: value})
        assert e.value.name == "InvalidArgument", key
    with pytest.raises(shmr_amd.Error):
        shmr_amd.set_tuning(no_such_knob=1)
    # uvec=0 (the realigning kernels a device without the unaligned access mode
    # runs: exact results) is a product knob; uvec=1 stays tools-only
    shmr_amd.set_tuning(uvec=0)
    assert shmr_amd.get_tuning("uvec") == 0
    shmr_amd.set_tuning(uvec=-2)
    assert "diag=0" in shmr_amd.describe_variant(False, 8, 3)
    # the measured policy: 4 output rows -> 2 chunks/lane; NT loads and stores; ring depth 2
    assert "chunks=2" in shmr_amd.describe_variant(False, 10, 4)
    assert "nt_load=1 nt_store=1" in shmr_amd.describe_variant(False, 4, 2)
    assert "nt_load=1" in shmr_amd.describe_variant(True, 8, 1)
    assert "depth=2" in shmr_amd.describe_variant(True, 8, 1)
    assert "early=1" in shmr_amd.describe_variant(False, 4, 2)
    assert "early=1" in shmr_amd.describe_variant(False, 8, 3)
    assert "early=0" in shmr_amd.describe_variant(False, 10, 3)
    assert "early=0" in shmr_amd.describe_variant(True, 4, 2)
    assert "fuse_tail=1" in shmr_amd.describe_variant(False, 10, 4)
    assert "fuse_tail=1" in shmr_amd.describe_variant(True, 10, 2)
    # reconstructs into a compact output (decode=2) store with sc1, no residency cap
    assert "sc1_store=1" in shmr_amd.describe_variant(2, 10, 2)
    # reconstructs peel the shard ring's tail; encodes keep the look-ahead
    assert "peel=1" in shmr_amd.describe_variant(2, 10, 2) and "peel=1" in shmr_amd.describe_variant(True, 8, 1)
    assert "peel=1" not in shmr_amd.describe_variant(False, 8, 3)
    # U = 2 launches (4-row encodes and rebuilds) take wave-contiguous runs
    assert "wave_run=1" in shmr_amd.describe_variant(False, 10, 4) and "wave_run=1" in shmr_amd.describe_variant(True, 10, 4)
    assert "wave_run=1" not in shmr_amd.describe_variant(False, 8, 3)
    assert "nt_store=0" in shmr_amd.describe_variant(2, 8, 1) and "wgs_per_cu=0" in shmr_amd.describe_variant(2, 8, 1)
    assert "sc1_store" not in shmr_amd.describe_variant(True, 8, 1)
    shmr_amd.set_tuning(sc1_store=-2)
    with pytest.raises(shmr_amd.Error):
        shmr_amd.set_tuning(sc1_store=0)
    saved = shmr_amd.get_tuning("bounce_kib")
    try:
        shmr_amd.set_tuning(bounce_kib=0)
        assert shmr_amd.get_tuning("bounce_kib") == 0
        shmr_amd.set_tuning(bounce_kib=-2)
        assert shmr_amd.get_tuning("bounce_kib") == 8192       # auto: 8 MiB blocks bounce (measured crossover)
        with pytest.raises(shmr_amd.Error):
            shmr_amd.set_tuning(bounce_kib=-5)
    finally:
        shmr_amd.set_tuning(bounce_kib=saved)
    # host-path knobs: set, read back, reset to the measured defaults
    for knob, value, default in (("ptrs_direct", 0, 16), ("sync_spin_us", 50, 0), ("mirror_zc", 0, 1), ("ptrs_segs", 0, 1)):
        shmr_amd.set_tuning(**{knob: value})
        assert shmr_amd.get_tuning(knob) == value
        shmr_amd.set_tuning(**{knob: -2})
        assert shmr_amd.get_tuning(knob) == default
    with pytest.raises(shmr_amd.Error):
        shmr_amd.set_tuning(ptrs_direct=-7)


def test_auto_policy_variants_are_compiled():
    """Every shape the auto policy can pick maps to a compiled kernel."""
    for decode in (0, 1, 2, 3, 4):   # 3 / 4: the *_ptrs_dev calls
        for k in range(1, 33):
            for rows in range(1, 5):
                d = shmr_amd.describe_variant(decode, k, rows)
                assert "compiled=1" in d, (decode, k, rows, d)
    assert "depth=2" in shmr_amd.describe_variant(False, 8, 3)


def test_native_library_is_required():
    """The package refuses to run without the in-tree .so (no fallback)."""
    assert os.path.exists(_native.LIB_PATH)
    assert _native.LIB_PATH.startswith(os.path.join(ROOT, "shmr_amd"))
    saved_paths, saved_libs = dict(_native._PATHS), dict(_native._libs)
    try:
        _native._libs.clear()
        _native._PATHS["product"] = "/nonexistent/libshmr_ec.so"
        with pytest.raises(_native.NativeLibraryMissing):
            _native.lib()
    finally:
        _native._PATHS.clear()
        _native._PATHS.update(saved_paths)
        _native._libs.clear()
        _native._libs.update(saved_libs)


def test_tools_build_is_separate():
    """Measurement-only variants (and the XOR-only diagnostic kernel) live in
    libshmr_ec_tools.so; objects keep the library they were created with."""
    with _native.tools() as T:
        assert T.shmr_ec_is_tools_build() == 1 and b"tools" in T.shmr_ec_version()
        # the tools ID hashes the product kernel TU and the tools-only TU
        assert re.fullmatch(rb"[0-9a-f]{12}", T.shmr_ec_build_id())
        assert T.shmr_ec_build_id() != _native._load("product").shmr_ec_build_id()
        saved = shmr_amd.get_tuning("encode.chunks")
        try:
            shmr_amd.set_tuning(**{"encode.chunks": 2})
            assert shmr_amd.get_tuning("encode.chunks") == 2
            assert "chunks=2" in shmr_amd.describe_variant(False, 8, 3)
            shmr_amd.set_tuning(**{"encode.diag": 1})
            assert "diag=1" in shmr_amd.describe_variant(False, 8, 3)
            with pytest.raises(shmr_amd.Error):
                shmr_amd.set_tuning(chunks=3)
            rs = shmr_amd.ReedSolomon(8, 3)
        finally:
            shmr_amd.set_tuning(**{"encode.chunks": saved, "encode.diag": 0})
    assert rs._L is _native._libs["tools"]
    assert shmr_amd.ReedSolomon(8, 3)._L is _native._libs["product"]
    assert _native.flavour() == "product"
    # the tools knobs never reached the product library
    assert shmr_amd.get_tuning("encode.chunks") == -2 and shmr_amd.get_tuning("encode.diag") == 0


def test_build_id_is_a_kernel_hash():
    bid = _native.lib().shmr_ec_build_id().decode()
    assert re.fullmatch(r"[0-9a-f]{12}", bid), bid


def test_host_register_rejects_non_contiguous():
    """A non-contiguous array would be registered through a temporary copy;
    the shim refuses it before any device call (no GPU needed)."""
    a = np.zeros((8, 8), np.uint8)[:, ::2]
    with pytest.raises(TypeError):
        shmr_amd.host_register(a)
    ro = np.zeros(16, np.uint8)
    ro.flags.writeable = False
    with pytest.raises(TypeError):
        shmr_amd.host_register(ro)
    with pytest.raises(ValueError):
        shmr_amd.host_register(np.zeros(0, np.uint8))


def test_batch_tensor_bounds_checked_before_launch():
    """The device-batch shim checks dtype, shard count and shard size against the
    tensors before the raw-pointer ABI call (a short tensor would be an
    out-of-bounds kernel access), then refuses memory the GPU cannot address."""
    import torch
    rs = shmr_amd.ReedSolomon(4, 2)
    data = torch.zeros((3, 4, 1024), dtype=torch.uint8)
    parity = torch.zeros((3, 2, 1024), dtype=torch.uint8)
    with pytest.raises(TypeError):
        rs.encode_batch_dev(data.float(), parity)
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode_batch_dev(data[:, :3], parity)
    assert e.value.name == "TooFewShards"
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode_batch_dev(data, torch.zeros((3, 3, 1024), dtype=torch.uint8))
    assert e.value.name == "TooManyShards"
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode_batch_dev(data, parity, shard_len=1025)
    assert e.value.name == "IncorrectShardSize"
    with pytest.raises(shmr_amd.Error) as e:                     # 2-D block rows too short for the pitch
        rs.encode_batch_dev(torch.zeros((3, 4000), dtype=torch.uint8), parity, shard_len=1000,
                            data_shard_pitch=1024)
    assert e.value.name == "IncorrectShardSize"
    with pytest.raises(ValueError):
        rs.encode_batch_dev(data, parity[:2])
    with pytest.raises(TypeError):                               # well formed, but pageable host memory
        rs.encode_batch_dev(data, parity, shard_len=1000)
    shards = torch.zeros((3, 6, 1024), dtype=torch.uint8)
    present = np.ones((3, 6), np.uint8)
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct_batch_dev(shards[:, :5], present[:, :5])
    assert e.value.name == "TooFewShards"
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct_batch_dev(shards, present, shard_len=2048)
    assert e.value.name == "IncorrectShardSize"
    with pytest.raises(ValueError):
        rs.reconstruct_batch_dev(shards, present[:2])
    with pytest.raises(TypeError):
        rs.reconstruct_batch_dev(shards, present)


def test_path_stats_api():
    z, s = shmr_amd.path_stats()
    assert z >= 0 and s >= 0


def _kernel_flags(path):
    """Template flags F of every gf_apply_kernel<R, U, MODE, F> in a library."""
    data = open(path, "rb").read()
    return {int(m) for m in re.findall(rb"gf_apply_kernelILi\d+ELi\d+ELi\d+ELi(\d+)E", data)}


def test_product_library_has_no_diagnostic_kernel():
    """The XOR-only kernel (flag 16, wrong results by design) and the other
    measurement-only instantiations are compiled into the tools build only."""
    KDIAG, KDEPTH2 = 16, 512
    product = _kernel_flags(_native._PATHS["product"])
    tools = _kernel_flags(_native._PATHS["tools"])
    assert product and not any(f & KDIAG for f in product)
    assert any(f & KDIAG for f in tools)
    # every product full-tile kernel (MODE 0) is a depth-2 ring with nontemporal
    # stores, or sc1 stores (reconstructs into a compact output)
    KSC1 = 1 << 23
    assert all(f & KDEPTH2 and (f & 2 or f & KSC1) for f in product if f != 0)
    assert product < tools


def test_device_list_and_stats_api():
    """Device-list checks that precede any device use (CPU-only here): a NULL
    list or ndev <= 0 is InvalidArgument; per-device counters read zero without
    a GPU; alias device IDs exist only in the tools build."""
    import ctypes
    L = _native.lib()
    h = ctypes.c_void_p()
    assert L.shmr_ec_new(8, 3, ctypes.byref(h)) == 0
    shard = np.zeros(4096, np.uint8)
    ptrs = (_native._u8p * 11)(*[shard.ctypes.data_as(_native._u8p)] * 11)
    devs = (ctypes.c_int * 1)(0)
    pr = np.ones(11, np.uint8)
    for d, n in ((None, 1), (devs, 0), (devs, -2)):
        assert L.shmr_ec_encode_blocks_host(h, ptrs, 1, 4096, d, n) == -100
        assert L.shmr_ec_reconstruct_blocks_host(h, ptrs, pr.ctypes.data_as(_native._u8p), 1, 4096, 0, d, n) == -100
    assert L.shmr_ec_set_device(h, -1) == -100
    L.shmr_ec_free(h)
    out = (ctypes.c_uint64 * 7)(*([7] * 7))
    assert L.shmr_ec_device_stats(-1, out, 7) == -100
    assert L.shmr_ec_device_stats(0, None, 7) == -100
    assert L.shmr_ec_device_stats(0, out, 7) == 0 and list(out) == [0] * 7
    assert L.shmr_ec_device_init(0) == -101          # NoDevice (no GPU here)
    assert L.shmr_ec_device_init(-1) in (-100, -101)
    assert shmr_amd.device_stats(3) == {k: 0 for k in shmr_amd.reed_solomon.DEVICE_COUNTERS}
    assert L.shmr_ec_set_tuning(b"alias_devices", 1) == -100
    assert L.shmr_ec_set_tuning(b"alias_devices", 0) == 0
    with _native.tools() as T:
        assert T.shmr_ec_set_tuning(b"alias_devices", 3) == 0 and T.shmr_ec_get_tuning(b"alias_devices") == 3
        assert T.shmr_ec_set_tuning(b"alias_devices", 33) == -100
        assert T.shmr_ec_set_tuning(b"alias_devices", 0) == 0
    assert L.shmr_ec_get_tuning(b"alias_devices") == 0


def test_pointer_table_rows_follow_the_plan():
    """Pointer tables go to the kernels in plan order (input t at [t], output
    row r at [k + r], ec_core permute_ptr_rows): for random presence patterns
    the permuted row names exactly the shards of the reconstruct plan the
    library runs (shmr_ec_reconstruct_plan: the crate's first k present shards,
    then the absent ones -- absent parity only without data_only), and encode
    rows stay as given.  CPU only (the host side of *_ptrs_dev and of the
    zero-copy mapped path)."""
    L = _native.lib()
    fn = L["_ZN4shmr4core16permute_ptr_rowsEPKmPKhmjjbPm"]   # shmr::core::permute_ptr_rows
    fn.restype = None
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_uint, ctypes.c_bool,
                   ctypes.c_void_p]
    rng = np.random.default_rng(404)
    for k, p in ((4, 2), (8, 3), (10, 4), (3, 5), (17, 7)):
        t = k + p
        rs = shmr_amd.ReedSolomon(k, p)
        n = 40
        src = (np.arange(n * t, dtype=np.uint64) + np.uint64(1 << 40)) * np.uint64(16)
        present = np.ones((n, t), np.uint8)
        for b in range(1, n):   # block 0 keeps every shard
            lost = rng.choice(t, size=int(rng.integers(1, p + 1)), replace=False)
            present[b, lost] = 0
        for data_only in (False, True):
            dst = np.zeros(n * t, np.uint64)
            fn(src.ctypes.data, present.ctypes.data, n, k, t, data_only, dst.ctypes.data)
            row = dst.reshape(n, t)
            assert np.array_equal(row[0], src[:t])
            for b in range(1, n):
                in_idx, out_idx, _ = rs.reconstruct_plan(present[b].astype(bool), data_only=data_only)
                base = src[b * t:(b + 1) * t]
                assert np.array_equal(row[b, :k], base[list(in_idx)]), (k, p, b)
                m = len(out_idx)
                assert np.array_equal(row[b, k:k + m], base[list(out_idx)]), (k, p, b)
                assert not row[b, k + m:].any()
        enc = np.zeros(n * t, np.uint64)
        fn(src.ctypes.data, None, n, k, t, False, enc.ctypes.data)
        assert np.array_equal(enc, src)
