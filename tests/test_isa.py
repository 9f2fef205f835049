"""The product code object's memory instructions (CPU-only: disassembles the
gfx950 code object embedded in libshmr_ec.so with the ROCm LLVM tools).

Misaligned device-resident shards (the reference's packed block buffer, shard
i at i * S, src/vfs/block.rs:408-419) run the same vector kernels as aligned
ones.  Their 16-byte accesses go through an under-aligned vector type (well-
defined C++ at any address); this pins that the compiler still lowers every
full-tile kernel's data path to global_load_dwordx4 / global_store_dwordx4 --
no byte-granular or split accesses -- and that the sc1 policy reaches the
compact-output kernels' stores (raw buffer stores: no global-store builtin
takes cache-policy bits).
"""
import os
import re
import subprocess

import pytest

from shmr_amd import _native

LLVM = "/opt/rocm/lib/llvm/bin"


def _disasm(lib_path, tmp_path):
    objcopy, bundler, objdump = (os.path.join(LLVM, n) for n in ("llvm-objcopy", "clang-offload-bundler",
                                                                  "llvm-objdump"))
    if not all(os.path.exists(x) for x in (objcopy, bundler, objdump)):
        pytest.skip("ROCm LLVM tools not available")
    fb, co = str(tmp_path / "lib.fatbin"), str(tmp_path / "lib.co")
    subprocess.check_call([objcopy, f"--dump-section=.hip_fatbin={fb}", lib_path, str(tmp_path / "discard")])
    subprocess.check_call([bundler, "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                           f"--input={fb}", f"--output={co}"])
    text = subprocess.check_output([objdump, "-d", co], text=True)
    kernels, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
        if m:
            cur = m.group(1)
            kernels[cur] = []
        elif cur and line.startswith("\t"):
            ins = line.split("//")[0].strip()
            if ins:
                kernels[cur].append(ins)
    return kernels


@pytest.fixture(scope="module")
def product_kernels(tmp_path_factory):
    return _disasm(_native._PATHS["product"], tmp_path_factory.mktemp("isa"))


def _apply_kernels(kernels):
    out = {}
    for name, body in kernels.items():
        m = re.search(r"gf_apply_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", name)
        if m:
            out[tuple(int(x) for x in m.groups())] = body
    return out


KFUSE, KPTRS, KSC1, KNTSTORE = 1 << 18, 1 << 19, 1 << 23, 2


def test_full_tile_kernels_use_dwordx4(product_kernels):
    """Every full-tile (MODE 0) kernel without the bounds-checked tail form
    moves shard data only with 16-byte vector loads and stores."""
    kern = _apply_kernels(product_kernels)
    full = {key: body for key, body in kern.items() if key[2] == 0 and not key[3] & KFUSE}
    assert len(full) >= 40, len(full)
    for (R, U, mode, F), body in full.items():
        ops = [i.split()[0] for i in body]
        assert "global_load_dwordx4" in ops, (R, U, F)
        store16 = "buffer_store_dwordx4" if F & KSC1 else "global_store_dwordx4"
        assert store16 in ops, (R, U, F)
        # no byte accesses at all; 16-bit loads only read the plan's u16 shard
        # indices (stage_plan), never shard data
        narrow = [o for o in ops if re.fullmatch(r"(global|flat|buffer)_(load_(ubyte|sbyte)|store_(byte|short))\w*", o)]
        assert not narrow, ((R, U, F), narrow[:4])
        # data stores: R outputs x U chunks per lane, all 16-byte
        stores = [o for o in ops if re.match(r"(global|buffer|flat)_store", o)]
        assert set(stores) == {store16}, ((R, U, F), set(stores))


def test_store_cache_policy(product_kernels):
    """sc1 kernels (compact rebuilt-shard outputs) store with sc1 through raw
    buffer stores -- never an inline-asm store, which would hide the >8-byte
    store-data hazard from the compiler -- and nontemporal-store kernels with nt."""
    kern = _apply_kernels(product_kernels)
    sc1 = [(k, b) for k, b in kern.items() if k[2] == 0 and k[3] & KSC1]
    nt = [(k, b) for k, b in kern.items() if k[2] == 0 and k[3] & KNTSTORE and not k[3] & KFUSE]
    assert sc1 and nt
    for key, body in sc1:
        st = [i for i in body if re.match(r"(global|buffer)_store_dwordx4", i)]
        assert st and all(i.startswith("buffer_store_dwordx4") and i.endswith(" sc1") for i in st), (key, st[:2])
    for key, body in nt:
        st = [i for i in body if i.startswith("global_store_dwordx4")]
        assert st and all(re.search(r"\bnt\b", i) for i in st), (key, st[:2])


def test_misaligned_path_kernels_exist(product_kernels):
    """The realigning fallback (MODE 3) and the byte-granular remainder (MODE 2)
    exist for every row count."""
    kern = _apply_kernels(product_kernels)
    for R in (1, 2, 3, 4):
        assert any(k[0] == R and k[2] == 3 for k in kern), R
        assert any(k[0] == R and k[2] == 2 for k in kern), R


def test_inventory_is_the_code_object(product_kernels):
    """shmr_ec_kernel_inventory (what the library can dispatch, derived from the
    launch policy at compile time) lists exactly the gf_apply kernels of the
    product code object -- nothing compiled that the policy cannot select."""
    import shmr_amd
    inv = {(e["rows"], e["chunks"], e["mode"], e["flags"]) for e in shmr_amd.kernel_inventory()}
    assert len(inv) == len(shmr_amd.kernel_inventory())
    assert set(_apply_kernels(product_kernels)) == inv
    # modes 1-3: one kernel per row count
    for mode in (1, 2, 3):
        assert sorted(r for r, u, m, f in inv if m == mode) == [1, 2, 3, 4]
    full = [key for key in inv if key[2] == 0]
    assert all(u == (2 if r == 4 else 1) for r, u, m, f in full), "U = 2 exactly for 4-row launches"


def _host_symbols(path):
    out = subprocess.check_output(["nm", path], text=True)
    stubs, handles = {}, {}
    for line in out.splitlines():
        parts = line.split()
        if len(parts) != 3 or "gf_apply_kernel" not in parts[2]:
            continue
        addr, kind, name = int(parts[0], 16), parts[1], parts[2]
        m = re.search(r"gf_apply_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", name)
        key = tuple(int(x) for x in m.groups())
        (stubs if "__device_stub__" in name else handles)[key] = (addr, kind)
    return stubs, handles


@pytest.mark.parametrize("flavour", ["product", "tools"])
def test_kernel_stubs_and_handles_are_distinct(flavour):
    """Every kernel instantiation has its own host launch stub and its own
    kernel handle (the address hipLaunchKernel passes and
    __hipRegisterFunction binds).  Two instantiations sharing either would make
    one launch run a sibling kernel -- the failure DESIGN.md §3 records for a
    UBSan build of the kernel TU."""
    stubs, handles = _host_symbols(_native._PATHS[flavour])
    assert stubs and set(stubs) == set(handles)
    assert len({a for a, _ in stubs.values()}) == len(stubs)
    assert len({a for a, _ in handles.values()}) == len(handles)
    assert {k for _, k in stubs.values()} <= {"t", "T"} and {k for _, k in handles.values()} <= {"d", "D"}


def _launch_protocol(path):
    """Calls of the HIP launch protocol in the library's own x86 code (outside
    the compiler's __device_stub__ functions): a launch pushes its
    configuration (__hipPushCallConfiguration) and the stub's code -- inlined or
    not -- pops it (__hipPopCallConfiguration) right before hipLaunchKernel."""
    text = subprocess.check_output(["objdump", "-d", "--no-show-raw-insn", path], text=True)
    func, push, pop = "", 0, 0
    for line in text.splitlines():
        h = re.match(r"^[0-9a-f]+ <(.*)>:", line)
        if h:
            func = h.group(1)
            continue
        if "__device_stub__" in func or "@plt" in func:
            continue
        push += "<__hipPushCallConfiguration@plt>" in line
        pop += "<__hipPopCallConfiguration@plt>" in line
    return push, pop


@pytest.mark.parametrize("flavour", ["product", "tools"])
def test_every_launch_reaches_its_kernel(flavour):
    """Every launch site in the library's host code goes on to launch its
    kernel.  Guards the failure DESIGN.md §3 records: with -fsanitize=function
    a kernel launched through a function-pointer variable lost its launch --
    only __hipPushCallConfiguration was left (no kernel ran, no report),
    because the sanitizer reads 8 bytes in front of the kernel handle, which
    the optimizer treats as out of bounds.  gf_tile.hpp launch_one launches by
    kernel name.  (Measured on a host-UBSan build of gf_apply.hip with the
    old pointer launch: 132 pushes, 1 pop; with launches by name: 143 / 143.)"""
    path = _native._PATHS[flavour]
    out = subprocess.check_output(["nm", path], text=True)
    handles = [l for l in out.splitlines() if len(l.split()) == 3 and l.split()[1] in "dD" and "gf_apply_kernel" in l]
    push, pop = _launch_protocol(path)
    assert push == pop and push >= len(handles) > 0, (push, pop, len(handles))
