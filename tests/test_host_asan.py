"""The C++ StorageBlock mirror's CPU cases under AddressSanitizer,
LeakSanitizer and UBSan, on the CPU.

tests/test_host_cpp.py runs the same cases against the plain build; here
shmr_amd/host/{vfs,record,vfs_test}.cpp are compiled with the sanitizers (the
codec library they link stays uninstrumented: none of these cases reaches the
GPU) and any report fails the case.  Leak detection is on -- it found a leak on
the error path of the topology record parser (GCC 11 does not destroy the
members a braced aggregate initialiser already built when a later one throws).
The GPU cases run under the sanitizers on the GPU box (tools/asan_host.sh).
"""
import os
import subprocess

import pytest

from test_host_cpp import CPU_CASES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "shmr_amd", "_lib")


@pytest.fixture(scope="module")
def asan_bin(tmp_path_factory):
    if not os.path.exists(os.path.join(LIB, "libshmr_ec.so")):
        pytest.fail("shmr_amd/_lib/libshmr_ec.so not built (run __graft_entry__.build())")
    exe = str(tmp_path_factory.mktemp("asan") / "vfs_test_asan")
    host = os.path.join(ROOT, "shmr_amd", "host")
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "include"), "-I", host,
           os.path.join(host, "vfs_test.cpp"), os.path.join(host, "vfs.cpp"), os.path.join(host, "record.cpp"),
           "-L", LIB, "-lshmr_ec", f"-Wl,-rpath,{LIB}", "-lpthread", "-o", exe]
    subprocess.run(cmd, check=True, timeout=600)
    return exe


@pytest.mark.parametrize("case", CPU_CASES)
def test_cpu_case_under_sanitizers(asan_bin, case, tmp_path):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([asan_bin, case, str(tmp_path)], capture_output=True, text=True, timeout=600, env=env)
    out = p.stdout.strip().splitlines()
    assert p.returncode == 0 and out and out[-1] == "PASS", f"{case}: rc={p.returncode}\n{p.stdout[-2000:]}\n" \
                                                            f"{p.stderr[-4000:]}"
    assert "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-4000:]
