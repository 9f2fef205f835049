#!/usr/bin/env bash
# Host-side AddressSanitizer + UBSan run of the C++ StorageBlock mirror
# (shmr_amd/host) and of libshmr_ec.so's host code: the sanitizers cover host
# code only (no GPU ASan).  Build here, run on a GPU box:
#
#   tools/asan_host.sh build
#   tools/asan_host.sh run [out_dir]      # every case of shmr_vfs_test
#   (no LeakSanitizer here: leaks are checked on the CPU build, tests/test_host_asan.py -- r06,
#   see the `run` case)
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
PROBE="${ASAN_DIR:-$ROOT/tools/_probe}"   # run: a copy of the build elsewhere (tools/_probe is not uploaded)
BIN="$PROBE/vfs_test_asan"
HIPCC=/opt/rocm/bin/hipcc
CPU_CASES="block_topology_try_from virtual_block_new_block virtual_block_unbuffered_backing virtual_block_unbuffered
virtual_block_buffered virtual_block_erasure_buffered block_errors virtual_file_1 virtual_file_2_4_mb virtual_file_errors
virtual_file_chunk_model erasure_f32_hazard virtual_file_record_roundtrip virtual_file_record_fuzz read_needed_shards_plan"
# GPU cases with the input sizes tests/test_host_cpp.py gives them
GPU_CASES="erasure_block_sync_load:700001 erasure_block_missing_shards:1048576 virtual_file_erasure_batch:6291456
replace_block_erasure:300000 virtual_file_batched_reconstruct:12582912 rewrite_erasure:2109497
virtual_file_mapped_per_block_flush:10485760 erasure_f32_hazard_release:16777217
rewrite_erasure_record_reload:2109497 read_needed_shards:4194304 virtual_block_erasure_fuzz virtual_file_erasure_fuzz
erasure_flush_encode_failure:2097152 direct_io_mapped:4194304 direct_io_pageable:4194304"
case "${1:-}" in
build)
    # libshmr_ec.so's host code (C ABI, launch core, host engine) instrumented
    # too; the kernels are unchanged (-Xarch_host: host compilation only)
    L="$ROOT/tools/_probe/asan_lib"
    mkdir -p "$L"
    SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
    CXXF="-O1 -g -std=c++17 -fPIC -Wall -I$ROOT/include -I$ROOT/shmr_amd/csrc"
    C="$ROOT/shmr_amd/csrc"
    # The kernel TU too (r04): UBSan there used to return wrong parity because
    # -fsanitize=function deleted launches made through a kernel function
    # pointer; launch_one now launches by kernel name, and
    # tests/test_isa.py checks every launch site still pops its configuration.
    $HIPCC $CXXF $SAN --offload-arch=gfx950 -x hip -c "$C/gf_apply.hip" -o "$L/gf_apply.o"
    for f in gf256 ec_core host_engine ptrs submit pool ec_api; do
        $HIPCC $CXXF $SAN -c "$C/$f.cpp" -o "$L/$f.o"
    done
    $HIPCC --offload-arch=gfx950 -shared -fPIC $SAN -o "$L/libshmr_ec.so" "$L"/*.o -Wl,-soname,libshmr_ec.so -lpthread
    rm -f "$L"/*.o
    $HIPCC -O1 -g -std=c++17 $SAN -I"$ROOT/include" -o "$ROOT/tools/_probe/abi_check_asan" "$ROOT/tools/abi_check.cpp" \
        -L"$L" -lshmr_ec -Wl,-rpath,'$ORIGIN/asan_lib'
    $HIPCC -O1 -g -std=c++17 $SAN -Wall -I"$ROOT/include" -I"$ROOT/shmr_amd/host" -o "$BIN" \
        "$ROOT/shmr_amd/host/vfs_test.cpp" "$ROOT/shmr_amd/host/vfs.cpp" "$ROOT/shmr_amd/host/record.cpp" \
        -L"$L" -lshmr_ec -Wl,-rpath,'$ORIGIN/asan_lib' -lpthread
    ;;
run)
    OUT="${2:-$ROOT/gpurun_out/asan}"
    mkdir -p "$OUT"
    # protect_shadow_gap=0: the ROCm runtime maps GPU apertures in the low shadow gap
    # LEAKS=1: LeakSanitizer on, the ROCm runtime's own allocations suppressed
    # (tools/lsan_rocm.supp); this repository's code stays checked
    # LeakSanitizer stays off on the GPU box (r06): twice (r05, profiles/r05/s27) a
    # case passed and then hung at exit with every thread stopped in
    # ptrace_stop by LeakSanitizer's exit-time StopTheWorld, while the leak scan
    # walked a process whose address space holds the ROCm runtime's device
    # apertures; the record lacks the tracer task, so the hang is the checker's
    # or the runtime's, not this code's, and re-running it costs GPU sessions
    # for no finding.  Leaks are checked where no runtime mapping exists: the
    # CPU build of every StorageBlock case under ASan + LSan + UBSan in the CPU
    # suite (tests/test_host_asan.py), which found the one leak there was.
    if [ "${LEAKS:-0}" = 1 ]; then
        echo "LEAKS=1 is not run on the GPU box (see the comment above; tests/test_host_asan.py checks leaks)" >&2
        exit 2
    fi
    export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1
    export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
    fail=0
    T="${CASE_TIMEOUT:-120}"     # seconds per case (LeakSanitizer's exit scan adds to the long cases)
    if timeout -k 10 "$T" "$PROBE/abi_check_asan" > "$OUT/abi_check.log" 2>&1; then
        echo "abi_check PASS"
    else
        echo "abi_check FAIL (see $OUT/abi_check.log)"; exit 1
    fi
    for cs in $CPU_CASES $GPU_CASES; do
        c="${cs%%:*}"
        if [ -n "${ONLY:-}" ] && [[ " $ONLY " != *" $c "* ]]; then continue; fi
        rm -rf "$OUT/b" && mkdir -p "$OUT/b"
        input=()
        if [ "$c" != "$cs" ]; then
            python3 -c "import numpy as np; np.random.default_rng(7).integers(0, 256, ${cs#*:}, dtype=np.uint8).tofile('$OUT/input.bin')"
            input=("$OUT/input.bin")
        fi
        if timeout -k 10 "$T" "$BIN" "$c" "$OUT/b" "${input[@]}" > "$OUT/$c.log" 2>&1 && [ "$(tail -1 "$OUT/$c.log")" = PASS ]; then
            echo "$c PASS"
        else
            echo "$c FAIL (see $OUT/$c.log)"; fail=1
            break
        fi
    done
    rm -rf "$OUT/b" "$OUT/input.bin"
    exit $fail
    ;;
*)
    echo "usage: $0 build | run [out_dir]" >&2; exit 2 ;;
esac
