#!/bin/bash
# Pointer-table layout: early-prologue / store-policy A/Bs (tools build), plus the affected GPU tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10 300"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptrs.py tests/test_gpu_compact.py \
  tests/test_gpu_capture.py > gpurun_out/pytest_ptrs2.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
$T python tools/tune.py --config encode83 --ptrs --rounds 9 \
  --variants "depth=2,nt_load=1,nt_store=1;depth=2,early=1,nt_load=1,nt_store=1" > gpurun_out/ptrs_encode83.txt 2>&1 || exit $?
E="chunks=2,depth=2,nt_load=1,nt_store=1,wave_run=1,fuse_tail=1"
$T python tools/tune.py --config encode104 --ptrs --rounds 9 \
  --variants "$E;$E,early=1,serial=1" > gpurun_out/ptrs_encode104.txt 2>&1 || exit $?
D="depth=2,nt_load=1,peel=1"
$T python tools/tune.py --config decode83 --ptrs --rounds 9 \
  --variants "$D,nt_store=1;$D,nt_store=1,wgs_per_cu=7;$D,sc1_store=1;$D,early=1,nt_store=1;$D,early=1,sc1_store=1" \
  > gpurun_out/ptrs_decode83.txt 2>&1 || exit $?
D="depth=2,nt_load=1,peel=1,fuse_tail=1"
$T python tools/tune.py --config decode104 --ptrs --rounds 9 \
  --variants "$D,nt_store=1;$D,sc1_store=1;$D,early=1,nt_store=1;$D,early=1,sc1_store=1" \
  > gpurun_out/ptrs_decode104.txt 2>&1
