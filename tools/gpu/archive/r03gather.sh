#!/bin/bash
# Pointer-table staging by ds_bpermute gather (current build) against the previous build, in one process.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for c in encode83 decode83 encode104 decode104; do
  timeout -k 10 300 python tools/ab_libs.py tools/ab_prev/libshmr_ec_3869.so --config $c --ptrs --rounds 11 \
    >> gpurun_out/ab_gather.txt 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptrs.py \
  > gpurun_out/pytest_gather.log 2>&1
