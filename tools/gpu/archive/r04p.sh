#!/bin/bash
# Round 4 (session 16): config 5 on three host-code builds, interleaved on one box -- no mirrored
# events (871d9b5), every readiness event mirrored through the private stream (996eb72), mirrored
# only for callers' streams (library-owned streams record their own) -- then the capture, soak
# slice and zero-copy tests on the last.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04p
mkdir -p $O /tmp/vb
for rep in 1 2; do
  for v in no_mirror mirror_all own; do
    timeout -k 10 400 tools/_abm/$v/shmr_vfs_bench /tmp/vb 256 4 0 3 >> $O/vf_$v.jsonl 2>> $O/vf.err || exit $?
  done
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_capture.py tests/test_gpu_soak.py tests/test_gpu_zero_copy.py > $O/pytest.log 2>&1 || exit $?
echo done-p
