#!/bin/bash
# Round 4 (session 27): the capture tests incl. host-buffer calls inside the caller's own capture.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04aa
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_capture.py > $O/pytest_capture.log 2>&1 || exit $?
echo done-aa
