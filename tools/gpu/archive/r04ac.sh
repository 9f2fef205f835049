#!/bin/bash
# Round 4 (session 29): the null-stream-during-a-blocking-capture case of the capture tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04ac
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_capture.py > $O/pytest_capture.log 2>&1 || exit $?
echo done-ac
