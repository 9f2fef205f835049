#!/bin/bash
# Round 4 (session 10): every entry point under the relaxed capture mode -- allocations in one
# thread while another captures (both capture modes), the capture tests, and the 120 s soak.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_capture.py > $O/pytest_capture.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/soak.py --seconds 120 --threads 12 > $O/soak.log 2>&1 || exit $?
echo done-j
