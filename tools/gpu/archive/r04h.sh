#!/bin/bash
# Round 4 (session 8): allocations in one thread while another captures -- the library before
# (tools/_pre) and after the relaxed-mode fix -- then the capture tests and the 120 s soak.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 240 python -u tools/capture_concurrency.py --lib tools/_pre/libshmr_ec.so > $O/probe_pre.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/capture_concurrency.py > $O/probe_fixed.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_capture.py > $O/pytest_capture.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/soak.py --seconds 120 --threads 12 > $O/soak.log 2>&1 || exit $?
echo done-h
