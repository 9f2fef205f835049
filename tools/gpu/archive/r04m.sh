#!/bin/bash
# Round 4 (session 13): events recorded on a stream before it captures (HIP probe), the regression
# test on the library before (tools/_pre) and after the mirrored events, the capture tests, soak.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 180 python -u tools/capture_probe_hip.py > $O/probe_hip.log 2>&1 || exit $?
T=test_events_recorded_before_a_capture_on_that_stream
timeout -k 10 240 python -u tools/capture_concurrency.py --test $T --lib tools/_pre/libshmr_ec.so > $O/events_pre.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/capture_concurrency.py --test $T > $O/events_fixed.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_capture.py tests/test_gpu_ptrs.py > $O/pytest_capture.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/soak.py --seconds 120 --threads 12 > $O/soak.log 2>&1 || exit $?
echo done-m
