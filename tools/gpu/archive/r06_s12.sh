#!/bin/bash
# r06 session 12: the soak slice failed in s11 (an exception in op 3); tracebacks now recorded
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s12
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_soak.py > $O/pytest_soak.log 2>&1
timeout -k 10 120 python -u tools/soak.py --seconds 30 --threads 12 --ops 8,9 > $O/soak_pool.jsonl 2>&1 || exit $?
timeout -k 10 120 python -u tools/soak.py --seconds 30 --threads 12 --ops 3,7 > $O/soak_37.jsonl 2>&1 || exit $?
echo done-s12
