#!/bin/bash
# Round 4 (session 12): the full 12-thread soak with HIP's API log filtered to failed calls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04l
mkdir -p $O
AMD_LOG_LEVEL=3 AMD_LOG_MASK=1 timeout -k 10 200 python -u tools/soak.py --seconds 90 --threads 12 > $O/soak.log 2> >(python -u tools/hiplog_filter.py > $O/hip_errors.txt)
rc=$?
sleep 5
echo "soak rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo done-l
