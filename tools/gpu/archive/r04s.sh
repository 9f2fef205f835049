#!/bin/bash
# Round 4 (session 19): a 10-minute 12-thread soak of the final library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 800 python -u tools/soak.py --seconds 600 --threads 12 > $O/soak600.log 2>&1 || exit $?
echo done-s
