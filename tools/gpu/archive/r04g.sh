#!/bin/bash
# Round 4 (session 7): 120 s soak of every entry point incl. started calls and graph captures
# (captures gated against the legacy default stream, tools/soak.py CaptureGate).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 300 python -u tools/soak.py --seconds 120 --threads 12 > $O/soak.log 2>&1 || exit $?
echo done-g
