#!/bin/bash
# Round 4 (session 9): which HIP calls in one thread break a capture in another (HIP only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 180 python -u tools/capture_probe_hip.py > $O/probe_hip2.log 2>&1 || exit $?
echo done-i
