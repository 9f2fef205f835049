#!/bin/bash
# Round 4 (session 20): does a mirrored event's private-stream wait hold back another stream?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 300 python -u tools/hol_probe.py tools/_hol/libshmr_ec_nomirror.so > $O/hol_probe.txt 2>&1 || exit $?
echo done-t
