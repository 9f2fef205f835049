#!/bin/bash
# Round 5 (session 13): a 300 s 12-thread soak of every entry point (slab/grid op included).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 420 python -u tools/soak.py --seconds 300 --threads 12 > $O/soak300.log 2>&1 || exit $?
echo done-m
