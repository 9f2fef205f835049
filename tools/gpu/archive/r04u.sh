#!/bin/bash
# Round 4 (session 21): the six bench lines on another box (box-to-box ranges for DESIGN §0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04u
mkdir -p $O
for c in encode83 decode83 encode104 decode104 encode42 codec104; do
  timeout -k 10 300 python bench.py --config $c >> $O/bench.jsonl 2>> $O/bench.err || exit $?
done
echo done-u
