#!/bin/bash
# Round 5 (session 9): the bench lines with the r05 defaults (K = 100, two-event timed region):
# the headline three times, then every config once.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05i
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python bench.py >> $O/bench_default.jsonl 2>> $O/bench.err || exit $?
done
for c in decode83 encode104 decode104 encode42 codec104; do
  timeout -k 10 300 python bench.py --config $c >> $O/bench_configs.jsonl 2>> $O/bench.err || exit $?
done
echo done-i
