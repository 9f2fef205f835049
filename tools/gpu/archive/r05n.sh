#!/bin/bash
# Round 5 (session 14): the final tree -- the whole GPU suite, smoke, the
# default bench line (as the driver runs it) and one line per BASELINE config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.jsonl 2>> $O/bench.err || exit $?
for c in decode83 encode104 decode104 encode42 codec104; do
  timeout -k 10 300 python bench.py --config $c --no-cpu >> $O/bench_configs.jsonl 2>> $O/bench.err || exit $?
done
echo done-n
