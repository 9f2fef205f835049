#!/bin/bash
# Round 4 (session 17): the final host code -- the whole GPU suite, smoke, the default bench line,
# the ptrs bench lines (table-cache hits on the caller's own events) and a 60 s soak.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.jsonl 2>> $O/bench.err || exit $?
for c in encode83 decode83; do
  timeout -k 10 300 python bench.py --config $c --layout ptrs >> $O/bench_ptrs.jsonl 2>> $O/bench.err || exit $?
done
timeout -k 10 200 python -u tools/soak.py --seconds 60 --threads 12 > $O/soak.log 2>&1 || exit $?
echo done-q
