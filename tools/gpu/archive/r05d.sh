#!/bin/bash
# Round 5 (session 4): the whole GPU suite, smoke, the default bench line and
# the pointer-table bench lines (slab buffers: a slot grid; torch buffers: the
# table kernels), then a 60 s soak that includes the slab/grid operation.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.jsonl 2>> $O/bench.err || exit $?
for c in encode83 decode83 encode104 decode104; do
  timeout -k 10 300 python bench.py --config $c --layout ptrs --no-cpu >> $O/bench_ptrs.jsonl 2>> $O/bench.err || exit $?
done
timeout -k 10 200 python -u tools/soak.py --seconds 60 --threads 12 > $O/soak.log 2>&1 || exit $?
echo done-d
