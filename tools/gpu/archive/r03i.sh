#!/bin/bash
# Round 3: the peeled-ring reconstruct policy build -- full GPU suite, smoke,
# one-process A/B against the r02 library, bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03i
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
$T 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
for c in decode83 decode104; do
  $T 300 python tools/ab_libs.py tools/_abr/libshmr_ec_r02.so --config $c > $O/ab_libs_$c.txt 2>&1 || exit 1
done &&
for i in 1 2; do
  for c in decode83 decode104 encode83; do
    $T 180 python bench.py --config $c --cpu-seconds 0.3 >> $O/bench_$c.jsonl 2>>$O/bench.err || exit 1
  done
done
