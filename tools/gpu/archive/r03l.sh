#!/bin/bash
# Round 3: wave-run policy build (U = 2 launches) -- GPU suite, smoke, A/B vs
# r02 in one process, bench lines incl. the packed layout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03l
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
$T 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
for c in encode104 decode104 encode83; do
  $T 300 python tools/ab_libs.py tools/_abr/libshmr_ec_r02.so --config $c > $O/ab_libs_$c.txt 2>&1 || exit 1
done &&
for i in 1 2; do
  for c in encode104 codec104; do
    $T 180 python bench.py --config $c --cpu-seconds 0.3 >> $O/bench_$c.jsonl 2>>$O/bench.err || exit 1
  done
  for c in encode104 decode104; do
    $T 180 python bench.py --config $c --pitch-align 1 --cpu-seconds 0.3 >> $O/bench_${c}_packed.jsonl 2>>$O/bench.err || exit 1
  done
done
