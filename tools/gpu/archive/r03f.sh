#!/bin/bash
# Round 3: RS(10,4) counter table; line vs page alignment of the shard pitch;
# a 90 s 12-thread soak with the compact rebuild; host ASan/UBSan run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03f
mkdir -p $O
T="timeout -k 10"
$T 900 bash tools/counter_passes.sh $O/ctr > $O/counter_passes.txt 2>&1 &&
python tools/counter_table.py $O/ctr --json $O/counters_encode104.json > $O/counters_encode104.md 2>&1 &&
for cfg in encode104 decode104; do
  for pa in 4096 128 64 32 16; do
    $T 180 python bench.py --config $cfg --pitch-align $pa --pitch-pad 0 --rebuild-out inplace --no-cpu >> $O/bench_${cfg}_pitch_align.jsonl 2>>$O/bench.err || exit 1
  done
done &&
$T 200 python -u tools/soak.py --seconds 90 --threads 12 > $O/soak.log 2>&1 &&
$T 600 bash tools/asan_host.sh run $O/asan > $O/asan_host.log 2>&1
