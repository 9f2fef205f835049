#!/bin/bash
# Round 3, second GPU pass: regression suite on the policy build, compact
# rebuild tuning, single-process model vs process model, packed-layout
# isolation (16-byte vs page alignment) and PMC traffic of the new layouts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03b
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
$T 300 python tools/tune.py --config decode83 --compact --pad 4096 --rounds 9 \
  --variants "nt_load=1,nt_store=1,depth=2,wgs_per_cu=7;nt_load=1,nt_store=1,depth=2,wgs_per_cu=6;nt_load=1,nt_store=1,depth=2;nt_load=1,nt_store=1,depth=2,early=1,wgs_per_cu=7;nt_load=1,nt_store=1,wgs_per_cu=7;nt_load=1,nt_store=1,depth=2,threads=512;nt_load=1,depth=2,sc1_store=1" > $O/tune_decode83_compact_sweep.txt 2>&1 &&
$T 300 python tools/tune.py --config decode83 --pad 4096 --rounds 9 \
  --variants "nt_load=1,nt_store=1,depth=2,wgs_per_cu=7;nt_load=1,nt_store=1,depth=2,wgs_per_cu=6;nt_load=1,nt_store=1,depth=2" > $O/tune_decode83_inplace_sweep.txt 2>&1 &&
$T 300 python tools/tune.py --config decode104 --compact --align 4096 --rounds 9 \
  --variants "nt_load=1,nt_store=1,depth=2,fuse_tail=1;nt_load=1,depth=2,fuse_tail=1,sc1_store=1;nt_load=1,nt_store=1,depth=2,fuse_tail=1,wgs_per_cu=7" > $O/tune_decode104_compact_4k.txt 2>&1 &&
$T 300 python tools/tune.py --config decode104 --align 4096 --rounds 9 \
  --variants "nt_load=1,nt_store=1,depth=2,fuse_tail=1;nt_load=1,nt_store=1,depth=2,fuse_tail=1,wgs_per_cu=7" > $O/tune_decode104_inplace_4k.txt 2>&1 &&
for i in 1 2; do
  $T 180 python bench.py --steps 200 --no-cpu >> $O/bench_process_s200.jsonl 2>>$O/bench.err &&
  $T 180 python bench.py --steps 200 --no-cpu --process-model single >> $O/bench_single_s200.jsonl 2>>$O/bench.err &&
  $T 180 python bench.py --steps 200 --no-cpu --process-model single --single-stream current >> $O/bench_single_cur_s200.jsonl 2>>$O/bench.err || exit 1
done &&
for cfg in encode104 decode104; do
  for pa in 4096 16 1; do
    $T 180 python bench.py --config $cfg --pitch-align $pa --pitch-pad 0 --no-cpu >> $O/bench_${cfg}_align.jsonl 2>>$O/bench.err || exit 1
  done
done &&
$T 180 python bench.py --config decode83 --rebuild-out compact > $O/bench_decode83_compact.jsonl 2>>$O/bench.err &&
$T 180 python bench.py --config decode104 --rebuild-out compact > $O/bench_decode104_compact.jsonl 2>>$O/bench.err &&
KEY=encode104+packed BENCH_EXTRA="--pitch-align 1" $T 600 bash tools/profile.sh r03b encode104 64 $((64 * 14 * 1677722)) > $O/prof_encode104_packed.txt 2>&1 &&
KEY=decode83+compact BENCH_EXTRA="--rebuild-out compact" $T 600 bash tools/profile.sh r03b decode83 512 2415919104 > $O/prof_decode83_compact.txt 2>&1
