#!/bin/bash
# Round 3, fourth GPU pass: the sc1 compact-rebuild policy build (suite +
# bench), cache policy on the packed layout, and the RS(10,4) counter table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03d
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
for i in 1 2; do
  for c in decode83 decode104; do
    $T 180 python bench.py --config $c --cpu-seconds 0.3 >> $O/bench_${c}_compact.jsonl 2>>$O/bench.err &&
    $T 180 python bench.py --config $c --rebuild-out inplace --cpu-seconds 0.3 >> $O/bench_${c}_inplace.jsonl 2>>$O/bench.err || exit 1
  done
done &&
$T 400 python tools/tune.py --config encode104 --packed --rounds 11 \
  --variants "chunks=2,nt_load=1,nt_store=1,depth=2,early=1,serial=1,fuse_tail=1;chunks=2,nt_load=0,nt_store=1,depth=2,early=1,serial=1,fuse_tail=1;chunks=2,nt_load=1,nt_store=0,depth=2,early=1,serial=1,fuse_tail=1;chunks=2,nt_load=0,nt_store=0,depth=2,early=1,serial=1,fuse_tail=1;chunks=2,nt_load=0,nt_store=1,depth=2,fuse_tail=1" > $O/tune_encode104_packed_cachepol.txt 2>&1 &&
$T 400 python tools/tune.py --config decode104 --packed --rounds 11 \
  --variants "nt_load=1,nt_store=1,depth=2,fuse_tail=1;nt_load=0,nt_store=1,depth=2,fuse_tail=1;nt_load=1,nt_store=0,depth=2,fuse_tail=1;nt_load=0,nt_store=0,depth=2,fuse_tail=1" > $O/tune_decode104_packed_cachepol.txt 2>&1 &&
$T 900 bash tools/counter_passes.sh $O/ctr > $O/counter_passes.txt 2>&1 &&
python tools/counter_table.py $O/ctr --json $O/counters_encode104.json > $O/counters_encode104.md 2>&1
