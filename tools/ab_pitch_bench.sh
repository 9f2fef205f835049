#!/bin/bash
# bench.py with 256 B vs 4 KiB shard pitch, alternating processes (3 pairs per config).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/ab_pitch_bench.jsonl
: > $OUT
for cfg in encode104 decode104 codec104; do
  for rep in 1 2 3; do
    for pa in 256 4096; do
      timeout -k 10 120 python bench.py --no-cpu --config $cfg --pitch-align $pa --steps 40 > gpurun_out/pb.log 2>&1 || { cat gpurun_out/pb.log; exit 1; }
      python -c "
import json,sys
l=json.loads([x for x in open('gpurun_out/pb.log') if x.startswith('{')][-1])
print(json.dumps({'config': '$cfg', 'pitch_align': $pa, 'rep': $rep, 'value': l['value'], 'frac': l['roofline']['frac'], 'ms': l['ms_per_step']}))" >> $OUT
    done
  done
done
cat $OUT
