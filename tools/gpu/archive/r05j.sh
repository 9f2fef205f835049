#!/bin/bash
# Round 5 (session 10): the driver's scaling launch shape at full size on one shared GPU:
# bench.py --gpus 2 / 4 / 8 with the default batch (B = 512 per rank) and K = 100.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05j
mkdir -p $O
for n in 2 4 8; do
  SHMR_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus $n >> $O/bench_shared_gpus.jsonl 2>> $O/bench.err || exit $?
done
echo done-j
