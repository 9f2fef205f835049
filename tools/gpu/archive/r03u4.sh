#!/bin/bash
# U = 4 wave-contiguous runs (4 KiB per wave and shard) against the policy, packed and aligned
# RS(10,4); then multi-rank rehearsals of the final build (torchrun and single-process, shared GPU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10 300"
E="depth=2,early=1,fuse_tail=1,nt_load=1,nt_store=1,serial=1,wave_run=1"
$T python tools/tune.py --config encode104 --packed --rounds 9 --variants "chunks=2,$E;chunks=4,$E" \
  > gpurun_out/u4_encode104_packed.txt 2>&1 || exit $?
$T python tools/tune.py --config encode104 --align 4096 --rounds 9 --variants "chunks=2,$E;chunks=4,$E" \
  > gpurun_out/u4_encode104.txt 2>&1 || exit $?
D="depth=2,nt_load=1,nt_store=1,peel=1,fuse_tail=1"
$T python tools/tune.py --config decode104 --packed --compact --rounds 9 --variants "$D;chunks=4,wave_run=1,$D" \
  > gpurun_out/u4_decode104_packed.txt 2>&1 || exit $?
export SHMR_BENCH_SHARE_GPU=1
$T python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench_torchrun_g2_shared.jsonl 2> gpurun_out/bench_torchrun_g2.err || exit $?
$T python bench.py --gpus 2 --process-model single --steps 20 > gpurun_out/bench_single_g2_shared.jsonl 2> gpurun_out/bench_single_g2.err
