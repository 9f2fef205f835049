#!/bin/bash
# Round 3, first GPU pass: new tests, full GPU suite, compact-output decode
# bench + store-policy A/B, and the split / new product library against r02.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03a
mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_capture.py tests/test_isa.py -x -v --timeout 120 --timeout-method thread > $O/pytest_new.log 2>&1 &&
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
for i in 1 2; do
  $T 180 python bench.py --config decode83 --cpu-seconds 0.5 >> $O/bench_decode83_inplace.jsonl 2>>$O/bench.err &&
  $T 180 python bench.py --config decode83 --rebuild-out compact --cpu-seconds 0.5 >> $O/bench_decode83_compact.jsonl 2>>$O/bench.err || exit 1
done &&
$T 300 python tools/tune.py --config decode83 --compact --pad 4096 --rounds 7 \
  --variants "nt_load=1,depth=2,sc1_store=1;nt_load=1,depth=2,nt_store=1;nt_load=1,depth=2;nt_load=1,depth=2,sc1_store=1,wgs_per_cu=7;nt_load=1,depth=2,nt_store=1,wgs_per_cu=7;nt_load=1,depth=2,wgs_per_cu=7" > $O/tune_decode83_compact.txt 2>&1 &&
$T 300 python tools/tune.py --config decode104 --compact --rounds 7 \
  --variants "nt_load=1,depth=2,sc1_store=1,fuse_tail=1;nt_load=1,depth=2,nt_store=1,fuse_tail=1;nt_load=1,depth=2,fuse_tail=1" > $O/tune_decode104_compact.txt 2>&1 &&
$T 180 python bench.py > $O/bench_encode83.jsonl 2>>$O/bench.err &&
$T 180 python bench.py --process-model single --no-cpu > $O/bench_single_g1.jsonl 2>>$O/bench.err &&
SHMR_BENCH_SHARE_GPU=1 $T 180 python bench.py --process-model single --gpus 2 --blocks 256 > $O/bench_single_g2_shared.jsonl 2>>$O/bench.err &&
SHMR_BENCH_SHARE_GPU=1 $T 180 python bench.py --process-model single --gpus 4 --config codec104 --blocks 16 > $O/bench_single_g4_shared_codec.jsonl 2>>$O/bench.err &&
for c in encode83 decode83 encode104 decode104; do
  $T 240 python tools/ab_libs.py tools/_abr/libshmr_ec_r02.so --config $c --pitch-align 4096 > $O/ab_r02_$c.txt 2>&1 || exit 1
done &&
# packed layout (the reference's i * S buffer): unaligned-vector policy vs the DPP realign tile, one process each
$T 300 python tools/tune.py --config encode104 --packed --rounds 7 \
  --variants "chunks=2,nt_load=1,nt_store=1,depth=2,early=1,serial=1,fuse_tail=1;chunks=2,nt_load=1,nt_store=1,depth=2,fuse_tail=1;chunks=2,nt_load=1,nt_store=1,depth=2,fuse_tail=1,realign=1;chunks=2,nt_load=1,nt_store=1,depth=2,fuse_tail=1,serial=1,realign=1" > $O/tune_encode104_packed_realign.txt 2>&1 &&
$T 300 python tools/tune.py --config decode104 --packed --rounds 7 \
  --variants "nt_load=1,nt_store=1,depth=2,fuse_tail=1;nt_load=1,nt_store=1,depth=2,fuse_tail=1,realign=1" > $O/tune_decode104_packed_realign.txt 2>&1 &&
$T 180 python bench.py --config encode104 --pitch-align 1 --cpu-seconds 0.5 > $O/bench_encode104_packed.jsonl 2>>$O/bench.err &&
$T 180 python bench.py --config decode104 --pitch-align 1 --cpu-seconds 0.5 > $O/bench_decode104_packed.jsonl 2>>$O/bench.err
