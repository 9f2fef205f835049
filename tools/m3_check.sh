#!/bin/bash
# Realigning kernel (mode 3) check: its parity cases, kernel times of
# misaligned layouts next to the aligned ones, then the rocprofv3 + PMC
# profiles of every bench config for the new build.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread \
    -k "contiguous_layout_realigned or encode_batch_dev or reconstruct" > gpurun_out/m3_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/m3_pytest.log; [ $rc -eq 0 ] || exit $rc
E="chunks=2,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1,serial=1"
for pad in 1536 2; do
  timeout -k 10 120 python -u tools/tune.py --config encode104 --pad $pad --rounds 5 --iters 10 --variants "$E" \
      > gpurun_out/m3_e104_$pad.txt 2>&1 || exit $?
  timeout -k 10 120 python -u tools/tune.py --config decode104 --pad $pad --rounds 5 --iters 10 \
      --variants "chunks=1,nt_load=1,nt_store=1,depth=2,fuse_tail=1" > gpurun_out/m3_d104_$pad.txt 2>&1 || exit $?
  echo "RS(10,4) pad=$pad encode $(tail -1 gpurun_out/m3_e104_$pad.txt | sed 's/.*"median_ms"/median_ms/') decode $(tail -1 gpurun_out/m3_d104_$pad.txt | sed 's/.*"median_ms"/median_ms/')"
done
for pad in 4096 4100; do
  timeout -k 10 120 python -u tools/tune.py --config encode83 --pad $pad --rounds 5 --iters 10 \
      --variants "chunks=1,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1" > gpurun_out/m3_e83_$pad.txt 2>&1 || exit $?
  echo "RS(8,3) pad=$pad encode $(tail -1 gpurun_out/m3_e83_$pad.txt | sed 's/.*"median_ms"/median_ms/')"
done
bash tools/profile_all.sh r02
