#!/bin/bash
# Misaligned-shard paths: the full GPU suite, the layout probe, kernel times of
# misaligned layouts next to aligned ones (auto policy, and the realigning
# kernel forced with uvec=0), then rocprofv3 + PMC profiles of every bench
# config for the new build.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/m3_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/m3_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/misaligned_probe.py --blocks 32 > gpurun_out/misaligned_auto.jsonl 2>&1 || exit $?
cat gpurun_out/misaligned_auto.jsonl | grep layout
E="chunks=2,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1,serial=1"
D="chunks=1,nt_load=1,nt_store=1,depth=2,fuse_tail=1"
for pad in 1536 2; do
  timeout -k 10 120 python -u tools/tune.py --config encode104 --pad $pad --rounds 5 --iters 10 --variants "$E;$E,uvec=0" \
      > gpurun_out/m3_e104_$pad.txt 2>&1 || exit $?
  timeout -k 10 120 python -u tools/tune.py --config decode104 --pad $pad --rounds 5 --iters 10 --variants "$D;$D,uvec=0" \
      > gpurun_out/m3_d104_$pad.txt 2>&1 || exit $?
  grep frac gpurun_out/m3_e104_$pad.txt | sed "s/^/RS(10,4) encode pad=$pad /"
  grep frac gpurun_out/m3_d104_$pad.txt | sed "s/^/RS(10,4) decode pad=$pad /"
done
P="chunks=1,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1"
for pad in 4096 4100; do
  timeout -k 10 120 python -u tools/tune.py --config encode83 --pad $pad --rounds 5 --iters 10 --variants "$P;$P,uvec=0" \
      > gpurun_out/m3_e83_$pad.txt 2>&1 || exit $?
  grep frac gpurun_out/m3_e83_$pad.txt | sed "s/^/RS(8,3) encode pad=$pad /"
done
bash tools/profile_all.sh r02
