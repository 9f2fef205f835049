#!/bin/bash
# Round 4 final (part 1): rocprofv3 kernel traces + PMC traffic of the six bench configs on the
# final build, the whole GPU suite, smoke and the bench lines (`bash tools/gpu/r04d.sh [part]`).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04d
mkdir -p $O
PART=${1:-1}
if [ "$PART" = 2 ]; then
  # pointer-table rebuilds in plan order: is the early prologue (+3.4 / +8.2 with the r03 chain) still the better tile?
  D="depth=2,fuse_tail=1,nt_load=1,peel=1,sc1_store=1,ptrs_segs=0"   # table launches in both (no segs build of the plain tile)
  timeout -k 10 300 python tools/tune.py --config decode83 --ptrs --rounds 11 --variants "$D,early=1;$D" \
    > $O/tune_decode83_ptrs_early.txt 2>&1 || exit $?
  timeout -k 10 300 python tools/tune.py --config decode104 --ptrs --rounds 11 --variants "$D,early=1;$D" \
    > $O/tune_decode104_ptrs_early.txt 2>&1 || exit $?
fi
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
bash tools/profile_all.sh r04 $PART > $O/profile_all_r04_part$PART.log 2>&1 || exit $?
find gpurun_out -name '*_kernel_trace.csv' -delete
find gpurun_out -name 'pmc_counter_collection.csv' -delete
if [ "$PART" = 1 ]; then
  cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json   # (the box's copy) bench lines then match traffic
  for c in encode83 decode83 encode104 decode104 encode42 codec104; do
    timeout -k 10 300 python bench.py --config $c >> $O/bench_final.jsonl 2>> $O/bench_final.err || exit $?
  done
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_final.log 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/pytest_gpu_final.log 2>&1 || exit $?
fi
if [ "$PART" = 2 ]; then   # config 5 on the final build (flush / copy-out overlapped with the GPU calls)
  mkdir -p /tmp/vb
  timeout -k 10 400 shmr_amd/_lib/shmr_vfs_bench /tmp/vb 256 4 0 3 > $O/e2e_virtual_file_nofsync.jsonl 2> $O/e2e_vf.err || exit $?
  timeout -k 10 300 python tools/e2e_bench.py > $O/e2e_host_path.json 2> $O/e2e_host_path.err || exit $?
fi
echo done-final-$PART
