#!/bin/bash
# Round 3 (session 2): profile part 2 (layout / output variants), the whole GPU suite, smoke, bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
bash tools/profile_all.sh r03 2 > gpurun_out/profile_all_r03_part2.log 2>&1 || exit $?
# the per-dispatch traces are merged already (pmc_traffic.json) and would push gpurun_out past
# the 64 MiB copy-back limit: keep the summaries only
find gpurun_out -name '*_kernel_trace.csv' -delete
find gpurun_out -name 'pmc_counter_collection.csv' -delete
du -sh gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_final.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit $?
for c in encode83 decode83 encode104 decode104 encode42 codec104; do
  timeout -k 10 300 python bench.py --config $c >> gpurun_out/bench_final.jsonl 2>> gpurun_out/bench_final.err || exit $?
done
timeout -k 10 300 python bench.py >> gpurun_out/bench_final.jsonl 2>> gpurun_out/bench_final.err || exit $?
# XCD-grouped tile order (tools knob xcd) against the policy, interleaved in one process:
# packed layouts (shared boundary lines between neighbouring tiles) and aligned slots
T="timeout -k 10 300"
E104="chunks=2,depth=2,early=1,fuse_tail=1,nt_load=1,nt_store=1,serial=1,wave_run=1"
$T python tools/tune.py --config encode104 --packed --rounds 9 --variants "$E104;$E104,xcd=1" \
  > gpurun_out/xcd_encode104_packed.txt 2>&1 || exit $?
D104P="depth=2,nt_load=1,nt_store=1,peel=1,fuse_tail=1"
$T python tools/tune.py --config decode104 --packed --compact --rounds 9 --variants "$D104P;$D104P,xcd=1" \
  > gpurun_out/xcd_decode104_packed.txt 2>&1 || exit $?
$T python tools/tune.py --config encode104 --align 4096 --rounds 9 --variants "$E104;$E104,xcd=1" \
  > gpurun_out/xcd_encode104.txt 2>&1 || exit $?
E83="depth=2,early=1,fuse_tail=1,nt_load=1,nt_store=1"
$T python tools/tune.py --config encode83 --pad 4096 --rounds 9 --variants "$E83;$E83,xcd=1" \
  > gpurun_out/xcd_encode83.txt 2>&1 || exit $?
D104="depth=2,nt_load=1,sc1_store=1,peel=1,fuse_tail=1"
$T python tools/tune.py --config decode104 --align 4096 --compact --rounds 9 --variants "$D104;$D104,xcd=1" \
  > gpurun_out/xcd_decode104.txt 2>&1
