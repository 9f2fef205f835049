#!/bin/bash
# Round 4 (session 1): the r04 build (policy-derived kernel list, plan-order
# pointer tables, capture reserve) -- the whole GPU suite first, then A/Bs
# against the r03 product library (tools/ablib/r03) in one process, the peeled
# RS(10,4) encode and the MODE 3 counters on the packed buffer (tools build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit $?
T="timeout -k 10 300"
R03=tools/ablib/r03/libshmr_ec.so
for c in encode83 decode83 encode104 decode104; do
  $T python tools/ab_libs.py $R03 --config $c --ptrs --rounds 11 > $O/ab_ptrs_$c.txt 2>&1 || exit $?
done
for c in decode104 decode83e3 decode83; do
  $T python tools/ab_libs.py $R03 --config $c --compact --pitch-align 4096 --rounds 11 > $O/ab_compact_$c.txt 2>&1 || exit $?
done
E104="chunks=2,depth=2,early=1,fuse_tail=1,nt_load=1,nt_store=1,serial=1,wave_run=1"
$T python tools/tune.py --config encode104 --align 4096 --rounds 11 --variants "$E104;$E104,peel=1" \
  > $O/tune_encode104_peel.txt 2>&1 || exit $?
$T python tools/tune.py --config encode104 --packed --rounds 9 --variants "$E104;$E104,uvec=0" \
  > $O/tune_encode104_packed_mode3.txt 2>&1 || exit $?
echo done-ab
# config 5 on the r04 build: VirtualFile end to end with per-block task phases, codec entry points
mkdir -p /tmp/vb
timeout -k 10 400 shmr_amd/_lib/shmr_vfs_bench /tmp/vb 256 4 0 3 > $O/e2e_virtual_file_nofsync.jsonl 2> $O/e2e_vf.err || exit $?
$T python tools/e2e_bench.py > $O/e2e_host_path.json 2> $O/e2e_host_path.err || exit $?
echo done-e2e
