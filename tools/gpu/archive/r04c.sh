#!/bin/bash
# Round 4 (session 2): memory-pipeline counters of the RS(10,4) encode -- policy kernel on slots,
# the same with the peeled ring, on the reference's packed buffer with the unaligned vector path
# and with the realigning kernel (MODE 3, knob uvec=0) -- one rocprofv3 --pmc pass per group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"
O=gpurun_out/r04c
mkdir -p $O/pmc
# pointer tables in plan order: does the early prologue now pay for the RS(10,4) encode (r03: -1.5)?
P104="chunks=2,depth=2,fuse_tail=1,nt_load=1,nt_store=1,wave_run=1"
timeout -k 10 300 python tools/tune.py --config encode104 --ptrs --rounds 11 --variants "$P104;$P104,early=1,serial=1" \
  > $O/tune_encode104_ptrs_early.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
B="--no-cpu --config encode104 --steps 5 --warmup 1 --ramp-seconds 0.2"
E104="chunks=2,depth=2,early=1,fuse_tail=1,nt_load=1,nt_store=1,serial=1,wave_run=1"
pass() {  # name tag counters -- program
  local name=$1 tag=$2 ctr=$3; shift 3
  timeout -s KILL 60 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/$O/pmc/${name}_$tag" -o pmc -- "$@" \
    > "$R/$O/pmc/${name}_$tag.log" 2>&1
  local rc=$?
  echo "$name $tag rc=$rc"
  return $rc
}
P1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE"
P2="TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_STREAMING_REQ_sum"
P4="TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_WRITE_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_UTCL1_TRANSLATION_MISS_sum GRBM_GUI_ACTIVE"
P5="TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum GRBM_GUI_ACTIVE"
for tag in p1 p2 p4 p5; do
  case $tag in p1) C=$P1;; p2) C=$P2;; p4) C=$P4;; p5) C=$P5;; esac
  pass gf $tag "$C" python3 $R/bench.py $B || exit $?
  pass gfpeel $tag "$C" python3 $R/bench.py $B --tune "$E104,peel=1" || exit $?
  pass gfpack $tag "$C" python3 $R/bench.py $B --pitch-align 1 || exit $?
  pass gfpack3 $tag "$C" python3 $R/bench.py $B --pitch-align 1 --tune uvec=0 || exit $?
done
cd $R
python3 tools/counter_table.py $O/pmc --json $O/counters_encode104_r04.json > $O/counters_encode104_r04.md || exit $?
find $O -name '*_kernel_trace.csv' -size +2M -delete
echo done-counters
# config 5: per-block task concurrency of the mapped-buffer read / flush (default 16)
mkdir -p /tmp/vb
for n in 24 32 16; do
  SHMR_VFS_TASKS=$n timeout -k 10 400 shmr_amd/_lib/shmr_vfs_bench /tmp/vb 256 4 0 3 > $O/e2e_vf_tasks$n.jsonl 2> $O/e2e_vf_tasks$n.err || exit $?
done
echo done-e2e
