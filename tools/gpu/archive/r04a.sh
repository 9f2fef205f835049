#!/bin/bash
# Round 4 (session 1), on the r03 product build plus two tools variants:
#  * the peeled ring on the RS(10,4) U = 2 early + serial encode,
#  * the realigning kernel (MODE 3, uvec=0) on the packed RS(10,4) buffer: time and
#    memory-pipeline counters against the unaligned-vector path (item 6),
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04a
mkdir -p $O
T="timeout -k 10 300"
E104="chunks=2,depth=2,early=1,fuse_tail=1,nt_load=1,nt_store=1,serial=1,wave_run=1"
$T python tools/tune.py --config encode104 --align 4096 --rounds 11 --variants "$E104;$E104,peel=1" \
  > $O/tune_encode104_peel.txt 2>&1 || exit $?
$T python tools/tune.py --config encode104 --packed --rounds 9 --variants "$E104;$E104,uvec=0" \
  > $O/tune_encode104_packed_mode3.txt 2>&1 || exit $?
# counters: one pass per group (tools/counter_passes.sh groups p1, p2, p4)
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
B="--no-cpu --config encode104 --steps 5 --warmup 1 --ramp-seconds 0.2"
pass() {  # name pass counters... -- program
  local name=$1 tag=$2 ctr=$3; shift 3
  timeout -s KILL 60 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/$O/pmc/${name}_$tag" -o pmc -- "$@" \
    > "$R/$O/pmc/${name}_$tag.log" 2>&1
  local rc=$?
  echo "$name $tag rc=$rc"
  return $rc
}
mkdir -p $R/$O/pmc
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
find $O -name '*_kernel_trace.csv' -size +2M -delete
echo done
