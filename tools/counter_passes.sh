#!/bin/bash
# Memory-pipeline counters of three RS(10,4)-shaped kernels, one rocprofv3
# --pmc pass per counter group (each within gfx950's per-block limits:
# <= 4 TCC, 4 TCP, 2 TA, 2 TD, 8 SQ, 2 GRBM):
#   gf      the product encode kernel, bench.py --config encode104 (page-aligned slots)
#   gfpack  the same on the reference's packed buffer (--pitch-align 1)
#   xor     the 10 -> 4 XOR replica of the tiling (tools/membench.hip, U = 1 and 2)
# tools/counter_table.py turns the passes into per-byte figures.
# Usage: tools/counter_passes.sh <outdir>
set -u
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$1"
OUT="$(cd "$1" && pwd)"
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "p1:TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE"
  "p2:TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_STREAMING_REQ_sum"
  "p3:TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE"
  "p4:TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_WRITE_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_UTCL1_TRANSLATION_MISS_sum GRBM_GUI_ACTIVE"
  "p5:TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum GRBM_GUI_ACTIVE"
  "p6:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_WAVES GRBM_GUI_ACTIVE"
)
subject() {  # name, then the program and its args
  local name=$1; shift
  for p in "${PASSES[@]}"; do
    local tag=${p%%:*} ctr=${p#*:}
    timeout -s KILL 60 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/${name}_$tag" -o pmc -- "$@" \
      > "$OUT/${name}_$tag.log" 2>&1
    local rc=$?
    echo "$name $tag rc=$rc"
    [ $rc -eq 0 ] || return $rc
  done
}
BENCH="--no-cpu --config encode104 --steps 5 --warmup 1 --ramp-seconds 0.2"
subject gf python3 "$ROOT/bench.py" $BENCH || exit 1
subject gfpack python3 "$ROOT/bench.py" $BENCH --pitch-align 1 || exit 1
export MEMBENCH_ONLY=104
subject xor "$ROOT/tools/_probe/membench" 1671168 64 5 || exit 1
