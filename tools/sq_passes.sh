#!/bin/bash
# One rocprofv3 pass of 8 SQ counters + GRBM_GUI_ACTIVE per kernel variant
# (bench.py short runs), summarised by tools/sq_split.py into
# gpurun_out/sq_split.json.  Separate pass per variant; stops at the first failure.
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
CTR="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
cd /tmp && export TMPDIR=/tmp
pass() {  # tag dwords_per_wave bench-args...
  local tag=$1 dw=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d "$ROOT/gpurun_out/sq_$tag" -o pmc -- \
    python3 "$ROOT/bench.py" --no-cpu --steps 5 --warmup 1 --ramp-seconds 0.2 "$@" > "$ROOT/gpurun_out/sq_$tag.log" 2>&1
  echo "sq pass $tag rc=$?"
  python3 "$ROOT/tools/sq_split.py" "$ROOT/gpurun_out/sq_$tag" --tag "$tag" --dwords-per-wave "$dw" \
    --merge "$ROOT/gpurun_out/sq_split.json" > /dev/null
}
pass encode83 32 --config encode83
pass encode104_u2 80 --config encode104
pass encode104_u1 40 --config encode104 --tune "chunks=1"
pass encode104_u1_serial 40 --config encode104 --tune "chunks=1,serial=1"
pass encode104_xor_u1 40 --config encode104 --tune "chunks=1,depth=3,fuse_tail=0,diag=1"
pass decode83 32 --config decode83
cat "$ROOT/gpurun_out/sq_split.json" | python3 -c "
import json,sys
d=json.load(sys.stdin)
for k,v in d.items(): print(k, v.get('wave_cycle_split'), v.get('valu_insts_per_loaded_dword'), v.get('valu_active_per_busy_cycle'), v.get('wave_quadcycles_per_wave'))"
