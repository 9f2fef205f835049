#!/bin/bash
# rocprofv3 passes for one bench config: kernel trace + stats, then one PMC
# pass per counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950),
# then tools/pmc_traffic.py merges the summary into gpurun_out/pmc_traffic.json.
# Usage: tools/profile.sh <tag> <config> <blocks> <algo_bytes_per_launch> [--sum-kernels]
# Env: BENCH_EXTRA (more bench.py flags, e.g. "--pitch-align 1" or "--rebuild-out compact") and
# KEY (the record's key, bench.py traffic_key(): e.g. encode104+packed, decode83+compact).
set -u
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
TAG=$1; CFG=$2; BLOCKS=$3; ALGO=$4; EXTRA=${5:-}
BX=${BENCH_EXTRA:-}; KEY=${KEY:-$CFG}
OUT="$ROOT/gpurun_out/prof_${TAG}_${KEY}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- \
  python3 "$ROOT/bench.py" --no-cpu --config "$CFG" --blocks "$BLOCKS" $BX > "$OUT/kt.log" 2>&1
rc=$?; echo "kernel-trace $CFG rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$C" -o pmc -- \
    python3 "$ROOT/bench.py" --no-cpu --config "$CFG" --blocks "$BLOCKS" --steps 5 --warmup 1 --ramp-seconds 0.2 $BX \
    > "$OUT/$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
# merge into a copy of the tracked table (gpurun_out/ is not pushed to the box)
[ -f "$ROOT/gpurun_out/pmc_traffic.json" ] || cp "$ROOT/profiles/pmc_traffic.json" "$ROOT/gpurun_out/pmc_traffic.json"
python3 "$ROOT/tools/pmc_traffic.py" "$OUT" --config "$KEY" --blocks "$BLOCKS" --algo-bytes "$ALGO" \
  --merge "$ROOT/gpurun_out/pmc_traffic.json" $EXTRA
