#!/bin/bash
# rocprofv3 passes for the bench command: kernel trace + stats, then one PMC
# pass per counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
# Usage: tools/profile.sh <tag> [bench args...]
set -u
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
TAG=${1:-r01}; shift || true
ARGS="$*"
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- \
  python3 "$ROOT/bench.py" --no-cpu $ARGS > "$OUT/kt.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$C" -o pmc -- \
    python3 "$ROOT/bench.py" --no-cpu --steps 5 --warmup 1 $ARGS > "$OUT/$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
find "$OUT" -name "*.csv" | head -20
