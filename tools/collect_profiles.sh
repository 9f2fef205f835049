#!/bin/bash
# Copies the rocprofv3 summaries tools/profile.sh left under gpurun_out/ into
# profiles/<round>/ (tracked) and the merged PMC traffic table into profiles/.
# Usage: tools/collect_profiles.sh <round-tag> <config>...
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
TAG=$1; shift
mkdir -p "$ROOT/profiles/$TAG"
for CFG in "$@"; do
  SRC="$ROOT/gpurun_out/prof_${TAG}_${CFG}"
  cp "$SRC/kt/kt_kernel_stats.csv" "$ROOT/profiles/$TAG/${CFG}_kernel_stats.csv"
  grep '^{' "$SRC/kt.log" > "$ROOT/profiles/$TAG/${CFG}_bench_under_rocprof.jsonl"
done
cp "$ROOT/gpurun_out/pmc_traffic.json" "$ROOT/profiles/pmc_traffic.json"
