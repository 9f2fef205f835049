#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, bench.  Every GPU step has its
# own time limit; a crash/abort/timeout ends the script (no further GPU work).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
stop_if_fatal() {  # pytest 0/1 (pass/fail) are fine; anything else ends the run
  local rc=$1 what=$2
  echo "$what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal in $what, stopping"; exit "$rc"; fi
}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/smoke.log; stop_if_fatal $rc smoke
timeout -k 10 600 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/bench.log; stop_if_fatal $rc bench
