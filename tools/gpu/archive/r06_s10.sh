#!/bin/bash
# r06 session 10: the round-end sequence on the frozen kernel build (suite, smoke),
# then the kernel traces + PMC passes of the six bench configs for that build
# (bench.py's roofline.traffic is keyed by the build ID), then the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s10
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/profile_all.sh r06 1 > $O/profile_all.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.jsonl 2>> $O/bench.err || exit $?
echo done-s10
