#!/bin/bash
# Round 5 (session 20): the final tree -- the whole GPU suite, smoke, the default bench line, and
# the host sanitizers (ASan + UBSan, kernel TU included) over the StorageBlock cases and abi_check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.jsonl 2>> $O/bench.err || exit $?
timeout -k 10 900 bash tools/asan_host.sh build > $O/asan_build.log 2>&1 || exit $?
timeout -k 10 900 bash tools/asan_host.sh run $O/asan > $O/asan_host.log 2>&1 || exit $?
echo done-y
