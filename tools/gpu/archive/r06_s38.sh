#!/bin/bash
# r06 session 38: round-end sequence on the final tree (rebuild lattices fitted
# over every present shard, queue trace base): GPU suite, smoke, default bench
# line, queue per-block rates, host per-block rates.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s38
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.jsonl 2>> $O/bench.err || exit $?
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 256 7 > $O/perblock256.jsonl 2> $O/perblock256.err || exit 1
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 > $O/perblock1024.jsonl 2> $O/perblock1024.err || exit 1
timeout -k 10 300 tools/_abx/perblock_host 128 5 > $O/perblock_host.jsonl 2> $O/perblock_host.err || exit 1
echo done-s38
