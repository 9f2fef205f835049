#!/bin/bash
# r06 session 41: scratch buffers grown without a free (grow_scratch): the HOL
# probe with growth during the hold, alone and after the queue / pool tests,
# then the round-end sequence on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s41
mkdir -p $O
timeout -k 10 120 python -u tools/hol_held.py > $O/hol_held.jsonl 2> $O/hol_held.err || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_submit.py tests/test_gpu_pool.py tests/test_gpu_hol.py > $O/pytest_hol_after.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.jsonl 2>> $O/bench.err || exit $?
timeout -k 10 300 tools/_abx/perblock_host 128 5 > $O/perblock_host.jsonl 2> $O/perblock_host.err || exit 1
timeout -k 10 120 python -u tools/soak.py --seconds 60 --threads 12 > $O/soak_all.jsonl 2>&1 || exit $?
echo done-s41
