#!/bin/bash
# r06 session 33: GPU suite, smoke and the default bench line on the final tree
# (host-path staging streams at the library's stream priority), the host-path
# per-block rates and the VirtualFile end to end.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s33
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.jsonl 2>> $O/bench.err || exit $?
timeout -k 10 300 tools/_abx/perblock_host 128 5 > $O/perblock_host.jsonl 2> $O/perblock_host.err || exit 1
mkdir -p /tmp/vb_s33 && timeout -k 10 300 shmr_amd/_lib/shmr_vfs_bench /tmp/vb_s33 256 4 0 3 > $O/vfs_bench.jsonl 2> $O/vfs_bench.err || exit 1
echo done-s33
