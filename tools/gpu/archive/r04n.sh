#!/bin/bash
# Round 4 (session 14): validation of the final host code (relaxed capture mode at every entry,
# mirrored events): bench lines (slots and pointer tables), smoke, the whole GPU suite, config 5
# with 16 vs 24 per-block tasks (second box of the three-box rule).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04n
mkdir -p $O
for c in encode83 decode83 encode104 decode104 encode42 codec104; do
  timeout -k 10 300 python bench.py --config $c >> $O/bench.jsonl 2>> $O/bench.err || exit $?
done
for c in encode83 decode83 encode104 decode104; do
  timeout -k 10 300 python bench.py --config $c --layout ptrs >> $O/bench_ptrs.jsonl 2>> $O/bench.err || exit $?
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
mkdir -p /tmp/vb
for n in 16 24 16 24; do
  SHMR_VFS_TASKS=$n timeout -k 10 400 shmr_amd/_lib/shmr_vfs_bench /tmp/vb 256 4 0 3 >> $O/e2e_vf_tasks$n.jsonl 2>> $O/e2e_vf.err || exit $?
done
echo done-n
