#!/bin/bash
# Round 5 (session 3): capture-block reuse behind a queued replay,
# the flush-failure path of the C++ mirror, and the relaxed-capture guard A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05c
mkdir -p $O
PT="python -u -m pytest -x -q -s --timeout 120 --timeout-method thread"
# where shard files would live on this box (config 5: O_DIRECT needs a real block device)
{ df -T /tmp . /dev/shm; findmnt -T /tmp; findmnt -T .; nproc; free -g; lsblk -d -o NAME,ROTA,SIZE,MODEL 2>/dev/null; } > $O/fs_probe.txt 2>&1
timeout -k 10 200 $PT tests/test_gpu_capture.py -k queued > $O/pytest_queued.log 2>&1
rc=$?; echo "queued rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 $PT tests/test_host_cpp.py -k "encode_failure or mapped_per_block or direct_io" > $O/pytest_flush_failure.log 2>&1
rc=$?; echo "flush rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 $PT tests/test_gpu_multidevice.py -k eight > $O/pytest_eight_ids.log 2>&1
rc=$?; echo "eight ids rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 500 $PT tests/test_gpu_dist.py > $O/pytest_dist.log 2>&1
rc=$?; echo "dist rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 tools/_abx/guard_ab shmr_amd/_lib/libshmr_ec.so tools/_abx/norelax/libshmr_ec.so 11 8 > $O/guard_ab.txt 2>&1 || exit $?
timeout -k 10 300 tools/_abx/guard_ab tools/_abx/norelax/libshmr_ec.so shmr_amd/_lib/libshmr_ec.so 11 8 > $O/guard_ab_swapped.txt 2>&1 || exit $?
# config 5 with and without O_DIRECT shard files (mapped Block Cache, fsync on and off)
for fsy in 0 1; do
  for d in 0 1; do
    SHMR_VFS_DIRECT=$d SHMR_VFS_PINNED_ONLY=1 timeout -k 10 300 shmr_amd/_lib/shmr_vfs_bench /tmp/vb_$d 256 4 $fsy 3 \
      > $O/vfs_direct${d}_fsync${fsy}.jsonl 2>&1 || exit $?
    rm -rf /tmp/vb_$d
  done
done
echo done-c
