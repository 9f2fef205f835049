#!/bin/bash
# r06: BASELINE config 5 with the reference CPU path beside the GPU path, in
# one session on one box: the C++ VirtualFile over the library (shmr_vfs_bench,
# mapped Block Cache, per-block tasks, fsync off / on) and the reference's own
# flow on 16 host threads with the oracle's AVX2 codec (tools/ref_cpu_vfs),
# interleaved twice; the CPU leg's shard files are compared byte for byte with
# the GPU leg's (same ino / idx naming).
set -o pipefail
O=gpurun_out/r06cfg5c
mkdir -p $O
B=/tmp/shmr_cfg5
for round in 1 2; do
  for fs in 0 1; do
    rm -rf $B && mkdir -p $B/gpu $B/cpu || exit 1
    SHMR_VFS_KEEP_FILES=1 SHMR_VFS_PINNED_ONLY=1 timeout -k 10 300 shmr_amd/_lib/shmr_vfs_bench $B/gpu 256 4 $fs 3 >> $O/gpu_vfs.jsonl 2>> $O/gpu_vfs.err || exit 1
    timeout -k 10 300 tools/_abx/ref_cpu_vfs $B/cpu 256 4 $fs 3 16 $B/gpu 1003 >> $O/cpu_ref.jsonl 2>> $O/cpu_ref.err || exit 1
    REF_CPU_REUSE=1 timeout -k 10 300 tools/_abx/ref_cpu_vfs $B/cpu 256 4 $fs 3 16 $B/gpu 1003 >> $O/cpu_ref.jsonl 2>> $O/cpu_ref.err || exit 1
  done
done
rm -rf $B
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $O/nproc.txt 2>/dev/null; grep -m1 "model name" /proc/cpuinfo >> $O/nproc.txt
echo "exit=$?"
