#!/bin/bash
# Round 5 (session 24): host sanitizers with LeakSanitizer on (ROCm runtime suppressed).  First
# pass: abi_check and 26 StorageBlock cases clean; the erasure fuzz outran the per-case limit
# under the exit-time leak scan.  This pass: the three short cases after it, buckets under /tmp.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 900 bash tools/asan_host.sh build > $O/asan_build.log 2>&1 || exit $?
SECONDS=0
LEAKS=1 CASE_TIMEOUT=150 ONLY="erasure_flush_encode_failure direct_io_mapped direct_io_pageable" \
  timeout -k 10 600 bash tools/asan_host.sh run /tmp/asan3 > $O/asan_host_leaks3.log 2>&1
echo "rc=$? seconds=$SECONDS" >> $O/asan_host_leaks3.log
mkdir -p $O/asan3 && cp /tmp/asan3/*.log $O/asan3/ 2>/dev/null
echo done-aa
