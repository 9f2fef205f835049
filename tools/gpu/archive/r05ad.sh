#!/bin/bash
# Round 5 (session 27): how long the two cases that outran 120-150 s under LeakSanitizer take
# (exit-time leak scan), with a 400 s limit each; a heartbeat file shows the run is alive.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ad
mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
timeout -k 10 900 bash tools/asan_host.sh build > $O/asan_build.log 2>&1 || { kill $HB; exit 1; }
for c in direct_io_pageable virtual_file_erasure_fuzz; do
  SECONDS=0
  LEAKS=1 CASE_TIMEOUT=400 ONLY="$c" timeout -k 10 450 bash tools/asan_host.sh run /tmp/asan_$c > $O/leaks_$c.log 2>&1
  echo "rc=$? seconds=$SECONDS" >> $O/leaks_$c.log
  cp /tmp/asan_$c/$c.log $O/$c.case.log 2>/dev/null
  rm -rf /tmp/asan_$c
done
kill $HB
echo done-ad
