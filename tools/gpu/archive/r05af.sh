#!/bin/bash
# Round 5 (session 29): direct_io_pageable under LeakSanitizer, four fresh processes through the
# asan_host.sh path (under `timeout`), each with line-buffered output: a stall is located before or
# after main() printed PASS, and the stalled process's threads are recorded from /proc.  Stops at
# the first stall.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05af
mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
timeout -k 10 900 bash tools/asan_host.sh build > $O/asan_build.log 2>&1 || { kill $HB; exit 1; }
BIN=tools/_probe/vfs_test_asan
python3 -c "import numpy as np; np.random.default_rng(7).integers(0, 256, 4194304, dtype=np.uint8).tofile('/tmp/in.bin')"
export ASAN_OPTIONS="detect_leaks=1:protect_shadow_gap=0:halt_on_error=1:verify_asan_link_order=0"
export LSAN_OPTIONS="suppressions=$PWD/tools/lsan_rocm.supp:print_suppressions=0"
for i in 1 2 3 4; do
  rm -rf /tmp/b && mkdir -p /tmp/b
  timeout -k 5 100 stdbuf -oL -eL $BIN direct_io_pageable /tmp/b /tmp/in.bin > $O/run$i.log 2>&1 &
  tpid=$!
  sleep 2
  pid=$(pgrep -P $tpid | head -1)
  for s in $(seq 1 80); do kill -0 $tpid 2>/dev/null || break; sleep 1; done
  if kill -0 $tpid 2>/dev/null; then
    { echo "run $i alive after ~80 s: pid $pid"; for t in /proc/$pid/task/*; do
        echo "$(basename $t) $(cat $t/comm) state=$(awk '{print $3}' $t/stat) wchan=$(cat $t/wchan 2>/dev/null) syscall=$(cut -d' ' -f1 $t/syscall 2>/dev/null)"; done; } > $O/run$i.threads.txt
    wait $tpid; echo "exit=$? (stalled)" >> $O/run$i.log
    break
  fi
  wait $tpid; echo "exit=$?" >> $O/run$i.log
done
kill $HB
echo done-af
