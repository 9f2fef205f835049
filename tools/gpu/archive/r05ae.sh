#!/bin/bash
# Round 5 (session 28): direct_io_pageable under LeakSanitizer does not finish.  Run it with
# line-buffered stdout (does main() complete?), and after 90 s record every thread's state,
# wait channel and current syscall from /proc before killing it; then the same run with the
# exit-time leak check off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ae
mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
timeout -k 10 900 bash tools/asan_host.sh build > $O/asan_build.log 2>&1 || { kill $HB; exit 1; }
BIN=tools/_probe/vfs_test_asan
python3 -c "import numpy as np; np.random.default_rng(7).integers(0, 256, 4194304, dtype=np.uint8).tofile('/tmp/in.bin')"
run_case() {   # $1 tag, $2 ASAN_OPTIONS
  rm -rf /tmp/b && mkdir -p /tmp/b
  ASAN_OPTIONS="$2:verify_asan_link_order=0" LSAN_OPTIONS="suppressions=$PWD/tools/lsan_rocm.supp:print_suppressions=0" \
    UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 stdbuf -oL -eL $BIN direct_io_pageable /tmp/b /tmp/in.bin > $O/$1.log 2>&1 &
  local pid=$!
  for i in $(seq 1 90); do kill -0 $pid 2>/dev/null || break; sleep 1; done
  if kill -0 $pid 2>/dev/null; then
    { echo "alive after 90 s: pid $pid"; for t in /proc/$pid/task/*; do
        echo "$(basename $t) $(cat $t/comm) state=$(awk '{print $3}' $t/stat) wchan=$(cat $t/wchan 2>/dev/null) syscall=$(cut -d' ' -f1 $t/syscall 2>/dev/null)"; done; } > $O/$1.threads.txt
    kill -9 $pid; wait $pid 2>/dev/null
    echo "killed" >> $O/$1.log
  else
    wait $pid; echo "exit=$?" >> $O/$1.log
  fi
}
run_case leaks "detect_leaks=1:protect_shadow_gap=0:halt_on_error=1"
run_case noexitcheck "detect_leaks=1:leak_check_at_exit=0:protect_shadow_gap=0:halt_on_error=1"
run_case noleaks "detect_leaks=0:protect_shadow_gap=0:halt_on_error=1"
kill $HB
echo done-ae
