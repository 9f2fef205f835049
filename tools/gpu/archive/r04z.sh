#!/bin/bash
# Round 4 (session 26): host sanitizers (ASan + UBSan, kernel TU included) on the final host code.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04z
mkdir -p $O
timeout -k 10 600 bash tools/asan_host.sh build > $O/asan_build.log 2>&1 || exit $?
timeout -k 10 600 bash tools/asan_host.sh run $O/asan > $O/asan_host.log 2>&1 || exit $?
echo done-z
