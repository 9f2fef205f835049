#!/bin/bash
# Round 3 final build: rocprofv3 kernel-trace + PMC (FETCH_SIZE / WRITE_SIZE) passes, part $1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/profile_all.sh r03 "${1:-1}" > gpurun_out/profile_all_r03_part${1:-1}.log 2>&1
