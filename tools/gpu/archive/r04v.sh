#!/bin/bash
# Round 4 (session 22): the long seeded random sweep (250 x the suite's cases) on the final library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/sweep_long.sh 250 || exit $?
echo done-v
