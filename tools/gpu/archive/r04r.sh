#!/bin/bash
# Round 4 (session 18): does the host code of this session (relaxed capture mode at every entry,
# mirrored events) cost the bench anything?  Product library now vs 6cec136, in one process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04r
mkdir -p $O
for c in encode83 decode83 encode104; do
  timeout -k 10 300 python tools/ab_libs.py tools/_abh/libshmr_ec_6cec136.so --config $c > $O/ab_$c.txt 2>&1 || exit $?
done
echo done-r
