#!/bin/bash
# Round 4 (session 6): the host sanitizer build -- ASan + UBSan on every host TU, the kernel TU
# included now that its launches are by name -- run on the GPU (bit-exact parity, no report),
# then a 120 s soak of every entry point incl. started calls and graph captures.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 bash tools/asan_host.sh build > $O/asan_build.log 2>&1 || exit $?
timeout -k 10 600 bash tools/asan_host.sh run $O/asan > $O/asan_host.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/soak.py --seconds 120 --threads 12 > $O/soak.log 2>&1 || exit $?
echo done-f
