#!/bin/bash
# r06 session 42: host ASan + UBSan (no LSan on the GPU box) on the final host
# code: abi_check and every StorageBlock case (build: tools/asan_host.sh build,
# copied to tools/_asanrun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s42
mkdir -p $O
ASAN_DIR=tools/_asanrun timeout -k 10 900 bash tools/asan_host.sh run $O/asan > $O/asan.log 2>&1 || exit $?
echo done-s42
