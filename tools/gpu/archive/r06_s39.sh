#!/bin/bash
# r06 session 39: table kernels with tile pairs (tools knob pair) against the
# policy's one tile per workgroup, torch per-shard buffers, four configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s39
mkdir -p $O
for c in encode83 decode83 encode104 decode104; do
  SHMR_EC_FLAVOUR=tools timeout -k 10 240 python tools/pair_ab.py --config $c --rounds 11 > $O/pair_ab_$c.jsonl 2> $O/pair_ab_$c.err || exit 1
done
for c in encode83 decode83; do
  SHMR_EC_FLAVOUR=tools timeout -k 10 240 python tools/pair_ab.py --config $c --rounds 11 > $O/pair_ab_${c}_rep.jsonl 2> $O/pair_ab_${c}_rep.err || exit 1
done
echo done-s39
