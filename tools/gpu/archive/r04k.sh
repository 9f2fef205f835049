#!/bin/bash
# Round 4 (session 11): the soak's remaining interaction (a host batch of RS(17,7) failing while
# another thread's captured encode is invalidated), reduced to ops 1 + 6, with HIP's API log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 120 python -u tools/soak.py --seconds 40 --threads 4 --ops 1,6 --shapes 4,6 > $O/soak_ops16.log 2>&1
rc=$?
echo "soak rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AMD_LOG_LEVEL=3 timeout -k 10 120 python -u tools/soak.py --seconds 20 --threads 4 --ops 1,6 --shapes 4,6 > $O/soak_ops16_log3.out 2> $O/hiplog.txt
rc=$?
echo "logged soak rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
python - <<'PY'
import re
lines = open("gpurun_out/r04k/hiplog.txt", errors="replace").read().splitlines()
bad = [i for i, l in enumerate(lines) if "Returned" in l and "hipSuccess" not in l and "hipErrorNotReady" not in l]
with open("gpurun_out/r04k/hiplog_errors.txt", "w") as f:
    f.write(f"{len(lines)} lines, {len(bad)} non-success returns\n")
    for i in bad[:40]:
        f.write("\n".join(lines[max(0, i - 12): i + 2]) + "\n----\n")
PY
rm -f $O/hiplog.txt
echo done-k
