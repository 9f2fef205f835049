#!/bin/bash
# Round 5 (session 8): inter-launch gaps of the headline step (tools/gap_probe.py), plus the
# kernel trace of the same run for the kernels' own durations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 300 python tools/gap_probe.py --rounds 11 --steps 20 > $O/gap_probe.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/gapkt -o kt -- \
  python3 $R/tools/gap_probe.py --rounds 3 --steps 20 > $R/$O/gap_probe_rocprof.txt 2>&1 || exit $?
cp /tmp/gapkt/*/kt_kernel_stats.csv $R/$O/ 2>/dev/null || find /tmp/gapkt -name '*kernel_stats.csv' -exec cp {} $R/$O/ \;
python3 - <<'PY' >> $R/$O/gap_probe_rocprof.txt
import csv, glob
rows = []
for p in glob.glob('/tmp/gapkt/**/*kernel_trace.csv', recursive=True):
    rows += [r for r in csv.DictReader(open(p)) if 'gf_apply_kernel' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
gaps = [int(b['Start_Timestamp']) - int(a['End_Timestamp']) for a, b in zip(rows, rows[1:])]
gaps = [g for g in gaps if g < 100000]
gaps.sort()
print({"kernels": len(rows), "gap_ns_median": gaps[len(gaps)//2] if gaps else None, "gap_ns_p10": gaps[len(gaps)//10] if gaps else None})
PY
echo done-h
