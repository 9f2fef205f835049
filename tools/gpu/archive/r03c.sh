#!/bin/bash
# Round 3, third GPU pass: in-place vs compact rebuilds interleaved in one
# process with real parity content; load/store cache policy on the packed
# layout; the available PMC counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03c
mkdir -p $O
T="timeout -k 10"
$T 60 rocprofv3 -L > $O/rocprofv3_avail.txt 2>&1
$T 400 python tools/tune.py --config decode83 --pad 4096 --rounds 11 \
  --variants "compact=0,nt_load=1,nt_store=1,depth=2,wgs_per_cu=7;compact=1,nt_load=1,nt_store=1,depth=2,wgs_per_cu=7;compact=0,nt_load=1,depth=2,sc1_store=1;compact=1,nt_load=1,depth=2,sc1_store=1;compact=0,nt_load=1,nt_store=1,depth=2,threads=512;compact=1,nt_load=1,nt_store=1,depth=2,threads=512;compact=1,nt_load=1,nt_store=1,depth=2" > $O/tune_decode83_inplace_vs_compact.txt 2>&1 &&
$T 400 python tools/tune.py --config decode104 --align 4096 --rounds 11 \
  --variants "compact=0,nt_load=1,nt_store=1,depth=2,fuse_tail=1;compact=1,nt_load=1,nt_store=1,depth=2,fuse_tail=1;compact=0,nt_load=1,depth=2,fuse_tail=1,sc1_store=1;compact=1,nt_load=1,depth=2,fuse_tail=1,sc1_store=1" > $O/tune_decode104_inplace_vs_compact.txt 2>&1 &&
$T 400 python tools/tune.py --config encode104 --packed --rounds 11 \
  --variants "chunks=2,nt_load=1,nt_store=1,depth=2,early=1,serial=1,fuse_tail=1;chunks=2,nt_load=0,nt_store=1,depth=2,early=1,serial=1,fuse_tail=1;chunks=2,nt_load=1,nt_store=0,depth=2,early=1,serial=1,fuse_tail=1;chunks=2,nt_load=0,nt_store=0,depth=2,early=1,serial=1,fuse_tail=1;chunks=2,nt_load=0,nt_store=1,depth=2,fuse_tail=1" > $O/tune_encode104_packed_cachepol.txt 2>&1 &&
$T 400 python tools/tune.py --config decode104 --packed --rounds 11 \
  --variants "nt_load=1,nt_store=1,depth=2,fuse_tail=1;nt_load=0,nt_store=1,depth=2,fuse_tail=1;nt_load=1,nt_store=0,depth=2,fuse_tail=1;nt_load=0,nt_store=0,depth=2,fuse_tail=1" > $O/tune_decode104_packed_cachepol.txt 2>&1 &&
for i in 1 2; do
  $T 180 python bench.py --config decode83 --cpu-seconds 0.3 >> $O/bench_decode83_inplace.jsonl 2>>$O/bench.err &&
  $T 180 python bench.py --config decode83 --rebuild-out compact --cpu-seconds 0.3 >> $O/bench_decode83_compact.jsonl 2>>$O/bench.err || exit 1
done
