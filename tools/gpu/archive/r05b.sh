#!/bin/bash
# Round 5 (session 2): shard-major slab legs of the pointer-table A/B, and the
# scalar-cache counters of the table kernels against the grid (strided)
# kernels over the same separate slabs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05b
mkdir -p $O
for c in encode83 decode83 encode104; do
  timeout -k 10 240 python -u tools/ptrs_ab.py --config $c --rounds 9 > $O/ptrs_ab_$c.txt 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
P1="SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P3="FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE"
for c in encode83 decode83; do
  legs=slab_sep,slab_sep_tab
  [ $c = decode83 ] && legs=slab,slab_tab
  n=1
  for P in "$P1" "$P2" "$P3"; do
    rm -rf /tmp/pmcraw
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d /tmp/pmcraw -o pmc -- \
      python3 $R/tools/ptrs_ab.py --config $c --rounds 2 --iters 5 --legs $legs > $R/$O/pmc_${c}_p$n.log 2>&1 || exit $?
    python3 $R/tools/pmc_summary.py /tmp/pmcraw --out $R/$O/pmc_${c}_p$n.json >> $R/$O/pmc_${c}_p$n.log 2>&1 || exit $?
    rm -rf /tmp/pmcraw
    n=$((n+1))
  done
done
echo done-b
