#!/bin/bash
# rocprofv3 kernel-trace + PMC passes for every bench config (tools/profile.sh),
# one after the other; stops at the first failure.  Algorithmic bytes per
# launch: B * (k + rows) * S -- for RS(10,4) (S = 1,677,722, not a multiple of
# the tile) the partial last tiles run at the head of the same launch.
# Usage: tools/profile_all.sh <round-tag> [part: 1 = the bench configs, 2 = the layout / output
# variants, 3 = the pointer-table layouts only, default 1 + 2 -- one part fits one 20-minute GPU call]
set -eu
T=$1
PART=${2:-all}
D="$(cd "$(dirname "$0")" && pwd)"
if [ "$PART" = all ] || [ "$PART" = 1 ]; then
bash "$D/profile.sh" "$T" encode83 512 2952790016
bash "$D/profile.sh" "$T" decode83 512 2415919104
bash "$D/profile.sh" "$T" encode104 64 $((64 * 14 * 1677722))
bash "$D/profile.sh" "$T" decode104 64 $((64 * 12 * 1677722))
bash "$D/profile.sh" "$T" encode42 1024 1610612736
bash "$D/profile.sh" "$T" codec104 64 $((64 * 26 * 1677722)) --sum-kernels
fi
[ "$PART" != 1 ] || exit 0
if [ "$PART" != 3 ]; then
# round 3: decodes rebuilt in place (the compact output, the crate's semantics, is the bench
# default) and the reference's packed / contiguous layouts (bench.py traffic_key)
KEY=decode83+inplace BENCH_EXTRA="--rebuild-out inplace" bash "$D/profile.sh" "$T" decode83 512 2415919104
KEY=decode104+inplace BENCH_EXTRA="--rebuild-out inplace" bash "$D/profile.sh" "$T" decode104 64 $((64 * 12 * 1677722))
KEY=encode104+packed BENCH_EXTRA="--pitch-align 1" bash "$D/profile.sh" "$T" encode104 64 $((64 * 14 * 1677722))
KEY=decode104+packed BENCH_EXTRA="--pitch-align 1" bash "$D/profile.sh" "$T" decode104 64 $((64 * 12 * 1677722))
KEY=encode83+contig BENCH_EXTRA="--pitch-pad 0" bash "$D/profile.sh" "$T" encode83 512 2952790016
KEY=decode83+contig BENCH_EXTRA="--pitch-pad 0" bash "$D/profile.sh" "$T" decode83 512 2415919104
fi
# every shard its own buffer, named by a pointer table (the crate's shape, --layout ptrs): r05 slab
# buffers from shmr_ec_device_alloc_shards (a slot grid: strided kernels), and torch allocations
KEY=encode83+ptrs_slab BENCH_EXTRA="--layout ptrs" bash "$D/profile.sh" "$T" encode83 512 2952790016
KEY=decode83+ptrs_slab BENCH_EXTRA="--layout ptrs" bash "$D/profile.sh" "$T" decode83 512 2415919104
KEY=encode104+ptrs_slab BENCH_EXTRA="--layout ptrs" bash "$D/profile.sh" "$T" encode104 64 $((64 * 14 * 1677722))
KEY=decode104+ptrs_slab BENCH_EXTRA="--layout ptrs" bash "$D/profile.sh" "$T" decode104 64 $((64 * 12 * 1677722))
KEY=encode83+ptrs_torch BENCH_EXTRA="--layout ptrs --ptrs-alloc torch" bash "$D/profile.sh" "$T" encode83 512 2952790016
KEY=decode83+ptrs_torch BENCH_EXTRA="--layout ptrs --ptrs-alloc torch" bash "$D/profile.sh" "$T" decode83 512 2415919104
KEY=encode104+ptrs_torch BENCH_EXTRA="--layout ptrs --ptrs-alloc torch" bash "$D/profile.sh" "$T" encode104 64 $((64 * 14 * 1677722))
