"""shmr_amd -- MI355X-native Reed-Solomon erasure path for shmr StorageBlocks.

Drop-in for the reference's ``reed_solomon_erasure::galois_8::ReedSolomon``
(src/vfs/block.rs:10) behind the C ABI in ``include/shmr_ec.h``; every byte
of GF(2^8) arithmetic runs in hand-written gfx950 HIP kernels
(``shmr_amd/csrc/gf_apply.hip``).  No CPU compute fallback exists.
"""
from .reed_solomon import (DeviceBuffer, Error, Op, capture_reserve, PinnedBuffer, ReedSolomon, ShardPool, ShardSlab, calculate_shard_size, describe_variant, device_count,  # noqa: F401
                           device_init, device_stats, get_tuning, host_register, host_unregister, kernel_inventory,
                           path_stats, queue_stats, set_tuning)

__version__ = "0.1.0"
