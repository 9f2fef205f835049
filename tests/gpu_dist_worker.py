"""One rank of the multi-process GPU parity check (tests/test_gpu_dist.py),
started by torch.distributed.run: whole blocks round-robin over ranks
(shmr_amd.placement, the reference's per-block fan-out src/vfs/mod.rs:93-96),
each rank encodes and rebuilds ITS blocks through the library on its GPU, and
rank 0 prints every block's digests (gathered over gloo -- test-side only, the
data path exchanges nothing).  Ranks may share one GPU (SHMR_BENCH_SHARE_GPU=1).
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import shmr_amd  # noqa: E402
from shmr_amd import placement  # noqa: E402

K, P, S, NBLOCKS, SEED = 8, 3, 65536 + 48, 13, 0x53484D52


def block_data(b):
    return np.random.default_rng([SEED, b]).integers(0, 256, (K, S), dtype=np.uint8)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % ndev if os.environ.get("SHMR_BENCH_SHARE_GPU") == "1" else local)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    mine = placement.blocks_for_rank(NBLOCKS, rank, world)
    rs = shmr_amd.ReedSolomon(K, P)
    data = torch.from_numpy(np.stack([block_data(b) for b in mine])).to(dev)
    parity = torch.zeros((len(mine), P, S), dtype=torch.uint8, device=dev)
    rs.encode_batch_dev(data, parity, shard_len=S)
    shards = torch.cat([data, parity], dim=1).contiguous()
    full = shards.clone()
    present = np.ones((len(mine), K + P), np.uint8)
    for j, b in enumerate(mine):   # two erasures per block, a different pattern per global block
        present[j, [b % (K + P), (b + 5) % (K + P)]] = 0
    shards[torch.from_numpy(present == 0).to(dev)] = 0
    rs.reconstruct_batch_dev(shards, present, shard_len=S)
    torch.cuda.synchronize(dev)
    out = {}
    host_par = parity.cpu().numpy()
    for j, b in enumerate(mine):
        out[b] = {"rank": rank, "parity_sha256": hashlib.sha256(host_par[j].tobytes()).hexdigest()}
    rebuilt_ok = bool(torch.equal(shards, full))
    gathered = [None] * world
    dist.all_gather_object(gathered, {"blocks": out, "rebuilt_ok": rebuilt_ok, "device": str(dev)})
    if rank == 0:
        print(json.dumps({"world": world, "ranks": gathered}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
