#!/usr/bin/env python3
"""Does the aligned vector kernel (mode 0) run correctly on shards that are not
16-byte aligned, i.e. does the hardware's unaligned global access serve
misaligned global_load/store_dwordx4?  Tools build, knob uvec=1; RS(10,4) and
RS(8,3) encodes of contiguous (shard i at i * L) layouts checked against the
oracle, guard bytes around the batch checked."""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

os.environ.setdefault("SHMR_EC_FLAVOUR", "tools")
import shmr_amd  # noqa: E402
from oracle import c_oracle  # noqa: E402   (checker only)


def main():
    gpu = torch.device("cuda", 0)
    ok_all = True
    for uvec in (0, 1):
        shmr_amd.set_tuning(uvec=uvec)
        for (k, p, L, B, off) in [(10, 4, 1677722, 2, 0), (8, 3, 524288 + 4096 + 5, 2, 3), (4, 4, 8192, 2, 9)]:
            t = k + p
            rng = np.random.default_rng(L + off)
            host = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
            flat = torch.full((off + B * t * L + 64,), 0x5A, dtype=torch.uint8, device=gpu)
            blocks = flat[off:off + B * t * L].view(B, t, L)
            blocks[:, :k] = torch.from_numpy(host).to(gpu)
            rs = shmr_amd.ReedSolomon(k, p)
            rs.encode_batch_dev(blocks[:, :k], blocks[:, k:], shard_len=L, data_shard_pitch=L, parity_shard_pitch=L)
            torch.cuda.synchronize()
            got = blocks.cpu().numpy()
            ok = True
            for b in range(B):
                sh = [host[b, i].copy() for i in range(k)] + [np.zeros(L, np.uint8) for _ in range(p)]
                c_oracle.encode(k, p, sh)
                for r in range(p):
                    ok = ok and np.array_equal(got[b, k + r], sh[k + r])
                ok = ok and np.array_equal(got[b, :k], host[b])
            edge = flat.cpu().numpy()
            ok = ok and bool((edge[:off] == 0x5A).all() and (edge[off + B * t * L:] == 0x5A).all())
            print(f"uvec={uvec} RS({k},{p}) L={L} off={off}: {'bit-exact' if ok else 'MISMATCH'}", flush=True)
            ok_all = ok_all and ok
    shmr_amd.set_tuning(uvec=0)
    sys.exit(0 if ok_all else 1)


if __name__ == "__main__":
    main()
