#!/usr/bin/env python3
"""Headline benchmark: GiB/s erasure-encoded (device-resident), RS(8,3) 4 MiB
StorageBlocks, on 1/2/4/8 MI355X (BASELINE.json ``metric``, ``configs[1]``).

A "step" is one pass of the hot path over one batch: encode every block of
the per-GPU batch (B blocks x 8 data shards x 524,288 B) into 3 parity shards,
inputs already resident in HBM (``--config`` selects the other BASELINE
configs: decodes, RS(10,4), RS(4,2), and ``codec104`` = encode + 2-erasure
rebuild per step).  Multi-GPU: one process per GPU, whole blocks
round-robin (global block b -> rank b % N), no collectives on the data path
(only the timing barrier / max-over-ranks reduction).  ``scaling`` is weak.

Prints ONE JSON line (rank 0).  ``roofline`` is computed from HIP events
recorded on the stream the kernel runs on; ``cpu_baseline`` times the CPU
restatement of the crate's AVX2 loop (oracle/, test infrastructure) on a
bounded sample of the same workload and checks the GPU parity of those sampled
blocks bit-for-bit.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import socket
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

# torch and shmr_amd are imported by the worker only (run()): the launcher
# parent of `--gpus N` must not touch the GPU before it starts its children.
np = torch = dist = shmr_amd = placement = _native = None

METRIC = "GiB/s erasure-encoded (device-resident), RS(8,3) 4 MiB StorageBlocks, 1/2/4/8 GPUs"
HBM_PEAK = 8.0e12          # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md)
SEED = 0x53484D52          # "SHMR"

CONFIGS = {
    # name: (k, p, block_bytes, erasures or None)
    "encode83": (8, 3, 4 << 20, None),
    "decode83": (8, 3, 4 << 20, 1),
    "encode104": (10, 4, 16 << 20, None),
    "decode104": (10, 4, 16 << 20, 2),
    "encode42": (4, 2, 1 << 20, None),
    # BASELINE config 4 as stated: encode, then rebuild 2 erased shards, per step
    "codec104": (10, 4, 16 << 20, -2),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100,
                    help="timed steps (default 100: ~46 ms of RS(8,3) encode, so the bracketing barrier / "
                         "synchronize costs < 0.5 %% of the timed region instead of ~2 %% at 20 steps)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="encode83", choices=sorted(CONFIGS))
    ap.add_argument("--blocks", type=int, default=0, help="blocks per GPU (default: 1024 for 1 MiB, 512 for 4 MiB, 64 for 16 MiB blocks)")
    ap.add_argument("--tune", default="", help="kernel knobs, e.g. 'chunks=2,grid=0' (default: library defaults)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=1.5, help="wall budget of the cpu_baseline sample")
    ap.add_argument("--backend", default="gloo", choices=["gloo", "nccl"],
                    help="process group for the timing barrier / max-over-ranks only (the data path "
                         "exchanges nothing between GPUs)")
    ap.add_argument("--contig", action="store_true",
                    help="batch buffers in physically contiguous VRAM (shmr_ec_device_alloc) instead of "
                         "torch's allocator; pays off on multi-GiB batches")
    ap.add_argument("--ramp-seconds", type=float, default=0.5,
                    help="untimed device clock ramp before the warmup steps (MI355X needs ~0.1 s of "
                         "sustained load to reach its steady clock)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the cpu_baseline leg (default: rayon's default pool size, "
                         "available_parallelism = sched affinity capped by the cgroup CPU quota; the "
                         "reference fans blocks out with rayon, mod.rs:93-96)")
    ap.add_argument("--pitch-align", type=int, default=4096,
                    help="device shard pitch = S rounded up to this many bytes (DESIGN.md section 4: 4 KiB "
                         "measured +0.7-1.0 point of HBM peak over 256 B for RS(10,4)'s S = 1,677,722); 1 = the "
                         "reference's packing, shard i at i * S (off 16-byte alignment for RS(10,4)); implies "
                         "--pitch-pad 0 unless the pad is given")
    ap.add_argument("--pitch-pad", type=int, default=-1,
                    help="bytes added to every shard slot after alignment; -1 (auto): one 4 KiB page when the "
                         "aligned pitch is a multiple of 64 KiB (power-of-two shard sizes: RS(8,3) 4 MiB, RS(4,2) "
                         "1 MiB: +1.7-1.8 points of HBM peak), none with --pitch-align 1; 0 = the reference's "
                         "contiguous block buffer for those sizes (DESIGN.md section 4)")
    ap.add_argument("--rebuild-out", default="compact", choices=["inplace", "compact"],
                    help="decode configs: rebuild the erased shards into a separate compact "
                         "[blocks][erasures][pitch] output -- the crate's semantics, every None shard rebuilt into "
                         "a fresh buffer (reference src/vfs/block.rs:556-565; shmr_ec_reconstruct_batch_dev_out; "
                         "default) -- or in place, in their block's own slots")
    ap.add_argument("--layout", default="batch", choices=["batch", "ptrs"],
                    help="batch: one [blocks][shards][pitch] tensor per role (shmr_ec_*_batch_dev); ptrs: every "
                         "shard its own GPU allocation named by a pointer table (shmr_ec_*_ptrs_dev) -- the "
                         "crate's shape, where each shard is a Vec<u8> of its own (reference block.rs:408-427) and "
                         "each rebuilt shard a fresh buffer (block.rs:556-565); not with codec104")
    ap.add_argument("--ptrs-alloc", default="slab", choices=["slab", "torch"],
                    help="--layout ptrs: where the shard buffers come from -- slab: shmr_ec_device_alloc_shards "
                         "(every shard of the batch in one slab at the slot pitch, rebuilt shards in a second "
                         "slab; the table forms a slot grid and runs through the strided kernels, knob ptrs_grid); "
                         "torch: one torch allocation per shard (table kernels)")
    ap.add_argument("--process-model", default="process", choices=["process", "single"],
                    help="process: one process per GPU (torchrun, or self-spawned for --gpus N); single: one "
                         "process drives all N GPUs with one host thread + stream each (the reference daemon's "
                         "shape, src/lib.rs:36-59)")
    ap.add_argument("--single-stream", default="own", choices=["own", "current"],
                    help=argparse.SUPPRESS)   # single model: a stream per device, or torch's current stream (A/B)
    ap.add_argument("--dump-dir", default="",
                    help="after the timed region, every rank writes the data and parity shards of its first "
                         "--dump-blocks blocks (encode configs) with their global block ids to "
                         "DIR/rank<r>.npz, for a test-side check against the CPU oracle")
    ap.add_argument("--dump-blocks", type=int, default=2)
    ap.add_argument("--no-host-probe", action="store_true",
                    help="skip the untimed host-path probe after the timed region (mapped Block-Cache blocks coded "
                         "zero-copy on this rank's GPU; rank 0 also over every visible GPU from one process)")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher rehearsal without a GPU: ranks join the process group, exchange their "
                         "identities and rank 0 prints one JSON line (tests/test_bench_launch.py)")
    return ap.parse_args()


_REAL_STDOUT = None


def quiet_stdout() -> None:
    """The contract is ONE JSON line on stdout, but native libraries print
    there too (Gloo: "[Gloo] Rank r is connected to n peer ranks ..." from
    every rank, interleaved): from here on fd 1 goes to stderr, and the line
    is written to the saved stdout (emit)."""
    global _REAL_STDOUT
    if _REAL_STDOUT is None:
        sys.stdout.flush()
        _REAL_STDOUT = os.dup(1)
        os.dup2(2, 1)


def emit(obj) -> None:
    line = (json.dumps(obj) + "\n").encode()
    if _REAL_STDOUT is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
        return
    sys.stdout.flush()
    view = memoryview(line)
    while view:                      # os.write may take only part of a long line
        view = view[os.write(_REAL_STDOUT, view):]


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(n: int, argv) -> int:
    """`bench.py --gpus N` started without a torch.distributed launcher: spawn
    N fresh worker processes of this script (rank r -> GPU r), wait for them
    and return the first failing exit status (0 if all succeed).  The parent
    never initialises the GPU and never re-execs itself; the children inherit
    stdout, where rank 0 prints the one JSON line.  Same partition as the
    torchrun launch: whole blocks round-robin, one process per GPU
    (reference per-block fan-out: src/vfs/mod.rs:91-103)."""
    port = os.environ.get("MASTER_PORT") or str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port,
                   SHMR_BENCH_LAUNCHER="spawn")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for pr in list(live):
            code = pr.poll()
            if code is None:
                continue
            live.remove(pr)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for other in live:          # a rank died: the others would wait in a collective forever
                    other.terminate()
        time.sleep(0.05)
    return rc


def launch_check(args) -> None:
    """Process-group rehearsal of a launch (no GPU, gloo): every rank reports
    its RANK / LOCAL_RANK / pid; rank 0 prints one JSON line."""
    import torch.distributed as dist_
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    me = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "pid": os.getpid(),
          "launcher": os.environ.get("SHMR_BENCH_LAUNCHER", "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ else "none")}
    ranks = [me]
    seen = 1
    if os.environ.get("SHMR_BENCH_LAUNCH_FAIL_RANK") == str(rank):
        sys.exit(3)      # test hook: a rank that dies before joining the group
    if world > 1:
        dist_.init_process_group("gloo")
        seen = dist_.get_world_size()
        ranks = [None] * seen
        dist_.all_gather_object(ranks, me)
    if rank == 0:
        emit({"launch_check": True, "n_gpus": args.gpus, "ranks_seen": seen, "ranks": ranks})
    if world > 1:
        dist_.destroy_process_group()


def main():
    args = parse()
    if args.process_model == "single":
        if "WORLD_SIZE" in os.environ and os.environ["WORLD_SIZE"] != "1":
            raise SystemExit("--process-model single runs as one process (not under a launcher)")
        quiet_stdout()
        return run_single(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args.gpus, sys.argv[1:]))
    quiet_stdout()
    if args.launch_check:
        return launch_check(args)
    run(args)


WORKLOADS = {"encode83": "RS(8,3) encode, 4 MiB StorageBlocks, device-resident",
             "decode83": "RS(8,3) reconstruct, 1 missing data shard (b mod 8), 4 MiB blocks",
             "encode104": "RS(10,4) encode, 16 MiB StorageBlocks, device-resident",
             "decode104": "RS(10,4) reconstruct, 2 erasures {b mod 10, (b+3) mod 10}, 16 MiB",
             "encode42": "RS(4,2) encode, 1 MiB StorageBlocks, device-resident",
             "codec104": "RS(10,4) encode + reconstruct of 2 erasures {b mod 10, (b+3) mod 10} per step, 16 MiB"}


class Shape:
    """The configuration's arithmetic and HBM layout (same on every device)."""

    def __init__(self, args):
        k, p, block_bytes, erasures = CONFIGS[args.config]
        self.k, self.p, self.block_bytes = k, p, block_bytes
        self.S = shmr_amd.calculate_shard_size(block_bytes, k)
        self.B = args.blocks or (1024 if block_bytes <= (1 << 20) else 512 if block_bytes <= (4 << 20) else 64)
        self.codec = erasures is not None and erasures < 0
        self.erasures = -erasures if self.codec else erasures
        self.compact = self.erasures is not None and args.rebuild_out == "compact"
        rows = p if self.erasures is None else self.erasures
        mode = 0 if self.erasures is None else 2 if self.compact else 1
        if args.layout == "ptrs":
            # slab buffers form a slot grid: the strided kernels run (encode, compact rebuild)
            mode = (0 if self.erasures is None else 2) if args.ptrs_alloc == "slab" else \
                (3 if self.erasures is None else 4)
        self.tuning = shmr_amd.describe_variant(mode, k, rows)
        if self.codec:
            self.tuning = f"encode: {shmr_amd.describe_variant(False, k, p)}; reconstruct: {self.tuning}"
        # HBM layout: shard i of block b at (b*k + i) * pitch with pitch = S
        # rounded up to 4 KiB, plus one 4 KiB page when that is a multiple of
        # 64 KiB: S = 524,288 (RS(8,3) 4 MiB) gets 528,384-byte slots (0.8 %
        # padding) instead of the reference's contiguous block buffer, whose
        # 2^19 shard stride measured 1.8 points of HBM peak slower (DESIGN.md
        # section 4); S = 1,677,722 (RS(10,4) 16 MiB) gets the page-aligned
        # 1,679,360-byte slots (0.1 %) and no page.
        a = max(1, args.pitch_align)          # 1: pitch = S, the reference's packing (any alignment)
        pitch = (self.S + a - 1) // a * a
        pad = args.pitch_pad
        if pad < 0:
            pad = 0 if a == 1 else (4096 if pitch % 65536 == 0 else 0)
        self.pitch = pitch + pad
        S, e = self.S, self.erasures
        self.algo_bytes_per_block = (k + p) * S if e is None else (k + e) * S + ((k + p) * S if self.codec else 0)
        self.payload_bytes_per_block = k * S


class Workload:
    """One device's batch: B whole blocks (global blocks rank + j * world,
    j < B: weak scaling, round-robin), synthetic data generated on the device,
    and the step that runs the hot path over all of them on `stream`."""

    def __init__(self, args, shape, dev, rank, world, rs, stream):
        self.shape, self.dev, self.rank, self.world, self.rs, self.stream = shape, dev, rank, world, rs, stream
        self.bufs = []
        k, p, S, B, pitch = shape.k, shape.p, shape.S, shape.B, shape.pitch
        g = torch.Generator(device=dev)
        g.manual_seed(SEED + rank)
        self.args = args
        self.ptrs = args.layout == "ptrs"
        if self.ptrs:
            self._init_ptrs(g)
            torch.cuda.synchronize(dev)
            return
        with torch.cuda.device(dev), torch.cuda.stream(stream):
            if shape.erasures is None:
                self.data = self.vram((B, k, pitch))
                self.data.copy_(torch.randint(0, 256, (B, k, pitch), dtype=torch.uint8, device=dev, generator=g))
                self.parity = self.vram((B, p, pitch))
            else:
                e = shape.erasures
                self.shards = self.vram((B, k + p, pitch))
                self.shards.zero_()
                self.shards[:, :k, :S] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
                rs.encode_batch_dev(self.shards[:, :k], self.shards[:, k:], shard_len=S,
                                    data_shard_pitch=pitch, parity_shard_pitch=pitch)
                present = np.ones((B, k + p), dtype=np.uint8)
                gb = np.array(placement.weak_batch(B, rank, world))         # global block ids of this device
                if e == 1:
                    present[np.arange(B), gb % k] = 0
                else:
                    present[np.arange(B), gb % 10] = 0                     # config 4: {b%10, (b+3)%10}
                    present[np.arange(B), (gb + 3) % 10] = 0
                self.present = present
                self.erased = torch.from_numpy(present == 0).to(dev)
                self.rebuilt = None
                self.reference = self.shards[:, :, :S].clone() if shape.codec else None
                if shape.compact:
                    # rebuilt shards into their own [B][erasures][pitch] array; for a
                    # pure rebuild the erased slots of the block buffer are zeroed
                    # (never read); codec104's encode needs every data shard, so
                    # there they stay
                    self.rebuilt = self.vram((B, e, pitch))
                    self.rebuilt.zero_()
                    self.originals = self.shards[self.erased][:, :S].clone().view(B, e, S)
                    if not shape.codec:
                        self.shards[self.erased] = 0
        torch.cuda.synchronize(dev)

    def _init_ptrs(self, g):
        """--layout ptrs: every shard a buffer of its own named by a pointer
        table (the crate's Vec<u8> per shard); the table is marshalled once, as
        a Rust shim would keep its Vec of pointers, and each step is one C call.
        --ptrs-alloc slab: the buffers come from shmr_ec_device_alloc_shards
        (INTEGRATION.md's Block Cache), torch: one torch allocation each."""
        sh, dev, rs = self.shape, self.dev, self.rs
        k, p, S, B = sh.k, sh.p, sh.S, sh.B
        t = k + p
        if sh.codec:
            raise SystemExit("--layout ptrs: encode and decode configs only (not codec104)")
        if self.args.ptrs_alloc == "slab":
            return self._init_slab(g)
        with torch.cuda.device(dev), torch.cuda.stream(self.stream):
            blocks = [[torch.randint(0, 256, (S,), dtype=torch.uint8, device=dev, generator=g) for _ in range(k)]
                      + [torch.zeros(S, dtype=torch.uint8, device=dev) for _ in range(p)] for _ in range(B)]
            self.stream_ptr = ctypes.c_void_p(self.stream.cuda_stream)
            self.blocks = blocks
            if sh.erasures is None:
                self.keep, _, _, self.ptab = rs._dev_table(blocks, lambda b, i: True)
                # [B, k|p, S] views for the cpu_baseline leg's parity check (copies, after timing)
                self.data = _Stacked(blocks, 0, k)
                self.parity = _Stacked(blocks, k, t)
                return
            rs.encode_ptrs_dev(blocks)
            present = np.ones((B, t), dtype=np.uint8)
            gb = np.array(placement.weak_batch(B, self.rank, self.world))     # global block ids of this device
            if sh.erasures == 1:
                present[np.arange(B), gb % k] = 0
            else:
                present[np.arange(B), gb % 10] = 0
                present[np.arange(B), (gb + 3) % 10] = 0
            self.present = present
            # absent entries: fresh output buffers (the crate allocates vec![0; len] per None)
            self.originals = [[blocks[b][i].clone() for i in np.flatnonzero(present[b] == 0)] for b in range(B)]
            self.outs = [[torch.zeros(S, dtype=torch.uint8, device=dev) for _ in np.flatnonzero(present[b] == 0)]
                         for b in range(B)]
            table = []
            for b in range(B):
                it = iter(self.outs[b])
                table.append([blocks[b][i] if present[b, i] else next(it) for i in range(t)])
            self.keep, _, _, self.ptab = rs._dev_table(table, lambda b, i: True)
            self.shards = _Stacked(blocks, 0, t)
            self.rebuilt = _Stacked(self.outs, 0, sh.erasures)

    def _init_slab(self, g):
        sh, dev, rs = self.shape, self.dev, self.rs
        k, p, S, B = sh.k, sh.p, sh.S, sh.B
        t = k + p
        self.stream_ptr = ctypes.c_void_p(self.stream.cuda_stream)
        with torch.cuda.device(dev), torch.cuda.stream(self.stream):
            if sh.erasures is None:
                # the encode's inputs and outputs in slabs of their own (measured: data and
                # parity interleaved in one slab run 1.7-3.6 points slower, profiles/r05/s1)
                self.dslab = shmr_amd.ShardSlab(B, k, S, device=dev.index)
                self.pslab = shmr_amd.ShardSlab(B, p, S, device=dev.index)
                self.data, self.parity = self.dslab.tensor(), self.pslab.tensor()
                self.data.zero_()
                self.parity.zero_()
                self.data[:, :, :S] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
                addrs = np.concatenate([self.dslab.ptrs.reshape(B, k), self.pslab.ptrs.reshape(B, p)], axis=1)
            else:
                self.slab = shmr_amd.ShardSlab(B, t, S, device=dev.index)
                view = self.slab.tensor()
                view.zero_()
                view[:, :k, :S] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
                addrs = self.slab.ptrs.reshape(B, t).copy()
                tab = np.ascontiguousarray(addrs.reshape(-1))
                _native_check(rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab.ctypes.data_as(ctypes.POINTER(
                    ctypes.POINTER(ctypes.c_uint8))), B, S, dev.index, self.stream_ptr))
                present = np.ones((B, t), dtype=np.uint8)
                gb = np.array(placement.weak_batch(B, self.rank, self.world))   # global block ids of this device
                if sh.erasures == 1:
                    present[np.arange(B), gb % k] = 0
                else:
                    present[np.arange(B), gb % 10] = 0
                    present[np.arange(B), (gb + 3) % 10] = 0
                self.present = present
                # a fresh buffer per None shard (the crate's vec![0; len]), from a second slab
                e = sh.erasures
                self.outs = shmr_amd.ShardSlab(B, e, S, device=dev.index)
                for b in range(B):
                    for j, i in enumerate(np.flatnonzero(present[b] == 0)):
                        addrs[b, i] = self.outs.ptrs[b * e + j]
                self.shards = view
                self.rebuilt = self.outs.tensor()
                self.rebuilt.zero_()
            self.ptab_arr = np.ascontiguousarray(addrs.reshape(-1))
            self.ptab = self.ptab_arr.ctypes.data_as(ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)))

    def vram(self, shape):
        """Batch tensor: torch's allocator, or with --contig physically
        contiguous VRAM from shmr_ec_device_alloc (footprint)."""
        if not self.args.contig:
            return torch.empty(shape, dtype=torch.uint8, device=self.dev)
        self.bufs.append(shmr_amd.DeviceBuffer(int(np.prod(shape)), device=self.dev.index, contiguous=True))
        return self.bufs[-1].tensor(shape)

    def encode(self):
        sh = self.shape
        if self.ptrs:
            _native_check(self.rs._L.shmr_ec_encode_ptrs_dev(self.rs._h, self.ptab, sh.B, sh.S, self.dev.index,
                                                             self.stream_ptr))
            return
        if sh.erasures is None:
            self.rs.encode_batch_dev(self.data, self.parity, shard_len=sh.S)
        else:
            self.rs.encode_batch_dev(self.shards[:, :sh.k], self.shards[:, sh.k:], shard_len=sh.S,
                                     data_shard_pitch=sh.pitch, parity_shard_pitch=sh.pitch)

    def rebuild(self):
        if self.ptrs:
            pr = self.present
            _native_check(self.rs._L.shmr_ec_reconstruct_ptrs_dev(
                self.rs._h, self.ptab, pr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), self.shape.B, self.shape.S,
                0, self.dev.index, self.stream_ptr))
            return
        if self.shape.compact:
            self.rs.reconstruct_batch_dev_out(self.shards, self.present, self.rebuilt, shard_len=self.shape.S)
        else:
            self.rs.reconstruct_batch_dev(self.shards, self.present, shard_len=self.shape.S)

    def step(self):
        """One pass of the hot path over the whole batch (enqueued on the
        current stream, which the callers set to self.stream)."""
        if self.shape.erasures is None:
            self.encode()
        elif self.shape.codec:
            # encode, then rebuild the erased shards: two launches per step,
            # algorithmic bytes of both ((k+p)S + (k+e)S per block)
            self.encode()
            self.rebuild()
        else:
            self.rebuild()

    def ramp_and_warmup(self):
        """Untimed clock ramp: the same step until ramp_seconds of wall time
        have passed (measured: with only 5 warmup steps, ~2 ms of work, the
        first timed steps run 10-15 % slow while the GPU clock ramps up), then
        the W warmup steps."""
        n, t = 0, time.perf_counter()
        with torch.cuda.device(self.dev), torch.cuda.stream(self.stream):
            while time.perf_counter() - t < self.args.ramp_seconds:
                for _ in range(8):
                    self.step()
                n += 8
                self.stream.synchronize()
            for _ in range(self.args.warmup):
                self.step()
            self.stream.synchronize()
        return n

    def timed(self, steps):
        """K steps bracketed by two HIP events on this device's stream (nothing
        else between the launches: an event after every step measured 0.9 %
        slower, profiles/r05/s8/gap_probe.txt); returns the region's
        milliseconds, one figure for the K steps (no per-step spread is
        measured; the stream is drained on return)."""
        with torch.cuda.device(self.dev), torch.cuda.stream(self.stream):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(self.stream)
            for _ in range(steps):
                self.step()
            e1.record(self.stream)
            self.stream.synchronize()
        return e0.elapsed_time(e1)

    def round_trip(self):
        """codec configs: the timed steps ran over already-consistent blocks --
        wipe the parity, encode, wipe the erased shards, rebuild them, and check
        every shard against the originals (device-side comparison)."""
        sh = self.shape
        with torch.cuda.device(self.dev), torch.cuda.stream(self.stream):
            self.shards[:, sh.k:] = 0
            self.encode()
            self.shards[self.erased] = 0
            if sh.compact:
                self.rebuilt.zero_()
            self.rebuild()
            self.stream.synchronize()
            if sh.compact:
                ok = bool(torch.equal(self.rebuilt[:, :, :sh.S], self.originals)) and bool(
                    torch.equal(self.shards[~self.erased][:, :sh.S], self.reference[~self.erased]))
                # put the rebuilt shards back into their slots (the buffer is whole
                # again for the cpu_baseline leg's parity check)
                self.shards[..., :sh.S][self.erased] = self.rebuilt[:, :, :sh.S].reshape(-1, sh.S)
            else:
                ok = bool(torch.equal(self.shards[:, :, :sh.S], self.reference))
        return ok


class _Stacked:
    """[B, rows, S] view of per-shard tensors for the cpu_baseline leg: indexing
    [:nb, :, :S] stacks the first nb blocks' shards (a copy, after the timed
    region)."""

    def __init__(self, blocks, lo, hi):
        self.blocks, self.lo, self.hi = blocks, lo, hi
        self.shape = (len(blocks), hi - lo, blocks[0][lo].numel() if blocks else 0)

    def __getitem__(self, idx):
        nb = range(len(self.blocks))[idx[0]] if isinstance(idx, tuple) else range(len(self.blocks))[idx]
        rest = idx[1:] if isinstance(idx, tuple) else ()
        st = torch.stack([torch.stack(self.blocks[b][self.lo:self.hi]) for b in nb])
        return st[(slice(None),) + rest] if rest else st


def _slot(S):
    pitch = (S + 4095) // 4096 * 4096
    return pitch + 4096 if pitch % 65536 == 0 else pitch


def _native_check(rc):
    if rc != 0:
        raise RuntimeError(f"shmr_ec call failed: {_native.lib().shmr_ec_status_name(rc).decode()}")


def device_identity(dev, rank):
    props = torch.cuda.get_device_properties(dev)
    return {"rank": rank, "device": dev.index,
            "pci_bus_id": f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}",
            "name": props.name}


def report(args, shape, world, ranks, elapsed, step_ms, ramp_steps, process_model, extra=None):
    """The one JSON line: value = payload of every block of every device over
    `elapsed` (max over devices); the roofline is the slowest device's."""
    B = shape.B
    value = shape.payload_bytes_per_block * B * world * args.steps / elapsed / 2 ** 30
    kern_s = float(np.mean(step_ms)) / 1e3          # one dominant launch per step (two for codec104)
    achieved = shape.algo_bytes_per_block * B / kern_s
    build_id = _native.lib().shmr_ec_build_id().decode()
    out = {
        "metric": METRIC if args.config == "encode83" else f"GiB/s {args.config} (device-resident)",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "process_model": process_model,
        "ranks_seen": len(ranks),
        "devices": ranks,
        "distinct_gpus": len({r["pci_bus_id"] for r in ranks}),
        "launcher": (os.environ.get("SHMR_BENCH_LAUNCHER", "torchrun" if world > 1 else "single")
                     if process_model == "process" else "threads"),
        "library": {"flavour": _native.flavour(), "build_id": build_id},
        "steps": args.steps,
        "warmup": args.warmup,
        "clock_ramp": {"seconds": args.ramp_seconds, "steps": ramp_steps},
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic uniform random bytes generated on-device (torch.randint, seeded per rank)",
        "config": {
            "workload": WORKLOADS[args.config] + ("" if args.layout != "ptrs" else
                                                   " +ptrs_slab (pointer tables over shmr_ec_device_alloc_shards "
                                                   "slabs: a slot grid, strided kernels)"
                                                   if args.ptrs_alloc == "slab" else
                                                   " +ptrs_torch (pointer tables over torch buffers: the table "
                                                   "kernels)"),
            "data_shards": shape.k, "parity_shards": shape.p, "shard_bytes": shape.S, "blocks_per_gpu": B,
            "global_batch_blocks": B * world,
            "parallelism": (f"blocks round-robin over {world} GPU(s), no data-path collectives " +
                            (f"({args.backend} only for the timing barrier / max-over-ranks)"
                             if process_model == "process" else
                             "(one process, one host thread + stream per GPU: the daemon's shape)")),
            "tuning": shape.tuning,
            "memory": ("physically contiguous VRAM (shmr_ec_device_alloc)" if args.contig
                       else "shmr_ec_device_alloc_shards slabs (hipMalloc)"
                       if args.layout == "ptrs" and args.ptrs_alloc == "slab"
                       else "torch caching allocator (hipMalloc)"),
            "shard_pitch_bytes": None if args.layout == "ptrs" else shape.pitch,
            "rebuild_out": (None if shape.erasures is None else
                            "a fresh buffer per None shard, named by the pointer table (crate semantics)"
                            if args.layout == "ptrs" else
                            "compact [blocks][erasures][pitch] output (crate semantics: a fresh buffer per None "
                            "shard)" if shape.compact else "in place, in the erased shards' own slots"),
            "shard_layout": (("every shard a buffer of its own from shmr_ec_device_alloc_shards "
                              f"({_slot(shape.S)} B slots; encode: data and parity shards in two slabs, rebuild: "
                              "every shard in one slab and the rebuilt shards in a second), named by a pointer table "
                              "(shmr_ec_*_ptrs_dev: the crate's Vec<u8> per shard); the table forms a slot grid, "
                              "which runs through the strided kernels"
                              if args.ptrs_alloc == "slab" else
                              "every shard a separate torch allocation, named by a pointer table (shmr_ec_*_ptrs_dev: "
                              "the crate's Vec<u8> per shard)") if args.layout == "ptrs" else
                             "contiguous shards (the reference's block buffer)" if shape.pitch == shape.S else
                             f"shard slots of {shape.pitch} B for {shape.S} B shards"
                             + (" (one 4 KiB page past the 4 KiB-aligned size for a power-of-two stride, "
                                "DESIGN.md section 4)" if shape.pitch - shape.S >= 4096 else " (4 KiB-aligned)")),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved / 1e9, 2),
            "peak": HBM_PEAK / 1e9,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK, 4),
            "traffic": None,
            "kernel_ms_avg": round(kern_s * 1e3, 4),
            "algorithmic_bytes_per_launch": shape.algo_bytes_per_block * B,
        },
        "cpu_baseline": None,
    }
    traffic, source = load_traffic(traffic_key(args), B, build_id, shape.tuning)
    out["roofline"]["traffic"] = traffic
    out["roofline"]["traffic_source"] = source
    if shape.codec:
        # two launches per step: the roofline figures are per step (both launches)
        out["roofline"]["launches_per_step"] = 2
        out["roofline"]["algorithmic_bytes_per_step"] = out["roofline"].pop("algorithmic_bytes_per_launch")
        out["roofline"]["step_ms_avg"] = out["roofline"].pop("kernel_ms_avg")
    out.update(extra or {})
    return out


def cpu_leg(args, shape, w):
    """cpu_baseline (rank 0 at N = 1 only): the oracle's restatement of the
    crate's loops timed on this host's cores, checking the GPU's outputs of
    the sampled blocks."""
    k, p, S = shape.k, shape.p, shape.S
    if shape.codec:
        enc = cpu_baseline(k, p, S, shape.block_bytes, w.shards[:, :k], w.shards[:, k:], args.cpu_seconds / 2,
                           args.cpu_threads)
        dec = cpu_baseline_decode(k, p, S, w.shards, w.present, args.cpu_seconds / 2, args.cpu_threads, w.rebuilt)
        rate = 1.0 / (1.0 / enc["value"] + 1.0 / dec["value"])
        return {
            "value": round(rate, 3), "unit": "GiB/s", "cores": enc["cores"], "kind": "port",
            "sample": "encode and reconstruct legs timed separately on bounded samples of the same "
                      "workload, combined as one step: 1 / (1/encode + 1/reconstruct); "
                      f"encode: {enc['sample']}; reconstruct: {dec['sample']}",
            "encode_GiBps": enc["value"], "reconstruct_GiBps": dec["value"],
            "cpu_model": enc["cpu_model"], "cpu_quota_cores": enc["cpu_quota_cores"],
            "gpu_parity_bit_exact_on_sample": enc["gpu_parity_bit_exact_on_sample"],
            "gpu_rebuilt_bit_exact_on_sample": dec["gpu_rebuilt_bit_exact_on_sample"],
        }
    if shape.erasures is None:
        return cpu_baseline(k, p, S, shape.block_bytes, w.data, w.parity, args.cpu_seconds, args.cpu_threads)
    return cpu_baseline_decode(k, p, S, w.shards, w.present, args.cpu_seconds, args.cpu_threads, w.rebuilt)


def import_runtime(args):
    global np, torch, dist, shmr_amd, placement, _native
    import numpy as np  # noqa: F811
    import torch  # noqa: F811  (before shmr_amd: share one HIP runtime)
    import torch.distributed as dist  # noqa: F811
    if args.tune:
        # kernel knobs are measurement variants: the tools build
        os.environ["SHMR_EC_FLAVOUR"] = "tools"
    import shmr_amd  # noqa: F811
    from shmr_amd import _native, placement  # noqa: F811
    for kv in filter(None, args.tune.split(",")):
        key, val = kv.split("=")
        shmr_amd.set_tuning(**{key: int(val)})


def run(args):
    """One process per GPU (torchrun or the self-launcher): this process's
    rank encodes / rebuilds its own B blocks on its GPU."""
    import_runtime(args)
    if args.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE')}")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if local >= ndev:
        # Rehearsal on a box with fewer GPUs than ranks (several ranks share a
        # GPU) is opt-in only; a real N-GPU run maps rank -> its own GPU.
        if os.environ.get("SHMR_BENCH_SHARE_GPU") != "1":
            raise SystemExit(f"LOCAL_RANK {local} but only {ndev} GPU(s) visible")
        local = local % ndev
    if world > 1:
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    ranks = [device_identity(dev, rank)]
    if world > 1:
        ranks = [None] * dist.get_world_size()
        dist.all_gather_object(ranks, device_identity(dev, rank))   # gloo by default: identities only

    shape = Shape(args)
    rs = shmr_amd.ReedSolomon(shape.k, shape.p)
    w = Workload(args, shape, dev, rank, world, rs, torch.cuda.current_stream(dev))
    ramp_steps = w.ramp_and_warmup()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    grids0 = shmr_amd.device_stats(dev.index)["ptr_table_grids"]
    t0 = time.perf_counter()
    region_ms = w.timed(args.steps)
    step_ms = region_ms / args.steps
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    grid_calls = shmr_amd.device_stats(dev.index)["ptr_table_grids"] - grids0
    if world > 1:
        dist.barrier()
    elapsed = max(wall, region_ms / 1e3)
    elapsed = placement.max_over_ranks(elapsed, device=dev if args.backend == "nccl" else None)
    out = report(args, shape, world, ranks, elapsed, step_ms, ramp_steps, "process")
    out["roofline"]["timed_region"] = {"steps": args.steps, "events_ms": round(region_ms, 4)}
    if args.layout == "ptrs":
        # pointer-table calls of the timed steps that ran as a slot grid (strided kernels)
        out["config"]["ptr_table_grid_calls_timed"] = grid_calls
    if shape.codec:
        out["roofline"]["round_trip_bit_exact"] = w.round_trip()
    if args.dump_dir and shape.erasures is None:
        dump_blocks(args, shape, w, rank, world)
    # per-rank figures (the line's roofline is the slowest rank's) and the host-path probe
    mine = {"rank": rank, "device": dev.index, "ms_per_step": round(float(np.mean(step_ms)), 4),
            "frac": round(shape.algo_bytes_per_block * shape.B / (float(np.mean(step_ms)) / 1e3) / HBM_PEAK, 4)}
    if not args.no_host_probe:
        mine["host_probe"] = host_probe(dev.index, all_devices=rank == 0)
    per_rank = [mine]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    out["per_rank"] = per_rank
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_leg(args, shape, w)
    if rank == 0:
        emit(out)
    if world > 1:
        dist.destroy_process_group()


def run_single(args):
    """The reference daemon's process model (src/lib.rs:36-59: one process;
    rayon fans blocks out, src/vfs/mod.rs:93-96): one process drives N GPUs,
    one host thread + HIP stream per GPU, whole blocks round-robin (device d
    owns global blocks d + j * N).  Aggregate = all devices' data / the slowest
    device's time (per-device HIP events, and the wall clock around all)."""
    import_runtime(args)
    n = args.gpus
    ndev = torch.cuda.device_count()
    if n > ndev and os.environ.get("SHMR_BENCH_SHARE_GPU") != "1":
        raise SystemExit(f"--gpus {n} but only {ndev} GPU(s) visible")
    devs = [torch.device("cuda", d % ndev) for d in range(n)]
    shape = Shape(args)
    rs = shmr_amd.ReedSolomon(shape.k, shape.p)
    for d in sorted({x.index for x in devs}):
        shmr_amd.device_init(d)                   # one-time per-device state, outside the timed region
    works = []
    for d, dev in enumerate(devs):
        st = torch.cuda.Stream(device=dev) if args.single_stream == "own" else torch.cuda.current_stream(dev)
        works.append(Workload(args, shape, dev, d, n, rs, st))
    ranks = [device_identity(dev, d) for d, dev in enumerate(devs)]
    results, wall = placement.fan_out([w.ramp_and_warmup for w in works], [lambda w=w: w.timed(args.steps)
                                                                             for w in works])
    ramp_steps = max(r[0] for r in results)
    per_dev_ms = [r[1] / args.steps for r in results]        # event-timed region / K steps
    dev_s = [r[1] / 1e3 for r in results]
    slowest = int(np.argmax(dev_s))
    elapsed = max(wall, max(dev_s))
    extra = {"per_device": [{"device": ranks[d], "ms_per_step": round(dev_s[d] / args.steps * 1e3, 4),
                             "frac": round(shape.algo_bytes_per_block * shape.B / (float(np.mean(per_dev_ms[d])) / 1e3)
                                           / HBM_PEAK, 4)} for d in range(n)]}
    out = report(args, shape, n, ranks, elapsed, per_dev_ms[slowest], ramp_steps, "single", extra)
    if shape.codec:
        out["roofline"]["round_trip_bit_exact"] = all(w.round_trip() for w in works)
    if n == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_leg(args, shape, works[0])
    emit(out)


def host_probe(local: int, all_devices: bool):
    """Untimed, after the timed region: the host path (BASELINE config 5's
    start and end in host memory) on this rank's GPU -- two RS(8,3) blocks in
    mapped Block-Cache memory coded zero-copy (shmr_ec_encode_blocks_host),
    their parity compared with a device-resident encode of the same bytes on
    the same GPU.  Rank 0 also codes 2 blocks per visible GPU from this one
    process, round-robin over all of them: on a multi-GPU node that is the
    check that mapped host memory is addressed the same way from every device
    (host_engine.cpp's zero-copy precondition)."""
    k, p, S = 8, 3, 65536
    ndev = torch.cuda.device_count()
    devices = list(range(ndev)) if all_devices else [local]
    nb = 2 * len(devices)
    rs = shmr_amd.ReedSolomon(k, p)
    buf = shmr_amd.PinnedBuffer(nb * (k + p) * S)
    arr = buf.array.reshape(nb, k + p, S)
    g = np.random.default_rng([SEED, local, nb])
    arr[:, :k] = g.integers(0, 256, (nb, k, S), dtype=np.uint8)
    arr[:, k:] = 0
    z0, s0 = shmr_amd.path_stats()
    before = {d: shmr_amd.device_stats(d)["blocks_encoded"] for d in devices}
    rs.encode_blocks_host(arr, devices=devices)
    z1, s1 = shmr_amd.path_stats()
    per_dev = {d: shmr_amd.device_stats(d)["blocks_encoded"] - before[d] for d in devices}
    with torch.cuda.device(local):
        data = torch.from_numpy(np.ascontiguousarray(arr[:, :k])).to(f"cuda:{local}")
        par = torch.zeros((nb, p, S), dtype=torch.uint8, device=f"cuda:{local}")
        rs.encode_batch_dev(data, par)
        torch.cuda.synchronize(local)
        same = bool(np.array_equal(par.cpu().numpy(), arr[:, k:]))
    del buf
    return {"devices": devices, "blocks": nb, "zero_copy_blocks": z1 - z0, "staged_blocks": s1 - s0,
            "blocks_per_device": [per_dev[d] for d in devices], "parity_equals_device_resident": same}


def dump_blocks(args, shape, w, rank, world):
    """--dump-dir: this rank's first blocks as coded (test-side oracle check of
    every rank's share, tests/test_gpu_dist.py)."""
    n = min(args.dump_blocks, shape.B)
    S = shape.S
    os.makedirs(args.dump_dir, exist_ok=True)
    np.savez(os.path.join(args.dump_dir, f"rank{rank}.npz"),
             data=w.data[:n, :, :S].cpu().numpy(), parity=w.parity[:n, :, :S].cpu().numpy(),
             blocks=np.array(placement.weak_batch(shape.B, rank, world)[:n]), device=w.dev.index)


def traffic_key(args) -> str:
    """Key of the PMC record for this run's configuration and layout: the
    config name, plus "+packed" for the reference's packing (--pitch-align 1),
    "+contig" for --pitch-pad 0 on a power-of-two shard, "+inplace" for a
    decode rebuilt in place (the compact output is the default)."""
    key = args.config
    if args.layout == "ptrs":
        # (r06: "+ptrs_slab" -- slab buffers on a slot grid, the strided kernels --
        # is not the table-kernel workload that "+ptrs" named before r05)
        return key + ("+ptrs_slab" if args.ptrs_alloc == "slab" else "+ptrs_torch")
    if args.pitch_align == 1:
        key += "+packed"
    elif args.pitch_pad == 0:
        key += "+contig"
    elif (args.pitch_align, args.pitch_pad) != (4096, -1):
        key += f"+pitch{args.pitch_align}_{args.pitch_pad}"
    if args.rebuild_out == "inplace" and CONFIGS[args.config][3] is not None:
        key += "+inplace"
    return key


def load_traffic(config: str, B: int, build_id: str, variant: str):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py), only if the
    record was measured on this kernel build and variant at this batch size;
    otherwise traffic is null and the source says why."""
    rel = os.path.join("profiles", "pmc_traffic.json")
    src = {"file": rel, "key": config, "build_id": build_id, "variant": variant}
    try:
        with open(os.path.join(HERE, rel)) as f:
            rec = json.load(f).get(config)
    except (OSError, ValueError):
        return None, dict(src, status="no record file")
    if not rec:
        return None, dict(src, status="no record for this config")
    for key, want in (("build_id", build_id), ("variant", variant), ("blocks", B)):
        if rec.get(key) != want:
            return None, dict(src, status=f"stale: recorded {key} {rec.get(key)!r} != running {want!r}")
    return rec.get("hbm_bytes_per_launch"), dict(src, status="match")


def affinity_cores() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_threads(requested: int) -> int:
    """rayon's default pool size: std::thread::available_parallelism(), i.e.
    the CPUs this process may run on (sched affinity) capped by the cgroup v2
    CPU quota rounded up (Rust std reads cpu.max on Linux).  On the GPU box
    the affinity set is 256 CPUs but the quota is 16 cores: 256 threads there
    are throttled to 16 cores' worth of time slices and measured 3.6x slower
    than 16 threads (36 vs 132 GiB/s, RS(8,3)), which is not what the
    reference's pool would do."""
    if requested > 0:
        return requested
    n = affinity_cores()
    q = cpu_quota()
    if q:
        n = min(n, max(1, int(-(-q // 1))))
    return n


def cpu_quota():
    """cgroup v2 CPU quota in cores (None if unlimited / unknown)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
        return None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        return None


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_baseline(k, p, S, block_bytes, data_t, parity_t, budget_s, threads=0):
    """CPU restatement of the crate's simd_c AVX2 loop (oracle/, "port"),
    one block per thread as rayon does over VirtualFile blocks, on every core
    this process may use (rayon's default pool); bounded sample of the same
    workload; also checks the GPU parity of the sampled blocks.  A 16-thread
    and a 1-core figure ride along."""
    from oracle import c_oracle   # cpu_baseline leg: oracle allowed here only
    cores = cpu_threads(threads)
    nb = min(max(256, 4 * cores), data_t.shape[0])   # >= 1 GiB of RS(8,3) data (past the host LLC), >= 4 blocks/thread
    host_data = data_t[:nb, :, :S].contiguous().cpu().numpy().reshape(-1)
    host_par = np.zeros(nb * p * S, dtype=np.uint8)
    reps, secs = 0, 0.0
    while secs < budget_s or reps == 0:
        secs += c_oracle.encode_batch(k, p, host_data, host_par, nb, S, cores, variant=1)
        reps += 1
    gpu_par = parity_t[:nb, :, :S].contiguous().cpu().numpy().reshape(-1)
    ok = bool(np.array_equal(gpu_par, host_par))
    gib = nb * k * S * reps / secs / 2 ** 30
    t16 = min(16, cores)
    reps16, secs16 = 0, 0.0
    while secs16 < budget_s / 3 or reps16 == 0:
        secs16 += c_oracle.encode_batch(k, p, host_data, host_par, nb, S, t16, variant=1)
        reps16 += 1
    single = c_oracle.encode_batch(k, p, host_data[: k * S], host_par[: p * S], 1, S, 1, variant=1)
    aff = affinity_cores()
    repsa, secsa = 0, 0.0
    while aff != cores and (secsa < budget_s / 3 or repsa == 0):
        secsa += c_oracle.encode_batch(k, p, host_data, host_par, nb, S, aff, variant=1)
        repsa += 1
    # the whole VirtualBlock::sync_data Erasure arm minus disk I/O (block.rs:406-430):
    # chunks(S).to_vec() copies, zero pad, zero shards, encode, per block
    ns = min(nb, max(1, (256 << 20) // block_bytes))
    src = np.zeros(ns * block_bytes, np.uint8)
    for b in range(ns):
        n = min(k * S, block_bytes)
        src[b * block_bytes:b * block_bytes + n] = host_data[b * k * S:b * k * S + n]
    sync_par = np.zeros(ns * p * S, np.uint8)
    sreps, ssecs = 0, 0.0
    while ssecs < budget_s / 3 or sreps == 0:
        ssecs += c_oracle.sync_data_batch(k, p, src, block_bytes, S, sync_par, ns, cores)
        sreps += 1
    sync_ok = bool(np.array_equal(sync_par, host_par[:ns * p * S])) if block_bytes >= k * S else None
    return {
        "value": round(gib, 3),
        "unit": "GiB/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{nb} blocks x {reps} reps of the same RS({k},{p}) workload ({secs:.1f} s wall, "
                  f"~{secs * cores:.0f} core-seconds), {cores} threads "
                  f"(one block per thread, AVX2 nibble-pshufb loop restating reed-solomon-erasure "
                  f"6.0.0 simd_c); encode only (erasure_encode_duration scope, block.rs:425-430)",
        "single_core_GiBps": round(k * S / single / 2 ** 30, 3),
        "threads16_GiBps": round(nb * k * S * reps16 / secs16 / 2 ** 30, 3),
        "affinity_cores": aff,
        "affinity_threads_GiBps": round(nb * k * S * repsa / secsa / 2 ** 30, 3) if repsa else round(gib, 3),
        "cpu_quota_cores": cpu_quota(),
        "threads_rule": "available_parallelism: sched affinity capped by the cgroup CPU quota (rayon's default pool)",
        "sync_data_GiBps": round(ns * block_bytes * sreps / ssecs / 2 ** 30, 3),
        "sync_data_sample": f"{ns} blocks x {sreps} reps: chunk to_vec copies + zero pad/shards + encode "
                            f"per block (block.rs:406-430), {cores} threads",
        "sync_data_parity_matches": sync_ok,
        "cpu_model": cpu_model(),
        "gpu_parity_bit_exact_on_sample": ok,
    }


def cpu_baseline_decode(k, p, S, shards_t, present, budget_s, threads=0, rebuilt_t=None):
    """CPU restatement of the crate's reconstruct (first k present shards,
    inverted sub-matrix, SIMD mul_slice loop; oracle/, "port"), one block per
    thread; bounded sample of the same decode workload.  The GPU's rebuilt
    shards of the sampled blocks (in place, or rows of the compact output
    `rebuilt_t`) are checked bit-for-bit against it."""
    from oracle import c_oracle   # cpu_baseline leg: oracle allowed here only
    cores = cpu_threads(threads)
    t = k + p
    nb = min(shards_t.shape[0], max(1, (1 << 30) // (t * S), 4 * cores))
    gpu = np.ascontiguousarray(shards_t[:nb, :, :S].cpu().numpy())
    pr = np.ascontiguousarray(present[:nb], dtype=np.uint8)
    if rebuilt_t is not None:   # compact output: row j = the j-th erased shard of the block
        rows = rebuilt_t[:nb, :, :S].cpu().numpy()
        for b in range(nb):
            for j, i in enumerate(np.flatnonzero(pr[b] == 0)):
                gpu[b, i] = rows[b, j]
    work = gpu.copy()
    work[pr == 0] = 0
    reps, secs = 0, 0.0
    while secs < budget_s or reps == 0:
        secs += c_oracle.reconstruct_batch(k, p, work, pr, S, cores)
        reps += 1
    ok = bool(np.array_equal(work, gpu))
    t16 = min(16, cores)
    reps16, secs16 = 0, 0.0
    while secs16 < budget_s / 3 or reps16 == 0:
        secs16 += c_oracle.reconstruct_batch(k, p, work, pr, S, t16)
        reps16 += 1
    single = c_oracle.reconstruct_batch(k, p, work[:1], pr[:1], S, 1)
    aff = affinity_cores()
    repsa, secsa = 0, 0.0
    while aff != cores and (secsa < budget_s / 3 or repsa == 0):
        secsa += c_oracle.reconstruct_batch(k, p, work, pr, S, aff)
        repsa += 1
    return {
        "value": round(nb * k * S * reps / secs / 2 ** 30, 3),
        "unit": "GiB/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{nb} blocks x {reps} reps of the same decode workload ({secs:.1f} s wall, "
                  f"~{secs * cores:.0f} core-seconds), {cores} threads (one block per thread; crate reconstruct "
                  f"restated: inv(M[first k present]) + AVX2 nibble-pshufb mul_slice)",
        "single_core_GiBps": round(k * S / single / 2 ** 30, 3),
        "threads16_GiBps": round(nb * k * S * reps16 / secs16 / 2 ** 30, 3),
        "affinity_cores": aff,
        "affinity_threads_GiBps": (round(nb * k * S * repsa / secsa / 2 ** 30, 3) if repsa
                                   else round(nb * k * S * reps / secs / 2 ** 30, 3)),
        "cpu_quota_cores": cpu_quota(),
        "threads_rule": "available_parallelism: sched affinity capped by the cgroup CPU quota (rayon's default pool)",
        "cpu_model": cpu_model(),
        "gpu_rebuilt_bit_exact_on_sample": ok,
    }


if __name__ == "__main__":
    main()
