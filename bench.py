#!/usr/bin/env python3
"""Benchmark: GiB/s of Merkle leaf-hash + tree-reduce over device-resident record values.

One step = the Merkle step of one SSTable build on each GPU: SHA-1 of every value
(NewLeaf, merklenode.go:27-34) + the full tree (build, merkletree.go:31-64) over
BASELINE config 2 -- 1 Mi values x 4 KiB, resident in HBM when timing starts.
With N > 1 ranks each GPU builds its own table (one run per GPU, as in
lsmtree compaction) and the 20-byte roots are all-gathered over RCCL every step.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints one JSON line (see DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md (chip table)
# Measured compute ceiling of the per-lane SHA-1 (no memory traffic, 8 waves/SIMD,
# 2.37-2.39 GHz): tools/sha1_rate.hip -> profiles/r01_sha1_compute_rate.txt.
SHA1_VALU_CEILING_GBS = 4100.0
# (The LDS-DMA loop streamed random bytes at ~2.04 GHz under the board power
# limit, profiles/r01_clock_power.txt; the register-load loop that replaced it
# runs faster than that clock allows, so no fixed streaming-clock ceiling is
# reported.)
# k_leaf_verify's block loop issues ~711 VALU per 64-B block (SHA-1's 614 plus
# 97 for the CRC's byte indices and three-input XORs; ISA count, DESIGN.md
# K1v) against ~618.5 for the plain leaf kernel, so its compute ceiling is the
# SHA-1 one scaled by that ratio.
VERIFY_VALU_RATIO = 618.5 / 711.0
SEED = 0x6E616B65
SEED_MIXED = 0x6E616B66


LEAF_KERNEL = {-1: "library default", 0: "k_leaf, one-block lookahead", 1: "k_leaf, deep register prefetch",
               2: "k_leaf_queue, deep register prefetch", 3: "k_leaf_queue, LDS chunk ring"}


def mixed_lengths(target_bytes: int, seed: int):
    """BASELINE configs[2]: L = floor(2^U(6,16)) (64 B - 64 KiB, log-uniform), values
    packed back to back (so mostly unaligned), until the payload reaches target_bytes."""
    import numpy as np
    rng = np.random.default_rng(seed)
    est = int(target_bytes / 9000) + 1024
    lens = np.floor(2.0 ** rng.uniform(6, 16, est)).astype(np.uint64)
    cs = np.cumsum(lens)
    k = int(np.searchsorted(cs, target_bytes, side="right"))
    lens = lens[:max(k, 1)]
    off = np.zeros(len(lens), np.uint64)
    off[1:] = np.cumsum(lens[:-1])
    return lens, off


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", choices=["sstable4k", "mixed", "records", "records_verify", "one_tree"],
                    default="sstable4k",
                    help="sstable4k = BASELINE configs[1] (the metric); mixed = configs[2]; records = the "
                         "compaction form: 1 Mi serialized 4 KiB records in a Data table, values located "
                         "from the record headers and hashed in place; records_verify = the same plus every "
                         "record's Crc checked (nkv_tree_verify_records_dev)")
    ap.add_argument("--mixed-bytes", type=int, default=4 << 30, help="payload of the mixed config")
    ap.add_argument("--no-bucket", action="store_true", help="hash ragged values in input order (--bucket 0)")
    ap.add_argument("--bucket", type=int, default=-1, help="NKV_OPT_BUCKET override (0 input order, 1 sorted, 2 auto)")
    ap.add_argument("--leaf-load", type=int, default=0, help="NKV_OPT_LEAF_LOAD override (0 = library default)")
    ap.add_argument("--deep", type=int, default=-1,
                    help="NKV_OPT_DEEP_PREFETCH override for ragged batches (-1 = library default)")
    ap.add_argument("--queue-split", type=int, default=-1, help="NKV_OPT_QUEUE_SPLIT override")
    ap.add_argument("--queue-waves", type=int, default=0, help="NKV_OPT_QUEUE_WAVES override")
    ap.add_argument("--queue-ring", type=int, default=0, help="NKV_OPT_QUEUE_RING override (2, 3, 4)")
    ap.add_argument("--records-fused", type=int, default=-1, help="NKV_OPT_RECORDS_FUSED override (0, 1)")
    ap.add_argument("--leaves", type=int, default=1 << 20)
    ap.add_argument("--key-bytes", type=int, default=16, help="records configs: KeySize (the Value starts at +30+key)")
    ap.add_argument("--value-bytes", type=int, default=4096)
    ap.add_argument("--preroll-s", type=float, default=0.3,
                    help="untimed steps for at least this long before the warmup (clock settling)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-leaves", type=int, default=1 << 20)
    ap.add_argument("--verify", action="store_true", help="check the root against the C oracle")
    ap.add_argument("--dist", action="store_true",
                    help="join the RCCL group and all-gather the roots even at world size 1 (exercises the N > 1 path on one GPU)")
    ap.add_argument("--gather", choices=["batch", "step"], default="batch",
                    help="root all-gather with N > 1 (or --dist): one collective per timed loop (batch) or one "
                         "per table, pipelined behind the next table (step)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="do not record per-kernel HIP events inside the timed loop")
    return ap.parse_args()


def cpu_baseline(n_leaves: int, vlen: int) -> dict:
    """The oracle (C restatement of ds/merkletree, one thread, like the Go reference)."""
    import numpy as np
    from oracle import oracle_c as oc
    oc.build()
    data = oc.splitmix64_bytes(n_leaves * vlen, SEED)
    t0 = time.perf_counter()
    leaves = oc.leaf_hashes_strided(data, vlen, vlen, n_leaves, threads=1)
    nodes = oc.tree_from_digests(leaves)
    dt = time.perf_counter() - t0
    # SURVEY 8(d) variant 2: the same port with the leaves spread over the host
    # cores this process may use (the box caps a GPU job's share at 16)
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), len(os.sched_getaffinity(0))))
    t3 = time.perf_counter()
    leaves_mt = oc.leaf_hashes_strided(data, vlen, vlen, n_leaves, threads=threads)
    nodes_mt = oc.tree_from_digests(leaves_mt)
    dt3 = time.perf_counter() - t3
    assert nodes_mt[-1].tobytes() == nodes[-1].tobytes()
    # informational: OpenSSL SHA-1 (hashlib) on one core over a 256 MiB slice
    k = min(n_leaves, (256 << 20) // vlen)
    t1 = time.perf_counter()
    for i in range(k):
        hashlib.sha1(memoryview(data)[i * vlen:(i + 1) * vlen]).digest()
    dt2 = time.perf_counter() - t1
    del data
    return {
        "value": round(n_leaves * vlen / dt / 2**30, 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{n_leaves} x {vlen} B values (splitmix64 seed {SEED:#x}), leaf hash + full tree, "
                  f"oracle/merkle_oracle.c single thread, {dt:.2f} s",
        "root": nodes[-1].tobytes().hex(),
        "openssl_leaf_hash_1core_GiBps": round(k * vlen / dt2 / 2**30, 4),
        "all_cores": {"value": round(n_leaves * vlen / dt3 / 2**30, 4), "unit": "GiB/s", "cores": threads,
                      "sample": "the same sample, leaves over pthreads, tree on one thread"},
    }


def launcher_cmd(argv, n: int, port: int):
    """The one-node launch of N rank processes (one per GPU) for this bench."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def ensure_ranks(args, argv, run=None) -> "int | None":
    """`--gpus N` must match the process group.  Under a launcher WORLD_SIZE is
    set and must equal N; without one, N > 1 starts the N ranks as a child
    torch.distributed.run (before this process touches a GPU) and returns its
    exit code; None means: run the bench in this process."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
            return 2
        return None
    if args.gpus <= 1:
        return None
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return (run or subprocess.call)(launcher_cmd(argv, args.gpus, port))


class RootGather:
    """Per-step RCCL all-gather of the table roots, overlapped with the next
    step: step i builds into bufs[i % 2] and gathers that buffer's 20-byte root
    asynchronously into outs[i % 2]; begin() of step i + 2 waits for gather i
    before bufs[i % 2] is rewritten.  dist None: one rank, nothing to gather."""

    def __init__(self, nodes, roots, dist=None):
        self.dist = dist
        self.bufs = [nodes, nodes.new_empty(nodes.shape)] if dist else [nodes]
        self.outs = [roots, roots.new_empty(roots.shape)] if dist else [roots]
        self.pending = []  # (step index, async work)
        self.i = -1

    def begin(self):
        self.i += 1
        while self.pending and self.pending[0][0] <= self.i - 2:
            self.pending.pop(0)[1].wait()
        return self.bufs[self.i % len(self.bufs)]

    def end(self, nodes):
        if self.dist:
            work = self.dist.all_gather_into_tensor(self.outs[self.i % 2], nodes[-20:], async_op=True)
            self.pending.append((self.i, work))

    def drain(self):
        while self.pending:
            self.pending.pop(0)[1].wait()

    def last_roots(self):
        return self.outs[self.i % 2]


def preroll(step, drain, sync, seconds, dist=None, flag=None) -> int:
    """Untimed steps, in chunks of 8, until every rank has run them for
    `seconds`; returns the count, which is the same on every rank (the ranks
    agree after each chunk through a MIN all-reduce of flag(done))."""
    steps, t0 = 0, time.perf_counter()
    while True:
        for _ in range(8):
            step()
        steps += 8
        drain()
        sync()
        done = time.perf_counter() - t0 >= seconds
        if dist is not None:
            f = flag(1 if done else 0)
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            done = int(f.item()) == 1
        if done:
            return steps


class BatchedRootGather:
    """The roots of a whole run of tables in one collective: each step copies
    its 20-byte root (on the compute stream, behind the tree) into the next
    slot, and drain() all-gathers the filled slots at once (world x k x 20 B),
    so a timed loop of K tables issues one RCCL call instead of K (SURVEY.md
    section 8e: the gather follows the builds; fewer, larger collectives).
    Every gather still completes inside the timed region (drain before the
    closing barrier).  dist None: one rank, nothing to gather."""

    def __init__(self, nodes, world, dist=None, cap=256):
        self.dist, self.nodes, self.world, self.cap = dist, nodes, world, max(1, cap)
        self.slots = nodes.new_empty(self.cap * 20)
        self.out = nodes.new_empty(world * self.cap * 20)
        self.k = 0
        self.last = None

    def begin(self):
        return self.nodes

    def end(self, nodes):
        if self.dist:
            if self.k == self.cap:
                self.drain()
            self.slots[20 * self.k:20 * (self.k + 1)].copy_(nodes[-20:])
            self.k += 1

    def drain(self):
        if self.dist and self.k:
            out = self.out[:self.world * self.k * 20]
            self.dist.all_gather_into_tensor(out, self.slots[:self.k * 20])
            self.last = out.view(self.world, self.k, 20)[:, self.k - 1].reshape(-1)
            self.k = 0

    def last_roots(self):
        return self.last


def main():
    args = parse()
    if args.config in ("records", "records_verify") and args.value_bytes <= 30 + args.key_bytes:
        raise SystemExit("bench.py: --value-bytes (the record size) must exceed the 30-B header + --key-bytes")
    rc = ensure_ranks(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_dist = world > 1 or args.dist
    if use_dist:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    from nakevaleng_amd import build as nb
    if rank == 0 or not os.path.exists(nb.SO):
        nb.build()
    if use_dist:
        dist.barrier()
    from nakevaleng_amd import _lib

    L = _lib.lib()
    dev = torch.cuda.current_device()
    ctx = _lib.Context(dev)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream.cuda_stream)

    if args.leaf_load:
        ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, args.leaf_load)
    if args.deep >= 0:
        ctx.set_option(_lib.NKV_OPT_DEEP_PREFETCH, args.deep)
    if args.queue_split >= 0:
        ctx.set_option(_lib.NKV_OPT_QUEUE_SPLIT, args.queue_split)
    if args.queue_waves:
        ctx.set_option(_lib.NKV_OPT_QUEUE_WAVES, args.queue_waves)
    if args.queue_ring:
        ctx.set_option(_lib.NKV_OPT_QUEUE_RING, args.queue_ring)
    if args.records_fused >= 0:
        ctx.set_option(_lib.NKV_OPT_RECORDS_FUSED, args.records_fused)
    if args.no_bucket:
        ctx.set_option(_lib.NKV_OPT_BUCKET, 0)
    elif args.bucket >= 0:
        ctx.set_option(_lib.NKV_OPT_BUCKET, args.bucket)
    roots = torch.empty(world * 20, dtype=torch.uint8, device="cuda")
    mixed = args.config == "mixed"
    one_tree = args.config == "one_tree"
    records = args.config in ("records", "records_verify")
    verify_crc = args.config == "records_verify"
    if records:
        import numpy as np
        n, rb = args.leaves, args.value_bytes
        ks = args.key_bytes
        vlen = rb - 30 - ks  # record.go:191-199 header 30 B, 16-B key, the rest is the Value
        stream_len = n * rb
        data = torch.empty(stream_len, dtype=torch.uint8, device="cuda")
        _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, data.data_ptr(), stream_len, SEED + rank))
        v = data.view(n, rb)
        v[:, 14:22] = torch.from_numpy(np.frombuffer(np.uint64(ks).tobytes(), np.uint8).copy()).cuda()
        v[:, 22:30] = torch.from_numpy(np.frombuffer(np.uint64(vlen).tobytes(), np.uint8).copy()).cuda()
        d_roff = torch.arange(n, dtype=torch.int64, device="cuda") * rb
        d_err = torch.zeros(1, dtype=torch.int32, device="cuda")
        nbytes = n * vlen  # payload: the hashed Values
        nodes = torch.empty(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
        if verify_crc:  # store each record's right checksum (computed on the device once)
            d_crc = torch.empty(n, dtype=torch.int32, device="cuda")
            d_stats = torch.zeros(3, dtype=torch.int64, device="cuda")
            _lib.check(L.nkv_record_crc_dev(ctx.h, data.data_ptr(), stream_len, d_roff.data_ptr(), n,
                                            d_crc.data_ptr(), d_stats.data_ptr()))
            v[:, 0:4] = d_crc.view(torch.uint8).view(n, 4)

            def tree():
                _lib.check(L.nkv_tree_verify_records_dev(ctx.h, data.data_ptr(), stream_len, d_roff.data_ptr(), n,
                                                         nodes.data_ptr(), None, d_stats.data_ptr()))
        else:
            def tree():
                _lib.check(L.nkv_tree_from_records_dev(ctx.h, data.data_ptr(), stream_len, d_roff.data_ptr(), n,
                                                       nodes.data_ptr(), d_err.data_ptr()))
    elif not mixed:
        n, vlen = args.leaves, args.value_bytes
        nbytes = n * vlen
        data = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, data.data_ptr(), nbytes, SEED + rank))
        nodes = torch.empty(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")

        def tree():
            _lib.check(L.nkv_tree_from_strided_dev(ctx.h, data.data_ptr(), vlen, vlen, n, nodes.data_ptr()))

        if one_tree:  # one tree over every rank's leaves (rank r holds leaves [r n, (r+1) n))
            from nakevaleng_amd import sharded_tree
            if n & (n - 1):
                raise SystemExit("--config one_tree needs a power-of-two --leaves (ranges aligned to 2^k)")
            ops = sharded_tree.DeviceOps(dev, ctx=ctx)

            def tree():
                nodes[-20:] = sharded_tree.sharded_root((data, vlen, vlen), n * world, ops=ops, host_root=False)
    else:
        import numpy as np
        lens_h, off_h = mixed_lengths(args.mixed_bytes, SEED_MIXED + rank)
        n, vlen = len(lens_h), None
        nbytes = int(lens_h.sum())
        data = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, data.data_ptr(), nbytes, SEED_MIXED + rank))
        d_off = torch.from_numpy(off_h.view(np.int64)).cuda()
        d_len = torch.from_numpy(lens_h.view(np.int64)).cuda()
        nodes = torch.empty(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")

        def tree():
            _lib.check(L.nkv_tree_from_values_dev(ctx.h, data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                                  n, nodes.data_ptr()))

    # C1, the root gather.  Default (--gather batch):
    # every table's root is kept and all of them are all-gathered in one call
    # at the end of the loop (BatchedRootGather).  --gather step: one gather
    # per table, overlapped with the next: step i builds into bufs[i % 2] and
    # all-gathers that buffer's root asynchronously on RCCL's stream while
    # step i + 1 hashes into the other buffer; step i + 2 first waits for
    # gather i before it rewrites bufs[i % 2].  Either way every gather
    # completes inside the timed region (the final synchronize waits for it).
    gdist = dist if (use_dist and not one_tree) else None
    if args.gather == "step":
        rg = RootGather(nodes, roots, gdist)
    else:
        rg = BatchedRootGather(nodes, world, gdist, cap=max(args.steps, args.warmup, 8))

    def step():
        nonlocal nodes
        nodes = rg.begin()
        tree()
        rg.end(nodes)

    drain = rg.drain

    # Untimed pre-roll, independent of --warmup: the shader clock settles only
    # after ~30 ms of back-to-back launches ("The clock"),
    # so run steps for at least PREROLL_S before the caller's warmup steps.
    torch.cuda.synchronize()
    # Steps go in chunks of 8 and, with several ranks, every rank runs the same
    # number of them (the gathers and the one_tree collectives are matched by
    # order, so a rank that ran one step more would wait forever): after each
    # chunk the ranks agree to stop only once every one of them has pre-rolled
    # for PREROLL_S.
    preroll_steps = preroll(step, drain, torch.cuda.synchronize, args.preroll_s, dist if use_dist else None,
                            lambda v: torch.tensor([v], dtype=torch.int32, device="cuda"))
    if records and (int(d_err.item()) != 0 or (verify_crc and int(d_stats[2].item()) != 0)):
        # a malformed synthetic stream would time empty hashes
        raise SystemExit("bench.py: the record stream failed the header checks")
    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.set_timing(not args.no_kernel_timing)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    calls, leaf_ms_tot, reduce_ms_tot = ctx.timing_summary()
    ctx.set_timing(False)
    if calls == 0:  # kernel split measured in a separate loop of the same steps
        ctx.set_timing(True)
        for _ in range(args.steps):
            step()
        drain()
        calls, leaf_ms_tot, reduce_ms_tot = ctx.timing_summary()
        ctx.set_timing(False)
    if use_dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    root = nodes[-20:].cpu().numpy().tobytes().hex()
    gathered_ok = None
    if rg.dist:  # every rank's slot of the last gather holds that rank's root
        got = rg.last_roots().cpu().numpy().reshape(world, 20)
        gathered_ok = got[rank].tobytes().hex() == root
    leaf_ms = leaf_ms_tot / max(calls, 1)
    reduce_ms = reduce_ms_tot / max(calls, 1)

    # K3 (Serialize image) timed separately: not part of the metric
    img = torch.empty(L.nkv_bfs_size(n), dtype=torch.uint8, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    _lib.check(L.nkv_bfs_image_dev(ctx.h, nodes.data_ptr(), n, img.data_ptr()))
    e0.record(stream)
    for _ in range(5):
        _lib.check(L.nkv_bfs_image_dev(ctx.h, nodes.data_ptr(), n, img.data_ptr()))
    e1.record(stream)
    torch.cuda.synchronize()
    bfs_ms = e0.elapsed_time(e1) / 5

    verified = None
    if args.verify and rank == 0:
        import numpy as np
        from oracle import oracle_c as oc
        if mixed:
            host = oc.splitmix64_bytes(nbytes, SEED_MIXED)
            want = oc.tree_from_digests(oc.leaf_hashes(host, off_h, lens_h, threads=16))
        elif records:
            host = data.cpu().numpy()
            voff = np.arange(n, dtype=np.uint64) * rb + 30 + ks
            want = oc.tree_from_digests(oc.leaf_hashes(host, voff, np.full(n, vlen, np.uint64), threads=16))
            assert int(d_err.item()) == 0
            if verify_crc:
                assert d_stats.cpu().tolist() == [0, -1, 0], d_stats.cpu().tolist()
        else:
            host = np.concatenate([oc.splitmix64_bytes(nbytes, SEED + r) for r in range(world if one_tree else 1)])
            want = oc.tree_from_digests(oc.leaf_hashes_strided(host, vlen, vlen, len(host) // vlen, threads=16))
        verified = want[-1].tobytes().hex() == root
        del host

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "sstable4k":
        cpu = cpu_baseline(min(args.cpu_sample_leaves, n), vlen)

    if rank == 0:
        total_bytes = nbytes * world * args.steps
        value = total_bytes / elapsed / 2**30
        achieved = nbytes / (leaf_ms * 1e-3) / 1e9  # algorithmic payload bytes per K1 launch
        valu_ceiling = SHA1_VALU_CEILING_GBS * (VERIFY_VALU_RATIO if verify_crc else 1.0)
        traffic, traffic_bounds = None, None
        # PMC-measured HBM bytes of this config's leaf kernel (separate rocprofv3
        # passes: tools/pmc_sizes.sh for cfg2, tools/pmc_config.sh for the others)
        # cfg2: the default 128-byte register runs (LOAD 4) or the LDS-DMA stage (--leaf-load 1)
        cfg2_pmc = {0: "pmc_traffic_cfg2_runs.json", 4: "pmc_traffic_cfg2_runs.json",
                    1: "pmc_traffic.json"}.get(args.leaf_load)
        pmc_name = {"sstable4k": cfg2_pmc, "records": "pmc_traffic_records.json",
                    "mixed": "pmc_traffic_mixed.json", "records_verify": "pmc_traffic_records_verify.json"}.get(args.config)
        pmc_path = os.path.join(ROOT, "profiles", pmc_name) if pmc_name else None
        if pmc_path and os.path.exists(pmc_path):
            with open(pmc_path) as f:
                pmc = json.load(f)
            same = pmc.get("leaves") == n and (pmc.get("value_bytes") in (None, vlen)) and \
                pmc.get("algorithmic_bytes_per_launch") in (None, nbytes)
            if same:
                traffic = pmc.get("hbm_bytes_per_launch")
                traffic_bounds = pmc.get("hbm_read_bytes_bounds_per_launch")
        out = {
            "metric": "GiB/s Merkle leaf-hash + tree-reduce over device-resident record blocks",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "preroll_steps": preroll_steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": f"synthetic: splitmix64 bytes (seed {SEED_MIXED if mixed else SEED:#x} + rank) generated in HBM",
            "config": {
                "workload": ("BASELINE configs[2]: mixed 64 B - 64 KiB log-uniform values packed back to back, "
                             + ("input order" if args.no_bucket else "length-bucketed")) if mixed else
                            (f"compaction form: {n} serialized {rb}-B records ({ks}-B key, {vlen}-B value) in a "
                             "Data table in HBM; values located from the headers and hashed in place, full tree"
                             + ("; every record's Crc (Key ++ Value) checked in the same pass" if verify_crc else ""))
                            if records else
                            (f"one tree over {world} GPU(s): {n} x {vlen} B values per rank, each rank builds the "
                             "levels of its aligned leaf range, sub-roots all-gathered, top levels on every rank")
                            if one_tree else
                            ("BASELINE configs[1]: single SSTable flush, 1 Mi x 4 KiB values, "
                             if (n, vlen) == (1 << 20, 4096) else
                             "BASELINE configs[4] per-GPU table (8 Mi x 4 KiB values), "
                             if (n, vlen) == (8 << 20, 4096) else
                             f"single SSTable flush, {n} x {vlen} B values, ")
                            + "leaf SHA-1 + full tree reduce (one table per GPU; roots all-gathered over RCCL when N>1)",
                "leaves_per_gpu": n,
                "value_bytes": vlen if not mixed else "64..65536 (mean %.0f)" % (nbytes / n),
                "parallelism": (f"1 tree split over {world} ranks" + (" + RCCL all_gather of sub-roots" if world > 1 else ""))
                               if one_tree else
                               f"{world} independent tables" + ((" + RCCL all_gather of roots, "
                                                                 + ("one call per timed loop" if args.gather == "batch"
                                                                    else "one per table")) if world > 1 else ""),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": ("leaf phase: length sort + ragged leaf SHA-1 (%s)" % LEAF_KERNEL.get(args.deep, "default"))
                          if mixed else
                          ("leaf phase: k_leaf_verify (header parse + record CRC + leaf SHA-1 from whole 128-byte lines in registers, input order)"
                           if verify_crc else
                           ("leaf phase: k_locate + k_leaf<offsets, aligned-segment stage> (input order)"
                            if args.records_fused == 0 else
                            "leaf phase: k_leaf_records (header parse + whole 128-byte lines into registers, input order)")) if records else
                          ("k_leaf<strided, LDS-DMA stage> (leaf SHA-1, level 0)" if args.leaf_load == 1 else
                           "k_leaf<strided, 128-byte register runs> (leaf SHA-1, level 0)" if args.leaf_load in (0, 4)
                           else f"k_leaf<strided, load path {args.leaf_load}> (leaf SHA-1, level 0)"),
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                # the whole step (leaf + tree + launches, N ranks): payload per
                # GPU / ms_per_step / peak
                "step_frac": round(nbytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_bounds": traffic_bounds,  # RDREQ x 64 .. x 128 B (profiles/pmc_traffic.json)
                "valu_ceiling": round(valu_ceiling, 1),
                "valu_frac": round(achieved / valu_ceiling, 4),
            },
            "kernel_ms": {"leaf": round(leaf_ms, 4), "tree_reduce": round(reduce_ms, 4),
                          "bfs_image": round(bfs_ms, 4)},
            "root": root,
            "cpu_baseline": cpu,
        }
        if verified is not None:
            out["verified_vs_oracle"] = verified
        if gathered_ok is not None:
            out["root_gather_ok"] = gathered_ok
        print(json.dumps(out), flush=True)
    ctx.close()
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
