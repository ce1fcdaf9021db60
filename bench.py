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
import ctypes
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md (chip table)
PCIE_SPEC_GBS = 63.0  # host link, PCIe Gen5 x16 (same table)
# The VALU-issue ceiling of the leaf kernel at the shader clock its waves
# actually ran at in the timed loop (the clock probe, sclk_mhz): every SIMD
# issuing one VALU instruction per VALU_CYCLES cycles (the half-rate ops
# v_add3 / v_alignbit / v_perm set the cadence, profiles/r01_valu_rate.txt),
# VALU_PER_WAVE_BLOCK instructions per wave per 64-byte block (PMC
# SQ_INSTS_VALU per launch / wave-blocks of payload: leaf from the register-run
# kernel with its padding block's schedule on the scalar unit,
# profiles/r04_pad_valu_pmc.json (39,689 per wave / 64; 623.0 before); records (k_leaf_records) and verify
# (k_leaf_verify) per 64 bytes of Value, profiles/r03_records_pmc.json), 4096 bytes per
# wave-block (64 lanes x 64 B):
#   ceiling = SIMDS x f / (VALU_PER_WAVE_BLOCK x VALU_CYCLES) x 4096 B.
SIMDS = 1024  # 256 CUs x 4
VALU_CYCLES = 4.0
VALU_PER_WAVE_BLOCK = {"leaf": 620.1, "records": 631.7, "verify": 737.9}
SHA1_VALU_CEILING_GBS = 4100.0  # fallback without a clock reading: tools/sha1_rate.hip at 2.37 GHz
# The mixed config's floor is its longest value: one lane's chain of dependent
# compressions, on a wave that issues one instruction every ~4.65 cycles when
# it runs alone on its SIMD -- 2,852 shader cycles per block for SHA-1 from
# registers (tools/lone_wave.hip, profiles/r02_lone_wave_ilp.txt).
LONE_WAVE_CYCLES_PER_BLOCK = 2852.0
SEED = 0x6E616B65
SEED_MIXED = 0x6E616B66




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


GOLDEN = os.path.join(ROOT, "tests", "golden", "bench_roots.json")
_golden = None


def golden():
    """The committed expected roots of the bench's synthetic tables
    (tests/golden/make_bench_roots.py, the C oracle in the build container)."""
    global _golden
    if _golden is None:
        try:
            with open(GOLDEN) as f:
                _golden = json.load(f)
        except OSError:  # no fixture: only --verify checks (verified_vs_oracle null)
            _golden = {"sstable4k": {"leaves": -1, "value_bytes": -1, "roots": {}},
                       "one_tree": {"leaves_per_rank": -1, "value_bytes": -1, "roots": {}}}
    return _golden


def expected_roots(config, leaves, value_bytes, rank, T, key_bytes=16, mixed_bytes=4 << 30):
    """Rank `rank`'s T table roots (hex) from the committed fixture, or None when
    the fixture does not cover this shape (then only --verify checks).
    value_bytes is the record size for the records configs."""
    g = golden()
    if config in ("records", "records_verify"):
        r = g.get("records")
        ok = r and T == 1 and (leaves, value_bytes, key_bytes) == (r["leaves"], r["record_bytes"], r["key_bytes"])
        return [r["roots"][str(rank)]] if ok and str(rank) in r["roots"] else None
    if config == "mixed":
        m = g.get("mixed")
        ok = m and T == 1 and mixed_bytes == m["payload_bytes"]
        return [m["roots"][str(rank)]] if ok and str(rank) in m["roots"] else None
    if config not in ("sstable4k", "runs4"):
        return None
    for key in ("sstable4k", "small", "config4"):  # configs[1]; configs[0]'s size (CPU tests); configs[4] per GPU
        g = golden().get(key)
        if g is None:
            continue
        if (leaves, value_bytes) == (g["leaves"], g["value_bytes"]):
            roots = g["roots"].get(str(rank))
            roots = [roots] if isinstance(roots, str) else roots
            return roots[:T] if roots is not None and T <= len(roots) else None
    return None


def expected_one_tree(leaves, value_bytes, world):
    """The root of one tree over ranks 0..world-1's leaves, or None."""
    g = golden()["one_tree"]
    if (leaves, value_bytes) != (g["leaves_per_rank"], g["value_bytes"]):
        return None
    return g["roots"].get(str(world))


def verdict(codes):
    """Per-rank check codes (1 ok, 0 wrong, -1 not covered) -> verified_vs_oracle:
    False if any rank is wrong, True if every rank checked out, else None."""
    if any(c == 0 for c in codes):
        return False
    return True if codes and all(c == 1 for c in codes) else None


def rank_codes(dist, world, rank, code, device):
    """Every rank's check code on every rank (one SUM all-reduce of a one-hot
    vector; `device` is where the backend wants its tensors)."""
    import torch
    flags = torch.zeros(world, dtype=torch.int32, device=device)
    flags[rank] = int(code) + 2  # 1 (not covered), 2 (wrong), 3 (ok): never 0
    if dist is not None and world > 1:
        dist.all_reduce(flags)
    return [int(v) - 2 for v in flags.cpu().tolist()]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", choices=["sstable4k", "mixed", "records", "records_verify", "one_tree", "runs4",
                                         "api_flush", "small_flush"],
                    default="sstable4k",
                    help="sstable4k = BASELINE configs[1] (the metric); mixed = configs[2]; records = the "
                         "compaction form: 1 Mi serialized 4 KiB records in a Data table, values located "
                         "from the record headers and hashed in place; records_verify = the same plus every "
                         "record's Crc checked (nkv_tree_verify_records_dev); runs4 = configs[3] per GPU: "
                         "lsm_run_max = 4 tables of 1 Mi x 4 KiB per step (sstable4k with --tables 4); "
                         "api_flush = the host-inclusive flush through the C++ Go-API mirror: NewLeaf x n "
                         "from host memory, New, Root, Serialize to a fresh file (tools/api_flush.cpp); "
                         "small_flush = microseconds per flush at the reference's default sizes (10 values "
                         "<= 200 B) up to configs[0], GPU paths beside one host core (tools/small_flush.cpp)")
    ap.add_argument("--small-reps", type=int, default=300, help="small_flush: flushes per shape and mode")
    ap.add_argument("--small-modes", default="1,3,3h,2,0",
                    help="small_flush: NKV_OPT_SMALL_PATH modes to time (1 one launch over pinned memory, 3 the "
                         "resident service, 3h the same with its requests in host memory, 2 one launch through HBM, "
                         "0 the grid path)")
    ap.add_argument("--api-cycles", type=int, default=4, help="api_flush: flushes per mode (the first allocates "
                                                              "the pinned arena)")
    ap.add_argument("--tables", type=int, default=0,
                    help="tables per step and GPU (0: 4 for runs4, else 1); more than one goes through "
                         "nkv_trees_dev, spread over --table-lanes streams")
    ap.add_argument("--table-lanes", type=int, default=0,
                    help="NKV_OPT_TABLE_LANES (0 = library default 2; 1 = the tables one after another on one stream)")
    ap.add_argument("--backend", choices=["torch", "capi"], default="torch",
                    help="torch: one process per GPU (torch.distributed over RCCL); capi: one process over all "
                         "--gpus through the library's group (nkv_group_*: a context per GPU, ncclCommInitAll, "
                         "the roots all-gathered by the library)")
    ap.add_argument("--no-clock", action="store_true", help="no shader-clock probe in the timed loop")
    ap.add_argument("--mixed-bytes", type=int, default=4 << 30, help="payload of the mixed config")
    ap.add_argument("--no-bucket", action="store_true", help="hash ragged values in input order (--bucket 0)")
    ap.add_argument("--bucket", type=int, default=-1, help="NKV_OPT_BUCKET override (0 input order, 1 sorted, 2 auto)")
    ap.add_argument("--side-gate", type=int, default=-1,
                    help="NKV_OPT_SIDE_GATE override (1 = library default: the gated input-order kernel on a second "
                         "stream; 0 = on the context's stream)")
    ap.add_argument("--leaf-load", type=int, default=0,
                    help="NKV_OPT_LEAF_LOAD override (0 = library default 4: 128-byte register runs for aligned "
                         "values; 11: the staged paths for every value)")
    ap.add_argument("--queue-split", type=int, default=-1, help="NKV_OPT_QUEUE_SPLIT override")
    ap.add_argument("--queue-waves", type=int, default=0, help="NKV_OPT_QUEUE_WAVES override (1..3)")
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
    ap.add_argument("--timing-every", type=int, default=1,
                    help="record the kernel-timing events on every k-th step of the timed loop only "
                         "(NKV_OPT_TIMING_EVERY; each record is a packet between two kernels)")
    ap.add_argument("--no-capi", action="store_true",
                    help="no capi_group / capi_one_tree sub-records (by default rank 0 runs the one-process C-ABI "
                         "group over the same N GPUs in a fresh child process once the ranks are done)")
    ap.add_argument("--capi-timeout", type=int, default=150,
                    help="seconds per C-ABI group child (a healthy 8-GPU child takes well under a minute; a hung "
                         "one must not cost the run its line)")
    ap.add_argument("--no-subconfigs", action="store_true",
                    help="no config2_mixed / config1_records sub-records (by default the N = 1 configs[1] line "
                         "runs both in fresh children, each with its own roofline and CPU baseline)")
    ap.add_argument("--child-budget-s", type=int, default=360,
                    help="seconds after the ranks finish within which the sub-config children must start")
    return ap.parse_args(argv)


_T0 = time.perf_counter()


def progress(msg: str) -> None:
    """One progress line on stderr (a long run shows it is alive)."""
    print(f"bench.py [{time.perf_counter() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def host_threads() -> int:
    """Host threads this process may use: its affinity set, capped by
    OMP_NUM_THREADS (the GPU box gives a one-GPU job 16 of its cores)."""
    return max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), len(os.sched_getaffinity(0))))


def cpu_model() -> str:
    """The host CPU's model name (/proc/cpuinfo, what lscpu prints)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_sample(args, rank: int = 0) -> dict:
    """The host-memory form of the workload the GPU line measured (rank `rank`'s
    first table, same seeds and layout as build_tables), bounded to
    --cpu-sample-leaves values (the mixed batch whole: its leaves are ragged,
    so a prefix would be a different workload).  Keys: data, n, nbytes and
    either (stride, L) or (off, lens); `text` says what it is."""
    import numpy as np
    from oracle import oracle_c as oc
    cfg = args.config
    if cfg == "mixed":
        lens, off = mixed_lengths(args.mixed_bytes, SEED_MIXED + rank)
        nbytes = int(lens.sum())
        return {"data": oc.splitmix64_bytes(nbytes, SEED_MIXED + rank), "off": off, "lens": lens, "n": len(lens),
                "nbytes": nbytes, "text": f"BASELINE configs[2]'s batch: {len(lens)} values of 64 B - 64 KiB "
                                          f"({nbytes} B, splitmix64 seed {SEED_MIXED + rank:#x})"}
    n = min(args.cpu_sample_leaves, args.leaves)
    if cfg == "records_verify":
        # the Data table build_tables writes (KeySize, ValueSize in every
        # header, each record's right Crc at +0: record.go:191-199, :51), which
        # the host reads back as merge does (record.go:163-169, lsmtree.go:210-211)
        rb, ks = args.value_bytes, args.key_bytes
        vlen = rb - 30 - ks
        data = oc.splitmix64_bytes(n * rb, SEED + rank)
        v = data.reshape(n, rb)
        v[:, 14:22] = np.frombuffer(np.uint64(ks).tobytes(), np.uint8)
        v[:, 22:30] = np.frombuffer(np.uint64(vlen).tobytes(), np.uint8)
        rec_off = np.arange(n, dtype=np.uint64) * rb
        oc.seal_records(data, rec_off, host_threads())
        return {"data": data, "rec_off": rec_off, "n": n, "nbytes": n * vlen,
                "text": f"{n} serialized {rb}-B records ({ks}-B key, {vlen}-B value; splitmix64 seed "
                        f"{SEED + rank:#x}), each record's Crc over Key ++ Value checked and its Value hashed"}
    if cfg == "records":
        rb, ks = args.value_bytes, args.key_bytes
        vlen = rb - 30 - ks
        # the Values sit at rec + 30 + KeySize (record.go:191-199); the header
        # words build_tables writes do not overlap them
        off = np.arange(n, dtype=np.uint64) * rb + 30 + ks
        return {"data": oc.splitmix64_bytes(n * rb, SEED + rank), "off": off, "lens": np.full(n, vlen, np.uint64),
                "n": n, "nbytes": n * vlen,
                "text": f"{n} serialized {rb}-B records ({ks}-B key, {vlen}-B value; splitmix64 seed "
                        f"{SEED + rank:#x}), the values hashed in place"}
    vlen = args.value_bytes
    return {"data": oc.splitmix64_bytes(n * vlen, SEED + rank), "stride": vlen, "L": vlen, "n": n,
            "nbytes": n * vlen, "text": f"{n} x {vlen} B values (splitmix64 seed {SEED + rank:#x})"}


# The four CPU variants of SURVEY.md 8(d): the portable C restatement
# (oracle/merkle_oracle.c, the reference's statements) and OpenSSL's SHA-1
# (oracle/merkle_openssl.c, libcrypto: SHA-NI where the host has it, the
# stand-in for Go's assembly crypto/sha1), each on one thread (the reference
# is single-threaded) and on every host thread this process may use.
CPU_VARIANTS = (("port_1core", "port", False), ("openssl_1core", "openssl", False),
                ("port_all_cores", "port", True), ("all_cores_openssl", "openssl", True))
# records_verify's variants add the record check: the port with a
# slicing-by-8 CRC-32, the OpenSSL variant with a PCLMULQDQ one (what Go's
# hash/crc32 runs on amd64), fused per record with the leaf SHA-1
# (oracle/record_crc_oracle.c nkvo_verify_records)
CPU_IMPL_TEXT = {"port": "the portable C restatement (oracle/merkle_oracle.c)",
                 "openssl": "the C restatement's tree over OpenSSL's SHA-1 (libcrypto, SHA-NI; "
                            "oracle/merkle_openssl.c)"}


def cpu_baseline(args, rank: int = 0) -> dict:
    """Leaf hash + full tree of cpu_sample() on the host, every variant of
    CPU_VARIANTS timed on the same bytes.  `value` is the STRONGEST figure
    (`best` names it), so every GPU/CPU ratio is against the best CPU; the
    one-core port is the reference-shaped figure.  Every variant's root must
    agree."""
    from oracle import oracle_c as oc
    oc.build()
    s = cpu_sample(args, rank)
    data, n, nbytes = s["data"], s["n"], s["nbytes"]
    threads = host_threads()
    out, roots = {}, set()
    for name, impl, allc in CPU_VARIANTS:
        t = threads if allc else 1
        t0 = time.perf_counter()
        if "rec_off" in s:  # records_verify: Crc check + leaf hash in one pass per record, then the tree
            leaves, bad = oc.verify_records(data, s["rec_off"], threads=t, openssl=impl == "openssl")
            if bad:
                raise SystemExit(f"bench.py: {bad} records failed the CPU Crc check")
            nodes = (oc.ossl_tree_from_digests(leaves, threads=t) if impl == "openssl"
                     else oc.tree_from_digests(leaves, threads=t))
        elif impl == "port":
            leaves = (oc.leaf_hashes_strided(data, s["stride"], s["L"], n, threads=t) if "stride" in s
                      else oc.leaf_hashes(data, s["off"], s["lens"], threads=t))
            nodes = oc.tree_from_digests(leaves, threads=t)
        else:
            leaves = (oc.ossl_leaf_hashes_strided(data, s["stride"], s["L"], n, threads=t) if "stride" in s
                      else oc.ossl_leaf_hashes(data, s["off"], s["lens"], threads=t))
            nodes = oc.ossl_tree_from_digests(leaves, threads=t)
        dt = time.perf_counter() - t0
        roots.add(nodes[-1].tobytes().hex())
        out[name] = {"value": round(nbytes / dt / 2**30, 4), "cores": t, "seconds": round(dt, 3)}
        progress(f"cpu_baseline {args.config} {name}: {out[name]['value']} GiB/s")
        del leaves, nodes
    if len(roots) != 1:
        raise SystemExit(f"bench.py: the CPU variants disagree on the root ({sorted(roots)})")
    best = max(out, key=lambda k: out[k]["value"])
    impl = dict((v[0], v[1]) for v in CPU_VARIANTS)[best]
    return {
        "value": out[best]["value"],
        "unit": "GiB/s",
        "cores": out[best]["cores"],
        # every variant is a CPU restatement timed on this host (the contract's
        # "port"; the Go reference cannot run here); `impl` names whose SHA-1
        # the strongest one, which `value` reports, runs
        "kind": "port",
        "impl": impl,
        "impl_text": CPU_IMPL_TEXT[impl] + (f" on {out[best]['cores']} threads" if out[best]["cores"] > 1
                                            else " on one thread"),
        "best": best,
        "sample": s["text"] + ", leaf hash + full tree",
        "cpu_model": cpu_model(),
        "host_threads": threads,
        "root": roots.pop(),
        **out,
    }


def vs_cpu(value, cpu) -> dict:
    """GPU/CPU ratios of a line: against the strongest CPU figure and the
    reference-shaped one (one core, portable SHA-1)."""
    if not cpu or not value:
        return {}
    return {"vs_cpu_best": round(value / cpu["value"], 2),
            "vs_cpu_port_1core": round(value / cpu["port_1core"]["value"], 2)}


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
    its tables' 20-byte roots (on the compute stream, behind the trees) into the
    next slots, and drain() all-gathers the filled slots at once (world x k x 20
    B), so a timed loop of K steps issues one RCCL call instead of K (SURVEY.md
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

    def end(self, nodes, more=()):
        """Queue the roots of this step's tables (nodes first, then `more`)."""
        if self.dist:
            group = (nodes,) + tuple(more)
            if self.k + len(group) > self.cap:
                self.drain()
            self.first = self.k  # slot of this step's first table
            for nb in group:
                self.slots[20 * self.k:20 * (self.k + 1)].copy_(nb[-20:])
                self.k += 1

    def drain(self):
        if self.dist and self.k:
            out = self.out[:self.world * self.k * 20]
            self.dist.all_gather_into_tensor(out, self.slots[:self.k * 20])
            # every rank's root of the latest step's first table
            self.last = out.view(self.world, self.k, 20)[:, self.first].reshape(-1)
            self.k = 0

    def last_roots(self):
        return self.last


TABLE_SEED_STEP = 7919  # table t of a step uses seed + rank + t * TABLE_SEED_STEP (t = 0: the single-table seeds)


def build_tables(args, torch, _lib, L, ctx, rank, T, device="cuda"):
    """T independent tables of the config's shape, resident in HBM on `device`.
    Each is a dict: nodes (device tensor), table (NkvTable for nkv_trees_dev),
    single() (the single-table entry on ctx), want() (the oracle root, host),
    plus its buffers."""
    import numpy as np
    tabs = []
    for t in range(T):
        seed_t = t * TABLE_SEED_STEP
        tab = {}
        if args.config in ("records", "records_verify"):
            n, rb, ks = args.leaves, args.value_bytes, args.key_bytes
            vlen = rb - 30 - ks  # record.go:191-199: 30-B header, the key, the rest is the Value
            stream_len = n * rb
            data = torch.empty(stream_len, dtype=torch.uint8, device=device)
            _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, data.data_ptr(), stream_len, SEED + rank + seed_t))
            v = data.view(n, rb)
            v[:, 14:22] = torch.from_numpy(np.frombuffer(np.uint64(ks).tobytes(), np.uint8).copy()).to(device)
            v[:, 22:30] = torch.from_numpy(np.frombuffer(np.uint64(vlen).tobytes(), np.uint8).copy()).to(device)
            d_roff = torch.arange(n, dtype=torch.int64, device=device) * rb
            nodes = torch.empty(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device=device)
            d_err = torch.zeros(1, dtype=torch.int32, device=device)
            tab.update(data=data, d_roff=d_roff, nodes=nodes, d_err=d_err, n=n, vlen=vlen, nbytes=n * vlen,
                       stream_len=stream_len, rb=rb, ks=ks)
            if args.config == "records_verify":  # store each record's right checksum (computed on the device once)
                d_crc = torch.empty(n, dtype=torch.int32, device=device)
                d_stats = torch.zeros(3, dtype=torch.int64, device=device)
                _lib.check(L.nkv_record_crc_dev(ctx.h, data.data_ptr(), stream_len, d_roff.data_ptr(), n,
                                                d_crc.data_ptr(), d_stats.data_ptr()))
                v[:, 0:4] = d_crc.view(torch.uint8).view(n, 4)
                tab.update(d_stats=d_stats)
                tab["table"] = _lib.table(_lib.NKV_TABLE_VERIFY, nodes.data_ptr(), n, base=data.data_ptr(),
                                          base_len=stream_len, off=d_roff.data_ptr(), stats=d_stats.data_ptr())

                def single(tab=tab):
                    _lib.check(L.nkv_tree_verify_records_dev(ctx.h, tab["data"].data_ptr(), tab["stream_len"],
                                                             tab["d_roff"].data_ptr(), tab["n"],
                                                             tab["nodes"].data_ptr(), None,
                                                             tab["d_stats"].data_ptr()))
            else:
                tab["table"] = _lib.table(_lib.NKV_TABLE_RECORDS, nodes.data_ptr(), n, base=data.data_ptr(),
                                          base_len=stream_len, off=d_roff.data_ptr(), err=d_err.data_ptr())

                def single(tab=tab):
                    _lib.check(L.nkv_tree_from_records_dev(ctx.h, tab["data"].data_ptr(), tab["stream_len"],
                                                           tab["d_roff"].data_ptr(), tab["n"],
                                                           tab["nodes"].data_ptr(), tab["d_err"].data_ptr()))

            def want(tab=tab):
                from oracle import oracle_c as oc
                host = tab["data"].cpu().numpy()
                voff = np.arange(tab["n"], dtype=np.uint64) * tab["rb"] + 30 + tab["ks"]
                return oc.tree_from_digests(oc.leaf_hashes(host, voff, np.full(tab["n"], tab["vlen"], np.uint64),
                                                           threads=16))[-1].tobytes().hex()
        elif args.config == "mixed":
            lens_h, off_h = mixed_lengths(args.mixed_bytes, SEED_MIXED + rank + seed_t)
            n = len(lens_h)
            nbytes = int(lens_h.sum())
            data = torch.empty(nbytes, dtype=torch.uint8, device=device)
            _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, data.data_ptr(), nbytes, SEED_MIXED + rank + seed_t))
            d_off = torch.from_numpy(off_h.view(np.int64)).to(device)
            d_len = torch.from_numpy(lens_h.view(np.int64)).to(device)
            nodes = torch.empty(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device=device)
            tab.update(data=data, d_off=d_off, d_len=d_len, nodes=nodes, n=n, vlen=None, nbytes=nbytes,
                       lens_h=lens_h, off_h=off_h, seed=SEED_MIXED + rank + seed_t)
            tab["table"] = _lib.table(_lib.NKV_TABLE_VALUES, nodes.data_ptr(), n, base=data.data_ptr(),
                                      off=d_off.data_ptr(), lens=d_len.data_ptr())

            def single(tab=tab):
                _lib.check(L.nkv_tree_from_values_dev(ctx.h, tab["data"].data_ptr(), tab["d_off"].data_ptr(),
                                                      tab["d_len"].data_ptr(), tab["n"], tab["nodes"].data_ptr()))

            def want(tab=tab):
                from oracle import oracle_c as oc
                host = oc.splitmix64_bytes(tab["nbytes"], tab["seed"])
                return oc.tree_from_digests(oc.leaf_hashes(host, tab["off_h"], tab["lens_h"],
                                                           threads=16))[-1].tobytes().hex()
        else:  # sstable4k, runs4, one_tree: n values of vlen bytes at base + i vlen
            n, vlen = args.leaves, args.value_bytes
            nbytes = n * vlen
            data = torch.empty(nbytes, dtype=torch.uint8, device=device)
            _lib.check(L.nkv_fill_splitmix64_dev(ctx.h, data.data_ptr(), nbytes, SEED + rank + seed_t))
            nodes = torch.empty(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device=device)
            tab.update(data=data, nodes=nodes, n=n, vlen=vlen, nbytes=nbytes, seed=SEED + rank + seed_t)
            tab["table"] = _lib.table(_lib.NKV_TABLE_STRIDED, nodes.data_ptr(), n, base=data.data_ptr(),
                                      stride=vlen, length=vlen)

            def single(tab=tab):
                _lib.check(L.nkv_tree_from_strided_dev(ctx.h, tab["data"].data_ptr(), tab["vlen"], tab["vlen"],
                                                       tab["n"], tab["nodes"].data_ptr()))

            def want(tab=tab):
                from oracle import oracle_c as oc
                host = oc.splitmix64_bytes(tab["nbytes"], tab["seed"])
                return oc.tree_from_digests(oc.leaf_hashes_strided(host, tab["vlen"], tab["vlen"], tab["n"],
                                                                   threads=16))[-1].tobytes().hex()
        tab["single"], tab["want"] = single, want
        tabs.append(tab)
    return tabs


def valu_kind(config):
    """Which VALU_PER_WAVE_BLOCK entry a config's leaf kernel is priced at."""
    return {"records_verify": "verify", "records": "records"}.get(config, "leaf")


def valu_ceiling(mhz, kind):
    """GB/s the leaf kernel would reach issuing one VALU per VALU_CYCLES on every
    SIMD at the measured clock (None without a clock reading)."""
    if not mhz:
        return None
    per = VALU_PER_WAVE_BLOCK[kind]
    return SIMDS * mhz * 1e6 / (per * VALU_CYCLES) * 4096 / 1e9


def pmc_traffic(args, n, vlen, nbytes):
    """PMC-measured HBM bytes of this config's leaf kernel, per launch (separate
    rocprofv3 passes, tools/pmc_config.sh; cfg2 on round 4's build,
    tools/r04_pmc_cfg2.sh)."""
    cfg2_pmc = {0: "pmc_traffic_cfg2_r04.json", 4: "pmc_traffic_cfg2_r04.json",
                1: "pmc_traffic.json"}.get(args.leaf_load)
    pmc_name = {"sstable4k": cfg2_pmc, "runs4": cfg2_pmc, "records": "pmc_traffic_records.json",
                "mixed": "pmc_traffic_mixed.json", "records_verify": "pmc_traffic_records_verify.json"}.get(args.config)
    pmc_path = os.path.join(ROOT, "profiles", pmc_name) if pmc_name else None
    if pmc_path and os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        same = pmc.get("leaves") == n and (pmc.get("value_bytes") in (None, vlen)) and \
            pmc.get("algorithmic_bytes_per_launch") in (None, nbytes)
        if same:
            return pmc.get("hbm_bytes_per_launch"), pmc.get("hbm_read_bytes_bounds_per_launch")
    return None, None


def set_options(args, _lib, ctx):
    if args.leaf_load:
        ctx.set_option(_lib.NKV_OPT_LEAF_LOAD, args.leaf_load)
    if args.queue_split >= 0:
        ctx.set_option(_lib.NKV_OPT_QUEUE_SPLIT, args.queue_split)
    if args.queue_waves:
        ctx.set_option(_lib.NKV_OPT_QUEUE_WAVES, args.queue_waves)
    if args.records_fused >= 0:
        ctx.set_option(_lib.NKV_OPT_RECORDS_FUSED, args.records_fused)
    if args.no_bucket:
        ctx.set_option(_lib.NKV_OPT_BUCKET, 0)
    elif args.bucket >= 0:
        ctx.set_option(_lib.NKV_OPT_BUCKET, args.bucket)
    if args.table_lanes:
        ctx.set_option(_lib.NKV_OPT_TABLE_LANES, args.table_lanes)
    if args.side_gate >= 0:
        ctx.set_option(_lib.NKV_OPT_SIDE_GATE, args.side_gate)


def workload_text(args, n, vlen, nbytes, world, T, rb=None, ks=None):
    mixed = args.config == "mixed"
    records = args.config in ("records", "records_verify")
    if args.config == "runs4" or T > 1:
        head = (f"BASELINE configs[3] per GPU: lsm_run_max = {T} runs per compaction, " if args.config == "runs4"
                else f"{T} tables per step, ")
    else:
        head = ""
    if mixed:
        body = ("BASELINE configs[2]: mixed 64 B - 64 KiB log-uniform values packed back to back, "
                + ("input order" if args.no_bucket else "length-bucketed"))
    elif records:
        body = (f"compaction form: {n} serialized {rb}-B records ({ks}-B key, {vlen}-B value) in a "
                "Data table in HBM; values located from the headers and hashed in place, full tree"
                + ("; every record's Crc (Key ++ Value) checked in the same pass"
                   if args.config == "records_verify" else ""))
    elif args.config == "one_tree":
        body = (f"one tree over {world} GPU(s): {n} x {vlen} B values per rank, each rank builds the "
                "levels of its aligned leaf range, sub-roots all-gathered, every rank reduces the top levels")
    else:
        body = (("BASELINE configs[1]: single SSTable flush, 1 Mi x 4 KiB values, "
                 if (n, vlen) == (1 << 20, 4096) and T == 1 else
                 "BASELINE configs[4] per-GPU table (8 Mi x 4 KiB values), "
                 if (n, vlen) == (8 << 20, 4096) else
                 f"tables of {n} x {vlen} B values, ")
                + "leaf SHA-1 + full tree reduce (one table per GPU; roots all-gathered over RCCL when N>1)")
    return head + body


def kernel_text(args, T):
    mixed = args.config == "mixed"
    records = args.config in ("records", "records_verify")
    if mixed:
        k = "leaf phase: length sort + ragged leaf SHA-1 (k_leaf_queue: work queue, LDS ring)"
    elif args.config == "records_verify":
        k = ("leaf phase: k_leaf_verify (header parse + record CRC + leaf SHA-1 from whole 128-byte lines in "
             "registers, input order)")
    elif records:
        k = ("leaf phase: k_locate + k_leaf<offsets, aligned-segment stage> (input order)"
             if args.records_fused == 0 else
             "leaf phase: k_leaf_records (header parse + whole 128-byte lines into registers, input order)")
    else:
        k = ("k_leaf<strided, LDS-DMA stage> (leaf SHA-1, level 0)" if args.leaf_load == 1 else
             "k_leaf<strided, 128-byte register runs> (leaf SHA-1, level 0)" if args.leaf_load in (0, 4)
             else f"k_leaf<strided, load path {args.leaf_load}> (leaf SHA-1, level 0)")
    if T > 1:
        k += f"; {T} tables per step over {args.table_lanes or 2} streams (per-table event spans overlap)"
    return k


def main():
    args = parse()
    if args.config in ("records", "records_verify") and args.value_bytes <= 30 + args.key_bytes:
        raise SystemExit("bench.py: --value-bytes (the record size) must exceed the 30-B header + --key-bytes")
    T = args.tables or (4 if args.config == "runs4" else 1)
    if args.config == "one_tree" and T != 1:
        raise SystemExit("bench.py: --config one_tree builds one tree per step (--tables 1)")
    if args.gather == "step" and T != 1:
        raise SystemExit("bench.py: --gather step gathers one table per step (--tables 1)")
    if args.backend == "capi":
        return main_capi(args, T)
    if args.config == "api_flush":
        return main_api_flush(args)
    if args.config == "small_flush":
        return main_small_flush(args)
    rc = ensure_ranks(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    out = run_ranks(args, T)
    if out is None:  # not rank 0: done
        return
    progress(f"{args.config}: ranks done, {out.get('value')} GiB/s")
    import gc
    import torch
    gc.collect()  # the tables and their closures hold this run's device buffers
    torch.cuda.empty_cache()
    # Rank 0, every rank's GPU state released: the one-process C-ABI group over
    # the same N GPUs (SURVEY 8e's process model, what the Go drop-in would use;
    # VERDICT r03 item 1), each in a fresh child process, then the CPU baseline.
    world = out["n_gpus"]
    t_start = time.perf_counter()

    def budget_left():  # the driver allows the whole run 600 s; keep the children well inside it
        return args.child_budget_s - (time.perf_counter() - t_start)
    if not args.no_capi and args.config in ("sstable4k", "runs4"):
        out["capi_group"] = capi_child(args, world, [], args.capi_timeout)
        progress("capi_group child done")
        if args.config == "sstable4k":
            if "error" in out["capi_group"]:  # the same group would fail again: no second wait
                out["capi_one_tree"] = {"error": "skipped: the group child failed"}
                out["capi_config4"] = {"error": "skipped: the group child failed"}
            else:
                out["capi_one_tree"] = capi_child(args, world, ["--config", "one_tree", "--tables", "1"],
                                                  args.capi_timeout)
                if (args.leaves, args.value_bytes, T) == (1 << 20, 4096, 1):
                    # BASELINE configs[4]'s per-GPU table: 8 Mi x 4 KiB = 32 GiB on each GPU
                    out["capi_config4"] = capi_child(args, world, ["--leaves", str(8 << 20), "--tables", "1"],
                                                     args.capi_timeout)
    if not args.no_subconfigs and args.config == "sstable4k" and world == 1 and T == 1 \
            and (args.leaves, args.value_bytes) == (1 << 20, 4096):
        # The other single-GPU BASELINE workloads, each a
        # fresh child with its own roofline, verification and CPU baseline on
        # the same sample: configs[2] (mixed) and the serialized-record form of
        # configs[1] (the literal sstable.go:58-74 / lsmtree.go:210-211 input).
        for key, cfg in SUBCONFIGS:
            left = budget_left()
            if left < 60:
                out[key] = {"error": f"skipped: {args.child_budget_s} s child budget spent"}
                continue
            out[key] = sub_child(args, cfg, int(min(args.capi_timeout, left)))
            progress(f"{key} child done: {out[key].get('value', out[key].get('error'))}")
    if not args.no_cpu_baseline:
        # at every N, on rank 0 once the ranks are done (the Go reference is
        # one process on the same host)
        out["cpu_baseline"] = cpu_baseline(args)
        out.update(vs_cpu(out.get("value"), out["cpu_baseline"]))
    print(json.dumps(out), flush=True)


# sub-record key -> the child's --config (bench.py --gpus 1 only): configs[2];
# configs[1] as serialized records (the flush's input, sstable.go:58-74); the
# compaction read as merge performs it, every record's Crc checked before its
# Value is hashed (record.go:163-169, lsmtree.go:210-211); the host-inclusive
# flush through the Go-API mirror (pinned arena, PCIe both ways)
SUBCONFIGS = (("config2_mixed", "mixed"), ("config1_records", "records"),
              ("config1_records_verify", "records_verify"), ("api_flush", "api_flush"))
SUB_KEYS = ("value", "unit", "n_gpus", "steps", "ms_per_step", "sclk_mhz", "roofline", "kernel_ms",
            "verified_vs_oracle", "verified_basis", "root", "cpu_baseline", "vs_cpu_best", "vs_cpu_port_1core",
            "crc_checked", "value_basis", "breakdown_ms", "first_flush", "first_over_steady_time", "reserve_ms",
            "first_flush_no_reserve", "bound_note")


def sub_child(args, config, timeout, run=None):
    """Run `bench.py --config <config> --gpus 1` (this run's step flags) in a
    fresh child and return the keys of its line that go into the parent's line
    (or {"error": ...}: a failed child never costs the parent its line)."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in CHILD_ENV_DROP}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = [sys.executable, os.path.abspath(__file__)] + list(sys.argv[1:]) + [
        "--config", config, "--gpus", "1", "--tables", "1", "--no-capi", "--no-subconfigs"]
    t0 = time.perf_counter()
    try:
        p = (run or subprocess.run)(cmd, stdout=subprocess.PIPE, text=True, timeout=timeout, env=env)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {timeout} s", "cmd": " ".join(cmd[1:])}
    lines = [x for x in (p.stdout or "").splitlines() if x.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"exit status {p.returncode}", "cmd": " ".join(cmd[1:])}
    d = json.loads(lines[-1])
    sub = {k: d[k] for k in SUB_KEYS if k in d}
    sub["workload"] = d.get("config", {}).get("workload")
    sub["wall_s"] = round(time.perf_counter() - t0, 1)
    return sub


CHILD_ENV_DROP = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                  "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT",
                  "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_RUN_ID",
                  "TORCHELASTIC_USE_AGENT_STORE", "TORCH_NCCL_ASYNC_ERROR_HANDLING", "TORCHELASTIC_ERROR_FILE")
CAPI_KEYS = ("value", "unit", "n_gpus", "steps", "ms_per_step", "backend", "sclk_mhz", "root_gather_ok",
             "verified_vs_oracle", "verified_members", "members_agree", "root", "kernel_ms")


def capi_cmd(args, world, extra):
    """The C-ABI group child's command line: this run's flags with the group
    backend over `world` GPUs (later flags win in argparse)."""
    argv = [a for a in sys.argv[1:]]
    return [sys.executable, os.path.abspath(__file__)] + argv + ["--backend", "capi", "--gpus", str(world),
                                                                  "--no-cpu-baseline"] + list(extra)


def capi_child(args, world, extra, timeout, run=None):
    """Run the one-process group bench (main_capi) in a fresh child, outside
    any launcher's process group, and return the keys of its JSON line that go
    into the parent's line (or {"error": ...}: a failed child never fails the
    bench)."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in CHILD_ENV_DROP}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = capi_cmd(args, world, extra)
    t0 = time.perf_counter()
    try:
        p = (run or subprocess.run)(cmd, stdout=subprocess.PIPE, text=True, timeout=timeout, env=env)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {timeout} s", "cmd": " ".join(cmd[1:])}
    lines = [x for x in (p.stdout or "").splitlines() if x.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"exit status {p.returncode}", "cmd": " ".join(cmd[1:])}
    d = json.loads(lines[-1])
    sub = {k: d[k] for k in CAPI_KEYS if k in d}
    sub["parallelism"] = d.get("config", {}).get("parallelism")
    sub["workload"] = d.get("config", {}).get("workload")
    sub["roofline_frac"] = d.get("roofline", {}).get("frac")
    sub["wall_s"] = round(time.perf_counter() - t0, 1)
    return sub


def run_ranks(args, T):
    """This rank's measurement (one process per GPU); returns the JSON line's
    dict on rank 0, None on the others.  Every GPU tensor of the run is
    released before it returns."""
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
    set_options(args, _lib, ctx)

    roots = torch.empty(world * 20, dtype=torch.uint8, device="cuda")
    mixed = args.config == "mixed"
    one_tree = args.config == "one_tree"
    records = args.config in ("records", "records_verify")
    verify_crc = args.config == "records_verify"
    tabs = build_tables(args, torch, _lib, L, ctx, rank, T)
    t0_ = tabs[0]
    n, vlen, nodes = t0_["n"], t0_["vlen"], t0_["nodes"]
    nbytes = sum(t["nbytes"] for t in tabs)  # payload per step on this GPU
    arr = (_lib.NkvTable * T)(*[t["table"] for t in tabs])

    if one_tree:  # one tree over every rank's leaves (rank r holds leaves [r n, (r+1) n))
        from nakevaleng_amd import sharded_tree
        if n & (n - 1):
            raise SystemExit("--config one_tree needs a power-of-two --leaves (ranges aligned to 2^k)")
        ops = sharded_tree.DeviceOps(dev, ctx=ctx)
        data = t0_["data"]

        def tree():
            nodes[-20:] = sharded_tree.sharded_root((data, vlen, vlen), n * world, ops=ops, host_root=False)
    elif T == 1:
        tree = t0_["single"]
    else:
        def tree():
            _lib.check(L.nkv_trees_dev(ctx.h, arr, T), "nkv_trees_dev")

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
        rg = BatchedRootGather(nodes, world, gdist, cap=T * max(args.steps, args.warmup, 8))
    more = tuple(t["nodes"] for t in tabs[1:])

    def step():
        nonlocal nodes
        nodes = rg.begin()
        if args.gather == "step":
            t0_["nodes"] = nodes
        tree()
        rg.end(nodes, more) if args.gather != "step" else rg.end(nodes)

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
    if records and any(int(t["d_err"].item()) != 0 or (verify_crc and int(t["d_stats"][2].item()) != 0)
                       for t in tabs):
        # a malformed synthetic stream would time empty hashes
        raise SystemExit("bench.py: the record stream failed the header checks")
    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.set_option(_lib.NKV_OPT_TIMING_EVERY, max(1, args.timing_every))
    ctx.set_timing(not args.no_kernel_timing, clock=not args.no_clock)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    sclk, clock_waves = ctx.clock() if not args.no_clock else (None, 0)
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

    # every rank's roots against the committed oracle roots (no flag needed;
    # VERDICT r03 item 1): one code per rank, gathered to all ranks
    if one_tree:  # every rank reduced the top levels itself (sharded_tree): its root must be the tree's
        want1 = expected_one_tree(n, vlen, world)
        code = -1 if want1 is None else int(root == want1)
    else:
        want = expected_roots(args.config, n, t0_.get("rb", vlen), rank, T, args.key_bytes, args.mixed_bytes)
        mine = [t["nodes"][-20:].cpu().numpy().tobytes().hex() for t in tabs]
        code = -1 if want is None else int(mine == want)
    crc_stats = None
    if verify_crc:  # the last step's record check: every stored Crc must have matched, no header outside
        crc_stats = [t["d_stats"].cpu().tolist() for t in tabs]
        if any(st != [0, -1, 0] for st in crc_stats):
            code = 0
    codes = rank_codes(dist if use_dist else None, world, rank, code, "cuda")
    verified = verdict(codes)
    if args.verify and rank == 0 and verified is None:
        import numpy as np
        from oracle import oracle_c as oc
        if records:
            assert all(int(t["d_err"].item()) == 0 for t in tabs)
            if verify_crc:
                assert all(t["d_stats"].cpu().tolist() == [0, -1, 0] for t in tabs), "a stored Crc failed"
        if one_tree:
            host = np.concatenate([oc.splitmix64_bytes(n * vlen, SEED + r) for r in range(world)])
            want = oc.tree_from_digests(oc.leaf_hashes_strided(host, vlen, vlen, len(host) // vlen, threads=16))
            verified = want[-1].tobytes().hex() == root
            del host
        else:
            verified = all(t["want"]() == t["nodes"][-20:].cpu().numpy().tobytes().hex() for t in tabs)

    out = None
    if rank == 0:
        total_bytes = nbytes * world * args.steps
        value = total_bytes / elapsed / 2**30
        table_bytes = t0_["nbytes"]
        achieved = table_bytes / (leaf_ms * 1e-3) / 1e9  # algorithmic payload bytes per K1 launch
        ceiling = valu_ceiling(sclk, valu_kind(args.config))
        traffic, traffic_bounds = pmc_traffic(args, n, vlen, table_bytes)
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
            "data": f"synthetic: splitmix64 bytes (seed {SEED_MIXED if mixed else SEED:#x} + rank"
                    + (f" + {TABLE_SEED_STEP} t for table t" if T > 1 else "") + ") generated in HBM",
            "config": {
                "workload": workload_text(args, n, vlen, table_bytes, world, T, t0_.get("rb"), t0_.get("ks")),
                "leaves_per_gpu": n * T,
                "tables_per_gpu": T,
                "value_bytes": vlen if not mixed else "64..65536 (mean %.0f)" % (table_bytes / n),
                "parallelism": (f"1 tree split over {world} ranks" + (" + RCCL all_gather of sub-roots" if world > 1 else ""))
                               if one_tree else
                               f"{world * T} independent tables" + ((" + RCCL all_gather of roots, "
                                                                     + ("one call per timed loop" if args.gather == "batch"
                                                                        else "one per table")) if world > 1 else ""),
            },
            "sclk_mhz": round(sclk, 1) if sclk else None,
            "roofline": {
                "bound": "hbm",
                "kernel": kernel_text(args, T),
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                # the whole step (leaf + tree + launches, N ranks): payload per
                # GPU / ms_per_step / peak
                "step_frac": round(nbytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_bounds": traffic_bounds,  # RDREQ x 64 .. x 128 B (profiles/pmc_traffic.json)
                # VALU-issue ceiling at the measured clock (sclk_mhz) and the
                # fraction of it the leaf kernel reached
                "valu_ceiling": round(ceiling, 1) if ceiling else SHA1_VALU_CEILING_GBS,
                "valu_ceiling_basis": (f"{SIMDS} SIMDs x {sclk:.0f} MHz / ({VALU_PER_WAVE_BLOCK[valu_kind(args.config)]}"
                                       f" VALU per wave-block x {VALU_CYCLES:g} cycles) x 4096 B") if ceiling else
                                      "tools/sha1_rate.hip at 2.37 GHz (no clock reading)",
                "valu_frac": round(achieved / (ceiling or SHA1_VALU_CEILING_GBS), 4),
            },
            "kernel_ms": {"leaf": round(leaf_ms, 4), "tree_reduce": round(reduce_ms, 4),
                          "bfs_image": round(bfs_ms, 4)},
            "clock_probe_waves": clock_waves,
            "root": root,
            "cpu_baseline": None,
        }
        if mixed and sclk:
            # the leaf phase can end no sooner than its longest value's chain
            longest = max(int((int(t["lens_h"].max()) + 9 + 63) // 64) for t in tabs)
            floor_ms = longest * LONE_WAVE_CYCLES_PER_BLOCK / (sclk * 1e6) * 1e3
            out["roofline"].update({"chain_floor_ms": round(floor_ms, 4),
                                    "chain_floor_basis": f"longest value {longest} compressions x "
                                                         f"{LONE_WAVE_CYCLES_PER_BLOCK:g} cycles at {sclk:.0f} MHz",
                                    "chain_frac": round(floor_ms / leaf_ms, 4)})
        if crc_stats is not None:
            out["crc_checked"] = {"records_per_table": n, "tables": T,
                                  "crc_mismatches": sum(st[0] for st in crc_stats),
                                  "header_errors": sum(st[2] for st in crc_stats),
                                  "basis": "d_stats of nkv_tree_verify_records_dev after the last timed step"}
        out["verified_vs_oracle"] = verified
        out["verified_ranks"] = [None if c < 0 else bool(c) for c in codes]
        out["verified_basis"] = ("tests/golden/bench_roots.json (C oracle roots of the same seeds, committed)"
                                 if all(c >= 0 for c in codes) else
                                 "the C oracle at run time (--verify)" if verified is not None else None)
        if gathered_ok is not None:
            out["root_gather_ok"] = gathered_ok
    # the ranks leave together; the caller releases this run's tensors (they
    # live in this frame and in the tables' closures) before any group child
    ctx.close()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()
    return out


def main_api_flush(args):
    """--config api_flush: the Merkle step of one memtable flush as the unchanged
    caller runs it (sstable.makeMetadata, core/sstable/sstable.go:58-74), through
    the C++ mirror of the Go API: NewLeaf per value from host memory (the copy
    into the pinned arena queued for the mirror's copy threads, the settled 32
    MiB chunks streamed to HBM during the loop), New (the device call + the
    pointer tree), Root.String(), Serialize to a fresh file.  Runs
    tools/api_flush.cpp with the copy threads (the default), then with the
    copies on the caller's thread (round 3's form); the first cycle of each
    allocates the arena, the steady state is the best later cycle.  The CPU
    baseline (the C restatement on one core and on every core this process may
    use) is measured in the same run, on the same values."""
    import subprocess
    import tempfile
    from nakevaleng_amd import build as nb
    exe = nb.build_api_flush()
    n, vlen = args.leaves, args.value_bytes
    runs = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        for mode, threads, retain, reserve in (("pool", -1, 1, 1), ("caller_thread", 0, 1, 1),
                                               ("pool_glibc_heap", -1, 0, 1), ("pool_no_reserve", -1, 1, 0)):
            out = subprocess.run([exe, str(n), str(vlen), str(max(3, args.api_cycles)), td, "1", hex(SEED), "1",
                                  str(threads), str(retain), str(reserve)], capture_output=True, text=True,
                                 timeout=900)
            if out.returncode != 0:
                raise SystemExit(f"api_flush failed: {out.stderr[-2000:]}")
            runs[mode] = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    # the steady state is the MEDIAN of the cycles after the first (VERDICT r04
    # item 3), reported beside the first (cold) and the best cycle
    def median_cycle(r):
        rest = sorted(r[1:], key=lambda c: c["gib_s"])
        return rest[(len(rest) - 1) // 2]
    best = {m: median_cycle(r) for m, r in runs.items()}
    root = best["pool"]["root"]
    # every cycle's root against the committed oracle root (1 Mi x 4 KiB), else
    # the oracle at run time under --verify
    want = (expected_roots("sstable4k", n, vlen, 0, 1) or [None])[0]
    if want is None and args.verify:
        from oracle import oracle_c as oc
        host = oc.splitmix64_bytes(n * vlen, SEED)
        want = oc.tree_from_digests(oc.leaf_hashes_strided(host, vlen, vlen, n, threads=16))[-1].tobytes().hex()
        del host
    verified = None if want is None else all(c["root"] == want for r in runs.values() for c in r)
    cpu = None if args.no_cpu_baseline else cpu_baseline(args)
    b, c0 = best["pool"], best["caller_thread"]
    first, top = runs["pool"][0], max(runs["pool"][1:], key=lambda c: c["gib_s"])
    keys = ("newleaf_ms", "new_call_ms", "upload_ms", "kernels_ms", "download_ms", "materialize_ms", "root_ms",
            "walk_ms", "write_ms", "total_ms")
    out = {
        "metric": "GiB/s host-inclusive Merkle step of one SSTable flush through the Go-API mirror "
                  "(NewLeaf x n from host memory, New, Root, Serialize)",
        "value": b["gib_s"],
        "unit": "GiB/s",
        "n_gpus": 1,
        "steps": len(runs["pool"]),
        "higher_is_better": True,
        "dtype": "u32",
        "data": f"synthetic: splitmix64 bytes (seed {SEED:#x}) in host memory (the memtable's values)",
        "config": {"workload": f"memtable flush: {n} x {vlen} B values, sstable.go:58-74 call sequence",
                   "leaves": n, "value_bytes": vlen, "copy_threads": b.get("copy_threads"),
                   "heap": "retained between flushes (M_MMAP_THRESHOLD 1 GiB, no trim), as a Go GC heap"},
        "value_basis": "median of the flushes after the first (steady state)",
        "breakdown_ms": {k: b[k] for k in keys},
        # the first flush of the process (arena and node storage allocated,
        # pages faulted in) and the best steady one
        "first_flush": {"gib_s": first["gib_s"], "arena_allocs": first.get("arena_allocs"),
                        **{k: first[k] for k in keys}},
        "first_over_steady_time": round(first["total_ms"] / b["total_ms"], 3),
        "reserve_ms": first.get("reserve_ms"),
        # the same without Session::Reserve: the first flush grows the arena
        "first_flush_no_reserve": {"gib_s": runs["pool_no_reserve"][0]["gib_s"],
                                   "arena_allocs": runs["pool_no_reserve"][0].get("arena_allocs"),
                                   **{k: runs["pool_no_reserve"][0][k] for k in keys}},
        "best_flush": {"gib_s": top["gib_s"], **{k: top[k] for k in keys}},
        "copies_on_caller_thread": {"gib_s": c0["gib_s"], **{k: c0[k] for k in keys}},
        # the same flush with glibc's default heap policy (every freed block over
        # 32 MiB unmapped: the next flush page-faults it again)
        "glibc_default_heap": {"gib_s": best["pool_glibc_heap"]["gib_s"],
                               **{k: best["pool_glibc_heap"][k] for k in keys}},
        "cycles": runs,
        "root": root,
        "verified_vs_oracle": verified,
        "cpu_baseline": cpu,
        # the path starts and ends in host memory: its bound is the host link,
        # not HBM (the payload crosses PCIe once, host -> HBM)
        "bound_note": {
            "bound": "pcie",
            "link_spec_gbs": PCIE_SPEC_GBS,
            "achieved_gbs": round(n * vlen / (b["total_ms"] * 1e-3) / 1e9, 2),
            "frac_of_link": round(n * vlen / (b["total_ms"] * 1e-3) / 1e9 / PCIE_SPEC_GBS, 3),
            "cpu_comparator": (f"cpu_baseline runs on the {cpu['host_threads']} host threads this job may use "
                               f"({cpu['cpu_model']}); a whole socket hashing in memory would beat this "
                               "PCIe-bound path" if cpu else None),
        },
    }
    out.update(vs_cpu(b["gib_s"], cpu))
    print(json.dumps(out), flush=True)


SMALL_MODE_KEYS = (("1", "small_pinned"), ("3", "small_resident"), ("3h", "small_resident_host_mailbox"),
                   ("2", "small_hbm"), ("0", "grid"))
# --config small_flush: (name, n, min value length, max value length); lengths
# uniform in [min, max], seed SMALL_SEED (tools/small_flush.cpp's generator)
SMALL_SEED = 0x6E616B67
SMALL_SHAPES = (
    ("flush_default", 10, 1, 200),     # MEMTABLE_CAPACITY = 10 under the 2 KB threshold (coreconf.go:33-34)
    ("compaction_default", 40, 1, 200),  # LSM_RUN_MAX = 4 such runs merged (coreconf.go:39)
    ("n100", 100, 1, 200),
    ("n256", 256, 1, 200),
    ("n1024", 1024, 1, 200),
    ("config0", 1024, 1024, 1024),     # BASELINE configs[0]: 1 Ki x 1 KiB
    ("n256_4k", 256, 4096, 4096),
    ("n1024_4k", 1024, 4096, 4096),    # 4 MiB: above the small path's 1 MiB bound
)


def small_shape_values(n, lo, hi, seed=SMALL_SEED):
    """tools/small_flush.cpp's memtable: len[i] = lo + splitmix(i) % (hi - lo + 1),
    then the bytes from the same stateful splitmix64 stream (host arrays)."""
    import numpy as np
    from oracle import oracle_c as oc
    used = 0
    if hi > lo:
        w = oc.splitmix64_bytes(8 * n, seed).view(np.uint64)
        lens = (lo + w % np.uint64(hi - lo + 1)).astype(np.uint64)
        used = n
    else:
        lens = np.full(n, lo, np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1])
    total = int(lens.sum())
    data = oc.splitmix64_bytes(total, seed, first=8 * used) if total else np.zeros(0, np.uint8)
    return data, off, lens


def main_small_flush(args):
    """--config small_flush: microseconds per flush at the reference engine's own
    default sizes and up to configs[0]'s 1 Ki x 1 KiB,
    through the C++ Go-API mirror (tools/small_flush.cpp: NewLeaf x n, New,
    Root.String(), the image; with the file write as well; and the bare C-ABI
    call), for each NKV_OPT_SMALL_PATH mode: 1 = the one-launch kernel over
    pinned host memory (default), 3 = the resident service (3h: with its
    requests in host memory, NKV_OPT_SERVICE_MAILBOX 1), 2 = the one launch
    through HBM, 0 = the grid path.  Beside each shape: the same flush in memory on one host core with the
    portable SHA-1 and with OpenSSL's (oracle/, nkvo_flush_reps), whose root every
    GPU run must reproduce."""
    import subprocess
    import tempfile
    from nakevaleng_amd import build as nb
    from oracle import oracle_c as oc
    exe = nb.build_small_flush()
    spec = [f"{n}:{lo}:{hi}:{SMALL_SEED:x}" for _, n, lo, hi in SMALL_SHAPES]
    gpu = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        modes = [m.strip() for m in args.small_modes.split(",") if m.strip()]
        for mode in modes:
            p = subprocess.run([exe, mode, str(args.small_reps), td] + spec, capture_output=True, text=True,
                               timeout=600)
            if p.returncode != 0:
                raise SystemExit(f"small_flush mode {mode} failed: {p.stderr[-2000:]}")
            gpu[mode] = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    shapes, verified = [], True
    for k, (name, n, lo, hi) in enumerate(SMALL_SHAPES):
        data, off, lens = small_shape_values(n, lo, hi)
        cpu = {}
        root = None
        for impl in ("port", "openssl"):
            est, root = oc.flush_us(data, off, lens, 3, openssl=impl == "openssl")
            reps = max(5, min(200000, int(0.25e6 / max(est, 0.05))))  # ~0.25 s per figure
            us_, r2 = oc.flush_us(data, off, lens, reps, openssl=impl == "openssl")
            assert r2 == root
            cpu[f"{impl}_1core_us"] = round(us_, 3)
        best_cpu = min(cpu.values())
        row = {"shape": name, "n": n, "value_bytes": [lo, hi], "payload_bytes": int(lens.sum()), "cpu": cpu,
               "root": root}
        for mode, key in SMALL_MODE_KEYS:
            if mode not in gpu:
                continue
            g = gpu[mode][k]
            ok = g["root"] == root
            verified = verified and ok
            row[key] = {"path": "small" if g["path"] == 1 else "grid", "mirror_us": g["mirror_us"],
                        "mirror_us_p10_p90": [g["mirror_us_p10"], g["mirror_us_p90"]], "file_us": g["file_us"],
                        "abi_us": g["abi_us"], "root_ok": ok}
        best_gpu = min(row[key]["mirror_us"] for mode, key in SMALL_MODE_KEYS if key in row)
        row["gpu_over_cpu_time"] = round(best_gpu / best_cpu, 2)
        shapes.append(row)
    # the smallest payload of the sweep at which the best GPU flush is at least as
    # fast as the best one-core CPU flush
    cross = next((r["payload_bytes"] for r in sorted(shapes, key=lambda r: r["payload_bytes"])
                  if r["gpu_over_cpu_time"] <= 1.0), None)
    head = shapes[0]
    out = {
        "metric": "microseconds per default-size flush (NewLeaf x 10 values <= 200 B, New, Root, image) "
                  "through the Go-API mirror",
        "value": head["small_pinned"]["mirror_us"],
        "unit": "us",
        "n_gpus": 1,
        "higher_is_better": False,
        "dtype": "u32",
        "data": f"synthetic: splitmix64 values (seed {SMALL_SEED:#x}) in host memory",
        "config": {"workload": "the reference engine's default flush (coreconf.go:33-34) and compaction (:39) "
                               "sizes, up to configs[0] and beyond the small path's bound",
                   "reps": args.small_reps},
        "shapes": shapes,
        "crossover_payload_bytes": cross,
        "verified_vs_oracle": verified,
        "cpu_model": cpu_model(),
    }
    print(json.dumps(out), flush=True)


def main_capi(args, T):
    """--backend capi: ONE process drives every GPU through the library's group
    (SURVEY.md 8e process model: nkv_group_create = a context per GPU +
    ncclCommInitAll).  A step builds T tables per GPU (nkv_group_trees_dev:
    table t on member t % N, the tables of a member over its streams) and
    all-gathers every root over RCCL inside the library; one_tree builds one
    tree split over the GPUs (nkv_group_tree_dev).  Inputs are resident in each
    GPU's HBM before timing starts; the timed region ends with every member
    synchronized."""
    if os.environ.get("WORLD_SIZE", "1") != "1":
        raise SystemExit("bench.py: --backend capi is one process for all GPUs (no launcher)")
    import numpy as np
    import torch
    from nakevaleng_amd import build as nb
    nb.build()
    from nakevaleng_amd import _lib
    L = _lib.lib()
    N = args.gpus
    if torch.cuda.device_count() < N:
        raise SystemExit(f"bench.py: --gpus {N} but {torch.cuda.device_count()} device(s) visible")
    grp = _lib.Group(list(range(N)))
    ctxs = []
    for m in range(N):
        c = grp.ctx(m)  # the member's context (owned by the group)
        set_options(args, _lib, c)
        ctxs.append(c)
    one_tree = args.config == "one_tree"
    per = []  # per member: its tables
    for m in range(N):
        with torch.cuda.device(m):
            # inputs are written on torch's stream (fills through the member's
            # context on that stream too); the member's own stream then waits
            # for them (nkv_ctx_use_own_stream orders the hand-over)
            ctxs[m].set_stream(torch.cuda.current_stream(m).cuda_stream)
            per.append(build_tables(args, torch, _lib, L, ctxs[m], m, T, device=f"cuda:{m}"))
            ctxs[m].set_stream(_lib._OWN)
    for m in range(N):
        torch.cuda.synchronize(m)
        _lib.check(L.nkv_ctx_sync(ctxs[m].h))
    n, vlen = per[0][0]["n"], per[0][0]["vlen"]
    nbytes = sum(t["nbytes"] for tabs in per for t in tabs)  # payload per step, all GPUs
    if one_tree:
        if n & (n - 1):
            raise SystemExit("--config one_tree needs a power-of-two --leaves (ranges aligned to 2^k)")
        parts = (_lib.NkvTable * N)(*[per[m][0]["table"] for m in range(N)])
        d_root = [torch.zeros(20, dtype=torch.uint8, device=f"cuda:{m}") for m in range(N)]
        droots = (ctypes.c_void_p * N)(*[d.data_ptr() for d in d_root])

        def step():
            _lib.check(L.nkv_group_tree_dev(grp.h, parts, n * N, droots, None), "nkv_group_tree_dev")
    else:
        order = [per[t % N][t // N] for t in range(N * T)]  # table t on member t % N
        arr = (_lib.NkvTable * (N * T))(*[t["table"] for t in order])

        def step():
            _lib.check(L.nkv_group_trees_dev(grp.h, arr, N * T, None), "nkv_group_trees_dev")

    t_pre, preroll_steps = time.perf_counter(), 0
    while preroll_steps < 8 or time.perf_counter() - t_pre < args.preroll_s:
        step()
        preroll_steps += 1
        if preroll_steps % 8 == 0:
            grp.sync()
    for _ in range(args.warmup):
        step()
    grp.sync()
    ctxs[0].set_option(_lib.NKV_OPT_TIMING_EVERY, max(1, args.timing_every))
    ctxs[0].set_timing(not args.no_kernel_timing, clock=not args.no_clock)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    grp.sync()
    elapsed = time.perf_counter() - t0
    sclk, clock_waves = ctxs[0].clock() if not args.no_clock else (None, 0)
    calls, leaf_ms_tot, _ = ctxs[0].timing_summary()
    ctxs[0].set_timing(False)
    # the gathered roots of the last step, checked against each table's own
    # nodes; every member's roots against the committed oracle roots
    members_agree = None
    if one_tree:
        got = [d.cpu().numpy().tobytes().hex() for d in d_root]  # every member reduced the top
        root = got[0]
        members_agree = all(r == root for r in got)
        gathered_ok = None
        want1 = expected_one_tree(n, vlen, N)
        codes = [-1 if want1 is None else int(r == want1) for r in got]
    else:
        roots = np.zeros(20 * N * T, np.uint8)
        _lib.check(L.nkv_group_trees_dev(grp.h, arr, N * T, _lib.p8(roots)))
        gathered_ok = all(roots[20 * t:20 * t + 20].tobytes() == order[t]["nodes"][-20:].cpu().numpy().tobytes()
                          for t in range(N * T))
        root = per[0][0]["nodes"][-20:].cpu().numpy().tobytes().hex()
        codes = []
        for m in range(N):
            want = expected_roots(args.config, n, per[0][0].get("rb", vlen), m, T, args.key_bytes, args.mixed_bytes)
            mine = [t["nodes"][-20:].cpu().numpy().tobytes().hex() for t in per[m]]
            codes.append(-1 if want is None else int(mine == want))
    verified = verdict(codes)
    if args.verify and verified is None:
        if one_tree:
            from oracle import oracle_c as oc
            host = np.concatenate([oc.splitmix64_bytes(n * vlen, SEED + r) for r in range(N)])
            verified = oc.tree_from_digests(oc.leaf_hashes_strided(host, vlen, vlen, n * N,
                                                                   threads=16))[-1].tobytes().hex() == root
        else:
            verified = all(t["want"]() == t["nodes"][-20:].cpu().numpy().tobytes().hex() for t in order)
    leaf_ms = leaf_ms_tot / max(calls, 1)
    table_bytes = per[0][0]["nbytes"]
    achieved = table_bytes / (leaf_ms * 1e-3) / 1e9 if calls else None
    ceiling = valu_ceiling(sclk, valu_kind(args.config))
    out = {
        "metric": "GiB/s Merkle leaf-hash + tree-reduce over device-resident record blocks",
        "value": round(nbytes * args.steps / elapsed / 2**30, 2),
        "unit": "GiB/s",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "preroll_steps": preroll_steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: splitmix64 bytes generated in each GPU's HBM",
        "backend": f"capi group: one process, {N} context(s), transport "
                   + ("RCCL" if grp.transport == _lib.NKV_TRANSPORT_RCCL else "copy"),
        "config": {
            "workload": workload_text(args, n, vlen, table_bytes, N, T, per[0][0].get("rb"), per[0][0].get("ks")),
            "leaves_per_gpu": n * T,
            "tables_per_gpu": T,
            "value_bytes": vlen,
            "parallelism": (f"1 tree split over {N} GPU(s), sub-roots all-gathered by the library" if one_tree else
                            f"{N * T} independent tables, every root all-gathered by the library each step"),
        },
        "sclk_mhz": round(sclk, 1) if sclk else None,
        "roofline": {
            "bound": "hbm",
            "kernel": kernel_text(args, T) + " (member 0)",
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "step_frac": round(nbytes / N / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
            "valu_ceiling": round(ceiling, 1) if ceiling else None,
            "valu_frac": round(achieved / ceiling, 4) if (ceiling and achieved) else None,
        },
        "kernel_ms": {"leaf": round(leaf_ms, 4)},
        "clock_probe_waves": clock_waves,
        "root": root,
        "cpu_baseline": None,
    }
    if gathered_ok is not None:
        out["root_gather_ok"] = gathered_ok
    if members_agree is not None:
        out["members_agree"] = members_agree
    out["verified_vs_oracle"] = verified
    out["verified_members"] = [None if c < 0 else bool(c) for c in codes]
    print(json.dumps(out), flush=True)
    grp.close()


if __name__ == "__main__":
    main()
