"""Per-run Merkle rebuild of core/lsmtree compaction, sharded over GPUs.

In the reference, compaction merges a level's runs (lsmtree.go:71-128), collects
NewLeaf(head.Rec.Value) for every output record (lsmtree.go:211) and builds the
output table's tree in MakeTableSecondaries (sstable.go:41-46).  Independent
table builds are independent trees, so they shard with no data-path exchange:
one process per GPU builds its tables, then the 20-byte roots are all-gathered
(RCCL over xGMI when the process group is "nccl"; gloo in CPU tests) so every
rank holds every table's root.  The k-way merge itself stays on the host.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

Table = Tuple[bytes, np.ndarray]  # (Data-table stream, RecSize per record)


def shard(num_tables: int, world: int, rank: int) -> List[int]:
    """Tables owned by `rank`: round-robin, one run per GPU when num_tables == world."""
    return list(range(rank, num_tables, world))


def rank_device(device=None) -> int:
    """The GPU this rank hashes on: `device` when given (an int or torch.device),
    else _lib.current_device() -- the same rule the mirrors' default contexts
    use (LOCAL_RANK modulo the visible devices, else torch's device if torch
    already set one up, else 0)."""
    if device is not None:
        return device.index if hasattr(device, "index") else int(device)
    from . import _lib
    return _lib.current_device()


def _call_build(build, table, dev):
    """build(table, device), or build(table) for a one-argument builder (the
    form compact_roots took before round 2)."""
    import inspect
    try:
        params = [p for p in inspect.signature(build).parameters.values()
                  if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)]
        takes_device = len(params) >= 2 or any(p.kind == p.VAR_POSITIONAL
                                               for p in inspect.signature(build).parameters.values())
    except (TypeError, ValueError):  # builtins without a signature: try the two-argument form
        takes_device = True
    return build(table, dev) if takes_device else build(table)


def gpu_table_root(table: Table, device: Optional[int] = None) -> bytes:
    """Root of one table's Merkle tree, values hashed in place on `device`
    (None: rank_device())."""
    from . import _lib
    stream, rec_sizes = table
    n = len(rec_sizes)
    L = _lib.lib()
    ctx = _lib.default_context(rank_device(device))
    buf = np.frombuffer(bytes(stream) + b"\0", dtype=np.uint8)
    rs = np.ascontiguousarray(rec_sizes, dtype=np.uint64)
    root = np.zeros(20, np.uint8)
    _lib.check(L.nkv_tree_from_records(ctx.h, _lib.p8(buf), buf.size - 1, _lib.p64(rs), n,
                                       _lib.p8(root), None, None), "compaction Merkle step")
    return root.tobytes()


def gather_roots(local: Dict[int, bytes], num_tables: int, device=None) -> List[bytes]:
    """All-gather {table index: 20-byte root} from every rank; returns roots by table index."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    per = (num_tables + world - 1) // world
    rec = 4 + 20  # table index (int32 LE, -1 = empty slot) + root
    mine = np.zeros((per, rec), np.uint8)
    mine[:, :4] = np.frombuffer(np.int32(-1).tobytes(), np.uint8)
    for slot, (idx, root) in enumerate(sorted(local.items())):
        mine[slot, :4] = np.frombuffer(np.int32(idx).tobytes(), np.uint8)
        mine[slot, 4:] = np.frombuffer(root, np.uint8)
    t = torch.from_numpy(mine.reshape(-1))
    if dist.get_backend() == "nccl":
        t = t.to(device if device is not None else torch.device("cuda", torch.cuda.current_device()))
    out = torch.empty(world * t.numel(), dtype=torch.uint8, device=t.device)
    dist.all_gather_into_tensor(out, t)
    allrec = out.cpu().numpy().reshape(-1, rec)
    roots: List[Optional[bytes]] = [None] * num_tables
    for r in allrec:
        idx = int(np.frombuffer(r[:4].tobytes(), np.int32)[0])
        if idx >= 0:
            roots[idx] = r[4:].tobytes()
    if any(x is None for x in roots):
        raise RuntimeError("gather_roots: a table root is missing")
    return roots  # type: ignore[return-value]


def compact_roots(tables: Sequence[Table], build: Callable[[Table, int], bytes] = None,
                  device=None) -> List[bytes]:
    """Build the Merkle tree of every table this rank owns and all-gather the roots.

    `build(table, device)` (or `build(table)`) maps one table to its root; the
    default hashes on this rank's GPU (rank_device(device): LOCAL_RANK under one
    process per GPU), and the roots are gathered from that same device over RCCL.
    """
    import torch.distributed as dist

    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    dev = rank_device(device)
    if build is None:
        build = gpu_table_root
    local = {i: _call_build(build, tables[i], dev) for i in shard(len(tables), world, rank)}
    if world == 1:
        return [local[i] for i in range(len(tables))]
    import torch
    return gather_roots(local, len(tables), torch.device("cuda", dev))
