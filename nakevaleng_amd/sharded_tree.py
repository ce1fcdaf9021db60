"""One Merkle tree over N GPUs ("single large tree").

The reference builds a table's tree on one goroutine (merkletree.go:31-64):
level by level, n_{j+1} = ceil(n_j / 2), an odd level padded with an empty
node so the lone last node's parent is SHA-1(node) (merkletree.go:32-34,44-46).
Parent i of level j+1 covers leaves [i 2^(j+1), (i+1) 2^(j+1)) and padding
only ever happens at a level's end, so a tree splits exactly at 2^k-aligned
leaf ranges:

- rank r takes leaves [r 2^k, (r+1) 2^k) with k = max(1, ceil(log2 ceil(n / N)));
- it builds the k levels of its range on its own GPU (the library's leaf and
  reduce kernels); the last, partial range keeps re-hashing its lone top node
  until level k, which is what the whole tree's padding does to it;
- the G = ceil(n / 2^k) level-k nodes (one per non-idle rank) are all-gathered
  (20 B per rank, RCCL over xGMI when the group is "nccl");
- every rank builds the top ceil(log2 G) levels from them (one small reduce),
  so every rank holds the root.

Level j <= k of the whole tree is the concatenation, in rank order, of every
range's level j (ceil(n_r / 2^j) nodes each), so the Serialize image
(merkletree.go:67-92: top level first, 21 B per node, one MERKLE_NODE_EMPTY
byte after each odd level below the top) is assembled on rank 0 from per-level
segments gathered there.

The device work goes through an ops object: DeviceOps calls the HIP library
(no CPU fallback); tests inject the oracle to run the same host logic on CPU.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

MERKLE_NODE_EMPTY = 1  # merklenode.go:11


# ---------------------------------------------------------------------------
# shape (mirrors capi.cpp levels_of / count_of: merkletree.go:31-64)

def levels_of(n: int) -> int:
    """Levels including the leaf level; build() always adds at least one."""
    if n == 0:
        return 0
    lv, c = 1, n
    while True:
        c = (c + 1) // 2
        lv += 1
        if c <= 1:
            return lv


def count_of(n: int, j: int) -> int:
    return n if j == 0 else ((n - 1) >> j) + 1


def plan(n: int, world: int) -> Tuple[int, List[Tuple[int, int]], int]:
    """(k, [(lo, hi) per rank], G): levels built per range, leaf ranges, ranges in use."""
    if n <= 0:
        raise ValueError("cannot build Merkle Tree from 0 nodes")  # merkletree.go:20
    if world < 1:
        raise ValueError("world must be >= 1")
    per = -(-n // world)
    k = max(1, (per - 1).bit_length())
    span = 1 << k
    ranges = [(min(n, r * span), min(n, (r + 1) * span)) for r in range(world)]
    return k, ranges, -(-n // span)


def range_level_counts(n_r: int, k: int) -> List[int]:
    """Node counts of levels 0..k of one range (0 for an idle rank)."""
    return [count_of(n_r, j) if n_r else 0 for j in range(k + 1)]


# ---------------------------------------------------------------------------
# device work

class DeviceOps:
    """The rank's GPU through the C-ABI, on torch's current stream."""

    def __init__(self, device: Optional[int] = None, ctx=None):
        import torch
        from . import _lib
        self.torch = torch
        self._lib = _lib
        self.L = _lib.lib()
        dev = torch.cuda.current_device() if device is None else device
        self.device = torch.device("cuda", dev)
        self.ctx = ctx if ctx is not None else _lib.Context(dev)
        self.ctx.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def empty(self, nbytes: int):
        return self.torch.empty(nbytes, dtype=self.torch.uint8, device=self.device)

    def range_tree(self, values, n_r: int):
        """Nodes (levels_of(n_r) levels, level-major) of one leaf range.

        values: (base, off, len) device tensors (uint8, int64, int64) or
        (base, stride, length) for equal-length values at base + i stride."""
        nodes = self.empty(20 * sum(count_of(n_r, j) for j in range(levels_of(n_r))))
        base, a, b = values
        if isinstance(a, int):
            rc = self.L.nkv_tree_from_strided_dev(self.ctx.h, base.data_ptr(), a, b, n_r, nodes.data_ptr())
        else:
            rc = self.L.nkv_tree_from_values_dev(self.ctx.h, base.data_ptr(), a.data_ptr(), b.data_ptr(), n_r,
                                                 nodes.data_ptr())
        self._lib.check(rc, "sharded range tree")
        return nodes

    def reduce(self, nodes, n: int):
        """Build the levels above n digests already in nodes[:20 n]."""
        self._lib.check(self.L.nkv_tree_reduce_dev(self.ctx.h, nodes.data_ptr(), n), "sharded top reduce")
        return nodes


def _rehash_chain(ops, top, m: int):
    """[top, SHA-1(top), SHA-1^2(top), ...]: m + 1 digests, the lone node's
    parents up to level k (an odd level of one node pads it: merkletree.go:32-34)."""
    chain = ops.empty(20 * (m + 1))
    chain[:20] = top
    pair = ops.empty(40)  # leaf + root of a one-leaf tree
    for i in range(m):
        pair[:20] = chain[20 * i:20 * i + 20]
        ops.reduce(pair, 1)
        chain[20 * (i + 1):20 * (i + 2)] = pair[20:40]
    return chain


def build_range_levels(ops, values, n_r: int, k: int):
    """Levels 0..k of one range as one flat uint8 tensor (level-major)."""
    if n_r == 0:
        return ops.empty(0)
    nodes = ops.range_tree(values, n_r)
    top_r = levels_of(n_r) - 1
    if top_r == k:
        return nodes
    chain = _rehash_chain(ops, nodes[-20:], k - top_r)
    out = ops.empty(nodes.numel() + chain.numel() - 20)
    out[:nodes.numel()] = nodes
    out[nodes.numel():] = chain[20:]
    return out


def _all_gather_roots(ops, sub_root, world: int):
    import torch
    import torch.distributed as dist
    out = torch.empty(world * 20, dtype=torch.uint8, device=sub_root.device)
    dist.all_gather_into_tensor(out, sub_root.contiguous())
    return out


def sharded_root(values, n: int, ops=None, return_image: bool = False, host_root: bool = True):
    """Root (20 bytes) of the tree over all ranks' leaves, on every rank.

    values: this rank's leaf range (see DeviceOps.range_tree); n: total leaves.
    With return_image, rank 0 also returns the Serialize image (bytes; None on
    other ranks).  host_root=False returns the root as a 20-byte tensor on the
    ops' device without waiting for it.  Every rank must call it (collective)."""
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    if ops is None:
        ops = DeviceOps()
    k, ranges, G = plan(n, world)
    lo, hi = ranges[rank]
    mine = build_range_levels(ops, values, hi - lo, k)
    sub_root = mine[-20:] if hi > lo else ops.empty(20).zero_()
    if world > 1:
        subs = _all_gather_roots(ops, sub_root, world)
    else:
        subs = sub_root
    if G == 1:
        top = ops.empty(20)
        top[:] = subs[:20]
    else:
        top = ops.empty(20 * sum(count_of(G, j) for j in range(levels_of(G))))
        top[:20 * G] = subs[:20 * G]
        ops.reduce(top, G)
    root = bytes(top[-20:].cpu().numpy().tobytes()) if host_root or return_image else top[-20:]
    if not return_image:
        return root
    image = _gather_image(mine, n, k, ranges, G, top, rank, world)
    return root, image


def _gather_image(mine, n: int, k: int, ranges, G: int, top, rank: int, world: int) -> Optional[bytes]:
    """Rank 0 collects every range's levels 0..k and lays out the image."""
    import torch
    counts = [range_level_counts(h - l, k) for l, h in ranges]
    sizes = [20 * sum(c) for c in counts]
    cap = max(sizes)
    buf = torch.zeros(cap, dtype=torch.uint8, device=mine.device)
    buf[:mine.numel()] = mine
    if world > 1:
        import torch.distributed as dist
        if rank == 0:
            parts = [torch.empty_like(buf) for _ in range(world)]
            dist.gather(buf, parts, dst=0)
        else:
            dist.gather(buf, None, dst=0)
            return None
    else:
        parts = [buf]
    host = [p.cpu().numpy() for p in parts]
    top_h = top.cpu().numpy()
    # levels bottom-up: 0..k from the ranges, k+1.. from the top tree
    levels: List[np.ndarray] = []
    offs = [0] * world
    for j in range(k + 1):
        segs = []
        for r in range(world):
            c = counts[r][j]
            segs.append(host[r][offs[r]:offs[r] + 20 * c])
            offs[r] += 20 * c
        levels.append(np.concatenate(segs).reshape(-1, 20))
    if G > 1:
        o = 0
        for j in range(levels_of(G)):
            c = count_of(G, j)
            if j > 0:
                levels.append(top_h[o:o + 20 * c].reshape(-1, 20))
            o += 20 * c
    return bfs_image(levels)


def bfs_image(levels: Sequence[np.ndarray]) -> bytes:
    """Serialize image from bottom-up levels of 20-byte nodes (merkletree.go:67-92,
    merklenode.go:37-63): top first, 0x00 + digest per node, MERKLE_NODE_EMPTY
    after an odd level below the top (the pad node, which has no children)."""
    out = []
    for j in range(len(levels) - 1, -1, -1):
        lv = levels[j]
        rows = np.zeros((lv.shape[0], 21), np.uint8)
        rows[:, 1:] = lv
        out.append(rows.tobytes())
        if j < len(levels) - 1 and lv.shape[0] % 2:
            out.append(bytes([MERKLE_NODE_EMPTY]))
    return b"".join(out)
