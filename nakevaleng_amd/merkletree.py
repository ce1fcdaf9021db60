"""Python mirror of the reference's ds/merkletree API, computed on the MI355X.

Same names, argument meaning and error behaviour as magley/nakevaleng
ds/merkletree (paths relative to the reference root):

  MerkleNode, MERKLE_NODE_EMPTY     merklenode.go:11-19
  NewLeaf                           merklenode.go:27-34   (deferred, batched on the GPU)
  MerkleNode.String/Serialize/...   merklenode.go:22-96
  MerkleTree, New                   merkletree.go:13-25   (raises "cannot build Merkle Tree from 0 nodes")
  MerkleTree.Serialize              merkletree.go:67-92   (O_WRONLY|O_CREATE, no O_TRUNC)
  MerkleTree.Deserialize            merkletree.go:97-157  (reproduces the root-only quirk)
  MerkleTree.Validate               merkletree.go:162-171

Every digest comes from libnkvmerkle.so (HIP, gfx950); there is no CPU hash
path.  NewLeaf records the value in a pending batch and returns a node whose
Data is filled when the batch is hashed -- by New(), or on first access to
Data -- so a sequence of NewLeaf calls becomes one kernel launch (the same
deferred-leaf design as the Go cgo shim in INTEGRATION.md).
"""
from __future__ import annotations

import ctypes
import io
from typing import List, Optional

import numpy as np

from . import _lib

MERKLE_NODE_EMPTY = 1  # merklenode.go:11


class MerkleTreeError(Exception):
    pass


class _LeafBatch:
    """Values handed to NewLeaf, hashed together on first need."""

    def __init__(self):
        self.values: List[bytes] = []
        self.digests: Optional[np.ndarray] = None
        self.device = None  # None: the process's device (_lib.current_device)

    def add(self, data: bytes) -> int:
        self.values.append(bytes(data))
        return len(self.values) - 1

    def packed(self):
        lens = np.fromiter((len(v) for v in self.values), dtype=np.uint64, count=len(self.values))
        off = np.zeros(len(self.values), np.uint64)
        if len(self.values) > 1:
            off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        base = np.frombuffer(b"".join(self.values) + b"\0", dtype=np.uint8)
        return base, off, lens

    def resolve(self) -> None:
        if self.digests is not None:
            return
        n = len(self.values)
        out = np.zeros((max(n, 1), 20), np.uint8)
        base, off, lens = self.packed()
        ctx = _lib.default_context(self.device)
        _lib.check(_lib.lib().nkv_leaf_hash(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(lens), n,
                                            _lib.p8(out)), "NewLeaf")
        self.set_digests(out[:n])

    def set_digests(self, d: np.ndarray) -> None:
        self.digests = d
        self.values = []  # the batch is sealed; NewLeaf opens a new one


_batch = _LeafBatch()


class MerkleNode:  # merklenode.go:15-19
    __slots__ = ("_data", "Left", "Right", "_pend")

    def __init__(self, Data: bytes = b"", Left: "MerkleNode" = None, Right: "MerkleNode" = None):
        self._data = bytes(Data)
        self.Left = Left
        self.Right = Right
        self._pend = None  # (batch, index) while the NewLeaf digest is pending

    @property
    def Data(self) -> bytes:
        if self._pend is not None:
            b, i = self._pend
            b.resolve()
            self._data = b.digests[i].tobytes()
            self._pend = None
        return self._data

    @Data.setter
    def Data(self, v: bytes) -> None:
        self._pend = None
        self._data = bytes(v)

    def _copy(self) -> "MerkleNode":  # Go value copy (`l := level[i]`, merkletree.go:41-42)
        c = MerkleNode.__new__(MerkleNode)
        c._data, c.Left, c.Right, c._pend = self._data, self.Left, self.Right, self._pend
        return c

    def String(self) -> str:  # merklenode.go:22-24
        return self.Data.hex()

    __str__ = String

    def Serialize(self, writer) -> None:  # merklenode.go:37-63
        d = self.Data
        if len(d) == 0:
            writer.write(bytes([MERKLE_NODE_EMPTY]))
        else:
            writer.write(b"\x00")
            writer.write(d)

    def Deserialize(self, reader) -> bool:  # merklenode.go:67-96; True = EOF
        fb = reader.read(1)
        if len(fb) < 1:
            return True
        if fb[0] & MERKLE_NODE_EMPTY:
            self.Data = b""
        else:
            d = reader.read(20)
            if len(d) < 20:
                return True
            self.Data = d
        return False


def NewLeaf(data: bytes) -> MerkleNode:  # merklenode.go:27-34
    global _batch
    if _batch.digests is not None:
        _batch = _LeafBatch()
    node = MerkleNode()
    node._pend = (_batch, _batch.add(data))
    return node


def _level_counts(n: int) -> List[int]:
    return [_lib.lib().nkv_level_count(n, L) for L in range(_lib.lib().nkv_num_levels(n))]


class MerkleTree:  # merkletree.go:13-15
    """A built tree.  Its digests live in `nodes` (every level, bottom-up); the
    pointer tree under Root is materialized on first access to Root."""

    def __init__(self):
        self._root: Optional[MerkleNode] = None
        self.nodes: Optional[np.ndarray] = None  # (total, 20) uint8 when built by New
        self.n = 0
        self._leaves: Optional[List[MerkleNode]] = None  # copies of the level given to New
        self._image: Optional[bytes] = None
        self._materialized = False

    # ---- Root (pointer tree) ----
    @property
    def Root(self) -> Optional[MerkleNode]:
        if self.nodes is not None and not self._materialized:
            self._materialize()
        return self._root

    @Root.setter
    def Root(self, v: Optional[MerkleNode]) -> None:
        self._root = v
        self._materialized = True
        self.nodes = None
        self._image = None

    def _materialize(self) -> None:
        counts = _level_counts(self.n)
        start = np.concatenate([[0], np.cumsum(counts)])
        below = list(self._leaves)  # level 0
        for L in range(1, len(counts)):
            cur = []
            s = int(start[L])
            prev = below
            if len(prev) % 2:
                prev = prev + [MerkleNode(b"")]  # merkletree.go:32-34
            for i in range(counts[L]):
                cur.append(MerkleNode(self.nodes[s + i].tobytes(), prev[2 * i], prev[2 * i + 1]))
            below = cur
        self._root = below[0]
        self._materialized = True

    # ---- Serialize ----
    def SerializeBytes(self) -> bytes:
        if not self._materialized and self._image is not None:
            return self._image
        out = io.BytesIO()  # merkletree.go:75-89
        queue = [self.Root]
        while queue:
            n = queue.pop(0)
            if n.Left is not None:
                queue.append(n.Left)
            if n.Right is not None:
                queue.append(n.Right)
            n.Serialize(out)
        return out.getvalue()

    def Serialize(self, fname: str) -> None:  # merkletree.go:67-92
        img = np.frombuffer(self.SerializeBytes() + b"\0", dtype=np.uint8)
        rc = _lib.lib().nkv_write_file(fname.encode(), _lib.p8(img), img.size - 1)
        if rc != _lib.NKV_OK:
            raise OSError(f"Serialize({fname!r}): {_lib.lib().nkv_strerror(rc).decode()}")

    # ---- Deserialize (root-only, as the reference) ----
    def Deserialize(self, fname: str) -> None:  # merkletree.go:97-157
        with open(fname, "rb") as f:
            self.DeserializeBytes(f.read())

    def DeserializeBytes(self, blob: bytes) -> None:
        r = io.BytesIO(blob)
        nodes: List[MerkleNode] = []
        while True:
            n = MerkleNode()
            if n.Deserialize(r):
                break
            nodes.append(n)
        # merkletree.go:129-156 pops the root, then tests `i >= len(queue)` against
        # the now-empty queue and breaks: the tree is the root alone.
        self.Root = nodes[0] if nodes else None

    # ---- Validate ----
    def Validate(self) -> bool:  # merkletree.go:162-171
        if self._leaves is not None and not self._materialized:
            # a tree New built whose pointer tree was never handed out: rehash
            # is the tree over its leaves -- one device call (nkv_tree_validate)
            return _validate_leaves(self._leaves, root_of(self))
        root = self.Root
        leaves = _new_shaped_leaves(root, self.n) if self.n else None
        if leaves is not None:
            # New's shape (checked link by link, pads empty and childless):
            # rehash is again the tree over the leaves' current Data
            return _validate_leaves(leaves, root.Data)
        h = _rehash(root)
        for i in range(20):
            if root.Data[i] != h[i]:
                return False
        return True


def _new_shaped_leaves(root: Optional[MerkleNode], n: int) -> Optional[List[MerkleNode]]:
    """The n level-0 nodes under root if the pointer tree has exactly the shape
    New builds for n leaves (merkletree.go:31-64: every internal node has two
    children, an odd level below the top ends in an empty childless pad,
    level-0 nodes are childless), else None.  On that shape rehash
    (merklenode.go:99-108) equals the tree rebuilt from the leaves' Data."""
    if root is None or n < 1:
        return None
    counts = _level_counts(n)
    top = len(counts) - 1
    cur = [root]
    for L in range(top, 0, -1):
        if len(cur) != counts[L] + (1 if (counts[L] & 1) and L < top else 0):
            return None
        if len(cur) > counts[L]:
            pad = cur[-1]
            if pad.Left is not None or pad.Right is not None or len(pad.Data) != 0:
                return None
        nxt: List[MerkleNode] = []
        for x in cur[:counts[L]]:
            if x.Left is None or x.Right is None:
                return None
            nxt.append(x.Left)
            nxt.append(x.Right)
        cur = nxt
    if len(cur) != counts[0] + (1 if (counts[0] & 1) and top > 0 else 0):
        return None
    if len(cur) > counts[0]:
        pad = cur[-1]
        if pad.Left is not None or pad.Right is not None or len(pad.Data) != 0:
            return None
    leaves = cur[:counts[0]]
    if any(x.Left is not None or x.Right is not None for x in leaves):
        return None
    return leaves


def _validate_leaves(leaves: List[MerkleNode], root: bytes) -> bool:
    """Validate of a tree New built from `leaves` (C-ABI nkv_tree_validate)."""
    if any(x.Left is not None or x.Right is not None for x in leaves):
        return _rehash_root_matches(leaves, root)
    datas = [x.Data for x in leaves]
    n = len(datas)
    lens = np.fromiter((len(d) for d in datas), dtype=np.uint64, count=n)
    off = np.zeros(n, np.uint64)
    if n > 1:
        off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    base = np.frombuffer(b"".join(datas) + b"\0", dtype=np.uint8)
    if len(root) < 20:
        raise MerkleTreeError("Validate: index out of range")  # Go: Root.Data[i], i < 20
    r = np.frombuffer(bytes(root[:20]), np.uint8).copy()
    ok = ctypes.c_int(0)
    _lib.check(_lib.lib().nkv_tree_validate(_lib.default_context().h, _lib.p8(base), _lib.p64(off),
                                            _lib.p64(lens), n, _lib.p8(r), ctypes.byref(ok)), "Validate")
    return bool(ok.value)


def _rehash_root_matches(leaves: List[MerkleNode], root: bytes) -> bool:
    """Leaves that are themselves subtrees: rehash them first, then the tree above."""
    return _validate_leaves([MerkleNode(_rehash(x)) for x in leaves], root)


def _rehash(node: MerkleNode) -> bytes:
    """merklenode.go:99-108 on the device.

    A childless node (leaf, or pad: empty Data) yields its Data; any other node
    SHA-1(rehash(Left) || rehash(Right)).  Pads make the tree ragged, so the
    pointer tree is walked by depth and every depth's internal nodes are hashed
    in one nkv_leaf_hash batch, deepest first."""
    levels: List[List[MerkleNode]] = [[node]]
    while True:
        nxt = []
        for n in levels[-1]:
            if (n.Left is None) != (n.Right is None):
                raise MerkleTreeError("Validate: node with a single child")  # Go: nil dereference
            if n.Left is not None:
                nxt.extend((n.Left, n.Right))
        if not nxt:
            break
        levels.append(nxt)
    val = {}
    for depth in range(len(levels) - 1, -1, -1):
        msgs, owners = [], []
        for n in levels[depth]:
            if n.Left is None:
                val[id(n)] = n.Data
            else:
                msgs.append(val[id(n.Left)] + val[id(n.Right)])
                owners.append(n)
        if msgs:
            for n, d in zip(owners, _sha1_many(msgs)):
                val[id(n)] = d
    return val[id(node)]


def _sha1_many(msgs: List[bytes]) -> List[bytes]:
    n = len(msgs)
    lens = np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=n)
    off = np.zeros(n, np.uint64)
    if n > 1:
        off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    base = np.frombuffer(b"".join(msgs) + b"\0", dtype=np.uint8)
    out = np.zeros((n, 20), np.uint8)
    ctx = _lib.default_context()
    _lib.check(_lib.lib().nkv_leaf_hash(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(lens), n,
                                        _lib.p8(out)), "Validate")
    return [out[i].tobytes() for i in range(n)]


def New(level: List[MerkleNode]) -> MerkleTree:  # merkletree.go:18-25
    n = len(level)
    if n == 0:
        raise MerkleTreeError("cannot build Merkle Tree from 0 nodes")
    ctx = _lib.default_context()
    L = _lib.lib()
    tree = MerkleTree()
    tree.n = n
    tree._leaves = [x._copy() for x in level]
    total = L.nkv_total_nodes(n)
    nodes = np.zeros((total, 20), np.uint8)
    img = None
    b0 = level[0]._pend[0] if level[0]._pend is not None else None
    same_batch = (b0 is not None and b0.digests is None and len(b0.values) == n
                  and all(x._pend is not None and x._pend[0] is b0 and x._pend[1] == i
                          for i, x in enumerate(level)))
    childless = all(x.Left is None and x.Right is None for x in level)
    if same_batch:
        # the flush/compaction pattern: n NewLeaf calls, then New -- one fused call
        base, off, lens = b0.packed()
        img = np.zeros(L.nkv_bfs_size(n), np.uint8)
        _lib.check(L.nkv_tree_from_values(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(lens), n,
                                          None, _lib.p8(nodes), _lib.p8(img)), "New")
        b0.set_digests(nodes[:n].copy())
    elif all(len(x.Data) == 20 for x in level):
        leaf20 = np.frombuffer(b"".join(x.Data for x in level), dtype=np.uint8).copy()
        img = np.zeros(L.nkv_bfs_size(n), np.uint8)
        _lib.check(L.nkv_tree_build(ctx.h, _lib.p8(leaf20), n, None, _lib.p8(nodes), _lib.p8(img)), "New")
    else:
        datas = [x.Data for x in level]
        lens = np.fromiter((len(d) for d in datas), dtype=np.uint64, count=n)
        off = np.zeros(n, np.uint64)
        if n > 1:
            off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        base = np.frombuffer(b"".join(datas) + b"\0", dtype=np.uint8)
        img = np.zeros(L.nkv_generic_bfs_size(_lib.p64(lens), n), np.uint8)
        up = np.zeros((total - n, 20), np.uint8)
        _lib.check(L.nkv_tree_generic(ctx.h, _lib.p8(base), _lib.p64(off), _lib.p64(lens), n, None,
                                      _lib.p8(up), _lib.p8(img)), "New")
        nodes[n:] = up
        for i, d in enumerate(datas):  # level 0 of `nodes` is only meaningful for 20-byte Data
            if len(d) == 20:
                nodes[i] = np.frombuffer(d, np.uint8)
    for x in tree._leaves:
        x.Data  # resolve pending digests into the copies
    tree.nodes = nodes
    tree._image = img.tobytes() if (img is not None and childless) else None
    if not childless:
        tree._materialize()
    return tree


def root_of(tree: MerkleTree) -> bytes:
    """Root digest without materializing the pointer tree."""
    if tree.nodes is not None and not tree._materialized:
        return tree.nodes[-1].tobytes()
    return tree.Root.Data
