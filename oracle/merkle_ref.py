"""Literal Python restatement of magley/nakevaleng ds/merkletree (TEST INFRASTRUCTURE ONLY).

Nothing in the product imports this module.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may use it, and only as the checker.

Parity status: SHA-1 is hashlib's (OpenSSL) and is pinned by the FIPS 180-4 known
answers in tests/test_oracle.py.  The tree layer is "parity unpinned": the reference
is Go (no toolchain in this image) and has no tests or fixtures for this package
(SURVEY.md sections 4 and 8c).  It is cross-checked against the independent C
restatement in oracle/merkle_oracle.c.

This module deliberately follows the Go code statement by statement, including the
pointer tree, the value copies made by `l := level[i]` / `Left: &l`, the recursive
build, the queue-based BFS writer and the root-only Deserialize.  It is meant for
small trees (pure-Python loops); the C oracle covers large ones.
"""
from __future__ import annotations

import hashlib
import io
from dataclasses import dataclass, field
from typing import List, Optional

MERKLE_NODE_EMPTY = 1  # ds/merkletree/merklenode.go:11


@dataclass
class MerkleNode:  # merklenode.go:15-19
    Data: bytes = b""
    Left: Optional["MerkleNode"] = None
    Right: Optional["MerkleNode"] = None

    def String(self) -> str:  # merklenode.go:22-24
        return self.Data.hex()

    def copy(self) -> "MerkleNode":  # Go value copy: `l := level[i]`
        return MerkleNode(self.Data, self.Left, self.Right)

    def Serialize(self, w: io.BufferedIOBase) -> None:  # merklenode.go:37-63
        flags = 0
        if len(self.Data) == 0:
            flags |= MERKLE_NODE_EMPTY
        w.write(bytes([flags]))
        if (flags & MERKLE_NODE_EMPTY) != MERKLE_NODE_EMPTY:
            w.write(self.Data)

    def Deserialize(self, r: io.BufferedIOBase) -> bool:  # merklenode.go:67-96
        fb = r.read(1)
        if len(fb) < 1:
            return True
        if (fb[0] & MERKLE_NODE_EMPTY) == MERKLE_NODE_EMPTY:
            self.Data = b""
        else:
            d = r.read(20)
            if len(d) < 20:
                return True
            self.Data = d
        return False

    def rehash(self) -> bytes:  # merklenode.go:99-108
        if self.Left is None and self.Right is None:
            return self.Data
        lh = self.Left.rehash()
        rh = self.Right.rehash()
        return hashlib.sha1(lh + rh).digest()


def NewLeaf(data: bytes) -> MerkleNode:  # merklenode.go:27-34
    return MerkleNode(hashlib.sha1(bytes(data)).digest(), None, None)


class MerkleTreeError(Exception):
    pass


@dataclass
class MerkleTree:  # merkletree.go:13-15
    Root: Optional[MerkleNode] = None

    def _build(self, level: List[MerkleNode]) -> List[MerkleNode]:  # merkletree.go:31-64
        if len(level) % 2 != 0:
            level = level + [MerkleNode(b"")]
        new_level: List[MerkleNode] = []
        i = 0
        while i < len(level) - 1:
            l = level[i].copy()
            r = level[i + 1].copy()
            h = hashlib.sha1(l.Data + r.Data).digest()
            new_level.append(MerkleNode(h, l, r))
            i += 2
        if len(new_level) == 1:
            return new_level
        return self._build(new_level)

    def Serialize(self, fname: str) -> None:  # merkletree.go:67-92 (O_WRONLY|O_CREATE, no O_TRUNC)
        import os
        fd = os.open(fname, os.O_WRONLY | os.O_CREAT, 0o666)
        with os.fdopen(fd, "r+b") as f:
            f.write(self.SerializeBytes())

    def SerializeBytes(self) -> bytes:
        out = io.BytesIO()
        queue = [self.Root]
        while queue:
            n = queue.pop(0)
            if n.Left is not None:
                queue.append(n.Left)
            if n.Right is not None:
                queue.append(n.Right)
            n.Serialize(out)
        return out.getvalue()

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
        if not nodes:
            self.Root = None
            return
        # The reference's loop compares `i` against the (just emptied) queue and
        # breaks on its first iteration: only the root survives (merkletree.go:135-143).
        queue = []
        i = 0
        self.Root = nodes[i]
        i += 1
        queue.append(self.Root.copy())
        while len(queue) != 0:
            n = queue.pop(0)
            if i >= len(queue):
                break
            n.Left = nodes[i]  # pragma: no cover  (unreachable, kept for fidelity)
            queue.append(nodes[i].copy())
            i += 1
            if i >= len(queue):
                break
            n.Right = nodes[i]
            i += 1
            queue.append(nodes[i].copy())

    def Validate(self) -> bool:  # merkletree.go:162-171
        h = self.Root.rehash()
        for i in range(20):
            if self.Root.Data[i] != h[i]:
                return False
        return True


def New(level: List[MerkleNode]) -> MerkleTree:  # merkletree.go:18-25
    if len(level) == 0:
        raise MerkleTreeError("cannot build Merkle Tree from 0 nodes")
    t = MerkleTree()
    t.Root = t._build(list(level))[0]
    return t


def levels_of(tree: MerkleTree) -> List[List[bytes]]:
    """Top-down list of levels (pads included as b"") read off the pointer tree."""
    out = []
    cur = [tree.Root]
    while cur:
        out.append([n.Data for n in cur])
        nxt = []
        for n in cur:
            if n.Left is not None:
                nxt.append(n.Left)
            if n.Right is not None:
                nxt.append(n.Right)
        cur = nxt
    return out
