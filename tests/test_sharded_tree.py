"""One tree over N ranks (nakevaleng_amd/sharded_tree.py) on CPU.

The device ops are replaced by the oracle (test infrastructure): the split,
the lone-node rehash, the sub-root gather, the top levels and the image
layout must give the whole tree's root and Serialize image exactly.  The
same host logic runs on the GPU in tests/test_gpu_sharded.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from nakevaleng_amd import sharded_tree as st


class OracleOps:
    def empty(self, nbytes):
        return torch.empty(nbytes, dtype=torch.uint8)

    def range_tree(self, values, n_r):
        from oracle import oracle_c as oc
        base, off, ln = values
        nodes = oc.tree_from_digests(oc.leaf_hashes(base, off, ln))
        return torch.from_numpy(nodes.reshape(-1).copy())

    def reduce(self, nodes, n):
        from oracle import oracle_c as oc
        full = oc.tree_from_digests(nodes[:20 * n].numpy().reshape(n, 20))
        nodes[:] = torch.from_numpy(full.reshape(-1))
        return nodes


def make_values(n, seed=5):
    rng = np.random.default_rng(seed)
    ln = rng.integers(0, 150, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln)[:-1]
    base = np.frombuffer(rng.bytes(int(ln.sum()) + 1), np.uint8)
    return base, off, ln


def range_values(vals, lo, hi):
    base, off, ln = vals
    return base, off[lo:hi], ln[lo:hi]


def whole(oracle, vals):
    nodes = oracle.tree_from_digests(oracle.leaf_hashes(*vals))
    return nodes[-1].tobytes(), oracle.bfs_image(nodes, len(vals[1]))


def test_plan_shapes():
    for n in range(1, 300):
        for world in range(1, 10):
            k, ranges, G = st.plan(n, world)
            assert k >= 1 and ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(h - l <= 1 << k for l, h in ranges)
            assert G == sum(1 for l, h in ranges if h > l)
            # every used range but the last is full (aligned to 2^k)
            assert all(h - l == 1 << k for l, h in ranges[:G - 1])
            assert st.levels_of(n) == (k + 1 if G == 1 else k + st.levels_of(G))
    with pytest.raises(ValueError, match="0 nodes"):
        st.plan(0, 2)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 7, 8, 9, 31, 33, 100, 257, 1000])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_split_equals_whole_tree(oracle, n, world):
    """Every rank's part computed in one process, combined as sharded_root does."""
    vals = make_values(n, seed=n)
    ops = OracleOps()
    k, ranges, G = st.plan(n, world)
    parts = [st.build_range_levels(ops, range_values(vals, l, h), h - l, k) for l, h in ranges]
    subs = torch.cat([p[-20:] for p in parts if p.numel()])
    assert subs.numel() == 20 * G
    if G == 1:
        top = subs.clone()
    else:
        top = ops.empty(20 * sum(st.count_of(G, j) for j in range(st.levels_of(G))))
        top[:20 * G] = subs
        ops.reduce(top, G)
    root, img = whole(oracle, vals)
    assert top[-20:].numpy().tobytes() == root
    # image from the per-level segments
    levels = []
    offs = [0] * world
    for j in range(k + 1):
        seg = []
        for r, (l, h) in enumerate(ranges):
            c = st.range_level_counts(h - l, k)[j]
            seg.append(parts[r][offs[r]:offs[r] + 20 * c].numpy())
            offs[r] += 20 * c
        levels.append(np.concatenate(seg).reshape(-1, 20))
    if G > 1:
        th, o = top.numpy(), 0
        for j in range(st.levels_of(G)):
            c = st.count_of(G, j)
            if j:
                levels.append(th[o:o + 20 * c].reshape(-1, 20))
            o += 20 * c
    assert st.bfs_image(levels) == img


def test_bfs_image_matches_oracle(oracle):
    for n in (1, 2, 3, 6, 7, 64, 65):
        nodes = oracle.tree_from_digests(oracle.leaf_hashes(*make_values(n)))
        levels, o = [], 0
        for j in range(st.levels_of(n)):
            c = st.count_of(n, j)
            levels.append(nodes[o:o + c])
            o += c
        assert st.bfs_image(levels) == oracle.bfs_image(nodes, n)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    vals = make_values(n, seed=n)
    k, ranges, G = st.plan(n, world)
    lo, hi = ranges[rank]
    root, img = st.sharded_root(range_values(vals, lo, hi), n, ops=OracleOps(), return_image=True)
    q.put((rank, root.hex(), None if img is None else img.hex()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1), (2, 5), (2, 1000), (3, 4), (3, 777)])
def test_sharded_root_gloo(oracle, world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    root, img = whole(oracle, make_values(n, seed=n))
    assert all(r[1] == root.hex() for r in res)  # every rank holds the root
    assert res[0][2] == img.hex() and all(r[2] is None for r in res[1:])
