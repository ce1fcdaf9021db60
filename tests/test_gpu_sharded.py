"""One tree over N ranks (sharded_tree.py) with the HIP library.

RCCL needs one GPU per rank, so the ranks' parts are built here one after
another on cuda:0 through DeviceOps (the path each rank runs), combined as
sharded_root combines them, and checked against the oracle (small trees) and
the library's whole-tree build (large ones).  world = 1 runs sharded_root
itself.  The collective paths are covered on CPU with gloo
(tests/test_sharded_tree.py).
"""
import numpy as np
import pytest
import torch

from nakevaleng_amd import sharded_tree as st

pytestmark = pytest.mark.gpu


def device_values(n, seed):
    rng = np.random.default_rng(seed)
    ln = rng.integers(0, 300, n).astype(np.int64)
    off = np.zeros(n, np.int64)
    off[1:] = np.cumsum(ln)[:-1]
    base = np.frombuffer(rng.bytes(int(ln.sum()) + 1), np.uint8).copy()
    return base, off, ln


def combine(ops, vals_h, n, world):
    base, off, ln = vals_h
    d_base = torch.from_numpy(base).cuda()
    k, ranges, G = st.plan(n, world)
    parts = []
    for lo, hi in ranges:
        d_off = torch.from_numpy(off[lo:hi].copy()).cuda()
        d_len = torch.from_numpy(ln[lo:hi].copy()).cuda()
        parts.append(st.build_range_levels(ops, (d_base, d_off, d_len), hi - lo, k))
    subs = torch.cat([p[-20:] for p in parts if p.numel()])
    if G == 1:
        top = subs.clone()
    else:
        top = ops.empty(20 * sum(st.count_of(G, j) for j in range(st.levels_of(G))))
        top[:20 * G] = subs
        ops.reduce(top, G)
    torch.cuda.synchronize()
    levels, offs = [], [0] * world
    host = [p.cpu().numpy() for p in parts]
    for j in range(k + 1):
        seg = []
        for r, (lo, hi) in enumerate(ranges):
            c = st.range_level_counts(hi - lo, k)[j]
            seg.append(host[r][offs[r]:offs[r] + 20 * c])
            offs[r] += 20 * c
        levels.append(np.concatenate(seg).reshape(-1, 20))
    if G > 1:
        th, o = top.cpu().numpy(), 0
        for j in range(st.levels_of(G)):
            c = st.count_of(G, j)
            if j:
                levels.append(th[o:o + 20 * c].reshape(-1, 20))
            o += 20 * c
    return top[-20:].cpu().numpy().tobytes(), st.bfs_image(levels)


@pytest.mark.parametrize("n", [1, 2, 3, 7, 64, 65, 1000, 4097])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_split_on_device_vs_oracle(oracle, n, world):
    vals = device_values(n, seed=n + world)
    root, img = combine(st.DeviceOps(0), vals, n, world)
    nodes = oracle.tree_from_digests(oracle.leaf_hashes(*vals))
    assert root == nodes[-1].tobytes()
    assert img == oracle.bfs_image(nodes, n)


@pytest.mark.parametrize("n,world", [(300001, 8), (262144, 4), (262145, 3)])
def test_split_on_device_vs_whole(nkv, n, world):
    _lib, ctx = nkv
    L = _lib.lib()
    vals = device_values(n, seed=7)
    root, img = combine(st.DeviceOps(0), vals, n, world)
    base, off, ln = vals
    nodes = torch.empty(L.nkv_total_nodes(n) * 20, dtype=torch.uint8, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    d_base = torch.from_numpy(base).cuda()
    d_off, d_len = torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()
    _lib.check(L.nkv_tree_from_values_dev(ctx.h, d_base.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                                          nodes.data_ptr()))
    d_img = torch.empty(L.nkv_bfs_size(n), dtype=torch.uint8, device="cuda")
    _lib.check(L.nkv_bfs_image_dev(ctx.h, nodes.data_ptr(), n, d_img.data_ptr()))
    torch.cuda.synchronize()
    assert root == nodes[-20:].cpu().numpy().tobytes()
    assert img == d_img.cpu().numpy().tobytes()


def test_sharded_root_world1_strided(oracle):
    n, L = 4099, 100
    data = np.frombuffer(np.random.default_rng(3).bytes(n * L), np.uint8).copy()
    d = torch.from_numpy(data).cuda()
    root, img = st.sharded_root((d, L, L), n, ops=st.DeviceOps(0), return_image=True)
    nodes = oracle.tree_from_digests(oracle.leaf_hashes_strided(data, L, L, n))
    assert root == nodes[-1].tobytes()
    assert img == oracle.bfs_image(nodes, n)
