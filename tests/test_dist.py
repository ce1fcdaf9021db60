"""CPU, world_size 2 over gloo: sharded per-run Merkle rebuild + root all-gather.

The table builder is injected (here: the oracle); on the GPU box the default
builder hashes on the rank's device and the group is RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from nakevaleng_amd import record


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_tables(k):
    rng = np.random.default_rng(11)
    tables = []
    for t in range(k):
        recs = [record.New(rng.bytes(8), rng.bytes(int(rng.integers(0, 200))), timestamp=t) for _ in range(37 + t)]
        tables.append(record.data_table(recs))
    return tables


def oracle_root(table):
    from oracle import oracle_c as oc
    stream, sizes = table
    off, ln = record.value_spans(stream, sizes)
    d = oc.leaf_hashes(np.frombuffer(stream, np.uint8), off, ln)
    return oc.tree_from_digests(d)[-1].tobytes()


def _worker(rank, world, port, k, q):
    import torch.distributed as dist
    from nakevaleng_amd import lsmtree
    # what torch.distributed.run sets for each rank of one node
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    devices = []

    def build(tb, device):
        devices.append(device)
        return oracle_root(tb)

    roots = lsmtree.compact_roots(make_tables(k), build=build)
    q.put((rank, devices, [r.hex() for r in roots]))
    dist.destroy_process_group()


@pytest.mark.parametrize("k", [2, 3, 4])
def test_compact_roots_world2(oracle, k):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, k, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    want = [oracle_root(t).hex() for t in make_tables(k)]
    assert res[0][2] == want and res[1][2] == want  # every rank holds every root
    assert len(res[0][1]) + len(res[1][1]) == k  # each table built exactly once
    assert len(res[0][1]) == (k + 1) // 2
    # each rank hashes on its own device (LOCAL_RANK), never all on device 0
    assert set(res[0][1]) == {0} and set(res[1][1]) == {1}


def test_rank_device_resolution(monkeypatch):
    """One device rule for lsmtree and the mirrors' default contexts:
    explicit device, else LOCAL_RANK modulo the visible devices, else torch's
    device only if torch already initialised its GPU state, else 0."""
    from nakevaleng_amd import _lib, lsmtree
    import torch
    monkeypatch.setattr(_lib, "device_count", lambda: 0)
    assert lsmtree.rank_device(3) == 3
    assert lsmtree.rank_device(torch.device("cuda", 5)) == 5
    monkeypatch.setenv("LOCAL_RANK", "6")
    assert lsmtree.rank_device() == 6 == _lib.current_device()
    monkeypatch.setattr(_lib, "device_count", lambda: 4)
    assert lsmtree.rank_device() == 2 == _lib.current_device()  # LOCAL_RANK modulo the visible devices
    monkeypatch.delenv("LOCAL_RANK")
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: False)
    assert lsmtree.rank_device() == 0 == _lib.current_device()
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: True)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 1)
    assert lsmtree.rank_device() == 1 == _lib.current_device()


def test_compact_roots_takes_one_or_two_argument_builders():
    """build(table) (the pre-round-2 form) and build(table, device) both work."""
    from nakevaleng_amd import lsmtree
    tables = [(b"x" * 10, [10]), (b"y" * 20, [20])]
    seen = []
    assert lsmtree.compact_roots(tables, build=lambda t: t[0][:1] * 20) == [b"x" * 20, b"y" * 20]
    assert lsmtree.compact_roots(tables, build=lambda t, d: seen.append(d) or t[0][:1] * 20, device=3) == \
        [b"x" * 20, b"y" * 20]
    assert seen == [3, 3]
