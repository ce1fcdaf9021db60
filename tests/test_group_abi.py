"""CPU: argument and error paths of the round-3 C-ABI entries -- the multi-GPU
group (one process, one context per GPU, RCCL), the multi-table
entry, arena streaming and the clock probe -- without touching a device, and the
split plan against the Python restatement (nakevaleng_amd/sharded_tree.py).

Reference: compaction merges a level's runs into one table
(core/lsmtree/lsmtree.go:71-128,211) whose tree MakeTableSecondaries builds
(core/sstable/sstable.go:35-47); padding only at a level's end
(ds/merkletree/merkletree.go:32-34) is what makes the 2^k split exact.
"""
import ctypes

import pytest


@pytest.fixture(scope="module")
def lib():
    from nakevaleng_amd import build as b
    b.build()
    from nakevaleng_amd import _lib
    return _lib


def test_split_span_matches_python_plan(lib):
    from nakevaleng_amd import sharded_tree as st
    L = lib.lib()
    for n in list(range(1, 300)) + [1 << 20, (1 << 20) + 1, 3 << 20, 8 << 23]:
        for g in range(1, 10):
            k, ranges, G = st.plan(n, g)
            span = L.nkv_split_span(n, g)
            assert span == 1 << k, (n, g)
            assert G == -(-n // span) <= g
            assert ranges[0][0] == 0 and ranges[-1][1] == n
    assert L.nkv_split_span(0, 4) == 0 and L.nkv_split_span(10, 0) == 0


def test_group_create_argument_checks(lib):
    L = lib.lib()
    out = ctypes.c_void_p(123)
    devs = (ctypes.c_int * 2)(0, 1)
    assert L.nkv_group_create(devs, 2, None) == lib.NKV_ERR_INVALID
    assert L.nkv_group_create(None, 2, ctypes.byref(out)) == lib.NKV_ERR_INVALID
    assert out.value is None  # *out cleared before any failure
    assert L.nkv_group_create(devs, 0, ctypes.byref(out)) == lib.NKV_ERR_INVALID
    assert L.nkv_group_create(devs, 65, ctypes.byref(out)) == lib.NKV_ERR_INVALID
    bad = (ctypes.c_int * 1)(-1)
    assert L.nkv_group_create(bad, 1, ctypes.byref(out)) in (lib.NKV_ERR_DEVICE,)


def test_group_create_without_device_fails_loudly(lib):
    if lib.device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(lib.NkvError):
        lib.Group([0])


def test_null_group_and_context_entries(lib):
    L = lib.lib()
    assert L.nkv_group_size(None) == 0
    assert L.nkv_group_transport(None) == 0
    L.nkv_group_destroy(None)  # no-op
    out = ctypes.c_void_p()
    assert L.nkv_group_ctx(None, 0, ctypes.byref(out)) == lib.NKV_ERR_INVALID
    assert L.nkv_group_sync(None) == lib.NKV_ERR_INVALID
    assert L.nkv_group_roots_allgather(None, None, None, None) == lib.NKV_ERR_INVALID
    assert L.nkv_group_trees_dev(None, None, 1, None) == lib.NKV_ERR_INVALID
    assert L.nkv_group_trees_from_values(None, None, 1) == lib.NKV_ERR_INVALID
    assert L.nkv_group_tree_dev(None, None, 5, None, None) == lib.NKV_ERR_INVALID
    assert L.nkv_group_tree_from_values(None, None, None, None, 5, None, None, None) == lib.NKV_ERR_INVALID
    assert L.nkv_group_tree_fetch(None, None, None) == lib.NKV_ERR_INVALID
    assert L.nkv_trees_dev(None, None, 0) == lib.NKV_ERR_INVALID
    assert L.nkv_host_stream(None, None, 0) == lib.NKV_ERR_INVALID
    mhz, waves = ctypes.c_double(), ctypes.c_uint64()
    assert L.nkv_ctx_clock(None, ctypes.byref(mhz), ctypes.byref(waves)) == lib.NKV_ERR_INVALID
    a = ctypes.c_float()
    assert L.nkv_ctx_last_host_timing(None, ctypes.byref(a), ctypes.byref(a), ctypes.byref(a)) == \
        lib.NKV_ERR_INVALID


def test_table_struct_layout_matches_header(lib):
    """The ctypes mirror of struct nkv_table / nkv_values has the C layout
    (int, then 8-byte fields: 12 x 8 bytes; nkv_values 7 x 8)."""
    assert ctypes.sizeof(lib.NkvTable) == 12 * 8
    assert lib.NkvTable.base.offset == 8 and lib.NkvTable.stats.offset == 88
    assert ctypes.sizeof(lib.NkvValues) == 7 * 8
    t = lib.table(lib.NKV_TABLE_RECORDS, nodes=0x1000, n=7, base=0x2000, base_len=99, off=0x3000)
    assert t.kind == 2 and t.n == 7 and t.base == 0x2000 and t.err is None
