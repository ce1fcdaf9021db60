"""CPU: the C-ABI library builds, loads and exports every symbol include/*.h
declares; pure shape helpers agree with the oracle; no compute without a GPU."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nkv_merkle.h")


@pytest.fixture(scope="module")
def lib():
    from nakevaleng_amd import build as b
    b.build()
    from nakevaleng_amd import _lib
    return _lib


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(nkv_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("nkv_leaf_hash", "nkv_tree_build", "nkv_tree_from_values", "nkv_tree_generic",
                 "nkv_tree_from_records", "nkv_bfs_size", "nkv_write_file", "nkv_tree_from_strided_dev",
                 "nkv_locate_values_dev", "nkv_ctx_create"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    so = lib.SO_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s(nkv_\w+)$", out, flags=re.M))
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, f"declared but not exported: {missing}"
    # and the ctypes table covers exactly the header
    assert sorted(lib.SIGNATURES) == declared_functions()
    L = lib.lib()
    for n in declared_functions():
        getattr(L, n)


def test_gfx950_code_object_present(lib):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", lib.SO_PATH],
                         capture_output=True, text=True, check=True).stdout
    assert ".hip_fatbin" in out
    assert b"amdgcn-amd-amdhsa--gfx950" in open(lib.SO_PATH, "rb").read()


def test_shape_helpers_match_oracle(lib, oracle):
    L = lib.lib()
    for n in list(range(1, 70)) + [255, 256, 257, 1000, 1023, 1024, 1025, 1 << 20, (1 << 20) + 1, 8 << 20]:
        assert L.nkv_num_levels(n) == oracle.num_levels(n)
        assert L.nkv_total_nodes(n) == oracle.total_nodes(n)
        assert L.nkv_bfs_size(n) == oracle.bfs_size(n)
        s = 0
        for lv in range(L.nkv_num_levels(n)):
            assert L.nkv_level_start(n, lv) == s
            s += L.nkv_level_count(n, lv)
        assert s == L.nkv_total_nodes(n)
        assert L.nkv_level_count(n, L.nkv_num_levels(n) - 1) == 1
    assert L.nkv_num_levels(0) == 0 and L.nkv_bfs_size(0) == 0
    assert L.nkv_bfs_size(1 << 20) == (2 * (1 << 20) - 1) * 21 == 44040171


def test_generic_bfs_size(lib):
    L = lib.lib()
    lens = np.array([1] * 7, np.uint64)  # README example: 162 bytes
    assert L.nkv_generic_bfs_size(lib.p64(lens), 7) == 162
    lens = np.array([0, 20, 5], np.uint64)
    # top (21) + level1 2 nodes (42) + level0: 0x01 | 0x00+20 | 0x00+5 | pad 0x01
    assert L.nkv_generic_bfs_size(lib.p64(lens), 3) == 21 + 42 + 1 + 21 + 6 + 1


def test_error_strings(lib):
    L = lib.lib()
    assert L.nkv_strerror(lib.NKV_ERR_EMPTY).decode() == "cannot build Merkle Tree from 0 nodes"
    assert L.nkv_strerror(lib.NKV_OK).decode() == "ok"


def test_write_file_has_no_truncate(lib, tmp_path):
    """Serialize opens O_WRONLY|O_CREATE without O_TRUNC (merkletree.go:68)."""
    L = lib.lib()
    f = str(tmp_path / "t-1-0-metadata.db")
    a = np.frombuffer(b"A" * 50, np.uint8).copy()
    b = np.frombuffer(b"B" * 20, np.uint8).copy()
    assert L.nkv_write_file(f.encode(), lib.p8(a), 50) == 0
    assert L.nkv_write_file(f.encode(), lib.p8(b), 20) == 0
    assert open(f, "rb").read() == b"B" * 20 + b"A" * 30  # stale tail kept, as in the reference
    assert L.nkv_write_file(str(tmp_path / "no/such/dir/x").encode(), lib.p8(b), 20) == lib.NKV_ERR_IO


def test_write_file_large(lib, tmp_path):
    """Images of tens of MiB: the file holds exactly the bytes written, and a
    longer stale file keeps its tail (no O_TRUNC)."""
    L = lib.lib()
    f = str(tmp_path / "big-1-0-metadata.db")
    rng = np.random.default_rng(7)
    old = rng.integers(0, 256, (70 << 20) + 13, dtype=np.uint8)
    assert L.nkv_write_file(f.encode(), lib.p8(old), old.size) == 0
    assert open(f, "rb").read() == old.tobytes()
    for n in [(8 << 20) - 1, 8 << 20, (44 << 20) + 40040171 % 997, (64 << 20) + 5]:
        new = rng.integers(0, 256, n, dtype=np.uint8)
        assert L.nkv_write_file(f.encode(), lib.p8(new), n) == 0
        got = open(f, "rb").read()
        assert len(got) == old.size
        assert got[:n] == new.tobytes()
        assert got[n:] == old.tobytes()[n:]
        old = np.frombuffer(got, np.uint8).copy()


def test_no_cpu_fallback_without_device(lib):
    """With no HIP device the product path fails loudly instead of hashing on the CPU."""
    if lib.device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(lib.NkvError):
        lib.Context(0)


def test_bloom_params_host_function_matches_oracle(oracle):
    """nkv_bloom_params is pure host math (no device): bloomfilter.go:18-24."""
    import ctypes
    from nakevaleng_amd import _lib
    L = _lib.lib()
    for n in (1, 7, 100, 4096, 1 << 20):
        for p in (0.01, 0.2, 0.001):
            m, k = ctypes.c_uint32(0), ctypes.c_uint32(0)
            assert L.nkv_bloom_params(n, p, ctypes.byref(m), ctypes.byref(k)) == 0
            assert (m.value, k.value) == oracle.bloom_params(n, p)
    m, k = ctypes.c_uint32(0), ctypes.c_uint32(0)
    assert L.nkv_bloom_params(0, 0.01, ctypes.byref(m), ctypes.byref(k)) == _lib.NKV_ERR_INVALID
    assert L.nkv_bloom_params(10, 1.5, ctypes.byref(m), ctypes.byref(k)) == _lib.NKV_ERR_INVALID


def test_build_id_is_the_source_hash(lib):
    """The library in the tree was compiled from these sources (nakevaleng_amd/build.py)."""
    from nakevaleng_amd import build as b
    want = b.source_hash()
    assert b.embedded_hash() == want
    assert lib.lib().nkv_build_id().decode() == "nkv-src-sha256:" + want


def test_validate_argument_checks_without_device(lib):
    import ctypes
    L = lib.lib()
    ok = ctypes.c_int(7)
    assert L.nkv_tree_validate(None, None, None, None, 0, None, ctypes.byref(ok)) == lib.NKV_ERR_INVALID
