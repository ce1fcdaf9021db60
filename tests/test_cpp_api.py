"""The C++ ds/merkletree mirror (include/nkv_merkletree.hpp): compiles on CPU;
on the GPU its outputs match the golden fixtures and the oracle."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "test_merkletree_api.cpp")
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "merkle_golden.json")))


def build_binary(tmpdir):
    from nakevaleng_amd import build as b
    so = b.build()
    out = os.path.join(tmpdir, "test_merkletree_api")
    libdir = os.path.dirname(so)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"), SRC,
                           "-L", libdir, "-lnkvmerkle", f"-Wl,-rpath,{libdir}", "-o", out])
    return out


def test_cpp_mirror_compiles(tmp_path):
    assert os.path.exists(build_binary(str(tmp_path)))


def test_arena_copy_in_cpu(tmp_path):
    """NewLeaf's arena copy (non-temporal stores from 256 bytes up) is exact for
    every length and source alignment, and writes nothing past the value."""
    from nakevaleng_amd import build as b
    so = b.build()
    libdir = os.path.dirname(so)
    exe = os.path.join(str(tmp_path), "test_copy_in")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "test_copy_in.cpp"), "-L", libdir, "-lnkvmerkle",
                           f"-Wl,-rpath,{libdir}", "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr


@pytest.mark.parametrize("sanitize", [False, True])
def test_task_team_cpu(tmp_path, sanitize):
    """The mirror's host thread team (New's materialization, Serialize's walk):
    every part of every run exactly once, runs back to back, clean shutdown;
    also under ThreadSanitizer (host code only)."""
    from nakevaleng_amd import build as b
    so = b.build()
    libdir = os.path.dirname(so)
    exe = os.path.join(str(tmp_path), "test_task_team")
    flags = ["-O1", "-g", "-fsanitize=thread"] if sanitize else ["-O2"]
    subprocess.check_call(["g++", "-std=c++17", "-Wall", "-pthread", *flags, "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "test_task_team.cpp"), "-L", libdir, "-lnkvmerkle",
                           f"-Wl,-rpath,{libdir}", "-o", exe])
    out = subprocess.run([exe, "3000" if sanitize else "20000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.startswith("ok") and "WARNING" not in out.stderr, \
        out.stdout + out.stderr[-3000:]


@pytest.mark.parametrize("sanitize", [False, True])
def test_session_shared_by_threads_cpu(tmp_path, sanitize):
    """trees serialized and destroyed on several threads at once
    (the session's recycled storage is locked; the host team runs one caller's
    run at a time, the others inline), no GPU needed; also under
    ThreadSanitizer (host code only)."""
    from nakevaleng_amd import build as b
    so = b.build()
    libdir = os.path.dirname(so)
    exe = os.path.join(str(tmp_path), "test_session_threads")
    flags = ["-O1", "-g", "-fsanitize=thread"] if sanitize else ["-O2"]
    subprocess.check_call(["g++", "-std=c++17", "-Wall", "-pthread", *flags, "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "test_session_threads.cpp"), "-L", libdir,
                           "-lnkvmerkle", f"-Wl,-rpath,{libdir}", "-o", exe])
    out = subprocess.run([exe, str(tmp_path), "300" if sanitize else "3000"], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0 and out.stdout.startswith("ok") and "WARNING" not in out.stderr, \
        out.stdout + out.stderr[-3000:]


@pytest.mark.gpu
def test_cpp_mirror_on_gpu(tmp_path, oracle):
    exe = build_binary(str(tmp_path))
    out = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    kv = dict(line.split(" ", 1) for line in out.stdout.strip().splitlines())
    g = GOLDEN["readme"]
    assert kv["readme_root"] == g["root"]
    assert kv["readme_bfs"] == g["bfs_hex"]
    assert kv["readme_validate"] == "1"
    assert kv["readme_deser_root"] == g["root"] and kv["readme_deser_children"] == "0"
    assert kv["readme_deser_validate"] == "1"
    assert kv["empty_null"] == "1" and kv["empty_err"] == "cannot build Merkle Tree from 0 nodes"
    trees = {c["n"]: c for c in GOLDEN["trees"] if c["value_bytes"] in (64, 100)}
    for n in (1, 2, 3, 255, 256, 257, 1000, 1025):
        c = trees[n]
        assert kv[f"tree{n}_root"] == c["root"]
        assert int(kv[f"tree{n}_bfs_len"]) == c["bfs_len"]
        assert kv[f"tree{n}_bfs_head"] == c["bfs_head_hex"]
        assert kv[f"tree{n}_validate"] == "1"
    for n in (1, 2, 3, 255, 256, 257, 1000, 1025, 70001):
        assert kv[f"tree{n}_file_eq"] == "1"  # Serialize(file) == SerializeBytes()
    assert kv["mut_file_eq"] == "1"  # a smaller image after a larger one
    assert kv["tree1000_corrupt_validate"] == "0"
    # a tree New materializes on several threads (70001 leaves of 64 bytes)
    data = oracle.splitmix64_bytes(70001 * 64, 0x6E616B65 + 70001)
    want = oracle.tree_from_digests(oracle.leaf_hashes_strided(data, 64, 64, 70001, threads=8))
    assert kv["tree70001_root"] == want[-1].tobytes().hex() and kv["tree70001_validate"] == "1"
    img = open(os.path.join(str(tmp_path), "tree70001.img"), "rb").read()
    assert img == oracle.bfs_image(want, 70001) and int(kv["tree70001_bfs_len"]) == len(img)
    vals = [bytes([ord("a") + i]) * (7 * i) for i in range(10)]
    assert kv["early_leaf3"] == hashlib.sha1(vals[3]).hexdigest()
    want = oracle.tree_from_digests(np.frombuffer(b"".join(hashlib.sha1(v).digest() for v in vals), np.uint8))
    assert kv["early_root"] == want[-1].tobytes().hex()
    # flush after flush: one pinned arena, allocated by the first cycle only
    assert int(kv["flush0_allocs_total"]) >= 1
    assert kv["flush1_allocs_total"] == kv["flush0_allocs_total"] == kv["flush2_allocs_total"]
    for k in range(3):
        data = oracle.splitmix64_bytes(4096 * 512, 0xF1 + k)
        want = oracle.tree_from_digests(oracle.leaf_hashes_strided(data, 512, 512, 4096))
        assert kv[f"flush{k}_root"] == want[-1].tobytes().hex()
        assert kv[f"flush{k}_validate"] == "1" and kv[f"flush{k}_bad_root_validate"] == "0"
        assert kv[f"flush{k}_swapped_validate"] == "0"  # rehash over swapped children differs
    # Serialize walks the live tree: Data changed after New shows in the image
    # exactly as the literal restatement's walk writes it (merkletree.go:75-89)
    from oracle import merkle_ref as ref
    data = oracle.splitmix64_bytes(37 * 50, 0xAB)
    t = ref.New([ref.NewLeaf(data[50 * i:50 * i + 50].tobytes()) for i in range(37)])
    leaf = t.Root
    while leaf.Left is not None:
        leaf = leaf.Left
    leaf.Data = bytes([0xAB]) * 20
    d = t.Root.Right.Data
    t.Root.Right.Data = bytes([d[0] ^ 0xFF]) + bytes(d[1:])
    assert kv["mut_img"] == t.SerializeBytes().hex()
    # flushes past the 32 MiB stream chunk, streamed or not, aligned or odd value sizes
    # -- with NewLeaf's copies on the default pool, on the caller's thread, on 3 threads
    assert int(kv["default_copy_threads"]) >= 1
    for vlen in (4096, 1001):
        data = oracle.splitmix64_bytes(20000 * vlen, 0x5EED + vlen)
        want = oracle.tree_from_digests(oracle.leaf_hashes_strided(data, vlen, vlen, 20000, threads=8))
        for t in (-1, 0, 3):
            assert kv[f"big{vlen}_t{t}_s1_root"] == kv[f"big{vlen}_t{t}_s0_root"] == want[-1].tobytes().hex()
    data = oracle.splitmix64_bytes(5000 * 9000, 0xBAD)
    off = np.arange(9000, dtype=np.uint64) * 5000
    ln = (np.arange(9000, dtype=np.uint64) * 37) % 5000
    want = oracle.tree_from_digests(oracle.leaf_hashes(data, off, ln, threads=8))
    for t in (-1, 0, 3):
        assert kv[f"ragged_t{t}_root"] == want[-1].tobytes().hex()
        assert kv[f"ragged_t{t}_leaf77"] == want[77].tobytes().hex()
    # CompactRoots over a group of one GPU (RCCL) and of device 0 twice (copy)
    from nakevaleng_amd import record
    assert kv["group1_transport"] == "1"
    for t in range(5):
        stream = open(os.path.join(str(tmp_path), f"table{t}.bin"), "rb").read()
        rs = np.full(300 + 77 * t, 30 + 16 + 100 + 13 * t, np.uint64)
        off, ln = record.value_spans(stream, rs)
        want = oracle.tree_from_digests(oracle.leaf_hashes(np.frombuffer(stream, np.uint8), off, ln))
        assert kv[f"compact_g1_root{t}"] == kv[f"compact_g2_root{t}"] == want[-1].tobytes().hex()
        if "groupall_size" in kv:  # several GPUs: the group over all of them, /opt/rocm's RCCL
            assert kv["groupall_transport"] == "1"
            assert kv[f"compact_gall_root{t}"] == want[-1].tobytes().hex()
