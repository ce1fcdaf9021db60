"""CPU: pin the oracle (C restatement + literal Python restatement) before trusting it.

SHA-1 is pinned by FIPS 180-4 vectors; the tree layer by the committed golden
fixtures (tests/golden/make_golden.py) and by agreement of the two independent
restatements.  Parity at tree level is "unpinned" against the Go binary itself
(no Go toolchain, no reference fixtures) -- see DESIGN.md.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import merkle_ref as mr
from tests.golden.make_golden import splitmix64_bytes

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "merkle_golden.json")))


@pytest.mark.parametrize("kat", GOLDEN["fips"])
def test_fips_vectors_c_oracle(oracle, kat):
    msg = bytes.fromhex(kat["msg_hex"]) * kat["repeat"]
    assert oracle.sha1(msg).hex() == kat["sha1"]
    assert hashlib.sha1(msg).hexdigest() == kat["sha1"]


def test_splitmix64_generators_agree(oracle):
    for n, seed in ((0, 1), (1, 2), (7, 3), (8, 4), (1001, 0x6E616B65)):
        assert oracle.splitmix64_bytes(n, seed).tobytes() == splitmix64_bytes(n, seed)


@pytest.mark.parametrize("case", GOLDEN["leaf_lengths"], ids=lambda c: f"len{c['len']}")
def test_leaf_lengths(oracle, case):
    data = splitmix64_bytes(case["len"], case["seed"])
    assert oracle.sha1(data).hex() == case["sha1"]
    assert mr.NewLeaf(data).String() == case["sha1"]


@pytest.mark.parametrize("case", GOLDEN["trees"], ids=lambda c: f"n{c['n']}x{c['value_bytes']}")
def test_trees_c_oracle_vs_golden(oracle, case):
    n, vlen = case["n"], case["value_bytes"]
    data = np.frombuffer(splitmix64_bytes(n * vlen, case["seed"]), np.uint8)
    leaves = oracle.leaf_hashes_strided(data, vlen, vlen, n)
    assert hashlib.sha1(leaves.tobytes()).hexdigest() == case["leaf_digests_sha1"]
    nodes = oracle.tree_from_digests(leaves)
    assert nodes[-1].tobytes().hex() == case["root"]
    img = oracle.bfs_image(nodes, n)
    assert len(img) == case["bfs_len"] == oracle.bfs_size(n)
    assert hashlib.sha1(img).hexdigest() == case["bfs_sha1"]
    assert img[:64].hex() == case["bfs_head_hex"]
    # level shape: real nodes per level plus the pad of every odd level below the top
    sizes = case["level_sizes_with_pads"]  # top-down
    counts = [n]
    while len(counts) < 2 or counts[-1] > 1:
        counts.append((counts[-1] + 1) // 2)
    want = [c + (c & 1 if L < len(counts) - 1 else 0) for L, c in enumerate(counts)][::-1]
    assert sizes == want


def test_readme_example_literal_restatement():
    g = GOLDEN["readme"]
    t = mr.New([mr.MerkleNode(x.encode()) for x in g["leaves"]])
    assert t.Root.String() == g["root"] == "40bd4db4f1ae6c7d962b3edd605aea88549b8dcb"
    assert t.SerializeBytes().hex() == g["bfs_hex"]
    assert len(bytes.fromhex(g["bfs_hex"])) == 162
    assert t.Validate()


def test_generic_c_oracle_vs_golden(oracle):
    for g in GOLDEN["generic"]:
        raw = splitmix64_bytes(4096, g["seed"])
        off = np.cumsum([g["offset0"]] + g["lens"][:-1]).astype(np.uint64)
        lens = np.asarray(g["lens"], np.uint64)
        up = oracle.tree_generic(np.frombuffer(raw, np.uint8), off, lens)
        assert up[-1].tobytes().hex() == g["root"]


def test_deserialize_is_root_only():
    """merkletree.go:135-143 breaks before linking any child."""
    img = bytes.fromhex(GOLDEN["readme"]["bfs_hex"])
    t = mr.MerkleTree()
    t.DeserializeBytes(img)
    assert t.Root.String() == GOLDEN["readme"]["root"]
    assert t.Root.Left is None and t.Root.Right is None
    assert t.Validate()


def test_validate_detects_corrupted_leaf():
    t = mr.New([mr.NewLeaf(bytes([i])) for i in range(9)])
    assert t.Validate()
    leaf = t.Root
    while leaf.Left is not None:
        leaf = leaf.Left
    leaf.Data = bytes(20)
    assert not t.Validate()


def test_empty_tree_error_text():
    with pytest.raises(mr.MerkleTreeError, match="^cannot build Merkle Tree from 0 nodes$"):
        mr.New([])


def test_literal_restatement_matches_c_oracle_random(oracle):
    rng = np.random.default_rng(3)
    for n in (1, 2, 3, 6, 31, 64, 129):
        lens = rng.integers(0, 300, n).astype(np.uint64)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(lens[:-1])
        data = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
        t = mr.New([mr.NewLeaf(data[int(o):int(o + l)].tobytes()) for o, l in zip(off, lens)])
        nodes = oracle.tree_from_digests(oracle.leaf_hashes(data, off, lens))
        assert nodes[-1].tobytes() == t.Root.Data
        assert oracle.bfs_image(nodes, n) == t.SerializeBytes()


# --- record checksum: CRC-32/IEEE over key ++ value ---

def test_crc32_published_check_value(oracle):
    # ISO-HDLC / Go crc32.ChecksumIEEE check value
    assert oracle.crc32(b"123456789") == 0xCBF43926
    assert oracle.crc32(b"") == 0


def test_crc32_matches_zlib(oracle):
    import zlib
    rng = np.random.default_rng(11)
    for n in (1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 65, 255, 4066, 10000):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.crc32(d) == zlib.crc32(d)


def test_record_crcs_on_serialized_stream(oracle):
    from nakevaleng_amd import record
    rng = np.random.default_rng(12)
    recs = [record.New(rng.integers(0, 256, int(k), dtype=np.uint8).tobytes(),
                       rng.integers(0, 256, int(v), dtype=np.uint8).tobytes(), timestamp=7)
            for k, v in zip(rng.integers(0, 40, 50), rng.integers(0, 3000, 50))]
    recs.append(record.New(b"", b"", timestamp=7))
    stream, sizes = record.data_table(recs)
    off = np.zeros(len(recs), np.uint64)
    off[1:] = np.cumsum(sizes[:-1])
    buf = np.frombuffer(stream, np.uint8).copy()
    crc, ok, bad = oracle.record_crcs(buf, off)
    assert bad == 0 and ok.all()
    assert [int(c) for c in crc] == [r.Crc for r in recs]
    buf[int(off[3]) + 30] ^= 1  # corrupt record 3's first key byte
    crc2, ok2, bad2 = oracle.record_crcs(buf, off)
    assert bad2 == 1 and not ok2[3] and ok2[[i for i in range(len(recs)) if i != 3]].all()


def test_fast_crc_forms_match_zlib(oracle):
    """The CPU baseline's CRC-32 forms (slicing-by-8; PCLMULQDQ folding, as Go's
    hash/crc32 on amd64) against zlib and the bitwise checker, every length
    around the folding loop's 16/64-byte steps and every start alignment."""
    import zlib
    rng = np.random.default_rng(13)
    big = rng.integers(0, 256, 70000, dtype=np.uint8)
    for n in list(range(0, 200)) + [255, 256, 257, 1023, 4066, 4096, 65536, 65599]:
        for a in (0, 1, 7) if n < 200 else range(16):
            d = big[a:a + n]
            want = zlib.crc32(d.tobytes())
            assert oracle.crc32_fast(d, clmul=False) == want
            assert oracle.crc32_fast(d, clmul=True) == want
    assert oracle.crc32_fast(b"123456789", clmul=True) == 0xCBF43926


def test_verify_records_cpu_baseline(oracle):
    """nkvo_seal_records / nkvo_verify_records (bench.py's records_verify CPU
    baseline): the sealed Crcs are the bitwise checker's, the digests are the
    leaf oracle's for every variant and thread count, and one flipped key byte
    is counted once."""
    rng = np.random.default_rng(14)
    ks = rng.integers(0, 40, 300).astype(np.uint64)
    vs = rng.integers(0, 5000, 300).astype(np.uint64)
    sizes = 30 + ks + vs
    off = np.zeros(300, np.uint64)
    off[1:] = np.cumsum(sizes[:-1])
    stream = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8)
    for i in range(300):
        o = int(off[i])
        stream[o + 14:o + 22] = np.frombuffer(np.uint64(ks[i]).tobytes(), np.uint8)
        stream[o + 22:o + 30] = np.frombuffer(np.uint64(vs[i]).tobytes(), np.uint8)
    oracle.seal_records(stream, off, 3)
    _, ok, bad = oracle.record_crcs(stream, off)
    assert bad == 0 and ok.all()
    want = oracle.leaf_hashes(stream, off + 30 + ks, vs)
    for ossl in (False, True):
        for t in (1, 4):
            d, b = oracle.verify_records(stream, off, threads=t, openssl=ossl)
            assert b == 0 and np.array_equal(d, want)
    stream[int(off[7]) + 30 + 0] ^= 1 if ks[7] + vs[7] else 0
    if ks[7] + vs[7]:
        assert oracle.verify_records(stream, off, threads=2, openssl=True)[1] == 1


# --- SSTable filter: murmur3 Bloom inserts ---

MURMUR3_VECTORS = [  # published MurmurHash3_x86_32 vectors (input, seed, hash)
    (b"", 0, 0x00000000), (b"", 1, 0x514E28B7), (b"", 0xFFFFFFFF, 0x81F16F39),
    (b"\x00\x00\x00\x00", 0, 0x2362F9DE), (b"\xff\xff\xff\xff", 0, 0x76293B50),
    (b"\x21\x43\x65\x87", 0, 0xF55B516B), (b"\x21\x43\x65\x87", 0x5082EDEE, 0x2362F9DE),
    (b"\x21\x43\x65", 0, 0x7E4A8634), (b"\x21\x43", 0, 0xA0F7B07A), (b"\x21", 0, 0x72661CF4),
    (b"aaaa", 0x9747B28C, 0x5A97808A), (b"Hello, world!", 0x9747B28C, 0x24884CBA),
    (b"The quick brown fox jumps over the lazy dog", 0x9747B28C, 0x2FA826CD),
]


@pytest.mark.parametrize("data,seed,want", MURMUR3_VECTORS)
def test_murmur3_published_vectors(oracle, data, seed, want):
    assert oracle.murmur3_32(data, seed) == want


def test_murmur3_matches_sklearn(oracle):
    from sklearn.utils import murmurhash3_32
    rng = np.random.default_rng(13)
    for n in list(range(0, 40)) + [100, 1000]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        seed = int(rng.integers(0, 2**32))
        assert oracle.murmur3_32(d, seed) == murmurhash3_32(d, seed=seed, positive=True)


def test_bloom_params_match_reference_formula(oracle):
    import math
    for n in (1, 2, 10, 100, 1000, 12345, 1 << 20):
        for p in (0.01, 0.1, 0.2, 0.001):
            m = math.ceil(n * abs(math.log(p)) / math.pow(math.log(2), 2))
            k = math.ceil((m / n) * math.log(2))
            assert oracle.bloom_params(n, p) == (m, k)
    assert oracle.bloom_params(1 << 20, 0.01) == (10050663, 7)


def test_bloom_insert_then_query(oracle):
    rng = np.random.default_rng(14)
    n = 2000
    ln = rng.integers(0, 40, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1])
    keys = rng.integers(0, 256, int(ln.sum()) + 1, dtype=np.uint8)
    m, k = oracle.bloom_params(n, 0.01)
    bits = oracle.bloom_insert(keys, off, ln, m, k, 12345)
    assert oracle.bloom_query(keys, off, ln, m, k, 12345, bits).all()  # no false negatives
    # the reference's bit numbering: Contents[idx / 8] |= 1 << (idx % 8)
    idx = oracle.murmur3_32(keys[int(off[0]):int(off[0] + ln[0])], 12345) % m
    assert bits[idx // 8] >> (idx % 8) & 1
    other = rng.integers(0, 256, 64 * 1000, dtype=np.uint8)
    qoff = np.arange(1000, dtype=np.uint64) * 64
    fp = oracle.bloom_query(other, qoff, np.full(1000, 64, np.uint64), m, k, 12345, bits).mean()
    assert fp < 0.05


def test_openssl_variant_kats_and_trees(oracle):
    """The CPU baseline's OpenSSL variant (oracle/merkle_openssl.c): FIPS 180-4
    known answers, and the same leaves and trees as the portable restatement on
    ragged values, one thread and several (wide levels split over threads)."""
    kats = {b"": "da39a3ee5e6b4b0d3255bfef95601890afd80709",
            b"abc": "a9993e364706816aba3e25717850c26c9cd0d89d",
            b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq": "84983e441c3bd26ebaae4aa1f95129e5e54670f1"}
    for m, want in kats.items():
        assert oracle.ossl_sha1(m).hex() == want
    assert oracle.ossl_sha1(b"a" * 1000000).hex() == "34aa973cd4c4daa4f61eeb2bdbad27316534016f"
    rng = np.random.default_rng(17)
    for n in (1, 2, 3, 7, 1000, 9001):
        ln = rng.integers(0, 300, n).astype(np.uint64)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(ln[:-1])
        base = np.frombuffer(rng.bytes(int(ln.sum()) + 1), np.uint8).copy()
        want = oracle.tree_from_digests(oracle.leaf_hashes(base, off, ln))
        for t in (1, 4):
            got = oracle.ossl_tree_from_digests(oracle.ossl_leaf_hashes(base, off, ln, threads=t), threads=t)
            assert np.array_equal(got, want), (n, t)
            assert np.array_equal(oracle.tree_from_digests(oracle.leaf_hashes(base, off, ln, threads=t), threads=t),
                                  want)
    data = oracle.splitmix64_bytes(5000 * 64, 3)
    assert np.array_equal(oracle.ossl_leaf_hashes_strided(data, 64, 64, 5000, threads=3),
                          oracle.leaf_hashes_strided(data, 64, 64, 5000))


def test_flush_reps_matches_the_tree(oracle):
    """nkvo_flush_reps (small_flush's one-core CPU column) builds the same root
    with either SHA-1."""
    rng = np.random.default_rng(5)
    for n in (1, 10, 40, 1025):
        ln = rng.integers(1, 200, n).astype(np.uint64)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(ln[:-1])
        base = np.frombuffer(rng.bytes(int(ln.sum()) + 1), np.uint8).copy()
        want = oracle.tree_from_digests(oracle.leaf_hashes(base, off, ln))[-1].tobytes().hex()
        for ossl in (False, True):
            us, root = oracle.flush_us(base, off, ln, 3, openssl=ossl)
            assert root == want and us > 0
