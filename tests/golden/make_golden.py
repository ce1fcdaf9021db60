#!/usr/bin/env python3
"""Generate tests/golden/merkle_golden.json (committed) -- run in the build container.

Every expected value here comes from oracle/merkle_ref.py, the literal Python
restatement of the reference's ds/merkletree (pointer tree, recursive build,
queue BFS, root-only Deserialize) over hashlib SHA-1.  The reference is Go and
cannot run in this image, and it ships no fixtures for this package, so these
vectors pin our restatement, not the reference binary ("parity unpinned" at tree
level).  SHA-1 itself is pinned by the FIPS 180-4 vectors.

Inputs are not stored: they are regenerated from (seed, sizes) with the
splitmix64 byte stream defined in splitmix64_bytes() below.
"""
import hashlib
import json
import os
import struct
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import merkle_ref as mr  # noqa: E402

M64 = (1 << 64) - 1


def splitmix64_bytes(nbytes: int, seed: int) -> bytes:
    """byte j = byte (j % 8), little endian, of splitmix64(seed, j // 8)."""
    out = bytearray()
    k = 0
    while len(out) < nbytes:
        z = (seed + (k + 1) * 0x9E3779B97F4A7C15) & M64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        z ^= z >> 31
        out += struct.pack("<Q", z)
        k += 1
    return bytes(out[:nbytes])


FIPS = [  # FIPS 180-4 / NIST CSRC example vectors
    {"msg_hex": b"".hex(), "repeat": 1, "sha1": "da39a3ee5e6b4b0d3255bfef95601890afd80709"},
    {"msg_hex": b"abc".hex(), "repeat": 1, "sha1": "a9993e364706816aba3e25717850c26c9cd0d89d"},
    {"msg_hex": b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq".hex(), "repeat": 1,
     "sha1": "84983e441c3bd26ebaae4aa1f95129e5e54670f1"},
    {"msg_hex": b"a".hex(), "repeat": 1000000, "sha1": "34aa973cd4c4daa4f61eeb2bdbad27316534016f"},
]

EDGE_N = [1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 255, 256, 257, 1000, 1023, 1024, 1025]
EDGE_LENS = [0, 1, 19, 20, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 1024, 4050, 4096, 65536]


def tree_case(n: int, vlen: int, seed: int) -> dict:
    data = splitmix64_bytes(n * vlen, seed)
    leaves = [mr.NewLeaf(data[i * vlen:(i + 1) * vlen]) for i in range(n)]
    t = mr.New(leaves)
    img = t.SerializeBytes()
    levels = mr.levels_of(t)
    return {
        "n": n, "value_bytes": vlen, "seed": seed,
        "root": t.Root.String(),
        "leaf_digests_sha1": hashlib.sha1(b"".join(x.Data for x in leaves)).hexdigest(),
        "level_sizes_with_pads": [len(lv) for lv in levels],
        "bfs_len": len(img),
        "bfs_sha1": hashlib.sha1(img).hexdigest(),
        "bfs_head_hex": img[:64].hex(),
    }


def main():
    out = {"about": __doc__.strip().splitlines()[0], "fips": FIPS}
    # NewLeaf over every padding boundary
    out["leaf_lengths"] = [{"len": L, "seed": 1000 + L,
                            "sha1": hashlib.sha1(splitmix64_bytes(L, 1000 + L)).hexdigest()} for L in EDGE_LENS]
    out["trees"] = [tree_case(n, 64 if n > 300 else 100, 0x6E616B65 + n) for n in EDGE_N]
    out["trees"].append(tree_case(1024, 1024, 0x6E616B65))  # BASELINE configs[0]

    # README example (ds/merkletree/README.md:44-57): 7 raw one-byte leaves
    t = mr.New([mr.MerkleNode(str(i).encode()) for i in range(1, 8)])
    img = t.SerializeBytes()
    t2 = mr.MerkleTree()
    t2.DeserializeBytes(img)
    out["readme"] = {"leaves": [str(i) for i in range(1, 8)], "root": t.Root.String(),
                     "bfs_hex": img.hex(), "validate": t.Validate(),
                     "deserialized_root": t2.Root.String(), "deserialized_has_children":
                         t2.Root.Left is not None or t2.Root.Right is not None,
                     "deserialized_validate": t2.Validate()}
    t = mr.New([mr.NewLeaf(b"x")])
    out["single_x"] = {"root": t.Root.String(), "bfs_hex": t.SerializeBytes().hex()}

    # generic leaves of mixed Data length, including empty Data (serialized as 0x01)
    gens = []
    for n, seed in ((1, 5), (2, 6), (5, 7), (33, 8), (100, 9)):
        raw = splitmix64_bytes(4096, seed)
        lens = [(raw[i] % 45) if (raw[i] % 7) else 0 for i in range(n)]
        datas, p = [], 100
        for L in lens:
            datas.append(raw[p:p + L])
            p += L
        t = mr.New([mr.MerkleNode(d) for d in datas])
        img = t.SerializeBytes()
        gens.append({"n": n, "seed": seed, "lens": lens, "offset0": 100, "root": t.Root.String(),
                     "bfs_len": len(img), "bfs_sha1": hashlib.sha1(img).hexdigest()})
    out["generic"] = gens

    # a serialized Data table (record.go:191-199) with fixed timestamps
    recs, vals = [], []
    raw = splitmix64_bytes(1 << 16, 77)
    p = 0
    for i in range(50):
        ks, vs = 1 + raw[i] % 20, (raw[50 + i] * 7) % 300
        key, val = raw[p:p + ks], raw[p + ks:p + ks + vs]
        p += ks + vs
        crc = zlib.crc32(key + val) & 0xFFFFFFFF
        recs.append(struct.pack("<IqBBQQ", crc, 1700000000 + i, 0, 0, ks, vs) + key + val)
        vals.append(val)
    stream = b"".join(recs)
    t = mr.New([mr.NewLeaf(v) for v in vals])
    out["records"] = {"seed": 77, "n": 50, "key_size": "1 + raw[i] % 20", "value_size": "(raw[50+i]*7) % 300",
                      "timestamp": "1700000000 + i", "stream_len": len(stream),
                      "stream_sha1": hashlib.sha1(stream).hexdigest(), "rec_sizes": [len(r) for r in recs],
                      "root": t.Root.String(), "bfs_sha1": hashlib.sha1(t.SerializeBytes()).hexdigest()}
    with open(os.path.join(HERE, "merkle_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "merkle_golden.json"))


if __name__ == "__main__":
    main()
