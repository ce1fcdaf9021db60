"""ds/bloomfilter-shaped mirror over the device filter build.

Reference: ds/bloomfilter/bloomfilter.go.  New(expectedElements,
falsePositiveRate) sizes M and K (:18-24, :54-74); hash j of an element is
murmur3.Sum32WithSeed(element, seed_j) % M with seeds t, t+1, .. (:28-39);
Insert sets Contents[idx / 8] |= 1 << (idx % 8) (:76-91); Query tests every bit
(:93-111).  Inserts are deferred and hashed in one device batch when the
filter is next read (Query, Contents, EncodeToDict) -- the same batching the
Merkle mirror does for NewLeaf.  Gob encoding (EncodeToFile/Bytes) is host
serialization and out of scope; EncodeToDict gives its fields.
"""
from __future__ import annotations

import ctypes
import time
from typing import List, Optional, Sequence

import numpy as np

from nakevaleng_amd import _lib


class BloomFilterError(ValueError):
    pass


def params(expected_elements: int, false_positive_rate: float):
    """(M, K) as calculateM / calculateK (bloomfilter.go:18-24)."""
    m, k = ctypes.c_uint32(0), ctypes.c_uint32(0)
    _lib.check(_lib.lib().nkv_bloom_params(expected_elements, false_positive_rate, ctypes.byref(m),
                                           ctypes.byref(k)))
    return m.value, k.value


def _pack(elements: Sequence[bytes]):
    lens = np.fromiter((len(e) for e in elements), dtype=np.uint64, count=len(elements))
    off = np.zeros(len(elements), np.uint64)
    if len(elements) > 1:
        off[1:] = np.cumsum(lens[:-1])
    data = np.frombuffer(b"".join(bytes(e) for e in elements) or b"\0", np.uint8)
    return data, off, lens


class BloomFilter:
    def __init__(self, M: int, K: int, HashSeeds: List[int], Contents: Optional[bytes] = None, ctx=None):
        self.M, self.K, self.HashSeeds = M, K, list(HashSeeds)
        if any(s != (self.HashSeeds[0] + j) & 0xFFFFFFFF for j, s in enumerate(self.HashSeeds)):
            raise BloomFilterError("HashSeeds must be consecutive (createHashFunctions, bloomfilter.go:31-36)")
        self._contents = bytearray(Contents) if Contents is not None else bytearray((M + 7) // 8)
        self._pending: List[bytes] = []
        self._ctx = ctx

    @property
    def _seed0(self) -> int:
        return self.HashSeeds[0] if self.HashSeeds else 0

    def _flush(self):
        if not self._pending:
            return
        ctx = self._ctx or _lib.default_context()
        data, off, lens = _pack(self._pending)
        bits = np.zeros((self.M + 7) // 8, np.uint8)
        _lib.check(_lib.lib().nkv_bloom_build(ctx.h, _lib.p8(data), _lib.p64(off), _lib.p64(lens), len(self._pending),
                                              self.M, self.K, self._seed0, _lib.p8(bits)))
        cur = np.frombuffer(self._contents, np.uint8)
        self._contents = bytearray((cur | bits).tobytes())
        self._pending.clear()

    def Insert(self, element: bytes) -> None:  # bloomfilter.go:76-91
        self._pending.append(bytes(element))

    def InsertMany(self, elements: Sequence[bytes]) -> None:
        self._pending.extend(bytes(e) for e in elements)

    @property
    def Contents(self) -> bytes:
        self._flush()
        return bytes(self._contents)

    def QueryMany(self, elements: Sequence[bytes]) -> np.ndarray:
        """Query (bloomfilter.go:93-111) for a batch, on the context's device.

        The inputs go to that device and the launch uses its current torch
        stream; the context's previous stream is restored afterwards."""
        import torch
        self._flush()
        if not elements:
            return np.zeros(0, bool)
        ctx = self._ctx or _lib.default_context()
        dev = torch.device("cuda", ctx.device)
        data, off, lens = _pack(elements)
        words = np.zeros(((self.M + 31) // 32) * 4, np.uint8)
        words[:len(self._contents)] = np.frombuffer(self._contents, np.uint8)
        d = [torch.from_numpy(a.view(np.uint8).copy()).to(dev) for a in (data, off, lens, words)]
        out = torch.zeros(len(elements), dtype=torch.uint8, device=dev)
        stream = torch.cuda.current_stream(dev)
        with ctx.on_stream(stream.cuda_stream):
            _lib.check(_lib.lib().nkv_bloom_query_dev(ctx.h, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                                      len(elements), self.M, self.K, self._seed0,
                                                      d[3].data_ptr(), out.data_ptr()))
        stream.synchronize()
        return out.cpu().numpy().astype(bool)

    def Query(self, element: bytes) -> bool:
        return bool(self.QueryMany([element])[0])

    def EncodeToDict(self) -> dict:
        return {"M": self.M, "K": self.K, "HashSeeds": list(self.HashSeeds), "Contents": self.Contents}


def New(expected_elements: int, false_positive_rate: float, seed: Optional[int] = None, ctx=None) -> BloomFilter:
    """bloomfilter.New (bloomfilter.go:54-74); seed defaults to
    uint32(time.Now().UnixNano()) like createHashFunctions."""
    if expected_elements < 0:
        raise BloomFilterError(
            f"expectedElements must be greater than or equal to zero, but {expected_elements} was given")
    if false_positive_rate < 0.0 or false_positive_rate > 1.0:
        raise BloomFilterError(f"falsePositiveRate must be between (0, 1), but {false_positive_rate:f} was given")
    m, k = params(expected_elements, false_positive_rate)
    t = (time.time_ns() if seed is None else seed) & 0xFFFFFFFF
    return BloomFilter(m, k, [(t + i) & 0xFFFFFFFF for i in range(k)], ctx=ctx)
