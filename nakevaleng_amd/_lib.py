"""ctypes binding of libnkvmerkle.so (the C-ABI in include/nkv_merkle.h).

The product path has no CPU fallback: if the HIP library is missing, or no
device is usable, every call raises.  Loading the library does not touch the GPU.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
SO_PATH = os.environ.get("NKV_LIB", os.path.join(_PKG, "libnkvmerkle.so"))

NKV_OK = 0
NKV_ERR_EMPTY = 1
NKV_ERR_INVALID = 2
NKV_ERR_DEVICE = 3
NKV_ERR_NOMEM = 4
NKV_ERR_IO = 5
NKV_OPT_LEAF_LOAD = 1
NKV_OPT_BUCKET = 2
NKV_OPT_QUEUE_SPLIT = 4
NKV_OPT_QUEUE_WAVES = 5
NKV_OPT_CRC_LOAD = 6
NKV_OPT_HOST_THREADS = 7
NKV_OPT_STAGE_CHUNK = 8
NKV_OPT_BLOOM_PATH = 10
NKV_OPT_RECORDS_FUSED = 11
NKV_OPT_TABLE_LANES = 12
NKV_OPT_TIMING_EVERY = 13
NKV_OPT_SMALL_PATH = 14
NKV_OPT_SMALL_MAX_N = 15
NKV_OPT_SMALL_MAX_BYTES = 16
NKV_OPT_ARENA_COHERENT = 17
NKV_OPT_SIDE_GATE = 18
NKV_OPT_QUEUE_PAIR = 19  # retired: accepts only 0
NKV_OPT_SERVICE_MAILBOX = 20
NKV_PATH_GRID = 0
NKV_PATH_SMALL = 1
NKV_OPT_DEEP_PREFETCH = 3  # retired: accepts only 3
NKV_OPT_QUEUE_RING = 9  # retired: accepts only 13
NKV_ABI_VERSION = 1  # include/nkv_merkle.h
NKV_TIMING_EVENTS = 1
NKV_TIMING_CLOCK = 2
NKV_TABLE_STRIDED = 0
NKV_TABLE_VALUES = 1
NKV_TABLE_RECORDS = 2
NKV_TABLE_VERIFY = 3
NKV_TRANSPORT_RCCL = 1
NKV_TRANSPORT_COPY = 2
NKV_PEER_NONE = 0
NKV_PEER_ENABLED = 1
NKV_PEER_SAME = 2

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64
_int = ctypes.c_int

class NkvTable(ctypes.Structure):
    """struct nkv_table (include/nkv_merkle.h): one table of device-resident leaves."""
    _fields_ = [("kind", _int), ("base", _vp), ("base_len", _u64), ("stride", _u64), ("len", _u64),
                ("off", _vp), ("lens", _vp), ("n", _u64), ("nodes", _vp), ("err", _vp), ("crc", _vp),
                ("stats", _vp)]


class NkvValues(ctypes.Structure):
    """struct nkv_values: one table of host values (nkv_group_trees_from_values)."""
    _fields_ = [("base", _vp), ("off", _vp), ("len", _vp), ("n", _u64), ("root20", _vp), ("nodes_out", _vp),
                ("img_out", _vp)]


_tabp = ctypes.POINTER(NkvTable)

# name -> (restype, argtypes); every symbol include/nkv_merkle.h declares
SIGNATURES = {
    "nkv_abi_version": (_int, []),
    "nkv_strerror": (ctypes.c_char_p, [_int]),
    "nkv_build_id": (ctypes.c_char_p, []),
    "nkv_device_count": (_int, [ctypes.POINTER(_int)]),
    "nkv_ctx_create": (_int, [_int, ctypes.POINTER(_vp)]),
    "nkv_ctx_destroy": (None, [_vp]),
    "nkv_ctx_set_stream": (_int, [_vp, _vp]),
    "nkv_ctx_use_own_stream": (_int, [_vp]),
    "nkv_ctx_sync": (_int, [_vp]),
    "nkv_ctx_last_path": (_int, [_vp, ctypes.POINTER(_int)]),
    "nkv_ctx_small_service_state": (_int, [_vp, ctypes.POINTER(ctypes.c_uint64)]),
    "nkv_ctx_small_service_trace": (_int, [_vp, _int, ctypes.POINTER(ctypes.c_uint64)]),
    "nkv_ctx_set_option": (_int, [_vp, _int, ctypes.c_int64]),
    "nkv_ctx_set_timing": (_int, [_vp, _int]),
    "nkv_ctx_last_timing": (_int, [_vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
    "nkv_ctx_timing_summary": (_int, [_vp, ctypes.POINTER(_int), ctypes.POINTER(ctypes.c_float),
                                      ctypes.POINTER(ctypes.c_float)]),
    "nkv_num_levels": (_int, [_u64]),
    "nkv_level_count": (_u64, [_u64, _int]),
    "nkv_level_start": (_u64, [_u64, _int]),
    "nkv_total_nodes": (_u64, [_u64]),
    "nkv_bfs_size": (_u64, [_u64]),
    "nkv_host_alloc": (_int, [_vp, _u64, ctypes.POINTER(_vp)]),
    "nkv_host_free": (_int, [_vp, _vp]),
    "nkv_leaf_hash": (_int, [_vp, _u8p, _u64p, _u64p, _u64, _u8p]),
    "nkv_tree_build": (_int, [_vp, _u8p, _u64, _u8p, _u8p, _u8p]),
    "nkv_tree_from_values": (_int, [_vp, _u8p, _u64p, _u64p, _u64, _u8p, _u8p, _u8p]),
    "nkv_generic_bfs_size": (_u64, [_u64p, _u64]),
    "nkv_tree_generic": (_int, [_vp, _u8p, _u64p, _u64p, _u64, _u8p, _u8p, _u8p]),
    "nkv_tree_validate": (_int, [_vp, _u8p, _u64p, _u64p, _u64, _u8p, ctypes.POINTER(_int)]),
    "nkv_tree_from_records": (_int, [_vp, _u8p, _u64, _u64p, _u64, _u8p, _u8p, _u8p]),
    "nkv_record_crc": (_int, [_vp, _u8p, _u64, _u64p, _u64, ctypes.POINTER(ctypes.c_uint32), _u64p, _u64p]),
    "nkv_bloom_params": (_int, [_u64, ctypes.c_double, ctypes.POINTER(ctypes.c_uint32),
                                ctypes.POINTER(ctypes.c_uint32)]),
    "nkv_bloom_build": (_int, [_vp, _u8p, _u64p, _u64p, _u64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                               _u8p]),
    "nkv_bloom_from_records": (_int, [_vp, _u8p, _u64, _u64p, _u64, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32, _u8p]),
    "nkv_write_file": (_int, [ctypes.c_char_p, _u8p, _u64]),
    "nkv_leaf_hash_dev": (_int, [_vp, _vp, _vp, _vp, _u64, _vp]),
    "nkv_leaf_hash_strided_dev": (_int, [_vp, _vp, _u64, _u64, _u64, _vp]),
    "nkv_tree_reduce_dev": (_int, [_vp, _vp, _u64]),
    "nkv_tree_from_values_dev": (_int, [_vp, _vp, _vp, _vp, _u64, _vp]),
    "nkv_tree_from_strided_dev": (_int, [_vp, _vp, _u64, _u64, _u64, _vp]),
    "nkv_bfs_image_dev": (_int, [_vp, _vp, _u64, _vp]),
    "nkv_record_offsets_dev": (_int, [_vp, _vp, _u64, _vp]),
    "nkv_locate_values_dev": (_int, [_vp, _vp, _u64, _vp, _u64, _vp, _vp]),
    "nkv_tree_from_records_dev": (_int, [_vp, _vp, _u64, _vp, _u64, _vp, _vp]),
    "nkv_crc32_dev": (_int, [_vp, _vp, _vp, _vp, _u64, _vp]),
    "nkv_record_crc_dev": (_int, [_vp, _vp, _u64, _vp, _u64, _vp, _vp]),
    "nkv_tree_verify_records_dev": (_int, [_vp, _vp, _u64, _vp, _u64, _vp, _vp, _vp]),
    "nkv_bloom_insert_dev": (_int, [_vp, _vp, _vp, _vp, _u64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                    _vp]),
    "nkv_bloom_insert_records_dev": (_int, [_vp, _vp, _u64, _vp, _u64, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, _vp]),
    "nkv_bloom_query_dev": (_int, [_vp, _vp, _vp, _vp, _u64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                   _vp, _vp]),
    "nkv_fill_splitmix64_dev": (_int, [_vp, _vp, _u64, _u64]),
    "nkv_ctx_clock": (_int, [_vp, ctypes.POINTER(ctypes.c_double), _u64p]),
    "nkv_ctx_last_host_timing": (_int, [_vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                        ctypes.POINTER(ctypes.c_float)]),
    "nkv_host_stream": (_int, [_vp, _vp, _u64]),
    "nkv_trees_dev": (_int, [_vp, _tabp, _int]),
    "nkv_group_create": (_int, [ctypes.POINTER(_int), _int, ctypes.POINTER(_vp)]),
    "nkv_group_destroy": (None, [_vp]),
    "nkv_group_size": (_int, [_vp]),
    "nkv_group_transport": (_int, [_vp]),
    "nkv_group_peer_access": (_int, [_vp, _int, _int, ctypes.POINTER(_int)]),
    "nkv_group_ctx": (_int, [_vp, _int, ctypes.POINTER(_vp)]),
    "nkv_group_sync": (_int, [_vp]),
    "nkv_group_roots_allgather": (_int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _u8p]),
    "nkv_group_trees_dev": (_int, [_vp, _tabp, _int, _u8p]),
    "nkv_group_trees_from_values": (_int, [_vp, ctypes.POINTER(NkvValues), _int]),
    "nkv_split_span": (_u64, [_u64, _int]),
    "nkv_group_tree_from_values": (_int, [_vp, _u8p, _u64p, _u64p, _u64, _u8p, _u8p, _u8p]),
    "nkv_group_tree_dev": (_int, [_vp, _tabp, _u64, ctypes.POINTER(_vp), _u8p]),
    "nkv_group_tree_fetch": (_int, [_vp, _u8p, _u8p]),
}

_lib = None
_OWN = object()  # Context.stream sentinel: the context's own stream


class NkvError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = lib().nkv_strerror(code).decode()
        super().__init__(f"{what}: {msg}" if what else msg)


def lib():
    """Load libnkvmerkle.so; raise loudly if it has not been built."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch wheels bundle their own
        # libamdhip64.so.7.  Importing torch first makes our DT_NEEDED
        # libamdhip64.so.7 bind to that already-loaded copy (same SONAME), so
        # device pointers and streams are shared with torch.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(SO_PATH):
            raise ImportError(
                f"{SO_PATH} is missing: build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()')")
        L = ctypes.CDLL(SO_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.nkv_abi_version() != NKV_ABI_VERSION:
            raise ImportError(f"{SO_PATH} implements C-ABI version {L.nkv_abi_version()}, "
                              f"this binding needs {NKV_ABI_VERSION}")
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != NKV_OK:
        raise NkvError(rc, what)


def p8(a: Optional[np.ndarray]):
    if a is None:
        return None
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_u8p)


def p64(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_u64p)


def device_count() -> int:
    c = _int(0)
    rc = lib().nkv_device_count(ctypes.byref(c))
    return c.value if rc == NKV_OK else 0


class Context:
    """One nkv_ctx: a device, a stream, device scratch and pinned staging."""

    def __init__(self, device: int = 0):
        h = _vp()
        check(lib().nkv_ctx_create(device, ctypes.byref(h)), f"nkv_ctx_create(device={device})")
        self.h = h
        self.device = device
        self.stream = _OWN  # the context's own stream until set_stream
        self.owned = True

    @classmethod
    def borrow(cls, handle, device: int) -> "Context":
        """A view of a context someone else owns (a group member): close() does not destroy it."""
        c = cls.__new__(cls)
        c.h, c.device, c.stream, c.owned = handle, device, _OWN, False
        return c

    def close(self) -> None:
        if getattr(self, "h", None):
            if getattr(self, "owned", True):
                lib().nkv_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_stream(self, stream_handle) -> None:
        """Launch on `stream_handle` (a hipStream_t as int, None = the null stream,
        _OWN = the context's own stream)."""
        if stream_handle is _OWN:
            check(lib().nkv_ctx_use_own_stream(self.h))
        else:
            check(lib().nkv_ctx_set_stream(self.h, stream_handle))
        self.stream = stream_handle

    def on_stream(self, stream_handle):
        """Context manager: launch on `stream_handle` inside the block, then restore."""
        ctx = self

        class _On:
            def __enter__(self_):
                self_.prev = ctx.stream
                ctx.set_stream(stream_handle)
                return ctx

            def __exit__(self_, *exc):
                ctx.set_stream(self_.prev)

        return _On()

    def set_option(self, key: int, value: int) -> None:
        check(lib().nkv_ctx_set_option(self.h, key, value), f"nkv_ctx_set_option({key}, {value})")

    def sync(self) -> None:
        check(lib().nkv_ctx_sync(self.h))

    def last_path(self) -> int:
        """NKV_PATH_* of the latest host-buffer tree call (small one-launch or grid)."""
        p = _int()
        check(lib().nkv_ctx_last_path(self.h, ctypes.byref(p)))
        return p.value

    def small_service_state(self) -> dict:
        """The resident small-tree service's mailbox and launch state (diagnostics)."""
        a = (ctypes.c_uint64 * 8)()
        check(lib().nkv_ctx_small_service_state(self.h, a))
        d = dict(zip(("doorbell", "served", "done", "launches", "live", "busy", "mailbox_dev"), list(a)))
        hw, d["xcc"] = a[7] & 0xFFFFFFFF, a[7] >> 32
        # HW_REG_HW_ID fields (gfx9): wave [3:0], SIMD [5:4], CU [11:8], SH [12], SE [15:13]
        d["simd"], d["cu"], d["sh"], d["se"] = (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7
        return d

    def small_service_trace(self, enable: bool) -> list:
        """Turn the service's phase stamps on/off; returns the latest traced request's
        seven (s_memrealtime, s_memtime) pairs (nkv_merkle.h)."""
        a = (ctypes.c_uint64 * 14)()
        check(lib().nkv_ctx_small_service_trace(self.h, 1 if enable else 0, a))
        return list(a)

    def set_timing(self, on, clock: bool = False) -> None:
        """Events around the leaf kernel / reduce (on) and the leaf kernels' clock probe (clock)."""
        flags = (NKV_TIMING_EVENTS if on else 0) | (NKV_TIMING_CLOCK if clock else 0)
        check(lib().nkv_ctx_set_timing(self.h, flags))

    def clock(self):
        """(MHz, waves): lifetime-weighted shader clock of the leaf-kernel waves since set_timing(clock=True)."""
        mhz, waves = ctypes.c_double(), _u64()
        check(lib().nkv_ctx_clock(self.h, ctypes.byref(mhz), ctypes.byref(waves)))
        return mhz.value, waves.value

    def trees(self, tables) -> None:
        """nkv_trees_dev over a list of NkvTable (asynchronous on the context's stream)."""
        arr = (NkvTable * len(tables))(*tables)
        check(lib().nkv_trees_dev(self.h, arr, len(tables)), "nkv_trees_dev")

    def timing_summary(self):
        """(calls, leaf_ms_total, reduce_ms_total) since set_timing(True)."""
        k, a, b = _int(), ctypes.c_float(), ctypes.c_float()
        check(lib().nkv_ctx_timing_summary(self.h, ctypes.byref(k), ctypes.byref(a), ctypes.byref(b)))
        return k.value, a.value, b.value

    def last_timing(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        check(lib().nkv_ctx_last_timing(self.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value


def table(kind: int, nodes: int, n: int, base: int = 0, base_len: int = 0, stride: int = 0, length: int = 0,
          off: int = 0, lens: int = 0, err: int = 0, crc: int = 0, stats: int = 0) -> NkvTable:
    """An nkv_table from device addresses (ints, 0 = NULL)."""
    return NkvTable(kind, base or None, base_len, stride, length, off or None, lens or None, n, nodes or None,
                    err or None, crc or None, stats or None)


class Group:
    """One host process over several GPUs (nkv_group_*): a context per listed
    device and one RCCL communicator (copy transport if a device repeats)."""

    def __init__(self, devices):
        devs = (_int * len(devices))(*devices)
        h = _vp()
        check(lib().nkv_group_create(devs, len(devices), ctypes.byref(h)), f"nkv_group_create({list(devices)})")
        self.h = h
        self.devices = list(devices)

    @property
    def size(self) -> int:
        return lib().nkv_group_size(self.h)

    @property
    def transport(self) -> int:
        return lib().nkv_group_transport(self.h)

    def peer_access(self, i: int, j: int) -> int:
        """NKV_PEER_* between member i's GPU and member j's."""
        s = _int()
        check(lib().nkv_group_peer_access(self.h, i, j, ctypes.byref(s)))
        return s.value

    def ctx_handle(self, i: int):
        out = _vp()
        check(lib().nkv_group_ctx(self.h, i, ctypes.byref(out)))
        return out

    def ctx(self, i: int) -> Context:
        """Member i's context (owned by the group)."""
        return Context.borrow(self.ctx_handle(i), self.devices[i])

    def sync(self) -> None:
        check(lib().nkv_group_sync(self.h))

    def close(self) -> None:
        if getattr(self, "h", None):
            lib().nkv_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


_default: dict = {}


def current_device() -> int:
    """The device this process works on, one rule for every caller
    (lsmtree.rank_device, the mirrors' default contexts): the launcher's
    LOCAL_RANK modulo the visible devices (one process per GPU), else the
    device torch already works on if this process initialised torch's GPU
    state, else 0.  It never initialises torch's GPU runtime itself."""
    local = os.environ.get("LOCAL_RANK")
    if local is not None:
        cnt = device_count()
        return int(local) % cnt if cnt else int(local)
    import sys
    torch = sys.modules.get("torch")
    if torch is not None:
        try:
            if torch.cuda.is_initialized():
                return int(torch.cuda.current_device())
        except Exception:
            pass
    return 0


def default_context(device: Optional[int] = None) -> Context:
    """One shared context per device; device None = current_device()."""
    if device is None:
        device = current_device()
    ctx = _default.get(device)
    if ctx is None:
        ctx = _default[device] = Context(device)
    return ctx
