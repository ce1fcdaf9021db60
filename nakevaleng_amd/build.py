"""Build libnkvmerkle.so in-tree (hipcc, gfx950).  Used by __graft_entry__.build().

The library embeds the SHA-256 of its sources, headers and compile flags
(nkv_build_id(), a string in .rodata).  build() compares it with the tree's
sources and recompiles on any mismatch, so a library that did not come from
these sources is never used -- on the GPU box as here (file times say nothing
once the tree has been copied).
"""
from __future__ import annotations

import hashlib
import os
import re
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
SO = os.path.join(PKG, "libnkvmerkle.so")
SOURCES = ["kernels.hip", "crc.hip", "bloom.hip", "capi.cpp", "group.cpp", "host_stage.cpp"]
HEADERS = ["internal.hpp", "context.hpp", "sha1_dev.hpp", "host_stage.hpp", "crc_dev.hpp"]
ARCH = os.environ.get("NKV_OFFLOAD_ARCH", "gfx950")
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread",
         "-Wall", "-Wno-unused-result"]
# RCCL for the multi-GPU group (nkv_group_*: ncclCommInitAll, ncclAllGather)
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
LIBS = [f"-L{ROCM}/lib", "-lrccl", "-lhsa-runtime64"]
_ID = re.compile(rb"nkv-src-sha256:([0-9a-f]{64})")


def source_hash(diag: bool = False) -> str:
    """SHA-256 over the compile flags and every source/header the library is built from."""
    h = hashlib.sha256()
    h.update(" ".join(FLAGS + LIBS + (["-DNKV_DIAG"] if diag else [])).encode())
    for path in [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "nkv_merkle.h")]:
        h.update(os.path.basename(path).encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def embedded_hash(so: str = SO):
    """The source hash compiled into `so` (None if absent or unreadable); no loading."""
    try:
        with open(so, "rb") as f:
            m = _ID.search(f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


DIAG_SO = os.path.join(PKG, "libnkvmerkle_diag.so")
last_status = ""  # what the latest build() did (printed by it, reported by the GPU tests)


def build(force: bool = False, verbose: bool = False, diag: bool = False, quiet: bool = False) -> str:
    """diag=True builds the stamp-instrumented library (tools/diag_timeline.py only)."""
    global last_status
    so = DIAG_SO if diag else SO
    want = source_hash(diag)
    have = embedded_hash(so)
    if not force and have == want:
        last_status = f"{os.path.basename(so)}: embedded source hash {want[:16]} matches the sources (no rebuild)"
        if not quiet:
            print(last_status, file=sys.stderr)
        return so
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = f"{so}.tmp{os.getpid()}"  # concurrent builders (ranks) never share a temp file
    cmd = [hipcc] + FLAGS + ["-I", os.path.join(ROOT, "include"), "-I", CSRC, f'-DNKV_SRC_HASH="{want}"']
    if diag:
        cmd.append("-DNKV_DIAG")
    cmd += [os.path.join(CSRC, f) for f in SOURCES] + LIBS + ["-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, so)
    if embedded_hash(so) != want:
        raise RuntimeError(f"{so}: the build did not embed source hash {want}")
    last_status = (f"{os.path.basename(so)}: rebuilt with hipcc --offload-arch={ARCH} "
                   f"(embedded hash was {have[:16] if have else 'none'}, sources {want[:16]})")
    if not quiet:
        print(last_status, file=sys.stderr)
    return so


API_FLUSH_SRC = os.path.join(ROOT, "tools", "api_flush.cpp")
API_FLUSH = os.path.join(ROOT, "build", "api_flush")


def build_tool(name: str) -> str:
    """tools/<name>.cpp over the C++ Go-API mirror -> build/<name> (g++, linked
    to the in-tree library; rebuilt when the source, the headers or the library
    are newer)."""
    build(quiet=True)
    src = os.path.join(ROOT, "tools", f"{name}.cpp")
    exe = os.path.join(ROOT, "build", name)
    deps = [src, SO] + [os.path.join(ROOT, "include", h) for h in ("nkv_merkle.h", "nkv_merkletree.hpp")]
    if os.path.exists(exe) and os.path.getmtime(exe) >= max(os.path.getmtime(d) for d in deps):
        return exe
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    tmp = f"{exe}.tmp{os.getpid()}"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "include"),
                           src, "-L", PKG, "-lnkvmerkle", "-Wl,-rpath,$ORIGIN/../nakevaleng_amd", "-o", tmp])
    os.replace(tmp, exe)
    return exe


def build_api_flush() -> str:
    """The end-to-end flush driver (tools/api_flush.cpp, bench.py --config api_flush)."""
    return build_tool("api_flush")


def build_small_flush() -> str:
    """The default-size flush driver (tools/small_flush.cpp, bench.py --config small_flush)."""
    return build_tool("small_flush")


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, diag="--diag" in sys.argv))
