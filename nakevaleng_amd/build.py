"""Build libnkvmerkle.so in-tree (hipcc, gfx950).  Used by __graft_entry__.build()."""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
SO = os.path.join(PKG, "libnkvmerkle.so")
SOURCES = ["kernels.hip", "crc.hip", "bloom.hip", "capi.cpp", "host_stage.cpp"]
HEADERS = ["internal.hpp", "sha1_dev.hpp", "host_stage.hpp"]
ARCH = os.environ.get("NKV_OFFLOAD_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(SO):
        return True
    t = os.path.getmtime(SO)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "nkv_merkle.h")]
    return any(os.path.getmtime(d) > t for d in deps)


DIAG_SO = os.path.join(PKG, "libnkvmerkle_diag.so")


def build(force: bool = False, verbose: bool = False, diag: bool = False) -> str:
    """diag=True builds the stamp-instrumented library (tools/diag_timeline.py only)."""
    so = DIAG_SO if diag else SO
    if not force and not diag and not _stale():
        return SO
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = so + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread",
           "-Wall", "-Wno-unused-result", "-I", os.path.join(ROOT, "include"), "-I", CSRC]
    if diag:
        cmd.append("-DNKV_DIAG")
    cmd += [os.path.join(CSRC, f) for f in SOURCES] + ["-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, so)
    return so


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, diag="--diag" in sys.argv))
