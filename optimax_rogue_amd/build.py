"""Builds the HIP engine in-tree: optimax_rogue_amd/liborx.so for gfx950.

    python -m optimax_rogue_amd.build [--force]
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
SRC = os.path.join(PKG_DIR, "csrc", "orx_engine.hip")
HDR = os.path.join(ROOT, "include", "orx.h")
OUT = os.path.join(PKG_DIR, "liborx.so")
ARCH = os.environ.get("ORX_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), "hipcc"):
        if os.path.sep not in c or os.path.exists(c):
            return c
    return "hipcc"


def built_id(path: str = OUT):
    """orx_build_id() of the library at `path` (None if it cannot be loaded),
    read in a child process so this one does not map a library that a later
    build replaces."""
    code = ("import ctypes,sys; L=ctypes.CDLL(sys.argv[1]); "
            "L.orx_build_id.restype=ctypes.c_char_p; print(L.orx_build_id().decode())")
    try:
        out = subprocess.run([sys.executable, "-c", code, path], capture_output=True, text=True,
                             timeout=60)
    except (OSError, subprocess.SubprocessError):
        return None
    return out.stdout.strip() if out.returncode == 0 else None


def source_id() -> str:
    """First 16 hex digits of SHA-256(orx_engine.hip || orx.h): the id
    orx_build_id() of a library built from these sources returns."""
    h = hashlib.sha256()
    for p in (SRC, HDR):
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and os.path.exists(OUT) and built_id() == source_id():
        return OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
           "-Wall", f'-DORX_BUILD_ID="{source_id()}"', "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
