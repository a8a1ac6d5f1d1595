"""Builds the HIP engine in-tree: optimax_rogue_amd/liborx.so for gfx950.

    python -m optimax_rogue_amd.build [--force]
"""
from __future__ import annotations

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


def build(force: bool = False, verbose: bool = False) -> str:
    newest = max(os.path.getmtime(SRC), os.path.getmtime(HDR))
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= newest:
        return OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
           "-Wall", "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
