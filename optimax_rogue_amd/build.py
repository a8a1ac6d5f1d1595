"""Builds the HIP engine in-tree: optimax_rogue_amd/liborx.so for gfx950.

    python -m optimax_rogue_amd.build [--force]

Diagnostic variants (results wrong by design; used by tools/ab_*.py and
tools/stamps.py to attribute time) are built by the same recipe with extra
preprocessor definitions, into tools/ab_libs/ by default:

    python -m optimax_rogue_amd.build --variant diag16     # -DORX_DIAG=16: no trajectory stores
    python -m optimax_rogue_amd.build --variant diag32     # -DORX_DIAG=32: trajectory stores only
    python -m optimax_rogue_amd.build --variant stamps     # -DORX_STAMPS: s_memtime timeline
    python -m optimax_rogue_amd.build --define ORX_STREAM_AUX=0 --out /tmp/x.so

The definitions are folded into the library's build id (``orx_build_id()``
= ``source_id(defines)``), so a diagnostic library can never pass for the
product build (tests/test_gpu_parity.py::test_loaded_library_is_the_trees_kernel).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from typing import Iterable, Optional

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
SRC = os.path.join(PKG_DIR, "csrc", "orx_engine.hip")
HDR = os.path.join(ROOT, "include", "orx.h")
OUT = os.path.join(PKG_DIR, "liborx.so")
ARCH = os.environ.get("ORX_OFFLOAD_ARCH", "gfx950")
AB_LIBS = os.path.join(ROOT, "tools", "ab_libs")

# named diagnostic variants: their -D sets
VARIANTS = {
    "diag16": ("ORX_DIAG=16",),   # rollout without its trajectory stores
    "diag32": ("ORX_DIAG=32",),   # the trajectory stores alone (no tick runs)
    "stamps": ("ORX_STAMPS",),    # per-wave s_memtime stamps + rare-block counts
    "diag64": ("ORX_DIAG=64",),   # the paired RandomBot tick block without Philox
    "noremap": ("ORX_XCD_REMAP=0",),  # workgroups in dispatch order (no XCD-aware remap)
    "lean": ("ORX_LEAN=1",),      # the paired StaircaseBot form with its lean spans (rejected)
    "split1": ("ORX_SPLIT_TICK=1",),  # split tick blocks in the compact form (rejected)
    "split2": ("ORX_SPLIT_TICK=2",),  # split tick blocks in every paired RandomBot form (rejected)
    "sepw0": ("ORX_SEP_WAVES=0",),    # the separation-damage StaircaseBot form uncapped (131 VGPRs)
    "envw5": ("ORX_ENV_WAVES=5",),    # orx_env_step_ex held to 5 waves per SIMD
    "envw6": ("ORX_ENV_WAVES=6",),    # ... to 6
    "envd1": ("ORX_ENV_DIAG=1",),     # orx_env_step without its tick (outputs of the loaded state)
    "envd2": ("ORX_ENV_DIAG=2",),     # orx_env_step without its observation rows
    "routl": ("ORX_RARE_OUTLINE=1",),  # the paired fallback rare tick out of line (rejected)
}


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


def source_id(defines: Iterable[str] = ()) -> str:
    """The id orx_build_id() of a library built from these sources returns:
    the first 16 hex digits of SHA-256(orx_engine.hip || orx.h), and for a
    build with extra definitions ``+`` and their sorted list (so the product
    id is exactly the sources' hash and no diagnostic build shares it)."""
    h = hashlib.sha256()
    for p in (SRC, HDR):
        with open(p, "rb") as f:
            h.update(f.read())
    d = sorted(defines)
    return h.hexdigest()[:16] + ("+" + ",".join(d) if d else "")


def build(force: bool = False, verbose: bool = False, defines: Iterable[str] = (),
          out: Optional[str] = None) -> str:
    defines = tuple(defines)
    out = out or (OUT if not defines else os.path.join(AB_LIBS, "custom.so"))
    sid = source_id(defines)
    if not force and os.path.exists(out) and built_id(out) == sid:
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    # one build per output at a time (parallel test workers in a fresh tree):
    # the others wait on the lock and then find the library built
    import fcntl
    with open(out + ".lock", "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        if not force and os.path.exists(out) and built_id(out) == sid:
            return out
        return _build_locked(out, sid, defines, verbose)


def _build_locked(out: str, sid: str, defines, verbose: bool) -> str:
    base = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
            f'-DORX_BUILD_ID="{sid}"'] + [f"-D{d}" for d in defines]
    if any(d.split("=")[0] == "ORX_STAMPS" for d in defines):
        # one translation unit (the stamps buffer is a device global read back
        # by the host side, so every kernel must live in the host's unit)
        cmd = base + ["-shared", "-o", out + ".tmp", SRC]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
    else:
        _build_parts(base, out + ".tmp", verbose)
    os.replace(out + ".tmp", out)
    return out


# The split build: orx_engine.hip compiled NPARTS times in parallel (part 0:
# the host side, every kernel instance declared extern; parts 1..NPARTS-1:
# their share of the explicit instantiations, orx_engine.hip "Kernel
# instances"), then linked -- about a minute on 8 cores instead of ~6 for one
# translation unit.
NPARTS = 16


def _build_parts(base, out, verbose=False, jobs=None):
    import tempfile
    jobs = jobs or max(1, min(NPARTS, int(os.environ.get("MAX_JOBS", 0)) or os.cpu_count() or 1))
    with tempfile.TemporaryDirectory(prefix="orx_build_") as tmp:
        objs = [os.path.join(tmp, f"part{k}.o") for k in range(NPARTS)]
        cmds = [base + ["-c", f"-DORX_NPARTS={NPARTS}", f"-DORX_PART={k}", "-o", objs[k], SRC]
                for k in range(NPARTS)]
        if verbose:
            print(" ".join(cmds[0]) + f"  (parts 0..{NPARTS - 1}, {jobs} at a time)")
        # the heaviest parts first (the paired and one-lane rollouts)
        order = list(range(1, NPARTS)) + [0]
        running, failed = [], []
        while order or running:
            while order and len(running) < jobs:
                k = order.pop(0)
                running.append((k, subprocess.Popen(cmds[k])))
            k, p = running.pop(0)
            if p.wait() != 0:
                failed.append(k)
        if failed:
            raise subprocess.CalledProcessError(1, f"hipcc part(s) {failed}")
        link = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs
        if verbose:
            print(" ".join(link))
        subprocess.check_call(link)


def build_variant(name: str, force: bool = False, verbose: bool = False) -> str:
    """tools/ab_libs/<name>.so for a named diagnostic variant (VARIANTS)."""
    return build(force, verbose, VARIANTS[name], os.path.join(AB_LIBS, name + ".so"))


def main(argv):
    force = "--force" in argv
    defines, out, variants = [], None, []
    it = iter(argv)
    for a in it:
        if a == "--define":
            defines.append(next(it))
        elif a == "--out":
            out = os.path.abspath(next(it))
        elif a == "--variant":
            variants.append(next(it))
    if len(variants) > 1 and out:
        raise SystemExit("--out names one library: give one --variant with it")
    for v in variants:   # --variant NAME [--out PATH]: that variant (plus any --define)
        print(build(force, True, VARIANTS[v] + tuple(defines),
                    out or os.path.join(AB_LIBS, v + ".so")))
    if not variants:
        print(build(force, verbose=True, defines=defines, out=out))


if __name__ == "__main__":
    main(sys.argv[1:])
