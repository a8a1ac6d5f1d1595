"""Static instruction census of the rollout kernel's common-path tick loop
(diagnostics): compiles orx_engine.hip to gfx950 assembly (extra -D flags
from the command line), finds the kernel's outermost loop header, and counts
the instructions on the fall-through path from the header to its back edge
(the common tick: the out-of-line rare block is not on it) by class.  A lone
wave per SIMD pays ~8 cycles per VALU instruction and next to nothing for
SALU (tools/ubench/isa_rate.hip, profiles/r02_v1/isa_rate.jsonl), so the VALU
count is the figure of merit.

    python tools/loop_isa.py [kernel-substring] [-DFOO ...]
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.environ.get("ORX_SRC", os.path.join(ROOT, "optimax_rogue_amd", "csrc", "orx_engine.hip"))


def assemble(defs):
    out = "/tmp/orx_loop_isa.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                           "--cuda-device-only", "-S", "-o", out, SRC] + defs,
                          stderr=subprocess.DEVNULL)
    return open(out).read().splitlines()


def kernel_lines(lines, pat):
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*%s\S*:\s*(;.*)?$" % pat, l):
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit(f"kernel {pat} not found")


def classify(op):
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def census(body):
    hdr = next(i for i, l in enumerate(body) if "Loop Header: Depth=1" in l)
    label = body[hdr].split(":")[0]
    counts = collections.Counter()
    ops = collections.Counter()
    for l in body[hdr + 1:]:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op = s.split()[0]
        counts[classify(op)] += 1
        ops[op] += 1
        if op == "s_branch" and s.split()[1] == label:
            break
    return counts, ops


def main():
    args = sys.argv[1:]
    defs = [a for a in args if a.startswith("-D")]
    pats = [a for a in args if not a.startswith("-")] or ["rollout_kernelILi8ELb1ELb0E"]
    lines = assemble(defs)
    for pat in pats:
        counts, ops = census(kernel_lines(lines, pat))
        print(pat, dict(counts), "total", sum(counts.values()))
        if "-v" in sys.argv:
            for op, n in ops.most_common():
                print(f"  {n:4d} {op}")


if __name__ == "__main__":
    main()
