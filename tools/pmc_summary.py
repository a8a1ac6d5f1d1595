"""Averages rocprofv3 --pmc counter_collection.csv values per (kernel, grid
size, counter); prints one line each, optionally only kernels matching a
substring."""
import collections
import csv
import sys


def short(name: str) -> str:
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def main(path, only=None):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = short(r["Kernel_Name"])
        if only and only not in name:
            continue
        agg[(name, int(r["Grid_Size"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (name, grid, ctr), v in agg.items():
        print(f"{name:28s} grid={grid:9d} {ctr:14s} dispatches={len(v)} mean={sum(v) / len(v):.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
