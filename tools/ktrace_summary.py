"""Summarizes a rocprofv3 kernel_trace.csv: consecutive dispatches of the same
kernel + grid size form a segment; prints each segment's count and median /
mean duration (us), in launch order."""
import csv
import statistics
import sys


def main(path, only=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    segs = []
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0]
        if only and only not in name:
            continue
        key = (name, r["Grid_Size_X"] if "Grid_Size_X" in r else r.get("Grid_Size"))
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if segs and segs[-1][0] == key:
            segs[-1][1].append(d)
        else:
            segs.append((key, [d]))
    for (name, grid), ds in segs:
        print(f"{name[:60]:60s} grid={grid:>9s} n={len(ds):4d} median={statistics.median(ds):10.2f}us "
              f"mean={statistics.mean(ds):10.2f}us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
