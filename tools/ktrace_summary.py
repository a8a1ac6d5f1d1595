"""Summarizes a rocprofv3 kernel_trace.csv: dispatches are grouped by kernel
+ grid size (--segments: consecutive runs of the same kernel + grid, in launch
order); prints each group's count and median / mean duration (us), ordered by
total time."""
import csv
import statistics
import sys


def main(path, only=None, segments=False):
    groups = {}
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    segs = []
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("orx_dev::", "").replace("void ", "")
        name = name.split("(")[0]
        if only and only not in name:
            continue
        key = (name, r["Grid_Size_X"] if "Grid_Size_X" in r else r.get("Grid_Size"))
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if segments:
            if segs and segs[-1][0] == key:
                segs[-1][1].append(d)
            else:
                segs.append((key, [d]))
        else:
            groups.setdefault(key, []).append(d)
    if not segments:
        segs = sorted(groups.items(), key=lambda kv: -sum(kv[1]))
    for (name, grid), ds in segs:
        print(f"{name[:60]:60s} grid={grid:>9s} n={len(ds):4d} median={statistics.median(ds):10.2f}us "
              f"mean={statistics.mean(ds):10.2f}us")


def span(path, kernel, grid, per_step):
    """Wall span of a kernel's dispatches at one grid size (first start to
    last end) divided by the steps they make (per_step dispatches a step):
    the per-step time of launches that overlap on several streams."""
    key = kernel.rstrip(">")   # the bench names "k<8, 1, 2>", rocprof "k<8, 1, 2, false>"
    rows = [r for r in csv.DictReader(open(path))
            if key in r["Kernel_Name"] and str(grid) in (r.get("Grid_Size_X"), r.get("Grid_Size"))]
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    t1 = max(int(r["End_Timestamp"]) for r in rows)
    steps = len(rows) / per_step
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows) / len(rows)
    print(f"{kernel} grid={grid}: {len(rows)} dispatches = {steps:g} steps, span "
          f"{(t1 - t0) / 1e3:.1f} us, {(t1 - t0) / 1e3 / steps:.2f} us per step, "
          f"mean dispatch duration {busy / 1e3:.2f} us")


if __name__ == "__main__":
    if "--span" in sys.argv:   # --span <trace.csv> <kernel substring> <grid> <dispatches per step>
        a = sys.argv[sys.argv.index("--span") + 1:]
        span(a[0], a[1], a[2], int(a[3]))
        sys.exit(0)
    args = [a for a in sys.argv[1:] if a != "--segments"]
    main(args[0], args[1] if len(args) > 1 else None, "--segments" in sys.argv)
