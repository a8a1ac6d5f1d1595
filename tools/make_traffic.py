"""Writes profiles/traffic.json from the two rocprofv3 PMC passes of
tools/_gpu_final.sh (FETCH_SIZE and WRITE_SIZE over tools/prof_kernels.py).

    python tools/make_traffic.py gpurun_out/prof/fetch gpurun_out/prof/write

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE is
doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B read requests at 64 B).
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        agg[(name.split("(")[0], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(fetch_dir, write_dir):
    import bench
    fe, wr = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    out = {"_source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                      "tools/prof_kernels.py (MI355X, ROCm 7.2), written by tools/make_traffic.py. "
                      "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE doubled per "
                      "MI355X_MICROARCH.md (gfx950 tallies 128-B read requests at 64 B). Per "
                      "launch, averaged over the profiled dispatches."}
    # (key, kernel prefix, grid, batch, ticks, algorithmic bytes per launch)
    K = 8
    rows = [("step_kernel", "step_kernel<8, false, false>", 1 << 21, 1 << 21, 1,
             bench.bytes_per_game("step", K) * (1 << 21)),
            ("rollout", "rollout_kernel<8, true, false>", 65536, 65536, 128,
             bench.bytes_per_game("rollout", K, 128) * 65536),
            ("rollout_large", "rollout_kernel<8, true, false>", 1 << 21, 1 << 21, 20,
             bench.bytes_per_game("rollout", K, 20) * (1 << 21))]
    for key, kname, grid, batch, ticks, alg in rows:
        f, w = fe.get((kname, grid)), wr.get((kname, grid))
        if f is None or w is None:
            print("missing", key, kname, grid, file=sys.stderr)
            continue
        out[key] = {"kernel": kname, "batch": batch, "ticks": ticks, "fetch_kb": round(f, 1),
                    "write_kb": round(w, 1), "hbm_bytes_per_launch": int((2 * f + w) * 1024),
                    "algorithmic_bytes_per_launch": int(alg)}
    json.dump(out, open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
