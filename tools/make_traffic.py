"""Writes profiles/traffic.json from two rocprofv3 PMC passes over the bench
command itself (tools/gpu_profile.sh):

    rocprofv3 --pmc FETCH_SIZE -d <fetch dir> ... -- python3 bench.py --gpus 1 --steps 20 --warmup 5
    rocprofv3 --pmc WRITE_SIZE -d <write dir> ... -- python3 bench.py --gpus 1 --steps 20 --warmup 5
    python tools/make_traffic.py <fetch dir> <write dir> [out.json]

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE is
doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B read requests at 64 B).
Only the dispatches of the headline kernel (the form orx_rollout_shape gives
for bench.py's concurrent stream shards) at its most-dispatched grid are averaged
(bench.py launches that kernel at no other shape by default); a bench step is
one dispatch per stream shard, so bytes per step = shards x the average.  The entry is
stamped with the library's build id: bench.py uses it only for that build.
"""
import collections
import ctypes
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
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("orx_dev::", "").replace("void ", "")
        agg[(name.split("(")[0], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in agg.items()}


def main(fetch_dir, write_dir, out_path=None, batch=65536, ticks=128, streams=2):
    import bench
    from optimax_rogue_amd import EnvConfig, _lib
    fe, wr = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    K = 8
    part = batch // streams                      # bench.py's stream shards (equal here)
    shape = _lib.OrxRolloutShape()
    lib = _lib.load()
    assert lib.orx_rollout_shape(ctypes.byref(EnvConfig.c3().to_c()), 1, 1, part, 1, streams,
                                 ctypes.byref(shape)) == 0
    shape = {"games_per_wave": shape.games_per_wave, "lanes_per_game": shape.lanes_per_game,
             "nontemporal": bool(shape.nontemporal)}
    kname = bench.rollout_kernel_name(K, shape)
    lanes = shape["games_per_wave"]
    # the headline kernel's grid: the dispatch shape it was profiled at most
    grids = [g for (n, g) in fe if n == kname]
    if not grids:
        raise SystemExit(f"no dispatches of {kname}: {sorted(fe)}")
    grid = max(grids, key=lambda g: fe[(kname, g)][1])
    out = {"_source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                      "`python3 bench.py --gpus 1 --steps 20 --warmup 5` (MI355X, ROCm 7.2), "
                      "written by tools/make_traffic.py. hbm_bytes = (2 * FETCH_SIZE + "
                      "WRITE_SIZE) * 1024: FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 "
                      "tallies 128-B read requests at 64 B). Per launch, averaged over the "
                      "profiled dispatches of the headline kernel at the headline grid."}
    f, w = fe.get((kname, grid)), wr.get((kname, grid))
    if f is None or w is None:
        raise SystemExit(f"no dispatches of {kname} at grid {grid}: {sorted(fe)}")
    alg = bench.bytes_per_game("rollout", K, ticks) * batch
    per_step = streams * (2 * f[0] + w[0]) * 1024
    out["rollout"] = {"kernel": kname, "batch": batch, "ticks": ticks, "streams": streams,
                      "grid": grid, "games_per_wave": lanes,
                      "lanes_per_game": shape["lanes_per_game"], "dispatches": [f[1], w[1]],
                      "fetch_kb_per_dispatch": round(f[0], 1),
                      "write_kb_per_dispatch": round(w[0], 1),
                      "hbm_bytes_per_step": int(per_step),
                      "algorithmic_bytes_per_step": int(alg),
                      "ratio": round(per_step / alg, 4),
                      "build_id": _lib.build_id()}
    out_path = out_path or os.path.join(ROOT, "profiles", "traffic.json")
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
