#!/usr/bin/env python3
"""bench.py -- env-steps/s of the batched Optimax Rogue tick engine on MI355X.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

`--gpus N` outside torchrun starts the N rank processes itself (one per GPU,
torch.distributed.run on 127.0.0.1, before this process touches the GPU) and
exits with their code; under torchrun WORLD_SIZE must equal N.

Workload (BASELINE.json configs[2], "C3"): 65,536 games per GPU on a 64x64
grid with enemies (K = 8 NPCs per game), both players driven by RandomBot,
Unreachable despawn, max_ticks 1000 with autoreset.  An env-step = one game
advanced one tick.  ONE BENCH STEP = one fused rollout launch of --chunk
(default 128) ticks over every game: the trajectory horizon a learner
consumes, the unit the hot path is called with.  `--steps K` times K such
launches (K x 128 ticks of every game); `value` = games x ranks x ticks /
time.  Games shard across GPUs by global game id (parallel.shard; weak
scaling, no data-path collective); after the timed region the per-game
episode returns are all-gathered over RCCL (the only collective).

Timed path: the fused rollout kernel; state stays in registers and EVERY
tick's full observation (14 int32 fields: both players' x, y, depth, health,
staircase, plus tick and status) and both actions are written to an HBM
trajectory buffer -- nothing is skipped.  The launches are issued through a
pre-bound launcher (one ctypes call each) with HIP events created beforehand,
so the timed region is the kernels back to back.

Extras (rank 0, 1 GPU): the unfused path (orx_policy + orx_step per tick,
captured in a HIP graph) at the config batch, the per-tick kernels at 2^21
games, C2 and C5.

Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
OBS_BYTES = 14 * 4      # one tick record: 14 int32 fields
ACT_BYTES = 2
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")
# the reference's own Python updater timed on the build container's cores
# (tools/ref_cpu_baseline.py; the reference never travels to the GPU box)
REF_CPU_FILE = os.path.join(ROOT, "profiles", "ref_cpu_c3.json")


def contract_bytes_per_env_step(K: int) -> int:
    """SURVEY.md §8(d)'s algorithmic bytes per env-step (the roofline contract):
    read actions 2 + players 32 + tick/status 8 + staircases 16 = 58, write
    players 32 + tick/status 8 = 40 -> 98 B; +8 B occupancy probe with NPCs
    (C3) -> 106 B.  A fused rollout keeps the state in registers and skips the
    re-read (its moved bytes, `traffic` / `materialized_bytes_per_launch`, are
    lower): the per-tick step kernel is priced with it, the fused rollout
    with its own bytes (`bytes_per_game("rollout", ...)`), the contract beside."""
    return 98 + (8 if K else 0)


def bytes_per_game(kernel: str, K: int, ticks: int = 1) -> int:
    """Bytes each kernel actually reads + writes per game per launch."""
    npc_read = (4 + 2 * K) if K else 0        # alive mask + K packed u16 positions
    if kernel == "step":
        # read: actions 2, players 32, staircases 16, tick/status/episode 12, NPCs
        # write: positions 16, tick 4 (depth, health and status only where they
        # changed: a descend, a combat, an episode end -- rare per game-tick)
        return 2 + 32 + 16 + 12 + npc_read + 20
    if kernel == "policy":
        return 4 + 4 + 2                       # tick, episode -> 2 int8 actions
    if kernel == "env_step":
        # orx_env_step_ex with int64 learner actions for player 1 and a RandomBot
        # opponent: read the actions 8, status/tick/episode 12, players and
        # staircases 48, the NPCs; write the action pair 2, positions 16, tick
        # 4, the observation row 56, reward 4, done 1, status 4 (depth, health
        # and staircases only where a descend or combat changed them)
        return 8 + 12 + 48 + npc_read + 2 + 16 + 4 + OBS_BYTES + 4 + 1 + 4
    # players, staircases, tick/status/episode, NPC positions + alive mask + health
    state_in = 32 + 16 + 12 + npc_read + K
    state_out = 32 + 12 + (4 + K if K else 0)  # players, tick/status/episode, alive, health
    return ticks * (OBS_BYTES + ACT_BYTES) + state_in + state_out


def rollout_kernel_name(K: int, shape: dict) -> str:
    """The kernel orx_rollout launches for this workload, as rocprofv3 names
    it: the RandomBot + trajectory specialization (PM=1), NPC capacity
    0/8/16, in the form orx_rollout_shape reports -- pair_rollout_kernel<NCAP,
    PM, AUX, SEP, CF, GRID> (two lanes per game; separation damage off, int32
    rows, empty dungeons) or rollout_kernel<NCAP, PM, GRID, AUX, CF> -- with
    its store policy (AUX 2 = nontemporal, 0 = default)."""
    ncap = 0 if K == 0 else 8 if K <= 8 else 16
    aux = 2 if shape["nontemporal"] else 0
    if shape["lanes_per_game"] == 2:
        return f"pair_rollout_kernel<{ncap}, 1, {aux}, false, false, false>"
    return f"rollout_kernel<{ncap}, 1, false, {aux}, false>"


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def physical_cores() -> int:
    """Physical cores of the host: unique (core, socket) pairs of `lscpu -p`
    (os.cpu_count() when lscpu is absent)."""
    try:
        out = subprocess.run(["lscpu", "-p=CORE,SOCKET"], capture_output=True, text=True,
                             timeout=20).stdout
        pairs = {tuple(l.split(",")[:2]) for l in out.splitlines() if l and l[0] != "#"}
        if pairs:
            return len(pairs)
    except (OSError, subprocess.SubprocessError):
        pass
    return os.cpu_count() or 1


def cpu_quota():
    """CPUs this job's cgroup may use at once (cgroup v2 cpu.max, v1
    cfs_quota_us / cfs_period_us), or None when it sets no limit."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def cpu_baseline(cfg_dict: dict, seconds: float) -> dict:
    """The C oracle (scalar port of the reference updater) on the host cores
    (the reference's own Python updater, timed in the build container, rides
    beside it as `reference_python`),
    same workload shape: one core for `seconds` * 0.4, then one thread per
    core of this job's CPU share (at most 16, the GPU box's share per GPU) for
    `seconds` * 1.5 / cores each -- about `seconds` * 2 of CPU work in all.
    Each thread owns an oracle of 256 games (disjoint game ids); ctypes
    releases the GIL inside the C calls, so the threads run in parallel."""
    import threading
    from oracle.oracle import Oracle, build
    build()
    B = 256

    def leg(k, wall, out):
        ora = Oracle(cfg_dict, B, 3, k * B)
        ora.reset()
        t0 = time.perf_counter()
        ticks = 0
        while True:
            ora.rollout(1, 1, 50)
            ticks += 50
            el = time.perf_counter() - t0
            if el >= wall:
                break
        out[k] = (ticks, el)

    one = {}
    leg(0, 0.4 * seconds, one)
    single = B * one[0][0] / one[0][1]
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    cores = max(1, min(16, avail))
    wall = max(1.0, 1.5 * seconds / cores)
    res = {}
    th = [threading.Thread(target=leg, args=(k, wall, res)) for k in range(cores)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    total = sum(B * n for n, _ in res.values())
    ref = None
    if os.path.exists(REF_CPU_FILE):
        rj = json.load(open(REF_CPU_FILE))
        full = rj["full"]
        ref = {"value": full["aggregate_env_steps_per_s"], "unit": "env-steps/s",
               "cores": full["procs"], "per_core": full["per_core_env_steps_per_s"],
               "single_core": full["single_core_env_steps_per_s"], "host": rj["host"],
               "where": "build container (the reference cannot run on the GPU box)",
               "sample": f"{rj['workload']}; the reference's RandomBot.move x2 + on_tick + "
                         f"Updater.update, one process per core for "
                         f"{full['seconds_per_proc']} s each ({full['env_steps']} env-steps); "
                         "tools/ref_cpu_baseline.py -> profiles/ref_cpu_c3.json"}
    # the pure-Python object-model restatement of the reference (oracle/pyref.py,
    # bit-exact vs the reference fixtures): the reference's cost profile timed
    # on THIS host's cores, one process per core (a child interpreter: the
    # processes fork from it, not from this GPU-initialized one)
    pyr = None
    try:
        r = subprocess.run([sys.executable, "-m", "oracle.pyref", "--bench",
                            f"--seconds={max(1.0, 0.2 * seconds)}",
                            f"--single={max(1.0, 0.3 * seconds)}", f"--procs={cores}"],
                           cwd=ROOT, capture_output=True, text=True, timeout=300)
        pyr = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
            {"error": r.stderr[-500:]}
    except (subprocess.SubprocessError, ValueError, IndexError) as e:
        pyr = {"error": repr(e)}
    # the restatement's cost relative to the reference's on one host (the
    # build container, tools/ref_cpu_baseline.py): the reference's own rate on
    # THIS host's cores, estimated as python_restatement / that ratio
    if ref is not None and "pyref_vs_reference" in rj and "per_core" in (pyr or {}):
        ratio = rj["pyref_vs_reference"]
        ref["pyref_vs_reference"] = {k: ratio[k] for k in ("single_core", "per_core")}
        pyr["reference_estimate_here"] = {
            "per_core": pyr["per_core"] / ratio["per_core"],
            "value": pyr["value"] / ratio["per_core"], "cores": pyr["cores"],
            "note": "python_restatement / pyref_vs_reference.per_core (both legs measured on "
                    "one host): the reference updater's estimated rate on this box's cores"}
    # the whole host (every physical core of the box, not the
    # per-GPU share above): the C port as one thread per physical core this
    # job may run on, and the Python restatement as one process per such core
    phys = physical_cores()
    n_all = max(1, min(phys, avail))
    res_all = {}
    th = [threading.Thread(target=leg, args=(k, 2.0, res_all)) for k in range(n_all)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    el_all = time.perf_counter() - t0
    tot_all = sum(B * n for n, _ in res_all.values())
    pyr_all = None
    try:
        r = subprocess.run([sys.executable, "-m", "oracle.pyref", "--bench", "--seconds=2.0",
                            "--single=0.5", f"--procs={n_all}"],
                           cwd=ROOT, capture_output=True, text=True, timeout=300)
        pyr_all = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
            {"error": r.stderr[-500:]}
        pyr_all.pop("lscpu", None)
    except (subprocess.SubprocessError, ValueError, IndexError) as e:
        pyr_all = {"error": repr(e)}
    quota = cpu_quota()
    whole = {"physical_cores": phys, "cpus_visible": os.cpu_count(), "cpus_in_affinity": avail,
             "cgroup_cpu_quota": quota, "cores_used": n_all, "host": _cpu_model(),
             "port": {"value": tot_all / el_all, "unit": "env-steps/s", "cores": n_all,
                      "per_core": tot_all / el_all / n_all,
                      "sample": f"{n_all} threads x 256 games for {el_all:.1f} s "
                                f"({tot_all} env-steps)"},
             "python_restatement": pyr_all,
             "note": "every physical core of the host this job may run on (lscpu: unique "
                     "(core, socket) pairs, capped by the process's CPU affinity); the "
                     "top-level value is the per-GPU share of 16 threads"
                     + ("" if quota is None else
                        f"; this job's cgroup allows {quota:g} CPUs at once, so these threads "
                        "time-share them and the whole-host figure is bounded by the quota, "
                        "not by the cores")}
    return {"value": total / el, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "whole_host": whole,
            "python_restatement": pyr,
            "reference_python": ref,
            "per_core": total / el / cores, "single_core": single,
            "sample": f"C oracle (scalar C restatement of Updater.update + RandomBot) on the "
                      f"same C3 workload: {cores} threads x 256 games for {el:.1f} s "
                      f"({total} env-steps), plus 1 core alone for "
                      f"{one[0][1]:.1f} s; host {_cpu_model()}, {os.cpu_count()} CPUs visible, "
                      f"{avail} in this job's affinity"}


def timed_launches(torch, launch, n):
    """Runs `launch` n times with HIP events around each (on torch's current
    stream, the stream the engine launches on); returns per-launch seconds."""
    evs = []
    for _ in range(n):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        launch()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    return [a.elapsed_time(b) * 1e-3 for a, b in evs]


def extras(torch, cfg, dev, B_cfg, K, large_rollout=False):
    """Unfused path at the config batch (HIP graph), the per-tick kernels at
    2^21 games (and, with `large_rollout`, the headline rollout kernel there:
    off by default so that a profile of the bench command sees that kernel at
    the headline shape only), C2 and C5."""
    from optimax_rogue_amd import OBS_FIELDS
    from optimax_rogue_amd.engine import BatchedEngine, StreamShardedEngine
    out = {}
    # (1) unfused policy+step, 50 ticks captured in one HIP graph, config batch
    eng = BatchedEngine(cfg, B_cfg, seed=3, device=dev)
    for _ in range(3):
        eng.step(eng.policy(1, 1))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(50):
                eng.step(eng.policy(1, 1))
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n_rep = 20
    for _ in range(n_rep):
        g.replay()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out["unfused_graph"] = {"value": B_cfg * 50 * n_rep / el, "unit": "env-steps/s",
                            "us_per_tick": el / (50 * n_rep) * 1e6,
                            "note": "orx_policy + orx_step per tick, 50 ticks per HIP graph"}
    del eng, g
    torch.cuda.empty_cache()
    # (1b) the learner's per-tick path: VecEnv.step (one orx_env_step_ex launch:
    # int64 learner actions for player 1, RandomBot opponent, observation /
    # reward / done / status out, the deferred refused-action count, no host
    # sync), called eagerly from Python at the config batch, 400 ticks, wall
    # clock -- with fresh output tensors per step (the default) and from a
    # ring of two preallocated sets (out_buffers=2)
    from optimax_rogue_amd import VecEnv
    pool = torch.randint(1, 6, (16, B_cfg), dtype=torch.int64, device=dev)
    n_ve = 400
    eager = {}
    for ring in (0, 2):
        env = VecEnv(cfg, B_cfg, seed=3, device=dev, opponent=1, out_buffers=ring)
        for k in range(20):
            env.step(pool[k % 16])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(n_ve):
            env.step(pool[k % 16])
        torch.cuda.synchronize()
        eager[ring] = time.perf_counter() - t0
    el = eager[0]
    # the same 50 calls captured in one HIP graph (no host sync inside
    # VecEnv.step makes it capturable): the device's time per tick
    gv = torch.cuda.CUDAGraph()
    sv = torch.cuda.Stream(device=dev)
    sv.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(sv):
        with torch.cuda.graph(gv, stream=sv):
            for k in range(50):
                env.step(pool[k % 16])
    torch.cuda.current_stream().wait_stream(sv)
    gv.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        gv.replay()
    torch.cuda.synchronize()
    gel = (time.perf_counter() - t0) / 500
    out["vecenv_step"] = {"value": B_cfg * n_ve / el, "unit": "env-steps/s",
                          "us_per_tick": el / n_ve * 1e6,
                          "ring_us_per_tick": eager[2] / n_ve * 1e6,
                          "graph_us_per_tick": gel * 1e6,
                          "note": "VecEnv.step called eagerly from Python (int64 learner actions "
                                  "+ RandomBot opponent -> obs, reward, done, status): one "
                                  "learner-tick launch per tick (env_step_kernel), no host "
                                  "sync; us_per_tick with fresh output tensors "
                                  "(orx_env_step_ex), ring_us_per_tick with out_buffers=2 (one "
                                  "prebuilt orx_env_step_args block per output set); "
                                  "graph_us_per_tick: 50 calls captured in one HIP graph"}
    del env, pool, gv
    torch.cuda.empty_cache()
    # (1c) a replay: orx_step_n over a 128-tick move log (int8 [128, B, 2],
    # uniform 1..5) at the config batch, every tick's observation rows
    # written -- the paired LOG form (pair_rollout_kernel PM 6, two lanes per
    # game, round 6) as two stream shards, the headline's recipe
    # (StreamShardedEngine.replay_launcher: each shard's log its own
    # contiguous slice, 3 warmup + 20 timed launches per shard between one
    # fork and one join); one launch over the whole log and the one-lane
    # replay_kernel timed beside it
    T = 128
    log = torch.randint(1, 6, (T, B_cfg, 2), dtype=torch.int8, device=dev)
    se = StreamShardedEngine(cfg, B_cfg, seed=3, device=dev, n_streams=2)
    slogs = se.split_log(log)
    sobs, _ = se.trajectory_buffers(T)
    go = se.replay_launcher(slogs, sobs)
    se.fork()
    for _ in range(3):
        go()
    se.join()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    ev0.record()
    se.fork()
    for _ in range(20):
        go()
    se.join()
    ev1.record()
    torch.cuda.synchronize()
    rmed = ev0.elapsed_time(ev1) * 1e-3 / 20
    del se, slogs, sobs, go
    eng = BatchedEngine(cfg, B_cfg, seed=3, device=dev)
    robs = torch.empty((T, len(OBS_FIELDS), B_cfg), dtype=torch.int32, device=dev)
    eng.step_n(log, obs=robs)
    rs = timed_launches(torch, lambda: eng.step_n(log, obs=robs), 10)
    one_launch = sorted(rs)[len(rs) // 2]
    os.environ["ORX_REPLAY_PAIRED"] = "0"   # the one-lane replay_kernel, for the record
    try:
        r1 = timed_launches(torch, lambda: eng.step_n(log, obs=robs), 10)
    finally:
        del os.environ["ORX_REPLAY_PAIRED"]
    one_lane = sorted(r1)[len(r1) // 2]
    # the rows (56 B a tick) and the log read (2 B a tick, in place of the
    # rollout's action rows: a replay writes none) + the state once
    rb = bytes_per_game("rollout", K, T) * B_cfg
    out["replay_step_n"] = {"games": B_cfg, "ticks_per_launch": T, "streams": 2,
                            "us_per_launch": rmed * 1e6,
                            "env_steps_per_s": B_cfg * T / rmed,
                            "achieved_GBps": rb / rmed / 1e9,
                            "frac": rb / rmed / 1e9 / HBM_PEAK_GBS,
                            "one_launch_us": one_launch * 1e6,
                            "one_lane_us_per_launch": one_lane * 1e6,
                            "note": "orx_step_n: a 128-tick move log of both players replayed "
                                    "with every tick's observation rows, the paired LOG form "
                                    "(pair_rollout_kernel PM 6, 32 games per wave) as two "
                                    "32,768-game stream shards (us_per_launch: per step of both "
                                    "shards, 20 timed); one_launch_us = orx_step_n over the "
                                    "whole batch in one launch, one_lane_us_per_launch = the "
                                    "one-lane replay_kernel (ORX_REPLAY_PAIRED=0), medians of "
                                    "10; bytes: rows 56 + log 2 per env-step + the state once"}
    del eng, log, robs
    torch.cuda.empty_cache()
    # (2) large batch: the chip full (2^21 games)
    BL = 1 << 21
    eng = BatchedEngine(cfg, BL, seed=3, device=dev)
    for _ in range(2):
        eng.step(eng.policy(1, 1))
    step_s = timed_launches(torch, lambda: eng.step(), 30)
    pol_s = timed_launches(torch, lambda: eng.policy(1, 1), 30)
    # the learner's fused tick (orx_env_step_ex) at the same batch, its
    # buffers allocated once
    la = torch.randint(1, 6, (BL,), dtype=torch.int64, device=dev)
    lo = torch.empty((BL, len(OBS_FIELDS)), dtype=torch.int32, device=dev)
    lr = torch.empty(BL, dtype=torch.float32, device=dev)
    ld = torch.empty(BL, dtype=torch.bool, device=dev)
    ls = torch.empty(BL, dtype=torch.int32, device=dev)
    lb = torch.zeros(1, dtype=torch.int32, device=dev)
    env_s = timed_launches(torch, lambda: eng.env_step(la, 1, lo, lr, ld, ls, lb), 30)
    del la, lo, lr, ld, ls, lb
    med = lambda v: sorted(v)[len(v) // 2]
    sb = contract_bytes_per_env_step(K) * BL
    eb = bytes_per_game("env_step", K) * BL
    out["large_batch"] = {
        "games": BL,
        "step_kernel": {"avg_us": med(step_s) * 1e6, "achieved_GBps": sb / med(step_s) / 1e9,
                        "frac": sb / med(step_s) / 1e9 / HBM_PEAK_GBS,
                        "bytes_per_env_step": contract_bytes_per_env_step(K),
                        "moved_bytes_per_env_step": bytes_per_game("step", K)},
        "policy_kernel": {"avg_us": med(pol_s) * 1e6},
        "env_step": {"avg_us": med(env_s) * 1e6, "env_steps_per_s": BL / med(env_s),
                     "achieved_GBps": eb / med(env_s) / 1e9,
                     "frac": eb / med(env_s) / 1e9 / HBM_PEAK_GBS,
                     "bytes_per_env_step": bytes_per_game("env_step", K),
                     "note": "orx_env_step_ex (int64 learner actions, RandomBot opponent, obs / "
                             "reward / done / status / refused-action count), median of 30 "
                             "launches between HIP events"},
    }
    if large_rollout:
        T = 20
        obs = torch.empty((T, len(OBS_FIELDS), BL), dtype=torch.int32, device=dev)
        act = torch.empty((T, BL, 2), dtype=torch.int8, device=dev)
        eng.rollout(T, 1, 1, obs=obs, act=act)
        roll_s = timed_launches(torch, lambda: eng.rollout(T, 1, 1, obs=obs, act=act), 5)
        rb = bytes_per_game("rollout", K, T) * BL
        rc = contract_bytes_per_env_step(K) * BL * T
        out["large_batch"]["rollout_kernel"] = {
            "avg_us": med(roll_s) * 1e6, "ticks": T, "env_steps_per_s": BL * T / med(roll_s),
            "achieved_GBps": rb / med(roll_s) / 1e9, "frac": rb / med(roll_s) / 1e9 / HBM_PEAK_GBS,
            "contract_frac": rc / med(roll_s) / 1e9 / HBM_PEAK_GBS}
        del obs, act
    del eng
    torch.cuda.empty_cache()
    # (3) the other BASELINE.json GPU configs, fused rollout with trajectories:
    # C2 (4,096 games, 32x32, RandomBot) and C5 (128x128, StaircaseBot "ladder"
    # policy, separation damage off and on) at its per-GPU share of 131,072
    # games on 8 GPUs and at the whole 131,072 on this one
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.enums import EXT_SEPARATION_DAMAGE

    def rollout_rate(c, games, pol, T=128, reps=6, streams=1):
        """µs per T-tick launch of `games` (median of `reps`); with streams > 1
        the games run as that many stream shards, as the headline step does
        (StreamShardedEngine; a step = one launch per shard, fork/join).
        ``pol``: both players' policy, or a (player 1, player 2) pair."""
        p1, p2 = (pol, pol) if isinstance(pol, int) else pol
        if streams > 1:
            # as the headline step: the shards' launches back to back on their
            # streams between one fork and one join, HIP events around them all
            # (3 warmup steps and 20 timed, as the headline: the shards' tails
            # overlap the next steps' launches, which a short run under-counts)
            e = StreamShardedEngine(c, games, seed=5, device=dev, n_streams=streams)
            o, a = e.trajectory_buffers(T)
            go = e.rollout_launcher(T, p1, p2, obs=o, act=a)
            e.fork()
            for _ in range(3):
                go()
            e.join()
            reps = max(reps, 20)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            ev0.record()
            e.fork()
            for _ in range(reps):
                go()
            e.join()
            ev1.record()
            torch.cuda.synchronize()
            us = ev0.elapsed_time(ev1) * 1e-3 / reps
        else:
            e = BatchedEngine(c, games, seed=5, device=dev)
            o = torch.empty((T, len(OBS_FIELDS), games), dtype=torch.int32, device=dev)
            a = torch.empty((T, games, 2), dtype=torch.int8, device=dev)
            go = e.rollout_launcher(T, p1, p2, obs=o, act=a)
            go()
            d = timed_launches(torch, go, reps)
            us = sorted(d)[len(d) // 2]
        shape = e.rollout_shape(p1, p2)
        del e, o, a, go
        return {"games": games, "ticks_per_launch": T, "games_per_wave": shape["games_per_wave"],
                "lanes_per_game": shape["lanes_per_game"], "nontemporal": shape["nontemporal"],
                "streams": streams, "us_per_launch": us * 1e6, "env_steps_per_s": games * T / us}

    # (3a) the headline step with ORX_OBS_COMPACT trajectory rows (24 B per
    # env-step instead of 56: u8 cells and staircases, int16 healths,
    # tick | status << 27; the same launches, shards and stream layout)
    from optimax_rogue_amd.enums import OBS_COMPACT
    sh = StreamShardedEngine(cfg, B_cfg, seed=3, device=dev, n_streams=2)
    T = 128
    co, ca = sh.trajectory_buffers(T, OBS_COMPACT)
    go = sh.rollout_launcher(T, 1, 1, obs=co, act=ca, obs_format=OBS_COMPACT)
    sh.fork()
    for _ in range(3):
        go()
    sh.join()
    reps = 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    sh.fork()
    for _ in range(reps):
        go()
    sh.join()
    e1.record()
    torch.cuda.synchronize()
    step_s = e0.elapsed_time(e1) * 1e-3 / reps
    cb = (bytes_per_game("rollout", K, T) - T * OBS_BYTES + T * 24) * B_cfg
    out["compact_rows"] = {
        "games": B_cfg, "ticks_per_step": T, "streams": 2, "us_per_step": step_s * 1e6,
        "env_steps_per_s": B_cfg * T / step_s, "bytes_per_env_step": cb / (B_cfg * T),
        "achieved_GBps": cb / step_s / 1e9, "frac": cb / step_s / 1e9 / HBM_PEAK_GBS,
        "note": "bench step with obs_format=ORX_OBS_COMPACT (6 uint32 rows per tick: cells, "
                "staircases, healths, depths, tick|status; decode_compact gives the 14 int32 "
                "fields back bit-exact) -- an opt-in trajectory format, not the headline"}
    del sh, co, ca, go
    torch.cuda.empty_cache()
    out["c2"] = dict(rollout_rate(EnvConfig.c2(), 4096, 1), policy="2x RandomBot", grid="32x32")
    # the explicit-grid generator (dungeon bank): C3's shape on 16 random
    # 64x64 layouts, tiles staged in LDS by the rollout
    from optimax_rogue_amd import DungeonBank
    bank = DungeonBank.random(64, 64, 16, seed=7)
    out["bank"] = dict(rollout_rate(EnvConfig(width=64, height=64, n_npcs=8, layouts=bank.layouts),
                                    65536, 1, streams=2),
                       policy="2x RandomBot", grid="64x64, 16 layouts (15% walls)",
                       note="two stream shards timed as the headline step (the paired form, "
                            "tiles staged in LDS: 64 KiB); us_per_launch = one step")
    # configs[2] read literally, "64x64 grid with enemies+items enabled": C3 with
    # the readme's character mechanics on (build extensions, no reference
    # semantics, so not the bit-exact headline)
    from optimax_rogue_amd.enums import EXT_RPG
    out["c3_rpg"] = dict(rollout_rate(EnvConfig(width=64, height=64, n_npcs=8, flags=EXT_RPG),
                                      65536, 1, streams=2),
                         policy="2x RandomBot", grid="64x64, 8 NPCs",
                         note="mana, heal, experience, item drops/pickup on (EXT_RPG; engine "
                              "vs oracle bit-exact, parity unpinned vs the reference); two "
                              "stream shards timed as the headline step (the paired form); "
                              "us_per_launch = one step")
    # a learner's baseline evaluation: C3 with a RandomBot against a
    # StaircaseBot (the paired mixed-bot form since round 5)
    out["c3_mixed"] = dict(rollout_rate(cfg, 65536, (1, 2), streams=2),
                           policy="RandomBot vs StaircaseBot", grid="64x64, 8 NPCs",
                           note="two stream shards timed as the headline step (the paired "
                                "PM 4 form); us_per_launch = one step")
    # moving NPCs (round 6): C3 with the enemy AI plugged into
    # Updater.decide_npc_move (npc_policy RANDOM / CHASE, reference-pinned):
    # the literal ordered tick, one lane per game (mov_rollout_kernel)
    from optimax_rogue_amd.enums import NpcPolicy
    for pol_name, npol in (("c3_moving_npcs", NpcPolicy.Random), ("c3_chasing_npcs",
                                                                  NpcPolicy.Chase)):
        r = rollout_rate(EnvConfig(width=64, height=64, n_npcs=8, npc_policy=int(npol)), 65536, 1)
        mb = bytes_per_game("rollout", 8, 128) * 65536
        r.update(achieved_GBps=mb / r["us_per_launch"] / 1e3,
                 frac=mb / r["us_per_launch"] / 1e3 / HBM_PEAK_GBS)
        out[pol_name] = dict(r, policy="2x RandomBot", grid="64x64, 8 NPCs",
                             note=f"npc_policy {npol.name}: every NPC's move decided, shuffled "
                                  "and resolved per tick (updater.py:116-145) in the generic "
                                  "one-lane form; frac by the rollout's own bytes")
    c5 = {}
    for flag in (0, EXT_SEPARATION_DAMAGE):
        c = EnvConfig.c5()
        if flag:
            c.flags, c.sep_period = flag, 8
        key = "separation_damage_on" if flag else "separation_damage_off"
        # the 8-GPU share as two stream shards timed as the headline step (one
        # shard's next launch runs while the other's slowest waves finish:
        # 64 vs 70 us, profiles/r04_v18/shard_small.jsonl), then as one launch,
        # then the whole 131,072 on one GPU
        c5[key] = [rollout_rate(c, 131072 // 8, 2, streams=2), rollout_rate(c, 131072 // 8, 2),
                   rollout_rate(c, 131072, 2, streams=2), rollout_rate(c, 131072, 2)]
    out["c5"] = dict(c5, policy="2x StaircaseBot", grid="128x128",
                     note="separation damage = build extension EXT_SEPARATION_DAMAGE, "
                          "sep_period 8 (parity unpinned: engine vs oracle only); entries: "
                          "16,384 games (the 8-GPU share) as two stream shards "
                          "(us_per_launch = one step) and as one launch, 131,072 (C5 on one "
                          "GPU) as two stream shards and as one launch")
    torch.cuda.empty_cache()
    return out


C5_GLOBAL = 131072   # BASELINE.json configs[4]: 131,072 games on 128x128 over 8 GPUs


def c5_sharded(torch, dist, dev, rank, world, coll_dev, steps, warmup=3, T=128):
    """BASELINE.json configs[4] (C5) as a multi-GPU job: the 131,072 games
    strong-sharded over the ranks by parallel.shard (16,384 per rank at 8
    GPUs), both players StaircaseBots (staircasebot.py:9-21; their descends are
    updater.py:259-296), separation damage off and on.  Every rank runs its
    share as two stream shards (the paired form, as the 1-GPU extra), timed
    like the headline: `warmup` untimed steps, then `steps` 128-tick launches
    bracketed by barrier + synchronize, the max over ranks; then its own
    returns all-gather.  Returns rank 0's block (None elsewhere)."""
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine
    from optimax_rogue_amd.enums import EXT_SEPARATION_DAMAGE
    from optimax_rogue_amd.parallel import gather_returns, shard
    off, n = shard(C5_GLOBAL, rank, world)
    block = {"global_batch": C5_GLOBAL, "ticks_per_step": T, "steps": steps, "warmup": warmup,
             "policy": "2x StaircaseBot", "grid": "128x128", "scaling": "strong",
             "note": "configs[4]: 131,072 games strong-sharded over the ranks by global id; "
                     "value = 131,072 x ticks x steps / max over ranks of the timed span "
                     "(barrier + synchronize on both sides); separation damage = build "
                     "extension EXT_SEPARATION_DAMAGE, sep_period 8"}
    for flag in (0, EXT_SEPARATION_DAMAGE):
        c = EnvConfig.c5()
        if flag:
            c.flags, c.sep_period = flag, 8
        e = StreamShardedEngine(c, n, seed=5, game_offset=off, device=dev, n_streams=2)
        o, a = e.trajectory_buffers(T)
        go = e.rollout_launcher(T, 2, 2, obs=o, act=a)
        e.fork()
        for _ in range(warmup):
            go()
        e.join()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.fork()
        for _ in range(steps):
            go()
        e.join()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        mine = {"rank": rank, "offset": off, "count": n, "elapsed_s": el}
        el_max = el
        ranks = [mine]
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_max = float(t.item())
            ranks = [None] * world
            dist.all_gather_object(ranks, mine)
        rets = gather_returns(e.episode_returns(), C5_GLOBAL)
        shape = e.rollout_shape(2, 2)
        key = "separation_damage_on" if flag else "separation_damage_off"
        block[key] = {"value": C5_GLOBAL * T * steps / el_max, "unit": "env-steps/s",
                      "ms_per_step": el_max / steps * 1e3,
                      "episodes_finished": int(rets[1].sum().item()),
                      "games_per_wave": shape["games_per_wave"],
                      "lanes_per_game": shape["lanes_per_game"], "ranks": ranks}
        del e, o, a, go
        torch.cuda.empty_cache()
    return block if rank == 0 else None


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv, same_device: bool = False) -> int:
    """`--gpus N` outside torchrun: N rank processes, one per GPU, started
    before this process touches the GPU (torch.distributed.run on 127.0.0.1,
    the same form the driver uses), with this script's own arguments; returns
    their exit code.  Rank 0's JSON line goes straight to this stdout.
    torch.cuda.device_count() does not initialize the GPU on this image."""
    import torch
    if not same_device:
        have = torch.cuda.device_count()
        if have < n:
            raise SystemExit(f"--gpus {n}: only {have} GPU(s) visible (use --same-device to "
                             "rehearse N ranks on one card)")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=env)


def launch_check(args) -> None:
    """--launch-check: the rank plumbing alone, no GPU (a CPU test of
    launch_ranks): every rank joins a gloo group, rank 0 prints the line's
    n_gpus and ranks entries."""
    import torch.distributed as dist
    from optimax_rogue_amd.parallel import env_rank, init, shard
    rank, world, local = env_rank()
    init("gloo" if world > 1 else None)
    G = args.global_batch if args.strong else args.batch * world
    offset, count = shard(G, rank, world)
    c5_off, c5_count = shard(C5_GLOBAL, rank, world)
    mine = {"rank": rank, "local_rank": local, "offset": offset, "count": count,
            "c5": {"offset": c5_off, "count": c5_count}}
    ranks = [mine]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    if rank == 0:
        line = {"n_gpus": world, "global_batch": G, "ranks": ranks}
        if world > 1 and not args.no_c5:
            # the configs[4] block the N > 1 line carries (c5_sharded)
            line["c5"] = {"global_batch": C5_GLOBAL,
                          "ranks": [{"rank": x["rank"], **x.pop("c5")} for x in ranks]}
        for x in ranks:
            x.pop("c5", None)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20,
                    help="timed steps; one step = one --chunk-tick rollout launch of every game")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=65536,
                    help="games per GPU (weak scaling, the default)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: a fixed --global-batch split over the ranks by "
                         "parallel.shard (SURVEY s8(d) C4) instead of --batch games per GPU")
    ap.add_argument("--global-batch", type=int, default=524288,
                    help="games of the whole job with --strong (C4: 524,288)")
    ap.add_argument("--chunk", type=int, default=128,
                    help="ticks per step (one rollout launch: the trajectory horizon a learner "
                         "consumes)")
    ap.add_argument("--streams", type=int, default=2,
                    help="shards of the GPU's batch on concurrent HIP streams")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--large", action="store_true",
                    help="extras also time the headline rollout kernel at 2^21 games")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, default) or gloo (multi-rank rehearsal on one GPU)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank uses cuda:0 (rehearsing N ranks on a 1-GPU box)")
    ap.add_argument("--no-c5", action="store_true",
                    help="with N > 1 ranks, skip the configs[4] block (C5: 131,072 StaircaseBot "
                         "games strong-sharded over the ranks, c5_sharded)")
    ap.add_argument("--c5-steps", type=int, default=20,
                    help="timed steps of each C5 block (N > 1 ranks)")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.steps < 1 or args.chunk < 1 or args.warmup < 0 or args.gpus < 1:
        raise SystemExit("--gpus, --steps and --chunk must be >= 1, --warmup >= 0")
    # --gpus N: under torchrun the world size must be N; outside it this
    # process starts the N ranks itself (before any GPU call) and waits
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}")
    elif args.gpus > 1:
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:], args.same_device))
    if args.launch_check:
        return launch_check(args)

    import torch
    import torch.distributed as dist

    from optimax_rogue_amd import EnvConfig, OBS_FIELDS, _lib
    from optimax_rogue_amd.engine import StreamShardedEngine
    from optimax_rogue_amd.parallel import env_rank, gather_returns, init, shard

    rank, world, local = env_rank()
    if args.same_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    init(args.dist_backend if world > 1 else None, dev)
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")

    cfg = EnvConfig.c3()
    # weak scaling: --batch games per GPU; strong: --global-batch games in all
    G = args.global_batch if args.strong else args.batch * world
    offset, B = shard(G, rank, world)
    chunk = args.chunk
    # the GPU's games as --streams shards on concurrent HIP streams (the
    # multi-GPU sharding within a device: one shard's launch ramp and tail
    # overlap the others' steady state)
    eng = StreamShardedEngine(cfg, B, seed=3, game_offset=offset, device=dev,
                              n_streams=args.streams)
    obs, act = eng.trajectory_buffers(chunk)
    launch = eng.rollout_launcher(chunk, 1, 1, obs=obs, act=act)
    eng.fork()
    for _ in range(args.warmup):
        launch()
    eng.join()
    # HIP events on the launch stream (torch's current stream, the one the
    # engine launches on), created before the timed region, bracketing the K
    # back-to-back launches
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    eng.fork()
    for _ in range(args.steps):
        launch()
    eng.join()
    e1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rank_elapsed = elapsed
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # every rank's shard and its own timed span (rank 0 reports them)
    mine = {"rank": rank, "offset": offset, "count": B, "elapsed_s": rank_elapsed,
            "device": str(dev)}
    ranks = [mine]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)

    # dominant kernel: the timed rollout launches, per step (one launch per
    # shard, the shards' launches overlapping on their streams).
    # roofline.achieved prices a launch with the bytes the fused kernel must
    # move (its trajectory rows + the state once per launch);
    # SURVEY s8(d)'s per-tick contract figure (106 B/env-step: state re-read
    # and re-written every tick) is reported beside it as contract_*.
    avg_launch_s = e0.elapsed_time(e1) * 1e-3 / args.steps
    materialized = bytes_per_game("rollout", cfg.n_npcs, chunk) * B
    achieved_gbs = materialized / avg_launch_s / 1e9
    contract_bytes = contract_bytes_per_env_step(cfg.n_npcs) * B * chunk
    shape = eng.rollout_shape(1, 1)   # the 2x RandomBot trajectory launches timed above
    lanes = shape["games_per_wave"]
    eng_parts = list(eng.parts)

    # the only collective: all-gather of per-game episode returns (RCCL / xGMI)
    torch.cuda.synchronize()
    g0 = time.perf_counter()
    allrets = gather_returns(eng.episode_returns(), G)
    torch.cuda.synchronize()
    gather_ms = (time.perf_counter() - g0) * 1e3 if world > 1 else None
    episodes = int(allrets[1].sum().item())
    mean_ret = float(allrets[0].sum().item()) / max(1, episodes)

    value = G * chunk * args.steps / elapsed
    # BASELINE.json configs[4] on the same ranks: C5's 131,072 games
    # strong-sharded over them (every rank takes part: barriers, collectives)
    c5 = None
    if world > 1 and not args.no_c5:
        del obs, act, launch, eng
        torch.cuda.empty_cache()
        c5 = c5_sharded(torch, dist, dev, rank, world, coll_dev, args.c5_steps)
    if rank == 0:
        traffic = None
        if os.path.exists(TRAFFIC_FILE):
            tr = json.load(open(TRAFFIC_FILE)).get("rollout", {})
            if tr.get("batch") == B and tr.get("ticks") == chunk \
                    and tr.get("streams") == len(eng_parts) \
                    and tr.get("build_id") == _lib.build_id():
                traffic = tr.get("hbm_bytes_per_step")
        extra = None
        if not args.no_extras and world == 1:
            del obs, act, launch, eng
            torch.cuda.empty_cache()
            extra = extras(torch, cfg, dev, B, cfg.n_npcs, args.large)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(cfg.to_dict(), args.cpu_seconds)
        if args.strong:
            metric = (f"env-steps/sec (whole node) at global batch={G}, 64x64 grid; "
                      "bit-exact vs ref")
            workload = (f"C4 strong scaling: {G} games in all (fixed), sharded by global id "
                        f"over {world} GPU(s)")
        else:
            metric = "env-steps/sec (whole node) at batch=65536, 64x64 grid; bit-exact vs ref"
            workload = f"C3: {args.batch} games/GPU"
        result = {
            "metric": metric,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (Philox-seeded dungeons and RandomBot actions)",
            "config": {
                "workload": f"{workload}, 64x64 grid, 8 NPCs/game, 2x RandomBot, "
                            "Unreachable despawn, max_ticks 1000, autoreset; one step = one "
                            f"{chunk}-tick rollout launch of every game, every tick's "
                            "observation + actions written to HBM",
                "batch_per_gpu": B, "global_batch": G, "grid": "64x64",
                "n_npcs": cfg.n_npcs, "ticks_per_step": chunk, "streams": len(eng_parts),
                "env_steps_per_step": G * chunk, "games_per_wave": lanes,
                "lanes_per_game": shape["lanes_per_game"],
                "nontemporal_stores": shape["nontemporal"],
                "parallelism": f"games sharded by global id over {world} GPU(s)",
                "build_id": _lib.build_id(),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": rollout_kernel_name(cfg.n_npcs, shape),
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "bytes_per_step": materialized,
                "bytes_per_env_step": materialized / (B * chunk),
                "env_steps_per_step": B * chunk,
                "avg_step_us": avg_launch_s * 1e6,
                "launches": args.steps * len(eng_parts),
                "per": f"step = {len(eng_parts)} concurrent launches (one per stream shard) "
                       f"of {chunk} ticks over {B // len(eng_parts)} games each; achieved = "
                       "bytes_per_step / avg_step_us (HIP events around the timed steps)",
                "contract_bytes_per_env_step": contract_bytes_per_env_step(cfg.n_npcs),
                "contract_bytes_per_step": contract_bytes,
                "contract_GBps": contract_bytes / avg_launch_s / 1e9,
                "contract_frac": contract_bytes / avg_launch_s / 1e9 / HBM_PEAK_GBS,
                "note": "achieved = the fused rollout's own algorithmic bytes (56 B observation "
                        "+ 2 B actions per env-step, state read and written once per launch); "
                        "traffic = PMC HBM bytes per launch of this command (profiles/"
                        "traffic.json, same build id); contract_* = SURVEY s8(d)'s per-tick "
                        "106 B/env-step, which counts a state re-read every tick that the "
                        "fused kernel never makes, hence contract_frac can exceed 1",
            },
            "cpu_baseline": cpu,
            "episodes_finished": episodes,
            "mean_return_p1": mean_ret,
            "returns_gather_ms": gather_ms,
            "returns_gather_backend": dist.get_backend() if world > 1 else None,
            "ranks": ranks,
            "extras": extra,
        }
        if world > 1:
            result["c5"] = c5
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
