"""GPU: the sharded HIP path.  Two (and four) torchrun ranks on cuda:0 (gloo), each
stepping its parallel.shard() of the global batch with BatchedEngine at its
game_offset, all-gathered with parallel.gather_returns, equal a single
BatchedEngine over the whole batch -- for even and odd global batches
(bit-identical for any rank count).
(The 8-GPU RCCL run is the driver's; this covers the same code path on one
card.)"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CFG = dict(width=64, height=64, n_npcs=8, max_ticks=90)
TICKS = 240


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("ranks,global_batch", [(2, 6000), (2, 6001), (4, 4097)])
def test_ranks_equal_one_process(tmp_path, ranks, global_batch):
    import torch
    from dist_worker import rows_of
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    out = str(tmp_path / "gathered.npy")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(HERE, "dist_worker.py"), "--global-batch", str(global_batch),
           "--ticks", str(TICKS), "--cfg", json.dumps(CFG), "--policy", "1,2", "--out", out]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    got = np.load(out)
    eng = BatchedEngine(EnvConfig.from_dict(CFG), global_batch, seed=23,
                        device=torch.device("cuda", 0))
    eng.rollout(TICKS, 1, 2)
    want = rows_of(eng).cpu().numpy()
    assert got.shape == want.shape
    assert np.array_equal(got, want)
    assert want[1].sum() >= global_batch  # every game finished an episode


def test_c4_eight_shards_equal_whole_batch():
    """BASELINE configs[3] (C4) at its full size: 524,288 games as the eight
    per-GPU shards of parallel.shard (each a BatchedEngine at its game_offset,
    here on one card) equal one engine over all 524,288 games -- state, and
    the per-game returns gather_returns would assemble in global id order."""
    import torch
    from golden_util import STATE_KEYS
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    from optimax_rogue_amd.parallel import shard
    G, T, dev = 524288, 64, torch.device("cuda", 0)
    cfg = EnvConfig.c4()
    cfg.max_ticks = 40          # episodes end inside the window
    whole = BatchedEngine(cfg, G, seed=4, device=dev)
    whole.rollout(T, 1, 1)
    want = whole.snapshot()
    want_ret = whole.episode_returns().cpu().numpy()
    del whole
    parts, rets = [], []
    for r in range(8):
        off, cnt = shard(G, r, 8)
        e = BatchedEngine(cfg, cnt, seed=4, game_offset=off, device=dev)
        e.rollout(T, 1, 1)
        parts.append(e.snapshot())
        rets.append(e.episode_returns().cpu().numpy())
        del e
    for k in STATE_KEYS:
        got = np.concatenate([p[k] for p in parts], axis=np.asarray(want[k]).ndim - 1)
        assert np.array_equal(got, want[k]), k
    assert np.array_equal(np.concatenate(rets, axis=1), want_ret)
    assert want_ret[1].sum() >= G   # every game finished at least one episode
    torch.cuda.synchronize()


def test_bench_gpus_2_runs_two_ranks():
    """`python bench.py --gpus 2` (no torchrun around it) starts two ranks by
    itself: here both on cuda:0 with the gloo gather (--same-device; RCCL takes
    one rank per device), as the driver's SCALE run does with one GPU each.
    The line reports n_gpus 2, both ranks' shards and the returns gather,
    and the configs[4] (C5) block timed on the same ranks."""
    root = os.path.dirname(HERE)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--same-device", "--dist-backend", "gloo", "--batch", "8192",
                        "--steps", "2", "--warmup", "1", "--no-extras", "--no-cpu-baseline",
                        "--c5-steps", "2"],
                       env=env, capture_output=True, text=True, timeout=110, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 16384
    assert [(x["rank"], x["offset"], x["count"]) for x in line["ranks"]] == \
        [(0, 0, 8192), (1, 8192, 8192)]
    assert line["returns_gather_ms"] is not None and line["returns_gather_backend"] == "gloo"
    assert line["value"] > 0
    # configs[4]: C5's 131,072 StaircaseBot games strong-sharded over the two
    # ranks, separation damage off and on, max over ranks
    c5 = line["c5"]
    assert c5["global_batch"] == 131072 and c5["steps"] == 2
    for key in ("separation_damage_off", "separation_damage_on"):
        b = c5[key]
        assert [(x["rank"], x["offset"], x["count"]) for x in b["ranks"]] == \
            [(0, 0, 65536), (1, 65536, 65536)]
        assert b["value"] > 0 and b["lanes_per_game"] == 2
        assert abs(b["ms_per_step"] * 1e-3 * 2 - max(x["elapsed_s"] for x in b["ranks"])) < 1e-6


def test_rccl_process_group_on_the_device():
    """The nccl (= RCCL) path of parallel.init / gather_returns on hardware:
    a process group bound to cuda:0 (init_process_group's device_id), the
    all-gather run on device tensors (no host round trip), the result equal
    to the input in global id order.  One rank: the box has one GPU and RCCL
    takes one rank per device; the 2/4/8-rank RCCL runs are the driver's
    SCALE bench, whose code path this is."""
    code = (
        "import sys, torch, torch.distributed as dist\n"
        f"sys.path.insert(0, {os.path.dirname(HERE)!r})\n"
        "from optimax_rogue_amd.parallel import init, gather_returns\n"
        "dev = torch.device('cuda', 0)\n"
        "torch.cuda.set_device(dev)\n"
        "init('nccl', dev, force=True)\n"
        "assert dist.get_backend() == 'nccl', dist.get_backend()\n"
        "x = torch.arange(2 * 1001, dtype=torch.int32, device=dev).reshape(2, 1001)\n"
        "y = gather_returns(x, 1001)\n"
        "torch.cuda.synchronize()\n"
        "assert y.device == dev and torch.equal(x, y)\n"
        "dist.destroy_process_group()\n"
        "print('RCCL_OK')\n")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0 and "RCCL_OK" in r.stdout, (r.stdout + r.stderr)[-3000:]
