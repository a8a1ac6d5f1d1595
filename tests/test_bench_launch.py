"""CPU: bench.py's rank plumbing.  `python bench.py --gpus N` outside torchrun
starts N rank processes itself (torch.distributed.run on 127.0.0.1) and rank
0 reports every rank's shard; under torchrun a --gpus / WORLD_SIZE mismatch
is refused.  `--launch-check` stops each rank before any GPU work (gloo
group, shard, all_gather_object), so this runs without a GPU; the same launch
with the engine is the GPU rehearsal (tests/test_gpu_distributed.py)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=120):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT)


def _line(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_starts_n_ranks(n):
    r = _run(["--gpus", str(n), "--same-device", "--launch-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["n_gpus"] == n
    assert out["global_batch"] == 65536 * n          # weak scaling: --batch per GPU
    assert [x["rank"] for x in out["ranks"]] == list(range(n))
    assert [x["local_rank"] for x in out["ranks"]] == list(range(n))
    assert [x["offset"] for x in out["ranks"]] == [65536 * k for k in range(n)]


def test_gpus_n_carries_the_c5_block():
    """configs[4] (C5: 131,072 StaircaseBot games over 8 GPUs) on the N > 1
    line: every rank's strong share of the 131,072 games by parallel.shard;
    a single rank has none (its C5 figures are the 1-GPU extras)."""
    r = _run(["--gpus", "2", "--same-device", "--launch-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["c5"]["global_batch"] == 131072
    assert [(x["rank"], x["offset"], x["count"]) for x in out["c5"]["ranks"]] == \
        [(0, 0, 65536), (1, 65536, 65536)]
    r = _run(["--gpus", "3", "--same-device", "--launch-check"])
    out = _line(r.stdout)
    assert [(x["offset"], x["count"]) for x in out["c5"]["ranks"]] == \
        [(0, 43691), (43691, 43691), (87382, 43690)]
    out = _line(_run(["--gpus", "1", "--launch-check"]).stdout)
    assert "c5" not in out
    out = _line(_run(["--gpus", "2", "--same-device", "--launch-check", "--no-c5"]).stdout)
    assert "c5" not in out


def test_gpus_n_strong_shards_the_global_batch():
    r = _run(["--gpus", "2", "--same-device", "--launch-check", "--strong",
              "--global-batch", "1001"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["n_gpus"] == 2
    assert [(x["offset"], x["count"]) for x in out["ranks"]] == [(0, 501), (501, 500)]


def test_gpus_1_is_one_process():
    r = _run(["--gpus", "1", "--launch-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["n_gpus"] == 1 and len(out["ranks"]) == 1


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "4", "--launch-check"],
             {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_more_gpus_than_visible_refused():
    """No GPU in this container: --gpus 2 without --same-device is refused
    before any rank starts."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("enough GPUs visible")
    r = _run(["--gpus", "2", "--launch-check"])
    assert r.returncode != 0 and "GPU(s) visible" in r.stderr


def test_cpu_quota_and_physical_cores():
    """The whole-host CPU baseline's host facts: the physical core count (lscpu
    (core, socket) pairs) is positive and at most the visible CPUs, and the
    cgroup CPU quota is either absent (None) or a positive CPU count."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    phys = bench.physical_cores()
    assert 1 <= phys <= (os.cpu_count() or phys)
    q = bench.cpu_quota()
    assert q is None or q > 0
