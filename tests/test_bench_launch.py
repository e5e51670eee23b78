"""bench.py --gpus G launches G ranks by itself (the driver's `python3 bench.py --gpus N` form):
torch.distributed.run as a child process, before anything loads libgm. --dry-launch stops each
rank after the gloo rendezvous, so this runs on CPU. Reference: the BSP tick that makes the
shards legal, Application.cpp:121-164."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(extra)
    return env


def _run(args, **extra):
    return subprocess.run([sys.executable, BENCH] + args, env=_env(**extra), capture_output=True, text=True,
                          timeout=240)


def test_gpus_2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--dry-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints ONE JSON line
    out = json.loads(lines[0])
    assert out["dry_launch"] and out["n_gpus"] == 2
    ranks = out["ranks"]
    assert sorted(x["rank"] for x in ranks) == [0, 1]
    assert all(x["world_size"] == 2 for x in ranks)
    assert sorted(x["local_rank"] for x in ranks) == [0, 1]
    assert len({x["pid"] for x in ranks}) == 2  # two processes
    assert all(x["master"].startswith("127.0.0.1:") for x in ranks)
    assert out["companion"] == "S-B"  # every S-A line of a --gpus sweep also measures the S-B cluster


def test_gpus_1_stays_one_process():
    r = _run(["--gpus", "1", "--dry-launch", "--scenario", "S-B"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip())
    assert out["n_gpus"] == 1 and out["scenario"] == "S-B"
    assert [x["world_size"] for x in out["ranks"]] == [1]
    assert out["ranks"][0]["pid"] != os.getpid()
    assert out["companion"] is None  # S-B is the cluster itself


def test_no_companion_flag():
    r = _run(["--dry-launch", "--no-companion"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip())["companion"] is None


def test_world_size_mismatch_fails_loudly():
    r = _run(["--gpus", "1", "--dry-launch"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr


def test_gpus_zero_rejected():
    r = _run(["--gpus", "0", "--dry-launch"])
    assert r.returncode == 2
