"""Two PROCESSES, each owning a real libgm SCALED column-shard context on the one GPU of the box,
tick the cluster with the per-tick exchanges (per-row counts all-gather, MAX-allreduce of the
resolved draws, pending-row agreement) done over gloo through the host-collective hook
(gm_shard_export / gm_shard_import; RCCL refuses two ranks on one device). Rank 0 compares every
tick with the single-context kernel: tables, node state, events (VERDICT r3 missing 3 / next 6).
Reference: the BSP tick, Application.cpp:121-164; the draw it shards, MP1Node.cpp:449-489."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("n,world,drop,ncrash", [(777, 2, 20, 24), (600, 3, 0, 300)])
def test_processes_with_real_shard_contexts_match_fused_kernel(n, world, drop, ncrash, tmp_path):
    out = str(tmp_path / "result.json")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 1000),
           os.path.join(HERE, "gloo_shard_worker.py"), str(n), "32", str(drop), str(ncrash), out]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-3000:]
    with open(out) as f:
        res = json.load(f)
    assert res["ok"], res
    assert res["ticks"] == 32 and res["world"] == world
    assert res["err"] == [0] * world and res["ref_err"] == 0
    if ncrash * 2 >= n:  # half the cluster crashed: rows run out of their first 16 draws
        assert max(res["rounds"]) > 1, res["rounds"]
