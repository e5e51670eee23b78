"""Worker of tests/test_gpu_gloo_shards.py (one process per column shard, launched by
torch.distributed.run): each rank owns a REAL libgm SCALED shard context on the box's GPU and
ticks it with membership.sharded.host_tick -- the exchanges cross the process boundary over gloo
through gm_shard_export / gm_shard_import. Rank 0 also runs the single-context (fused) tick of
the same cluster and compares, every tick, the merged tables + node state and the events.
Reference: the BSP tick that makes the shards legal, Application.cpp:121-164."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "distributed-membership_amd"))


def main():
    n, ticks, drop, ncrash, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    from membership import GM_MODE_SCALED, Simulator, crash_set, load_library
    from membership.sharded import host_tick
    load_library()  # libgm (system HIP runtime + RCCL) before torch brings its own copies
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    kw = dict(rd_seed=7, drop_pct=drop, drop_from=3, drop_to=1 << 20, drop_seed=42, init_mode=1, init_t0=6,
              init_seed=5)
    sim = Simulator(n, GM_MODE_SCALED, shard_rank=rank, shard_count=world, **kw)
    ref = Simulator(n, GM_MODE_SCALED, **kw) if rank == 0 else None
    c0, w = sim.shard_layout()
    crash = crash_set(n, ncrash, 42)
    result = {"ok": True, "ticks": 0, "rounds": [], "world": world}
    for _ in range(ticks):
        t = sim.time
        result["rounds"].append(host_tick(sim, dist))
        if ref is not None:
            ref.tick()
        if t == 8:
            sim.set_failed(crash)
            if ref is not None:
                ref.set_failed(crash)
        hb, ts = sim.read_table()
        nodes = sim.read_nodes()
        ev = sim.drain_events()
        parts = [None] * world
        dist.all_gather_object(parts, (c0, w, hb, ts, nodes, ev))
        if rank == 0:
            parts.sort(key=lambda p: p[0])
            mhb = np.concatenate([p[2] for p in parts], axis=1)
            mts = np.concatenate([p[3] for p in parts], axis=1)
            owner = np.zeros(n, dtype=int)
            for g, p in enumerate(parts):
                owner[p[0]:p[0] + p[1]] = g
            st = np.stack([p[4] for p in parts])[owner, np.arange(n)]
            rhb, rts = ref.read_table()
            same = (np.array_equal(mhb, rhb) and np.array_equal(mts, rts) and np.array_equal(st, ref.read_nodes())
                    and sorted(e for p in parts for e in p[5]) == sorted(ref.drain_events()))
            if not same:
                result.update(ok=False, bad_tick=t)
        flag = torch.tensor([0 if result["ok"] else 1])
        dist.broadcast(flag, 0)
        result["ticks"] += 1
        if int(flag):
            break
    errs = [None] * world
    dist.all_gather_object(errs, sim.tick_stats()["err"])
    result["err"] = errs
    if rank == 0:
        result["ref_err"] = ref.tick_stats()["err"]
        with open(out, "w") as f:
            json.dump(result, f)
    sim.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
