#!/usr/bin/env python3
"""Measurement tool: G column-shard contexts of one N cluster on ONE device, ticked
through the in-process loopback collectives (membership.sharded.loopback_tick), to
time the sharded tick's kernels (run under rocprofv3 --kernel-trace --stats). The
collectives are device copies here, not RCCL, so only kernel times carry over."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-membership_amd"))

from membership import GM_MODE_SCALED, Simulator, crash_set, load_library  # noqa: E402
from membership.abi import shard_loopback  # noqa: E402
from membership.sharded import D_FIRST, D_MORE, loopback_tick  # noqa: E402


def serial_tick(sims):
    """loopback_tick with every shard's phase run alone on the device (clean kernel times)."""
    for s in sims:
        s.shard_merge()
        s.sync()
    shard_loopback(sims, 0)
    rnd, d = 0, D_FIRST
    while True:
        for s in sims:
            s.shard_draw(rnd, d)
            s.sync()
        shard_loopback(sims, 1, d)
        pend = [s.shard_accept(d) for s in sims]
        if pend[0] == 0:
            break
        rnd, d = rnd + 1, D_MORE
    for s in sims:
        s.shard_end_tick()
    return rnd + 1


def one_shard(a):
    """--sb: ONE rank-g column shard of the S-B cluster (N = 262,144, G = 8: 262,144 rows x
    32,768 columns) alone on this device, ticked by gm_tick in gm_shard_stub mode (peers'
    counts mirrored, peer-column draws resolved as fresh column ix): the real merge / draw /
    accept kernels at the true shard shape, without the collectives. Prints one JSON line."""
    import json
    n, g, rank = a.cluster or 262144, a.shards, a.rank
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, shard_rank=rank, shard_count=g, init_mode=1, init_t0=8, init_seed=11)
    sim.keep_events(0)
    sim.shard_stub(1)
    crash = crash_set(n, n // 100, 42)
    while sim.time <= a.prologue:
        t = sim.time
        sim.tick()
        if t == 10:
            sim.set_failed(crash)
    for _ in range(3):
        sim.tick()
    sim.sync()
    sim.set_timing(1)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        sim.tick()
    sim.sync()
    dt = (time.perf_counter() - t0) / a.steps
    band_ms = sim.last_kernel_ms()
    st = sim.tick_stats()
    c0, w = sim.shard_layout()
    b_alg = (9 * st["live"] + st["lists"]) * w // 2
    out = {"what": "one S-B column shard alone on one MI355X (gm_shard_stub: collectives replaced by local stand-ins)",
           "n": n, "shards": g, "rank": rank, "columns": w, "ms_per_tick": dt * 1e3, "band_kernel_ms": band_ms,
           "other_kernels_ms": dt * 1e3 - band_ms, "live": st["live"], "lists": st["lists"], "err": st["err"],
           "band_alg_bytes": b_alg, "band_achieved_gbps": b_alg / (band_ms * 1e-3) / 1e9 if band_ms > 0 else None,
           "node_ticks_per_s_if_8_such_gpus": n / (dt if dt > 0 else 1)}
    print(json.dumps(out), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--cluster", type=int, default=0)
    p.add_argument("--shards", type=int, default=8)
    p.add_argument("--rank", type=int, default=3)
    p.add_argument("--prologue", type=int, default=25)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--sb", action="store_true", help="one S-B shard alone on the device (gm_shard_stub)")
    a = p.parse_args()
    load_library()
    if a.sb:
        return one_shard(a)
    a.cluster = a.cluster or 65536
    n, g = a.cluster, a.shards
    sims = [Simulator(n, GM_MODE_SCALED, rd_seed=7, shard_rank=r, shard_count=g, init_mode=1, init_t0=8, init_seed=11)
            for r in range(g)]
    crash = crash_set(n, n // 100, 42)
    while sims[0].time <= a.prologue:
        t = sims[0].time
        loopback_tick(sims)
        if t == 10:
            for s in sims:
                s.set_failed(crash)
    for s in sims:
        s.sync()
    t0 = time.perf_counter()
    rounds = 0
    for _ in range(a.steps):
        rounds += serial_tick(sims)
    for s in sims:
        s.sync()
    dt = (time.perf_counter() - t0) / a.steps
    st = sims[0].tick_stats()
    print(f"N={n} G={g}: {dt * 1e3:.3f} ms/tick (all shards, one device, loopback), draw rounds/tick "
          f"{rounds / a.steps:.2f}, err={st['err']}", flush=True)


if __name__ == "__main__":
    main()
