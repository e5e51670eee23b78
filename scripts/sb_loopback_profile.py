#!/usr/bin/env python3
"""Measurement tool for S-B column shards: G SCALED column-shard contexts of one N cluster on ONE
device, ticked through membership.sharded.loopback_tick (the per-tick exchanges as in-process
device copies / MAX kernels in place of RCCL). The shards run one after the other, so the wall
time per tick is the SUM of the G shards' own costs -- the per-GPU tick of a G-GPU node is about
that / G plus the RCCL collectives (all-gather of 2 x 4 B per row, MAX-allreduce of 4 B x 16 draws
per row). Run under rocprofv3 --kernel-trace --stats for the per-kernel split. The S-A schedule:
warm start, 1 % crash at tick 10, the timed ticks inside the TREMOVE window as in bench.py."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-membership_amd"))

from membership import GM_MODE_SCALED, Simulator, crash_set, load_library  # noqa: E402
from membership.abi import shard_loopback_tick  # noqa: E402
from membership.sharded import loopback_tick  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cluster", type=int, default=262144)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--ticks", type=int, default=20)
    ap.add_argument("--prologue", type=int, default=28)
    ap.add_argument("--pipelined", action="store_true",
                    help="time gm_shard_loopback_tick (the pipelined RCCL tick's chunk order, one stream) "
                         "instead of the phase-API loopback")
    a = ap.parse_args()
    load_library()
    n, G = a.cluster, a.shards
    kw = dict(rd_seed=7, init_mode=1, init_t0=8, init_seed=11)
    sims = [Simulator(n, GM_MODE_SCALED, shard_rank=g, shard_count=G, **kw) for g in range(G)]
    for s in sims:
        s.keep_events(0)
    print(f"created {G} column shards of n={n}", file=sys.stderr, flush=True)
    crash = crash_set(n, int(round(n * 0.01)), 42)
    while sims[0].time <= a.prologue:
        t = sims[0].time
        loopback_tick(sims)
        if t == 10:
            for s in sims:
                s.set_failed(crash)
    for s in sims:
        s.sync()
    rounds = []
    t0 = time.perf_counter()
    for _ in range(a.ticks):
        w = time.perf_counter()
        if a.pipelined:
            shard_loopback_tick(sims)
            rounds.append(1)
        else:
            rounds.append(loopback_tick(sims))
        print(f"tick {sims[0].time - 1}: {(time.perf_counter() - w) * 1e3:.1f} ms", file=sys.stderr, flush=True)
    for s in sims:
        s.sync()
    el = (time.perf_counter() - t0) / a.ticks
    errs = [s.tick_stats()["err"] for s in sims]
    removed = sum(s.event_totals()["removed"] for s in sims)
    print(json.dumps({"n": n, "shards": G, "ticks": a.ticks, "mode": "pipelined" if a.pipelined else "phase API", "ms_per_tick_all_shards_serialised": el * 1e3,
                      "ms_per_shard_tick": el * 1e3 / G, "draw_rounds": rounds, "err": errs,
                      "removed_total": removed}), flush=True)


if __name__ == "__main__":
    main()
