#!/usr/bin/env python3
"""Measurement tool for S-C row shards: G PARTIAL row-shard contexts of one N cluster on
ONE device, ticked through gm_partial_loopback_tick (the exchange as device copies in
the all-to-allv layout). Reports the wall time per tick (the G shards serialised) and the
bytes each shard receives per tick -- the xGMI volume of the RCCL exchange. Run under
rocprofv3 --kernel-trace --stats for per-shard kernel times."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-membership_amd"))

from membership import GM_MODE_PARTIAL, Simulator, crash_set, load_library  # noqa: E402
from membership.abi import partial_loopback_tick  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cluster", type=int, default=1 << 24)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--ticks", type=int, default=8)
    ap.add_argument("--prologue", type=int, default=14)
    a = ap.parse_args()
    load_library()
    n, G = a.cluster, a.shards
    kw = dict(rd_seed=7, view=32, view_seed=5, init_mode=1, init_t0=8, init_seed=11, drop_pct=5, drop_from=0,
              drop_to=1 << 20, drop_seed=42)
    sims = [Simulator(n, GM_MODE_PARTIAL, shard_rank=g, shard_count=G, **kw) for g in range(G)]
    for s in sims:
        s.keep_events(0)  # join records are counted on the device, not staged on the host
    print(f"created {G} shards of n={n}", file=sys.stderr, flush=True)
    crash = crash_set(n, n // 100, 42)
    while sims[0].time <= a.prologue:
        t = sims[0].time
        w = time.perf_counter()
        partial_loopback_tick(sims)
        print(f"prologue tick {t}: {(time.perf_counter() - w) * 1e3:.1f} ms", file=sys.stderr, flush=True)
        if t == 10:
            for s in sims:
                s.set_failed(crash)
    t0 = time.perf_counter()
    for _ in range(a.ticks):
        partial_loopback_tick(sims)
    for s in sims:
        s.sync()
    el = (time.perf_counter() - t0) / a.ticks
    rb = [s.exchange_bytes() for s in sims]
    print(json.dumps({"n": n, "shards": G, "ms_per_tick_all_shards_serialised": el * 1e3,
                      "recv_bytes_per_shard_per_tick": rb, "recv_mb_mean": sum(rb) / G / 1e6}), flush=True)


if __name__ == "__main__":
    main()
