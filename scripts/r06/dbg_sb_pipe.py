#!/usr/bin/env python3
"""Diagnostics: the full-size S-B pipelined loopback (G = 8 column shards of N = 262,144 on one
device, gm_shard_loopback_tick) tick by tick, printing each shard's error bits after every tick;
stops at the first error. Run with GM_LIBRARY pointing at a build that prints unresolved draws."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "distributed-membership_amd"))
from membership import GM_MODE_SCALED, GmError, Simulator, crash_set  # noqa: E402
from membership.abi import shard_loopback_tick  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
G = int(sys.argv[2]) if len(sys.argv) > 2 else 8
kw = dict(rd_seed=7, init_mode=1, init_t0=8, init_seed=11)
crash = crash_set(n, int(round(n * 0.01)), 42)
shards = [Simulator(n, GM_MODE_SCALED, shard_rank=g, shard_count=G, **kw) for g in range(G)]
for s in shards:
    s.keep_events(0)
print("layout", [s.shard_layout() for s in shards], flush=True)
while shards[0].time <= 48:
    t = shards[0].time
    t0 = time.time()
    try:
        shard_loopback_tick(shards)
    except GmError as e:
        print(f"tick {t}: {e}", flush=True)
        print("err", [s.tick_stats()["err"] for s in shards], flush=True)
        break
    if t == 10:
        for s in shards:
            s.set_failed(crash)
    errs = [s.tick_stats()["err"] for s in shards]
    print(f"tick {t}: err {errs} {time.time() - t0:.2f}s", flush=True)
    if any(errs):
        break
