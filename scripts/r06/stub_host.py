#!/usr/bin/env python3
"""Diagnostics: host time per gm_tick call of the S-A stub shard (rank 3 of 8) vs the tick period,
to tell a host-bound tick (the host enqueues slower than the GPU runs) from a device-bound one."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-membership_amd"))
from membership import GM_MODE_SCALED, Simulator, crash_set  # noqa: E402

n, g, rank = int(sys.argv[1]) if len(sys.argv) > 1 else 65536, 8, 3
sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, shard_rank=rank, shard_count=g, init_mode=1, init_t0=8, init_seed=11)
sim.keep_events(0)
sim.shard_stub(1)
crash = crash_set(n, n // 100, 42)
while sim.time <= 25:
    t = sim.time
    sim.tick()
    if t == 10:
        sim.set_failed(crash)
sim.sync()
calls = []
t0 = time.perf_counter()
for _ in range(20):
    a = time.perf_counter()
    sim.tick()
    calls.append(time.perf_counter() - a)
sim.sync()
dt = (time.perf_counter() - t0) / 20
calls.sort()
print(f"n={n} period {dt * 1e3:.4f} ms; host per gm_tick call: median {calls[10] * 1e3:.4f} ms, "
      f"min {calls[0] * 1e3:.4f}, max {calls[-1] * 1e3:.4f}")
