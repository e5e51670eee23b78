"""Headroom of the SCALED layout's semantic ceilings under the worst loss the protocol survives
(VERDICT r3 missing 4). The reference stores hb / ts as C `long` (Member.h:62-81) and delivers
every buffered message (EmulNet.cpp:144-177); the byte-cell layout fails loudly (GM_ERANGE) on a
present entry whose heartbeat lags more than 125 ticks (gm_scaled.h), and the inbox holds 64 lists.

The oracle (oracle/ref_cpu.c SCALED, the reference's merge / sweep / draw) runs 1,000 ticks at
95 % and 98 % keyed per-entry loss and records the largest heartbeat lag of any present entry:
a present entry's age is < TREMOVE = 20 and it was raised from a sender entry of age < TFAIL = 5,
so lags stay ~40 ticks -- a third of the ceiling. The inbox depth does not depend on loss (lists
are delivered, their entries lost): it is the max of ~Poisson(5) draws, checked here on the
oracle's own S2 streams via the GPU test's tick_stats at S-A / S-C sizes (test_gpu_limits.py)."""
import numpy as np
import pytest

import oracle_py

LAG_CEILING = 125  # ticks: h = 254 - 2 lag must stay >= 3 (gm_scaled.h, GM_ERR_LAG)


@pytest.mark.parametrize("n,pct", [(128, 95), (128, 98), (256, 95)])
def test_heavy_loss_lag_stays_far_below_the_ceiling(n, pct):
    o = oracle_py.Oracle(n, oracle_py.OC_SCALED, rd_seed=7, drop_pct=pct, drop_from=0, drop_to=1 << 30, drop_seed=5,
                         init_mode=1, init_t0=8, init_seed=11)
    worst = 0
    removed = joined = 0
    for k in range(1000):
        o.tick()
        t = o.time - 1
        for e in o.events():
            removed += e[2] == 2
            joined += e[2] == 1
        if k % 4 == 0:
            hb, _ = o.table()
            present = hb >= 0
            lag = (2 * t - 1 - hb[present]) // 2
            worst = max(worst, int(lag.max()))
    assert removed > 0  # the loss really churns the views: false removals ...
    if pct < 98:
        assert joined > 0  # ... and re-joins (at 98 % every view collapses to self: nobody gossips any more)
    assert worst <= 50, worst          # measured: 40 / 33 / 42 ticks
    assert worst < LAG_CEILING // 2
