"""The SCALED oracle's state between two ticks is exactly (tables, heartbeat counters, crash flags,
last targets): an oracle loaded with another's state continues identically (oc_load_scaled). This is
what lets the long CPU baseline run (scripts/cpu_hour.py) start its timed ticks from a state the HIP
path reached (tests/test_gpu_scaled.py::test_oracle_continues_from_gpu_state checks that leg)."""
import numpy as np
import pytest

import oracle_py
from golden_util import digest64


@pytest.mark.parametrize("n,drop", [(96, 0), (130, 30)])
def test_oracle_continues_from_loaded_state(n, drop):
    kw = dict(rd_seed=7, init_mode=1, init_t0=8, init_seed=11, crash_tick=10, crash_count=max(2, n // 20),
              crash_seed=42, drop_pct=drop, drop_from=0, drop_to=1000, drop_seed=5)
    a = oracle_py.Oracle(n, oracle_py.OC_SCALED, **kw)
    while a.time <= 24:  # through the crash and into the TFAIL / TREMOVE window
        a.tick()
    hb, ts = a.table()
    st = a.nodes()
    tg, cnt = a.targets()
    b = oracle_py.Oracle(n, oracle_py.OC_SCALED, **kw)  # a fresh context (its own tick-9 state), overwritten
    b.load_state(a.time, hb, ts, st[:, 3], st[:, 2], tg, cnt)
    assert b.time == a.time and digest64(b.dump()) == digest64(a.dump())
    for _ in range(14):
        t = a.time
        a.tick()
        b.tick()
        assert b.events() == a.events(), f"events differ at tick {t}"
        assert digest64(b.dump()) == digest64(a.dump()), f"tables differ at tick {t}"
    (tb, cb), (ta, ca) = b.targets(), a.targets()
    used = np.arange(5)[None, :] < ca[:, None]  # slots past a node's count hold older ticks' targets
    assert np.array_equal(cb, ca) and np.array_equal(np.where(used, tb, 0), np.where(used, ta, 0))
