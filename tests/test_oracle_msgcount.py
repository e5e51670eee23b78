"""The oracle's msgcount analogue for SCALED / PARTIAL (oc_last_msgcount / op_last_msgcount),
checked against conservation laws on CPU: without loss every entry a node puts on the wire
at tick t arrives at t+1 (EmulNet delivers everything in its buffer, EmulNet.cpp:144-177);
with keyed loss p % the arrivals are the sends thinned by ~p %."""
import numpy as np
import pytest

import oracle_py


def series(ora, ticks):
    out = []
    for _ in range(ticks):
        ora.tick()
        out.append(ora.last_msgcount())
    return out


@pytest.mark.parametrize("drop", [0, 30])
def test_scaled_counts_conserve_entries(drop):
    ora = oracle_py.Oracle(256, oracle_py.OC_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=11,
                           drop_pct=drop, drop_from=0, drop_to=1 << 30, drop_seed=5)
    s = series(ora, 12)
    for t in range(len(s) - 1):
        sent, recv = s[t][0].sum(), s[t + 1][1].sum()
        assert sent > 0
        if drop == 0:
            assert recv == sent
        else:
            assert abs(recv / sent - (1 - drop / 100)) < 0.02
    fresh = s[-1][0] // 5  # every live node of a warm, loss-free cluster gossips to 5 targets
    if drop == 0:
        assert np.all(s[-1][0] % 5 == 0) and np.all(fresh > 0)


@pytest.mark.parametrize("drop", [0, 20])
def test_partial_counts_conserve_entries(drop):
    ora = oracle_py.PartialOracle(2000, v=32, rd_seed=7, view_seed=5, init_t0=8, init_seed=11, drop_pct=drop,
                                  drop_from=0, drop_to=1 << 20, drop_seed=42)
    s = series(ora, 8)
    for t in range(len(s) - 1):
        sent, recv = s[t][0].sum(), s[t + 1][1].sum()
        # a node merges at most 16 lists: the (rare) lists beyond that are sent but not received
        assert 0 < recv <= sent
        assert recv / sent > (1 - drop / 100) - 0.03
