"""PARTIAL-view parity (scenario S-C semantics, oracle/ref_cpu.c "PARTIAL"): the HIP
V-entry-view tick against the oracle, tick by tick -- every node's list (dump),
node state and the join / remove event set -- with a crash set and keyed drops."""
import pytest

import oracle_py
from golden_util import digest64
from membership import GM_EV_JOINED, GM_MODE_PARTIAL, Simulator, crash_set

pytestmark = pytest.mark.gpu


def run_pair(n, v, ticks, crash_tick=-1, crash_count=0, drop_pct=0, drop_from=0, drop_to=0, seed=42):
    kw = dict(rd_seed=7, view_seed=5, init_t0=8, init_seed=11)
    ora = oracle_py.PartialOracle(n, v=v, crash_tick=crash_tick, crash_count=crash_count, crash_seed=seed,
                                  drop_pct=drop_pct, drop_from=drop_from, drop_to=drop_to, drop_seed=seed, **kw)
    sim = Simulator(n, GM_MODE_PARTIAL, rd_seed=7, view=v, view_seed=5, init_mode=1, init_t0=8, init_seed=11,
                    drop_pct=drop_pct, drop_from=drop_from, drop_to=drop_to, drop_seed=seed)
    crash = crash_set(n, crash_count, seed)
    assert sim.dump_tables() == ora.dump(), "initial views differ"
    joins = removes = 0
    for _ in range(ticks):
        t = sim.time
        assert ora.time == t
        ora.tick()
        sim.tick()
        if t == crash_tick:
            sim.set_failed(crash)
        ev = [(e[0], e[1], 1 if e[2] == GM_EV_JOINED else 2, e[3]) for e in sim.drain_events()]
        assert ev == ora.events(), f"events differ at tick {t}"
        joins += sum(e[2] == 1 for e in ev)
        removes += sum(e[2] == 2 for e in ev)
        assert digest64(sim.dump_tables()) == digest64(ora.dump()), f"views differ at tick {t}"
    assert sim.tick_stats()["err"] == 0
    return joins, removes


@pytest.mark.parametrize("n,v", [(64, 8), (300, 16), (1000, 32)])
def test_partial_matches_oracle(n, v):
    joins, _ = run_pair(n, v, 36, crash_tick=12, crash_count=max(1, n // 50))
    assert joins > 0


def test_partial_with_drops_matches_oracle():
    run_pair(400, 32, 40, crash_tick=10, crash_count=8, drop_pct=30, drop_from=5, drop_to=30)


def test_partial_sparse_views_remove_stale_entries():
    # heavy drops starve views of fresh entries: entries age past TREMOVE and are removed
    _, removes = run_pair(128, 4, 60, drop_pct=90, drop_from=2, drop_to=60)
    assert removes > 0


def test_partial_large_cluster_matches_oracle():
    # N = 131,072: ~1.4 % of the nodes receive more than P_KSMALL = 10 lists per tick
    # (the big-table kernel), ~2 per tick more than P_KP = 16 (the lowest-sender rule);
    # 5 % drops as in S-C, a crash set inside the window
    n, v = 131072, 32
    kw = dict(rd_seed=7, view_seed=5, init_t0=8, init_seed=11)
    ora = oracle_py.PartialOracle(n, v=v, crash_tick=10, crash_count=1311, crash_seed=42, drop_pct=5, drop_from=0,
                                  drop_to=1000, drop_seed=42, **kw)
    sim = Simulator(n, GM_MODE_PARTIAL, rd_seed=7, view=v, view_seed=5, init_mode=1, init_t0=8, init_seed=11,
                    drop_pct=5, drop_from=0, drop_to=1000, drop_seed=42)
    crash = crash_set(n, 1311, 42)
    for step in range(6):
        t = sim.time
        ora.tick()
        sim.tick()
        if t == 10:
            sim.set_failed(crash)
        ev = [(e[0], e[1], 1 if e[2] == GM_EV_JOINED else 2, e[3]) for e in sim.drain_events()]
        assert ev == ora.events(), f"events differ at tick {t}"
        if step in (2, 5):
            assert digest64(sim.dump_tables()) == digest64(ora.dump()), f"views differ at tick {t}"
    st = sim.tick_stats()
    assert st["err"] == 0 and st["max_inbox"] == 16, st
