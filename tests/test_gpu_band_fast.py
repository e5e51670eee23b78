"""gm_s_band's fast path (B = 1024: merge and sweep on the stored bytes, SWAR counts, the rare
cells redone one by one; gm_scaled.hip unit_fast) against the general path (GM_BAND_FAST=0),
tick by tick: events in order, tick statistics, membership tables, msgcount. The schedules drive
every branch of the fast path: the crash window (cells aging to 15 escape, then TREMOVE removes
them: the per-cell pass, the quick case of a slice whose escapes only age, and the removal events), cold start (every cell escaped: escape lists read
back), a loss window (DROP ticks take the general kernel; the ticks after it deliver stale and
lagging entries, so units are handed back to the general path), and column shards. The oracle
parity of both paths is test_gpu_scaled.py's (bands 1024 included). Reference: the merge
MP1Node.cpp:278-299, the sweep MP1Node.cpp:426-444, sendMemberList MP1Node.cpp:360-395."""
import numpy as np
import pytest

from membership import GM_MODE_SCALED, Simulator, crash_set
from membership.sharded import loopback_tick

pytestmark = pytest.mark.gpu


def _pair(monkeypatch, n, **kw):
    monkeypatch.setenv("GM_BAND_FAST", "0")
    gen = Simulator(n, GM_MODE_SCALED, **kw)
    monkeypatch.setenv("GM_BAND_FAST", "1")
    fast = Simulator(n, GM_MODE_SCALED, **kw)
    monkeypatch.delenv("GM_BAND_FAST")
    return gen, fast


def _same_tables(a, b, n, t):
    ha, ta = a.read_table(0, n)
    hb, tb = b.read_table(0, n)
    assert np.array_equal(ha, hb) and np.array_equal(ta, tb), f"tables differ at tick {t}"


@pytest.mark.parametrize("init_mode,loss,ncrash", [(1, 0, 41), (1, 0, 20), (0, 0, 41), (1, 1, 41), (0, 2, 41)])
def test_fast_path_matches_general_path(monkeypatch, init_mode, loss, ncrash):
    # ncrash 20 (1 %, S-A's share): ~10 escaped cells per 1024-column slice, so most units of the
    # crash window take the fast path's quick case (inline list, stale, undelivered; removals by the
    # gone-entry loop); 41 (2 %): ~20 per slice, past the inline slot, the park path
    n = 2048
    kw = dict(rd_seed=7, init_mode=init_mode, init_t0=8 if init_mode else 0, init_seed=11, band=1024)
    if loss == 1:  # 40 % loss for ticks 12..19: stale and lagging entries afterwards
        kw.update(drop_pct=40, drop_from=12, drop_to=20, drop_seed=5)
    elif loss == 2:  # one keyed-loss tick between fast ticks of the same parity (the hand-back
        # list's count of tick 14 must not survive into tick 16), after a cold start's hand-backs
        kw.update(drop_pct=20, drop_from=15, drop_to=16, drop_seed=5)
    gen, fast = _pair(monkeypatch, n, **kw)
    for s in (gen, fast):
        s.msgcount_record(64)
    crash = crash_set(n, ncrash, 42)
    for _ in range(56):
        t = fast.time
        gen.tick()
        fast.tick()
        if t == 10:
            gen.set_failed(crash)
            fast.set_failed(crash)
        assert gen.drain_events() == fast.drain_events(), f"events differ at tick {t}"
        assert gen.tick_stats() == fast.tick_stats(), f"tick stats differ at tick {t}"
        if t % 4 == 0 or 24 <= t <= 40:
            _same_tables(gen, fast, n, t)
        (sg, rg), (sf, rf) = gen.msgcount(t), fast.msgcount(t)
        assert np.array_equal(sg, sf) and np.array_equal(rg, rf), f"msgcount differs at tick {t}"
    assert fast.tick_stats()["err"] == 0


def test_fast_path_column_shards_match_general_path(monkeypatch):
    # G = 2 column shards (loopback exchange), fast path on vs off: the shards' own columns
    # (c0 offsets, the own cell in one shard only) through the same schedule
    n, G = 4096, 2
    kw = dict(rd_seed=7, init_mode=1, init_t0=8, init_seed=11, band=1024)
    sims = {}
    for fast in (0, 1):
        monkeypatch.setenv("GM_BAND_FAST", str(fast))
        sims[fast] = [Simulator(n, GM_MODE_SCALED, shard_rank=g, shard_count=G, **kw) for g in range(G)]
    monkeypatch.delenv("GM_BAND_FAST")
    crash = crash_set(n, 41, 42)
    for _ in range(44):
        t = sims[1][0].time
        for f in (0, 1):
            loopback_tick(sims[f])
            if t == 10:
                for s in sims[f]:
                    s.set_failed(crash)
        for g in range(G):
            assert sims[0][g].drain_events() == sims[1][g].drain_events(), f"events differ at tick {t}, shard {g}"
            if t % 6 == 0 or 30 <= t <= 38:
                w = sims[0][g].shard_layout()[1]
                for r in (0, 1, 2047, 2048, n - 1):
                    a = sims[0][g].read_row(r, 0, w)
                    b = sims[1][g].read_row(r, 0, w)
                    assert all(np.array_equal(x, y) for x, y in zip(a, b)), f"row {r} differs at tick {t}"
    for g in range(G):
        assert sims[1][g].tick_stats()["err"] == 0
