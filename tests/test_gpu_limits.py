"""Bounded resources fail loudly: an inbox that overflows sets
GM_ERR_INBOX and the context returns GM_ERANGE -- never a silent divergence. The
diagnostics knob GM_INBOX_CAP lowers the compiled capacity (64 lists) so that an ordinary
cluster overflows it on its first ticks; at the real capacity the same runs stay clean.
(The other narrow-layout limit, GM_ERR_LAG -- a present entry lagging > ~126 ticks -- is
not reachable under the protocol: the oracle's largest lag of a present entry at 90-98 %
keyed loss over 300 ticks is 40 ticks)"""
import pytest

from membership import GM_MODE_PARTIAL, GM_MODE_SCALED, GmError, Simulator

pytestmark = pytest.mark.gpu

GM_ERANGE, GM_ERR_INBOX = -4, 1


def first_error(sim, ticks):
    for _ in range(ticks):
        try:
            sim.tick()
            sim.sync()
        except GmError as e:
            return e.code
    return 0


@pytest.mark.parametrize("mode", [GM_MODE_SCALED, GM_MODE_PARTIAL])
@pytest.mark.parametrize("cap", [2, None])
def test_inbox_overflow_fails_loudly(mode, cap, monkeypatch):
    if cap is None:
        monkeypatch.delenv("GM_INBOX_CAP", raising=False)
    else:
        monkeypatch.setenv("GM_INBOX_CAP", str(cap))
    kw = dict(rd_seed=7, init_mode=1, init_t0=8, init_seed=11)
    if mode == GM_MODE_PARTIAL:
        kw.update(view=32, view_seed=5)
    sim = Simulator(512, mode, **kw)
    code = first_error(sim, 6)
    if cap is None:
        assert code == 0 and sim.tick_stats()["err"] == 0
    else:  # Poisson(5) inboxes: some receiver gets more than 2 lists on the first ticks
        assert code == GM_ERANGE
    sim.close()


GM_ERR_ESC = 128


def test_escape_pool_overflow_fails_loudly(monkeypatch):
    """The compact escape storage (gm_scaled.h): a cold start escapes every cell, so a pool smaller
    than the cluster refuses the context; a warm start fits a tiny pool until a crash window
    escapes the crashed nodes' entries (lag > 14 ticks) -- 64 of them per row, more than a
    list's 16 inline cells -- then the tick fails with GM_ERANGE."""
    n = 1024
    monkeypatch.setenv("GM_ESC_CAP", str(n * n // 2))
    with pytest.raises(GmError) as e:
        Simulator(n, GM_MODE_SCALED, rd_seed=7)
    assert e.value.code == GM_ERANGE
    monkeypatch.setenv("GM_ESC_CAP", "64")
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=11)
    assert first_error(sim, 3) == 0
    crash = list(range(3, 1024, 16))  # 64 nodes
    sim.set_failed(crash)
    code = first_error(sim, 30)  # 64 x 960 observers' cells escape ~10 ticks after the crash
    assert code == GM_ERANGE
    sim.close()
    monkeypatch.delenv("GM_ESC_CAP")  # the default pool: the same run stays clean through the removals
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=11)
    assert first_error(sim, 3) == 0
    sim.set_failed(crash)
    assert first_error(sim, 30) == 0 and sim.tick_stats()["err"] == 0
    assert sim.event_totals()["removed"] == 64 * (n - 64)
