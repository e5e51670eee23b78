"""Bounded resources fail loudly: an inbox that overflows sets
GM_ERR_INBOX and the context returns GM_ERANGE -- never a silent divergence. The
diagnostics knob GM_INBOX_CAP lowers the compiled capacity (64 lists) so that an ordinary
cluster overflows it on its first ticks; at the real capacity the same runs stay clean.
The other narrow-layout limit, GM_ERR_LAG -- a present entry lagging > 125 ticks -- is not
reachable under the protocol (the oracle's largest lag at 95 / 98 % keyed loss over 1,000 ticks
is 40 / 33 ticks, tests/test_oracle_limits.py); GM_LAG_CAP lowers it to show that it too fails
loudly."""
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


GM_ERR_LAG = 64


@pytest.mark.parametrize("cap,fails", [(20, True), (45, False)])
def test_lag_ceiling_fails_loudly(cap, fails, monkeypatch):
    """The heartbeat-lag ceiling of the byte-cell layout (125 ticks, gm_scaled.h) lowered by the
    diagnostics knob GM_LAG_CAP: a crashed node's entries lag L0 + age ticks until their TREMOVE
    removal at age 20 (L0 <= ~5 at N = 1,024), so a 20-tick ceiling is crossed in the crash
    window and the tick returns GM_ERANGE (GM_ERR_LAG), while a 45-tick one never is. The
    protocol's own worst case is ~40 ticks at 95 % loss (tests/test_oracle_limits.py)."""
    monkeypatch.setenv("GM_LAG_CAP", str(cap))
    n = 1024
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=11)
    assert first_error(sim, 3) == 0
    sim.set_failed(list(range(5, n, 64)))
    code = first_error(sim, 30)
    if fails:
        assert code == GM_ERANGE
    else:
        assert code == 0 and sim.tick_stats()["err"] == 0
        assert sim.event_totals()["removed"] == 16 * (n - 16)
    sim.close()


def test_heavy_loss_long_run_stays_inside_the_ceilings():
    """95 % keyed loss for 400 ticks at N = 2,048: false removals and re-joins churn every row, the
    lags and the escape pools stay bounded (no GM_ERR_LAG / GM_ERR_ESC) and no inbox nears 64."""
    n = 2048
    sim = Simulator(n, GM_MODE_SCALED, rd_seed=7, init_mode=1, init_t0=8, init_seed=11, drop_pct=95, drop_from=0,
                    drop_to=1 << 20, drop_seed=5)
    sim.keep_events(0)
    worst_inbox = 0
    for _ in range(400):
        sim.tick()
        worst_inbox = max(worst_inbox, sim.tick_stats()["max_inbox"])
    st = sim.tick_stats()
    tot = sim.event_totals()
    assert st["err"] == 0, st
    assert tot["removed"] > 0 and tot["joined"] > 0, tot
    assert worst_inbox < 32, worst_inbox
    sim.close()


GM_ERR_DRAWS = 8


@pytest.mark.parametrize("diag", [True, False])
def test_shard_draw_without_holder_fails_loudly(diag, monkeypatch):
    """gm_s_draw0 (round 0 of the column-shard draws) resolves a draw that lands in its columns
    from the row's band records and cells. If they disagree, no lane holds the drawn rank, and the
    status slot would keep an older tick's value for the MAX-allreduce: the kernel sets
    GM_ERR_DRAWS instead. GM_DIAG_ZERO_ROW clears one row's cells after its band kernels (the
    records keep their counts) on a one-rank RCCL shard; without it the same run stays clean."""
    from membership.abi import comm_unique_id
    n = 2048
    monkeypatch.setenv("GM_FORCE_SHARD", "1")
    if diag:
        monkeypatch.setenv("GM_DIAG_ZERO_ROW", "700")
    sh = Simulator(n, GM_MODE_SCALED, shard_rank=0, shard_count=1, rd_seed=7, init_mode=1, init_t0=6, init_seed=5)
    monkeypatch.delenv("GM_FORCE_SHARD")
    monkeypatch.delenv("GM_DIAG_ZERO_ROW", raising=False)
    sh.comm_init(comm_unique_id(), 1, 0)
    code = first_error(sh, 3)
    if diag:
        assert code == GM_ERANGE
        assert sh.tick_stats()["err"] & GM_ERR_DRAWS
    else:
        assert code == 0 and sh.tick_stats()["err"] == 0
    sh.close()
