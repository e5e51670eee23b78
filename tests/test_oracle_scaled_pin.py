"""Pins the SCALED oracle to the reference itself (SURVEY.md §8(c) parity chain).

SCALED (`oracle/ref_cpu.c`, OC_SCALED) swaps the reference's EmulNet for an
unbounded order-free network with keyed drops and emits a canonical event
stream; its join ramp (`init_mode` 2) is the reference's own lifecycle
(`/root/reference/Application.cpp:121-164`, `MP1Node.cpp:126-163,226-251`).
Where the reference's network does nothing SCALED does not — no drops, and
N < 78 so the 30000-entry EmulNet buffer (`EmulNet.cpp:92`) never fills —
the two must produce the same cluster tick by tick. This test runs the SCALED
oracle through every golden case with N <= 70 and checks, against fixtures
generated from the seeded reference build (`tests/golden/make_golden.py`):

* every tick's table digest (inited, inGroup, bFailed, heartbeat and the
  whole member list of every node) — all 700 ticks without drops; up to
  tick 50 in the DROP_MSG cases (the reference starts dropping at tick 51
  through glibc `rand()`, SCALED drops are keyed, so they diverge there);
* every tick's join / remove events against the golden dbg.log lines, per
  logger: the reference logs joins in EmulNet delivery order, SCALED in
  ascending id, so joins compare as sets, removals in order (descending id
  in both, `MP1Node.cpp:429-444`).

The failure victims of `Application::fail` (glibc `rand()`, `Application.cpp:
184-196`) are read from the golden dbg.log's "Node failed" lines and applied
with `Oracle.set_failed`. Every SCALED HIP test inherits this pin: the HIP
SCALED path is compared with this oracle tick by tick.
"""
import collections
import re

import pytest

import oracle_py
from golden_util import digest64, load_case, load_index, parse_conf

_LINE = re.compile(rb"^ (?:(-?\d+)\.(-?\d+)\.(-?\d+)\.(-?\d+):0 )?\[(\d+)\] (.*)$")
_EVENT = re.compile(rb"Node (-?\d+)\.(-?\d+)\.(-?\d+)\.(-?\d+):0 (joined|removed) at time (\d+)")


def _addr_id(*b):
    """inverse of Log.cpp's "%d.%d.%d.%d" over the signed address bytes (id LE, Member.h:29-55)"""
    return int.from_bytes(bytes(int(x) & 255 for x in b), "little", signed=True)


def _parse_dbg(dbg):
    """golden dbg.log -> {t: [(logger_idx, kind, subject_id)]}, {t: [failed idx]}"""
    ev, fails = collections.defaultdict(list), collections.defaultdict(list)
    for ln in dbg.split(b"\n"):
        m = _LINE.match(ln)
        if not m or m.group(1) is None:  # the first record carries no address (Log.cpp:46-60)
            continue
        logger, t, text = _addr_id(*m.group(1, 2, 3, 4)) - 1, int(m.group(5)), m.group(6)
        e = _EVENT.match(text)
        if e:
            ev[t].append((logger, 1 if e.group(5) == b"joined" else 2, _addr_id(*e.group(1, 2, 3, 4))))
        elif text.startswith(b"Node failed"):
            fails[t].append(logger)
    return ev, fails


def _canon(events):
    """SCALED's canonical order: loggers descending, joins ascending id, removals descending id"""
    return sorted(events, key=lambda e: (-e[0], e[1], e[2] if e[1] == 1 else -e[2]))


SMALL = [c for c in load_index() if parse_conf(load_case(c)["conf"])[0] <= 70]


def test_small_case_grid_is_complete():
    assert len(SMALL) == 79  # 3 testcases x 25 seed pairs + n20_single, n20_multi_drop, n50_multi_drop, n70_single


@pytest.mark.parametrize("case", SMALL)
def test_scaled_ramp_equals_reference(case):
    m = load_case(case)
    n, _single, drop, _p = parse_conf(m["conf"])
    ev, fails = _parse_dbg(m["dbg"])
    ticks = 51 if drop else m["ticks"]
    ora = oracle_py.Oracle(n, oracle_py.OC_SCALED, rd_seed=m["rd_seed"], init_mode=2)
    joins = 0
    for t in range(ticks):
        ora.tick()
        if fails.get(t):
            ora.set_failed(fails[t])
        assert digest64(ora.dump()) == int(m["tick_digests"][t]), f"{case}: tables differ at t={t}"
        got = [(e[1], e[2], e[3]) for e in ora.events()]
        assert got == _canon(ev.get(t, [])), f"{case}: events differ at t={t}"
        joins += sum(1 for e in got if e[1] == 1)
    assert joins > 0
    if not drop:
        assert fails, "the no-drop cases run through the tick-100 failure"
