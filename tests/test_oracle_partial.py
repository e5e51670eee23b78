"""PARTIAL mode (V-entry views, scenario S-C) has no reference to pin it: the
oracle restatement (oracle/ref_cpu.c "PARTIAL") IS the specification. This test
pins the specification itself against regressions: 40-tick digests of every
view dump and event list for six configurations, recorded from the oracle when
GM_MODE_PARTIAL was specified (tests/golden/partial/oracle_digests.json;
regenerate only on a deliberate semantic change). The HIP path is checked
against the live oracle in test_gpu_partial.py."""
import hashlib
import json
import os

import pytest

import oracle_py

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "partial", "oracle_digests.json")))


def oracle_digest(c):
    ora = oracle_py.PartialOracle(c["n"], v=c["v"], rd_seed=7, view_seed=5, init_t0=8, init_seed=11,
                                  crash_tick=c["crash_tick"], crash_count=c["crash_count"], crash_seed=42,
                                  drop_pct=c["drop_pct"], drop_from=c["drop_from"], drop_to=c["drop_to"], drop_seed=42)
    md = hashlib.sha256()
    for _ in range(c["ticks"]):
        ora.tick()
        md.update(ora.dump())
        md.update(repr(ora.events()).encode())
    return md.hexdigest()


@pytest.mark.parametrize("c", CASES, ids=[f"n{c['n']}_v{c['v']}_drop{c['drop_pct']}" for c in CASES])
def test_partial_oracle_digest(c):
    assert oracle_digest(c) == c["sha256"]


def test_sc_regime_has_no_removals():
    """Pins what test_gpu_baseline_configs asserts at N = 16M on the specification:
    under the S-C schedule (5 % drops every tick, 1 % crash at tick 10) eviction keeps
    every view full and fresh, so the TREMOVE sweep never fires; crashed nodes leave
    the views by eviction."""
    n = 4000
    ora = oracle_py.PartialOracle(n, v=32, rd_seed=7, view_seed=5, init_t0=8, init_seed=11, crash_tick=10,
                                  crash_count=n // 100, crash_seed=42, drop_pct=5, drop_from=0, drop_to=1 << 20,
                                  drop_seed=42)
    for _ in range(30):
        ora.tick()
        assert all(e[2] == 1 for e in ora.events())
