"""The oracle (oracle/ref_cpu.c) against the seeded reference's golden fixtures.

Pins the CPU restatement before it is trusted as the checker of the HIP path:
dbg.log, msgcount.log and stdout byte-for-byte and the per-tick membership
tables (digest of the dump of every tick) for the 3 reference testcases x 25
seed pairs and 10 synthetic clusters (N=20..1000, the largest EmulNet admits: healthy, drop, multi-failure,
EmulNet-buffer overflow, signed-char addresses, updateMyPos quirk regimes).
"""
import numpy as np
import pytest

import oracle_py
from golden_util import load_case, load_index, tick_digests_from_dump

ALL = load_index()
FAST = [n for n in ALL if not n.startswith("n") or n.split("_")[0] in ("n20", "n50", "n70")]
SLOW = [n for n in ALL if n not in FAST]


def _check(name, tmp_path):
    m = load_case(name)
    dbg, msgc, out, dump = oracle_py.run_cli(m["conf"], m["time_seed"], m["rd_seed"], str(tmp_path), dump=True)
    assert dbg == m["dbg"], "dbg.log differs"
    assert msgc == m["msgcount"], "msgcount.log differs"
    assert out == m["stdout"], "stdout differs"
    d = tick_digests_from_dump(dump)
    assert len(d) == len(m["tick_digests"])
    bad = np.nonzero(d != m["tick_digests"])[0]
    assert bad.size == 0, f"table digest differs first at tick {bad[:1]}"
    if m["tables"] is not None:
        assert dump == m["tables"]


@pytest.mark.parametrize("name", FAST)
def test_oracle_matches_reference(name, tmp_path):
    _check(name, tmp_path)


@pytest.mark.slow
@pytest.mark.parametrize("name", SLOW)
def test_oracle_matches_reference_large(name, tmp_path):
    _check(name, tmp_path)


def test_fixture_inventory():
    # 3 testcases x (8x3 seed grid + the survey's 42/7 pair) + 10 synthetic clusters
    assert len(ALL) == 3 * 25 + 10
    for name in ALL:
        m = load_case(name)
        assert m["ticks"] == 700 and m["dbg"].startswith(b"131\n")
