"""The reference's own grader scores this build's logs exactly as tests/grader.py does.

Runs /root/reference/Grader_verbose.sh UNMODIFIED (bash, in a scratch directory) with a no-op
`make` first on PATH and an `./Application` stub that drops in a chosen dbg.log for each
testcase, then compares its "Final grade" with tests/grader.py on the same three logs: golden
logs of the seeded reference (90/90) and deliberately broken ones (a missing join, a false
removal, a lost failure detection, duplicated lines). CPU only; skipped where the reference
checkout is absent (the GPU box).
"""
import os
import re
import shutil
import subprocess

import pytest

from golden_util import load_case
from grader import grade

GRADER = "/root/reference/Grader_verbose.sh"
CASES = ("singlefailure", "multifailure", "msgdropsinglefailure")

pytestmark = pytest.mark.skipif(not os.path.exists(GRADER) or shutil.which("bash") is None,
                                reason="reference grader not present (GPU box)")


def run_reference_grader(tmp_path, logs):
    """Final grade of the unmodified script with logs[case] as the dbg.log of each run."""
    d = tmp_path / "g"
    (d / "testcases").mkdir(parents=True)
    (d / "bin").mkdir()
    for c in CASES:
        (d / "testcases" / f"{c}.conf").write_text("")
        (d / f"{c}.log").write_bytes(logs[c])
    make = d / "bin" / "make"
    make.write_text("#!/bin/sh\nexit 0\n")
    app = d / "Application"
    app.write_text('#!/bin/sh\nc=$(basename "$1" .conf)\ncp "$c.log" dbg.log\n')
    for f in (make, app):
        f.chmod(0o755)
    env = dict(os.environ, PATH=f"{d / 'bin'}:{os.environ.get('PATH', '/usr/bin:/bin')}", LC_ALL="C")
    r = subprocess.run(["bash", GRADER], cwd=d, env=env, capture_output=True, timeout=120)
    m = re.search(rb"Final grade (\d+)", r.stdout)
    assert m, r.stdout[-2000:] + r.stderr[-2000:]
    return int(m.group(1))


def _replace_lines(dbg, fn):
    return "\n".join(fn(dbg.decode().split("\n"))).encode()


def _keep_removals_of_first_failed(keep):
    def f(lines):
        fl = sorted(ln for ln in lines if "Node failed at time" in ln)
        who = fl[0].split()[0]
        out, seen = [], 0
        for ln in lines:
            if "removed" in ln and f"Node {who} removed" in ln:
                seen += 1
                if seen > keep:
                    continue
            out.append(ln)
        return out
    return f


def _add_false_removal(lines):
    fl = [ln.split()[0] for ln in lines if "Node failed at time" in ln]
    ok = [f"{i}.0.0.0:0" for i in range(1, 11) if f"{i}.0.0.0:0" not in fl]
    return lines + [f" {ok[0]} [650] Node {ok[1]} removed at time 650"]


def _duplicate_removals(lines):
    return lines + [ln for ln in lines if "removed" in ln][:3]


BROKEN = {
    "missing_join": {"singlefailure": lambda lines: [ln for ln in lines
                                                     if not (ln.startswith(" 3.0.0.0:0 ") and "Node 4.0.0.0:0 joined" in ln)]},
    "false_removal": {"singlefailure": _add_false_removal, "multifailure": _add_false_removal},
    "lost_detection": {"singlefailure": _keep_removals_of_first_failed(8),
                       "multifailure": _keep_removals_of_first_failed(4),
                       "msgdropsinglefailure": _keep_removals_of_first_failed(8)},
    "duplicated_lines": {"multifailure": _duplicate_removals},
    "no_joins": {"msgdropsinglefailure": lambda lines: [ln for ln in lines if "joined" not in ln]},
    "no_failure_line": {"singlefailure": lambda lines: [ln for ln in lines if "Node failed" not in ln]},
}


@pytest.mark.parametrize("seed", ["T1_R1", "T8_R3", "T42_R7"])
def test_reference_grader_agrees_on_golden_logs(tmp_path, seed):
    logs = {c: load_case(f"{c}_{seed}")["dbg"] for c in CASES}
    ours = sum(grade(logs[c], c) for c in CASES)
    assert ours == 90
    assert run_reference_grader(tmp_path, logs) == ours


@pytest.mark.parametrize("kind", sorted(BROKEN))
def test_reference_grader_agrees_on_broken_logs(tmp_path, kind):
    logs = {c: load_case(f"{c}_T4_R2")["dbg"] for c in CASES}
    for c, fn in BROKEN[kind].items():
        logs[c] = _replace_lines(logs[c], fn)
    ours = sum(grade(logs[c], c) for c in CASES)
    ref = run_reference_grader(tmp_path, logs)
    assert ref == ours, (kind, ref, ours)
    if kind != "duplicated_lines":
        assert ours < 90, kind  # each break costs points
