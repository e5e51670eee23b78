"""Property checks of the reference's grader (Grader_verbose.sh:41-181), restated.

TEST INFRASTRUCTURE. Operates on dbg.log bytes; returns (points, details).
"""
import re

JOIN_RE = re.compile(r"^ (\S+) \[\d+\] Node (\S+) joined at time")
REM_RE = re.compile(r"^ (\S+) \[\d+\] Node (\S+) removed at time")
FAIL_RE = re.compile(r"^ (\S+) \[\d+\] Node failed at time")


def _lines(dbg):
    return dbg.decode(errors="replace").split("\n")


def join_ok(dbg, n=10):
    pairs = set()
    per = {}
    for ln in _lines(dbg):
        m = JOIN_RE.match(ln)
        if m:
            pairs.add((m.group(1), m.group(2)))
            per.setdefault(m.group(1), set()).add(m.group(2))
    if len(pairs) == n * n:
        return True
    return len(per) == n and all(len(v) >= n - 1 for v in per.values())


def failed_nodes(dbg):
    out = []
    for ln in _lines(dbg):
        m = FAIL_RE.match(ln)
        if m:
            out.append(m.group(1))
    return out


def removals(dbg):
    return [(m.group(1), m.group(2)) for m in (REM_RE.match(ln) for ln in _lines(dbg)) if m]


def grade(dbg, case):
    """Points the reference grader would award for one testcase."""
    pts = 0
    fails = failed_nodes(dbg)
    rem = removals(dbg)
    if case == "singlefailure":
        pts += 10 if join_ok(dbg) else 0
        f = fails[0]
        pts += 10 if sum(1 for (_, s) in rem if s == f) >= 9 else 0
        pts += 10 if sum(1 for (_, s) in rem if s != f) == 0 else 0
    elif case == "multifailure":
        pts += 10 if join_ok(dbg) else 0
        ok_c = all(sum(1 for (_, s) in rem if s == f) >= 5 for f in fails)
        pts += 10 if ok_c else 0
        ok_a = all(sum(1 for (_, s) in rem if s != f) == 20 for f in fails)
        pts += 10 if ok_a else 0
    elif case == "msgdropsinglefailure":
        pts += 15 if join_ok(dbg) else 0
        f = fails[0]
        pts += 15 if sum(1 for (_, s) in rem if s == f) >= 9 else 0
    return pts
