"""The reference's grader (Grader_verbose.sh:41-181), restated line for line in Python.

TEST INFRASTRUCTURE. Operates on dbg.log bytes; `grade(dbg, case)` returns the points the
script adds to its "Final grade" for one testcase. The script's text pipelines are modelled
with their exact semantics, not their intent:

* `grep P` keeps the lines in which the basic regex P matches anywhere (addresses are used
  as patterns, so '.' matches any character and a node's address also matches the lines it
  logged itself); `grep -v P` keeps the others; with no pattern (an empty `$failednode`)
  grep prints nothing.
* `sort -u` keeps distinct lines; `wc -l` counts them.
* `cut -d" " -f2,4-7` splits on single spaces: a record line starts with a space, so field 2
  is the logger's address and fields 4-7 are "Node <addr> joined at".
* The multi-failure loops stop after their sixth node (completeness, `cnt -gt 5`) or once ten
  points are reached (accuracy, `tmp -gt 9`).

tests/test_grader_reference.py runs the unmodified script on the same logs (golden ones and
deliberately broken ones) and requires the same score.
"""
import re


def _lines(dbg):
    # grep sees the file's lines; the file has no trailing newline (Log.cpp writes "\n" + record)
    return dbg.decode(errors="replace").split("\n")


def _grep(lines, pat, invert=False):
    if pat is None:  # `grep` with no pattern argument: usage error, no output
        return []
    rx = re.compile(pat)
    return [ln for ln in lines if (rx.search(ln) is None) == invert]


def _cut(ln, fields):
    parts = ln.split(" ")
    return " ".join(parts[f - 1] for f in fields if f - 1 < len(parts))


def _join_points(lines, full):
    joined = _grep(lines, "joined")
    if len({_cut(ln, (2, 4, 5, 6, 7)) for ln in joined}) == 100:
        return full
    cnt = 0
    for i in sorted({_cut(ln, (2,)) for ln in joined}):
        mine = _grep(joined, "^ " + i)
        others = _grep([_cut(ln, (4, 5, 6, 7)) for ln in mine], i, invert=True)
        if len(set(others)) == 9:
            cnt += 1
    return full if cnt == 10 else 0


def failed_nodes(dbg):
    """`grep "Node failed at time" dbg.log | sort -u | awk '{print $1}'`, in sort order."""
    fl = sorted(set(_grep(_lines(dbg), "Node failed at time")))
    return [ln.split()[0] for ln in fl if ln.split()]


def grade(dbg, case):
    """Points the reference grader awards for one testcase."""
    lines = _lines(dbg)
    rem = sorted(set(_grep(lines, "removed")))  # grep removed dbg.log | sort -u
    fails = failed_nodes(dbg)
    first = fails[0] if fails else None  # `grep $failednode`: the first word is the pattern
    if case in ("singlefailure", "msgdropsinglefailure"):
        w = 10 if case == "singlefailure" else 15
        pts = _join_points(lines, w)
        failcount = len(_grep(rem, first)) if len(fails) <= 1 else 0
        pts += w if failcount >= 9 else 0
        if case == "singlefailure":
            acc = len(_grep(rem, first, invert=True)) if fails else 0
            pts += 10 if acc == 0 and failcount > 0 and len(fails) == 1 else 0
        return pts
    if case == "multifailure":
        pts = _join_points(lines, 10)
        cnt = 0
        for i in fails:
            if len(_grep(rem, i)) >= 5:
                pts += 2
            cnt += 1
            if cnt > 5:
                break
        tmp = 0
        for i in fails:
            if len(_grep(rem, i, invert=True)) == 20:
                tmp += 2
            if tmp > 9:
                break
        return pts + tmp
    raise ValueError(case)
