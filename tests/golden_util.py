"""Helpers shared by the golden-fixture generator and the parity tests.

Pure data handling (no reference code): 64-bit digests of the per-tick table
dump format written by oracle/shim/dump_main.cpp, and loaders for the
committed fixtures under tests/golden/.

Dump line format (one per node, per tick, after `mp1Run(); fail();`):
    "t i inited inGroup bFailed heartbeat n id:hb:ts id:hb:ts ...\\n"
with the membership list in ascending id order (the reference keeps it sorted:
MP1Node.cpp:297,319,446).
"""
import gzip
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FAITHFUL = os.path.join(GOLDEN, "faithful")


def digest64(data: bytes) -> int:
    """64-bit digest used for every fixture: blake2b with an 8-byte digest, read little-endian."""
    return int.from_bytes(hashlib.blake2b(data, digest_size=8).digest(), "little")


def tick_digests_from_dump(text: bytes) -> np.ndarray:
    """digest64 of each tick's block of dump lines (line bytes incl. '\\n')."""
    out = []
    pos = 0
    n = len(text)
    while pos < n:
        sp = text.index(b" ", pos)
        t = text[pos:sp]
        # the block of tick t ends where the first line of another tick starts
        end = pos
        while end < n:
            nl = text.index(b"\n", end) + 1
            end = nl
            if end >= n or not text.startswith(t + b" ", end):
                break
        out.append(digest64(text[pos:end]))
        pos = end
    return np.array(out, dtype=np.uint64)


def dump_lines_for_tick(t, inited, in_group, failed, heartbeat, present, hb, ts):
    """Render one tick of per-node state (dense-table form) in the dump format.

    present/hb/ts are [N][N] arrays: column c is subject id c+1.
    """
    n = len(inited)
    parts = []
    for i in range(n):
        cols = np.nonzero(present[i])[0]
        ent = " ".join(f"{c + 1}:{int(hb[i][c])}:{int(ts[i][c])}" for c in cols)
        line = f"{t} {i} {int(inited[i])} {int(in_group[i])} {int(failed[i])} {int(heartbeat[i])} {len(cols)}"
        if len(cols):
            line += " " + ent
        parts.append(line + "\n")
    return "".join(parts).encode()


def load_index():
    with open(os.path.join(FAITHFUL, "index.json")) as f:
        return json.load(f)


def load_case(name):
    with open(os.path.join(FAITHFUL, name + ".json")) as f:
        meta = json.load(f)

    def gz(suffix):
        p = os.path.join(FAITHFUL, name + suffix)
        if not os.path.exists(p):
            return None
        with gzip.open(p, "rb") as g:
            return g.read()

    meta["dbg"] = gz(".dbg.log.gz")
    meta["msgcount"] = gz(".msgcount.gz")
    meta["stdout"] = gz(".stdout.gz")
    meta["tables"] = gz(".tables.gz")
    meta["tick_digests"] = np.load(os.path.join(FAITHFUL, name + ".ticks.npy"))
    return meta


def parse_conf(text):
    """Params::setparams (Params.cpp:19-40) key order: MAX_NNB, SINGLE_FAILURE, DROP_MSG, MSG_DROP_PROB."""
    vals = {}
    for line in text.splitlines():
        if ":" in line:
            k, v = line.split(":", 1)
            vals[k.strip()] = v.strip()
    return (int(vals["MAX_NNB"]), int(vals["SINGLE_FAILURE"]), int(vals["DROP_MSG"]), float(vals["MSG_DROP_PROB"]))


def same_state(sim, ora):
    """HIP context vs oracle by binary readbacks: every table cell (hb, ts) and every node's
    state -- the content of the text dump, without rendering it (parity tests at larger N)."""
    import numpy as np
    hb, ts = sim.read_table()
    ohb, ots = ora.table()
    return np.array_equal(hb, ohb) and np.array_equal(ts, ots) and np.array_equal(sim.read_nodes(), ora.nodes())
