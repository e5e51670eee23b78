"""Reference-shaped driver in Python (Application.cpp:27-202, Params.cpp, Log.cpp).

`Application(conf).run()` produces the same dbg.log / msgcount.log / stdout
bytes as the C++ ./Application and as the reference, in memory.
"""
import struct

from .abi import (GM_EV_JOINED, GM_EV_REMOVED, GM_EV_START_GROUP, GM_EV_TIME_MARK, GM_EV_TRY_JOIN,
                  GM_MODE_FAITHFUL, Simulator)

TOTAL_RUNNING_TIME = 700  # Application.h:27


class Params:
    """Params::setparams (Params.cpp:19-40): MAX_NNB, SINGLE_FAILURE, DROP_MSG, MSG_DROP_PROB."""

    def __init__(self, MAX_NNB=10, SINGLE_FAILURE=1, DROP_MSG=0, MSG_DROP_PROB=0.1):
        self.MAX_NNB = self.EN_GPSZ = MAX_NNB
        self.SINGLE_FAILURE, self.DROP_MSG, self.MSG_DROP_PROB = SINGLE_FAILURE, DROP_MSG, MSG_DROP_PROB
        self.STEP_RATE = 0.25
        self.MAX_MSG_SIZE = 4000

    @classmethod
    def from_conf_text(cls, text):
        vals = {}
        for line in text.splitlines():
            if ":" in line:
                k, v = line.split(":", 1)
                vals[k.strip()] = v.strip()
        return cls(int(vals["MAX_NNB"]), int(vals["SINGLE_FAILURE"]), int(vals["DROP_MSG"]),
                   float(vals["MSG_DROP_PROB"]))

    @classmethod
    def from_conf(cls, path):
        with open(path) as f:
            return cls.from_conf_text(f.read())


def log_addr(i):
    """%d.%d.%d.%d:%d over the signed-char address bytes (Log.cpp:73)."""
    b = struct.unpack("4b", struct.pack("<i", i))
    return f"{b[0]}.{b[1]}.{b[2]}.{b[3]}:0"


class Log:
    def __init__(self):
        self.parts = []
        self.opened = False
        self.first = False

    def LOG(self, node_id, t, text):
        prefix = ""
        if not self.opened:
            self.opened = True
        else:
            prefix = log_addr(node_id) + " "
        if not self.first:
            self.parts.append("%x\n" % sum(map(ord, "CS425")))
            self.first = True
        self.parts.append(f"\n {prefix}[{t}] {text}")

    def logNodeAdd(self, logger_id, added_id, t):
        self.LOG(logger_id, t, f"Node {log_addr(added_id)} joined at time {t}")

    def logNodeRemove(self, logger_id, removed_id, t):
        self.LOG(logger_id, t, f"Node {log_addr(removed_id)} removed at time {t}")

    def data(self):
        return "".join(self.parts).encode()


def format_msgcount(sent, recv):
    """EmulNet::ENcleanup (EmulNet.cpp:184-220), node 67 special-cased."""
    n, T = sent.shape
    out = []
    for i in range(1, n + 1):
        out.append("node %3d " % i)
        st = rt = 0
        for j in range(T):
            s, r = int(sent[i - 1, j]), int(recv[i - 1, j])
            st += s
            rt += r
            if i != 67:
                out.append(" (%4d, %4d)" % (s, r))
                if j % 10 == 9:
                    out.append("\n         ")
            else:
                out.append("special %4d %4d %4d\n" % (j, s, r))
        out.append("\n")
        out.append("node %3d sent_total %6u  recv_total %6u\n\n" % (i, st, rt))
    return "".join(out).encode()


class Application:
    def __init__(self, params, time_seed=0, rd_seed=0, device=0, ticks=TOTAL_RUNNING_TIME, dump_tables=False):
        self.par = params if isinstance(params, Params) else Params.from_conf(params)
        self.ticks = ticks
        self.log = Log()
        self.stdout = []
        self.dumps = [] if dump_tables else None
        n = self.par.EN_GPSZ
        for i in range(n):
            self.log.LOG(i + 1, 0, "APP")  # Application.cpp:66
        self.sim = Simulator(n, GM_MODE_FAITHFUL, self.par.SINGLE_FAILURE, self.par.DROP_MSG, self.par.MSG_DROP_PROB,
                             time_seed, rd_seed, device=device)
        self.t = 0

    def mp1Run(self):
        self.sim.tick()
        for (t, logger, kind, subject) in self.sim.drain_events():
            nid = logger + 1
            if kind == GM_EV_JOINED:
                self.log.logNodeAdd(nid, subject, t)
            elif kind == GM_EV_REMOVED:
                self.log.logNodeRemove(nid, subject, t)
            elif kind == GM_EV_START_GROUP:
                self.log.LOG(nid, t, "Starting up group...")
            elif kind == GM_EV_TRY_JOIN:
                self.log.LOG(nid, t, "Trying to join...")
            elif kind == GM_EV_TIME_MARK:
                self.log.LOG(nid, t, f"@@time={t}")
        for i in range(self.par.EN_GPSZ - 1, -1, -1):
            if self.t == int(self.par.STEP_RATE * i):
                self.stdout.append(f"{i}-th introduced node is assigned with the address: {i + 1}:0\n")

    def fail(self):
        t, n = self.t, self.par.EN_GPSZ
        if self.par.DROP_MSG and t == 50:
            self.sim.set_dropmsg(1)
        if self.par.SINGLE_FAILURE and t == 100:
            removed = self.sim.rand() % n
            self.log.LOG(removed + 1, t, f"Node failed at time={t}")
            self.sim.set_failed([removed])
        elif t == 100:
            removed = (self.sim.rand() % n) // 2
            idx = list(range(removed, removed + n // 2))
            for i in idx:
                self.log.LOG(i + 1, t, f"Node failed at time = {t}")
            self.sim.set_failed(idx)
        if self.par.DROP_MSG and t == 300:
            self.sim.set_dropmsg(0)

    def run(self):
        for self.t in range(self.ticks):
            self.mp1Run()
            self.fail()
            if self.dumps is not None:
                self.dumps.append(self.sim.dump_tables())
        self.t = self.ticks
        sent, recv = self.sim.msgcount(self.ticks)
        self.msgcount = format_msgcount(sent, recv)
        self.dbg = self.log.data()
        self.out = "".join(self.stdout).encode()
        return self
