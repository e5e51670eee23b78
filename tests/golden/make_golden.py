#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the SEEDED reference.

TEST INFRASTRUCTURE. Runs only in the build container, where /root/reference
exists: `make -C oracle -f Makefile.ref` compiles the unmodified reference
sources in place (plus the oracle/shim seed shim) into oracle/_ref/, and this
script executes those binaries and stores ONLY their outputs (data, no source):

  faithful/<name>.json        run metadata + md5 of dbg.log / msgcount.log / stdout
  faithful/<name>.dbg.log.gz  dbg.log bytes            (Log.cpp:44-131 contract)
  faithful/<name>.msgcount.gz msgcount.log bytes       (EmulNet.cpp:184-220)
  faithful/<name>.stdout.gz   stdout bytes             (Application.cpp:146)
  faithful/<name>.ticks.npy   uint64 digest64 of the per-tick table dump
                              (oracle/shim/dump_main.cpp line format), one per tick
  faithful/<name>.tables.gz   full table dump (only for a few runs)
  kat_glibc_rand.npz          glibc TYPE_3 rand() first draws for several seeds
  kat_mt19937_lemire.npz      mt19937(seed) + uniform_int_distribution<int>(0,n-1)

The per-tick digest is golden_util.digest64 (blake2b-64) over the bytes of that tick's dump lines
(each line including its trailing '\n'), exactly as tests/golden_util.py
recomputes it from any implementation's state.
"""
import gzip
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
REFBIN = os.path.join(REPO, "oracle", "_ref")
OUT = os.path.join(HERE, "faithful")

sys.path.insert(0, os.path.join(REPO, "tests"))
from golden_util import digest64, parse_conf, tick_digests_from_dump  # noqa: E402


def conf_text(n, single, drop, prob):
    # Params.cpp:22-25 fscanf keys
    return f"MAX_NNB: {n}\nSINGLE_FAILURE: {single}\nDROP_MSG: {drop}\nMSG_DROP_PROB: {prob} \n"


def run_case(name, conf, time_seed, rd_seed, keep_tables=False):
    with tempfile.TemporaryDirectory() as td:
        cpath = os.path.join(td, "case.conf")
        with open(cpath, "w") as f:
            f.write(conf)
        env = dict(os.environ, TIME_SEED=str(time_seed), RD_SEED=str(rd_seed), DUMP_FILE=os.path.join(td, "tables.txt"))
        # plain seeded binary: dbg.log / msgcount.log / stdout
        p = subprocess.run([os.path.join(REFBIN, "Application_seeded"), cpath], cwd=td, env=env,
                           capture_output=True, check=True)
        stdout = p.stdout
        dbg = open(os.path.join(td, "dbg.log"), "rb").read()
        msgc = open(os.path.join(td, "msgcount.log"), "rb").read()
        # dump harness: per-tick tables (must reproduce dbg.log byte for byte)
        d2 = os.path.join(td, "d2")
        os.mkdir(d2)
        subprocess.run([os.path.join(REFBIN, "dump_seeded"), cpath], cwd=d2, env=env, capture_output=True, check=True)
        dbg2 = open(os.path.join(d2, "dbg.log"), "rb").read()
        assert dbg2 == dbg, f"{name}: dump harness diverged from plain oracle"
        tables = open(os.path.join(td, "tables.txt"), "rb").read()
    digs = tick_digests_from_dump(tables)
    meta = dict(name=name, conf=conf, time_seed=time_seed, rd_seed=rd_seed,
                md5_dbg=hashlib.md5(dbg).hexdigest(), md5_msgcount=hashlib.md5(msgc).hexdigest(),
                md5_stdout=hashlib.md5(stdout).hexdigest(), ticks=len(digs),
                digest_of_digests=f"{digest64(digs.tobytes()):016x}",
                removed_lines=dbg.count(b"removed at time"), joined_lines=dbg.count(b"joined at time"))
    with open(os.path.join(OUT, name + ".json"), "w") as f:
        json.dump(meta, f, indent=1)
    for suffix, data in ((".dbg.log.gz", dbg), (".msgcount.gz", msgc), (".stdout.gz", stdout)):
        with gzip.GzipFile(os.path.join(OUT, name + suffix), "wb", mtime=0, compresslevel=9) as g:
            g.write(data)
    np.save(os.path.join(OUT, name + ".ticks.npy"), digs)
    if keep_tables:
        with gzip.GzipFile(os.path.join(OUT, name + ".tables.gz"), "wb", mtime=0, compresslevel=9) as g:
            g.write(tables)
    print(name, meta["md5_dbg"], meta["removed_lines"], meta["joined_lines"], flush=True)
    return meta


def kat_rand():
    src = r'''
#include <stdio.h>
#include <stdlib.h>
int main(int c, char **v) { unsigned s = strtoul(v[1],0,10); int n = atoi(v[2]); srand(s);
  for (int i = 0; i < n; i++) { int r = rand(); fwrite(&r, 4, 1, stdout); } return 0; }'''
    src2 = r'''
#include <random>
#include <stdio.h>
#include <stdlib.h>
int main(int c, char **v) { unsigned s = strtoul(v[1],0,10); int n = atoi(v[2]); int k = atoi(v[3]);
  std::mt19937 mt(s); std::uniform_int_distribution<> d(0, n - 1);
  for (int i = 0; i < k; i++) { int r = d(mt); fwrite(&r, 4, 1, stdout); } return 0; }'''
    with tempfile.TemporaryDirectory() as td:
        open(os.path.join(td, "r.c"), "w").write(src)
        open(os.path.join(td, "m.cpp"), "w").write(src2)
        subprocess.run(["gcc", "-O1", "-o", os.path.join(td, "r"), os.path.join(td, "r.c")], check=True)
        subprocess.run(["g++", "-O1", "-o", os.path.join(td, "m"), os.path.join(td, "m.cpp")], check=True)
        seeds = [0, 1, 42, 1234567, 4294967295]
        rand = {f"seed_{s}": np.frombuffer(subprocess.run([os.path.join(td, "r"), str(s), "100000"],
                                                          capture_output=True, check=True).stdout, dtype=np.int32)
                for s in seeds}
        np.savez_compressed(os.path.join(HERE, "kat_glibc_rand.npz"), **rand)
        rng = np.random.default_rng(2024)
        mseeds = rng.integers(0, 2**32, size=200, dtype=np.uint64)
        ranges = [1, 2, 3, 7, 10, 11, 64, 100, 1000, 65536, 1 << 20, 2**31 - 1]
        arrs = {}
        for n in ranges:
            rows = []
            for s in mseeds:
                out = subprocess.run([os.path.join(td, "m"), str(int(s)), str(n), "40"], capture_output=True,
                                     check=True).stdout
                rows.append(np.frombuffer(out, dtype=np.int32))
            arrs[f"n_{n}"] = np.stack(rows)
        arrs["seeds"] = mseeds.astype(np.uint32)
        np.savez_compressed(os.path.join(HERE, "kat_mt19937_lemire.npz"), **arrs)


def synth_cases():
    return [
        ("n20_single", conf_text(20, 1, 0, "0.1"), 5, 9),
        ("n20_multi_drop", conf_text(20, 0, 1, "0.1"), 5, 9),
        ("n50_multi_drop", conf_text(50, 0, 1, "0.1"), 5, 9),
        ("n70_single", conf_text(70, 1, 0, "0.1"), 3, 4),
        ("n100_single", conf_text(100, 1, 0, "0.1"), 3, 4),
        ("n130_multi_drop", conf_text(130, 0, 1, "0.1"), 3, 4),
        ("n300_single", conf_text(300, 1, 0, "0.1"), 3, 4),
        ("n300_drop50_single", conf_text(300, 1, 1, "0.5"), 11, 12),
        ("n520_single", conf_text(520, 1, 0, "0.1"), 3, 4),
        # the largest cluster EmulNet admits (EmulNet.cpp:108 asserts id <= 1000): saturated
        # 30000-message buffer, multi-failure, drops
        ("n1000_multi_drop", conf_text(1000, 0, 1, "0.1"), 3, 4),
    ]


def main():
    if not os.path.isdir(REF):
        sys.exit("needs /root/reference (build container only)")
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "-f", "Makefile.ref"], check=True)
    os.makedirs(OUT, exist_ok=True)
    synth = synth_cases()
    if len(sys.argv) > 2 and sys.argv[1] == "--only":  # regenerate one synthetic case, keep the rest
        with open(os.path.join(OUT, "index.json")) as f:
            names = json.load(f)
        for name, conf, ts, rs in synth:
            if name == sys.argv[2]:
                run_case(name, conf, ts, rs)
                if name not in names:
                    names.append(name)
        with open(os.path.join(OUT, "index.json"), "w") as f:
            json.dump(names, f, indent=0)
        return
    kat_rand()
    testcases = {"singlefailure": (10, 1, 0, "0.1"), "multifailure": (10, 0, 0, "0.1"),
                 "msgdropsinglefailure": (10, 1, 1, "0.1")}
    index = []
    for case, (n, s, d, p) in testcases.items():
        conf = open(os.path.join(REF, "testcases", case + ".conf")).read()
        assert parse_conf(conf) == (n, s, d, float(p)), case
        for ts in range(1, 9):
            for rs in range(1, 4):
                keep = (ts == 1 and rs == 1)
                index.append(run_case(f"{case}_T{ts}_R{rs}", conf, ts, rs, keep_tables=keep))
        index.append(run_case(f"{case}_T42_R7", conf, 42, 7))
    for name, conf, ts, rs in synth:
        index.append(run_case(name, conf, ts, rs, keep_tables=(name == "n20_multi_drop")))
    with open(os.path.join(OUT, "index.json"), "w") as f:
        json.dump([m["name"] for m in index], f, indent=0)


if __name__ == "__main__":
    main()
