"""Known-answer tests of the two RNG streams the simulator replays.

S1: glibc TYPE_3 rand() (srand seeds; EmulNet.cpp:90, Application.cpp:182,189).
S2: libstdc++-11 mt19937 + uniform_int_distribution<int> (Lemire) (MP1Node.cpp:450-452).
Vectors in tests/golden/kat_*.npz were produced by glibc / libstdc++ themselves
(tests/golden/make_golden.py). Also pins the seed contract's splitmix64 step.
"""
import os

import numpy as np

import oracle_py
from golden_util import GOLDEN


def test_glibc_rand_kat():
    kat = np.load(os.path.join(GOLDEN, "kat_glibc_rand.npz"))
    for key in kat.files:
        seed = int(key.split("_")[1])
        got = oracle_py.glibc_rand(seed, 2000)
        assert np.array_equal(got, kat[key][:2000]), key


def test_mt19937_lemire_kat():
    kat = np.load(os.path.join(GOLDEN, "kat_mt19937_lemire.npz"))
    seeds = kat["seeds"]
    for key in kat.files:
        if key == "seeds":
            continue
        n = int(key.split("_")[1])
        exp = kat[key]
        for row in range(0, len(seeds), 7):
            got = oracle_py.mt_uniform(int(seeds[row]), n, exp.shape[1])
            assert np.array_equal(got, exp[row]), (key, row)


def test_rd_seed_contract():
    # splitmix64 finalizer over RD_SEED ^ (t<<32 | id), low 32 bits
    def ref(rd, t, i):
        m = (1 << 64) - 1
        z = (rd ^ ((t << 32) | i)) & m
        z = (z + 0x9E3779B97F4A7C15) & m
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
        z ^= z >> 31
        return z & 0xFFFFFFFF
    for rd, t, i in [(0, 0, 1), (7, 5, 3), (2**63 + 5, 699, 1000), (42, 12345, 65536)]:
        assert oracle_py.lib().oc_rd_seed(rd, t, i) == ref(rd, t, i)


def test_shard_model_mt19937_matches_kat():
    # the protocol model's pure-Python mt19937 (raw outputs, Lemire on top) must be the
    # libstdc++ stream the golden KATs hold
    from shard_model import lemire_draws
    kat = np.load(os.path.join(GOLDEN, "kat_mt19937_lemire.npz"))
    seeds = kat["seeds"]
    for key in kat.files:
        if key == "seeds":
            continue
        n = int(key.split("_")[1])
        exp = kat[key]
        for row in range(0, len(seeds), 97):
            assert lemire_draws(int(seeds[row]), n, exp.shape[1]) == list(exp[row]), (key, row)
