"""C-ABI boundary checks that need no GPU: libgm.so loads and exports exactly the
entry points include/gm_abi.h declares; the host-only helpers agree with the oracle."""
import os
import re

import numpy as np
import pytest

import oracle_py
from membership import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    text = open(os.path.join(REPO, "include", "gm_abi.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char \*)\s*(gm_\w+)\(", text, re.M)))


def test_header_lists_every_binding():
    assert set(declared()) == set(abi.EXPORTS)


def test_library_exports_all_symbols():
    lib = abi.load_library()
    for name in declared():
        assert hasattr(lib, name), name


def test_product_is_built_for_gfx950():
    data = open(abi.lib_path(), "rb").read()
    assert b"gfx950" in data


def test_crash_set_host_helper_matches_oracle():
    for n, k, seed in [(10, 1, 42), (65536, 655, 42), (1000, 37, 7), (5, 5, 1)]:
        assert np.array_equal(abi.crash_set(n, k, seed), oracle_py.crash_set(n, k, seed))


def test_parse_conf_matches_params(tmp_path):
    import ctypes
    p = tmp_path / "x.conf"
    p.write_text("MAX_NNB: 10\nSINGLE_FAILURE: 0\nDROP_MSG: 1\nMSG_DROP_PROB: 0.1 \n")
    cfg = abi.GmConfig()
    assert abi.load_library().gm_parse_conf(str(p).encode(), ctypes.byref(cfg)) == 0
    assert (cfg.n, cfg.single_failure, cfg.drop_msg, cfg.drop_prob) == (10, 0, 1, 0.1)


def test_no_silent_cpu_path():
    # Without a usable GPU the product must fail loudly, never fall back.
    try:
        sim = abi.Simulator(10)
    except abi.GmError as e:
        assert e.code in (-3, -2)
        return
    sim.close()
    pytest.skip("a GPU is present; the loud-failure path is exercised only without one")
