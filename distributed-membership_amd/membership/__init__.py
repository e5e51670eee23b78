"""Python host surface of the MI355X gossip-membership simulator.

Mirrors the reference's driver interface (Application / Params / Log,
Application.cpp:27-202, Params.cpp:19-40, Log.cpp:44-131) over the C ABI of
include/gm_abi.h (libgm.so: hand-written HIP kernels for gfx950). There is no
CPU fallback: constructing a Simulator without the built library, or without a
GPU, raises.
"""
from .abi import (GM_EV_JOINED, GM_EV_REMOVED, GM_EV_START_GROUP, GM_EV_TIME_MARK, GM_EV_TRY_JOIN,  # noqa: F401
                  GM_MODE_FAITHFUL, GM_MODE_PARTIAL, GM_MODE_SCALED, GmError, Simulator, crash_set, lib_path, load_library)
from .app import Application, Params, format_msgcount, log_addr  # noqa: F401
