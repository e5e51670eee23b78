"""CPU lint over the product sources (csrc/, app/).

Every copy and fill of a context must go through the context's own non-blocking stream
(`ctx_memset` / `ctx_memcpy` / `ctx_memcpy2d`, gm_host.hip): a synchronous null-stream call
(`hipMemset`, `hipMemcpy`, `hipMemcpy2D`, the symbol copies) is not ordered against the
context's kernels. One such fill at creation raced `gm_p_init` and zeroed S-C rows
(intermittent GM_ERR_SELF in rounds r04u / r04z, profiles/r04/sc_self_flake/README.md).
`hipDeviceSynchronize` would also wait for every other context's work on the device.

Measurement-only variants (ablations, dropped routes, the per-section clock builds
GM_P_PROFILE / GM_F_PROFILE) live as patches under profiles/ (e.g.
profiles/r06/profile_patches/), not as #ifdef blocks in the product kernels.
"""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC_DIRS = [os.path.join(REPO, "distributed-membership_amd", d) for d in ("csrc", "app")]

# synchronous / null-stream runtime calls (the async forms take an explicit stream)
FORBIDDEN = re.compile(
    r"\b(hipMemset|hipMemsetD8|hipMemsetD16|hipMemsetD32|hipMemcpy|hipMemcpy2D|hipMemcpy3D|"
    r"hipMemcpyToSymbol|hipMemcpyFromSymbol|hipMemcpyHtoD|hipMemcpyDtoH|hipMemcpyDtoD|"
    r"hipDeviceSynchronize)\s*\(")
# an async copy / fill enqueued on the null stream by a literal 0 / nullptr stream argument
NULL_STREAM = re.compile(r"\bhip(Memset|Memcpy\w*)Async\s*\([^;]*,\s*(0|nullptr|NULL)\s*\)\s*[;)]")
ABLATION = re.compile(r"GM_ABL_\w+|GM_P_ROUTE|GM_\w+_PROFILE")


def _sources():
    for d in SRC_DIRS:
        for name in sorted(os.listdir(d)):
            if name.endswith((".hip", ".h", ".cpp", ".hpp")):
                yield os.path.join(d, name)


def _strip_comments(text):
    text = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), text, flags=re.S)
    return re.sub(r"//[^\n]*", "", text)


def test_sources_found():
    assert len(list(_sources())) >= 8


def test_no_null_stream_copies_or_device_syncs():
    bad = []
    for p in _sources():
        code = _strip_comments(open(p).read())
        for ln, line in enumerate(code.splitlines(), 1):
            if FORBIDDEN.search(line) or NULL_STREAM.search(line):
                bad.append(f"{os.path.relpath(p, REPO)}:{ln}: {line.strip()}")
    assert not bad, "null-stream / device-wide synchronous calls in product sources:\n" + "\n".join(bad)


def test_no_ablation_variants_in_product_kernels():
    bad = []
    for p in _sources():
        for ln, line in enumerate(open(p).read().splitlines(), 1):
            if ABLATION.search(line):
                bad.append(f"{os.path.relpath(p, REPO)}:{ln}: {line.strip()}")
    assert not bad, "measurement-only variants in product sources:\n" + "\n".join(bad)


def test_lint_catches_the_r04_race_pattern():
    # the exact call shape behind the r04u / r04z GM_ERR_SELF, and its async form on the null stream
    assert FORBIDDEN.search("  HIPCHECK(hipMemset(p.lists, 0, bytes));")
    assert NULL_STREAM.search("  HIPCHECK(hipMemsetAsync(p.lists, 0, bytes, 0));")
    assert not FORBIDDEN.search("  HIPCHECK(hipMemsetAsync(p.lists, 0, bytes, c->stream));")
    assert not NULL_STREAM.search("  HIPCHECK(hipMemsetAsync(p.lists, 0, bytes, c->stream));")


def test_lint_catches_profile_blocks():
    assert ABLATION.search("#ifdef GM_P_PROFILE")
    assert ABLATION.search("#ifdef GM_F_PROFILE")
    assert ABLATION.search("#if defined(GM_S_PROFILE)")
