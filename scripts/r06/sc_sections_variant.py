#!/usr/bin/env python3
"""Measurement build (not product code): a copy of gm_partial.hip whose node ticks stop after one
section on chosen ticks, so the SQ instruction mix per dispatch attributes the per-node VALU / SALU /
LDS instructions to the sections (the ablated tick minus the same tick's cumulative predecessor).
Only the LAST tick of the bench run (tick 42 of `bench.py --scenario S-C --steps 16 --warmup 1`)
is cut, so the state it runs on is the normal one (an ablated tick sends nothing and writes no list:
the ticks after it are not representative). Level -> last section kept:
  1: loads + table clear + own insert + delivered-list inserts
  2: + self bump + sweep / compaction
  3: + dense read + eviction
  4: + compaction of the kept entries + id rank + list store + joins / numfailed
  5: + gossip draw (everything but the inbox appends and the row records)
  6: loads .. sweep + the dense read (inside level 3)
  7: + the distance histogram and the keep / bucket masks
  8: + the eviction keys of the cut bucket (before the key histogram)
Writes build_dbg/sc_l<level>/gm_partial.hip for levels 1..8.
usage: scripts/r06/sc_sections_variant.py"""
import os

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(REPO, "distributed-membership_amd/csrc/gm_partial.hip")).read()


def ins(s, anchor, text, before=True, nth=0):
    i = -1
    for _ in range(nth + 1):
        i = s.index(anchor, i + 1)
    return s[:i] + text + s[i:] if before else s[:i + len(anchor)] + text + s[i + len(anchor):]


# finer cuts inside the eviction (levels 6..8): after the dense read; after the distance histogram and
# the keep / bucket masks; after the eviction keys (a uint32_t mask keeps "v" constraints simple)
FINE = [("  mask_t keep = 0;\n  if (m <= V) {", 'asm volatile("" :: "v"(dw[0]), "v"(dw[1]), "v"(dw[2]), "v"(dh[0]), "v"(dh[1]), "v"(dh[2]))'),
        ("    if (needb == bsz) {", 'asm volatile("" :: "v"(keep), "v"(bucket))'),
        ("      p_wsync();\n      hist[lane] = 0;", 'asm volatile("" :: "v"(key[0]), "v"(key[1]), "v"(key[2]), "v"(keep))')]
CUTS = [("  // ---- 3. self bump", 'asm volatile("" :: "v"(hslot))'),
        ("  // ---- 4. dense entries", 'asm volatile("" :: "v"(m), "v"(removed), "v"(nrem))'),
        ("  // ---- 5. compact the kept entries", 'asm volatile("" :: "v"(keep))'),
        ("  // ---- 6. gossip draw", 'asm volatile("" :: "v"(numfailed), "v"(nj), "v"(jb))'),
        ("  // ---- sends: one parallel round", 'asm volatile("" :: "v"(ng))')]
for level, (anchor, use) in list(enumerate(CUTS, 1)) + list(enumerate(FINE, 6)):
    s = ins(src, anchor, f"  if (t == 42) {{ {use}; return; }}\n")
    out = os.path.join(REPO, "build_dbg", f"sc_l{level}")
    os.makedirs(out, exist_ok=True)
    open(os.path.join(out, "gm_partial.hip"), "w").write(s)
    print("wrote", os.path.join(out, "gm_partial.hip"))
