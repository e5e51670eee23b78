#!/usr/bin/env python3
"""Measurement build (not product code): a copy of gm_partial.hip whose node ticks stop after one
section on chosen ticks, so the SQ instruction mix per dispatch attributes the per-node VALU / SALU /
LDS instructions to the sections (the ablated tick minus the same tick's cumulative predecessor).
Tick -> last section kept:
  29: loads + table clear + own insert + delivered-list inserts
  32: + self bump + sweep / compaction
  35: + dense read + eviction
  38: + compaction of the kept entries + id rank + list store + joins / numfailed
  41: + gossip draw (everything but the inbox appends and the row records)
Two normal ticks separate the ablated ones (an ablated tick sends nothing, so the next tick's inboxes
are empty). Writes build_dbg/sc_sections/gm_partial.hip.
usage: scripts/r06/sc_sections_variant.py"""
import os

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(REPO, "distributed-membership_amd/csrc/gm_partial.hip")).read()


def ins(s, anchor, text, before=True, nth=0):
    i = -1
    for _ in range(nth + 1):
        i = s.index(anchor, i + 1)
    return s[:i] + text + s[i:] if before else s[:i + len(anchor)] + text + s[i + len(anchor):]


s = src
s = ins(s, "  // ---- 3. self bump", '  if (t == 29) { asm volatile("" :: "v"(hslot)); return; }\n')
s = ins(s, "  // ---- 4. dense entries", '  if (t == 32) { asm volatile("" :: "v"(m), "v"(removed), "v"(nrem)); return; }\n')
s = ins(s, "  // ---- 5. compact the kept entries", '  if (t == 35) { asm volatile("" :: "v"(keep)); return; }\n')
s = ins(s, "  // ---- 6. gossip draw", '  if (t == 38) { asm volatile("" :: "v"(numfailed), "v"(nj), "v"(jb)); return; }\n')
s = ins(s, "  // ---- sends: one parallel round", '  if (t == 41) { asm volatile("" :: "v"(ng)); return; }\n')
out = os.path.join(REPO, "build_dbg", "sc_sections")
os.makedirs(out, exist_ok=True)
open(os.path.join(out, "gm_partial.hip"), "w").write(s)
print("wrote", os.path.join(out, "gm_partial.hip"))
