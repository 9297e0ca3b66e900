"""Index-width audit (the r03b incident): at N = 1e9 a
friends-table index `v * stride + j` passes 2^32 (1e9 nodes x 6..32 slots),
so every such product in the device code must be formed in 64 bits -- the
node variable declared 64-bit, or cast before the multiply.  The r03b call's
log was lost, so its fault cannot be named; this CPU test pins the property
that was audited instead, for every kernel source that indexes the table.
"""
from __future__ import annotations

import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gossip_simulator_amd", "csrc")
WIDE = ("uint64_t", "size_t", "unsigned long long", "int64_t")
# an index into a friends table: <table>[<var> * <...>stride + ...] or a row
# pointer <table> + <var> * <...>stride
PAT = re.compile(r"\b((?:s\.|w\.|p\.)?ids)\s*(?:\[|\+)\s*(\(\s*(?:uint64_t|size_t)\s*\)\s*)?(\w+)\s*\*\s*"
                 r"(?:s\.|p\.|w\.)?stride")


def declared_type(src: str, pos: int, name: str) -> str | None:
    """Type of the nearest declaration of `name` before `pos` (parameters and
    locals alike), or None."""
    decl = re.compile(r"\b(uint64_t|size_t|unsigned long long|int64_t|uint32_t|int|unsigned)\s+(?:const\s+)?"
                      r"(?:\w+\s*=\s*[^,;]*,\s*)*" + re.escape(name) + r"\b")
    last = None
    for m in decl.finditer(src, 0, pos):
        last = m.group(1)
    return last


@pytest.mark.parametrize("fname", ["gs_pushpull.hip", "gs_overlay.hip", "gs_window.hip", "gs_broadcast.hip"])
def test_table_indices_are_64_bit(fname):
    path = os.path.join(CSRC, fname)
    src = open(path).read()
    found, bad = 0, []
    for m in PAT.finditer(src):
        found += 1
        if m.group(2):  # explicit 64-bit cast
            continue
        var = m.group(3)
        t = declared_type(src, m.start(), var)
        if t not in WIDE:
            line = src.count("\n", 0, m.start()) + 1
            bad.append(f"{fname}:{line}: `{var}` is {t or 'undeclared'} in {src[m.start():m.end() + 8]!r}")
    assert not bad, "32-bit table index products:\n" + "\n".join(bad)
    if fname in ("gs_pushpull.hip", "gs_overlay.hip"):
        assert found > 0  # the audit sees the indexing it is meant to check
