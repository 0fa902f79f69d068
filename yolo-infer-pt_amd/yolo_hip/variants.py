"""YOLOv11 variant tables.

Mirrors the constructor tables of the reference (nets/nn.py:308-347): every
variant is described by the channel widths of its five pyramid levels, the
repeat count of each C3k2 block and whether the C3k2 blocks of the shallow /
deep stages use nested C3k modules.
"""
from dataclasses import dataclass
from typing import Tuple


@dataclass(frozen=True)
class Variant:
    name: str
    width: Tuple[int, int, int, int, int, int]
    depth: Tuple[int, int, int, int, int, int]
    csp: Tuple[bool, bool]


_SHALLOW = (False, True)   # n/t/s: plain bottlenecks in the shallow C3k2 blocks
_DEEP = (True, True)       # m/l/x: C3k everywhere

VARIANTS = {
    # nets/nn.py:308-312
    "n": Variant("n", (3, 16, 32, 64, 128, 256), (1,) * 6, _SHALLOW),
    # nets/nn.py:315-319
    "t": Variant("t", (3, 24, 48, 96, 192, 384), (1,) * 6, _SHALLOW),
    # nets/nn.py:322-326
    "s": Variant("s", (3, 32, 64, 128, 256, 512), (1,) * 6, _SHALLOW),
    # nets/nn.py:329-333
    "m": Variant("m", (3, 64, 128, 256, 512, 512), (1,) * 6, _DEEP),
    # nets/nn.py:336-340
    "l": Variant("l", (3, 64, 128, 256, 512, 512), (2,) * 6, _DEEP),
    # nets/nn.py:343-347
    "x": Variant("x", (3, 96, 192, 384, 768, 768), (2,) * 6, _DEEP),
}


def lookup(width, depth, csp) -> Variant:
    """Return the Variant matching a (width, depth, csp) triple, or an ad-hoc one."""
    w, d, c = tuple(int(v) for v in width), tuple(int(v) for v in depth), tuple(bool(v) for v in csp)
    for v in VARIANTS.values():
        if v.width == w and v.depth == d and v.csp == c:
            return v
    return Variant("custom", w, d, c)
