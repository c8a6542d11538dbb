#!/usr/bin/env python3
"""Build diagnostic variants of libmapfx.so next to the shipped one (A/B timing on the
GPU box via MAPFX_LIB=...): python tools/build_variants.py NAME=-DFLAG=V[,-DFLAG2=V2] ..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g  # noqa: E402

for spec in sys.argv[1:]:
    name, flags = spec.split("=", 1)
    out = os.path.join(g.PKG_ROOT, "mapfx", "libmapfx_%s.so" % name)
    g.build_hip(extra_flags=[f for f in flags.split(",") if f], out_lib=out)
    print("built", out)
