#!/usr/bin/env python3
"""Map data for the F1 full-range tests (build container only): the obstacle grids of
the reference's shipped maps with a side above 256 or a non-square shape
(MARL-curve-main/src/mapf_baseline/mapf-map/*.map -- MovingAI benchmark maps: data,
not source), packed LSB-first as tests/golden/big_maps.npz so that the GPU box,
which has no /root/reference, can load them.  Keys: <name>_bits (uint8), <name>_hw.

Usage:  python tests/golden/gen_big_maps.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_fixtures as G  # noqa: E402

NAMES = ("warehouse-20-40-10-2-1", "den520d", "brc202d", "orz900d", "w_woundedcoast",
         "ht_mansion_n", "warehouse-20-40-10-2-2")


def main():
    out = {}
    for n in NAMES:
        g = G.read_map_grid(os.path.join(G.MAP_DIR, n + ".map"))
        key = n.replace("-", "_")
        out[key + "_bits"] = np.packbits((g != 0).reshape(-1), bitorder="little")
        out[key + "_hw"] = np.array(g.shape, dtype=np.int32)
    path = os.path.join(G.OUT_DIR, "big_maps.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
