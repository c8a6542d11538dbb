#!/usr/bin/env python3
"""Per-phase cycle counts of one MARL_PARTIAL step launch (partial_kernel), block 0 /
lane 0, from the diagnostic build libmapfx_pstamps.so
(tools/build_variant.sh pstamps "" -DPARTIAL_STAMPS).

  python tools/pstamps_partial.py [E]
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MAPFX_LIB", os.path.join(REPO, "mapf-marl_amd", "mapfx", "libmapfx_pstamps.so"))
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import bench
    import mapfx
    from mapfx.maps import synthetic_instances
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    S, N = 8, 15
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.0, seed=1)
    b = mapfx.MarlPartialBatch(inst["init_pos"], inst["goals"], grids=np.zeros((1, S, S), np.int8),
                               **bench.PARTIAL_YAML)
    b.reset()
    ga = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S), obs=(),
                             track_steps=False)
    acts = ga.gen_actions(40, seed=2)
    lib = mapfx.lib
    lib.mapfx_partial_debug_stamps.restype = ctypes.c_int
    names = ["entry", "loads issued, bitmap staged", "map build",
             "state + action decoded (+ fallback lookups)", "agents counted", "step: moves, count atomics",
             "step: node / edge collisions, rewards", "step: reward fold", "neighbour lookups issued",
             "feature rows", "window + KNN rows (registers)", "staged copy-out",
             "avail / state / write-back issued", "stores drained"]
    rows = []
    for k in range(40):
        b.step(acts[k])
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 16)()
        assert lib.mapfx_partial_debug_stamps(buf) == 0
        st = np.array(buf, dtype=np.int64)[:len(names)]
        if k >= 8:
            rows.append(np.diff(st) % (1 << 32))  # (32-bit stamps)
    d = np.array(rows)
    print("E=%d partial_kernel, block 0 / lane 0: s_memtime cycles per phase (median / mean of %d launches)"
          % (E, len(rows)))
    for i, nm in enumerate(names[1:]):
        print("  %-36s %7.0f %7.0f" % (nm, np.median(d[:, i]), d[:, i].mean()))
    print("  %-36s %7.0f" % ("TOTAL entry -> drained", np.median(d.sum(1))))
    # every block of the last launch: s_memrealtime (10 ns ticks) relative to the first start
    nb = (E + 3) // 4
    bb = (ctypes.c_uint * (nb * 6))()
    if hasattr(lib, "mapfx_partial_debug_blocks") and lib.mapfx_partial_debug_blocks(bb, nb) == 0:
        t = np.array(bb, dtype=np.int64).reshape(nb, 6)
        t = (t - t[:, 0].min()) % (1 << 32)
        print("every block of the last launch, us after the first block's start (p0 / p50 / p90 / p100):")
        for i, nm in enumerate(["start", "loads + bitmap", "pre-obs done", "obs rows in registers",
                                "copy-out done", "drained"]):
            v = t[:, i] / 100.0
            print("  %-24s %6.2f %6.2f %6.2f %6.2f" % (nm, *np.percentile(v, [0, 50, 90, 100])))


if __name__ == "__main__":
    main()
