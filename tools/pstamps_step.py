#!/usr/bin/env python3
"""Per-phase cycle counts of one per-step launch (mapf_wave_kernel, T = 1) at the C2 shape,
block 0 / lane 0, from the diagnostic build libmapfx_stamps.so
(tools/build_variant.sh stamps "" -DMAPFX_STAMPS).

  python tools/pstamps_step.py
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MAPFX_LIB", os.path.join(REPO, "mapf-marl_amd", "mapfx", "libmapfx_stamps.so"))
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import bench
    import mapfx
    from mapfx.maps import synthetic_instances
    S, N, E, p, _ = bench.CONFIGS["c2"]
    inst = synthetic_instances(E, S, S, N, p_obstacle=p, seed=1)
    b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                            episode_limit=2 ** 31 - 1, obs=("window",), window=5, track_steps=False)
    b.reset()
    acts = b.gen_actions(48, seed=2)
    mapfx.lib.mapfx_debug_stamps.restype = ctypes.c_int
    rows = []
    for k in range(48):
        b.step(acts[k])
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (256 * 8))()
        assert mapfx.lib.mapfx_debug_stamps(buf) == 0
        st = np.array(buf, dtype=np.int64).reshape(256, 8)
        pro, s0 = st[255], st[0]
        # prologue 6 -> 0 -> 1 -> 2 -> 3, step 0 -> 2 -> 1 -> 3 -> 4 -> 6, epilogue 4 -> 5
        seq = [pro[6], pro[0], pro[1], pro[2], pro[3], s0[0], s0[2], s0[1], s0[3], s0[4], s0[6], pro[4], pro[5]]
        if k >= 8:
            rows.append(np.diff(seq))
    d = np.array(rows)
    names = ["state loads issued", "bitmap in registers / staged", "map built", "agents + neighbours",
             "-> step", "A move + atomics", "B rows", "C heavy (records, stores)", "D neighbours + dones",
             "end of step", "outputs + state write-back issued", "stores drained"]
    print("C2 shape (E=%d, %dx%d, N=%d), per-step launch, block 0 / lane 0: s_memtime cycles" % (E, S, S, N))
    for i, nm in enumerate(names):
        print("  %-34s %7.0f %7.0f" % (nm, np.median(d[:, i]), d[:, i].mean()))
    print("  %-34s %7.0f" % ("TOTAL", np.median(d.sum(1))))


if __name__ == "__main__":
    main()
