#!/usr/bin/env python3
"""Per-phase cycle counts of the generic rollout step at C5 (128x128, 256 agents, one
env per block), block 0 / thread 0 (wave 0's lane 0, the fold lane): diagnostic build
libmapfx_stamps.so (tools/build_variant.sh stamps "" -DMAPFX_STAMPS).

  python tools/stamps_c5.py
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
    S, N, E, p, _ = bench.CONFIGS["c5"]
    inst = synthetic_instances(E, S, S, N, p_obstacle=p, seed=1)
    b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                            episode_limit=2 ** 31 - 1, obs=("window_occ",), window=5, track_steps=False)
    b.reset()
    T = 64
    acts = b.gen_actions(T * 3, seed=2)
    traj = b._alloc_out(T)
    outs = ("reward", "term", "node", "edge", "avail", "obs_window_occ", "traj_pos", "traj_done", "traj_t")
    for i in range(3):
        b.rollout(T, actions=acts[i * T:(i + 1) * T], traj=traj, outputs=outs)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (256 * 8))()
    mapfx.lib.mapfx_debug_stamps.restype = ctypes.c_int
    assert mapfx.lib.mapfx_debug_stamps(buf) == 0
    st = np.array(buf, dtype=np.int64).reshape(256, 8)[:T]
    names = ["P0 move + B1", "P1 atomics + B2", "edge scan", "P2 per-agent outputs",
             "B2b + tail/fold", "window records", "B3"]
    fold = (np.arange(T) % 8) == 7
    rows = np.arange(1, T - 1)
    print("C5 E=%d T=%d: s_memtime cycles per phase, block 0 thread 0 (median: plain steps / fold steps)" % (E, T))
    for k in range(7):
        d = st[rows, k + 1] - st[rows, k]
        print("  %-22s %7.0f %7.0f" % (names[k], np.median(d[~fold[rows]]), np.median(d[fold[rows]])))
    nxt = st[2:, 0] - st[1:-1, 7]
    print("  %-22s %7.0f" % ("P3 + B4 -> next step", np.median(nxt)))
    tot = st[2:, 0] - st[1:-1, 0]
    print("  %-22s %7.0f %7.0f" % ("step total", np.median(tot[~fold[1:-1]]), np.median(tot[fold[1:-1]])))


if __name__ == "__main__":
    main()
