#!/usr/bin/env python3
"""Prologue / step / epilogue cycle stamps of block 0, lane 0 of the wave kernel
(diagnostic build libmapfx_stamps.so: tools/build_variant.sh stamps
mapf-marl_amd/csrc/mapfx.hip -DMAPFX_STAMPS), for the per-step kernel (mapfx_step)
and a T-step rollout at C2 (32x32, 16 agents, window 5).

  python tools/pstamps.py [--envs 64,4096] [--T 20]
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MAPFX_LIB", os.path.join(REPO, "mapf-marl_amd", "mapfx", "libmapfx_stamps.so"))
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def read(mapfx):
    buf = (ctypes.c_ulonglong * (256 * 8))()
    mapfx.lib.mapfx_debug_stamps.restype = ctypes.c_int
    assert mapfx.lib.mapfx_debug_stamps(buf) == 0
    return np.array(buf, dtype=np.int64).reshape(256, 8)


def show(tag, st, T):
    p = st[255]
    pro = [("entry->loads issued", 6, 0), ("HBM loads + bits->LDS", 0, 1), ("map build", 1, 2),
           ("agent atomics + nbrs", 2, 3)]
    out = ["%s:" % tag]
    for name, a, b in pro:
        out.append("  %-24s %6d" % (name, p[b] - p[a]))
    out.append("  %-24s %6d  (%d steps, %.0f / step)" % ("loop", st[T - 1, 6] - p[3] if T > 0 else 0, T,
                                                        (st[T - 1, 6] - p[3]) / max(T, 1)))
    out.append("  %-24s %6d" % ("drain + state stores", p[4] - st[T - 1, 6]))
    out.append("  %-24s %6d" % ("wait stores (vmcnt 0)", p[5] - p[4]))
    out.append("  %-24s %6d" % ("TOTAL entry->exit", p[5] - p[6]))
    print("\n".join(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", default="64,4096")
    ap.add_argument("--T", type=int, default=20)
    a = ap.parse_args()
    import mapfx
    from mapfx.maps import synthetic_instances
    S, N, W = 32, 16, 5
    outs = ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos", "traj_done", "traj_t")
    pouts = ("reward", "term", "node", "edge", "avail", "obs_window")
    for E in [int(x) for x in a.envs.split(",")]:
        inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=1)
        b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                                episode_limit=2 ** 31 - 1, obs=("window",), window=W,
                                track_steps=False)
        b.reset()
        acts = b.gen_actions(64, seed=2)
        for k in range(8):
            b.step(acts[k], outputs=pouts)
        torch.cuda.synchronize()
        show("E=%d per-step kernel (mapfx_step)" % E, read(mapfx), 1)
        traj = b._alloc_out(a.T)
        for i in range(3):
            b.rollout(a.T, actions=acts[:a.T], traj=traj, outputs=outs)
        torch.cuda.synchronize()
        show("E=%d rollout T=%d" % (E, a.T), read(mapfx), a.T)


if __name__ == "__main__":
    main()
