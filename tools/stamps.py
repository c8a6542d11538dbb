#!/usr/bin/env python3
"""Per-segment cycle shares of one rollout step (diagnostic build libmapfx_stamps.so)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MAPFX_LIB"] = os.path.join(REPO, "mapf-marl_amd", "mapfx", "libmapfx_stamps.so")
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
    T = 64
    acts = b.gen_actions(T * 3, seed=2)
    traj = b._alloc_out(T)
    traj.pop("reward_f32")
    outs = ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos", "traj_done", "traj_t")
    for i in range(3):
        b.rollout(T, actions=acts[i * T:(i + 1) * T], traj=traj, outputs=outs)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (256 * 8))()
    mapfx.lib.mapfx_debug_stamps.restype = ctypes.c_int
    assert mapfx.lib.mapfx_debug_stamps(buf) == 0
    st8 = np.array(buf, dtype=np.int64).reshape(256, 8)[:T]
    st = st8[:, [0, 7, 1, 2, 3, 4, 5, 6]]
    names = ["cand read", "tail(prev)", "move+atomics", "edge", "rows/window", "reward+stage",
             "stores+fence"]
    d = np.diff(st, axis=1)
    nxt = st[1:, 0] - st[:-1, 6]
    print("per-step cycles (median over steps 1..T-1)")
    for k in range(d.shape[1]):
        print("  %-16s median %6.0f  mean %6.0f" % (names[k], np.median(d[1:, k]), d[1:, k].mean()))
    nxt = st[1:, 0] - st[:-1, -1]
    print("  %-16s median %6.0f  mean %6.0f" % ("fence+loop+acts", np.median(nxt), nxt.mean()))
    tot = st[1:, 0] - st[:-1, 0]
    print("  step total       median %6.0f  mean %6.0f  (steps%%16==0: %s)" % (np.median(tot), tot.mean(), tot[15::16]))


if __name__ == "__main__":
    main()
