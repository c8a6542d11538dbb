#!/usr/bin/env python3
"""Per-segment cycle counts of one rollout step, block 0 / lane 0 (diagnostic build
libmapfx_stamps.so: tools/build_variant.sh stamps "" -DMAPFX_STAMPS).

  MAPFX_PROBE_E=4096 python tools/stamps.py
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
    E = int(os.environ.get("MAPFX_PROBE_E", E))
    inst = synthetic_instances(E, S, S, N, p_obstacle=p, seed=1)
    b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                            episode_limit=2 ** 31 - 1, obs=("window",), window=5, track_steps=False)
    b.reset()
    T = int(os.environ.get("MAPFX_PROBE_T", 64))
    acts = b.gen_actions(T * 3, seed=2)
    traj = b._alloc_out(T)
    outs = ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos", "traj_done", "traj_t")
    for i in range(3):
        b.rollout(T, actions=acts[i * T:(i + 1) * T], traj=traj, outputs=outs)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (256 * 8))()
    mapfx.lib.mapfx_debug_stamps.restype = ctypes.c_int
    assert mapfx.lib.mapfx_debug_stamps(buf) == 0
    full = np.array(buf, dtype=np.int64).reshape(256, 8)
    st = full[:T]
    pro = full[255]  # prologue: 6 entry, 0 state loads issued, 1 bitmap, 2 map built, 3 agents + neighbours
    if pro[6] and pro[3]:
        seq = [pro[6], pro[0], pro[1], pro[2], pro[3], st[0, 0]]
        print("prologue (block 0 / lane 0, cycles): state loads issued %d, bitmap %d, map built %d, "
              "agents + neighbours %d, -> step 0 %d" % tuple(np.diff(seq)))
    order = [0, 2, 1, 3, 4, 6]
    names = ["A move+atomics", "B rows+fold", "C heavy+tail", "D nbrs+dones", "end barrier/fence"]
    print("E=%d  s_memtime cycles per step segment (median / mean over steps 1..T-2)" % E)
    for k in range(len(order) - 1):
        d = st[1:-1, order[k + 1]] - st[1:-1, order[k]]
        print("  %-18s %7.0f %7.0f" % (names[k], np.median(d), d.mean()))
    nxt = st[2:, 0] - st[1:-1, 6]
    print("  %-18s %7.0f %7.0f" % ("loop+actions", np.median(nxt), nxt.mean()))
    tot = st[2:, 0] - st[1:-1, 0]
    print("  %-18s %7.0f %7.0f" % ("step total", np.median(tot), tot.mean()))
    # the first steps of a launch against the rest (cold instruction / scalar caches,
    # every block in the same phase)
    per = st[1:, 0] - st[:-1, 0]
    print("  step totals, steps 0..9:", " ".join("%d" % v for v in per[:10]),
          "| median of steps 10..%d: %.0f" % (T - 2, np.median(per[10:])))
    if st[2:T - 1, 5].any():  # store-wave split: busy time of each wave per barrier interval
        rel = st[1:T - 2, 6]          # release of barrier s (the step wave's stamp 6 of s - 1)
        rows = slice(2, T - 1)
        iv = st[rows, 6] - rel
        print("  split path, cycles per barrier interval (median / mean), from the release:")
        for name, col in (("step wave busy", 4), ("store wave 0 busy", 5), ("store wave 1 busy", 7)):
            d = st[rows, col] - rel
            print("  %-18s %7.0f %7.0f" % (name, np.median(d), d.mean()))
        print("  %-18s %7.0f %7.0f" % ("interval", np.median(iv), iv.mean()))
        for par, col in ((0, 5), (1, 7)):
            d = st[rows, col] - rel
            q = np.arange(2, T - 1) - 2
            a_, b_ = d[(q & 1) == par], d[(q & 1) != par]
            print("  store wave %d: a parts %6.0f, b parts %6.0f (median)" % (par, np.median(a_), np.median(b_)))


if __name__ == "__main__":
    main()
