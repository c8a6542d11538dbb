#!/usr/bin/env python3
"""Kernel time of one C2 rollout launch (bench.py's output set, int8 actions in HBM) vs T,
from launch-recorded events (mapfx_rollout_timed), median of 7 replays from the same
state: separates the per-launch fixed cost from the per-step cost.

  python tools/tsweep.py [--T 1,2,4,8,16,20,32,33,48,64] [--config c2]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", default="1,2,4,8,16,20,32,33,48,64")
    ap.add_argument("--config", default="c2")
    a = ap.parse_args()
    import bench
    import mapfx
    from mapfx import _abi
    from mapfx.maps import synthetic_instances, warehouse_grid
    S, N, E, p, shared = bench.CONFIGS[a.config]
    inst = synthetic_instances(E, S, S, N, p_obstacle=p or 0.0, seed=1,
                               shared_grid=warehouse_grid(S) if shared else None)
    b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                            episode_limit=2 ** 31 - 1, obs=("window",), window=5, track_steps=False)
    b.reset()
    outs = ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos", "traj_done", "traj_t")
    stream = torch.cuda.current_stream()
    state0 = [x.clone() for x in (b.pos, b.done, b.t)]
    rows = []
    for T in [int(x) for x in a.T.split(",")]:
        acts = b.gen_actions(T, seed=2)
        traj = b._alloc_out(T)
        traj.pop("reward_f32")
        ms = []
        for _ in range(7):
            for x, x0 in zip((b.pos, b.done, b.t), state0):
                x.copy_(x0)
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(stream)
            ev[1].record(stream)
            b.rollout_plan(T, actions=acts, traj=traj, outputs=outs, stream=stream, events=ev)()
            torch.cuda.synchronize()
            ms.append(ev[0].elapsed_time(ev[1]))
        k = _abi.last_kernel()
        med = float(np.median(ms)) * 1e3
        rows.append((T, med))
        print("T=%3d  kernel %8.2f us  %6.3f us/step  %s" % (T, med, med / T, k[k.find("<"):k.find(">") + 1]),
              flush=True)
    for short in (True, False):
        sel = [(t, m) for t, m in rows if (t <= 32) == short and t >= 4]
        if len(sel) >= 2:
            ts, ms_ = np.array(sel).T
            slope, icpt = np.polyfit(ts, ms_, 1)
            print("%s: fixed %.2f us + %.3f us/step (fit over T = %s)"
                  % ("T <= 32 (8-step action block)" if short else "T > 32 (16-step block)", icpt, slope,
                     ",".join("%d" % t for t in ts)))


if __name__ == "__main__":
    main()
