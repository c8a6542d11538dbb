#!/usr/bin/env python3
"""One env step at the C2 shape two ways, each as a HIP graph of 200 launches replayed
(the bench's per-step method): mapfx_step with the drop-in output set, and a T = 1
mapfx_rollout with the bench's rollout output set (the split kernel: a step wave and
two store waves).  Prints us per launch and the kernel instance of each.
usage: python3 tools/step_vs_split.py [--reps 5]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ks", type=int, default=200)
    a = ap.parse_args()
    import bench
    import mapfx
    from mapfx import _abi
    from mapfx.maps import synthetic_instances
    S, N, E, p, shared = bench.CONFIGS["c2"]
    inst = synthetic_instances(E, S, S, N, p_obstacle=p or 0.0, seed=1)
    b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                            episode_limit=2 ** 31 - 1, obs=("window",), window=5, track_steps=False)
    b.reset()
    ks = a.ks
    acts = b.gen_actions(ks, seed=2)
    pouts = ("reward", "term", "node", "edge", "avail", "obs_window")
    routs = ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos", "traj_done", "traj_t")
    traj = b._alloc_out(1)
    traj.pop("reward_f32")
    stream = torch.cuda.current_stream()

    def by_step():
        for k in range(ks):
            b.step(acts[k], outputs=pouts)

    def by_rollout():
        for k in range(ks):
            b.rollout(1, actions=acts[k:k + 1], traj=traj, outputs=routs)

    for name, fn in (("mapfx_step", by_step), ("rollout T=1", by_rollout)):
        side = torch.cuda.Stream()
        side.wait_stream(stream)
        with torch.cuda.stream(side):
            fn()
        stream.wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        g.replay()
        torch.cuda.synchronize()
        kern = _abi.last_kernel()
        us = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            g.replay()
            e1.record(stream)
            torch.cuda.synchronize()
            us.append(e0.elapsed_time(e1) * 1e3 / ks)
        print("%-12s %6.3f us per launch (median of %d graph replays)  %s"
              % (name, float(np.median(us)), a.reps, kern[kern.find("<"):kern.find(">") + 1]), flush=True)


if __name__ == "__main__":
    main()
