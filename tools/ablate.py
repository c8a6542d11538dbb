#!/usr/bin/env python3
"""A/B timing of the fused rollout with output subsets (one process, interleaved
rounds, MI355X).  Tells which part of a step costs what.

  python tools/ablate.py [--config c2] [--T 64] [--rounds 5]
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
    ap.add_argument("--config", default="c2")
    ap.add_argument("--T", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=8)
    ap.add_argument("--quick", action="store_true", help="runner rollout + per-step only")
    a = ap.parse_args()
    import bench
    import mapfx
    from mapfx.maps import synthetic_instances, warehouse_grid
    S, N, E, p, shared = bench.CONFIGS[a.config]
    inst = synthetic_instances(E, S, S, N, p_obstacle=p or 0.0, seed=1,
                               shared_grid=warehouse_grid(S) if shared else None)
    b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                            episode_limit=2 ** 31 - 1, obs=("window", "full"), window=5,
                            track_steps=False)
    b.reset()
    T = a.T
    acts = b.gen_actions(T * a.launches, seed=2)
    traj = b._alloc_out(T)
    full = ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos", "traj_done",
            "traj_t")
    variants = {
        "all": full,
        "no_window": tuple(k for k in full if k != "obs_window"),
        "window_only": ("obs_window",),
        "reward_term": ("reward", "term"),
        "nothing": (),
        "all+full_obs": full + ("obs_full",),
    }
    if a.quick:
        variants = {"all": full, "nothing": ()}
    res = {k: [] for k in variants}
    for rnd in range(a.rounds + 1):
        for name, outs in variants.items():
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for i in range(a.launches):
                b.rollout(T, actions=acts[i * T:(i + 1) * T], traj=traj, outputs=outs)
            ev[1].record()
            torch.cuda.synchronize()
            if rnd:
                res[name].append(ev[0].elapsed_time(ev[1]) / (a.launches * T) * 1e3)
    for name, v in res.items():
        print("%-14s us/step median %.3f  min %.3f" % (name, np.median(v), np.min(v)))
    # per-step drop-in path: one mapfx_step launch per env step
    pouts = ("reward", "term", "node", "edge", "avail", "obs_window")
    ks = 100
    for k in range(10):
        b.step(acts[k], outputs=pouts)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(ks)]
    for k in range(ks):
        ev[k][0].record()
        b.step(acts[k], outputs=pouts)
        ev[k][1].record()
    torch.cuda.synchronize()
    print("%-14s us/step median %.3f" % ("per_step", np.median([x.elapsed_time(y) * 1e3 for x, y in ev])))
    if a.quick:
        return
    # rng actions instead of HBM actions
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for i in range(a.launches):
        b.rollout(T, actions=None, seed=3, traj=traj, outputs=full)
    ev[1].record()
    torch.cuda.synchronize()
    print("%-14s us/step %.3f" % ("rng_actions", ev[0].elapsed_time(ev[1]) / (a.launches * T) * 1e3))
    print("info", b.info())


if __name__ == "__main__":
    main()
