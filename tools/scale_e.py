#!/usr/bin/env python3
"""Fused-rollout throughput vs number of envs (waves per SIMD) at 32x32 / 16 agents:
tells whether a step is bound per wave (latency / issue) or by a shared resource.

  python tools/scale_e.py [--T 64]
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
    ap.add_argument("--T", type=int, default=64)
    ap.add_argument("--launches", type=int, default=6)
    ap.add_argument("--envs", default="256,1024,2048,4096,8192,16384,32768")
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--S", type=int, default=32, help="grid side (C5: 128)")
    ap.add_argument("--Ts", default="", help="comma list of T at E=4096 instead of the E sweep")
    ap.add_argument("--rng", action="store_true", help="device-generated actions (no action loads)")
    a = ap.parse_args()
    import mapfx
    from mapfx.maps import synthetic_instances
    S, N, T = a.S, a.n, a.T
    outs = ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos", "traj_done",
            "traj_t")
    runs = [(int(x), T) for x in a.envs.split(",")]
    if a.Ts:
        runs = [(4096, int(t)) for t in a.Ts.split(",")]
    for E, T in runs:
        inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=1)
        b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                                episode_limit=2 ** 31 - 1, obs=("window",), window=5,
                                track_steps=False)
        b.reset()
        launches = max(2, a.launches * a.T // T)
        acts = b.gen_actions(T * launches, seed=2)
        traj = b._alloc_out(T)
        res = []
        for rnd in range(3):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(launches):
                if a.rng:
                    b.rollout(T, seed=2, t0=i * T, traj=traj, outputs=outs)
                else:
                    b.rollout(T, actions=acts[i * T:(i + 1) * T], traj=traj, outputs=outs)
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / (launches * T) * 1e3)
        us = float(np.min(res))
        print("E=%6d T=%4d waves=%6d  us/step %.3f  G agent-steps/s %.2f"
              % (E, T, E * N // 64, us, E * N / us * 1e-3))
        del b, traj, acts


if __name__ == "__main__":
    main()
