#!/usr/bin/env python3
"""Per-step launch (mapfx_step) time vs env count at 32x32 / 16 agents, window obs:
HIP-graph replay of 100 launches, so it is kernel time plus the graph's
back-to-back launch gap.  Tells fixed per-launch latency from per-env cost.

  python tools/scale_step.py [--envs 256,1024,4096,16384]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", default="64,256,1024,4096,16384")
    ap.add_argument("--n", type=int, default=16)
    a = ap.parse_args()
    import mapfx
    from mapfx.maps import synthetic_instances
    S, N, ks = 32, a.n, 100
    for E in [int(x) for x in a.envs.split(",")]:
        inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=1)
        b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                                episode_limit=2 ** 31 - 1, obs=("window",), window=5, track_steps=False)
        b.reset()
        acts = b.gen_actions(ks, seed=2)
        outs = ("reward", "term", "node", "edge", "avail", "obs_window")
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for k in range(ks):
                b.step(acts[k], outputs=outs)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for k in range(ks):
                b.step(acts[k], outputs=outs)
        g.replay()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / ks * 1e3)
        print("E=%6d  us/step %.3f  G agent-steps/s %.2f" % (E, best, E * N / best * 1e-3), flush=True)
        del g, b


if __name__ == "__main__":
    main()
