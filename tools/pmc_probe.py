#!/usr/bin/env python3
"""Minimal driver for PMC passes: a few fused-rollout launches of the C2 bench
workload (optionally one output subset), nothing else on the GPU."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]
import torch  # noqa: E402


def main():
    import bench
    import mapfx
    from mapfx.maps import synthetic_instances
    variant = sys.argv[1] if len(sys.argv) > 1 else "all"
    S, N, E, p, _ = bench.CONFIGS["c2"]
    E = int(os.environ.get("MAPFX_PROBE_E", E))
    inst = synthetic_instances(E, S, S, N, p_obstacle=p, seed=1)
    b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                            episode_limit=2 ** 31 - 1, obs=("window",), window=5,
                            track_steps=False)
    b.reset()
    T = 64
    acts = b.gen_actions(T * 4, seed=2)
    traj = b._alloc_out(T)
    outs = {"all": ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos",
                    "traj_done", "traj_t"), "nothing": ()}[variant]
    for i in range(4):
        b.rollout(T, actions=acts[i * T:(i + 1) * T], traj=traj, outputs=outs)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
