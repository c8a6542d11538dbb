#!/usr/bin/env python3
"""Diagnose C5 full-size rollout obs_window vs C oracle mismatches."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]
import numpy as np
import torch
import mapfx
from mapfx.maps import synthetic_instances
from oracle import corc
E = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
T = int(sys.argv[2]) if len(sys.argv) > 2 else 8
S, N = 128, 256
inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=1)
b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                        episode_limit=2000, obs=("window",))
ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], S, S, limit=2000)
b.reset()
traj = b.rollout(T, seed=2, t0=0)
ref = ob.rollout(T, seed=2, t0=0)
g = traj["obs_window"][-1].cpu().numpy()
print("dtypes", g.dtype, ref["obs_window"].dtype, g.shape, ref["obs_window"].shape)
d = g != ref["obs_window"]
print("mismatch elems", d.sum(), "envs", np.unique(np.nonzero(d)[0]).size)
idx = np.argwhere(d)
print("first", idx[:10])
if len(idx):
    e, a = idx[0][0], idx[0][1]
    print("gpu\n", g[e, a]); print("ref\n", ref["obs_window"][e, a])
    print("pos", ob.pos[e, a])
# observe-pass on the final state
o2 = b.observe() if hasattr(b, "observe") else None
if o2 is not None and "obs_window" in o2:
    g2 = o2["obs_window"].cpu().numpy()
    print("observe() vs ref mismatches", (g2 != ref["obs_window"]).sum(), "observe vs traj", (g2 != g).sum())
