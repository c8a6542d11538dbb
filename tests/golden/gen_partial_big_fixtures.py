#!/usr/bin/env python3
"""MARL_PARTIAL_ENV goldens on maps larger than 64x64, by RUNNING THE REFERENCE
(build container only; SURVEY.md §8(f) F1, VERDICT r01 "F1 at reference map sizes").

Same recording as gen_partial_fixtures.py (mp_*.npz): the reference's own A*
goal-distance tables (networkx, :947-955), reset observation and every step's
reward / flags / positions / obs / state / avail.  Cases:
  * mp_maze128_n2: the reference's maze-128-128-10.map (mapf_baseline/mapf-map),
    2 agents, window 5, K 2;
  * mp_rand80_n4: a connected random 80x80 map (20% obstacles), 4 agents, window 3, K 3;
  * mp_out8_n5: output=True (collision repair, :262-275 / :645-820) on an 8x8
    map, 5 agents, random actions.
The A* tables make each case minutes of CPU (one A* per (goal, free cell), at
construction and again at reset).

Usage:  python tests/golden/gen_partial_big_fixtures.py [maze128] [rand80] [out8]
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_fixtures as G  # noqa: E402
import gen_partial_fixtures as P  # noqa: E402


def main():
    tmp = tempfile.mkdtemp(prefix="mp_big_")
    only = sys.argv[1:]   # case names to (re)generate; each case has its own seed

    if not only or "maze128" in only:
        rng = np.random.default_rng(77)
        mpz = os.path.join(G.MAP_DIR, "maze-128-128-10.map")
        gz = G.read_map_grid(mpz)
        cells = P.free_cells(gz)
        pick = rng.choice(len(cells), size=4, replace=False)
        starts, goals = [cells[i] for i in pick[:2]], [cells[i] for i in pick[2:]]
        sc = P.write_scen(tmp, "maze128", 128, starts, goals)
        env, args = P.make(mpz, sc, 2, py_seed=31, obs_window=5, obs_knn_agents=2, episode_limit=30)
        acts = rng.integers(0, 5, size=(25, 2)).astype(np.int64)
        P.run("maze128_n2", env, args, acts, reset_seed=37, grid=gz)

    if not only or "rand80" in only:
        rng = np.random.default_rng(78)
        g80 = P.connected_random_grid(rng, 80, 0.2)
        mp80, _ = G.write_map(tmp, "rand80", g80)
        cells = P.free_cells(g80)
        pick = rng.choice(len(cells), size=8, replace=False)
        sc = P.write_scen(tmp, "rand80", 80, [cells[i] for i in pick[:4]], [cells[i] for i in pick[4:]])
        env, args = P.make(mp80, sc, 4, py_seed=41, obs_window=3, obs_knn_agents=3, episode_limit=40,
                           move_reward=-0.01, stay_reward=-0.02, stay_goal_reward=0,
                           node_collide_reward=-1, edge_collide_reward=-1, env_collide_reward=-1)
        acts = rng.integers(0, 5, size=(30, 4)).astype(np.int64)
        P.run("rand80_n4", env, args, acts, reset_seed=43, grid=g80)

    if not only or "out8" in only:
        # output mode (:262-275, :645-820): no collision may remain -- the reference
        # repairs node / edge collisions with random.shuffle'd tries after the rewards
        rng = np.random.default_rng(79)
        g6 = np.zeros((8, 8), dtype=np.int8)
        g6[3, 3] = g6[5, 6] = -1
        mp6, _ = G.write_map(tmp, "out8", g6)
        cells = P.free_cells(g6)
        pick = rng.choice(len(cells), size=10, replace=False)
        starts, goals = [cells[i] for i in pick[:5]], [cells[i] for i in pick[5:]]
        sc = P.write_scen(tmp, "out8", 8, starts, goals)
        env, args = P.make(mp6, sc, 5, py_seed=47, episode_limit=60, output=True)
        acts = rng.integers(0, 5, size=(50, 5)).astype(np.int64)
        P.run("out8_n5", env, args, acts, reset_seed=53, grid=g6)
        # what a replay needs to redraw the same instance with the same `random` calls:
        # the scen file lines (write_scen order) and both seeds
        path = os.path.join(G.OUT_DIR, "mp_out8_n5.npz")
        rec = dict(np.load(path, allow_pickle=False))
        rec.update(scen_starts=np.array(starts, np.int32), scen_goals=np.array(goals, np.int32),
                   meta_py_seed=np.array(47), meta_reset_seed=np.array(53))
        np.savez_compressed(path, **rec)


if __name__ == "__main__":
    main()
