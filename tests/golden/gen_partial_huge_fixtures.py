#!/usr/bin/env python3
"""MARL_PARTIAL_ENV goldens at the reference's full input range, by RUNNING THE
REFERENCE (build container only; SURVEY.md §8(f) F1, VERDICT r02 "F1 at the
reference's full input range"): N > 64 agents and sides > 256.

The reference runs on SQUARE maps only: MARL_PARTIAL_ENV.__create_grid
(marl_partial.py:523-533) indexes `_grid[i][j]` with i over the columns and j over
the rows, the same quirk as MAPF_GRID, and raises IndexError on
every non-square map -- which includes all seven shipped maps with a side above
256 (brc202d, den520d, ht_mansion_n, orz900d, w_woundedcoast, warehouse-20-40-*).
Those run here against the CPU restatement (oracle/partial_oracle.py, pinned by
these goldens) in tests/test_gpu_partial.py; the goldens below are square.

Same recording as gen_partial_fixtures.py (mp_*.npz).  Cases:
  * mp_rand64_n100: the reference's random-64-64-10 map, 100 agents, the yaml
    config (window 5, K 5), A* tables exactly as the reference builds them;
  * mp_sq300_n70: a connected random 300 x 300 map (sides above 256 AND N above 64),
    70 agents, window 7;
  * mp_orzcrop512_n3: the top-left 512 x 512 square of the reference's orz900d map
    (its largest), 3 agents in its largest component.
Goal-distance tables: the reference builds them with one networkx A* per (goal,
free cell) (:931-955), O(cells^2) per agent -- hours on the 90K+ cell maps.  The
`bfs` cases replace only __setup_agent_goal_dist by networkx's own
single_source_shortest_path_length from the goal on the same graph: on this
unweighted undirected graph it returns the same lengths as A* with the admissible
L2 heuristic (pinned where both ran: mp_rand64_n100 and every earlier mp_*
fixture), in O(cells).  The mode is stored as meta_goal_dist_mode.  Everything
else (moves, collisions, rewards, KNN observations, state, avail) is the
reference's own code.

Usage:  python tests/golden/gen_partial_huge_fixtures.py [case ...]
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_fixtures as G  # noqa: E402
import gen_partial_fixtures as P  # noqa: E402

MP = G.MP


def bfs_goal_dist(self):
    """__setup_agent_goal_dist (:931-945) with networkx BFS lengths instead of one A*
    per cell (same lengths on the unweighted graph)."""
    import networkx as nx
    coord = type(next(iter(self._global_graph.nodes)))
    for i, goal in enumerate(self._agent_goal_pos):
        lengths = nx.single_source_shortest_path_length(self._global_graph, coord(goal[0], goal[1]))
        ncol = self._grid_shape[1]
        self._goal_dist[i] = {v.row * ncol + v.col: d for v, d in lengths.items()}


def case(name, grid, n, seed, T, mode, map_name, **kw):
    tmp = tempfile.mkdtemp(prefix="mp_huge_")
    rng = np.random.default_rng(seed)
    mpath, _ = G.write_map(tmp, name, grid)
    cells = P.free_cells(grid)
    pick = rng.choice(len(cells), size=2 * n, replace=False)
    starts, goals = [cells[i] for i in pick[:n]], [cells[i] for i in pick[n:]]
    sc = P.write_scen(tmp, name, grid.shape[0], starts, goals)
    cls = MP.MARL_PARTIAL_ENV
    orig = cls._MARL_PARTIAL_ENV__setup_agent_goal_dist
    if mode == "bfs":
        cls._MARL_PARTIAL_ENV__setup_agent_goal_dist = bfs_goal_dist
    try:
        env, args = P.make(mpath, sc, n, py_seed=seed + 1, **kw)
        acts = rng.integers(0, 5, size=(T, n)).astype(np.int64)
        P.run(name, env, args, acts, reset_seed=seed + 2, grid=grid)
    finally:
        cls._MARL_PARTIAL_ENV__setup_agent_goal_dist = orig
    path = os.path.join(G.OUT_DIR, "mp_%s.npz" % name)
    rec = dict(np.load(path, allow_pickle=False))
    rec["meta_goal_dist_mode"] = np.array(mode)
    rec["meta_map_name"] = np.array(map_name)
    np.savez_compressed(path, **rec)


def largest_component_only(grid):
    """Obstacles everywhere outside the largest 4-connected free component (agents are
    drawn there; the reference's lookups then always find a distance)."""
    from collections import deque
    h, w = grid.shape
    seen = np.zeros(grid.shape, dtype=bool)
    best = []
    for s in zip(*np.nonzero(grid == 0)):
        if seen[s]:
            continue
        comp, q = [], deque([s])
        seen[s] = True
        while q:
            r, c = q.popleft()
            comp.append((r, c))
            for dr, dc in ((1, 0), (-1, 0), (0, 1), (0, -1)):
                rr, cc = r + dr, c + dc
                if 0 <= rr < h and 0 <= cc < w and grid[rr, cc] == 0 and not seen[rr, cc]:
                    seen[rr, cc] = True
                    q.append((rr, cc))
        if len(comp) > len(best):
            best = comp
    out = np.full_like(grid, -1)
    rr, cc = np.array(best).T
    out[rr, cc] = 0
    return out


def ref_map(name):
    return G.read_map_grid(os.path.join(G.MAP_DIR, name + ".map"))


CASES = {
    "rand64": lambda: case("rand64_n100", ref_map("random-64-64-10"), 100, 201, 20, "astar",
                           "random-64-64-10", episode_limit=30),
    "sq300": lambda: case("sq300_n70", P.connected_random_grid(np.random.default_rng(205), 300, 0.2),
                          70, 205, 15, "bfs", "synthetic random 300x300 p=0.2 (largest component)",
                          obs_window=7, obs_knn_agents=5, episode_limit=25),
    "orzcrop512": lambda: case("orzcrop512_n3", largest_component_only(ref_map("orz900d")[:512, :512]),
                               3, 204, 20, "bfs", "orz900d[:512, :512] (largest component)",
                               obs_window=5, obs_knn_agents=3, episode_limit=30),
}


def main():
    only = sys.argv[1:] or list(CASES)
    for k in only:
        CASES[k]()


if __name__ == "__main__":
    main()
