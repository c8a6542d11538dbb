#!/usr/bin/env python3
"""Pin the drop-ins' scenario draws by RUNNING THE REFERENCE (build container only).

For fixed `random.seed` values this constructs the reference's MAPF_GRID
(envs/mapf_gridworld.py:21-55, draws at :37, :432, :437) and MARL_PARTIAL_ENV
(envs/marl_partial.py:26-111 and every reset(), draws at :60, :907, :915) and
records the start / goal positions they end up with.  The MovingAI `.map` and
`.scen` files those draws read are benchmark DATA from
MARL-curve-main/src/mapf_baseline/ (mapf-map/, scen-random/); only the files a
draw actually opened are copied to tests/golden/scen/, so the CPU test can
replay the same draw through mapfx.envs without /root/reference.

Usage:  python tests/golden/gen_scen_fixtures.py   (writes tests/golden/scen/)
"""
from __future__ import annotations

import builtins
import contextlib
import io
import os
import random
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_fixtures as gf  # noqa: E402  (installs the stubs, imports the reference envs)

OUT = os.path.join(HERE, "scen")

# (case, env class, map, n_agents, py_seed, resets)
CASES = [
    ("grid_empty8_n2_s1", "grid", "empty-8-8.map", 2, 1, 0),        # = c1_empty8_n2's draw
    ("grid_random32_n16_s3", "grid", "random-32-32-10.map", 16, 3, 0),
    ("grid_maze32_n16_s4", "grid", "maze-32-32-4.map", 16, 4, 0),
    ("grid_empty8_n5_s2", "grid", "empty-8-8.map", 5, 2, 0),
    ("partial_empty8_n15_s21", "partial", "empty-8-8.map", 15, 21, 3),
    ("partial_empty8_n4_s22", "partial", "empty-8-8.map", 4, 22, 2),
]


class _OpenLog:
    """Record every .scen path the reference opens."""

    def __init__(self):
        self.paths = []
        self._open = builtins.open

    def __enter__(self):
        def logged(path, *a, **k):
            if isinstance(path, str) and path.endswith(".scen"):
                self.paths.append(path)
            return self._open(path, *a, **k)
        builtins.open = logged
        return self

    def __exit__(self, *exc):
        builtins.open = self._open


def main():
    os.makedirs(OUT, exist_ok=True)
    rec = {}
    files = set()
    for case, kind, map_name, n, seed, resets in CASES:
        map_path = os.path.join(gf.MAP_DIR, map_name)
        prefix = os.path.join(gf.SCEN_DIR, map_name[:-4] + "-random-")
        random.seed(seed)
        starts, goals = [], []
        with _OpenLog() as log, contextlib.redirect_stdout(io.StringIO()):
            if kind == "grid":
                env = gf.MG.MAPF_GRID(map_path, prefix, n_agents=n)
                starts.append(list(env.agent_starts))
                goals.append(list(env.agent_goals))
            else:
                env = gf.MP.MARL_PARTIAL_ENV(map_path, prefix, n_agents=n)
                starts.append(list(env._agent_init_pos))
                goals.append(list(env._agent_goal_pos))
                for _ in range(resets):
                    env.reset()
                    starts.append(list(env._agent_init_pos))
                    goals.append(list(env._agent_goal_pos))
        rec[case + "_starts"] = np.array(starts, np.int32)
        rec[case + "_goals"] = np.array(goals, np.int32)
        rec[case + "_scen"] = np.array([os.path.basename(p) for p in log.paths])
        files.update(log.paths)
        files.add(map_path)
        print(case, [os.path.basename(p) for p in log.paths])
    for p in sorted(files):
        shutil.copy(p, os.path.join(OUT, os.path.basename(p)))
    rec["cases"] = np.array([c[0] for c in CASES])
    rec["meta"] = np.array(["%s|%s|%s|%d|%d|%d" % c for c in CASES])
    np.savez_compressed(os.path.join(OUT, "scen_draws.npz"), **rec)


if __name__ == "__main__":
    main()
