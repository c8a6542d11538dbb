#!/usr/bin/env python3
"""Golden vectors of PRIMAL's random world generator by RUNNING THE REFERENCE
(build container only).

MAPFEnv(num_agents, SIZE, PROB) without world0 runs _setWorld
(MARL-curve-main/src/envs/mapf_primal.py:248-341): triangular obstacle density,
a side drawn from three sizes, agents on random free cells, goals drawn from each
agent's connected region.  With blank_world=True it places agents and goals on a
given world (:290-306).  Each case seeds the global np.random and random the
same way before constructing the env and stores the resulting initial world and
goals (`pw_*.npz`).

Usage:  python tests/golden/gen_primal_world_fixtures.py
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_fixtures as G  # noqa: E402  (installs the reference stubs)

PR = G.PR
OUT_DIR = G.OUT_DIR

CASES = [
    # name, seed, num_agents, SIZE, PROB, blank world (None = random)
    ("rand_a4_s0", 0, 4, (10, 40), (0, .5), None),
    ("rand_a8_s1", 1, 8, (10, 40), (0, .5), None),
    ("rand_a16_s7", 7, 16, (10, 20), (.1, .3), None),
    ("rand_a32_s11", 11, 32, (20, 40), (0, .2), None),
    ("blank12_a6_s5", 5, 6, None, None, (12, ((3, 3), (3, 4), (8, 1), (5, 9)))),
]


def main():
    for name, seed, n, size, prob, blank in CASES:
        np.random.seed(seed)
        random.seed(seed)
        if blank is None:
            env = PR.MAPFEnv(num_agents=n, SIZE=size, PROB=prob)
            extra = {"SIZE": np.array(size, dtype=np.float64), "PROB": np.array(prob, dtype=np.float64)}
        else:
            side, walls = blank
            w0 = np.zeros((side, side), dtype=int)
            for r, c in walls:
                w0[r, c] = -1
            env = PR.MAPFEnv(num_agents=n, world0=w0.copy(), blank_world=True)
            extra = {"world0": w0.astype(np.int8)}
        out = {"seed": np.array(seed), "num_agents": np.array(n),
               "world": np.asarray(env.initial_world).astype(np.int32),
               "goals": np.asarray(env.initial_goals).astype(np.int32)}
        out.update(extra)
        path = os.path.join(OUT_DIR, "pw_%s.npz" % name)
        np.savez_compressed(path, **out)
        print("wrote", path, out["world"].shape)


if __name__ == "__main__":
    main()
