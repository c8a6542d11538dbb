#!/usr/bin/env python3
"""Golden vectors of PRIMAL's sequential dynamics by RUNNING THE REFERENCE
(build container only).

Drives MAPFEnv._step((agent_id, action)) (MARL-curve-main/src/envs/mapf_primal.py:549-637)
-- State.moveAgent (:103-135), the reward table (:579-596), _observe (:343-386),
world.done (:159-166) and _listNextValidActions (:639-667) -- agent after agent,
and records every call's outputs as .npz fixtures (`pd_*.npz`).

The "stay on goal" reward adds get_blocking_reward (:513-546), which needs the
un-vendored od_mstar3 planner: it is replaced by 0 on the instance here, so that
term is "parity unpinned"  and the port defines it as 0.
JOINT = False (the reference's default, :27); DIAGONAL_MOVEMENT (:175) is False
(the default) in the first four fixtures and True in `pd_diag_*` (actions 5..8,
agents_past, State.diagonalCollision :77-99).

Usage:  python tests/golden/gen_primal_dyn_fixtures.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_fixtures as G  # noqa: E402  (installs the reference stubs)

PR = G.PR
OUT_DIR = G.OUT_DIR


def make_env(grid, starts, goals, size, diagonal=False):
    world = grid.astype(np.int64).copy()
    gg = np.zeros(grid.shape, dtype=np.int64)
    for a, ((r, c), (gr, gc)) in enumerate(zip(starts, goals)):
        world[r, c] = a + 1
        gg[gr, gc] = a + 1
    env = PR.MAPFEnv(num_agents=len(starts), observation_size=size, world0=world, goals0=gg,
                     DIAGONAL_MOVEMENT=diagonal)
    env.get_blocking_reward = lambda agent_id: 0  # od_mstar3 absent: term unpinned, defined 0
    return env


def run(name, grid, starts, goals, size, rounds, rng, script=None, diagonal=False):
    env = make_env(grid, starts, goals, size, diagonal)
    n = len(starts)
    calls = []
    if script is None:
        script = [(a + 1, int(rng.integers(0, 9 if diagonal else 5)))
                  for _ in range(rounds) for a in range(n)]
    rec = {k: [] for k in ("agent", "action", "reward", "done", "next_mask", "on_goal", "valid",
                           "blocking", "pos", "obs", "vec", "past")}
    for aid, act in script:
        state, reward, done, nxt, on_goal, blocking, valid = env._step((aid, act))
        mask = 0
        for x in nxt:
            mask |= 1 << int(x)
        rec["agent"].append(aid)
        rec["action"].append(act)
        rec["reward"].append(float(reward))
        rec["done"].append(bool(done))
        rec["next_mask"].append(mask)
        rec["on_goal"].append(bool(on_goal))
        rec["valid"].append(bool(valid))
        rec["blocking"].append(bool(blocking))
        rec["pos"].append(np.array(env.getPositions(), dtype=np.int32))
        rec["past"].append(np.array(env.world.agents_past, dtype=np.int32))
        m, v = state
        rec["obs"].append(np.stack([np.asarray(x) for x in m]).astype(np.uint8))
        rec["vec"].append(np.array(v, dtype=np.float64))
        calls.append((aid, act))
    out = {"grid": grid.astype(np.int8), "starts": np.array(starts, dtype=np.int32),
           "goals": np.array(goals, dtype=np.int32), "size": np.array(size),
           "diagonal": np.array(bool(diagonal))}
    for k, v in rec.items():
        out[k] = np.array(v)
    out["reward"] = out["reward"].astype(np.float64)
    path = os.path.join(OUT_DIR, "pd_%s.npz" % name)
    np.savez_compressed(path, **out)
    print("wrote", path, len(script), "calls, done at",
          int(np.argmax(out["done"])) if out["done"].any() else None)


def free_pick(rng, grid, k):
    free = np.argwhere(grid == 0)
    idx = rng.choice(len(free), size=k, replace=False)
    return [tuple(int(v) for v in free[i]) for i in idx]


def main():
    rng = np.random.default_rng(77)
    # 1. 10x10 random obstacles, 8 agents, 30 rounds of random actions, s = 10
    g = (rng.random((10, 10)) < 0.2).astype(np.int8) * -1
    cells = free_pick(rng, g, 16)
    run("rand10_n8", g, cells[:8], cells[8:], 10, 30, rng)
    # 2. crowded 6x6, 12 agents, s = 5 (robot collisions, blocked moves)
    g = np.zeros((6, 6), dtype=np.int8)
    g[2, 2] = g[3, 4] = -1
    cells = free_pick(rng, g, 24)
    run("crowd6_n12", g, cells[:12], cells[12:], 5, 25, rng)
    # 3. scripted: reach goal, stay on it, leave it (status 2), walls and bounds, finish
    g = np.zeros((5, 5), dtype=np.int8)
    g[1, 1] = -1
    starts, goals = [(0, 0), (4, 4)], [(0, 2), (4, 3)]
    # actions: 1 (0,+1), 2 (+1,0), 3 (0,-1), 4 (-1,0); 0 stay
    script = [(1, 4), (2, 0), (1, 1), (1, 2), (1, 1), (1, 0), (1, 2), (2, 3), (1, 4), (2, 1),
              (2, 3), (1, 0), (2, 0), (1, 3), (1, 1)]
    run("script5", g, starts, goals, 7, 0, rng, script=script)
    # 4. larger world, 20 agents, s = 9, random order of agents
    g = (rng.random((16, 16)) < 0.15).astype(np.int8) * -1
    cells = free_pick(rng, g, 40)
    order = [(int(a) + 1, int(rng.integers(0, 5))) for _ in range(12) for a in rng.permutation(20)]
    run("rand16_n20_perm", g, cells[:20], cells[20:], 9, 0, rng, script=order)
    # --- DIAGONAL_MOVEMENT = True (actions 0..8) ---
    rng = np.random.default_rng(1234)
    # 5. 10x10 random obstacles, 8 agents, s = 10, 30 rounds of random actions 0..8
    g = (rng.random((10, 10)) < 0.2).astype(np.int8) * -1
    cells = free_pick(rng, g, 16)
    run("diag_rand10_n8", g, cells[:8], cells[8:], 10, 30, rng, diagonal=True)
    # 6. crowded 6x6, 14 agents, s = 5: many crossings of past moves
    g = np.zeros((6, 6), dtype=np.int8)
    g[0, 5] = -1
    cells = free_pick(rng, g, 28)
    run("diag_crowd6_n14", g, cells[:14], cells[14:], 5, 30, rng, diagonal=True)
    # 7. scripted diagonal crossings: agent 1 (2,2) -> 5 (1,1) to (3,3); agent 2 at (2,3)
    #    tries 6 (1,-1) to (3,2): same midpoint -> -3, also in agent 2's next-action mask;
    #    a stay resets agents_past; the opposite of a diagonal move leaves the mask
    g = np.zeros((6, 6), dtype=np.int8)
    g[4, 4] = -1
    starts, goals = [(2, 2), (2, 3), (0, 0)], [(5, 5), (5, 0), (0, 5)]
    script = [(1, 5), (2, 6), (2, 0), (1, 0), (2, 6), (3, 5), (3, 8), (1, 7), (2, 5), (3, 6),
              (1, 5), (1, 5), (2, 7), (3, 2), (2, 8), (1, 6), (3, 0), (2, 1)]
    run("diag_script6", g, starts, goals, 4, 0, rng, script=script, diagonal=True)
    # 8. 16x16, 20 agents, s = 7 (odd: the byte path), random order, actions 0..8
    g = (rng.random((16, 16)) < 0.15).astype(np.int8) * -1
    cells = free_pick(rng, g, 40)
    order = [(int(a) + 1, int(rng.integers(0, 9))) for _ in range(10) for a in rng.permutation(20)]
    run("diag_rand16_n20_perm", g, cells[:20], cells[20:], 7, 0, rng, script=order, diagonal=True)


if __name__ == "__main__":
    main()
