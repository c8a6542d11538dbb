#!/usr/bin/env python3
"""Golden vectors of MARL_PARTIAL_ENV by RUNNING THE REFERENCE (build container only).

SURVEY.md §8(f) F1: the env actually registered by the reference
(MARL-curve-main/src/envs/__init__.py:60).  Drives
envs/marl_partial.py:25-310 (ctor, reset, step) and :312-375 (get_obs,
KNN features), :377-391 (get_state), :393-428 (avail) on fixed seeds and writes
the observed inputs/outputs as .npz fixtures (`mp_*.npz`) next to this file.
The reference is imported read-only through the stubs of gen_fixtures.py.

Recorded per step t (after step t): reward (fp64), terminated, positions,
at-goal flags, dones, per-agent step counts, node/edge collision vectors,
obs [N, 2W^2 + 13K] (fp64), state [3], avail [N, 5].  Plus the reset
observation and the instance (map, starts, goals) the reference drew.

Usage:  python tests/golden/gen_partial_fixtures.py
"""
from __future__ import annotations

import contextlib
import io
import os
import random
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_fixtures as G  # noqa: E402  (installs the reference stubs)

MP = G.MP
OUT_DIR = G.OUT_DIR

YAML_ARGS = dict(  # config/envs/marl_partial.yaml:3-23
    obs_window=5, obs_knn_agents=5, episode_limit=100, move_reward=0, stay_reward=-0.1,
    stay_goal_reward=1, node_collide_reward=-2000, edge_collide_reward=-2000,
    env_collide_reward=-2000, complete_reward=1000, complete_fac=1.5, gamma=0.99)


def write_scen(tmpdir, name, s, starts, goals):
    """25 identical scen files holding exactly the given (row, col) starts/goals
    (+1 spare line: the reference asserts len(lines) > n_agents, :897)."""
    prefix = os.path.join(tmpdir, name + "-random-")
    lines = ["version 1"]
    for (sr, sc), (gr, gc) in list(zip(starts, goals)) + [(starts[0], goals[0])]:
        # MovingAI: bucket map w h start_x start_y goal_x goal_y dist (x = col, y = row)
        lines.append("0\t%s.map\t%d\t%d\t%d\t%d\t%d\t%d\t0" % (name, s, s, sc, sr, gc, gr))
    for k in range(1, 26):
        with open(prefix + "%d.scen" % k, "w") as f:
            f.write("\n".join(lines) + "\n")
    return prefix


def make(map_path, scen_prefix, n, py_seed, **kw):
    random.seed(py_seed)
    args = dict(YAML_ARGS)
    args.update(kw)
    with contextlib.redirect_stdout(io.StringIO()):
        env = MP.MARL_PARTIAL_ENV(map_path, scen_prefix, n_agents=n, **args)
    return env, args


def snapshot(env):
    n = env._n_agents
    return dict(
        pos=np.array(env._agent_positions, dtype=np.int32).reshape(n, 2),
        at_goal=np.array(env._agent_at_goals, dtype=np.uint8),
        done=np.array(env._agent_dones, dtype=np.uint8),
        steps=np.array(env._agent_step_count, dtype=np.int32),
        node=np.array(env._node_collision_agents, dtype=np.int32),
        edge=np.array(env._edge_collision_agents, dtype=np.int32),
        obs=np.array(env.get_obs(), dtype=np.float64),
        state=np.array(env.get_state(), dtype=np.float64),
        avail=np.array(env.get_avail_actions(), dtype=np.uint8),
    )


def run(name, env, args, actions, reset_seed, grid):
    random.seed(reset_seed)
    with contextlib.redirect_stdout(io.StringIO()):
        obs0 = np.array(env.reset(), dtype=np.float64)
    n = env._n_agents
    rec = {"grid": grid, "init_pos": np.array(env._agent_init_pos, dtype=np.int32),
           "goals": np.array(env._agent_goal_pos, dtype=np.int32), "obs0": obs0,
           "avail0": np.array(env.get_avail_actions(), dtype=np.uint8),
           "state0": np.array(env.get_state(), dtype=np.float64), "actions": actions}
    # goal distance tables the reference computed (A* lengths), [N, H*W], -1 off-graph
    h, w = grid.shape
    gd = np.full((n, h * w), -1, dtype=np.int32)
    for a in range(n):
        for k, v in env._goal_dist[a].items():
            gd[a, k] = v
    rec["goal_dist"] = gd
    steps = []
    rew, term = [], []
    for t in range(actions.shape[0]):
        with contextlib.redirect_stdout(io.StringIO()):
            r, done, info = env.step(list(int(x) for x in actions[t]))
        rew.append(float(r))
        term.append(bool(done))
        steps.append(snapshot(env))
    for k in steps[0]:
        rec[k] = np.stack([s[k] for s in steps])
    rec["reward"] = np.array(rew, dtype=np.float64)
    rec["terminated"] = np.array(term, dtype=np.uint8)
    for k, v in args.items():
        rec["meta_" + k] = np.array(v)
    path = os.path.join(OUT_DIR, "mp_%s.npz" % name)
    np.savez_compressed(path, **rec)
    print("wrote", path, "T=%d N=%d" % (actions.shape[0], n), "terminated at",
          int(np.argmax(rec["terminated"])) if rec["terminated"].any() else None)


def connected_random_grid(rng, s, p):
    """Random obstacles, then everything outside the largest 4-connected free
    component becomes an obstacle (the reference's A* tables need one component)."""
    g = (rng.random((s, s)) < p).astype(np.int8) * -1
    seen = np.zeros_like(g, dtype=bool)
    best = []
    for r in range(s):
        for c in range(s):
            if g[r, c] == 0 and not seen[r, c]:
                comp, stack = [], [(r, c)]
                seen[r, c] = True
                while stack:
                    y, x = stack.pop()
                    comp.append((y, x))
                    for dy, dx in ((1, 0), (-1, 0), (0, 1), (0, -1)):
                        yy, xx = y + dy, x + dx
                        if 0 <= yy < s and 0 <= xx < s and g[yy, xx] == 0 and not seen[yy, xx]:
                            seen[yy, xx] = True
                            stack.append((yy, xx))
                if len(comp) > len(best):
                    best = comp
    out = np.full_like(g, -1)
    for y, x in best:
        out[y, x] = 0
    return out


def free_cells(grid):
    return [tuple(x) for x in np.argwhere(grid == 0)]


def main():
    tmp = tempfile.mkdtemp(prefix="mp_fixtures_")
    rng = np.random.default_rng(2024)

    # 1. the yaml config on the reference's own empty-8-8 map + scen files
    mp8 = os.path.join(G.MAP_DIR, "empty-8-8.map")
    sc8 = os.path.join(G.SCEN_DIR, "empty-8-8-random-")
    env, args = make(mp8, sc8, 15, py_seed=5)
    acts = rng.integers(0, 5, size=(120, 15)).astype(np.int64)
    run("yaml_empty8_n15", env, args, acts, reset_seed=7, grid=G.read_map_grid(mp8))

    # 2. random 16x16 (one component), 8 agents, float rewards, limit 60
    g16 = connected_random_grid(rng, 16, 0.2)
    mp16, _ = G.write_map(tmp, "rand16", g16)
    cells = free_cells(g16)
    pick = rng.choice(len(cells), size=16, replace=False)
    starts, goals = [cells[i] for i in pick[:8]], [cells[i] for i in pick[8:]]
    sc16 = write_scen(tmp, "rand16", 16, starts, goals)
    env, args = make(mp16, sc16, 8, py_seed=3, episode_limit=60, move_reward=-0.01,
                     stay_reward=-0.02, stay_goal_reward=0, node_collide_reward=-1,
                     edge_collide_reward=-1, env_collide_reward=-1)
    acts = rng.integers(0, 5, size=(70, 8)).astype(np.int64)
    run("rand16_n8", env, args, acts, reset_seed=11, grid=g16)

    # 3. scripted completion: 2 agents one move from their goals on a 4x4 map, stay
    #    at goal, then swap-collide; completion reward gamma**(limit - t)
    g4 = np.zeros((4, 4), dtype=np.int8)
    g4[1, 2] = -1
    mp4, _ = G.write_map(tmp, "tiny4", g4)
    sc4 = write_scen(tmp, "tiny4", 4, [(0, 0), (3, 3)], [(0, 1), (3, 2)])
    env, args = make(mp4, sc4, 2, py_seed=1, episode_limit=12)
    # the reference samples which scen line is agent 0: script from what it drew
    random.seed(13)
    with contextlib.redirect_stdout(io.StringIO()):
        env.reset()
    ip = list(env._agent_init_pos)
    gl = list(env._agent_goal_pos)
    def toward(a):
        (r, c), (gr, gc) = ip[a], gl[a]
        return 1 if gr > r else 0 if gr < r else 3 if gc > c else 2
    acts = np.array([[4, 4], [toward(0), 4], [4, toward(1)], [4, 4], [0, 1], [2, 3], [1, 0],
                     [3, 2], [4, 4]], dtype=np.int64)
    run("tiny4_complete", env, args, acts, reset_seed=13, grid=g4)

    # 4. collision-heavy: 6 agents crowded on a 5x5 map with a wall, K=3 < N
    g5 = np.zeros((5, 5), dtype=np.int8)
    g5[2, 1:4] = -1
    mp5, _ = G.write_map(tmp, "wall5", g5)
    cells = free_cells(g5)
    pick = rng.choice(len(cells), size=12, replace=False)
    sc5 = write_scen(tmp, "wall5", 5, [cells[i] for i in pick[:6]], [cells[i] for i in pick[6:]])
    env, args = make(mp5, sc5, 6, py_seed=2, obs_knn_agents=3, obs_window=3, episode_limit=25,
                     move_reward=-0.01, stay_reward=-0.02, stay_goal_reward=0.5,
                     node_collide_reward=-3, edge_collide_reward=-5, env_collide_reward=-7)
    acts = rng.integers(0, 5, size=(30, 6)).astype(np.int64)
    run("wall5_n6_k3", env, args, acts, reset_seed=17, grid=g5)

    # 5. window 7, K larger than N (rows of -1), 12x12 maze-ish map
    g12 = connected_random_grid(rng, 12, 0.3)
    mp12, _ = G.write_map(tmp, "rand12", g12)
    cells = free_cells(g12)
    pick = rng.choice(len(cells), size=8, replace=False)
    sc12 = write_scen(tmp, "rand12", 12, [cells[i] for i in pick[:4]], [cells[i] for i in pick[4:]])
    env, args = make(mp12, sc12, 4, py_seed=4, obs_window=7, obs_knn_agents=6, episode_limit=40)
    acts = rng.integers(0, 5, size=(45, 4)).astype(np.int64)
    run("rand12_w7_k6", env, args, acts, reset_seed=19, grid=g12)


if __name__ == "__main__":
    main()
