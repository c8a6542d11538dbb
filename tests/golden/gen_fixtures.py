#!/usr/bin/env python3
"""Generate golden vectors by RUNNING THE REFERENCE (build container only).

This script imports the reference Python envs read-only from
`/root/reference/MARL-curve-main/src/envs/` through five stub modules
(cv2, gym, smac.env.multiagentenv, od_mstar3.cpp_mstar,
od_mstar3.col_set_addition — none of them is on the path being pinned; see
SURVEY.md §8(c) C-1), drives them on fixed seeds and writes the observed
outputs as small `.npz` fixtures next to this file.  The reference itself never
leaves this container: only the data (inputs + outputs) is committed.

Reference entry points exercised (paths relative to MARL-curve-main/src/):
  * MAPF_GRID.__init__/reset/step/get_obs/get_state/get_avail_actions
    (envs/mapf_gridworld.py:21-224)
  * MARL_PARTIAL_ENV.get_obs_agent window part (envs/marl_partial.py:319-375),
    evaluated on MAPF_GRID's `_full_obs` / positions
  * MAPFEnv._observe (envs/mapf_primal.py:343-386) on collision-free states

Usage:  python tests/golden/gen_fixtures.py   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import contextlib
import io
import os
import random
import sys
import tempfile
import textwrap

import numpy as np

REF_SRC = "/root/reference/MARL-curve-main/src"
MAP_DIR = os.path.join(REF_SRC, "mapf_baseline", "mapf-map")
SCEN_DIR = os.path.join(REF_SRC, "mapf_baseline", "scen-random")
OUT_DIR = os.path.dirname(os.path.abspath(__file__))

STUBS = {
    "cv2.py": "def imshow(*a, **k):\n    pass\n\ndef waitKey(*a, **k):\n    return -1\n",
    "gym/__init__.py": "from . import spaces\n\nclass Env(object):\n    pass\n",
    "gym/spaces.py": textwrap.dedent("""
        class Discrete(object):
            def __init__(self, n):
                self.n = n
        class Tuple(object):
            def __init__(self, spaces):
                self.spaces = spaces
        """),
    "smac/__init__.py": "",
    "smac/env/__init__.py": "",
    # alias the reference's own interface (envs/multiagentenv.py)
    "smac/env/multiagentenv.py": "from multiagentenv import MultiAgentEnv\n",
    "od_mstar3/__init__.py": "",
    "od_mstar3/cpp_mstar.py": "def find_path(*a, **k):\n    raise RuntimeError('od_mstar3 not vendored')\n",
    "od_mstar3/col_set_addition.py": "class NoSolutionError(Exception):\n    pass\n\nclass OutOfTimeError(Exception):\n    pass\n",
}


def install_stubs():
    sys.dont_write_bytecode = True
    d = tempfile.mkdtemp(prefix="mapf_ref_stubs_")
    for rel, text in STUBS.items():
        p = os.path.join(d, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(text)
    sys.path[:0] = [d, os.path.join(REF_SRC, "envs"), REF_SRC]
    import mapf_gridworld  # noqa: E402
    import marl_partial  # noqa: E402
    import mapf_primal  # noqa: E402
    return mapf_gridworld, marl_partial, mapf_primal


MG, MP, PR = install_stubs()


# ----------------------------------------------------------------------------
# helpers
# ----------------------------------------------------------------------------
def write_map(tmpdir, name, grid):
    """grid: (S,S) int8 -1/0 -> MovingAI text; returns (map_path, scen_prefix)."""
    s = grid.shape[0]
    lines = ["type octile", "height %d" % s, "width %d" % s, "map"]
    for r in range(s):
        lines.append("".join("." if grid[r, c] == 0 else "@" for c in range(s)))
    mp = os.path.join(tmpdir, name + ".map")
    with open(mp, "w") as f:
        f.write("\n".join(lines) + "\n")
    # 25 placeholder scen files (positions are injected after construction)
    prefix = os.path.join(tmpdir, name + "-random-")
    for k in range(1, 26):
        with open(prefix + "%d.scen" % k, "w") as f:
            f.write("version 1\n")
            for i in range(300):
                f.write("0\t%s.map\t%d\t%d\t0\t0\t0\t0\t0\n" % (name, s, s))
    return mp, prefix


def read_map_grid(path):
    with open(path) as f:
        rows = [row.rstrip() for row in f.readlines()][4:]
    g = np.array([[0 if ch == "." else -1 for ch in row] for row in rows], dtype=np.int8)
    return g


def make_env(map_path, scen_prefix, n, limit, py_seed, step_reward=-0.01, collide_reward=-10):
    random.seed(py_seed)
    with contextlib.redirect_stdout(io.StringIO()):
        env = MG.MAPF_GRID(map_path, scen_prefix, n_agents=n, episode_limit=limit,
                           step_reward=step_reward, collide_reward=collide_reward)
    return env


def inject(env, init_pos, goals):
    n = len(init_pos)
    for a in range(n):
        env._agent_init_pos[a] = (int(init_pos[a][0]), int(init_pos[a][1]))
        env._agent_goal_pos[a] = (int(goals[a][0]), int(goals[a][1]))
    env.agent_starts = [env._agent_init_pos[i] for i in range(n)]
    env.agent_goals = [env._agent_goal_pos[i] for i in range(n)]


def marl_partial_window(env, window):
    """Run MARL_PARTIAL_ENV.get_obs_agent (envs/marl_partial.py:319-375) on
    MAPF_GRID's occupancy + positions; keep the 2*W*W window part."""
    n = env._n_agents
    mp = object.__new__(MP.MARL_PARTIAL_ENV)
    mp._n_agents = n
    mp._agent_positions = list(env.agent_positions)
    mp._obs_window = window
    mp._window_shape = (window, window)
    mp._full_obs = env._full_obs
    mp._grid_shape = env._grid_shape
    mp._obs_knn_agents = 1
    mp._n_features = 13
    mp.agent_distance_matrix = np.zeros((n, n))
    mp._agent_init_pos = list(env.agent_starts)
    mp._agent_goal_pos = list(env.agent_goals)
    mp._dir_unit_vectors = [[0, 0] for _ in range(n)]
    mp._norm_unit_vectors = [0 for _ in range(n)]
    mp._node_collision_agents = [0] * n
    mp._edge_collision_agents = [0] * n
    mp._agent_step_count = [0] * n
    out = np.zeros((n, 2 * window * window), dtype=np.int64)
    for a in range(n):
        o = mp.get_obs_agent(a)
        out[a] = o[: 2 * window * window].astype(np.int64)
        assert np.array_equal(o[: 2 * window * window], out[a])  # integral values
    return out.reshape(n, 2, window, window)


def primal_observe(grid, pos, goals, size):
    """MAPFEnv._observe (envs/mapf_primal.py:343-386) on a collision-free state."""
    n = len(pos)
    world = grid.astype(np.int64).copy()
    gg = np.zeros(grid.shape, dtype=np.int64)
    for a in range(n):
        world[pos[a][0], pos[a][1]] = a + 1
        gg[goals[a][0], goals[a][1]] = a + 1
    env = PR.MAPFEnv(num_agents=n, observation_size=size, world0=world, goals0=gg)
    maps = np.zeros((n, 4, size, size), dtype=np.uint8)
    vec = np.zeros((n, 3), dtype=np.float64)
    for a in range(n):
        m, v = env._observe(a + 1)
        for k in range(4):
            assert set(np.unique(m[k])).issubset({0.0, 1.0})
            maps[a, k] = m[k].astype(np.uint8)
        vec[a] = np.array(v, dtype=np.float64)
    return maps, vec


def run_scenario(env, actions, window_every=1, windows=(5,), record_occ=True):
    """Reset + T steps of the reference; returns dict of recorded arrays."""
    T, n = actions.shape
    h = env._grid_shape[0]
    with contextlib.redirect_stdout(io.StringIO()):
        obs0 = env.reset()
    occ0 = np.array(env._full_obs, dtype=np.int64)
    assert obs0.shape == (n, occ0.size) and obs0.dtype == np.int64
    assert all(np.array_equal(obs0[a], occ0.reshape(-1)) for a in range(n))
    assert np.array_equal(env.get_state(), occ0.reshape(-1))
    odt = np.int8 if n < 127 else np.int16
    rec = {
        "init_pos": np.array(env.agent_positions, dtype=np.int32),
        "goals": np.array(env.agent_goals, dtype=np.int32),
        "occ0": occ0.astype(odt),
        "avail0": np.array(env.get_avail_actions(), dtype=np.uint8),
        "actions": actions.astype(np.int8),
        "pos": np.zeros((T, n, 2), np.int32),
        "done": np.zeros((T, n), np.uint8),
        "reward": np.zeros(T, np.float64),
        "reward_is_int": np.zeros(T, np.uint8),
        "node": np.zeros((T, n), np.uint8),
        "edge": np.zeros((T, n), np.uint8),
        "avail": np.zeros((T, n, 5), np.uint8),
        "t": np.zeros(T, np.int32),
    }
    if record_occ:
        rec["occ"] = np.zeros((T,) + occ0.shape, odt)
    wsteps = list(range(0, T, window_every))
    rec["window_steps"] = np.array(wsteps, np.int32)
    for w in windows:
        rec["window%d" % w] = np.zeros((len(wsteps), n, 2, w, w), odt)
    wi = 0
    for t in range(T):
        with contextlib.redirect_stdout(io.StringIO()):
            R, dones, info = env.step(actions[t].astype(np.int64))
        assert dones is env._agent_dones  # aliased list (quirk 6)
        rec["pos"][t] = np.array(env.agent_positions, dtype=np.int32)
        rec["done"][t] = np.array(dones, dtype=np.uint8)
        rec["reward"][t] = float(R)
        rec["reward_is_int"][t] = 1 if isinstance(R, int) else 0
        rec["node"][t] = env._node_collision_agents
        rec["edge"][t] = env._edge_collision_agents
        rec["avail"][t] = np.array(env.get_avail_actions(), dtype=np.uint8)
        rec["t"][t] = info["_step_count"]
        occ = np.array(env._full_obs, dtype=np.int64)
        if record_occ:
            rec["occ"][t] = occ
        if t == T - 1:
            o = env.get_obs()
            assert all(np.array_equal(o[a], occ.reshape(-1)) for a in range(n))
            assert np.array_equal(env.get_state(), occ.reshape(-1))
        if wi < len(wsteps) and wsteps[wi] == t:
            for w in windows:
                rec["window%d" % w][wi] = marl_partial_window(env, w)
            wi += 1
    assert max(int(rec["edge"].max()), int(rec["node"].max())) < 256
    return rec


def random_positions(rng, grid, n, distinct=True, allow_obstacle=0.0):
    s = grid.shape[0]
    free = [(r, c) for r in range(s) for c in range(s) if grid[r, c] == 0]
    obst = [(r, c) for r in range(s) for c in range(s) if grid[r, c] != 0]
    out = []
    used = set()
    while len(out) < n:
        if obst and rng.random_sample() < allow_obstacle:
            p = obst[rng.randint(len(obst))]
        else:
            p = free[rng.randint(len(free))]
        if distinct and p in used:
            continue
        used.add(p)
        out.append(p)
    return out


def save(name, meta, rec):
    path = os.path.join(OUT_DIR, name + ".npz")
    arrays = dict(rec)
    for k, v in meta.items():
        arrays["meta_" + k] = np.array(v)
    np.savez_compressed(path, **arrays)
    print("wrote %-28s %7.1f KB" % (name + ".npz", os.path.getsize(path) / 1024.0))


# ----------------------------------------------------------------------------
# scenarios
# ----------------------------------------------------------------------------
def scen_real(name, map_file, n, limit, T, py_seed, act_seed, window_every=1,
              windows=(5,), record_occ=True, step_reward=-0.01, collide_reward=-10):
    """Real MovingAI map + the reference's own scenario draw (quirk 2)."""
    mp = os.path.join(MAP_DIR, map_file)
    prefix = os.path.join(SCEN_DIR, map_file[:-4] + "-random-")
    env = make_env(mp, prefix, n, limit, py_seed, step_reward, collide_reward)
    grid = read_map_grid(mp)
    actions = np.random.RandomState(act_seed).randint(0, 5, size=(T, n))
    rec = run_scenario(env, actions, window_every, windows, record_occ)
    rec["grid"] = grid
    save(name, dict(limit=limit, step_reward=step_reward, collide_reward=collide_reward,
                    collide_is_int=isinstance(collide_reward, int),
                    step_is_int=isinstance(step_reward, int), source=map_file), rec)
    return rec


def scen_synthetic(name, tmp, grid, init_pos, goals, actions, limit,
                   step_reward=-0.01, collide_reward=-10, window_every=1, windows=(5,)):
    mp, prefix = write_map(tmp, name, grid)
    n = len(init_pos)
    env = make_env(mp, prefix, n, limit, 0, step_reward, collide_reward)
    inject(env, init_pos, goals)
    rec = run_scenario(env, np.asarray(actions), window_every, windows)
    rec["grid"] = grid
    save(name, dict(limit=limit, step_reward=step_reward, collide_reward=collide_reward,
                    collide_is_int=isinstance(collide_reward, int),
                    step_is_int=isinstance(step_reward, int), source="synthetic"), rec)
    return rec


def primal_fixture(name, grid, states, goals, sizes=(10,)):
    """states: list of position lists (distinct); goals distinct."""
    rec = {"grid": grid, "goals": np.array(goals, np.int32),
           "pos": np.array(states, np.int32)}
    for s in sizes:
        mm, vv = [], []
        for pos in states:
            m, v = primal_observe(grid, pos, goals, s)
            mm.append(m)
            vv.append(v)
        rec["maps%d" % s] = np.stack(mm)
        rec["vec%d" % s] = np.stack(vv)
    save(name, {"sizes": list(sizes)}, rec)


def main():
    tmp = tempfile.mkdtemp(prefix="mapf_fixture_maps_")
    rng = np.random.RandomState(12345)

    # --- C1: empty-8-8, 2 agents, reference scen draw, T=2000 (BASELINE configs[0])
    scen_real("c1_empty8_n2", "empty-8-8.map", 2, 2000, 2000, py_seed=1, act_seed=11)
    # yaml default agent count (config/envs/mapf_gridworld.yaml:7)
    scen_real("empty8_n5", "empty-8-8.map", 5, 2000, 600, py_seed=2, act_seed=12, windows=(3, 5))
    # real 32x32 maps with the transposed scen coordinates (quirk 2)
    scen_real("random32_10_n16", "random-32-32-10.map", 16, 2000, 400, py_seed=3, act_seed=13,
              window_every=4)
    scen_real("maze32_4_n16", "maze-32-32-4.map", 16, 2000, 300, py_seed=4, act_seed=14,
              window_every=4, windows=(5, 7))
    # larger maps (C3/C5 sizes); occupancy and windows sub-sampled
    scen_real("random64_10_n64", "random-64-64-10.map", 64, 2000, 60, py_seed=5, act_seed=15,
              window_every=10)
    scen_real("maze128_10_n256", "maze-128-128-10.map", 256, 2000, 12, py_seed=6, act_seed=16,
              window_every=6, record_occ=False)
    # integer rewards: sum() stays a Python int (quirk 4)
    scen_real("empty8_int_rewards", "empty-8-8.map", 4, 2000, 200, py_seed=7, act_seed=17,
              step_reward=-1, collide_reward=-3)

    # --- synthetic 32x32 maps, 10% / 20% obstacles, some agents on obstacles (quirk 1)
    for pct, tag in ((0.10, "p10"), (0.20, "p20")):
        g = -(rng.random_sample((32, 32)) < pct).astype(np.int8)
        init = random_positions(rng, g, 16, allow_obstacle=0.1)
        goals = random_positions(rng, g, 16, allow_obstacle=0.05)
        acts = rng.randint(0, 5, size=(500, 16))
        scen_synthetic("syn32_%s_n16" % tag, tmp, g, init, goals, acts, 2000, window_every=5)

    # --- dense 8x8: stacked starts, swaps with multiplicity, many collisions
    g = -(rng.random_sample((8, 8)) < 0.15).astype(np.int8)
    init = random_positions(rng, g, 30, distinct=False, allow_obstacle=0.2)
    goals = random_positions(rng, g, 30, distinct=False, allow_obstacle=0.1)
    acts = rng.randint(0, 5, size=(300, 30))
    scen_synthetic("dense8_n30", tmp, g, init, goals, acts, 2000, windows=(3, 5))

    # --- scripted edge cases on a 6x6 map
    g = np.zeros((6, 6), np.int8)
    g[2, 3] = -1
    g[4, 1] = -1
    # a0,a1 stacked at (1,1); a2 at (1,2). a0,a1 move right (3), a2 moves left (2):
    # swap with multiplicity -> a2 edge=2 (quirk 3); a3 sits on obstacle (2,3);
    # a4 moves onto the occupied obstacle (2,3) (passable, quirk 1); a5 reaches its
    # goal while colliding; a6 is done and gets run into.
    init = [(1, 1), (1, 1), (1, 2), (2, 3), (3, 3), (5, 5), (0, 5), (0, 4)]
    goals = [(5, 0), (5, 1), (0, 0), (5, 3), (2, 3), (5, 4), (0, 5), (3, 0)]
    acts = [
        [3, 3, 2, 4, 0, 2, 4, 3],   # swap x2, onto occupied obstacle, a5 -> goal, a7 -> done a6
        [4, 4, 4, 1, 4, 4, 4, 4],   # a3 leaves obstacle (2,3)->(3,3)
        [2, 3, 3, 0, 0, 4, 0, 2],   # out of bounds (a6 done), obstacle (a4 on goal/done)
        [0, 1, 2, 3, 4, 0, 1, 2],
    ] + rng.randint(0, 5, size=(40, 8)).tolist()
    scen_synthetic("edge6_scripted", tmp, g, init, goals, acts, 2000, windows=(3, 5, 7))
    # episode limit hit mid-run: every agent done at t == limit, collisions after
    scen_synthetic("edge6_limit", tmp, g, init, goals, acts, 5, windows=(5,))
    # float collide reward (-10.0 * 0 == -0.0 products)
    scen_synthetic("edge6_float_collide", tmp, g, init, goals, acts, 2000,
                   step_reward=-0.25, collide_reward=-10.0, windows=(5,))

    # --- PRIMAL _observe on collision-free states (distinct positions and goals)
    g = -(rng.random_sample((32, 32)) < 0.15).astype(np.int8)
    goals = random_positions(rng, g, 16)
    states = [random_positions(rng, g, 16, allow_obstacle=0.1) for _ in range(6)]
    primal_fixture("primal32_n16", g, states, goals, sizes=(10, 5, 7))
    # 64x64: far goals so mag = (dx^2+dy^2)**.5 hits n >= 2921 (pow != sqrt, quirk 8)
    g = -(rng.random_sample((64, 64)) < 0.1).astype(np.int8)
    goals = random_positions(rng, g, 32)
    goals[0] = (54, 25)  # from (0,0): n = 54^2 + 25^2 = 3541, pow(n,.5) != sqrt(n)
    corner = [(0, 0), (63, 63), (0, 63), (63, 0)]
    states = []
    for k in range(4):
        st = random_positions(rng, g, 32)
        st = [p for p in st if p != corner[k]][:31]
        states.append([corner[k]] + st)
    assert len(set(goals)) == len(goals)
    assert all(len(set(s)) == len(s) for s in states)
    primal_fixture("primal64_n32", g, states, goals, sizes=(10,))


if __name__ == "__main__":
    main()
