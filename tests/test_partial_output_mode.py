"""output=True collision repair of MARL_PARTIAL_ENV (marl_partial.py:262-275,
:645-820) on the CPU, against tests/golden/mp_out8_n5.npz (written by running the
reference with output=True, tests/golden/gen_partial_big_fixtures.py).

The repair is host code in the drop-in (mapfx.envs.marl_partial: _check_node,
_check_edge, _solve_node, _solve_edge), exactly as in the reference.  Here the
pre-repair step comes from the CPU restatement (oracle/partial_oracle.py); the
drop-in's repair functions then move the agents, drawing from the global `random`
stream seeded and consumed as the reference's was (construction draw, reset draw),
and every step's positions, rewards and observations must equal the reference's."""
import random

import numpy as np

from conftest import load_fixture

KW = ("obs_window", "obs_knn_agents", "episode_limit", "move_reward", "stay_reward",
      "stay_goal_reward", "node_collide_reward", "edge_collide_reward", "env_collide_reward",
      "complete_reward", "complete_fac", "gamma")


def _draw(lines, n):
    """MARL_PARTIAL_ENV.__setup_agent's draws (:907-927) on the given scen lines."""
    random.randint(1, 25)
    picked = random.sample(lines, n)
    return [(l[1], l[0]) for l in picked], [(l[3], l[2]) for l in picked]


def test_output_mode_repair_matches_reference():
    from mapfx.envs import marl_partial as M
    from oracle.partial_oracle import PartialEnvState
    fx = load_fixture("mp_out8_n5")
    assert bool(fx["meta_output"])
    kw = {k: fx["meta_" + k].item() for k in KW}
    n = fx["init_pos"].shape[0]
    # scen lines as write_scen wrote them: (x=col, y=row) per start / goal, + a spare line
    st, gl = fx["scen_starts"], fx["scen_goals"]
    lines = [(int(s[1]), int(s[0]), int(g[1]), int(g[0])) for s, g in zip(st, gl)]
    lines.append(lines[0])
    random.seed(int(fx["meta_py_seed"]))
    random.randint(0, 9999)            # __init__ (:60)
    _draw(lines, n)                    # __init__ -> __setup_agent (:107)
    random.seed(int(fx["meta_reset_seed"]))
    starts, goals = _draw(lines, n)    # reset -> __setup_agent (:130)
    assert np.array_equal(np.array(starts), fx["init_pos"])
    assert np.array_equal(np.array(goals), fx["goals"])
    env = PartialEnvState(fx["grid"], starts, goals, **kw)
    grid = np.asarray(fx["grid"], dtype=np.int64)
    repaired = 0
    for t in range(fx["actions"].shape[0]):
        acts = [int(a) for a in fx["actions"][t]]
        old = list(env.pos)
        r, term = env.step(acts)
        new = list(env.pos)
        n_node, node_vec = M._check_node(new)
        n_edge, _, pairs = M._check_edge(old, new)
        if n_node or n_edge:
            occ_old = grid.copy()
            for p in old:
                occ_old[p] += 1
            ctx = (grid.shape, occ_old, old, acts)
            while n_node > 0:
                new = M._solve_node(ctx, new, node_vec)
                n_node, node_vec = M._check_node(new)
            if n_edge > 0:
                while n_edge > 0:
                    new = M._solve_edge(ctx, new, pairs)
                    n_edge, _, _ = M._check_edge(old, new)
            env.pos = [tuple(int(v) for v in p) for p in new]
            env.node = [0] * n
            env.edge = [0] * n
            env._refresh()
            repaired += 1
        assert np.float64(r).view(np.uint64) == fx["reward"][t].view(np.uint64), t
        assert np.array_equal(np.array(env.pos), fx["pos"][t]), t
        assert np.array_equal(env.obs().astype(np.float32), fx["obs"][t].astype(np.float32)), t
        assert np.array_equal(env.state(), fx["state"][t]), t
    assert repaired >= 5     # the fixture exercises the repair (node and edge) on several steps
