"""The drop-ins' scenario draws equal the reference's own draws (CPU).

tests/golden/gen_scen_fixtures.py constructed the REFERENCE envs under fixed
`random.seed` values and recorded where their agents start and go, plus the
MovingAI map / scen files those draws opened (tests/golden/scen/).  Here the
same seeds drive mapfx.envs.MAPF_GRID (draw order envs/mapf_gridworld.py:37,
:432, :437; scen (x, y) used as (row, col), quirk 2) and
mapfx.envs.MARL_PARTIAL_ENV (envs/marl_partial.py:60, :907, :915, re-drawn at
every reset; scen (x, y) read as (col, row)).  No GPU: the envs draw in
__init__ / __setup_agent before any device work.
"""
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN, load_fixture

SCEN = os.path.join(GOLDEN, "scen")
D = np.load(os.path.join(SCEN, "scen_draws.npz"), allow_pickle=False)
CASES = [tuple(m.split("|")) for m in D["meta"]]


def _paths(map_name):
    return os.path.join(SCEN, map_name), os.path.join(SCEN, map_name[:-4] + "-random-")


@pytest.mark.parametrize("case,kind,map_name,n,seed,resets",
                         [c for c in CASES if c[1] == "grid"])
def test_mapf_grid_draw_matches_reference(case, kind, map_name, n, seed, resets):
    from mapfx.envs.mapf_gridworld import MAPF_GRID
    mp, prefix = _paths(map_name)
    random.seed(int(seed))
    env = MAPF_GRID(mp, prefix, n_agents=int(n))
    assert np.array_equal(np.array(env.agent_starts, np.int32), D[case + "_starts"][0])
    assert np.array_equal(np.array(env.agent_goals, np.int32), D[case + "_goals"][0])
    # the constructor leaves `random` where the reference's leaves it
    random.seed(int(seed))
    MAPF_GRID(mp, prefix, n_agents=int(n))
    after = random.random()
    random.seed(int(seed))
    random.randint(0, 9999)
    random.randint(1, 25)
    with open(os.path.join(SCEN, str(D[case + "_scen"][0]))) as f:
        random.sample([r.rstrip() for r in f.readlines()][1:], int(n))
    assert after == random.random()


def test_c1_fixture_draw_through_drop_in():
    """BASELINE configs[0]: random.seed(1) -> MAPF_GRID(empty-8-8, n_agents=2) starts
    and goals equal those recorded in the reference-run c1_empty8_n2 golden."""
    from mapfx.envs.mapf_gridworld import MAPF_GRID
    fx = load_fixture("c1_empty8_n2")
    mp, prefix = _paths("empty-8-8.map")
    random.seed(1)
    env = MAPF_GRID(mp, prefix, n_agents=2)
    assert np.array_equal(np.array(env.agent_starts, np.int32), fx["init_pos"])
    assert np.array_equal(np.array(env.agent_goals, np.int32), fx["goals"])
    assert np.array_equal(env._grid, fx["grid"])


@pytest.mark.parametrize("case,kind,map_name,n,seed,resets",
                         [c for c in CASES if c[1] == "partial"])
def test_marl_partial_draws_match_reference(case, kind, map_name, n, seed, resets):
    from mapfx.envs.marl_partial import MARL_PARTIAL_ENV
    mp, prefix = _paths(map_name)
    random.seed(int(seed))
    env = MARL_PARTIAL_ENV(mp, prefix, n_agents=int(n))
    starts, goals = D[case + "_starts"], D[case + "_goals"]
    assert np.array_equal(np.array(env._agent_init_pos, np.int32), starts[0])
    assert np.array_equal(np.array(env._agent_goal_pos, np.int32), goals[0])
    for r in range(1, int(resets) + 1):    # reset() re-draws first (:130) -- the draw alone
        env._MARL_PARTIAL_ENV__setup_agent()
        assert np.array_equal(np.array(env._agent_init_pos, np.int32), starts[r]), r
        assert np.array_equal(np.array(env._agent_goal_pos, np.int32), goals[r]), r


def test_map_parsing_matches_readlines_semantics(tmp_path):
    """lines split like text-mode readlines (\\n, \\r\\n, \\r only), a
    short row raises IndexError like the reference's _original_grid[i][j]."""
    from mapfx.maps import load_map, parse_map_text
    hdr = "type octile\nheight 3\nwidth 3\nmap\n"
    g = parse_map_text(hdr + "..@\r\n.@.\r@..\n")
    assert g.tolist() == [[0, 0, -1], [0, -1, 0], [-1, 0, 0]]
    # \x0c (form feed) and   are cell characters (obstacles), not line breaks
    g = parse_map_text(hdr + ".\x0c.\n. .\n...\n")
    assert g.tolist() == [[0, -1, 0], [0, -1, 0], [0, 0, 0]]
    with pytest.raises(IndexError):
        parse_map_text(hdr + "...\n..\n...\n")
    with pytest.raises(IndexError):                 # trailing blanks are rstrip()ed away
        parse_map_text(hdr + "...\n.. \n...\n")
    assert parse_map_text(hdr + "...\n....\n...\n").shape == (3, 3)   # row 0 sets W
    p = tmp_path / "m.map"
    p.write_bytes((hdr + "...\r\n.@.\r\n...\r\n").encode())
    assert load_map(str(p)).tolist() == [[0, 0, 0], [0, -1, 0], [0, 0, 0]]
