"""Pin the CPU oracle (oracle/mapf_oracle.py) against the reference's own
outputs recorded in tests/golden/*.npz by tests/golden/gen_fixtures.py."""
import numpy as np
import pytest

from conftest import fixture_rewards, load_fixture, primal_fixtures, step_fixtures
from oracle import mapf_oracle as O


@pytest.mark.parametrize("name", step_fixtures())
def test_step_matches_reference(name):
    fx = load_fixture(name)
    sr, cr = fixture_rewards(fx)
    env = O.GridEnvState(fx["grid"], fx["init_pos"], fx["goals"],
                         episode_limit=int(fx["meta_limit"]), step_reward=sr, collide_reward=cr)
    assert np.array_equal(env.occ, fx["occ0"])
    assert np.array_equal(np.array(env.avail(), np.uint8), fx["avail0"])
    wsteps = list(fx["window_steps"])
    windows = sorted(int(k[6:]) for k in fx if k.startswith("window") and k != "window_steps")
    for t in range(fx["actions"].shape[0]):
        R, done, node, edge, _ = env.step(fx["actions"][t])
        # bit-exact fp64 (compare the bit patterns) and the Python type (quirk 4)
        assert np.float64(R).view(np.uint64) == fx["reward"][t].view(np.uint64), t
        assert isinstance(R, int) == bool(fx["reward_is_int"][t]), t
        assert np.array_equal(np.array(env.pos, np.int32), fx["pos"][t]), t
        assert np.array_equal(np.array(done, np.uint8), fx["done"][t]), t
        assert np.array_equal(np.array(node, np.uint8), fx["node"][t]), t
        assert np.array_equal(np.array(edge, np.uint8), fx["edge"][t]), t
        assert np.array_equal(np.array(env.avail(), np.uint8), fx["avail"][t]), t
        assert env.t == fx["t"][t]
        if "occ" in fx:
            assert np.array_equal(env.occ, fx["occ"][t]), t
        if t in wsteps:
            wi = wsteps.index(t)
            for w in windows:
                got = O.window_obs(env.occ, env.pos, w)
                assert np.array_equal(got, fx["window%d" % w][wi]), (t, w)


@pytest.mark.parametrize("name", primal_fixtures())
def test_primal_observe_matches_reference(name):
    fx = load_fixture(name)
    for s in [int(v) for v in np.atleast_1d(fx["meta_sizes"])]:
        for k, pos in enumerate(fx["pos"]):
            pos = [tuple(p) for p in pos]
            goals = [tuple(p) for p in fx["goals"]]
            maps, vec = O.primal_obs(fx["grid"], pos, goals, s)
            assert np.array_equal(maps, fx["maps%d" % s][k]), (s, k)
            assert np.array_equal(vec.view(np.uint64), fx["vec%d" % s][k].view(np.uint64)), (s, k)
