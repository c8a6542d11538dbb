"""The MARL_PARTIAL_ENV restatement (oracle/partial_oracle.py) against the
reference's own outputs (tests/golden/mp_*.npz, made by running
envs/marl_partial.py).  Bit-exact: fp64 rewards by bit pattern, obs/state exactly."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN

FIXTURES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "mp_*.npz")))
KW = ("obs_window", "obs_knn_agents", "episode_limit", "move_reward", "stay_reward",
      "stay_goal_reward", "node_collide_reward", "edge_collide_reward", "env_collide_reward",
      "complete_reward", "complete_fac", "gamma")


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
        return {k: z[k] for k in z.files}


def kwargs(fx):
    return {k: fx["meta_" + k].item() for k in KW}


@pytest.mark.parametrize("name", FIXTURES)
def test_partial_oracle_matches_reference(name):
    from oracle.partial_oracle import PartialEnvState
    fx = load(name)
    if "meta_output" in fx and bool(fx["meta_output"]):
        pytest.skip("output=True: the repair is checked in test_partial_output_mode.py")
    env = PartialEnvState(fx["grid"], fx["init_pos"], fx["goals"], **kwargs(fx))
    n = len(fx["init_pos"])
    for a in range(n):
        ref = fx["goal_dist"][a]
        on = ref >= 0
        assert np.array_equal(env.goal_dist[a][on], ref[on]), a
    assert np.array_equal(env.obs(), fx["obs0"])
    assert np.array_equal(env.avail(), fx["avail0"])
    assert np.array_equal(env.state(), fx["state0"])
    for t in range(fx["actions"].shape[0]):
        r, term = env.step(fx["actions"][t])
        assert np.float64(r).view(np.uint64) == fx["reward"][t].view(np.uint64), (t, r, fx["reward"][t])
        assert bool(term) == bool(fx["terminated"][t]), t
        assert np.array_equal(np.array(env.pos), fx["pos"][t]), t
        assert np.array_equal(np.array(env.at_goal, dtype=np.uint8), fx["at_goal"][t]), t
        assert np.array_equal(np.array(env.done, dtype=np.uint8), fx["done"][t]), t
        assert np.array_equal(np.array(env.steps), fx["steps"][t]), t
        assert np.array_equal(np.array(env.node), fx["node"][t]), t
        assert np.array_equal(np.array(env.edge), fx["edge"][t]), t
        assert np.array_equal(env.obs(), fx["obs"][t]), t
        assert np.array_equal(env.state(), fx["state"][t]), t
        assert np.array_equal(env.avail(), fx["avail"][t]), t
