"""PRIMAL random world generator (mapfx.maps.primal_world)
against the reference's own worlds (tests/golden/pw_*.npz, made by
MAPFEnv._setWorld, MARL-curve-main/src/envs/mapf_primal.py:248-341, under the
same seeds of np.random and random).  Host code: no GPU."""
import glob
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN

FIXTURES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "pw_*.npz")))


@pytest.mark.parametrize("name", FIXTURES)
def test_primal_world_matches_reference(name):
    from mapfx.maps import primal_world
    with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
        fx = {k: z[k] for k in z.files}
    np.random.seed(int(fx["seed"]))
    random.seed(int(fx["seed"]))
    n = int(fx["num_agents"])
    if "world0" in fx:
        world, goals = primal_world(n, world0=fx["world0"].astype(int), blank_world=True)
    else:
        world, goals = primal_world(n, SIZE=tuple(fx["SIZE"]), PROB=tuple(fx["PROB"]))
    assert np.array_equal(world, fx["world"])
    assert np.array_equal(goals, fx["goals"])


def test_primal_world_private_generators_are_deterministic():
    from mapfx.maps import primal_world
    a = primal_world(12, np_random=np.random.RandomState(4), py_random=random.Random(4))
    b = primal_world(12, np_random=np.random.RandomState(4), py_random=random.Random(4))
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    world, goals = a
    for k in range(1, 13):
        assert (world == k).sum() == 1 and (goals == k).sum() == 1
        assert world[tuple(np.argwhere(goals == k)[0])] != -1
