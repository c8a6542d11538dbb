"""PRIMAL sequential-dynamics restatement (oracle/primal_dyn_oracle.py) against the
reference's own outputs (tests/golden/pd_*.npz)."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN

FIXTURES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "pd_*.npz")))


@pytest.mark.parametrize("name", FIXTURES)
def test_primal_dyn_oracle_matches_reference(name):
    from oracle.primal_dyn_oracle import PrimalWorld
    with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
        fx = {k: z[k] for k in z.files}
    diag = bool(fx.get("diagonal", False))
    w = PrimalWorld(fx["grid"], fx["starts"], fx["goals"], int(fx["size"]), diagonal=diag)
    for k in range(len(fx["agent"])):
        maps, vec, r, done, mask, on_goal, blocking, valid = w.step(int(fx["agent"][k]) - 1,
                                                                    int(fx["action"][k]))
        assert np.float64(r).view(np.uint64) == fx["reward"][k].view(np.uint64), k
        assert done == bool(fx["done"][k]), k
        assert mask == int(fx["next_mask"][k]), k
        assert on_goal == bool(fx["on_goal"][k]), k
        assert valid == bool(fx["valid"][k]), k
        assert np.array_equal(np.array(w.pos), fx["pos"][k]), k
        if "past" in fx:   # agents_past (moves and stays update it; DIAGONAL_MOVEMENT reads it)
            assert np.array_equal(np.array(w.past), fx["past"][k]), k
        assert np.array_equal(maps, fx["obs"][k]), k
        assert np.array_equal(vec.view(np.uint64), fx["vec"][k].view(np.uint64)), k
