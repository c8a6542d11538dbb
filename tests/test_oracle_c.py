"""Pin the C oracle (oracle/liboracle.so) against the reference golden vectors,
and cross-check it against the Python oracle on random batched instances."""
import numpy as np
import pytest

from conftest import fixture_rewards, load_fixture, primal_fixtures, step_fixtures
from oracle import corc
from oracle import mapf_oracle as O


@pytest.fixture(scope="module", autouse=True)
def _built():
    corc.lib()


def _batch_from_fixture(fx, nthreads=1):
    sr, cr = fixture_rewards(fx)
    h, w = fx["grid"].shape
    bits = np.packbits((fx["grid"] != 0).reshape(-1), bitorder="little")
    b = np.zeros(corc.stride(h, w), np.uint8)
    b[: bits.size] = bits
    return corc.OracleBatch(b[None], fx["init_pos"][None], fx["goals"][None], h, w,
                            limit=int(fx["meta_limit"]), step_reward=sr, collide_reward=cr,
                            nthreads=nthreads)


@pytest.mark.parametrize("name", step_fixtures())
def test_c_oracle_matches_reference(name):
    fx = load_fixture(name)
    ob = _batch_from_fixture(fx)
    h, w = fx["grid"].shape
    o = ob.observe(window=5, win=False)
    assert np.array_equal(o["obs_full"][0].reshape(h, w), fx["occ0"])
    assert np.array_equal(o["avail"][0], (fx["avail0"] << np.arange(5)).sum(-1).astype(np.uint8))
    wsteps = list(fx["window_steps"])
    windows = sorted(int(k[6:]) for k in fx if k.startswith("window") and k != "window_steps")
    for t in range(fx["actions"].shape[0]):
        s = ob.step(fx["actions"][t][None].astype(np.int32))
        assert s["bad"] == 0
        assert s["reward"][0].view(np.uint64) == fx["reward"][t].view(np.uint64), t
        assert np.array_equal(ob.pos[0], fx["pos"][t]), t
        assert np.array_equal(ob.done[0], fx["done"][t]), t
        assert np.array_equal(s["node"][0], fx["node"][t]), t
        assert np.array_equal(s["edge"][0], fx["edge"][t]), t
        assert ob.t[0] == fx["t"][t]
        o = ob.observe(window=5, win=False)
        mask = (fx["avail"][t] << np.arange(5)).sum(-1).astype(np.uint8)
        assert np.array_equal(o["avail"][0], mask), t
        if "occ" in fx:
            assert np.array_equal(o["obs_full"][0].reshape(h, w), fx["occ"][t]), t
        if t in wsteps:
            wi = wsteps.index(t)
            for win in windows:
                ow = ob.observe(window=win, full=False)["obs_window"][0]
                assert np.array_equal(ow, fx["window%d" % win][wi]), (t, win)


@pytest.mark.parametrize("name", primal_fixtures())
def test_c_oracle_primal_matches_reference(name):
    fx = load_fixture(name)
    h, w = fx["grid"].shape
    bits = np.zeros(corc.stride(h, w), np.uint8)
    pb = np.packbits((fx["grid"] != 0).reshape(-1), bitorder="little")
    bits[: pb.size] = pb
    for s in [int(v) for v in np.atleast_1d(fx["meta_sizes"])]:
        for k, pos in enumerate(fx["pos"]):
            ob = corc.OracleBatch(bits[None], pos[None], fx["goals"][None], h, w, nthreads=1)
            o = ob.observe(psize=s, full=False, win=False, primal=True)
            assert np.array_equal(o["obs_primal"][0], fx["maps%d" % s][k]), (s, k)
            assert np.array_equal(o["primal_vec"][0].view(np.uint64),
                                  fx["vec%d" % s][k].view(np.uint64)), (s, k)


def test_c_oracle_batched_matches_python_oracle():
    """Random synthetic batch (stacked starts allowed) vs the Python oracle."""
    rs = np.random.RandomState(5)
    E, N, S, T = 6, 12, 10, 40
    grids = -(rs.random_sample((E, S, S)) < 0.2).astype(np.int8)
    init = rs.randint(0, S, size=(E, N, 2)).astype(np.int32)
    goals = rs.randint(0, S, size=(E, N, 2)).astype(np.int32)
    bits = np.zeros((E, corc.stride(S, S)), np.uint8)
    for e in range(E):
        pb = np.packbits((grids[e] != 0).reshape(-1), bitorder="little")
        bits[e, : pb.size] = pb
    ob = corc.OracleBatch(bits, init, goals, S, S, limit=30, nthreads=3)
    envs = [O.GridEnvState(grids[e], init[e], goals[e], episode_limit=30) for e in range(E)]
    acts = rs.randint(0, 5, size=(T, E, N))
    for t in range(T):
        s = ob.step(acts[t].astype(np.int32))
        o = ob.observe(window=5)
        for e in range(E):
            R, done, node, edge, _ = envs[e].step(acts[t, e])
            assert np.float64(R).view(np.uint64) == s["reward"][e].view(np.uint64)
            assert np.array_equal(np.array(envs[e].pos, np.int32), ob.pos[e])
            assert np.array_equal(np.array(done, np.uint8), ob.done[e])
            assert np.array_equal(np.array(node, np.uint8), s["node"][e])
            assert np.array_equal(np.array(edge, np.uint8), s["edge"][e])
            assert np.array_equal(envs[e].occ.reshape(-1), o["obs_full"][e])
            assert np.array_equal(O.window_obs(envs[e].occ, envs[e].pos, 5), o["obs_window"][e])


def test_c_oracle_rejects_bad_actions():
    fx = load_fixture("edge6_scripted")
    ob = _batch_from_fixture(fx)
    pos0 = ob.pos.copy()
    a = np.array([[0, 1, 2, 3, 4, 5, 0, 1]], np.int32)
    assert ob.step(a)["bad"] == 1
    assert np.array_equal(ob.pos, pos0) and ob.t[0] == 0


@pytest.mark.parametrize("N", [16, 200])
def test_c_oracle_rollout_window_equals_observe(N):
    """orc_rollout's last-step window equals orc_observe on the final state,
    including the int16 layout used when N > 127."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "mapf-marl_amd"))
    from mapfx.maps import synthetic_instances
    S, E, T = 24, 4, 6
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.05, seed=1)
    ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], S, S, limit=2000,
                          nthreads=2)
    r = ob.rollout(T, seed=2)
    o = ob.observe()
    assert r["obs_window"].dtype == (np.int16 if N > 127 else np.int8)
    assert np.array_equal(r["obs_window"], o["obs_window"])
    assert np.array_equal(r["avail"], o["avail"])
