"""GPU parity of batched PRIMAL sequential dynamics through the
C ABI (include/mapfx_primal.h): against the reference's own outputs
(tests/golden/pd_*.npz) and against the CPU restatement (oracle/primal_dyn_oracle.py)
on batched random worlds.  Everything bit-exact: rewards and goal vectors as fp64
bit patterns, observation maps, masks, flags and positions exactly."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

FIXTURES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "pd_*.npz")))


@pytest.fixture(scope="module")
def mapfx_mod():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mapfx
    return mapfx


def _load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
        return {k: z[k] for k in z.files}


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("chunk", [0, 1, 7])
def test_primal_matches_reference_goldens(mapfx_mod, name, chunk):
    """All calls in one launch (chunk 0) or split over launches of `chunk` calls:
    the world state carries over between launches."""
    fx = _load(name)
    diag = bool(fx.get("diagonal", False))
    b = mapfx_mod.PrimalBatch(fx["starts"][None], fx["goals"][None], grids=fx["grid"][None],
                              observation_size=int(fx["size"]), diagonal=diag)
    n = len(fx["agent"])
    step = n if chunk == 0 else chunk
    for k0 in range(0, n, step):
        k1 = min(n, k0 + step)
        o = b.act(fx["agent"][None, k0:k1], fx["action"][None, k0:k1])
        sl = slice(k0, k1)
        assert np.array_equal(_np(o["reward"])[0].view(np.uint64), fx["reward"][sl].view(np.uint64))
        assert np.array_equal(_np(o["done"])[0].astype(bool), fx["done"][sl])
        assert np.array_equal(_np(o["next_mask"])[0], fx["next_mask"][sl])
        assert np.array_equal(_np(o["on_goal"])[0].astype(bool), fx["on_goal"][sl])
        assert np.array_equal(_np(o["valid"])[0].astype(bool), fx["valid"][sl])
        assert np.array_equal(_np(o["obs"])[0], fx["obs"][sl])
        assert np.array_equal(_np(o["vec"])[0].view(np.uint64), fx["vec"][sl].view(np.uint64))
        assert np.array_equal(_np(b.pos)[0], fx["pos"][k1 - 1])
        if diag:
            assert np.array_equal(_np(b.past)[0], fx["past"][k1 - 1])
    b.check_err()


@pytest.mark.parametrize("name", ["pd_script5", "pd_diag_script6"])
def test_primal_dropin_matches_reference_goldens(mapfx_mod, name):
    from mapfx.primal import MAPFEnv
    fx = _load(name)
    world = fx["grid"].astype(np.int64)
    gg = np.zeros_like(world)
    for a, ((r, c), (gr, gc)) in enumerate(zip(fx["starts"], fx["goals"])):
        world[r, c] = a + 1
        gg[gr, gc] = a + 1
    env = MAPFEnv(num_agents=len(fx["starts"]), observation_size=int(fx["size"]), world0=world,
                  goals0=gg, DIAGONAL_MOVEMENT=bool(fx["diagonal"]))
    for k in range(len(fx["agent"])):
        (maps, vec), r, done, nxt, on_goal, blocking, valid = env._step(
            (int(fx["agent"][k]), int(fx["action"][k])))
        assert np.float64(r).view(np.uint64) == fx["reward"][k].view(np.uint64)
        assert done == bool(fx["done"][k]) and on_goal == bool(fx["on_goal"][k])
        assert valid == bool(fx["valid"][k]) and blocking is False
        assert sum(1 << a for a in nxt) == int(fx["next_mask"][k])
        assert np.array_equal(np.stack(maps), fx["obs"][k])
        assert np.array_equal(np.array(vec).view(np.uint64), fx["vec"][k].view(np.uint64))
        assert env.getPositions() == [tuple(p) for p in fx["pos"][k].tolist()]
    assert env.finished == bool(fx["done"].any())


def _random_worlds(rng, E, H, W, N, density, shared):
    n_maps = 1 if shared else E
    grids = np.where(rng.random((n_maps, H, W)) < density, -1, 0).astype(np.int8)
    starts = np.zeros((E, N, 2), np.int32)
    goals = np.zeros((E, N, 2), np.int32)
    for e in range(E):
        free = np.argwhere(grids[0 if shared else e] == 0)
        idx = rng.choice(len(free), size=2 * N, replace=False)
        starts[e] = free[idx[:N]]
        goals[e] = free[idx[N:]]
    return grids, starts, goals


@pytest.mark.parametrize("diag", [False, True])
@pytest.mark.parametrize("lanes", ["", "16", "32"])  # host's choice (64 at E = 64) / packed lane groups
@pytest.mark.parametrize("H,W,N,s,K,shared,density", [
    (12, 12, 10, 7, 60, False, 0.2),
    (9, 13, 30, 4, 90, True, 0.1),      # crowded, even window, non-square
    (40, 33, 100, 11, 150, False, 0.15),  # N > 64 (agent loops), s*s > 64
    (128, 128, 255, 32, 40, True, 0.1),   # the ABI limits: N 255, H*W 16384, s 32 (s*s > 4 * 64: the rest loop)
    (20, 20, 12, 9, 70, False, 0.1),      # 16-lane groups: s*s = 81 > 4 * 16 (the rest loop)
    (32, 32, 16, 10, 70, False, 0.1),     # observation_size 10 (the default): specialised kernels
    (15, 17, 40, 10, 66, True, 0.1),      # s = 10 at 64 lanes (N > 32)
])
def test_primal_batch_matches_oracle(mapfx_mod, monkeypatch, lanes, H, W, N, s, K, shared, density,
                                    diag):
    from oracle.primal_dyn_oracle import PrimalWorld
    monkeypatch.setenv("MAPFX_PRIMAL_LANES", lanes)
    rng = np.random.default_rng(H * 1000 + N + (7 if diag else 0))
    E = 64
    grids, starts, goals = _random_worlds(rng, E, H, W, N, density, shared)
    ids = rng.integers(1, N + 1, size=(E, K)).astype(np.int32)
    # bias toward moves; some stays
    if diag:
        acts = rng.choice(9, size=(E, K), p=[0.04] + [0.12] * 8).astype(np.int32)
    else:
        acts = rng.choice(5, size=(E, K), p=[0.1, 0.225, 0.225, 0.225, 0.225]).astype(np.int32)
    b = mapfx_mod.PrimalBatch(starts, goals, grids=grids, observation_size=s, diagonal=diag)
    o = {k: _np(v).copy() for k, v in b.act(ids, acts).items()}
    pos = _np(b.pos)
    b.check_err()
    for e in range(E):     # every world of the batch (the restatement takes < 1 s per world)
        w = PrimalWorld(grids[0 if shared else e], starts[e], goals[e], s, diagonal=diag)
        for k in range(K):
            maps, vec, r, done, mask, on_goal, _, valid = w.step(int(ids[e, k]) - 1, int(acts[e, k]))
            assert np.float64(r).view(np.uint64) == o["reward"][e, k].view(np.uint64), (e, k)
            assert done == bool(o["done"][e, k]) and mask == int(o["next_mask"][e, k]), (e, k)
            assert on_goal == bool(o["on_goal"][e, k]) and valid == bool(o["valid"][e, k]), (e, k)
            assert np.array_equal(maps, o["obs"][e, k]), (e, k)
            assert np.array_equal(vec.view(np.uint64), o["vec"][e, k].view(np.uint64)), (e, k)
        assert np.array_equal(np.array(w.pos), pos[e]), e
        if diag:
            assert np.array_equal(np.array(w.past), _np(b.past)[e]), e


@pytest.mark.parametrize("N,lanes,s,diag", [
    (3, "16", 5, False), (20, "16", 5, False), (40, "16", 5, False),  # lane groups (forced)
    # the host's own choice: even s -> primal_seq_kernel (one world per wave, its
    # badm / kstop path), s = 4 and 10, and a refused diagonal action 9
    (3, "", 10, False), (20, "", 4, False), (40, "", 10, False), (20, "", 10, True),
    (20, "16", 5, True)])
def test_primal_bad_call_stops_only_its_world(mapfx_mod, monkeypatch, N, lanes, s, diag):
    """E not a multiple of the worlds per wave, K past one 64-call block, and a bad
    call in world 2 (an agent id past N, or DIAGONAL_MOVEMENT's action 9) in the second
    block that ends that world's calls (the reference asserts, :552-557) while the
    other worlds -- wave neighbours on the lane-group kernel -- run on."""
    from oracle.primal_dyn_oracle import PrimalWorld
    rng = np.random.default_rng(N + 100 * s + (7 if diag else 0))
    E, H, W, K, kbad = 7, 14, 11, 80, 70
    grids, starts, goals = _random_worlds(rng, E, H, W, N, 0.1, False)
    ids = rng.integers(1, N + 1, size=(E, K)).astype(np.int32)
    acts = rng.integers(0, 9 if diag else 5, size=(E, K)).astype(np.int32)
    if diag:
        acts[2, kbad] = 9
    else:
        ids[2, kbad] = N + 1
    monkeypatch.setenv("MAPFX_PRIMAL_LANES", lanes)
    b = mapfx_mod.PrimalBatch(starts, goals, grids=grids, observation_size=s, diagonal=diag)
    o = {k: _np(v).copy() for k, v in b.act(ids, acts).items()}
    with pytest.raises(AssertionError, match="world 2"):
        b.check_err()
    pos = _np(b.pos)
    for e in range(E):
        w = PrimalWorld(grids[e], starts[e], goals[e], s, diagonal=diag)
        for k in range(kbad if e == 2 else K):
            maps, vec, r, done, mask, on_goal, _, valid = w.step(int(ids[e, k]) - 1, int(acts[e, k]))
            assert np.float64(r).view(np.uint64) == o["reward"][e, k].view(np.uint64), (e, k)
            assert done == bool(o["done"][e, k]) and mask == int(o["next_mask"][e, k]), (e, k)
            assert on_goal == bool(o["on_goal"][e, k]) and valid == bool(o["valid"][e, k]), (e, k)
            assert np.array_equal(maps, o["obs"][e, k]), (e, k)
            assert np.array_equal(vec.view(np.uint64), o["vec"][e, k].view(np.uint64)), (e, k)
        assert np.array_equal(np.array(w.pos), pos[e]), e


def test_primal_bench_shape_matches_oracle(mapfx_mod):
    """bench.py --env primal's shape through the host's kernel choice
    (primal_seq_kernel): 4096 worlds of 32 x 32 (10 % obstacles), 16 agents, s = 10,
    64 calls per world in one launch, agents round robin with random actions --
    every 64th world and the last against the restatement, call by call."""
    from mapfx.maps import synthetic_instances
    from oracle.primal_dyn_oracle import PrimalWorld
    E, S, N, s, K = 4096, 32, 16, 10, 64
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.10, seed=1)
    b = mapfx_mod.PrimalBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                              observation_size=s)
    rng = np.random.default_rng(7)
    ids = np.tile((np.arange(K) % N + 1).astype(np.int32), (E, 1))
    acts = rng.integers(0, 5, size=(E, K)).astype(np.int32)
    o = {k: _np(v).copy() for k, v in b.act(torch.from_numpy(ids).cuda(),
                                             torch.from_numpy(acts).cuda()).items()}
    pos = _np(b.pos)
    b.check_err()
    for e in list(range(0, E, 64)) + [E - 1]:
        w = PrimalWorld(inst["grid"][e % inst["grid"].shape[0]], inst["init_pos"][e],
                        inst["goals"][e], s)
        for k in range(K):
            maps, vec, r, done, mask, on_goal, _, valid = w.step(int(ids[e, k]) - 1, int(acts[e, k]))
            assert np.float64(r).view(np.uint64) == o["reward"][e, k].view(np.uint64), (e, k)
            assert done == bool(o["done"][e, k]) and mask == int(o["next_mask"][e, k]), (e, k)
            assert on_goal == bool(o["on_goal"][e, k]) and valid == bool(o["valid"][e, k]), (e, k)
            assert np.array_equal(maps, o["obs"][e, k]), (e, k)
            assert np.array_equal(vec.view(np.uint64), o["vec"][e, k].view(np.uint64)), (e, k)
        assert np.array_equal(np.array(w.pos), pos[e]), e


def test_primal_rejects_bad_past(mapfx_mod):
    g = np.zeros((4, 4), np.int8)
    st, gl = [[[0, 0], [1, 1]]], [[[3, 3], [2, 2]]]
    for past in ([[[0, 0]]], [[[0, 0], [4, 1]]], [[[0, -1], [1, 1]]]):
        with pytest.raises(ValueError):
            mapfx_mod.PrimalBatch(st, gl, grids=g, diagonal=True, past=past)
    mapfx_mod.PrimalBatch(st, gl, grids=g, diagonal=True, past=[[[0, 1], [1, 2]]])


def test_primal_done_when_all_on_goals(mapfx_mod):
    """Agents already on their goals: staying is status 1 (GOAL_REWARD) and done."""
    g = np.zeros((4, 4), np.int8)
    st = np.array([[[0, 0], [3, 3]]], np.int32)
    b = mapfx_mod.PrimalBatch(st, st, grids=g, observation_size=3)
    o = b.act([[1, 2, 1]], [[0, 0, 1]])
    assert _np(o["reward"])[0].tolist() == [0.0, 0.0, -0.3]
    assert _np(o["done"])[0].tolist() == [1, 1, 0]
    assert _np(o["valid"])[0].tolist() == [1, 1, 1]


def test_primal_bad_call_sets_err(mapfx_mod):
    g = np.zeros((4, 4), np.int8)
    b = mapfx_mod.PrimalBatch([[[0, 0]], [[1, 1]]], [[[3, 3]], [[2, 2]]], grids=g[None],
                              observation_size=3)
    b.act([[1, 1], [1, 2]], [[1, 2], [0, 0]])  # world 1: agent id 2 does not exist
    with pytest.raises(AssertionError, match="world 1"):
        b.check_err()
    b.act([[1], [1]], [[0], [5]])  # action 5 (diagonal) not available
    with pytest.raises(AssertionError, match="world 1"):
        b.check_err()


def test_primal_diagonal_action_range(mapfx_mod):
    """DIAGONAL_MOVEMENT: actions 5..8 are moves, 9 is refused (:552-557)."""
    g = np.zeros((5, 5), np.int8)
    b = mapfx_mod.PrimalBatch([[[2, 2]], [[0, 0]]], [[[4, 4]], [[1, 1]]], grids=g[None],
                              observation_size=3, diagonal=True)
    o = b.act([[1, 1], [1, 1]], [[5, 7], [5, 9]])    # world 1, call 1: action 9 is invalid
    with pytest.raises(AssertionError, match="world 1"):
        b.check_err()
    assert _np(b.pos).tolist() == [[[2, 2]], [[1, 1]]]  # world 0: (2,2) -> (3,3) -> (2,2)
    assert _np(b.past).tolist() == [[[3, 3]], [[0, 0]]]
    assert _np(o["valid"])[0].tolist() == [1, 1] and _np(o["on_goal"])[1, 0] == 1
    assert o["next_mask"].dtype == torch.int16 and int(_np(o["next_mask"])[0, 0]) & (1 << 7) == 0


def test_primal_rejects_bad_placement(mapfx_mod):
    g = np.zeros((4, 4), np.int8)
    g[1, 1] = -1
    with pytest.raises(ValueError):
        mapfx_mod.PrimalBatch([[[1, 1]]], [[[0, 0]]], grids=g)
    with pytest.raises(ValueError):
        mapfx_mod.PrimalBatch([[[0, 0], [0, 0]]], [[[2, 2], [3, 3]]], grids=g)


@pytest.mark.parametrize("name", sorted(os.path.basename(p)[:-4]
                                        for p in glob.glob(os.path.join(GOLDEN, "pw_*.npz"))))
def test_primal_dropin_random_world_matches_reference(mapfx_mod, name):
    """MAPFEnv without world0 (or with blank_world) builds the reference's world for
    the same seeds (tests/golden/pw_*.npz), then steps it on the device; _reset
    reports the stay-free valid moves and on_goal of the new world."""
    import random
    from mapfx.primal import MAPFEnv
    fx = _load(name)
    n = int(fx["num_agents"])
    np.random.seed(int(fx["seed"]))
    random.seed(int(fx["seed"]))
    if "world0" in fx:
        env = MAPFEnv(num_agents=n, world0=fx["world0"].astype(int), blank_world=True)
    else:
        env = MAPFEnv(num_agents=n, SIZE=tuple(fx["SIZE"]), PROB=tuple(fx["PROB"]))
    for a in range(1, n + 1):
        assert env.getPositions()[a - 1] == tuple(int(v) for v in np.argwhere(fx["world"] == a)[0])
        assert env.getGoals()[a - 1] == tuple(int(v) for v in np.argwhere(fx["goals"] == a)[0])
    assert np.array_equal(env.getObstacleMap(), (fx["world"] == -1).astype(int))
    world = fx["world"]
    for a in (1, n):
        nxt, on_goal, blocking = env._reset(a, world0=fx["world"], goals0=fx["goals"])
        r, c = np.argwhere(world == a)[0]
        want = [0]
        for act, (dr, dc) in ((1, (0, 1)), (2, (1, 0)), (3, (0, -1)), (4, (-1, 0))):  # dirDict :28
            rr, cc = r + dr, c + dc
            if 0 <= rr < world.shape[0] and 0 <= cc < world.shape[1] and world[rr, cc] == 0:
                want.append(act)
        assert nxt == want and blocking is False
        assert on_goal == (tuple(np.argwhere(fx["goals"] == a)[0]) == (r, c))
