"""GPU parity of the batched MARL_PARTIAL_ENV through the C ABI
(include/mapfx_partial.h): against the reference's own outputs
(tests/golden/mp_*.npz) and against the CPU restatement (oracle/partial_oracle.py)
on batched random instances.  Rewards bit-exact (fp64 bit patterns); obs equal
to the reference's float64 values rounded to float32 (PyMARL's storage dtype);
state / avail / positions / flags exact."""
import numpy as np
import pytest
import torch

from conftest import load_fixture, partial_fixtures

pytestmark = pytest.mark.gpu

KW = ("obs_window", "obs_knn_agents", "episode_limit", "move_reward", "stay_reward",
      "stay_goal_reward", "node_collide_reward", "edge_collide_reward", "env_collide_reward",
      "complete_reward", "complete_fac", "gamma")


@pytest.fixture(scope="module")
def mapfx_mod():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mapfx
    return mapfx


def _np(t):
    return t.detach().cpu().numpy()


def _mask5(avail):
    return (np.asarray(avail, dtype=np.uint8) << np.arange(5, dtype=np.uint8)).sum(-1)


@pytest.mark.parametrize("name", partial_fixtures())
def test_partial_matches_reference_goldens(mapfx_mod, name):
    fx = load_fixture(name)
    if "meta_output" in fx and bool(fx["meta_output"]):
        pytest.skip("output=True repairs positions on the host: test_partial_dropin_output_mode")
    kw = {k: fx["meta_" + k].item() for k in KW}
    b = mapfx_mod.MarlPartialBatch(fx["init_pos"][None], fx["goals"][None], grids=fx["grid"][None],
                                   **kw)
    gd = _np(b.goal_dist[0]).astype(np.int64)
    ref = fx["goal_dist"]
    assert np.array_equal(gd[ref >= 0], ref[ref >= 0])
    out = b.reset()
    assert np.array_equal(_np(out["obs"][0]), fx["obs0"].astype(np.float32))
    assert np.array_equal(_np(out["avail"][0]), _mask5(fx["avail0"]))
    assert np.array_equal(_np(out["state"][0]), fx["state0"].astype(np.float32))
    acts = torch.from_numpy(fx["actions"]).cuda()
    for t in range(fx["actions"].shape[0]):
        out = b.step(acts[t][None])
        r = _np(out["reward"])[0]
        assert r.view(np.uint64) == fx["reward"][t].view(np.uint64), (t, r, fx["reward"][t])
        assert bool(_np(b.terminated)[0]) == bool(fx["terminated"][t]), t
        assert np.array_equal(_np(b.pos[0]), fx["pos"][t]), t
        assert np.array_equal(_np(b.at_goal[0]), fx["at_goal"][t]), t
        assert np.array_equal(_np(b.done[0]), fx["done"][t]), t
        assert np.array_equal(_np(b.steps[0]), fx["steps"][t]), t
        assert np.array_equal(_np(b.node[0]).astype(np.int32), fx["node"][t]), t
        assert np.array_equal(_np(b.edge[0]), fx["edge"][t]), t
        assert np.array_equal(_np(out["obs"][0]), fx["obs"][t].astype(np.float32)), t
        assert np.array_equal(_np(out["state"][0]), fx["state"][t].astype(np.float32)), t
        assert np.array_equal(_np(out["avail"][0]), _mask5(fx["avail"][t])), t


@pytest.mark.parametrize("S,N,E,K,win,T", [(16, 8, 64, 5, 5, 40), (32, 16, 32, 5, 5, 30),
                                           (12, 5, 40, 8, 3, 25), (24, 30, 6, 5, 7, 20),
                                           # past 64 x 64: the multi-wave BFS, > 64 KB LDS maps
                                           (100, 8, 3, 5, 5, 15), (65, 64, 2, 5, 3, 12),
                                           (194, 16, 2, 4, 7, 10), (256, 6, 1, 5, 5, 8)])
def test_partial_batch_matches_oracle(mapfx_mod, S, N, E, K, win, T):
    """Batched random instances (one free component, distinct starts / goals)."""
    from oracle.partial_oracle import PartialEnvState
    rng = np.random.default_rng(S * 100 + N)
    grids, inits, goals = [], [], []
    for e in range(E):
        g = (rng.random((S, S)) < 0.15).astype(np.int8) * -1
        # keep the largest component (the reference's A* tables need one)
        from tests_helpers_partial import largest_component
        g = largest_component(g)
        free = np.argwhere(g == 0)
        pick = rng.choice(len(free), size=2 * N, replace=False)
        grids.append(g)
        inits.append(free[pick[:N]])
        goals.append(free[pick[N:]])
    grids, inits, goals = np.array(grids), np.array(inits), np.array(goals)
    kw = dict(obs_window=win, obs_knn_agents=K, episode_limit=T - 5, move_reward=-0.01,
              stay_reward=-0.02, stay_goal_reward=0.5, node_collide_reward=-1.5,
              edge_collide_reward=-2, env_collide_reward=-3, complete_reward=1000,
              complete_fac=1.5, gamma=0.99)
    b = mapfx_mod.MarlPartialBatch(inits, goals, grids=grids, **kw)
    refs = [PartialEnvState(grids[e], inits[e], goals[e], **kw) for e in range(E)]
    out = b.reset()
    assert np.array_equal(_np(out["obs"]), np.stack([r.obs() for r in refs]).astype(np.float32))
    acts = rng.integers(0, 5, size=(T, E, N))
    for t in range(T):
        out = b.step(torch.from_numpy(acts[t]).cuda())
        rr = [r.step(acts[t, e]) for e, r in enumerate(refs)]
        rew = np.array([x[0] for x in rr], dtype=np.float64)
        assert np.array_equal(_np(out["reward"]).view(np.uint64), rew.view(np.uint64)), t
        assert np.array_equal(_np(b.terminated).astype(bool), np.array([x[1] for x in rr])), t
        assert np.array_equal(_np(b.pos), np.array([r.pos for r in refs])), t
        assert np.array_equal(_np(out["obs"]), np.stack([r.obs() for r in refs]).astype(np.float32)), t
        assert np.array_equal(_np(out["state"]), np.stack([r.state() for r in refs]).astype(np.float32)), t
        assert np.array_equal(_np(out["avail"]), np.stack([_mask5(r.avail()) for r in refs])), t


def test_partial_dropin_env(mapfx_mod, tmp_path):
    """MARL_PARTIAL_ENV drop-in through the registry, against the yaml-config
    golden (same RNG draws select the same scen file / lines)."""
    import random
    from mapfx.envs import REGISTRY
    fx = load_fixture("mp_yaml_empty8_n15")
    # the golden was generated with the reference's own empty-8-8 map + scen files,
    # which do not travel; rebuild an equivalent instance file from the fixture
    grid = fx["grid"]
    mp = tmp_path / "m.map"
    mp.write_text("type octile\nheight 8\nwidth 8\nmap\n" +
                  "\n".join("".join("." if v == 0 else "@" for v in row) for row in grid) + "\n")
    prefix = str(tmp_path / "m-random-")
    lines = ["version 1"] + ["0\tm.map\t8\t8\t%d\t%d\t%d\t%d\t0" % (s[1], s[0], g[1], g[0])
                             for s, g in zip(fx["init_pos"], fx["goals"])] + \
            ["0\tm.map\t8\t8\t0\t0\t0\t0\t0"]
    for k in range(1, 26):
        (tmp_path / ("m-random-%d.scen" % k)).write_text("\n".join(lines) + "\n")
    kw = {k: fx["meta_" + k].item() for k in KW}
    random.seed(0)
    env = REGISTRY["marl_partial"](grid_file_path=str(mp), agents_path=prefix, n_agents=15, **kw)
    # pin the instance to the golden's draw (the scen file lines here are in agent order)
    env._MARL_PARTIAL_ENV__setup_agent = lambda: None
    env._agent_init_pos = [tuple(p) for p in fx["init_pos"]]
    env._agent_goal_pos = [tuple(p) for p in fx["goals"]]
    obs = env.reset()
    assert np.array_equal(obs, fx["obs0"].astype(np.float32))
    assert env.get_env_info()["obs_shape"] == fx["obs0"].shape[1]
    for t in range(fx["actions"].shape[0]):
        r, term, info = env.step(list(fx["actions"][t]))
        assert np.float64(r).view(np.uint64) == fx["reward"][t].view(np.uint64), t
        assert term == bool(fx["terminated"][t])
        assert info["_step_count"] == t + 1
        assert np.array_equal(env.get_obs(), fx["obs"][t].astype(np.float32)), t
        assert np.array_equal(env.get_state(), fx["state"][t].astype(np.int64)), t
        assert env.get_avail_actions() == fx["avail"][t].astype(int).tolist(), t


def test_partial_bench_shape_matches_oracle(mapfx_mod):
    """The bench's marl_partial workload itself (bench.py --env marl_partial: yaml config,
    empty 8x8, 15 agents, 4096 envs, synthetic starts / goals) for a few steps, every
    env against the CPU restatement."""
    from mapfx.maps import synthetic_instances
    from oracle.partial_oracle import PartialEnvState
    import bench
    S, N, E, T = 8, 15, 4096, 3
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.0, seed=1)
    grid = np.zeros((S, S), dtype=np.int8)
    b = mapfx_mod.MarlPartialBatch(inst["init_pos"], inst["goals"], grids=grid[None],
                                   **bench.PARTIAL_YAML)
    refs = [PartialEnvState(grid, inst["init_pos"][e], inst["goals"][e], **bench.PARTIAL_YAML)
            for e in range(E)]
    b.reset()
    rng = np.random.default_rng(5)
    for t in range(T):
        acts = rng.integers(0, 5, size=(E, N))
        out = b.step(torch.from_numpy(acts).cuda())
        rr = [r.step(acts[e]) for e, r in enumerate(refs)]
        rew = np.array([x[0] for x in rr], dtype=np.float64)
        assert np.array_equal(_np(out["reward"]).view(np.uint64), rew.view(np.uint64)), t
        assert np.array_equal(_np(b.pos), np.array([r.pos for r in refs])), t
        assert np.array_equal(_np(out["obs"]), np.stack([r.obs() for r in refs]).astype(np.float32)), t
        assert np.array_equal(_np(out["avail"]), np.stack([_mask5(r.avail()) for r in refs])), t


def _bench_actions(mapfx_mod, inst, S, N, T):
    """bench.py --env marl_partial's actions: the device generator (seed 2) of a
    MapfGridBatch over the same instances, [T, E, N] int8 in HBM."""
    ga = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                                 obs=(), track_steps=False)
    return ga.gen_actions(T, seed=2)


def test_partial_bench_episode_matches_oracle(mapfx_mod):
    """the bench's whole replayed episode at its shape (yaml config, empty
    8x8, 15 agents, 4096 envs, the generator's int8 actions): reset + 100 steps (the
    episode limit: every env terminates at t = 100) + a second reset + 5 steps, every
    64th env and the last against the CPU restatement at every step.  Every other
    sampled env has its goals on its starts and stays put at steps 0 and 40, so the
    completion bonus (marl_partial.py:291-299) fires at 4096 envs; the second reset
    re-initialises the carried goal distances (pdist / pnbr, ABI 4) that every step
    after it uses."""
    from mapfx.maps import synthetic_instances
    from oracle.partial_oracle import PartialEnvState
    import bench
    S, N, E = 8, 15, 4096
    limit = bench.PARTIAL_YAML["episode_limit"]
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.0, seed=1)
    sample = list(range(5, E, 64)) + [E - 1]
    complete = sample[::2]
    goals = inst["goals"].copy()
    goals[complete] = inst["init_pos"][complete]
    grid = np.zeros((S, S), dtype=np.int8)
    b = mapfx_mod.MarlPartialBatch(inst["init_pos"], goals, grids=grid[None], **bench.PARTIAL_YAML)
    refs = {e: PartialEnvState(grid, inst["init_pos"][e], goals[e], **bench.PARTIAL_YAML) for e in sample}
    acts = _bench_actions(mapfx_mod, inst, S, N, limit)
    acts[0, complete] = 4
    acts[40, complete] = 4
    ah = _np(acts).astype(np.int64)
    idx = torch.tensor(sample, device="cuda")
    bonus_seen = 0

    def check(out, t, rr=None):
        nonlocal bonus_seen
        obs = _np(out["obs"][idx])
        for j, e in enumerate(sample):
            r = refs[e]
            assert np.array_equal(obs[j], r.obs().astype(np.float32)), (t, e)
            assert np.array_equal(_np(out["avail"][e]), _mask5(r.avail())), (t, e)
            assert np.array_equal(_np(out["state"][e]), r.state().astype(np.float32)), (t, e)
            assert np.array_equal(_np(b.pos[e]), np.array(r.pos)), (t, e)
            if rr is not None:
                rew, term = rr[e]
                got = _np(out["reward"][e:e + 1])
                assert got.view(np.uint64)[0] == np.float64(rew).view(np.uint64), (t, e, got, rew)
                assert bool(_np(b.terminated[e:e + 1])[0]) == bool(term), (t, e)
                bonus_seen += int(rew > 100)

    for ep in range(2):
        out = b.reset()
        for r in refs.values():
            r.reset()
        check(out, -1)
        for t in range(limit if ep == 0 else 5):
            out = b.step(acts[t])
            rr = {e: refs[e].step(ah[t, e]) for e in sample}
            check(out, t, rr)
        if ep == 0:
            assert _np(b.terminated).all() and (_np(b.t) == limit).all()   # the episode limit
    assert bonus_seen >= len(complete)


def test_partial_carried_distances_equal_lookup(mapfx_mod):
    """the carried goal distances (pdist / pnbr, ABI 4) give the same episode
    as the table lookups a binding without them gets (NULL pointers), and a step right
    after set_agents() (new goals, new tables, no reset) uses the new tables: equal to
    the lookup path and to the restatement with the new goals."""
    from oracle.partial_oracle import PartialEnvState, bfs_goal_dist
    from tests_helpers_partial import largest_component
    rng = np.random.default_rng(11)
    S, N, E, T = 12, 6, 24, 12
    kw = dict(obs_window=5, obs_knn_agents=5, episode_limit=60, move_reward=-0.01,
              stay_reward=-0.02, stay_goal_reward=0.5, node_collide_reward=-1.5,
              edge_collide_reward=-2, env_collide_reward=-3, complete_reward=1000,
              complete_fac=1.5, gamma=0.99)
    grid = largest_component((rng.random((S, S)) < 0.15).astype(np.int8) * -1)
    free = np.argwhere(grid == 0)
    picks = [rng.choice(len(free), size=3 * N, replace=False) for _ in range(E)]
    inits = np.array([free[p[:N]] for p in picks])
    goals = np.array([free[p[N:2 * N]] for p in picks])
    goals2 = np.array([free[p[2 * N:]] for p in picks])
    carried = mapfx_mod.MarlPartialBatch(inits, goals, grids=grid[None], **kw)
    lookup = mapfx_mod.MarlPartialBatch(inits, goals, grids=grid[None], **kw)
    lookup._state.pdist = None
    lookup._state.pnbr = None
    assert carried.pnbr is not None          # u8 tables (144 cells): the carried path is on
    refs = [PartialEnvState(grid, inits[e], goals[e], **kw) for e in range(E)]
    carried.reset()
    lookup.reset()
    acts = rng.integers(0, 5, size=(2 * T, E, N))
    for t in range(2 * T):
        if t == T:   # new goals mid-episode, tables rebuilt, no reset
            mask = np.zeros(E, dtype=bool)
            mask[::2] = True
            g_new = np.where(mask[:, None, None], goals2, goals)
            for bb in (carried, lookup):
                bb.set_agents(inits, g_new, env_mask=mask)
            for e in np.flatnonzero(mask):
                refs[e].goals = [tuple(int(v) for v in p) for p in goals2[e]]
                refs[e].goal_dist = [bfs_goal_dist(refs[e].grid, g) for g in refs[e].goals]
                refs[e]._refresh()
        a = torch.from_numpy(acts[t]).cuda()
        oc = carried.step(a)
        rc = _np(oc["reward"]).copy()
        obs_c = _np(oc["obs"]).copy()
        ol = lookup.step(a)
        assert np.array_equal(rc.view(np.uint64), _np(ol["reward"]).view(np.uint64)), t
        assert np.array_equal(obs_c, _np(ol["obs"])), t
        ref = np.array([r.step(acts[t, e])[0] for e, r in enumerate(refs)], dtype=np.float64)
        assert np.array_equal(rc.view(np.uint64), ref.view(np.uint64)), t
        assert np.array_equal(obs_c, np.stack([r.obs() for r in refs]).astype(np.float32)), t


def test_partial_dropin_output_mode(mapfx_mod, tmp_path):
    """MARL_PARTIAL_ENV(output=True) through the registry against the reference run
    with output=True (mp_out8_n5): the drop-in draws the same instance with the same
    `random` calls, steps on the GPU, repairs collisions on the host (the global
    `random` stream, as the reference) and re-observes on the GPU."""
    import random
    from mapfx.envs import REGISTRY
    fx = load_fixture("mp_out8_n5")
    grid = fx["grid"]
    s = grid.shape[0]
    mp = tmp_path / "m.map"
    mp.write_text("type octile\nheight %d\nwidth %d\nmap\n" % (s, s) +
                  "\n".join("".join("." if v == 0 else "@" for v in row) for row in grid) + "\n")
    st, gl = fx["scen_starts"], fx["scen_goals"]
    rows = ["0\tm.map\t%d\t%d\t%d\t%d\t%d\t%d\t0" % (s, s, a[1], a[0], b[1], b[0])
            for a, b in zip(st, gl)]
    rows.append(rows[0])
    for k in range(1, 26):
        (tmp_path / ("m-random-%d.scen" % k)).write_text("version 1\n" + "\n".join(rows) + "\n")
    kw = {k: fx["meta_" + k].item() for k in KW}
    random.seed(int(fx["meta_py_seed"]))
    env = REGISTRY["marl_partial"](grid_file_path=str(mp), agents_path=str(tmp_path / "m-random-"),
                                   n_agents=int(fx["init_pos"].shape[0]), output=True, **kw)
    random.seed(int(fx["meta_reset_seed"]))
    obs = env.reset()
    assert np.array_equal(obs, fx["obs0"].astype(np.float32))
    for t in range(fx["actions"].shape[0]):
        r, term, info = env.step(list(fx["actions"][t]))
        assert np.float64(r).view(np.uint64) == fx["reward"][t].view(np.uint64), t
        assert term == bool(fx["terminated"][t])
        assert [env.agent_pos(i) for i in range(len(fx["pos"][t]))] == \
            [tuple(p) for p in fx["pos"][t].tolist()], t
        assert np.array_equal(env.get_obs(), fx["obs"][t].astype(np.float32)), t
        assert np.array_equal(env.get_state(), fx["state"][t].astype(np.int64)), t
        assert env.get_avail_actions() == fx["avail"][t].astype(int).tolist(), t
