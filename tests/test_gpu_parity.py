"""GPU parity: the HIP path (through the C ABI) vs the reference golden vectors
and vs the C oracle on seeded batched inputs.  Bit-exact for every output:
positions, dones, node/edge collisions, fp64 rewards (bit patterns), avail
masks, occupancy / window / PRIMAL observations."""
import numpy as np
import pytest
import torch

from conftest import fixture_rewards, load_fixture, primal_fixtures, step_fixtures

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mapfx_mod():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mapfx
    return mapfx


def _u64(x):
    return np.ascontiguousarray(x).view(np.uint64)


def _np(t):
    return t.detach().cpu().numpy()


# ---------------------------------------------------------------------------
# 1. golden vectors from the reference (single env)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", step_fixtures())
def test_step_matches_reference_goldens(mapfx_mod, name):
    fx = load_fixture(name)
    sr, cr = fixture_rewards(fx)
    windows = sorted(int(k[6:]) for k in fx if k.startswith("window") and k != "window_steps")
    wsteps = list(fx["window_steps"])
    h, w = fx["grid"].shape
    for win in windows:
        b = mapfx_mod.MapfGridBatch(fx["init_pos"][None], fx["goals"][None],
                                    grids=fx["grid"][None], episode_limit=int(fx["meta_limit"]),
                                    step_reward=sr, collide_reward=cr, obs=("full", "window"),
                                    window=win)
        out = b.reset()
        assert np.array_equal(_np(out["obs_full"][0]).reshape(h, w), fx["occ0"])
        mask0 = (fx["avail0"].astype(np.uint8) << np.arange(5, dtype=np.uint8)).sum(-1)
        assert np.array_equal(_np(out["avail"][0]), mask0)
        acts = torch.from_numpy(fx["actions"].astype(np.int64)).cuda()  # PyMARL hands int64
        for t in range(fx["actions"].shape[0]):
            out = b.step(acts[t][None])
            assert _u64(_np(out["reward"]))[0] == _u64(fx["reward"][t:t + 1])[0], (t, win)
            assert np.array_equal(_np(b.pos[0]), fx["pos"][t]), t
            assert np.array_equal(_np(b.done[0]), fx["done"][t]), t
            assert np.array_equal(_np(out["node"][0]), fx["node"][t]), t
            assert np.array_equal(_np(out["edge"][0]), fx["edge"][t]), t
            assert np.array_equal(_np(b.avail_actions()[0]), fx["avail"][t].astype(np.int64)), t
            assert int(_np(b.t)[0]) == int(fx["t"][t])
            assert bool(_np(out["term"])[0]) == bool(fx["done"][t].all())
            if "occ" in fx:
                assert np.array_equal(_np(out["obs_full"][0]).reshape(h, w), fx["occ"][t]), t
            if t in wsteps:
                wi = wsteps.index(t)
                assert np.array_equal(_np(out["obs_window"][0]), fx["window%d" % win][wi]), \
                    (t, win)
        assert int(b.err.item()) == 0


@pytest.mark.parametrize("name", primal_fixtures())
def test_primal_matches_reference_goldens(mapfx_mod, name):
    fx = load_fixture(name)
    E = fx["pos"].shape[0]
    goals = np.broadcast_to(fx["goals"][None], (E,) + fx["goals"].shape)
    for s in [int(v) for v in np.atleast_1d(fx["meta_sizes"])]:
        b = mapfx_mod.MapfGridBatch(fx["pos"], goals, grids=fx["grid"][None].repeat(E, 0),
                                    obs=("primal",), primal_size=s)
        out = b.reset()
        assert np.array_equal(_np(out["obs_primal"]), fx["maps%d" % s]), s
        assert np.array_equal(_u64(_np(out["primal_vec"])), _u64(fx["vec%d" % s])), s


# ---------------------------------------------------------------------------
# 2. batched parity vs the C oracle (configs of BASELINE.json + odd shapes)
# ---------------------------------------------------------------------------
CONFIGS = [
    # name, E, H(=W), N, p_obst, steps, window, shared_warehouse, limit
    ("c1_8x8_n2", 64, 8, 2, 0.0, 60, 5, False, 2000),
    ("c2_32x32_n16", 4096, 32, 16, 0.10, 24, 5, False, 2000),
    ("c3_wh64_n64", 512, 64, 64, None, 12, 5, True, 2000),
    ("c5_128_n256", 32, 128, 256, 0.10, 6, 5, False, 2000),
    ("odd_13x13_n5_w7", 300, 13, 5, 0.25, 40, 7, False, 17),
    ("dense_10x10_n90", 40, 10, 90, 0.05, 30, 3, False, 2000),
    ("n200_24x24", 12, 24, 200, 0.05, 10, 5, False, 2000),
    ("n300_40x40_apl2", 6, 40, 300, 0.05, 8, 4, False, 2000),
]


def _instances(mapfx_mod, E, S, N, p, shared, seed=3):
    from mapfx.maps import synthetic_instances, warehouse_grid
    if shared:
        return synthetic_instances(E, S, S, N, seed=seed, shared_grid=warehouse_grid(S))
    return synthetic_instances(E, S, S, N, p_obstacle=p, seed=seed)


@pytest.mark.parametrize("cfg", CONFIGS, ids=[c[0] for c in CONFIGS])
def test_batched_step_matches_oracle(mapfx_mod, cfg):
    from oracle import corc
    name, E, S, N, p, T, win, shared, limit = cfg
    inst = _instances(mapfx_mod, E, S, N, p, shared)
    init = inst["init_pos"].copy()
    if name.startswith("dense"):   # stacked starts / starts on obstacles (quirks 1, 3)
        rs = np.random.RandomState(1)
        init = rs.randint(0, S, size=(E, N, 2)).astype(np.int32)
    b = mapfx_mod.MapfGridBatch(init, inst["goals"], bits=inst["bits"], hw=(S, S),
                                episode_limit=limit, obs=("full", "window"), window=win)
    ob = corc.OracleBatch(inst["bits"], init, inst["goals"], S, S, limit=limit)
    out = b.reset()
    ref = ob.observe(window=win)
    assert np.array_equal(_np(out["obs_full"]), ref["obs_full"])
    assert np.array_equal(_np(out["obs_window"]), ref["obs_window"])
    rs = np.random.RandomState(7)
    for t in range(T):
        a = rs.randint(0, 5, size=(E, N)).astype(np.int8)
        out = b.step(torch.from_numpy(a).cuda())
        rstep = ob.step(a.astype(np.int32))
        ref = ob.observe(window=win)
        assert np.array_equal(_np(b.pos), ob.pos), (name, t)
        assert np.array_equal(_np(b.done), ob.done), (name, t)
        assert np.array_equal(_np(b.t), ob.t), (name, t)
        assert np.array_equal(_np(b.steps), ob.steps), (name, t)
        assert np.array_equal(_u64(_np(out["reward"])), _u64(rstep["reward"])), (name, t)
        assert np.array_equal(_np(out["reward_f32"]), rstep["reward"].astype(np.float32))
        assert np.array_equal(_np(out["node"]), rstep["node"]), (name, t)
        assert np.array_equal(_np(out["edge"]), rstep["edge"]), (name, t)
        assert np.array_equal(_np(out["avail"]), ref["avail"]), (name, t)
        assert np.array_equal(_np(out["term"]), ref["term"]), (name, t)
        assert np.array_equal(_np(out["obs_full"]), ref["obs_full"]), (name, t)
        assert np.array_equal(_np(out["obs_window"]), ref["obs_window"]), (name, t)


@pytest.mark.parametrize("cfg", CONFIGS, ids=[c[0] for c in CONFIGS])
def test_window_occ_matches_oracle(mapfx_mod, cfg):
    """obs_window_occ (one occupancy plane, generic kernel's block-cooperative writer)
    decodes to the oracle's {obstacle, agents} window planes, every step."""
    from mapfx.batch import window_planes
    from oracle import corc
    name, E, S, N, p, T, win, shared, limit = cfg
    inst = _instances(mapfx_mod, E, S, N, p, shared)
    init = inst["init_pos"].copy()
    if name.startswith("dense"):
        init = np.random.RandomState(1).randint(0, S, size=(E, N, 2)).astype(np.int32)
    b = mapfx_mod.MapfGridBatch(init, inst["goals"], bits=inst["bits"], hw=(S, S),
                                episode_limit=limit, obs=("window_occ",), window=win)
    ob = corc.OracleBatch(inst["bits"], init, inst["goals"], S, S, limit=limit)
    out = b.reset()
    assert np.array_equal(_np(window_planes(out["obs_window_occ"])), ob.observe(window=win)["obs_window"])
    rs = np.random.RandomState(7)
    for t in range(min(T, 6)):
        a = rs.randint(0, 5, size=(E, N)).astype(np.int8)
        out = b.step(torch.from_numpy(a).cuda())
        rstep = ob.step(a.astype(np.int32))
        ref = ob.observe(window=win)
        assert np.array_equal(_u64(_np(out["reward"])), _u64(rstep["reward"])), (name, t)
        assert np.array_equal(_np(out["avail"]), ref["avail"]), (name, t)
        assert np.array_equal(_np(window_planes(out["obs_window_occ"])), ref["obs_window"]), (name, t)


def test_window_occ_full_stack(mapfx_mod):
    """N = 256 agents stacked on one free cell: the occupancy value 256 needs the
    int16 cells; both window formats carry it exactly."""
    from mapfx.batch import window_planes
    E, S, N = 3, 16, 256
    init = np.full((E, N, 2), 7, dtype=np.int32)
    goals = np.zeros((E, N, 2), dtype=np.int32)
    grid = np.zeros((S, S), dtype=np.uint8)
    grid[7, 9] = 1
    b = mapfx_mod.MapfGridBatch(init, goals, grids=grid, episode_limit=100,
                                obs=("window", "window_occ"), window=5)
    out = b.reset()
    occ = _np(out["obs_window_occ"])
    assert occ.dtype == np.int16 and (occ[:, :, 2, 2] == 256).all()
    assert (occ[:, :, 2, 4] == -1).all()                     # the obstacle at (7, 9)
    assert np.array_equal(_np(window_planes(out["obs_window_occ"])), _np(out["obs_window"]))
    out = b.step(torch.full((E, N), 4, dtype=torch.int8, device="cuda"))   # all stay
    occ = _np(out["obs_window_occ"])
    assert (occ[:, :, 2, 2] == 256).all()
    assert np.array_equal(_np(window_planes(out["obs_window_occ"])), _np(out["obs_window"]))


@pytest.mark.parametrize("S,N,s,E", [(32, 16, 10, 64), (64, 32, 10, 16), (20, 30, 7, 50),
                                     (128, 200, 11, 4)])
def test_batched_primal_matches_oracle(mapfx_mod, S, N, s, E):
    from mapfx.maps import synthetic_instances
    from oracle import corc
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.15, seed=4)
    b = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                                obs=("primal", "window"), primal_size=s, window=5)
    ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], S, S)
    rs = np.random.RandomState(2)
    b.reset()
    for t in range(6):
        a = rs.randint(0, 5, size=(E, N)).astype(np.int8)
        out = b.step(torch.from_numpy(a).cuda())
        ob.step(a.astype(np.int32))
        ref = ob.observe(psize=s, full=False, win=True, primal=True)
        assert np.array_equal(_np(out["obs_primal"]), ref["obs_primal"]), t
        assert np.array_equal(_u64(_np(out["primal_vec"])), _u64(ref["primal_vec"])), t
        assert np.array_equal(_np(out["obs_window"]), ref["obs_window"]), t


# ---------------------------------------------------------------------------
# 3. fused rollout == repeated steps; device generator == host generator
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("S,N,E,T,obs,win", [
    (32, 16, 1000, 20, ("full", "window", "primal"), 5),   # generic kernel (PRIMAL)
    (32, 16, 1000, 20, ("full", "window"), 5),             # wave-local fast path
    (8, 2, 300, 50, ("full", "window"), 3),
    (13, 7, 200, 30, ("full", "window"), 7),
    (8, 2, 300, 50, ("full", "window", "primal"), 5),
    (64, 64, 40, 8, ("full", "window"), 5),
    (64, 64, 40, 8, ("full", "window", "primal"), 5),
    (128, 256, 4, 4, ("full", "window", "primal"), 5),
    # C5 shape with the occupancy window (+ reward_f32 and the full output set: feature
    # set 0, NOT the bench's FEAT_RUN instance -- that one is test_bench_leg_matches_oracle)
    (128, 256, 6, 6, ("window_occ",), 5),
    (100, 300, 5, 5, ("window", "window_occ"), 7),          # APL 2
    (32, 16, 300, 12, ("window_occ",), 3)])                 # u8 cells, 16 envs per block
def test_rollout_equals_repeated_steps(mapfx_mod, S, N, E, T, obs, win):
    from mapfx import rng
    from mapfx.maps import synthetic_instances
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=5)
    kw = dict(bits=inst["bits"], hw=(S, S), episode_limit=35, obs=obs, window=win,
              primal_size=10)
    b1 = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], env_offset=1000, **kw)
    b2 = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], env_offset=1000, **kw)
    b1.reset()
    b2.reset()
    seed, t0 = 99, 3
    acts = b2.gen_actions(T, seed, t0=t0)
    host = rng.gen_actions(seed, np.arange(1000, 1000 + E), np.arange(t0, t0 + T), N)
    assert np.array_equal(_np(acts), host)
    traj = b1.rollout(T, seed=seed, t0=t0)
    traj_buf = b2.rollout(T, actions=acts.to(torch.int32))  # actions read from HBM
    b3 = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], env_offset=1000, **kw)
    b3.reset()
    for k in range(T):
        out = b3.step(acts[k])
        for key in ("reward", "node", "edge", "avail", "term", "obs_full", "obs_window",
                    "obs_window_occ", "obs_primal", "primal_vec"):
            if key not in out:
                continue
            x = _np(out[key])
            for tr in (traj, traj_buf):
                y = _np(tr[key][k])
                if x.dtype == np.float64:
                    assert np.array_equal(_u64(x), _u64(y)), (key, k)
                else:
                    assert np.array_equal(x, y), (key, k)
        for tr in (traj, traj_buf):
            assert np.array_equal(_np(tr["traj_pos"][k]), _np(b3.pos)), k
            assert np.array_equal(_np(tr["traj_done"][k]), _np(b3.done)), k
            assert np.array_equal(_np(tr["traj_t"][k]), _np(b3.t)), k
    for bb in (b1, b2):
        assert np.array_equal(_np(bb.pos), _np(b3.pos))
        assert np.array_equal(_np(bb.done), _np(b3.done))
        assert np.array_equal(_np(bb.t), _np(b3.t))
        assert np.array_equal(_np(bb.steps), _np(b3.steps))


@pytest.mark.parametrize("E,T,win,autoreset,N", [
    (4096, 64, 5, False, 16),   # the bench shape
    (4096, 20, 5, False, 16),   # the driver's shape: T <= 32 takes the 8-step action-block instance
    (256, 1, 5, False, 16), (256, 2, 5, False, 16), (256, 3, 3, False, 16), (252, 17, 7, False, 16),
    # T = 15 / 16: either side of the preloaded "T >= 16" bit (the first action block
    # fetched without a clamp to T)
    (256, 15, 5, False, 16), (256, 16, 5, False, 16), (128, 16, 5, False, 64),
    (64, 40, 5, True, 16),
    (250, 12, 5, False, 12), (130, 9, 3, True, 7), (66, 10, 5, False, 40),  # N < L
    (130, 12, 5, False, 64), (64, 40, 3, True, 64), (40, 9, 7, False, 64),  # 64-agent store wave
    # obs_window_occ records from the store wave (the gather payload of bench --gpus N)
    (4096, 20, 5, False, -16), (256, 3, 3, False, -16), (252, 17, 7, False, -16),
    (64, 40, 5, True, -16)])
def test_runner_rollout_every_step(mapfx_mod, E, T, win, autoreset, N):
    """Runner rollouts (every PyMARL output, no full map; N = 16 takes the store-wave
    kernel): each step's outputs must equal one step launch's, step by step.
    N < 0: the occupancy window (obs_window_occ) instead of the two planes; the
    single steps write it with the generic kernel, the rollout with the store wave."""
    from mapfx.maps import synthetic_instances
    occ = N < 0
    N = abs(N)
    wkey = "obs_window_occ" if occ else "obs_window"
    S = 32 if not autoreset else (8 if N <= 16 else 12)
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=12)
    kw = dict(bits=inst["bits"], hw=(S, S), episode_limit=2000 if not autoreset else 9,
              obs=("window_occ",) if occ else ("window",), window=win)
    b1 = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], **kw)
    b2 = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], **kw)
    b1.reset()
    b2.reset()
    acts = b2.gen_actions(T, 21, t0=0)
    traj = b1.rollout(T, actions=acts, autoreset=autoreset)
    keys = ("reward", "reward_f32", "term", "node", "edge", "avail", wkey)
    for k in range(T):
        out = b2.step(acts[k])
        for key in keys:
            x, y = _np(out[key]), _np(traj[key][k])
            if x.dtype == np.float64:
                assert np.array_equal(_u64(x), _u64(y)), (key, k)
            else:
                assert np.array_equal(x, y), (key, k)
        assert np.array_equal(_np(traj["traj_pos"][k]), _np(b2.pos)), k
        assert np.array_equal(_np(traj["traj_done"][k]), _np(b2.done)), k
        assert np.array_equal(_np(traj["traj_t"][k]), _np(b2.t)), k
        if autoreset and out["term"].any():
            b2.reset(env_mask=out["term"].clone())
    assert np.array_equal(_np(b1.pos), _np(b2.pos))
    assert np.array_equal(_np(b1.done), _np(b2.done))
    assert np.array_equal(_np(b1.t), _np(b2.t))


@pytest.mark.parametrize("autoreset", [False, True])
def test_runner_rollout_agents_on_obstacles(mapfx_mod, autoreset):
    """The store-wave kernel runs the dynamics from static obstacle flags only in blocks
    where no agent stands (or is reset) on an obstacle; a block with such an agent
    (quirk 1: the obstacle becomes enterable while occupied) takes the one-wave step
    side.  Mixed blocks, every step equal to single step launches."""
    from mapfx.maps import synthetic_instances
    E, S, N, T, win = 256, 8, 16, 40, 5
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.15, seed=31)
    bits = np.asarray(inst["bits"])
    init = np.array(inst["init_pos"])
    rng = np.random.default_rng(3)
    for e in range(0, E, 3):          # every third env: one agent starts on an obstacle
        b_ = bits[e if bits.shape[0] > 1 else 0]
        cells = [c for c in range(S * S) if (b_[c >> 3] >> (c & 7)) & 1]
        if cells:
            c = int(rng.choice(cells))
            init[e, int(rng.integers(N))] = (c // S, c % S)
    kw = dict(bits=inst["bits"], hw=(S, S), episode_limit=2000 if not autoreset else 9,
              obs=("window",), window=win)
    b1 = mapfx_mod.MapfGridBatch(init, inst["goals"], **kw)
    b2 = mapfx_mod.MapfGridBatch(init, inst["goals"], **kw)
    b1.reset()
    b2.reset()
    acts = b2.gen_actions(T, 23, t0=0)
    traj = b1.rollout(T, actions=acts, autoreset=autoreset)
    for k in range(T):
        out = b2.step(acts[k])
        for key in ("reward", "term", "node", "edge", "avail", "obs_window"):
            x, y = _np(out[key]), _np(traj[key][k])
            if x.dtype == np.float64:
                assert np.array_equal(_u64(x), _u64(y)), (key, k)
            else:
                assert np.array_equal(x, y), (key, k)
        assert np.array_equal(_np(traj["traj_pos"][k]), _np(b2.pos)), k
        assert np.array_equal(_np(traj["traj_done"][k]), _np(b2.done)), k
        if autoreset and out["term"].any():
            b2.reset(env_mask=out["term"].clone())
    assert np.array_equal(_np(b1.pos), _np(b2.pos))
    assert np.array_equal(_np(b1.t), _np(b2.t))


# the instance pick_wave_win chooses for the bench's C2 launch (mapfx.hip): T <= 32 takes
# the 8-step action block, longer launches the default 16-step one (template arg 0)
C2_SPLIT_INSTANCE = {20: "mapf_wave_kernel<5, true, true, true, 16, true, false, 8>",
                     64: "mapf_wave_kernel<5, true, true, true, 16, true, false, 0>"}

# every timed mapf_grid leg of bench.py: (config, T).  T = 20 is the driver's
# `--steps 20`, T = 64 the default --chunk; T = 33 is the first C2 launch past the
# short-action-block threshold.
BENCH_LEGS = [("c2", 20), ("c2", 64), ("c2", 33), ("c1", 64), ("c1", 20), ("c3", 64),
              ("c3", 20), ("c5", 64), ("c5", 20)]


def _profile_kernel(config, T, E):
    """The kernel instance profiles/pmc_<config>.json was taken of, when that profile is
    of this (config, T, E) workload; else None."""
    import json
    import os
    import bench
    path = os.path.join(bench.REPO, "profiles", "pmc_%s.json" % config)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        pm = json.load(f)
    if pm.get("config") != config or pm.get("T") != T or pm.get("E") != E:
        return None
    return bench.kernel_instance(pm.get("kernel", ""))


@pytest.mark.parametrize("config,T", BENCH_LEGS, ids=["%s-T%d" % x for x in BENCH_LEGS])
def test_bench_leg_matches_oracle(mapfx_mod, config, T):
    """Every timed bench leg, structurally: the batch, output set and trajectory buffers
    come from bench.mapf_workload / bench.bench_traj -- the code the bench times -- and
    the launch is the bench's prepared rollout_plan with int8 actions resident in HBM.
    Against the C oracle at EVERY step, on every env (C1, C2) or an env slice (C3 every
    2nd, C5 every 8th, plus the last env): reward bits, node, edge, avail, term, the
    window (the planes of obs_window_occ at C5), positions, dones and t.  The launched
    instance must be the one the leg's PMC profile names when that profile is of the
    same workload (config, T, E)."""
    from mapfx import _abi
    from mapfx.batch import window_planes
    from oracle import corc
    import bench
    wl = bench.mapf_workload(config, 5, "cuda:0")
    b, S, N, E, inst, wkey = (wl[k] for k in ("batch", "S", "N", "E", "inst", "wkey"))
    b.reset()
    acts = b.gen_actions(T, seed=bench.ACT_SEED)
    traj = bench.bench_traj(b, T)
    b.rollout_plan(T, actions=acts, traj=traj, outputs=wl["outs"],
                   stream=torch.cuda.current_stream())()
    name = _abi.last_kernel()
    if config == "c2" and T in C2_SPLIT_INSTANCE:
        assert C2_SPLIT_INSTANCE[T] in name, name
    if config == "c5":      # the FEAT_RUN instance (runner output set, no f32 reward)
        assert "mapf_rollout_kernel<unsigned short, 1, 4>" in name, name
    stride = {"c3": 2, "c5": 8}.get(config, 1)
    envs = np.unique(np.append(np.arange(0, E, stride), E - 1))
    bits = inst["bits"] if inst["bits"].shape[0] == 1 else inst["bits"][envs]
    ob = corc.OracleBatch(bits, inst["init_pos"][envs], inst["goals"][envs], S, S,
                          limit=wl["limit"])
    torch.cuda.synchronize()
    ei = torch.from_numpy(envs).cuda()
    tr = {k: _np(v.index_select(1, ei)) for k, v in traj.items()}
    if wkey == "obs_window_occ":
        tr["obs_window"] = _np(window_planes(traj[wkey].index_select(1, ei)))
    ah = _np(acts).astype(np.int32)[:, envs]
    for k in range(T):
        r = ob.step(ah[k])
        o = ob.observe(window=5, full=False)
        assert np.array_equal(_u64(tr["reward"][k]), _u64(r["reward"])), k
        assert np.array_equal(tr["node"][k], r["node"]), k
        assert np.array_equal(tr["edge"][k], r["edge"]), k
        assert np.array_equal(tr["avail"][k], o["avail"]), k
        assert np.array_equal(tr["term"][k], o["term"]), k
        assert np.array_equal(tr["obs_window"][k], o["obs_window"]), k
        assert np.array_equal(tr["traj_pos"][k], ob.pos), k
        assert np.array_equal(tr["traj_done"][k], ob.done), k
        assert np.array_equal(tr["traj_t"][k], ob.t), k
    assert np.array_equal(_np(b.pos)[envs], ob.pos) and np.array_equal(_np(b.t)[envs], ob.t)
    assert np.array_equal(_np(b.done)[envs], ob.done)
    # last: the leg's committed profile must be of this instance (re-profile after a change)
    prof = _profile_kernel(config, T, E)
    if prof is not None:
        assert bench.kernel_instance(name) == prof, (name, prof)


def test_back_to_back_rollout_launches(mapfx_mod):
    """Launches that read the state the previous launch wrote back, enqueued back to back
    with no host wait between them (the bench's timed region: C3, 2048 envs of 64
    agents on the shared warehouse map, 8 launches), equal the oracle's one long
    rollout: every launch's last step and the final state.  A launch overlapping its
    predecessor would read stale positions here."""
    from mapfx import _abi
    from oracle import corc
    import bench
    S, N, E, _, shared = bench.CONFIGS["c3"]
    inst = _instances(mapfx_mod, E, S, N, None, shared, seed=1)
    b = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                                episode_limit=2 ** 31 - 1, obs=("window",), window=5,
                                track_steps=False)
    ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], S, S, limit=2 ** 31 - 1)
    b.reset()
    T, L = 16, 8
    acts = b.gen_actions(T * L, seed=2)
    outs = ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos", "traj_done", "traj_t")
    trajs = []
    for i in range(L):
        tr = b._alloc_out(T)
        tr.pop("reward_f32")
        trajs.append(tr)
    plans = [b.rollout_plan(T, actions=acts[i * T:(i + 1) * T], traj=trajs[i], outputs=outs,
                            stream=torch.cuda.current_stream()) for i in range(L)]
    torch.cuda.synchronize()
    for pl in plans:
        pl()
    assert "mapf_wave_kernel<5, true, true, true, 64" in _abi.last_kernel(), _abi.last_kernel()
    torch.cuda.synchronize()
    ah = _np(acts).astype(np.int32)
    for i in range(L):
        for k in range(T):
            r = ob.step(ah[i * T + k])
        o = ob.observe(window=5, full=False)
        tr = trajs[i]
        assert np.array_equal(_u64(_np(tr["reward"][-1])), _u64(r["reward"])), i
        assert np.array_equal(_np(tr["edge"][-1]), r["edge"]), i
        assert np.array_equal(_np(tr["obs_window"][-1]), o["obs_window"]), i
        assert np.array_equal(_np(tr["traj_pos"][-1]), ob.pos), i
        assert np.array_equal(_np(tr["traj_t"][-1]), ob.t), i
    assert np.array_equal(_np(b.pos), ob.pos) and np.array_equal(_np(b.done), ob.done)


def test_rollout_matches_oracle_long_horizon(mapfx_mod):
    """C2 shape (32x32, 16 agents, 4096 envs), 64 fused steps vs the C oracle."""
    from mapfx.maps import synthetic_instances
    from oracle import corc
    E, S, N, T = 4096, 32, 16, 64
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=1)
    b = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                                episode_limit=2000, obs=("window",))
    ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], S, S, limit=2000)
    b.reset()
    traj = b.rollout(T, seed=2, t0=0)
    ref = ob.rollout(T, seed=2, t0=0)
    assert np.array_equal(_np(b.pos), ob.pos)
    assert np.array_equal(_np(b.done), ob.done)
    assert np.array_equal(_np(b.t), ob.t)
    assert np.array_equal(_u64(_np(traj["reward"][-1])), _u64(ref["reward"]))
    assert np.array_equal(_np(traj["node"][-1]), ref["node"])
    assert np.array_equal(_np(traj["edge"][-1]), ref["edge"])
    assert np.array_equal(_np(traj["avail"][-1]), ref["avail"])
    assert np.array_equal(_np(traj["obs_window"][-1]), ref["obs_window"])



@pytest.mark.parametrize("name,E,S,N,T,shared", [
    ("c3_full_2048x64_warehouse", 2048, 64, 64, 32, True),
    ("c5_full_1024x256", 1024, 128, 256, 16, False)])
def test_rollout_matches_oracle_full_size(mapfx_mod, name, E, S, N, T, shared):
    """BASELINE C3 and C5 at their full env counts: a fused
    generator-action rollout equals the C oracle's, every env, bit for bit."""
    from oracle import corc
    from mapfx.batch import window_planes
    inst = _instances(mapfx_mod, E, S, N, 0.10, shared, seed=1)
    wkind = "window_occ" if N > 127 else "window"     # what bench.py emits for the config
    b = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                                episode_limit=2000, obs=(wkind,))
    ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], S, S, limit=2000)
    b.reset()
    traj = b.rollout(T, seed=2, t0=0)
    ref = ob.rollout(T, seed=2, t0=0)
    assert np.array_equal(_np(b.pos), ob.pos), name
    assert np.array_equal(_np(b.done), ob.done), name
    assert np.array_equal(_np(b.t), ob.t), name
    assert np.array_equal(_u64(_np(traj["reward"][-1])), _u64(ref["reward"])), name
    assert np.array_equal(_np(traj["node"][-1]), ref["node"]), name
    assert np.array_equal(_np(traj["edge"][-1]), ref["edge"]), name
    assert np.array_equal(_np(traj["avail"][-1]), ref["avail"]), name
    win = traj["obs_window"][-1] if wkind == "window" else window_planes(traj["obs_window_occ"][-1])
    assert np.array_equal(_np(win), ref["obs_window"]), name
    # size-independent: every agent stays in bounds and the window's agent plane
    # counts each agent's own cell (>= 1)
    pos = _np(b.pos)
    assert pos.min() >= 0 and pos.max() < S
    assert (_np(win)[:, :, 1, 2, 2] >= 1).all()


def test_autoreset(mapfx_mod):
    """Envs whose agents are all done restart from init_pos in the fused rollout,
    identically to step + reset(mask)."""
    from mapfx.maps import synthetic_instances
    E, S, N, T, limit = 64, 8, 3, 30, 7
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=6)
    kw = dict(bits=inst["bits"], hw=(S, S), episode_limit=limit, obs=("window",))
    b1 = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], **kw)
    b2 = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], **kw)
    b1.reset()
    b2.reset()
    acts = b2.gen_actions(T, 5)
    traj = b1.rollout(T, actions=acts, autoreset=True)
    resets = 0
    for k in range(T):
        out = b2.step(acts[k])
        assert np.array_equal(_u64(_np(out["reward"])), _u64(_np(traj["reward"][k]))), k
        assert np.array_equal(_np(out["obs_window"]), _np(traj["obs_window"][k])), k
        assert np.array_equal(_np(b2.pos), _np(traj["traj_pos"][k])), k
        term = out["term"].clone()
        resets += int(term.sum())
        if term.any():
            b2.reset(env_mask=term)
    assert resets >= E  # limit 7 over 30 steps: every env resets several times
    assert np.array_equal(_np(b1.pos), _np(b2.pos))
    assert np.array_equal(_np(b1.t), _np(b2.t))
    assert np.array_equal(_np(b1.done), _np(b2.done))


def test_invalid_action_sets_err_and_skips_env(mapfx_mod):
    from mapfx.maps import synthetic_instances
    E, S, N = 8, 8, 4
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=8)
    b = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S))
    b.reset()
    a = torch.full((E, N), 1, dtype=torch.int64, device="cuda")
    a[3, 2] = 7
    pos0 = _np(b.pos).copy()
    b.step(a)
    assert np.array_equal(_np(b.pos)[3], pos0[3]) and int(_np(b.t)[3]) == 0
    assert int(_np(b.t)[0]) == 1
    with pytest.raises(AssertionError):
        b.check_err()
    b.step(torch.full((E, N), 4, dtype=torch.int64, device="cuda"))
    b.check_err()


# ---------------------------------------------------------------------------
# 4. the MAPF_GRID drop-in class (plugin surface) on the golden vectors
# ---------------------------------------------------------------------------
def _write_map_and_scen(tmp_path, grid, n):
    s = grid.shape[0]
    mp = tmp_path / "g.map"
    rows = ["".join("." if v == 0 else "@" for v in row) for row in grid]
    mp.write_text("type octile\nheight %d\nwidth %d\nmap\n" % (s, s) + "\n".join(rows) + "\n")
    prefix = str(tmp_path / "g-random-")
    for k in range(1, 26):
        with open(prefix + "%d.scen" % k, "w") as f:
            f.write("version 1\n")
            for i in range(max(n, 30)):
                f.write("0\tg.map\t%d\t%d\t%d\t%d\t%d\t%d\t0\n" % (s, s, i % s, (i // s) % s,
                                                                 (i * 7) % s, (i * 3) % s))
    return str(mp), prefix


@pytest.mark.parametrize("name", ["c1_empty8_n2", "edge6_scripted", "empty8_int_rewards",
                                  "dense8_n30", "edge6_float_collide"])
def test_dropin_mapf_grid_on_goldens(mapfx_mod, tmp_path, name):
    from mapfx.envs import REGISTRY
    fx = load_fixture(name)
    sr, cr = fixture_rewards(fx)
    n = fx["init_pos"].shape[0]
    mp, prefix = _write_map_and_scen(tmp_path, fx["grid"], n)
    env = REGISTRY["mapf_gridworld"](grid_file_path=mp, agents_path=prefix, n_agents=n,
                                     episode_limit=int(fx["meta_limit"]), step_reward=sr,
                                     collide_reward=cr)
    for a in range(n):   # inject the fixture's scenario, as gen_fixtures.py did
        env._agent_init_pos[a] = tuple(int(v) for v in fx["init_pos"][a])
        env._agent_goal_pos[a] = tuple(int(v) for v in fx["goals"][a])
    env.agent_starts = [env._agent_init_pos[i] for i in range(n)]
    env.agent_goals = [env._agent_goal_pos[i] for i in range(n)]
    obs = env.reset()
    assert obs.shape == (n, fx["occ0"].size) and obs.dtype == np.int64
    assert np.array_equal(obs[0], fx["occ0"].reshape(-1))
    assert env.get_avail_actions() == fx["avail0"].astype(int).tolist()
    info = env.get_env_info()
    assert info["n_actions"] == 5 and info["state_shape"] == fx["occ0"].size
    dones_ref = None
    for t in range(fx["actions"].shape[0]):
        R, dones, inf = env.step(fx["actions"][t].astype(np.int64))
        if dones_ref is None:
            dones_ref = dones
        assert dones is dones_ref is env._agent_dones   # aliased list (quirk 6)
        assert isinstance(R, int) == bool(fx["reward_is_int"][t])
        assert np.float64(R).view(np.uint64) == fx["reward"][t:t + 1].view(np.uint64)[0]
        assert [int(v) for v in dones] == fx["done"][t].tolist()
        assert env.agent_positions == [tuple(p) for p in fx["pos"][t].tolist()]
        assert env.get_avail_actions() == fx["avail"][t].astype(int).tolist()
        assert inf == {"_step_count": int(fx["t"][t])}
        if "occ" in fx:
            assert np.array_equal(env.get_state(), fx["occ"][t].reshape(-1))
            assert np.array_equal(env.get_obs()[n - 1], fx["occ"][t].reshape(-1))
        assert env.episode_done() == bool(fx["done"][t].all())
    with pytest.raises(AssertionError):
        env.step([0] * (n + 1))
    with pytest.raises(AssertionError):
        env.step([5] + [0] * (n - 1))


# ---------------------------------------------------------------------------
# 5. env sharding: shards keyed by global env id
# ---------------------------------------------------------------------------
def test_sharded_batches_equal_full_batch(mapfx_mod):
    """Three env_offset shards of uneven size (as mapfx.dist.shard hands to 3
    ranks) stepped with generator actions equal one unsharded batch, env for env."""
    from mapfx.dist import shard
    from mapfx.maps import synthetic_instances
    E, S, N, T, world = 1000, 32, 16, 40, 3
    full = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=5)
    b = mapfx_mod.MapfGridBatch(full["init_pos"], full["goals"], bits=full["bits"], hw=(S, S),
                                episode_limit=30, obs=("window",))
    b.reset()
    ref = b.rollout(T, seed=9, t0=0, autoreset=True)
    for r in range(world):
        off, cnt = shard(E, r, world)
        inst = synthetic_instances(cnt, S, S, N, p_obstacle=0.1, seed=5, env_offset=off)
        assert np.array_equal(inst["bits"], full["bits"][off:off + cnt])
        bs = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"],
                                     hw=(S, S), episode_limit=30, obs=("window",), env_offset=off)
        bs.reset()
        tr = bs.rollout(T, seed=9, t0=0, autoreset=True)
        for k in ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos",
                  "traj_done", "traj_t"):
            assert np.array_equal(_np(tr[k]), _np(ref[k])[:, off:off + cnt]), (r, k)
        assert np.array_equal(_np(bs.pos), _np(b.pos)[off:off + cnt])


def test_overlapped_gather_single_rank(mapfx_mod):
    """OverlappedGather on a 1-rank RCCL group, read the way a consumer does: each
    chunk's gathered tensors are cloned on the current stream right after
    step_chunk (result() orders the read after the gather with a stream wait, no
    device sync), for 5 chunks through both receive buffers.  Every clone must
    equal a plain rollout of the same chunk."""
    import os
    import socket
    import torch.distributed as dist
    from mapfx.dist import OverlappedGather
    from mapfx.maps import synthetic_instances
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        E, S, N, T = 256, 32, 16, 8
        inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=2)
        mk = lambda: mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"],
                                             hw=(S, S), episode_limit=100, obs=("window",))
        b, bref = mk(), mk()
        b.reset()
        bref.reset()
        og = OverlappedGather(b, T)
        got = []
        for i in range(5):
            og.step_chunk(seed=4, t0=i * T)
            got.append({k: v[0].clone() for k, v in og.result(i).items()})
        ref = [{k: v.clone() for k, v in bref.rollout(T, seed=4, t0=i * T).items()}
               for i in range(5)]
        torch.cuda.synchronize()
        assert og.bytes_per_chunk() % 16 == 0
        for i in range(5):
            for k in og.keys:
                assert torch.equal(got[i][k], ref[i][k]), (i, k)
    finally:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# 7. the drop-in step's host traffic: one packed D2H copy, one synchronisation
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("env_name", ["mapf_gridworld", "marl_partial"])
def test_dropin_step_syncs_once(mapfx_mod, monkeypatch, env_name):
    """A drop-in step waits on the device exactly once (the packed pull) and never
    through an implicit sync (.item() / .cpu() / .tolist() / bool of a tensor)."""
    import os
    import random
    from mapfx.envs import REGISTRY
    scen = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "scen")
    random.seed(1)   # draws empty-8-8-random-19.scen (kept in tests/golden/scen)
    env = REGISTRY[env_name](grid_file_path=os.path.join(scen, "empty-8-8.map"),
                             agents_path=os.path.join(scen, "empty-8-8-random-"), n_agents=4)
    if env_name == "marl_partial":   # reset re-draws: pin the draw to a scen file that is present
        env._MARL_PARTIAL_ENV__setup_agent = lambda: None
    env.reset()
    torch.cuda.synchronize()
    calls = {"sync": 0}
    real_sync = torch.cuda.Stream.synchronize

    def counting_sync(self):
        calls["sync"] += 1
        return real_sync(self)

    def guard(name):
        real = getattr(torch.Tensor, name)

        def f(self, *a, **k):
            if self.is_cuda:
                raise AssertionError("implicit device sync (%s) in a drop-in step" % name)
            return real(self, *a, **k)
        return f

    monkeypatch.setattr(torch.cuda.Stream, "synchronize", counting_sync)
    for name in ("item", "cpu", "tolist", "__bool__"):
        monkeypatch.setattr(torch.Tensor, name, guard(name))
    rs = np.random.RandomState(0)
    for k in range(20):
        env.step(rs.randint(0, 5, size=4).tolist())
        assert calls["sync"] == k + 1
    monkeypatch.undo()


def test_rollout_timed_equals_rollout(mapfx_mod):
    """mapfx_rollout_timed (the bench's timed launch, hipExtLaunchKernel with start /
    stop events) writes exactly what mapfx_rollout writes, and its events time it."""
    from mapfx.maps import synthetic_instances
    E, S, N, T = 512, 32, 16, 20
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=8)
    mk = lambda: mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"],
                                         hw=(S, S), episode_limit=50, obs=("window",),
                                         track_steps=False)
    b1, b2 = mk(), mk()
    b1.reset()
    b2.reset()
    acts = b1.gen_actions(T, seed=3)
    outs = ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos", "traj_done",
            "traj_t")
    t1 = b1.rollout(T, actions=acts, outputs=outs)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    ev[0].record()
    ev[1].record()
    t2 = b2.rollout_plan(T, actions=acts, outputs=outs, events=ev)()
    torch.cuda.synchronize()
    for k in outs:
        assert torch.equal(t1[k], t2[k]), k
    assert torch.equal(b1.pos, b2.pos) and torch.equal(b1.t, b2.t)
    assert ev[0].elapsed_time(ev[1]) > 0.0


@pytest.mark.parametrize("N,win", [(12, 5), (100, 3)])
def test_nonsquare_highway_map(mapfx_mod, tmp_path, N, win):
    """A non-square map in the highway generator's format (mapfx.highway, SURVEY
    §8(f) F4) through the kernels (wave path at N = 12, generic at N = 100) and
    the C oracle, step by step."""
    from mapfx import highway as hw
    from mapfx.maps import synthetic_instances
    from oracle import corc
    H, W = 13, 37
    rows = ["".join("@" if (r % 4 in (1, 2) and c % 6 in (1, 2, 3, 4)) else "ewns"[(r + c) % 4]
                    for c in range(W)) for r in range(H)]
    hw.write_highway_outputs(str(tmp_path), rows, {}, {}, [], {"g_map": rows})
    grid, _ = hw.read_highways(str(tmp_path / "highways.txt"))
    E = 96
    inst = synthetic_instances(E, H, W, N, seed=9, shared_grid=-grid.astype(np.int8))
    b = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(H, W),
                                episode_limit=40, obs=("full", "window"), window=win)
    ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], H, W, limit=40)
    b.reset()
    rs = np.random.RandomState(3)
    for t in range(20):
        a = rs.randint(0, 5, size=(E, N)).astype(np.int8)
        out = b.step(torch.from_numpy(a).cuda())
        rstep = ob.step(a.astype(np.int32))
        ref = ob.observe(window=win)
        assert np.array_equal(_np(b.pos), ob.pos), t
        assert np.array_equal(_u64(_np(out["reward"])), _u64(rstep["reward"])), t
        assert np.array_equal(_np(out["avail"]), ref["avail"]), t
        assert np.array_equal(_np(out["obs_full"]), ref["obs_full"]), t
        assert np.array_equal(_np(out["obs_window"]), ref["obs_window"]), t


def test_edge_shapes(mapfx_mod):
    """Edge shapes the reference admits: an empty shard (E = 0: every call a no-op),
    a 1 x 1 map with one agent (nothing is ever available but stay), window 1, and
    the ABI's maximum N = 1024 (generic kernel, 4 agents per lane) against the C oracle."""
    from mapfx.maps import synthetic_instances
    from oracle import corc
    # E = 0
    b0 = mapfx_mod.MapfGridBatch(np.zeros((0, 3, 2), np.int32), np.zeros((0, 3, 2), np.int32),
                                 grids=np.zeros((4, 4), np.uint8), obs=("full", "window"))
    b0.reset()
    b0.step(torch.zeros((0, 3), dtype=torch.int8, device="cuda"))
    tr = b0.rollout(3, seed=1)
    assert tr["reward"].shape == (3, 0)
    # 1 x 1 map, one agent, window 1
    b1 = mapfx_mod.MapfGridBatch(np.zeros((2, 1, 2), np.int32), np.zeros((2, 1, 2), np.int32),
                                 grids=np.zeros((1, 1), np.uint8), obs=("full", "window"), window=1,
                                 episode_limit=5)
    out = b1.reset()
    assert _np(out["avail"]).tolist() == [[16], [16]]
    assert _np(out["obs_window"]).reshape(2, 2).tolist() == [[0, 1], [0, 1]]
    out = b1.step(torch.tensor([[0], [3]], dtype=torch.int8, device="cuda"))
    assert _np(b1.pos).reshape(2, 2).tolist() == [[0, 0], [0, 0]]
    assert _np(out["term"]).tolist() == [1, 1]          # the start is the goal
    # N = 1024 on 64 x 64
    E, S, N = 3, 64, 1024
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.05, seed=6)
    b = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                                episode_limit=50, obs=("full", "window", "window_occ"), window=5)
    assert b.info()["agents_per_lane"] == 4
    ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], S, S, limit=50)
    b.reset()
    rs = np.random.RandomState(4)
    from mapfx.batch import window_planes
    for t in range(5):
        a = rs.randint(0, 5, size=(E, N)).astype(np.int8)
        out = b.step(torch.from_numpy(a).cuda())
        rstep = ob.step(a.astype(np.int32))
        ref = ob.observe(window=5)
        assert np.array_equal(_np(b.pos), ob.pos), t
        assert np.array_equal(_u64(_np(out["reward"])), _u64(rstep["reward"])), t
        assert np.array_equal(_np(out["edge"]), rstep["edge"]), t
        assert np.array_equal(_np(out["obs_full"]), ref["obs_full"]), t
        assert np.array_equal(_np(out["obs_window"]), ref["obs_window"]), t
        assert np.array_equal(_np(window_planes(out["obs_window_occ"])), ref["obs_window"]), t


@pytest.mark.parametrize("N", [3, 6, 9, 11, 12, 13, 14, 15, 17, 24, 33, 47])
def test_wave_partial_lane_groups(mapfx_mod, N):
    """N below its lane group L = pow2ceil(N) (lanes past N carry no agent): the
    per-step kernel and the fused rollout against the C oracle, E not a multiple of
    the envs per wave.  (N = 9..14 once folded the next env's rewards.)"""
    from mapfx.maps import synthetic_instances
    from oracle import corc
    E, S, T = 51, 12, 8
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=N)
    kw = dict(bits=inst["bits"], hw=(S, S), episode_limit=30, obs=("window",), window=5)
    b = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], **kw)
    ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], S, S, limit=30)
    b.reset()
    acts = b.gen_actions(T, 7)
    traj = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], **kw).rollout(T, actions=acts)
    for t in range(T):
        a = _np(acts[t])
        out = b.step(acts[t])
        rstep = ob.step(a.astype(np.int32))
        ref = ob.observe(window=5)
        for got in (out, {k: v[t] for k, v in traj.items()}):
            assert np.array_equal(_u64(_np(got["reward"])), _u64(rstep["reward"])), (N, t)
            assert np.array_equal(_np(got["node"]), rstep["node"]), (N, t)
            assert np.array_equal(_np(got["edge"]), rstep["edge"]), (N, t)
            assert np.array_equal(_np(got["avail"]), ref["avail"]), (N, t)
            assert np.array_equal(_np(got["obs_window"]), ref["obs_window"]), (N, t)
        assert np.array_equal(_np(b.pos), ob.pos), (N, t)


@pytest.mark.parametrize("N", [256, 300])
def test_stacked_swap_edge_count_exact(mapfx_mod, N):
    """__count_edge_collision (:364-383) counts every stacked agent that swaps
    back: N - 1 agents stacked on one cell move right while the agent on the
    right moves left, so that agent's edge count is N - 1 (255 at N = 256, the
    u8 limit; 299 at N = 300, where `edge` is u16, mapfx_edge_elem_size)."""
    from oracle import corc
    from mapfx.maps import pack_bits
    E, S = 3, 20
    init = np.zeros((E, N, 2), np.int32)
    init[:, :, :] = (5, 5)
    init[:, N - 1] = (5, 6)
    goals = np.zeros((E, N, 2), np.int32)
    goals[:, :, :] = (15, 15)
    bits = pack_bits(np.zeros((1, S, S), np.int8))
    b = mapfx_mod.MapfGridBatch(init, goals, bits=bits, hw=(S, S), obs=("window",), window=5)
    ob = corc.OracleBatch(bits, init, goals, S, S)
    b.reset()
    a = np.full((E, N), 3, np.int8)
    a[:, N - 1] = 2
    a[1, :] = 4                                  # env 1 stays: no collisions
    out = b.step(torch.from_numpy(a).cuda())
    ref = ob.step(a.astype(np.int32))
    edge = _np(out["edge"]).astype(np.int64)
    assert edge[0, N - 1] == N - 1 and (edge[0, :N - 1] == 1).all()
    assert (edge[1] == 0).all()
    assert np.array_equal(edge, ref["edge"].astype(np.int64))
    assert np.array_equal(_u64(_np(out["reward"])), _u64(ref["reward"]))
    assert out["edge"].dtype == (torch.uint8 if N <= 256 else torch.int16)
    # the fused rollout (same kernel body, trajectory slots) agrees
    b2 = mapfx_mod.MapfGridBatch(init, goals, bits=bits, hw=(S, S), obs=("window",), window=5)
    b2.reset()
    traj = b2.rollout(1, actions=torch.from_numpy(a[None]).cuda())
    assert np.array_equal(_np(traj["edge"][0]).astype(np.int64), edge)
    # its reward row comes from the deferred fold's codes (edge >= 4: the arithmetic path)
    assert np.array_equal(_u64(_np(traj["reward"][0])), _u64(_np(out["reward"])))


def test_split64_stacked_swap_edges(mapfx_mod):
    """The store-wave split at 64 agents per env (C3's runner rollout): reward codes are
    u16 there because an edge count reaches N - 1 = 63 (4 bits hold 15).  Two stacks of
    32 agents swap cells in step 0 (edge = 32 for every agent), then random steps; every
    output of every step equals single step launches, and the launch is the split
    instance."""
    from mapfx import _abi
    E, S, N, T = 64, 8, 64, 12
    grid = np.zeros((S, S), np.int8)
    init = np.zeros((E, N, 2), np.int32)
    init[:, :32] = (3, 3)
    init[:, 32:] = (3, 4)
    goals = np.zeros((E, N, 2), np.int32)
    goals[:, :, 0] = 7
    goals[:, :, 1] = np.arange(N) % S
    kw = dict(grids=np.repeat(grid[None], E, 0), episode_limit=2000, obs=("window",), window=5)
    b1 = mapfx_mod.MapfGridBatch(init, goals, **kw)
    b2 = mapfx_mod.MapfGridBatch(init, goals, **kw)
    b1.reset()
    b2.reset()
    acts = b2.gen_actions(T, 41, t0=0)
    acts[0, :, :32] = 3            # right: (3,3) -> (3,4)
    acts[0, :, 32:] = 2            # left:  (3,4) -> (3,3)
    acts[0, 1, :] = 4              # env 1 stays put
    traj = b1.rollout(T, actions=acts)
    assert "mapf_wave_kernel<5, true, true, true, 64, true" in _abi.last_kernel(), _abi.last_kernel()
    for k in range(T):
        out = b2.step(acts[k])
        if k == 0:
            e0 = _np(out["edge"]).astype(np.int64)
            assert (e0[0] == 32).all() and (e0[1] == 0).all()
        for key in ("reward", "reward_f32", "term", "node", "edge", "avail", "obs_window"):
            x, y = _np(out[key]), _np(traj[key][k])
            if x.dtype == np.float64:
                assert np.array_equal(_u64(x), _u64(y)), (key, k)
            else:
                assert np.array_equal(x, y), (key, k)
        assert np.array_equal(_np(traj["traj_pos"][k]), _np(b2.pos)), k
        assert np.array_equal(_np(traj["traj_done"][k]), _np(b2.done)), k
        assert np.array_equal(_np(traj["traj_t"][k]), _np(b2.t)), k
    assert np.array_equal(_np(b1.pos), _np(b2.pos))


def test_rollout_does_not_pin_trajectories(mapfx_mod):
    """rollout() without a caller buffer allocates a fresh trajectory per
    call; the batch must not keep those alive (device memory stays flat)."""
    from mapfx.maps import synthetic_instances
    inst = synthetic_instances(256, 16, 16, 8, p_obstacle=0.1, seed=2)
    b = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(16, 16),
                                obs=("window",), window=5)
    b.reset()
    for _ in range(3):
        b.rollout(8, seed=1)
    torch.cuda.synchronize()
    m0 = torch.cuda.memory_allocated()
    for _ in range(80):
        b.rollout(8, seed=1)
    torch.cuda.synchronize()
    assert torch.cuda.memory_allocated() == m0
    # a caller-owned buffer is still reused through the struct cache
    traj = b._alloc_out(8)
    b.rollout(8, seed=1, traj=traj)
    n = len(b._traj_cache)
    b.rollout(8, seed=1, traj=traj)
    assert len(b._traj_cache) == n


@pytest.mark.parametrize("S,N,E,T,p,obs,runset", [
    (128, 256, 40, 21, 0.10, ("window_occ",), False),  # C5 shape: folds at steps 7, 15, partial ring at 20
    (24, 256, 24, 19, 0.05, ("window_occ",), False),   # dense: stacked agents, edge counts >= 4 (codes >= 32)
    (64, 300, 8, 10, 0.10, ("window_occ",), False),    # APL 2
    # the fold placement after B3 (no window writer to overlap it with): no window
    # outputs at L = 256, and a window at L = 128 with one env per block (the map's LDS)
    (128, 256, 12, 19, 0.10, (), False),
    (128, 256, 12, 19, 0.10, ("full",), False),
    (160, 100, 10, 12, 0.10, ("window_occ",), False),
    # FEAT_RUN: exactly the runner output set, no f32 reward (the C5 bench leg's
    # feature set) at APL 1, 2 and 4, and with the two window planes
    (128, 256, 40, 21, 0.10, ("window_occ",), True),
    (24, 256, 24, 19, 0.05, ("window_occ",), True),
    (64, 300, 8, 10, 0.10, ("window_occ",), True),
    (64, 600, 6, 10, 0.10, ("window_occ",), True),
    (160, 100, 10, 12, 0.10, ("window",), True)])
def test_generic_rollout_every_step(mapfx_mod, S, N, E, T, p, obs, runset):
    """Generic-kernel rollouts (one env per block) fold the rewards from per-agent codes
    every 8 steps; every step's outputs must equal single step launches (per-step fold),
    bit for bit, including an env whose step 9 is skipped for an invalid action.
    runset: the rollout writes exactly the runner output set (FEAT_RUN instance)."""
    from mapfx import _abi
    from mapfx.maps import synthetic_instances
    inst = synthetic_instances(E, S, S, N, p_obstacle=p, seed=17)
    kw = dict(bits=inst["bits"], hw=(S, S), episode_limit=2000, obs=obs, window=5)
    b1 = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], **kw)
    b2 = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], **kw)
    assert b1.info()["envs_per_block"] == 1      # the deferred-fold layout
    b1.reset()
    b2.reset()
    acts = b2.gen_actions(T, 5, t0=0).to(torch.int32)
    acts[9, 2, 0] = 7                            # env 2 skips step 9
    if runset:
        traj = b1._alloc_out(T)
        traj.pop("reward_f32")
        outs = ("reward", "term", "node", "edge", "avail", "obs_" + obs[0], "traj_pos",
                "traj_done", "traj_t")
        traj = b1.rollout(T, actions=acts, traj=traj, outputs=outs)
        apl = b1.info()["agents_per_lane"]
        apl = apl if apl <= 2 else 4          # the instance an APL of 3 or 4 runs (pick_kernel_run)
        name = _abi.last_kernel()
        assert "mapf_rollout_kernel<" in name and ", %d, 4>" % apl in name, (name, apl)
    else:
        traj = b1.rollout(T, actions=acts)
    with pytest.raises(AssertionError):
        b1.check_err()
    max_edge = 0
    for k in range(T):
        out = b2.step(acts[k])
        if k == 9:
            with pytest.raises(AssertionError):
                b2.check_err()
        for key in ("reward", "reward_f32", "term", "node", "edge", "avail", "obs_window_occ",
                    "obs_window", "obs_full"):
            if key not in out or key not in traj:
                continue
            x, y = _np(out[key]), _np(traj[key][k])
            if x.dtype == np.float64:
                assert np.array_equal(_u64(x), _u64(y)), (key, k)
            else:
                assert np.array_equal(x, y), (key, k)
        max_edge = max(max_edge, int(_np(out["edge"]).max()))
        assert np.array_equal(_np(traj["traj_pos"][k]), _np(b2.pos)), k
        assert np.array_equal(_np(traj["traj_t"][k]), _np(b2.t)), k
    assert int(_np(traj["traj_t"][9])[2]) == int(_np(traj["traj_t"][8])[2])
    if S == 24:
        assert max_edge >= 4, max_edge
    assert np.array_equal(_np(b1.steps), _np(b2.steps))


@pytest.mark.parametrize("dtype", [torch.int8, torch.int32, torch.int64])
@pytest.mark.parametrize("T", [1, 3, 4, 5, 13])
def test_generic_rollout_action_blocks(mapfx_mod, dtype, T):
    """The generic rollout reads int8 / int32 actions GAB = 4 steps per block (dword loads,
    rows clamped at T - 1; int64 keeps the one-step load): every launch length around the
    block size, each action dtype, invalid values (7, -1, and 300 / -300 where the dtype
    holds them) in several envs and steps -- every step's outputs equal single step launches
    and the error flag is raised as they raise it."""
    from mapfx.maps import synthetic_instances
    S, N, E = 24, 100, 10                     # N > 64: the generic kernel, one env per block
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=23)
    kw = dict(bits=inst["bits"], hw=(S, S), episode_limit=2000, obs=("window_occ",), window=5)
    b1 = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], **kw)
    b2 = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], **kw)
    b1.reset()
    b2.reset()
    acts = b2.gen_actions(T, 9, t0=0).to(dtype)
    bad = {torch.int8: (7, -1), torch.int32: (7, -1, 300), torch.int64: (7, -1, -300)}[dtype]
    for i, v in enumerate(bad):
        acts[min(T - 1, i + 1), (3 * i + 1) % E, (17 * i) % N] = v
    traj = b1.rollout(T, actions=acts)
    err1 = int(b1.err.item())
    for k in range(T):
        out = b2.step(acts[k])
        for key in ("reward", "term", "node", "edge", "avail", "obs_window_occ"):
            x, y = _np(out[key]), _np(traj[key][k])
            if x.dtype == np.float64:
                assert np.array_equal(_u64(x), _u64(y)), (key, k)
            else:
                assert np.array_equal(x, y), (key, k)
        assert np.array_equal(_np(traj["traj_pos"][k]), _np(b2.pos)), k
        assert np.array_equal(_np(traj["traj_t"][k]), _np(b2.t)), k
    assert err1 != 0 and int(b2.err.item()) != 0
    assert np.array_equal(_np(b1.pos), _np(b2.pos)) and np.array_equal(_np(b1.t), _np(b2.t))


def test_last_kernel_names_the_launched_instance(mapfx_mod):
    """mapfx_last_kernel (ABI 5) names the env kernel each entry point launched, as
    rocprofv3 does: what bench.py records and checks a profile against."""
    from mapfx import _abi
    from mapfx.maps import synthetic_instances
    inst = synthetic_instances(8, 8, 8, 4, p_obstacle=0.1, seed=3)
    b = mapfx_mod.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(8, 8),
                                obs=("window",), window=5)
    b.reset()
    b.step(torch.full((8, 4), 4, dtype=torch.int8, device="cuda"))
    assert _abi.last_kernel().startswith("void (anonymous namespace)::mapf_wave_kernel<5, false"), \
        _abi.last_kernel()
    p = mapfx_mod.MarlPartialBatch(inst["init_pos"], inst["goals"], grids=inst["grid"][:1])
    p.reset()
    p.step(torch.full((8, 4), 4, dtype=torch.int64, device="cuda"))
    assert "partial_kernel<" in _abi.last_kernel(), _abi.last_kernel()
    q = mapfx_mod.PrimalBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(8, 8),
                              observation_size=5)
    q.act(torch.ones((8, 2), dtype=torch.int32, device="cuda"),
          torch.full((8, 2), 4, dtype=torch.int32, device="cuda"))
    assert "primal_" in _abi.last_kernel() and "<" in _abi.last_kernel(), _abi.last_kernel()
    assert _abi.build_id().startswith("src=")
