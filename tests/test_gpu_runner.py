"""GPU test of the batched ParallelRunner (mapfx/runners.py)
against the REFERENCE runner: tests/golden/runner_*.npz were written by
tests/golden/gen_runner_fixtures.py running MARL-curve-main/src/runners/
parallel_runner.py (forked env workers, Pipe protocol) into the reference
components/episode_buffer.py EpisodeBatch with PyMARL's scheme and OneHot actions
preprocess, under the scripted MAC restated below.  Every transition field of
every run (state, obs, avail_actions, actions, actions_onehot, reward,
terminated, filled), t_env and the logged stats must be equal; the fixtures have
envs that terminate early at different steps (the stale not-terminated list)."""
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REWARDS = dict(move_reward=0, stay_reward=-0.1, stay_goal_reward=1, node_collide_reward=-2000,
               edge_collide_reward=-2000, env_collide_reward=-2000, complete_reward=1000,
               complete_fac=1.5, gamma=0.99)
CASES = ["runner_open5_n2", "runner_wall6_n3", "runner_solo4_n1"]


def scripted_action(b, t, n, avail_row):
    """= gen_runner_fixtures.scripted_action"""
    a = (3 * b + 7 * t + 5 * n + (b * t) % 3) % 5
    return a if avail_row[a] else 4


class ScriptedMAC:
    action_selector = types.SimpleNamespace()

    def __init__(self):
        self.bs_lens = []

    def init_hidden(self, batch_size):
        pass

    def select_actions(self, batch, t_ep, t_env, bs=slice(None), test_mode=False):
        avail = batch["avail_actions"][:, t_ep]
        idx = bs.tolist() if isinstance(bs, torch.Tensor) else list(range(avail.shape[0]))[bs]
        av = avail.cpu().numpy()
        n = av.shape[1]
        out = [[scripted_action(b, t_ep, k, av[b, k]) for k in range(n)] for b in idx]
        return torch.tensor(out, dtype=torch.long, device=avail.device).view(len(idx), n)


class Logger:
    def __init__(self):
        self.stats = []

    def log_stat(self, k, v, t):
        self.stats.append((k, float(v), int(t)))


def _make_runner(tmp_path, fx, B, mac, **extra):
    from mapfx.episode import DeviceEpisodeBatch, OneHot
    from mapfx.runners import ParallelRunner
    rows = [str(r) for r in fx["map"]]
    s = len(rows)
    mp = tmp_path / "m.map"
    mp.write_text("type octile\nheight %d\nwidth %d\nmap\n%s\n" % (s, s, "\n".join(rows)))
    N, limit = int(fx["n_agents"]), int(fx["limit"])
    starts, goals = fx["inst_starts"], fx["inst_goals"]   # [episodes, N, 2], one per run

    def instance_fn(ep):
        i = ep % starts.shape[0]
        return np.repeat(starts[i][None], B, 0), np.repeat(goals[i][None], B, 0)

    args = types.SimpleNamespace(
        env="marl_partial", batch_size_run=B, device="cuda",
        env_args=dict(REWARDS, grid_file_path=str(mp), agents_path=str(tmp_path / "x-"),
                      n_agents=N, obs_window=int(fx["obs_window"]),
                      obs_knn_agents=int(fx["obs_knn_agents"]), episode_limit=limit),
        episode_batch_cls=DeviceEpisodeBatch, test_nepisode=B, runner_log_interval=1, **extra)
    logger = Logger()
    runner = ParallelRunner(args, logger, instance_fn=instance_fn)
    info = runner.get_env_info()
    scheme = {"state": {"vshape": info["state_shape"]},
              "obs": {"vshape": info["obs_shape"], "group": "agents"},
              "actions": {"vshape": (1,), "group": "agents", "dtype": torch.long},
              "avail_actions": {"vshape": (info["n_actions"],), "group": "agents", "dtype": torch.int},
              "reward": {"vshape": (1,)}, "terminated": {"vshape": (1,), "dtype": torch.uint8}}
    runner.setup(scheme, {"agents": N}, {"actions": ("actions_onehot", [OneHot(out_dim=5)])}, mac)
    return runner, logger


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("name", CASES)
def test_runner_matches_reference_parallel_runner(tmp_path, name, fused):
    """fused=False: the runner state without bs_inv (a binding that predates ABI 4), so
    mapfx_runner_step takes the separate actions / env step / post kernels instead of
    the fused env step; both must fill the batch exactly as the reference runner.
    Every batch run() returned must still hold its run's rows after the later runs."""
    from conftest import load_fixture
    fx = load_fixture(name)
    runner, logger = _make_runner(tmp_path, fx, int(fx["B"]), ScriptedMAC())
    if not fused:
        runner._rs.bs_inv = None

    def check(r, batch):
        for k, v in batch.data.transition_data.items():
            ref = fx["run%d_%s" % (r, k)]
            got = v.cpu().numpy()
            assert got.shape == ref.shape and got.dtype == ref.dtype, (r, k)
            assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), (r, k)

    batches = []
    for r in range(int(fx["runs"])):
        batch = runner.run(test_mode=False)
        check(r, batch)
        batches.append(batch)
        assert runner.t_env == int(fx["run%d_t_env" % r])
    assert len({b.data.transition_data["obs"].data_ptr() for b in batches}) == len(batches)
    for r, batch in enumerate(batches):
        check(r, batch)
    assert [k for k, _, _ in logger.stats] == fx["log_stats"].tolist()
    assert [v for _, v, _ in logger.stats] == fx["log_values"].tolist()
    assert [t for _, _, t in logger.stats] == fx["log_t"].tolist()


class TiledMAC:
    """ScriptedMAC for a batch that tiles a fixture's B_fx envs: env b acts as
    fixture env b % B_fx (the same scripted_action), vectorised on the device so
    the runner loop stays free of host reads.  Accepts a padded or exact `bs`."""

    action_selector = types.SimpleNamespace()

    def __init__(self, bfx):
        self.bfx = bfx

    def init_hidden(self, batch_size):
        pass

    def select_actions(self, batch, t_ep, t_env, bs, test_mode=False):
        avail = batch["avail_actions"][:, t_ep]                 # [B, N, 5] int32
        bb = bs % self.bfx
        n = torch.arange(avail.shape[1], device=avail.device)
        a = (3 * bb[:, None] + 7 * t_ep + 5 * n[None, :] + ((bb * t_ep) % 3)[:, None]) % 5
        ok = torch.gather(avail[bs], 2, a[..., None]).squeeze(-1) != 0
        return torch.where(ok, a, torch.full_like(a, 4))


@pytest.mark.parametrize("B", [4096, 4100, 1100, 1102])
@pytest.mark.parametrize("name", CASES)
def test_runner_tiled_matches_reference_at_bench_shape(tmp_path, name, B):
    """the runner's multi-wave `bs` compaction (runner.hip, per-thread
    chunks + wave scans, reached only at large B) pinned at the bench's B = 4096 and
    at ragged sizes (1100; 1102, not a multiple of 4; 4100, whose per-thread chunks of
    5 envs leave the last threads empty).  Every env of the batch is the fixture instance and acts
    as fixture env b % B_fx, so env b's rows must equal the REFERENCE runner's rows
    of env b % B_fx byte for byte (envs never interact), every run.  Per-env returns
    and lengths must equal those of the B_fx-env run (itself pinned to the fixture's
    t_env and logged stats), so t_env and the logged stats follow exactly."""
    from conftest import load_fixture
    fx = load_fixture(name)
    bfx = int(fx["B"])
    (tmp_path / "base").mkdir()
    base, _ = _make_runner(tmp_path / "base", fx, bfx, TiledMAC(bfx))
    tiled, logger = _make_runner(tmp_path, fx, B, TiledMAC(bfx))
    src = np.arange(B) % bfx
    t_env = 0
    exp_log = []
    for r in range(int(fx["runs"])):
        base.run(test_mode=False)
        assert base.t_env == int(fx["run%d_t_env" % r])
        blen = base._ep_length.cpu().numpy()
        bret = base._ep_return.cpu().numpy()
        batch = tiled.run(test_mode=False)
        for k, v in batch.data.transition_data.items():
            ref = fx["run%d_%s" % (r, k)][src]
            got = v.cpu().numpy()
            assert got.shape == ref.shape and got.dtype == ref.dtype, (r, k)
            assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), (r, k, B)
        assert np.array_equal(tiled._ep_length.cpu().numpy(), blen[src]), r
        assert np.array_equal(tiled._ep_return.cpu().numpy().view(np.uint64),
                              bret[src].view(np.uint64)), r
        t_env += int(blen[src].sum())
        assert tiled.t_env == t_env
        rets = bret[src].tolist()
        total_len = int(blen[src].sum())
        exp_log += [("return_mean", float(np.mean(rets)), t_env),
                    ("return_std", float(np.std(rets)), t_env),
                    ("_step_count_mean", total_len / B, t_env),
                    ("ep_length_mean", total_len / B, t_env)]
    assert logger.stats == exp_log


def test_runner_exact_bs_mode(tmp_path):
    """args.runner_exact_bs: the MAC gets bs[:len(bs)], rows unchanged."""
    from conftest import load_fixture
    fx = load_fixture("runner_solo4_n1")   # envs terminate at different steps in run 0
    bfx, B = int(fx["B"]), 1100
    seen = []

    class Recording(TiledMAC):
        def select_actions(self, batch, t_ep, t_env, bs, test_mode=False):
            seen.append(int(bs.shape[0]))
            return super().select_actions(batch, t_ep, t_env, bs, test_mode)

    runner, _ = _make_runner(tmp_path, fx, B, Recording(bfx), runner_exact_bs=True)
    batch = runner.run(test_mode=False)
    src = np.arange(B) % bfx
    for k, v in batch.data.transition_data.items():
        assert np.array_equal(v.cpu().numpy().view(np.uint8),
                              fx["run0_%s" % k][src].view(np.uint8)), k
    assert seen[0] == B and min(seen) < B      # shrinks once envs terminate


def test_runner_step_needs_no_host_sync(tmp_path, monkeypatch):
    """Inside run(), between reset and the end-of-run totals, nothing reads a device
    value on the host (no .item() / .tolist() / .cpu() / bool(tensor)); the only
    waits are on the pinned ring's events, two steps old."""
    from mapfx.episode import DeviceEpisodeBatch, OneHot
    from mapfx.maps import synthetic_instances
    from mapfx.runners import ParallelRunner
    S, N, B = 8, 6, 64
    mp = tmp_path / "e.map"
    mp.write_text("type octile\nheight 8\nwidth 8\nmap\n" + "\n".join(["." * 8] * 8) + "\n")
    inst = synthetic_instances(B, S, S, N, p_obstacle=0.0, seed=4)
    args = types.SimpleNamespace(
        env="marl_partial", batch_size_run=B, device="cuda",
        env_args=dict(REWARDS, grid_file_path=str(mp), agents_path=str(tmp_path / "x-"),
                      n_agents=N, episode_limit=30),
        episode_batch_cls=DeviceEpisodeBatch, test_nepisode=B, runner_log_interval=1 << 62)
    runner = ParallelRunner(args, None, instance_fn=lambda ep: (inst["init_pos"], inst["goals"]))
    info = runner.get_env_info()

    class DeviceMAC:
        def init_hidden(self, batch_size):
            pass

        def select_actions(self, batch, t_ep, t_env, bs, test_mode=False):
            av = batch["avail_actions"][bs, t_ep].float()
            return torch.argmax(av * torch.rand(av.shape, device=av.device), dim=-1)

    scheme = {"state": {"vshape": 3}, "obs": {"vshape": info["obs_shape"], "group": "agents"},
              "actions": {"vshape": (1,), "group": "agents", "dtype": torch.long},
              "avail_actions": {"vshape": (5,), "group": "agents", "dtype": torch.int},
              "reward": {"vshape": (1,)}, "terminated": {"vshape": (1,), "dtype": torch.uint8}}
    runner.setup(scheme, {"agents": N}, {"actions": ("actions_onehot", [OneHot(out_dim=5)])},
                 DeviceMAC())
    runner.run()                       # warm: first batch, caches
    state = {"on": False}
    real = {n: getattr(torch.Tensor, n) for n in ("item", "tolist", "cpu", "__bool__")}
    steps_ptr = runner._env_steps.data_ptr()

    def make(n):
        def f(self, *a, **k):
            if n == "item" and self.data_ptr() == steps_ptr:
                state["on"] = False    # the end-of-run totals: the loop is over
            if state["on"] and self.is_cuda:
                raise AssertionError("%s() of a device tensor inside the runner loop" % n)
            return real[n](self, *a, **k)
        return f

    for n in real:
        monkeypatch.setattr(torch.Tensor, n, make(n))
    real_step = runner.env.step

    def step(a):
        state["on"] = True
        return real_step(a)

    monkeypatch.setattr(runner.env, "step", step)
    t_env0 = runner.t_env
    runner.run()
    monkeypatch.undo()
    assert 0 < runner.t_env - t_env0 <= B * 30
