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


@pytest.mark.parametrize("name", CASES)
def test_runner_matches_reference_parallel_runner(tmp_path, name):
    from conftest import load_fixture
    from mapfx.episode import DeviceEpisodeBatch, OneHot
    from mapfx.runners import ParallelRunner
    fx = load_fixture(name)
    rows = [str(r) for r in fx["map"]]
    s = len(rows)
    mp = tmp_path / "m.map"
    mp.write_text("type octile\nheight %d\nwidth %d\nmap\n%s\n" % (s, s, "\n".join(rows)))
    B, N, limit = int(fx["B"]), int(fx["n_agents"]), int(fx["limit"])
    starts, goals = fx["inst_starts"], fx["inst_goals"]   # [episodes, N, 2], one per run

    def instance_fn(ep):
        i = ep % starts.shape[0]
        return np.repeat(starts[i][None], B, 0), np.repeat(goals[i][None], B, 0)

    args = types.SimpleNamespace(
        env="marl_partial", batch_size_run=B, device="cuda",
        env_args=dict(REWARDS, grid_file_path=str(mp), agents_path=str(tmp_path / "x-"),
                      n_agents=N, obs_window=int(fx["obs_window"]),
                      obs_knn_agents=int(fx["obs_knn_agents"]), episode_limit=limit),
        episode_batch_cls=DeviceEpisodeBatch, test_nepisode=B, runner_log_interval=1)
    logger = Logger()
    runner = ParallelRunner(args, logger, instance_fn=instance_fn)
    info = runner.get_env_info()
    scheme = {"state": {"vshape": info["state_shape"]},
              "obs": {"vshape": info["obs_shape"], "group": "agents"},
              "actions": {"vshape": (1,), "group": "agents", "dtype": torch.long},
              "avail_actions": {"vshape": (info["n_actions"],), "group": "agents", "dtype": torch.int},
              "reward": {"vshape": (1,)}, "terminated": {"vshape": (1,), "dtype": torch.uint8}}
    runner.setup(scheme, {"agents": N}, {"actions": ("actions_onehot", [OneHot(out_dim=5)])},
                 ScriptedMAC())
    for r in range(int(fx["runs"])):
        batch = runner.run(test_mode=False)
        for k, v in batch.data.transition_data.items():
            ref = fx["run%d_%s" % (r, k)]
            got = v.cpu().numpy()
            assert got.shape == ref.shape and got.dtype == ref.dtype, (r, k)
            assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), (r, k)
        assert runner.t_env == int(fx["run%d_t_env" % r])
    assert [k for k, _, _ in logger.stats] == fx["log_stats"].tolist()
    assert [v for _, v, _ in logger.stats] == fx["log_values"].tolist()
    assert [t for _, _, t in logger.stats] == fx["log_t"].tolist()


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
