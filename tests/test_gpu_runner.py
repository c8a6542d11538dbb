"""GPU test of the batched ParallelRunner (mapfx/runners.py)
against the reference runner's semantics (runners/parallel_runner.py:62-173)
replayed on the CPU restatement of MARL_PARTIAL_ENV (oracle/partial_oracle.py):
every EpisodeBatch field (state, obs, avail_actions, actions, reward, terminated,
filled) equal, with some envs terminating early (completion) to exercise the
runner's not-terminated bookkeeping."""
import types

import numpy as np
import pytest
import torch

from mapfx.episode import DeviceEpisodeBatch

pytestmark = pytest.mark.gpu

YAML = dict(obs_window=5, obs_knn_agents=5, episode_limit=20, move_reward=0, stay_reward=-0.1,
            stay_goal_reward=1, node_collide_reward=-2000, edge_collide_reward=-2000,
            env_collide_reward=-2000, complete_reward=1000, complete_fac=1.5, gamma=0.99)


class ScriptedMAC:
    """select_actions(batch, t_ep, t_env, bs, test_mode) from a fixed table; envs with
    index % 4 == 0 always stay (they start on their goals and complete at t = 1)."""

    def __init__(self, table):
        self.table = table  # [T, B, N] int64 (device)
        self.calls = []

    def init_hidden(self, batch_size):
        pass

    def select_actions(self, batch, t_ep, t_env, bs, test_mode=False):
        self.calls.append(list(bs))
        return self.table[t_ep][torch.as_tensor(bs, dtype=torch.long, device=self.table.device)]


def _instances(B, S, N, seed=5):
    rng = np.random.default_rng(seed)
    cells = [(r, c) for r in range(S) for c in range(S)]
    out = []
    for e in range(B):
        pick = rng.choice(len(cells), size=2 * N, replace=False)
        st = [cells[i] for i in pick[:N]]
        gl = list(st) if e % 4 == 0 else [cells[i] for i in pick[N:]]
        out.append((st, gl))
    return out


def _reference_run(inst, table, S, N, T1):
    """The reference runner loop (:62-173) over the CPU restatement."""
    from oracle.partial_oracle import PartialEnvState
    B = len(inst)
    grid = np.zeros((S, S), dtype=np.int8)
    envs = [PartialEnvState(grid, s, g, **YAML) for s, g in inst]
    D = envs[0].obs().shape[1]
    buf = {"state": np.zeros((B, T1, 3), np.float32), "obs": np.zeros((B, T1, N, D), np.float32),
           "avail_actions": np.zeros((B, T1, N, 5), np.int32),
           "actions": np.zeros((B, T1, N, 1), np.int64), "reward": np.zeros((B, T1, 1), np.float32),
           "terminated": np.zeros((B, T1, 1), np.uint8), "filled": np.zeros((B, T1, 1), np.int64)}
    for e, env in enumerate(envs):
        buf["state"][e, 0] = env.state()
        buf["obs"][e, 0] = env.obs()
        buf["avail_actions"][e, 0] = env.avail()
        buf["filled"][e, 0] = 1
    terminated = [False] * B
    not_term = list(range(B))
    t = 0
    while True:
        for b in not_term:
            buf["actions"][b, t, :, 0] = table[t, b]
        stepping = [b for b in not_term if not terminated[b]]
        not_term = [b for b in range(B) if not terminated[b]]
        if all(terminated):
            break
        for b in stepping:
            r, term = envs[b].step(table[t, b])
            buf["reward"][b, t, 0] = np.float32(r)
            buf["terminated"][b, t, 0] = term
            terminated[b] = term
        t += 1
        for b in not_term:
            buf["state"][b, t] = envs[b].state()
            buf["obs"][b, t] = envs[b].obs()
            buf["avail_actions"][b, t] = envs[b].avail()
            buf["filled"][b, t] = 1
    return buf


def test_runner_matches_reference_runner_semantics(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mapfx.runners import ParallelRunner
    S, N, B = 8, 6, 16
    mp = tmp_path / "e.map"
    mp.write_text("type octile\nheight 8\nwidth 8\nmap\n" + "\n".join(["." * 8] * 8) + "\n")
    inst = _instances(B, S, N)
    args = types.SimpleNamespace(env="marl_partial", batch_size_run=B, device="cuda",
                                 env_args=dict(grid_file_path=str(mp), agents_path=str(tmp_path / "x-"),
                                               n_agents=N, **YAML),
                                 episode_batch_cls=DeviceEpisodeBatch, test_nepisode=B,
                                 runner_log_interval=10 ** 9)
    runner = ParallelRunner(args, None, instance_fn=lambda e: inst[e])
    info = runner.get_env_info()
    T1 = info["episode_limit"] + 1
    rng = np.random.default_rng(9)
    table = rng.integers(0, 5, size=(T1, B, N))
    table[:, ::4, :] = 4
    scheme = {"state": {"vshape": info["state_shape"]}, "obs": {"vshape": info["obs_shape"], "group": "agents"},
              "actions": {"vshape": (1,), "group": "agents", "dtype": torch.long},
              "avail_actions": {"vshape": (info["n_actions"],), "group": "agents", "dtype": torch.int},
              "reward": {"vshape": (1,)}, "terminated": {"vshape": (1,), "dtype": torch.uint8}}
    mac = ScriptedMAC(torch.as_tensor(table, device="cuda"))
    runner.setup(scheme, {"agents": N}, None, mac)
    batch = runner.run(test_mode=False)
    ref = _reference_run(inst, table, S, N, T1)
    for k in ("state", "obs", "avail_actions", "actions", "reward", "terminated", "filled"):
        got = batch.data.transition_data[k].cpu().numpy()
        assert np.array_equal(got, ref[k].astype(got.dtype)), k
    assert runner.t_env == int(ref["filled"].sum() - B)
    # envs 0, 4, 8, 12 complete at t = 1; the others run to the episode limit
    assert mac.calls[1] == list(range(B)) and 0 not in mac.calls[2]
