"""Batched, device-resident ParallelRunner.

Same public surface as MARL-curve-main/src/runners/parallel_runner.py
(`ParallelRunner.__init__(args, logger)`, `setup(scheme, groups, preprocess, mac)`,
`get_env_info`, `reset`, `run(test_mode)`, `close_env`, `save_replay`, the
`t_env` counter and the return / stat logging), but the `batch_size_run` envs are
one MarlPartialBatch on the GPU instead of one subprocess + Pipe each: no
pickling, no numpy round trip, and `batch.update` receives device tensors.

The EpisodeBatch the runner fills is whatever `setup` is given (PyMARL passes
`components.episode_buffer.EpisodeBatch`); the runner only calls its constructor
and `update(data, bs, ts, mark_filled)` exactly as the reference runner does
(parallel_runner.py:62-76 reset, :91-173 run).

Per-env instances: every reset draws each env's scenario like
MARL_PARTIAL_ENV.__setup_agent (:896-920: random.randint(1, 25) then
random.sample of the scen lines), from a per-env `random.Random(seed + e)`
stream (the reference's forked workers would all share one stream).
"""
from __future__ import annotations

import os
import random
from functools import partial

import numpy as np
import torch

from .maps import load_map
from .partial import MarlPartialBatch


def _scen_draw(rng, agents_path, n):
    """:896-920 with an explicit Random: (starts, goals) as (row, col)."""
    path = agents_path + str(rng.randint(1, 25)) + ".scen"
    assert os.path.exists(path)
    with open(path) as f:
        lines = [row.rstrip() for row in f.readlines()][1:]
    assert len(lines) > n
    starts, goals = [], []
    for line in rng.sample(lines, n):
        v = line.replace("\t", ",").split(",")
        starts.append((int(v[5]), int(v[4])))
        goals.append((int(v[7]), int(v[6])))
    return starts, goals


class ParallelRunner:
    """runners/parallel_runner.py:9-226 over one batched GPU env."""

    def __init__(self, args, logger, instance_fn=None):
        self.args = args
        self.logger = logger
        self.batch_size = int(args.batch_size_run)
        if args.env != "marl_partial":
            raise ValueError("the batched runner drives the marl_partial env (got %r)" % args.env)
        ea = dict(args.env_args)
        self.n_agents = int(ea.pop("n_agents", 4))
        grid_path, self.agents_path = ea.pop("grid_file_path"), ea.pop("agents_path")
        for k in ("seed", "render", "debug", "visual", "output"):
            ea.pop(k, None)
        self.device = torch.device(getattr(args, "device", "cuda"))
        self.grid = load_map(grid_path)
        seed = int(getattr(args, "seed", 0) or 0)
        self._rngs = [random.Random(seed + e) for e in range(self.batch_size)]
        # instance_fn(env_index) -> (starts, goals) overrides the scen draw (tests)
        self._instance_fn = instance_fn
        starts, goals = self._draw()
        self.env = MarlPartialBatch(starts, goals, grids=self.grid[None], device=self.device, **ea)
        self.env_info = {"state_shape": 3, "obs_shape": self.env.obs_dim, "n_actions": 5,
                         "n_agents": self.n_agents, "episode_limit": self.env.episode_limit}
        self.episode_limit = self.env_info["episode_limit"]
        self.t = 0
        self.t_env = 0
        self.train_returns = []
        self.test_returns = []
        self.train_stats = {}
        self.test_stats = {}
        self.log_train_stats_t = -100000

    def _draw(self):
        st, gl = [], []
        for e in range(self.batch_size):
            s, g = (self._instance_fn(e) if self._instance_fn else
                    _scen_draw(self._rngs[e], self.agents_path, self.n_agents))
            st.append(s)
            gl.append(g)
        return np.array(st, dtype=np.int32), np.array(gl, dtype=np.int32)

    def setup(self, scheme, groups, preprocess, mac):
        device = getattr(self.args, "device", "cuda")
        self.new_batch = partial(self._batch_cls(), scheme, groups, self.batch_size,
                                 self.episode_limit + 1, preprocess=preprocess, device=device)
        self.mac = mac
        self.scheme = scheme
        self.groups = groups
        self.preprocess = preprocess

    def _batch_cls(self):
        cls = getattr(self.args, "episode_batch_cls", None)
        if cls is None:
            from components.episode_buffer import EpisodeBatch  # PyMARL's, when run inside it
            cls = EpisodeBatch
        return cls

    def get_env_info(self):
        return self.env_info

    def save_replay(self):
        pass

    def close_env(self):
        pass

    def _pre_transition(self, bs=None):
        o = self.env.out
        sel = (lambda x: x) if bs is None else (lambda x: x[bs])
        return {"state": sel(o["state"]), "avail_actions": sel(self.env.avail_actions()),
                "obs": sel(o["obs"])}

    def reset(self):
        """:62-76: new batch, every env reset (instances re-drawn, :130), t = 0 data."""
        self.batch = self.new_batch()
        starts, goals = self._draw()
        self.env.set_agents(starts, goals)
        self.env.reset()
        self.batch.update(self._pre_transition(), ts=0)
        self.t = 0
        self.env_steps_this_run = 0

    def run(self, test_mode=False):
        """:78-206 with the envs stepped as one batch on the device."""
        self.reset()
        B, N = self.batch_size, self.n_agents
        dev = self.device
        episode_returns = torch.zeros(B, dtype=torch.float64, device=dev)
        episode_lengths = torch.zeros(B, dtype=torch.int64, device=dev)
        self.mac.init_hidden(batch_size=B)
        terminated = torch.zeros(B, dtype=torch.bool, device=dev)
        envs_not_terminated = list(range(B))
        full_actions = torch.full((B, N), 4, dtype=torch.int64, device=dev)
        while True:
            actions = self.mac.select_actions(self.batch, t_ep=self.t, t_env=self.t_env,
                                              bs=envs_not_terminated, test_mode=test_mode)
            self.batch.update({"actions": actions.unsqueeze(1)}, bs=envs_not_terminated, ts=self.t,
                              mark_filled=False)
            # actions reach the envs of the list that have not terminated (:116-121); the
            # list itself is refreshed only afterwards (:123), as in the reference
            sel = torch.as_tensor(envs_not_terminated, dtype=torch.int64, device=dev)
            full_actions.fill_(4)  # envs that are not stepped take "stay" (rows never written)
            if len(envs_not_terminated):
                full_actions[sel] = actions.to(dev).view(-1, N).to(torch.int64)
            bs_idx = torch.nonzero(~terminated).flatten()
            envs_not_terminated = bs_idx.tolist()
            if bool(terminated.all()):
                break
            out = self.env.step(full_actions)
            reward = out["reward"][bs_idx]
            term_now = self.env.terminated[bs_idx].bool()
            episode_returns[bs_idx] += reward
            episode_lengths[bs_idx] += 1
            if not test_mode:
                self.env_steps_this_run += len(envs_not_terminated)
            # env_terminated = terminated and not info["episode_limit"] (:147-150);
            # MARL_PARTIAL's info carries no "episode_limit" key
            self.batch.update({"reward": reward.unsqueeze(1),
                               "terminated": term_now.unsqueeze(1)},
                              bs=envs_not_terminated, ts=self.t, mark_filled=False)
            terminated[bs_idx] = term_now
            self.t += 1
            self.batch.update(self._pre_transition(bs_idx), bs=envs_not_terminated, ts=self.t,
                              mark_filled=True)
        if not test_mode:
            self.t_env += self.env_steps_this_run
        cur_stats = self.test_stats if test_mode else self.train_stats
        cur_returns = self.test_returns if test_mode else self.train_returns
        log_prefix = "test_" if test_mode else ""
        cur_stats["n_episodes"] = B + cur_stats.get("n_episodes", 0)
        cur_stats["ep_length"] = int(episode_lengths.sum().item()) + cur_stats.get("ep_length", 0)
        cur_returns.extend(episode_returns.cpu().tolist())
        n_test_runs = max(1, getattr(self.args, "test_nepisode", B) // B) * B
        if test_mode and (len(self.test_returns) == n_test_runs):
            self._log(cur_returns, cur_stats, log_prefix)
        elif self.t_env - self.log_train_stats_t >= getattr(self.args, "runner_log_interval", 1 << 62):
            self._log(cur_returns, cur_stats, log_prefix)
            sel = getattr(self.mac, "action_selector", None)
            if self.logger is not None and hasattr(sel, "epsilon"):
                self.logger.log_stat("epsilon", sel.epsilon, self.t_env)
            self.log_train_stats_t = self.t_env
        return self.batch

    def _log(self, returns, stats, prefix):
        if self.logger is not None:
            self.logger.log_stat(prefix + "return_mean", np.mean(returns), self.t_env)
            self.logger.log_stat(prefix + "return_std", np.std(returns), self.t_env)
        returns.clear()
        for k, v in stats.items():
            if k != "n_episodes" and self.logger is not None:
                self.logger.log_stat(prefix + k + "_mean", v / stats["n_episodes"], self.t_env)
        stats.clear()
