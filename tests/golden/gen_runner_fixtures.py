#!/usr/bin/env python3
"""Pin the batched runner by RUNNING THE REFERENCE ParallelRunner (build container only).

Drives MARL-curve-main/src/runners/parallel_runner.py (ParallelRunner: one
MARL_PARTIAL_ENV per forked worker process, Pipe protocol, :62-206) filling the
reference's own components/episode_buffer.py EpisodeBatch (with PyMARL's
standard scheme and the OneHot actions preprocess, components/transforms.py),
under a scripted deterministic MAC, and records every field of the returned
batches plus t_env / returns / stats.

Two things are supplied from outside the reference, both recorded here:
  * the envs are a subclass of the reference MARL_PARTIAL_ENV whose
    __setup_agent (:902-929) takes the episode's starts / goals from a fixed
    list instead of a scen file (every forked worker inherits the same `random`
    state, so in the reference all workers draw the same instance anyway), and
    which defines get_stats() -> {} (neither MARL_PARTIAL_ENV nor MultiAgentEnv
    has it, so the reference runner's ("get_stats") request at :179-185 would kill
    the worker: that is a reference bug, outside the path being pinned);
  * the MAC: actions are a fixed function of (env index, t_ep, agent), replaced by
    "stay" where the batch's avail_actions row forbids them.

Usage:  python tests/golden/gen_runner_fixtures.py   (writes tests/golden/runner_*.npz)
"""
from __future__ import annotations

import contextlib
import io
import os
import sys
import types
from functools import partial

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_fixtures as gf  # noqa: E402  (stubs + reference envs on sys.path)

import torch  # noqa: E402

# a scripted, deterministic MAC: action of agent n of env b at t
def scripted_action(b, t, n, avail_row):
    a = (3 * b + 7 * t + 5 * n + (b * t) % 3) % 5
    return a if avail_row[a] else 4


class ScriptedMAC:
    action_selector = types.SimpleNamespace()   # no epsilon (parallel_runner.py:202)

    def init_hidden(self, batch_size):
        pass

    def select_actions(self, batch, t_ep, t_env, bs=slice(None), test_mode=False):
        avail = batch["avail_actions"][:, t_ep]
        if isinstance(bs, slice):
            idx = list(range(avail.shape[0]))[bs]
        elif isinstance(bs, torch.Tensor):
            idx = bs.tolist()
        else:
            idx = list(bs)
        av = avail.cpu().numpy()
        n_agents = av.shape[1]
        out = [[scripted_action(b, t_ep, n, av[b, n]) for n in range(n_agents)] for b in idx]
        return torch.tensor(out, dtype=torch.long, device=avail.device).view(len(idx), n_agents)


CASES = {
    # name: (map rows, n_agents, episode_limit, batch_size_run, runs, yaml-style rewards, instances)
    "runner_open5_n2": dict(
        grid=[".....", ".....", ".....", ".....", "....."], n=2, limit=9, B=6, runs=2,
        inst=[([(0, 0), (4, 4)], [(0, 1), (4, 3)]), ([(2, 2), (0, 4)], [(2, 3), (1, 4)])]),
    "runner_wall6_n3": dict(
        grid=["......", ".@@...", "......", "...@..", "......", "......"], n=3, limit=7, B=5, runs=2,
        inst=[([(0, 0), (5, 5), (2, 2)], [(0, 1), (5, 4), (2, 3)]),
              ([(3, 0), (0, 5), (5, 2)], [(3, 1), (1, 5), (5, 3)])]),
    # one agent: an env completes whenever its agent stands on the goal -> early
    # terminations at different t across the batch (the stale-list path)
    "runner_solo4_n1": dict(
        grid=["....", "....", ".@..", "...."], n=1, limit=8, B=8, runs=2,
        inst=[([(1, 1)], [(1, 2)]), ([(3, 3)], [(2, 3)])]),
}
REWARDS = dict(move_reward=0, stay_reward=-0.1, stay_goal_reward=1, node_collide_reward=-2000,
               edge_collide_reward=-2000, env_collide_reward=-2000, complete_reward=1000,
               complete_fac=1.5, gamma=0.99)


def make_env_cls(instances):
    Base = gf.MP.MARL_PARTIAL_ENV

    class FixtureEnv(Base):
        _episode = -1

        def _MARL_PARTIAL_ENV__setup_agent(self):
            FixtureEnv._episode += 1      # per process: each worker counts its own resets
            starts, goals = instances[max(FixtureEnv._episode - 1, 0) % len(instances)]
            for a in range(self._n_agents):
                self._agent_init_pos[a] = tuple(starts[a])
                self._agent_goal_pos[a] = tuple(goals[a])
            self._MARL_PARTIAL_ENV__setup_agent_goal_dist()

        def get_stats(self):
            return {}

    return FixtureEnv


class _Logger:
    def __init__(self):
        self.stats = []

    def log_stat(self, k, v, t):
        self.stats.append((k, float(v), int(t)))


def run_case(name, c, tmpdir):
    import runners.parallel_runner as PR
    from components.episode_buffer import EpisodeBatch
    from components.transforms import OneHot
    s = len(c["grid"])
    mp = os.path.join(tmpdir, name + ".map")
    with open(mp, "w") as f:
        f.write("type octile\nheight %d\nwidth %d\nmap\n%s\n" % (s, s, "\n".join(c["grid"])))
    env_cls = make_env_cls(c["inst"])
    PR.env_REGISTRY["fixture_partial"] = partial(lambda env, **kw: env(**kw), env=env_cls)
    env_args = dict(REWARDS, grid_file_path=mp, agents_path=os.path.join(tmpdir, "unused-"),
                    n_agents=c["n"], obs_window=3, obs_knn_agents=2, episode_limit=c["limit"])
    args = types.SimpleNamespace(batch_size_run=c["B"], env="fixture_partial", env_args=env_args,
                                 device="cpu", test_nepisode=c["B"], runner_log_interval=1)
    logger = _Logger()
    with contextlib.redirect_stdout(io.StringIO()):
        runner = PR.ParallelRunner(args, logger)
    info = runner.get_env_info()
    scheme = {"state": {"vshape": info["state_shape"]},
              "obs": {"vshape": info["obs_shape"], "group": "agents"},
              "actions": {"vshape": (1,), "group": "agents", "dtype": torch.long},
              "avail_actions": {"vshape": (info["n_actions"],), "group": "agents", "dtype": torch.int},
              "reward": {"vshape": (1,)},
              "terminated": {"vshape": (1,), "dtype": torch.uint8}}
    groups = {"agents": info["n_agents"]}
    preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=info["n_actions"])])}
    runner.setup(scheme, groups, preprocess, ScriptedMAC())
    rec = {"map": np.array(c["grid"]), "n_agents": c["n"], "limit": c["limit"], "B": c["B"],
           "runs": c["runs"], "obs_window": 3, "obs_knn_agents": 2,
           "inst_starts": np.array([i[0] for i in c["inst"]], np.int32),
           "inst_goals": np.array([i[1] for i in c["inst"]], np.int32)}
    for r in range(c["runs"]):
        with contextlib.redirect_stdout(io.StringIO()):
            batch = runner.run(test_mode=False)
        for k, v in batch.data.transition_data.items():
            rec["run%d_%s" % (r, k)] = v.cpu().numpy()
        rec["run%d_t_env" % r] = runner.t_env
    rec["log_stats"] = np.array([k for k, _, _ in logger.stats])
    rec["log_values"] = np.array([v for _, v, _ in logger.stats], np.float64)
    rec["log_t"] = np.array([t for _, _, t in logger.stats], np.int64)
    runner.close_env()
    for p in runner.ps:
        p.join(timeout=10)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **rec)
    filled = [rec["run%d_filled" % r][..., 0].sum(1).tolist() for r in range(c["runs"])]
    print(name, "filled steps per env:", filled, "t_env:", [rec["run%d_t_env" % r] for r in range(c["runs"])])


def main():
    import tempfile
    sys.path.insert(0, gf.REF_SRC)
    tmp = tempfile.mkdtemp(prefix="mapf_runner_fx_")
    for name, c in CASES.items():
        run_case(name, c, tmp)


if __name__ == "__main__":
    main()
