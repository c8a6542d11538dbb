"""Batched, device-resident ParallelRunner.

Same public surface as MARL-curve-main/src/runners/parallel_runner.py
(`ParallelRunner.__init__(args, logger)`, `setup(scheme, groups, preprocess, mac)`,
`get_env_info`, `reset`, `run(test_mode)`, `close_env`, `save_replay`, the
`t_env` counter and the return / stat logging), but the `batch_size_run` envs are
one MarlPartialBatch on the GPU instead of one subprocess + Pipe each, and a
runner step is: the MAC's select_actions, then three device launches
(include/mapfx_runner.h) -- actions rows, the env step, the step's rows straight
into the EpisodeBatch tensors with the runner's bookkeeping (running envs, the
MAC's `bs`, returns, lengths, env steps) kept on the device.  No per-step host
synchronisation: the loop-exit test reads the count of running envs from a pinned
ring, written by the step two launches back (the reference stops one MAC call after
the last env terminated; the calls the lag adds find no running env and record
nothing; see `run`).

The EpisodeBatch is whatever `setup` is given (PyMARL passes
components.episode_buffer.EpisodeBatch); the runner writes its
`data.transition_data` tensors (PyMARL's scheme: obs / state float32,
avail_actions int32, actions int64 (+ actions_onehot float32 from the OneHot
preprocess), reward float32, terminated uint8, filled int64) on the batch's device.

Row semantics are the reference's (tests/golden/runner_*.npz were produced by the
reference ParallelRunner itself), including its stale list: the MAC's `bs` and the
actions row at step t cover the envs that were running before step t - 1.  The
MAC gets `bs` as a device LongTensor of length B (ascending running env ids,
padded with the first one), a form the reference EpisodeBatch / BasicMAC index
with (episode_buffer.py:186-190); `args.runner_exact_bs` passes the exact-length
list instead (one host sync per step, for stochastic action selectors whose RNG
consumption must follow the reference's).

Per-env instances: every reset draws each env's scenario like
MARL_PARTIAL_ENV.__setup_agent (:896-920: random.randint(1, 25) then
random.sample of the scen lines), from a per-env `random.Random(seed + e)` stream
(the reference's forked workers all share one stream and draw identical instances).
`instance_fn(episode) -> (starts [B, N, 2], goals [B, N, 2])` overrides the draw.
"""
from __future__ import annotations

import ctypes
import os
import random
from functools import partial

import numpy as np
import torch

from . import _abi
from ._abi import MAPFX_I8, MAPFX_I32, MAPFX_I64, check, lib, ptr
from .maps import load_map
from .partial import MarlPartialBatch

_ADT = {torch.int8: MAPFX_I8, torch.int32: MAPFX_I32, torch.int64: MAPFX_I64}
_ROW_DTYPES = {"obs": torch.float32, "state": torch.float32, "avail_actions": torch.int32,
               "actions": torch.int64, "actions_onehot": torch.float32, "reward": torch.float32,
               "terminated": torch.uint8, "filled": torch.int64}
_ROW_FIELDS = {"obs": "obs", "state": "state", "avail_actions": "avail", "actions": "actions",
               "actions_onehot": "onehot", "reward": "reward", "terminated": "terminated",
               "filled": "filled"}
_RING = 4


_SCEN_CACHE = {}


def _scen_lines(path):
    lines = _SCEN_CACHE.get(path)
    if lines is None:
        assert os.path.exists(path)
        with open(path) as f:
            lines = _SCEN_CACHE[path] = [row.rstrip() for row in f.readlines()][1:]
    return lines


def _scen_draw(rng, agents_path, n):
    """:896-920 with an explicit Random: (starts, goals) as (row, col)."""
    lines = _scen_lines(agents_path + str(rng.randint(1, 25)) + ".scen")
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
        dev = torch.device(getattr(args, "device", "cuda"))
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.grid = load_map(grid_path)
        seed = int(getattr(args, "seed", 0) or 0)
        self._rngs = [random.Random(seed + e) for e in range(self.batch_size)]
        self._instance_fn = instance_fn
        self._episode = 0
        starts, goals = self._draw()
        self.env = MarlPartialBatch(starts, goals, grids=self.grid[None], device=self.device, **ea)
        self._loaded = (starts.tobytes(), goals.tobytes())
        self.env_info = {"state_shape": 3, "obs_shape": self.env.obs_dim, "n_actions": 5,
                         "n_agents": self.n_agents, "episode_limit": self.env.episode_limit}
        self.episode_limit = self.env_info["episode_limit"]
        B, N, dev = self.batch_size, self.n_agents, self.device
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=dev)  # noqa: E731
        self._alive, self._alive_prev = z((B,), torch.uint8), z((B,), torch.uint8)
        self._bs = z((B,), torch.int64)
        self._counts = z((2,), torch.int32)
        self._ep_return, self._ep_length = z((B,), torch.float64), z((B,), torch.int64)
        self._env_steps = z((1,), torch.int64)
        self._env_actions = torch.full((B, N), 4, dtype=torch.int8, device=dev)
        # row of env b in bs (-1: not in it): the fused step reads b's actions there;
        # two halves by step parity (the compaction inside step k writes step k + 1's)
        self._bs_inv = torch.full((2, B), -1, dtype=torch.int32, device=dev)
        self._rs = _abi.RState(B=B, N=N, D=self.env.obs_dim, alive=ptr(self._alive),
                               alive_prev=ptr(self._alive_prev), bs=ptr(self._bs),
                               counts=ptr(self._counts), ep_return=ptr(self._ep_return),
                               ep_length=ptr(self._ep_length), env_steps=ptr(self._env_steps),
                               env_actions=ptr(self._env_actions), bs_inv=ptr(self._bs_inv))
        # counts {len(bs), running} of step k land in slot k % _RING of a mapped host
        # buffer, written by the compaction kernel itself (no copy launch); the slot's
        # event marks them final
        hp, dp = ctypes.c_void_p(), ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.mapfx_host_ring_alloc(2 * _RING, ctypes.byref(hp), ctypes.byref(dp)),
                  "mapfx_host_ring_alloc")
        self._ring_host = hp
        host = np.ctypeslib.as_array(ctypes.cast(hp, ctypes.POINTER(ctypes.c_int32)),
                                     shape=(_RING, 2))
        self._ring = [(torch.cuda.Event(), host[i], dp.value + 8 * i) for i in range(_RING)]
        self.t = 0
        self.t_env = 0
        self.train_returns = []
        self.test_returns = []
        self.train_stats = {}
        self.test_stats = {}
        self.log_train_stats_t = -100000

    def _draw(self):
        if self._instance_fn is not None:
            st, gl = self._instance_fn(self._episode)
        else:
            st, gl = [], []
            for e in range(self.batch_size):
                s, g = _scen_draw(self._rngs[e], self.agents_path, self.n_agents)
                st.append(s)
                gl.append(g)
        return np.asarray(st, dtype=np.int32), np.asarray(gl, dtype=np.int32)

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

    def __del__(self):
        hp = getattr(self, "_ring_host", None)
        if hp is not None and hp.value:
            lib.mapfx_host_ring_free(hp)
            self._ring_host = None

    def get_env_info(self):
        return self.env_info

    def save_replay(self):
        pass

    def close_env(self):
        pass

    # ------------------------------------------------------------------ rows
    def _rows(self, batch):
        """mapfx_episode_rows over the batch's transition tensors (checked)."""
        td = batch.data.transition_data
        r = _abi.ERows(max_t=int(batch.max_seq_length))
        B, N, D = self.batch_size, self.n_agents, self.env.obs_dim
        shapes = {"obs": (N, D), "state": (3,), "avail_actions": (N, 5), "actions": (N, 1),
                  "actions_onehot": (N, 5), "reward": (1,), "terminated": (1,), "filled": (1,)}
        for key, field in _ROW_FIELDS.items():
            t = td.get(key)
            if t is None:
                if key != "actions_onehot":
                    raise KeyError("EpisodeBatch has no %r field" % key)
                continue
            if t.dtype != _ROW_DTYPES[key] or tuple(t.shape[2:]) != shapes[key] or \
                    t.shape[0] != B or t.device != self.device:
                raise ValueError("EpisodeBatch %r is %s %s on %s; the runner writes %s %s on %s"
                                 % (key, t.dtype, tuple(t.shape), t.device, _ROW_DTYPES[key],
                                    (B, r.max_t) + shapes[key], self.device))
            inner = 1
            for s in shapes[key]:
                inner *= s
            if t.stride(-1) != 1 or t.stride(1) < inner or (len(shapes[key]) > 1 and
                                                             t.stride(2) != shapes[key][1]):
                raise ValueError("EpisodeBatch %r rows are not contiguous" % key)
            setattr(r, field, ptr(t))
            setattr(r, field + "_sb", t.stride(0))
            setattr(r, field + "_st", t.stride(1))
        if "actions_onehot" in td:
            pre = (self.preprocess or {}).get("actions")
            tf = pre[1] if pre else []
            if not (pre and pre[0] == "actions_onehot" and len(tf) == 1
                    and type(tf[0]).__name__ == "OneHot" and getattr(tf[0], "out_dim", 5) == 5):
                raise ValueError("actions_onehot must come from the OneHot(out_dim=5) preprocess")
        return r

    def _call(self, fn, *args):
        return fn(*args, torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------------ loop
    def reset(self):
        """:62-76: new batch, every env reset (instances re-drawn, :130), row 0."""
        self.batch = self.new_batch()
        starts, goals = self._draw()
        key = (starts.tobytes(), goals.tobytes())
        if key != self._loaded:           # same instances: the BFS tables still hold
            self.env.set_agents(starts, goals)
            self._loaded = key
        self._episode += 1
        self.env.reset()
        self._erows = self._rows(self.batch)
        check(self._call(lib.mapfx_runner_begin, ctypes.byref(self._rs),
                         ctypes.byref(self.env._obs_out), ctypes.byref(self._erows)),
              "mapfx_runner_begin")
        self.t = 0
        self.env_steps_this_run = 0

    def run(self, test_mode=False):
        """:78-206 with the envs stepped as one batch on the device.

        Iteration k of the reference calls the MAC (bs = envs running before step
        k - 1), writes the actions rows, then stops if no env is running after step
        k - 1, else steps and writes the step's rows.  Here iteration k first stops
        if the ring slot of launch k - 2 says no env is running: with the post pass
        and the next MAC call's compaction fused into the env step (one launch per
        step, mapfx_runner_step) that slot counts the envs running after step k - 3,
        else (the separate post / compaction kernels) after step k - 2 -- two
        iterations old either way, so no wait in the steady state.  The iterations
        the lag adds past the reference's last MAC call find no running env (empty
        `bs`, no action rows, nothing stepped) and write nothing; the loop also ends
        when the batch has no row k (every env has met its episode limit by then)."""
        self.reset()
        self.mac.init_hidden(batch_size=self.batch_size)
        r, rs, env = self._erows, ctypes.byref(self._rs), self.env
        stream = torch.cuda.current_stream(self.device)
        sh = stream.cuda_stream
        fixed = (env._h, ctypes.byref(env._state), ctypes.byref(env._out), rs)
        step = lib.mapfx_runner_step
        # The MAC gets `bs` padded to B (no host sync per step); a stochastic selector
        # then draws random numbers for B rows, not len(bs) as the reference does
        # (parallel_runner.py:106), so its RNG stream diverges once an env has
        # terminated.  args.runner_exact_bs = True passes bs[:len(bs)] instead, at the
        # cost of one host sync per step (the count of the previous step's compaction).
        exact_bs = bool(getattr(self.args, "runner_exact_bs", False))
        k = 0
        max_t = int(r.max_t)
        while k < max_t:
            if k >= 2:   # none running (after step k - 3 fused, k - 2 unfused): stop
                ev, hc, _ = self._ring[(k - 2) % _RING]
                ev.synchronize()
                if int(hc[1]) == 0:
                    break
            bs = self._bs
            if exact_bs and k >= 1:   # len(bs) from step k - 1's compaction (one sync)
                ev, hc, _ = self._ring[(k - 1) % _RING]
                ev.synchronize()
                bs = self._bs[:int(hc[0])]
            actions = self.mac.select_actions(self.batch, t_ep=k, t_env=self.t_env, bs=bs,
                                              test_mode=test_mode)
            a = actions.reshape(-1, self.n_agents)   # row j is env bs[j] (j < len(bs) read)
            if a.device != self.device:
                a = a.to(self.device)
            if a.dtype not in _ADT:
                a = a.to(torch.int64)
            a = a.contiguous()
            ev, _, dslot = self._ring[k % _RING]
            rc = step(*fixed, a.data_ptr(), _ADT[a.dtype], a.stride(0), k, dslot, ctypes.byref(r), sh)
            if rc:
                check(rc, "mapfx_runner_step")
            ev.record(stream)
            k += 1
        self.t = k
        # the run's totals: one transfer at the end
        env_steps = int(self._env_steps.item())
        # an env given an action outside 0..4 was not stepped (its rows say reward 0):
        # the reference asserts at marl_partial.py:177
        env.check_err()
        returns = self._ep_return.cpu().tolist()
        lengths = self._ep_length.cpu()
        self.env_steps_this_run = 0 if test_mode else env_steps
        if not test_mode:
            self.t_env += env_steps
        cur_stats = self.test_stats if test_mode else self.train_stats
        cur_returns = self.test_returns if test_mode else self.train_returns
        log_prefix = "test_" if test_mode else ""
        # infos of terminated envs carry `_step_count` (marl_partial.py:310) and every env
        # has terminated when the loop ends: their sum is the sum of the episode lengths
        total_len = int(lengths.sum())
        cur_stats["_step_count"] = total_len + cur_stats.get("_step_count", 0)
        cur_stats["n_episodes"] = self.batch_size + cur_stats.get("n_episodes", 0)
        cur_stats["ep_length"] = total_len + cur_stats.get("ep_length", 0)
        cur_returns.extend(returns)
        n_test_runs = max(1, getattr(self.args, "test_nepisode", self.batch_size)
                          // self.batch_size) * self.batch_size
        if test_mode and (len(self.test_returns) == n_test_runs):
            self._log(cur_returns, cur_stats, log_prefix)
        elif self.t_env - self.log_train_stats_t >= getattr(self.args, "runner_log_interval",
                                                            1 << 62):
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
