"""MarlPartialBatch -- E device-resident MARL_PARTIAL_ENV instances.

Batched counterpart of MARL-curve-main/src/envs/marl_partial.py over the C ABI
in include/mapfx_partial.h: goal-distance tables by a bit-parallel BFS kernel
(:906-928), reset (:125-163), step (:165-310) and get_obs / get_state /
get_avail_actions (:312-433) as HIP kernels.  Observations are float32 (the dtype
PyMARL's EpisodeBatch stores them in); rewards are fp64 in the reference's
operation order.  Nothing here computes env semantics on the host.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _abi
from ._abi import MAPFX_I8, MAPFX_I32, MAPFX_I64, check, lib, ptr
from .maps import map_stride, pack_bits

_DTYPES = {torch.int8: MAPFX_I8, torch.int32: MAPFX_I32, torch.int64: MAPFX_I64}

DEFAULTS = dict(  # MARL_PARTIAL_ENV.__init__ defaults (:25-47)
    obs_window=5, obs_knn_agents=5, episode_limit=100, move_reward=-0.01, stay_reward=-0.02,
    stay_goal_reward=0, node_collide_reward=-1, edge_collide_reward=-1, env_collide_reward=-1,
    complete_reward=1000, complete_fac=1.5, gamma=0.99)


class MarlPartialBatch:
    """E independent MARL_PARTIAL_ENV envs on one GPU.  `grids` [E|1, H, W]
    (nonzero = obstacle) or `bits` [E|1, map_stride]; init_pos / goals [E, N, 2]."""

    def __init__(self, init_pos, goals, grids=None, bits=None, hw=None, device=None, env_offset=0,
                 packed=False, **params):
        unknown = set(params) - set(DEFAULTS)
        if unknown:
            raise TypeError("unknown MARL_PARTIAL_ENV parameters: %s" % sorted(unknown))
        p = dict(DEFAULTS)
        p.update(params)
        self.params = p
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("MarlPartialBatch runs on a HIP device only (got %s)" % self.device)
        init_pos = np.array(init_pos, dtype=np.int32)
        goals = np.array(goals, dtype=np.int32)
        if init_pos.ndim != 3 or init_pos.shape[-1] != 2 or goals.shape != init_pos.shape:
            raise ValueError("init_pos/goals must both be [E, N, 2]")
        self.E, self.N = int(init_pos.shape[0]), int(init_pos.shape[1])
        if bits is None:
            g = np.asarray(grids)
            if g.ndim == 2:
                g = g[None]
            self.H, self.W = int(g.shape[1]), int(g.shape[2])
            bits = pack_bits(g)
        else:
            self.H, self.W = hw
        bits = np.array(bits, dtype=np.uint8)
        if bits.ndim == 1:
            bits = bits[None]
        if bits.shape[1] != map_stride(self.H, self.W) or bits.shape[0] not in (1, self.E):
            raise ValueError("bits must be [E or 1, %d]" % map_stride(self.H, self.W))
        self.map_shared = bits.shape[0] == 1 and self.E != 1
        self.episode_limit = int(p["episode_limit"])
        cfg = _abi.PCfg(H=self.H, W=self.W, n_agents=self.N, n_envs=self.E,
                        env_offset=int(env_offset), episode_limit=self.episode_limit,
                        obs_window=int(p["obs_window"]), obs_knn_agents=int(p["obs_knn_agents"]),
                        map_shared=1 if self.map_shared else 0,
                        move_reward=float(p["move_reward"]), stay_reward=float(p["stay_reward"]),
                        stay_goal_reward=float(p["stay_goal_reward"]),
                        node_collide_reward=float(p["node_collide_reward"]),
                        edge_collide_reward=float(p["edge_collide_reward"]),
                        env_collide_reward=float(p["env_collide_reward"]),
                        complete_reward=float(p["complete_reward"]),
                        complete_fac=float(p["complete_fac"]), gamma=float(p["gamma"]))
        with torch.cuda.device(self.device):
            h = ctypes.c_void_p()
            check(lib.mapfx_partial_create(ctypes.byref(cfg), ctypes.byref(h)),
                  "mapfx_partial_create")
        self._h = h
        self._dev_index = self.device.index if self.device.index is not None \
            else torch.cuda.current_device()
        self.obs_dim = int(lib.mapfx_partial_obs_dim(h))
        E, N, dev = self.E, self.N, self.device
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=dev)  # noqa: E731
        self.bits = torch.as_tensor(bits).to(dev)
        self.init_pos = torch.as_tensor(init_pos).to(dev).contiguous()
        self.goal = torch.as_tensor(goals).to(dev).contiguous()
        # `packed`: what the drop-in env reads after a step (positions, flags and the
        # outputs) are views of ONE flat buffer, pulled to the host with one copy
        spec = {"pos": ((E, N, 2), torch.int32), "done": ((E, N), torch.uint8),
                "terminated": ((E,), torch.uint8), "t": ((E,), torch.int32),
                "err": ((1,), torch.int32), "reward": ((E,), torch.float64),
                "obs": ((E, N, self.obs_dim), torch.float32), "state": ((E, 3), torch.float32),
                "avail": ((E, N), torch.uint8)}
        self.packed = bool(packed)
        if self.packed:
            from .dist import ChunkLayout
            self._layout = ChunkLayout(spec)
            self._flat = self._layout.alloc(dev)
            v = self._layout.views(self._flat)
        else:
            self._layout = self._flat = None
            v = {k: z(shape, dt) for k, (shape, dt) in spec.items()}
        self.pos, self.done, self.terminated, self.t, self.err = (
            v["pos"], v["done"], v["terminated"], v["t"], v["err"])
        self.pos.copy_(self.init_pos)
        self.steps = z((E, N), torch.int32)
        self.at_goal = z((E, N), torch.uint8)
        self.goal_cost = z((E, N), torch.int32)
        self.node = z((E, N), torch.uint8)
        self.edge = z((E, N), torch.int32)
        self.total_coll = z((E,), torch.int32)
        # goal distance of each agent's current cell, carried by the kernels (INT32_MIN:
        # not known yet, looked up; reset / observe set it)
        self.pdist = torch.full((E, N), -2 ** 31, dtype=torch.int32, device=dev)
        # u8 (255 = -1) while H * W <= 255, int16 up to 32767 cells, else int32
        gd_dt = {1: torch.uint8, 2: torch.int16, 4: torch.int32}[
            int(lib.mapfx_partial_goal_dist_elem_size(self.H, self.W))]
        self.goal_dist = z((E, N, self.H * self.W), gd_dt)
        # the goal distances of each agent's 4 neighbour cells, carried with pdist (u8 /
        # int16 tables): a step reads a moving agent's npd from it
        self.pnbr = z((E, N, 4), torch.int16) if gd_dt != torch.int32 else None
        self.out = {k: v[k] for k in ("reward", "obs", "state", "avail")}
        self._state = _abi.PState(
            pos=ptr(self.pos), goal=ptr(self.goal), init_pos=ptr(self.init_pos),
            steps=ptr(self.steps), at_goal=ptr(self.at_goal), done=ptr(self.done),
            goal_cost=ptr(self.goal_cost), node=ptr(self.node), edge=ptr(self.edge), t=ptr(self.t),
            terminated=ptr(self.terminated), total_coll=ptr(self.total_coll),
            map_bits=ptr(self.bits), goal_dist=ptr(self.goal_dist), pdist=ptr(self.pdist),
            pnbr=ptr(self.pnbr) if self.pnbr is not None else None)
        self._out = _abi.POut(reward=ptr(self.out["reward"]), obs=ptr(self.out["obs"]),
                              state=ptr(self.out["state"]), avail=ptr(self.out["avail"]),
                              err=ptr(self.err))
        self._obs_out = _abi.POut(reward=None, obs=ptr(self.out["obs"]),
                                  state=ptr(self.out["state"]), avail=ptr(self.out["avail"]),
                                  err=ptr(self.err))
        self.compute_goal_dist()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.mapfx_partial_destroy(h)
            self._h = None

    def _call(self, fn, *args):
        """Run a C-ABI call with self.device current (no context switch when it already is)."""
        if torch.cuda.current_device() == self._dev_index:
            return fn(*args, torch.cuda.current_stream().cuda_stream)
        with torch.cuda.device(self.device):
            return fn(*args, torch.cuda.current_stream().cuda_stream)

    # ------------------------------------------------------------------ API
    def compute_goal_dist(self, env_mask=None):
        """BFS tables of the (masked) envs' goals (:906-928)."""
        m = None if env_mask is None else \
            torch.as_tensor(env_mask, device=self.device).to(torch.uint8).contiguous()
        check(self._call(lib.mapfx_partial_goal_dist, self._h, ctypes.byref(self._state), ptr(m)),
              "mapfx_partial_goal_dist")

    def set_agents(self, init_pos, goals, env_mask=None):
        """New starts / goals (the reference re-samples them at every reset, :130)
        for the masked envs, and their goal-distance tables."""
        ip = torch.as_tensor(np.array(init_pos, dtype=np.int32), device=self.device)
        gl = torch.as_tensor(np.array(goals, dtype=np.int32), device=self.device)
        if env_mask is None:
            self.init_pos.copy_(ip)
            self.goal.copy_(gl)
        else:
            m = torch.as_tensor(env_mask, device=self.device).bool()
            self.init_pos[m] = ip[m]
            self.goal[m] = gl[m]
        self.compute_goal_dist(env_mask)

    def reset(self, env_mask=None):
        """:125-163 for the masked envs (all if None); observations of every env."""
        m = None if env_mask is None else \
            torch.as_tensor(env_mask, device=self.device).to(torch.uint8).contiguous()
        check(self._call(lib.mapfx_partial_reset, self._h, ctypes.byref(self._state), ptr(m),
                         ctypes.byref(self._obs_out)), "mapfx_partial_reset")
        return self.out

    def observe(self):
        check(self._call(lib.mapfx_partial_observe, self._h, ctypes.byref(self._state),
                         ctypes.byref(self._obs_out)), "mapfx_partial_observe")
        return self.out

    def step(self, actions):
        """One step of all E envs (:165-310).  actions: [E, N] int8/int32/int64."""
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype not in _DTYPES:
            a = a.to(torch.int64)
        a = a.contiguous()
        if tuple(a.shape) != (self.E, self.N):
            raise AssertionError("actions must be [%d, %d]" % (self.E, self.N))
        check(self._call(lib.mapfx_partial_step, self._h, ctypes.byref(self._state), ptr(a),
                         _DTYPES[a.dtype], ctypes.byref(self._out)), "mapfx_partial_step")
        return self.out

    def host_mirror(self):
        """Pinned host copy of the packed buffer and its typed views (packed=True)."""
        if not self.packed:
            raise RuntimeError("host_mirror needs MarlPartialBatch(..., packed=True)")
        flat = torch.empty(self._layout.nbytes, dtype=torch.uint8, pin_memory=True)
        return flat, self._layout.views(flat)

    def pull(self, host_flat):
        """Copy the packed buffer into `host_flat` and wait for it (one sync)."""
        host_flat.copy_(self._flat, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return host_flat

    def check_err(self):
        e = int(self.err.item())
        if e:
            self.err.zero_()
            raise AssertionError("invalid action for env %d (actions must be in 0..4)" % (e - 1))

    def avail_actions(self):
        """[E, N, 5] int64 0/1 (get_avail_actions)."""
        bits = torch.arange(5, device=self.device, dtype=torch.uint8)
        return ((self.out["avail"].unsqueeze(-1) >> bits) & 1).to(torch.int64)
