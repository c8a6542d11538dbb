"""MapfGridBatch — E device-resident MAPF_GRID envs stepped by one HIP launch.

The batched counterpart of the reference's env + ParallelRunner pair
(MARL-curve-main/src/envs/mapf_gridworld.py, runners/parallel_runner.py:91-206):
state, actions and every output stay in HBM as torch tensors; the C ABI
(include/mapfx.h, via mapfx._abi) is called with their device pointers on the
current torch stream.  Nothing here computes env semantics on the host.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _abi
from ._abi import MAPFX_I8, MAPFX_I32, MAPFX_I64, MAPFX_OBS_FULL, MAPFX_OBS_PRIMAL, \
    MAPFX_OBS_WINDOW, check, lib, ptr
from .maps import map_stride, pack_bits

_DTYPES = {torch.int8: MAPFX_I8, torch.int32: MAPFX_I32, torch.int64: MAPFX_I64}
OBS_MODES = {"full": MAPFX_OBS_FULL, "window": MAPFX_OBS_WINDOW, "window_occ": MAPFX_OBS_WINDOW,
             "primal": MAPFX_OBS_PRIMAL}
_OBS_KEYS = ("term", "avail", "obs_full", "obs_window", "obs_window_occ", "obs_primal", "primal_vec")


def _stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


class MapfGridBatch:
    """E independent MAPF_GRID envs on one GPU.

    Parameters mirror MAPF_GRID.__init__ (envs/mapf_gridworld.py:21-32) plus the
    batch description: `grids` is [E|1, H, W] (nonzero = obstacle) or
    precomputed `bits` [E|1, map_stride]; `init_pos` / `goals` are [E, N, 2]
    (row, col).  `obs` selects which observation kinds are produced each step:
    "full" (get_obs/get_state occupancy), "window" (marl_partial window of
    `window`, [N, 2, w, w] obstacle / agents planes), "window_occ" (the same window
    as one [N, w, w] plane of occupancy values: obstacle = (v == -1), agents =
    max(v, 0); see window_planes), "primal" (PRIMAL _observe of `primal_size`).
    """

    def __init__(self, init_pos, goals, grids=None, bits=None, hw=None, episode_limit=10000,
                 step_reward=-0.01, collide_reward=-10, obs=("full",), window=5,
                 primal_size=10, device=None, env_offset=0, track_steps=True, packed=False):
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("MapfGridBatch runs on a HIP device only (got %s)" % self.device)
        init_pos = torch.as_tensor(np.array(init_pos, dtype=np.int32))
        goals = torch.as_tensor(np.array(goals, dtype=np.int32))
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
        ip, gl = init_pos.numpy(), goals.numpy()
        for name, arr in (("init_pos", ip), ("goals", gl)):
            if arr.size and (arr[..., 0].min() < 0 or arr[..., 0].max() >= self.H
                             or arr[..., 1].min() < 0 or arr[..., 1].max() >= self.W):
                raise ValueError("%s outside the %dx%d grid" % (name, self.H, self.W))
        self.map_shared = bits.shape[0] == 1 and self.E != 1
        self.episode_limit = int(episode_limit)
        self.step_reward = step_reward
        self.collide_reward = collide_reward
        self.obs_kinds = tuple(obs)
        mode = 0
        for k in self.obs_kinds:
            mode |= OBS_MODES[k]
        self.window, self.primal_size = int(window), int(primal_size)

        cfg = _abi.Cfg(H=self.H, W=self.W, n_agents=self.N, n_envs=self.E,
                       env_offset=int(env_offset), episode_limit=self.episode_limit,
                       step_reward=float(step_reward), collide_reward=float(collide_reward),
                       obs_mode=mode, window=self.window, primal_size=self.primal_size,
                       map_shared=1 if self.map_shared else 0)
        self._cfg = cfg
        with torch.cuda.device(self.device):
            h = ctypes.c_void_p()
            check(lib.mapfx_create(ctypes.byref(cfg), ctypes.byref(h)), "mapfx_create")
        self._h = h
        dev = self.device
        self.bits = torch.as_tensor(bits).to(dev)
        self.init_pos = init_pos.to(dev).contiguous()
        self.goal = goals.to(dev).contiguous()
        self.obs_elem = torch.int8 if lib.mapfx_obs_elem_size(self.N) == 1 else torch.int16
        self.edge_elem = torch.uint8 if lib.mapfx_edge_elem_size(self.N) == 1 else torch.int16  # counts < 2^15
        self.err = torch.zeros((1,), dtype=torch.int32, device=dev)
        # `packed`: the mutable state and every per-step output are views of ONE flat
        # device buffer (mapfx.dist.ChunkLayout), so a host mirror of all of it is a
        # single copy (the drop-in env pulls a step's results with one sync).
        spec = {"pos": ((self.E, self.N, 2), torch.int32), "done": ((self.E, self.N), torch.uint8),
                "t": ((self.E,), torch.int32), "err": ((1,), torch.int32)}
        if track_steps:
            spec["steps"] = ((self.E, self.N), torch.int32)
        spec.update(self.out_spec(None))
        self.packed = bool(packed)
        if self.packed:
            from .dist import ChunkLayout
            self._layout = ChunkLayout(spec)
            self._flat = self._layout.alloc(dev)
            v = self._layout.views(self._flat)
            self.pos, self.done, self.t, self.err = v["pos"], v["done"], v["t"], v["err"]
            self.pos.copy_(self.init_pos)
            self.steps = v.get("steps")
            self.out = {k: v[k] for k in self.out_spec(None)}
        else:
            self._layout = self._flat = None
            self.pos = self.init_pos.clone()
            self.done = torch.zeros((self.E, self.N), dtype=torch.uint8, device=dev)
            self.t = torch.zeros((self.E,), dtype=torch.int32, device=dev)
            self.steps = torch.zeros((self.E, self.N), dtype=torch.int32, device=dev) \
                if track_steps else None
            self.out = self._alloc_out(None)
        self._out_cache = {}          # outputs selection -> Out struct over self.out
        self._traj_cache = {}         # (outputs, buffer pointers) -> Out struct
        self._dev_index = self.device.index if self.device.index is not None \
            else torch.cuda.current_device()
        self._act_shape = (self.E, self.N)
        self._state = _abi.State(pos=ptr(self.pos), goal=ptr(self.goal),
                                 init_pos=ptr(self.init_pos), done=ptr(self.done), t=ptr(self.t),
                                 steps=ptr(self.steps), map_bits=ptr(self.bits))

    # ------------------------------------------------------------------ buffers
    def out_spec(self, T=None):
        """name -> (shape, dtype) of every output a step (T None) or a T-step
        rollout (leading [T]) can write (include/mapfx.h mapfx_out)."""
        E, N = self.E, self.N
        lead = () if T is None else (int(T),)
        o = {
            "reward": (lead + (E,), torch.float64),
            "reward_f32": (lead + (E,), torch.float32),
            "term": (lead + (E,), torch.uint8),
            "node": (lead + (E, N), torch.uint8),
            "edge": (lead + (E, N), self.edge_elem),
            "avail": (lead + (E, N), torch.uint8),
        }
        if "full" in self.obs_kinds:
            o["obs_full"] = (lead + (E, self.H * self.W), self.obs_elem)
        if "window" in self.obs_kinds:
            w = self.window
            o["obs_window"] = (lead + (E, N, 2, w, w), self.obs_elem)
        if "window_occ" in self.obs_kinds:
            w = self.window
            o["obs_window_occ"] = (lead + (E, N, w, w), self.obs_elem)
        if "primal" in self.obs_kinds:
            s = self.primal_size
            o["obs_primal"] = (lead + (E, N, 4, s, s), torch.uint8)
            o["primal_vec"] = (lead + (E, N, 3), torch.float64)
        if T is not None:
            o["traj_pos"] = ((T, E, N, 2), torch.int32)
            o["traj_done"] = ((T, E, N), torch.uint8)
            o["traj_t"] = ((T, E), torch.int32)
        return o

    def _alloc_out(self, T):
        return {k: torch.zeros(shape, dtype=dt, device=self.device)
                for k, (shape, dt) in self.out_spec(T).items()}

    def _own_out(self, keys):
        """Cached Out struct over the persistent self.out buffers."""
        k = None if keys is None else tuple(keys)
        s = self._out_cache.get(k)
        if s is None:
            s = self._out_cache[k] = self._out_struct(self.out, keys=k)
        return s

    def _call(self, fn, *args):
        """Run a C-ABI call with self.device current (no context switch when it already is)."""
        if torch.cuda.current_device() == self._dev_index:
            return fn(*args, torch.cuda.current_stream().cuda_stream)
        with torch.cuda.device(self.device):
            return fn(*args, torch.cuda.current_stream().cuda_stream)

    def _out_struct(self, o, keys=None):
        s = _abi.Out()
        for name, _ in _abi.Out._fields_:
            if name == "err":
                continue
            if keys is not None and name not in keys:
                continue
            if name in o:
                setattr(s, name, ptr(o[name]))
        s.err = ptr(self.err)
        return s

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.mapfx_destroy(h)
            self._h = None

    def info(self):
        inf = _abi.Info()
        check(lib.mapfx_query(self._h, ctypes.byref(inf)), "mapfx_query")
        return {k: getattr(inf, k) for k, _ in _abi.Info._fields_}

    # ------------------------------------------------------------------ API
    def reset(self, env_mask=None):
        """envs/mapf_gridworld.py:70-83 for the masked envs (all if None);
        refreshes obs/avail/term of every env.  Returns self.out."""
        m = None
        if env_mask is not None:
            m = torch.as_tensor(env_mask, device=self.device).to(torch.uint8).contiguous()
        o = self._own_out(_OBS_KEYS)
        check(self._call(lib.mapfx_reset, self._h, ctypes.byref(self._state), ptr(m),
                         ctypes.byref(o)), "mapfx_reset")
        return self.out

    def observe(self):
        o = self._own_out(_OBS_KEYS)
        check(self._call(lib.mapfx_observe, self._h, ctypes.byref(self._state), ctypes.byref(o)),
              "mapfx_observe")
        return self.out

    def step(self, actions, outputs=None):
        """One env step of all E envs.  actions: [E, N] int8/int32/int64 tensor.
        `outputs` optionally restricts which outputs are written (names of self.out)."""
        a = actions
        if not (isinstance(a, torch.Tensor) and a.device == self.device and a.dtype in _DTYPES
                and a.is_contiguous()):
            a = torch.as_tensor(a, device=self.device)
            if a.dtype not in _DTYPES:
                a = a.to(torch.int64)
            a = a.contiguous()
        if a.shape != self._act_shape:
            raise AssertionError("actions must be [%d, %d], got %s" % (self.E, self.N,
                                                                     tuple(a.shape)))
        o = self._own_out(outputs)
        check(self._call(lib.mapfx_step, self._h, ctypes.byref(self._state), a.data_ptr(),
                         _DTYPES[a.dtype], ctypes.byref(o)), "mapfx_step")
        return self.out

    def _traj_struct(self, traj, outputs):
        """Out struct over a trajectory dict, cached by the buffers' device pointers:
        repeated rollouts into the same buffers build no ctypes objects, and the
        cache holds no reference to any tensor (the struct is pointers only, so an
        entry keyed by equal pointers is the same struct)."""
        keys = None if outputs is None else tuple(outputs)
        k = (keys,) + tuple((n, v.data_ptr()) for n, v in traj.items()
                            if isinstance(v, torch.Tensor))
        s = self._traj_cache.get(k)
        if s is None:
            s = self._out_struct(traj, keys=keys)
            if len(self._traj_cache) >= 64:
                self._traj_cache.clear()
            self._traj_cache[k] = s
        return s

    def _rollout_actions(self, T, actions):
        if actions is None:
            return None, None, MAPFX_I8
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype not in _DTYPES:
            a = a.to(torch.int64)
        a = a.contiguous()
        if tuple(a.shape) != (T, self.E, self.N):
            raise AssertionError("actions must be [T, E, N]")
        return a, ptr(a), _DTYPES[a.dtype]

    def rollout(self, T, actions=None, seed=0, t0=0, autoreset=False, traj=None, outputs=None):
        """T fused steps in one launch.  actions: [T, E, N] tensor or None (device
        generator keyed by (seed, global env, t0+k, agent)).  Returns the
        trajectory dict ([T, ...] tensors), allocated unless `traj` is given."""
        if traj is None:
            traj = self._alloc_out(T)
        actions, ap, adt = self._rollout_actions(T, actions)
        o = self._traj_struct(traj, outputs)
        check(self._call(lib.mapfx_rollout, self._h, ctypes.byref(self._state), int(T), ap, adt,
                         int(seed) & 0xFFFFFFFFFFFFFFFF, int(t0), 1 if autoreset else 0,
                         ctypes.byref(o)), "mapfx_rollout")
        return traj

    def rollout_plan(self, T, actions=None, seed=0, t0=0, autoreset=False, traj=None,
                     outputs=None, stream=None, events=None):
        """A prepared `rollout` launch: every argument is converted once, so calling
        the returned plan is one ctypes call (no tensor checks, no struct building).
        The plan keeps `actions` / `traj` alive and launches on `stream` (default:
        the current stream now).  Used where host time per launch matters (bench)."""
        if traj is None:
            traj = self._alloc_out(T)
        actions, ap, adt = self._rollout_actions(T, actions)
        return RolloutPlan(self, int(T), actions, ap, adt, int(seed) & 0xFFFFFFFFFFFFFFFF,
                           int(t0), 1 if autoreset else 0, traj,
                           self._out_struct(traj, keys=None if outputs is None else tuple(outputs)),
                           stream if stream is not None else torch.cuda.current_stream(self.device),
                           events)

    def gen_actions(self, T, seed, t0=0, out=None):
        if out is None:
            out = torch.empty((T, self.E, self.N), dtype=torch.int8, device=self.device)
        with torch.cuda.device(self.device):
            check(lib.mapfx_gen_actions(self._h, int(seed) & 0xFFFFFFFFFFFFFFFF, int(t0), int(T),
                                        ptr(out), _stream_handle()), "mapfx_gen_actions")
        return out

    def pack_compact(self, traj_pos, traj_done, cell, done_bits):
        """cell[T,E,N] (int16 holding the u16 row * W + col) and done_bits
        [T,E,ceil(N/8)] (bit a & 7 of byte a >> 3) from a rollout's traj_pos /
        traj_done, on the current stream (mapfx_pack_compact)."""
        T = int(traj_pos.shape[0])
        nb = (self.N + 7) // 8
        for name, t, shape, dt in (("traj_pos", traj_pos, (T, self.E, self.N, 2), torch.int32),
                                   ("traj_done", traj_done, (T, self.E, self.N), torch.uint8),
                                   ("cell", cell, (T, self.E, self.N), torch.int16),
                                   ("done_bits", done_bits, (T, self.E, nb), torch.uint8)):
            if tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous() \
                    or t.device != self.device:
                raise ValueError("%s must be a contiguous %s %s tensor on %s"
                                 % (name, shape, dt, self.device))
        check(self._call(lib.mapfx_pack_compact, self._h, T, ptr(traj_pos), ptr(traj_done),
                         ptr(cell), ptr(done_bits)), "mapfx_pack_compact")

    def set_positions(self, pos, done=None, t=None):
        """Overwrite the device state (pos [E,N,2] int32 (row, col), optional done /
        t) -- e.g. positions unpacked from a compact gather, to rebuild their
        observations with observe().  Positions are checked to lie on the grid (one
        host sync): the kernels index their LDS cell maps with them.  A position on
        an obstacle cell is legal state (quirk 1: agents may stand on obstacles, e.g.
        transposed .scen starts) and is observed exactly as the reference would.
        Any strided input (a slice of unpack_compact's output) is accepted."""
        p = torch.as_tensor(pos, device=self.device)
        if p.dtype.is_floating_point or p.dtype.is_complex or p.dtype == torch.bool:
            raise TypeError("positions must be an integer tensor, got %s" % p.dtype)
        p = p.reshape(self.E, self.N, 2)
        # range check before the int32 cast: an int64 outside int32 must not wrap onto the grid
        p64 = p.to(torch.int64)
        lo = torch.tensor([0, 0], device=self.device, dtype=torch.int64)
        hi = torch.tensor([self.H, self.W], device=self.device, dtype=torch.int64)
        if p.numel() and not bool(((p64 >= lo) & (p64 < hi)).all()):
            raise ValueError("positions outside the %dx%d grid" % (self.H, self.W))
        self.pos.copy_(p.to(torch.int32))
        if done is not None:
            self.done.copy_(torch.as_tensor(done, device=self.device).reshape(self.E, self.N))
        if t is not None:
            self.t.copy_(torch.as_tensor(t, device=self.device).reshape(self.E))

    def host_mirror(self):
        """Pinned host copy of the packed buffer and its typed views (packed=True)."""
        if not self.packed:
            raise RuntimeError("host_mirror needs MapfGridBatch(..., packed=True)")
        flat = torch.empty(self._layout.nbytes, dtype=torch.uint8, pin_memory=True)
        return flat, self._layout.views(flat)

    def pull(self, host_flat):
        """Copy state + outputs into `host_flat` (host_mirror) and wait for it: the
        one synchronisation of a drop-in step."""
        host_flat.copy_(self._flat, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return host_flat

    def check_err(self):
        """Raise AssertionError like the reference (:91-92) if an env got an
        action outside 0..4 since the last call (synchronises)."""
        e = int(self.err.item())
        if e:
            self.err.zero_()
            raise AssertionError("invalid action for env %d (actions must be in 0..4)" % (e - 1))

    # --------------------------------------------------- PyMARL-shaped views
    def avail_actions(self, avail=None):
        """[E, N, 5] int64 0/1, the layout of get_avail_actions (:198-224)."""
        m = self.out["avail"] if avail is None else avail
        bits = torch.arange(5, device=m.device, dtype=torch.uint8)
        return ((m.unsqueeze(-1) >> bits) & 1).to(torch.int64)

    def full_obs(self):
        """[E, N, H*W] view: every agent observes the same occupancy map (:161-183)."""
        o = self.out["obs_full"]
        return o.unsqueeze(1).expand(self.E, self.N, o.shape[-1])


class RolloutPlan:
    """One prepared `mapfx_rollout` launch (MapfGridBatch.rollout_plan).

    Holds the ctypes arguments ready-made: __call__ is a single foreign call on
    the plan's stream.  `traj` is the trajectory dict the launch writes."""

    __slots__ = ("batch", "T", "actions", "traj", "_fn", "_args")

    def __init__(self, batch, T, actions, ap, adt, seed, t0, autoreset, traj, out, stream,
                 events=None):
        self.batch, self.T, self.actions, self.traj = batch, T, actions, traj
        # byref objects keep `out` and the state struct alive with the plan
        if events is None:
            self._fn = lib.mapfx_rollout
            self._args = (batch._h, ctypes.byref(batch._state), T, ap, adt, seed, t0, autoreset,
                          ctypes.byref(out), stream.cuda_stream)
        else:   # (start, stop) torch.cuda.Event, recorded at the kernel's own begin / end
            self._fn = lib.mapfx_rollout_timed
            self._args = (batch._h, ctypes.byref(batch._state), T, ap, adt, seed, t0, autoreset,
                          ctypes.byref(out), events[0].cuda_event, events[1].cuda_event,
                          stream.cuda_stream)

    def __call__(self):
        rc = self._fn(*self._args)
        if rc:
            check(rc, "mapfx_rollout")
        return self.traj


def window_planes(occ):
    """[..., w, w] occupancy window (obs_window_occ) -> [..., 2, w, w] {obstacle,
    agents} planes, i.e. obs_window (envs/marl_partial.py:323-342)."""
    return torch.stack(((occ == -1).to(occ.dtype), occ.clamp(min=0)), dim=-3)
