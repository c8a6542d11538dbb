"""PrimalBatch -- E device-resident PRIMAL worlds, sequential dynamics.

Batched counterpart of MARL-curve-main/src/envs/mapf_primal.py's
`MAPFEnv._step((agent_id, action))` (:549-637) over the C ABI in
include/mapfx_primal.h: every world takes K single-agent calls in order, each
one `State.moveAgent` (:103-135), the reward table (:579-596), `_observe`
(:343-386), `State.done` (:159-166) and `_listNextValidActions` (:639-667), all
in one HIP kernel.  `MAPFEnv` below is the single-world drop-in with the
reference's call signature.  Nothing here computes env semantics on the host.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _abi
from ._abi import check, lib, ptr
from .maps import map_stride, pack_bits, primal_world

_OUT_KEYS = ("reward", "done", "next_mask", "on_goal", "valid", "obs", "vec")


class PrimalBatch:
    """E PRIMAL worlds on one GPU.  `grids` [E|1, H, W] (negative = obstacle, as
    PRIMAL's world0) or `bits` [E|1, map_stride]; starts / goals [E, N, 2] (row, col)."""

    def __init__(self, starts, goals, grids=None, bits=None, hw=None, observation_size=10,
                 device=None, diagonal=False, past=None):
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("PrimalBatch runs on a HIP device only (got %s)" % self.device)
        starts = np.array(starts, dtype=np.int32)
        goals = np.array(goals, dtype=np.int32)
        if starts.ndim != 3 or starts.shape[-1] != 2 or goals.shape != starts.shape:
            raise ValueError("starts/goals must both be [E, N, 2]")
        self.E, self.N = int(starts.shape[0]), int(starts.shape[1])
        if bits is None:
            g = np.asarray(grids)
            if g.ndim == 2:
                g = g[None]
            self.H, self.W = int(g.shape[1]), int(g.shape[2])
            bits = pack_bits(g < 0)
        else:
            self.H, self.W = hw
        bits = np.array(bits, dtype=np.uint8)
        if bits.ndim == 1:
            bits = bits[None]
        if bits.shape[1] != map_stride(self.H, self.W) or bits.shape[0] not in (1, self.E):
            raise ValueError("bits must be [E or 1, %d]" % map_stride(self.H, self.W))
        self._check_placement(starts, goals, bits)
        self.map_shared = bits.shape[0] == 1 and self.E != 1
        self.s = int(observation_size)
        self.diagonal = bool(diagonal)
        self.n_actions = 9 if self.diagonal else 5
        cfg = _abi.QCfg(H=self.H, W=self.W, n_agents=self.N, n_envs=self.E, obs_size=self.s,
                        map_shared=1 if self.map_shared else 0, diagonal=1 if self.diagonal else 0)
        with torch.cuda.device(self.device):
            h = ctypes.c_void_p()
            check(lib.mapfx_primal_create(ctypes.byref(cfg), ctypes.byref(h)), "mapfx_primal_create")
        self._h = h
        dev = self.device
        self.bits = torch.as_tensor(bits).to(dev)
        self.pos = torch.as_tensor(starts).to(dev).contiguous()
        self.goal = torch.as_tensor(goals).to(dev).contiguous()
        self.err = torch.zeros((1,), dtype=torch.int32, device=dev)
        # agents_past (DIAGONAL_MOVEMENT): equal to the starts in a fresh world (:55-66)
        self.past = None
        if self.diagonal:
            pp = starts if past is None else np.array(past, dtype=np.int32)
            # the kernels read past as int2 at [e * N + i] and primal_seq_kernel packs it
            # as biased u8 (row, col) bytes: shape and bounds are checked here
            if pp.shape != starts.shape:
                raise ValueError("past must be [E, N, 2] like the starts, got %s" % (pp.shape,))
            if pp.size and ((pp[..., 0] < 0).any() or (pp[..., 0] >= self.H).any()
                            or (pp[..., 1] < 0).any() or (pp[..., 1] >= self.W).any()):
                raise ValueError("past outside the %dx%d grid" % (self.H, self.W))
            self.past = torch.as_tensor(pp).to(dev).contiguous()
        self._state = _abi.QState(pos=ptr(self.pos), goal=ptr(self.goal), map_bits=ptr(self.bits),
                                  past=ptr(self.past))
        self._K = -1
        self.out = None

    def _check_placement(self, starts, goals, bits):
        """Distinct in-bounds starts and goals on free cells: PRIMAL keeps agents,
        goals and obstacles in one array per kind (:44-66), so the kernel assumes it."""
        H, W = self.H, self.W
        for arr, what in ((starts, "starts"), (goals, "goals")):
            if (arr[..., 0] < 0).any() or (arr[..., 0] >= H).any() or (arr[..., 1] < 0).any() \
                    or (arr[..., 1] >= W).any():
                raise ValueError("%s out of bounds" % what)
            flat = arr[..., 0].astype(np.int64) * W + arr[..., 1]
            if any(len(np.unique(row)) != self.N for row in flat):
                raise ValueError("%s must be distinct within a world" % what)
        cells = starts[..., 0].astype(np.int64) * W + starts[..., 1]
        b = bits if bits.shape[0] == cells.shape[0] else np.repeat(bits, cells.shape[0], 0)
        blocked = (np.take_along_axis(b, cells >> 3, 1) >> (cells & 7)) & 1
        if blocked.any():
            raise ValueError("an agent starts on an obstacle")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.mapfx_primal_destroy(h)
            self._h = None

    def _alloc(self, K):
        E, s, dev = self.E, self.s, self.device
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=dev)  # noqa: E731
        self.out = {"reward": z((E, K), torch.float64), "done": z((E, K), torch.uint8),
                    "next_mask": z((E, K), torch.int16 if self.diagonal else torch.uint8),
                    "on_goal": z((E, K), torch.uint8),
                    "valid": z((E, K), torch.uint8), "obs": z((E, K, 4, s, s), torch.uint8),
                    "vec": z((E, K, 3), torch.float64)}
        self._out = _abi.QOut(err=ptr(self.err), **{k: ptr(self.out[k]) for k in _OUT_KEYS})
        self._K = K

    def act(self, agent_ids, actions, events=None):
        """K calls of `_step((agent_id, action))` per world, in order.
        agent_ids (1-based) / actions: [E, K] ints.  Returns the output dict,
        each entry [E, K, ...] (buffers reused by the next call with the same K).
        events: optional (start, stop) torch.cuda.Event pair recorded at the
        kernel's own begin / end (mapfx_primal_act_timed)."""
        ids = torch.as_tensor(agent_ids, device=self.device).to(torch.int32).contiguous()
        acts = torch.as_tensor(actions, device=self.device).to(torch.int32).contiguous()
        if ids.ndim != 2 or ids.shape[0] != self.E or acts.shape != ids.shape:
            raise AssertionError("agent_ids / actions must be [%d, K]" % self.E)
        K = int(ids.shape[1])
        if K != self._K:
            self._alloc(K)
        with torch.cuda.device(self.device):
            if events is None:
                check(lib.mapfx_primal_act(self._h, ctypes.byref(self._state), ptr(ids), ptr(acts), K,
                                           ctypes.byref(self._out),
                                           torch.cuda.current_stream().cuda_stream),
                      "mapfx_primal_act")
            else:
                check(lib.mapfx_primal_act_timed(self._h, ctypes.byref(self._state), ptr(ids), ptr(acts),
                                                 K, ctypes.byref(self._out), events[0].cuda_event,
                                                 events[1].cuda_event,
                                                 torch.cuda.current_stream().cuda_stream),
                      "mapfx_primal_act_timed")
        return self.out

    def check_err(self):
        e = int(self.err.item())
        if e:
            self.err.zero_()
            raise AssertionError("invalid (agent_id, action) for world %d" % (e - 1))


class MAPFEnv:
    """Single-world drop-in for mapf_primal.py MAPFEnv (:168-667) on the device.
    World set-up follows _setWorld (:248-341): a given world0 / goals0 (PRIMAL's
    int arrays: -1 obstacle, agent id at its start / goal cell), agents and goals
    placed on a given world (blank_world), or a random world from SIZE / PROB --
    the last two drawn on the host by mapfx.maps.primal_world from the global
    np.random / random generators, as the reference draws them.  Rendering is
    outside the hot path."""

    def __init__(self, num_agents=1, observation_size=10, world0=None, goals0=None,
                 DIAGONAL_MOVEMENT=False, SIZE=(10, 40), PROB=(0, .5), FULL_HELP=False,
                 blank_world=False, device=None):
        self.DIAGONAL_MOVEMENT = bool(DIAGONAL_MOVEMENT)
        self.n_actions = 9 if self.DIAGONAL_MOVEMENT else 5
        self.num_agents = int(num_agents)
        self.observation_size = int(observation_size)
        self.SIZE, self.PROB, self.FULL_HELP = SIZE, PROB, FULL_HELP
        self._device = device
        self._set_world(world0, goals0, blank_world)

    def _set_world(self, world0, goals0, blank_world=False):
        if world0 is None:
            world0, goals0 = primal_world(self.num_agents, SIZE=self.SIZE, PROB=self.PROB)
        elif blank_world:
            world0, goals0 = primal_world(self.num_agents, world0=world0, blank_world=True)
        elif goals0 is None:
            raise Exception("you gave a world with no goals!")
        world0 = np.asarray(world0)
        goals0 = np.asarray(goals0)
        starts, goals = [], []
        for a in range(1, self.num_agents + 1):
            starts.append(tuple(int(v) for v in np.argwhere(world0 == a)[0]))
            goals.append(tuple(int(v) for v in np.argwhere(goals0 == a)[0]))
        self.initial_world, self.initial_goals = world0.copy(), goals0.copy()
        self._grid = np.where(world0 < 0, -1, 0).astype(np.int8)
        self.batch = PrimalBatch([starts], [goals], grids=self._grid,
                                 observation_size=self.observation_size, device=self._device,
                                 diagonal=self.DIAGONAL_MOVEMENT)
        self.finished = False
        self.fresh = True
        self.individual_rewards = [0 for _ in range(self.num_agents)]

    def _reset(self, agent_id, world0=None, goals0=None):
        """:389-402 -> (next valid actions, on_goal, False)."""
        self._set_world(world0, goals0)
        o = self.batch.act([[agent_id]], [[0]])  # a stay call changes nothing; it reports
        mask = int(o["next_mask"][0, 0].item())  # the valid moves with no previous action
        return ([a for a in range(self.n_actions) if (mask >> a) & 1],
                bool(o["on_goal"][0, 0].item()), False)

    def getObstacleMap(self):
        return (self._grid == -1).astype(int)

    def getGoals(self):
        return [tuple(int(v) for v in g) for g in self.batch.goal[0].tolist()]

    def getPositions(self):
        return [tuple(int(v) for v in p) for p in self.batch.pos[0].tolist()]

    def _step(self, action_input, episode=0):
        """:549-637 -> (state, reward, done, nextActions, on_goal, blocking, valid)."""
        assert len(action_input) == 2, 'Action input should be a tuple with the form (agent_id, action)'
        assert action_input[1] in range(self.n_actions), 'Invalid action'
        assert action_input[0] in range(1, self.num_agents + 1)
        agent_id, action = action_input
        o = self.batch.act([[agent_id]], [[action]])
        obs = o["obs"][0, 0].cpu().numpy()
        vec = o["vec"][0, 0].cpu().tolist()
        reward = float(o["reward"][0, 0].item())
        done = bool(o["done"][0, 0].item())
        mask = int(o["next_mask"][0, 0].item())
        self.individual_rewards[agent_id - 1] = reward
        self.finished |= done
        next_actions = [a for a in range(self.n_actions) if (mask >> a) & 1]
        state = ([obs[i] for i in range(4)], vec)
        return (state, reward, done, next_actions, bool(o["on_goal"][0, 0].item()), False,
                bool(o["valid"][0, 0].item()))
