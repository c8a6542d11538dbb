"""ctypes loader of the C oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class OrcCfg(ctypes.Structure):
    _fields_ = [("H", ctypes.c_int32), ("W", ctypes.c_int32), ("N", ctypes.c_int32),
                ("E", ctypes.c_int32), ("env_offset", ctypes.c_int64), ("limit", ctypes.c_int32),
                ("step_rew", ctypes.c_double), ("collide_rew", ctypes.c_double),
                ("map_shared", ctypes.c_int32), ("map_stride", ctypes.c_int64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("oracle/liboracle.so not built (make -C oracle)")
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.orc_action.restype = ctypes.c_int
        _lib.orc_action.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32,
                                    ctypes.c_int32]
        _lib.orc_max_threads.restype = ctypes.c_int
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def stride(h, w):
    return ((h * w + 7) // 8 + 15) // 16 * 16


class OracleBatch:
    """E envs on the host, same array layouts as mapfx.MapfGridBatch."""

    def __init__(self, bits, init_pos, goals, h, w, limit=10000, step_reward=-0.01,
                 collide_reward=-10, env_offset=0, nthreads=None):
        self.init_pos = np.ascontiguousarray(init_pos, dtype=np.int32)
        self.goal = np.ascontiguousarray(goals, dtype=np.int32)
        self.E, self.N = self.init_pos.shape[:2]
        self.H, self.W = h, w
        self.bits = np.ascontiguousarray(bits, dtype=np.uint8)
        if self.bits.ndim == 1:
            self.bits = self.bits[None]
        self.cfg = OrcCfg(H=h, W=w, N=self.N, E=self.E, env_offset=env_offset, limit=limit,
                          step_rew=float(step_reward), collide_rew=float(collide_reward),
                          map_shared=1 if (self.bits.shape[0] == 1 and self.E != 1) else 0,
                          map_stride=stride(h, w))
        self.nthreads = nthreads or os.cpu_count() or 1
        self.obs_dt = np.int8 if self.N <= 127 else np.int16
        self.reset()

    def reset(self):
        self.pos = self.init_pos.copy()
        self.done = np.zeros((self.E, self.N), np.uint8)
        self.t = np.zeros(self.E, np.int32)
        self.steps = np.zeros((self.E, self.N), np.int32)

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.int32)
        out = {"reward": np.zeros(self.E, np.float64), "node": np.zeros((self.E, self.N), np.uint8),
               "edge": np.zeros((self.E, self.N), np.uint16)}
        bad = lib().orc_step(ctypes.byref(self.cfg), _p(self.pos), _p(self.goal), _p(self.done),
                             _p(self.t), _p(self.steps), _p(self.bits), _p(a), _p(out["reward"]),
                             _p(out["node"]), _p(out["edge"]), ctypes.c_int(self.nthreads))
        out["bad"] = bad
        return out

    def observe(self, window=5, psize=10, full=True, win=True, primal=False):
        E, N = self.E, self.N
        out = {"avail": np.zeros((E, N), np.uint8), "term": np.zeros(E, np.uint8)}
        if full:
            out["obs_full"] = np.zeros((E, self.H * self.W), self.obs_dt)
        if win:
            out["obs_window"] = np.zeros((E, N, 2, window, window), self.obs_dt)
        if primal:
            out["obs_primal"] = np.zeros((E, N, 4, psize, psize), np.uint8)
            out["primal_vec"] = np.zeros((E, N, 3), np.float64)
        lib().orc_observe(ctypes.byref(self.cfg), _p(self.pos), _p(self.goal), _p(self.done),
                          _p(self.bits), _p(out["avail"]), _p(out["term"]), _p(out.get("obs_full")),
                          _p(out.get("obs_window")), ctypes.c_int(window),
                          _p(out.get("obs_primal")), _p(out.get("primal_vec")), ctypes.c_int(psize),
                          ctypes.c_int(self.nthreads))
        return out

    def rollout(self, T, seed, t0=0, window=5):
        E, N = self.E, self.N
        out = {"reward": np.zeros(E, np.float64), "node": np.zeros((E, N), np.uint8),
               "edge": np.zeros((E, N), np.uint16), "avail": np.zeros((E, N), np.uint8),
               "obs_window": np.zeros((E, N, 2, window, window), self.obs_dt)}
        lib().orc_rollout(ctypes.byref(self.cfg), ctypes.c_int32(T), ctypes.c_uint64(seed),
                          ctypes.c_int32(t0), _p(self.pos), _p(self.goal), _p(self.done),
                          _p(self.t), _p(self.steps), _p(self.bits), _p(out["reward"]),
                          _p(out["node"]), _p(out["edge"]), _p(out["avail"]),
                          _p(out["obs_window"]), ctypes.c_int(window), ctypes.c_int(self.nthreads))
        return out
