"""ctypes binding of the C ABI declared in include/mapfx.h (libmapfx.so).

torch is imported first so that the HIP runtime torch already loaded
(libamdhip64.so.7) is the one libmapfx.so binds to: device pointers and
streams then come straight from torch tensors / torch.cuda streams.

There is no fallback: if the library is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede loading libmapfx.so: shared HIP runtime)

LIB_NAME = "libmapfx.so"
LIB_PATH = os.environ.get("MAPFX_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

MAPFX_OBS_FULL = 1
MAPFX_OBS_WINDOW = 2
MAPFX_OBS_PRIMAL = 4
MAPFX_I8, MAPFX_I32, MAPFX_I64 = 0, 1, 2

c_i32, c_i64, c_u64, c_f64, c_vp = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64,
                                    ctypes.c_double, ctypes.c_void_p)


class Cfg(ctypes.Structure):
    _fields_ = [("H", c_i32), ("W", c_i32), ("n_agents", c_i32), ("n_envs", c_i32),
                ("env_offset", c_i64), ("episode_limit", c_i32), ("step_reward", c_f64),
                ("collide_reward", c_f64), ("obs_mode", c_i32), ("window", c_i32),
                ("primal_size", c_i32), ("map_shared", c_i32)]


class State(ctypes.Structure):
    _fields_ = [("pos", c_vp), ("goal", c_vp), ("init_pos", c_vp), ("done", c_vp), ("t", c_vp),
                ("steps", c_vp), ("map_bits", c_vp)]


class Out(ctypes.Structure):
    _fields_ = [("reward", c_vp), ("reward_f32", c_vp), ("term", c_vp), ("node", c_vp),
                ("edge", c_vp), ("avail", c_vp), ("obs_full", c_vp), ("obs_window", c_vp),
                ("obs_primal", c_vp), ("primal_vec", c_vp), ("traj_pos", c_vp),
                ("traj_done", c_vp), ("traj_t", c_vp), ("err", c_vp), ("obs_window_occ", c_vp)]


class Info(ctypes.Structure):
    _fields_ = [("lanes_per_env", c_i32), ("agents_per_lane", c_i32), ("envs_per_block", c_i32),
                ("block_threads", c_i32), ("lds_bytes", c_i32), ("cell_bytes", c_i32),
                ("pad", c_i32)]


class PCfg(ctypes.Structure):  # include/mapfx_partial.h
    _fields_ = [("H", c_i32), ("W", c_i32), ("n_agents", c_i32), ("n_envs", c_i32),
                ("env_offset", c_i64), ("episode_limit", c_i32), ("obs_window", c_i32),
                ("obs_knn_agents", c_i32), ("map_shared", c_i32), ("move_reward", c_f64),
                ("stay_reward", c_f64), ("stay_goal_reward", c_f64),
                ("node_collide_reward", c_f64), ("edge_collide_reward", c_f64),
                ("env_collide_reward", c_f64), ("complete_reward", c_f64),
                ("complete_fac", c_f64), ("gamma", c_f64)]


class PState(ctypes.Structure):
    _fields_ = [(k, c_vp) for k in ("pos", "goal", "init_pos", "steps", "at_goal", "done",
                                    "goal_cost", "node", "edge", "t", "terminated", "total_coll",
                                    "map_bits", "goal_dist", "pdist", "pnbr")]


class POut(ctypes.Structure):
    _fields_ = [(k, c_vp) for k in ("reward", "obs", "state", "avail", "err")]


class QCfg(ctypes.Structure):  # include/mapfx_primal.h
    _fields_ = [(k, c_i32) for k in ("H", "W", "n_agents", "n_envs", "obs_size", "map_shared",
                                     "diagonal")]


class QState(ctypes.Structure):
    _fields_ = [(k, c_vp) for k in ("pos", "goal", "map_bits", "past")]


class QOut(ctypes.Structure):
    _fields_ = [(k, c_vp) for k in ("reward", "done", "next_mask", "on_goal", "valid", "obs", "vec",
                                    "err")]


# every symbol include/mapfx.h, include/mapfx_partial.h and include/mapfx_primal.h declare
# (checked by tests/test_abi_exports.py)
EXPORTS = ("mapfx_abi_version", "mapfx_last_error", "mapfx_build_id", "mapfx_last_kernel",
           "mapfx_map_stride", "mapfx_obs_elem_size",
           "mapfx_edge_elem_size",
           "mapfx_create", "mapfx_destroy", "mapfx_query", "mapfx_reset", "mapfx_step",
           "mapfx_observe", "mapfx_rollout", "mapfx_rollout_timed", "mapfx_gen_actions", "mapfx_action",
           "mapfx_pack_compact",
           "mapfx_partial_create", "mapfx_partial_destroy", "mapfx_partial_obs_dim",
           "mapfx_partial_goal_dist_elem_size",
           "mapfx_partial_goal_dist", "mapfx_partial_reset", "mapfx_partial_step",
           "mapfx_partial_observe", "mapfx_primal_create", "mapfx_primal_destroy",
           "mapfx_primal_act", "mapfx_primal_act_timed", "mapfx_runner_begin", "mapfx_runner_actions", "mapfx_runner_post",
           "mapfx_runner_step", "mapfx_host_ring_alloc", "mapfx_host_ring_free")


class ERows(ctypes.Structure):  # include/mapfx_runner.h mapfx_episode_rows
    _fields_ = [("max_t", c_i32)] + [f for k in ("obs", "state", "avail", "actions", "onehot",
                                                 "reward", "terminated", "filled")
                                     for f in ((k, c_vp), (k + "_sb", c_i64), (k + "_st", c_i64))]


class RState(ctypes.Structure):  # include/mapfx_runner.h mapfx_runner_state
    _fields_ = [("B", c_i32), ("N", c_i32), ("D", c_i32)] + [
        (k, c_vp) for k in ("alive", "alive_prev", "bs", "counts", "ep_return", "ep_length",
                            "env_steps", "env_actions", "bs_inv")]


ABI_VERSION = 6  # include/mapfx.h MAPFX_ABI_VERSION


class MapfxError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("%s not built: run `python -c 'import __graft_entry__ as g; g.build()'`"
                          % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    sig = {
        "mapfx_abi_version": (c_i32, []),
        "mapfx_last_error": (ctypes.c_char_p, []),
        "mapfx_build_id": (ctypes.c_char_p, []),
        "mapfx_last_kernel": (ctypes.c_char_p, []),
        "mapfx_map_stride": (c_i64, [c_i32, c_i32]),
        "mapfx_obs_elem_size": (c_i32, [c_i32]),
        "mapfx_edge_elem_size": (c_i32, [c_i32]),
        "mapfx_create": (c_i32, [P(Cfg), P(c_vp)]),
        "mapfx_destroy": (None, [c_vp]),
        "mapfx_query": (c_i32, [c_vp, P(Info)]),
        "mapfx_reset": (c_i32, [c_vp, P(State), c_vp, P(Out), c_vp]),
        "mapfx_step": (c_i32, [c_vp, P(State), c_vp, c_i32, P(Out), c_vp]),
        "mapfx_observe": (c_i32, [c_vp, P(State), P(Out), c_vp]),
        "mapfx_rollout": (c_i32, [c_vp, P(State), c_i32, c_vp, c_i32, c_u64, c_i32, c_i32, P(Out),
                                  c_vp]),
        "mapfx_rollout_timed": (c_i32, [c_vp, P(State), c_i32, c_vp, c_i32, c_u64, c_i32, c_i32,
                                        P(Out), c_vp, c_vp, c_vp]),
        "mapfx_gen_actions": (c_i32, [c_vp, c_u64, c_i32, c_i32, c_vp, c_vp]),
        "mapfx_action": (c_i32, [c_u64, c_i64, c_i32, c_i32]),
        "mapfx_pack_compact": (c_i32, [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
        "mapfx_partial_create": (c_i32, [P(PCfg), P(c_vp)]),
        "mapfx_partial_destroy": (None, [c_vp]),
        "mapfx_partial_obs_dim": (c_i32, [c_vp]),
        "mapfx_partial_goal_dist_elem_size": (c_i32, [c_i32, c_i32]),
        "mapfx_partial_goal_dist": (c_i32, [c_vp, P(PState), c_vp, c_vp]),
        "mapfx_partial_reset": (c_i32, [c_vp, P(PState), c_vp, P(POut), c_vp]),
        "mapfx_partial_step": (c_i32, [c_vp, P(PState), c_vp, c_i32, P(POut), c_vp]),
        "mapfx_partial_observe": (c_i32, [c_vp, P(PState), P(POut), c_vp]),
        "mapfx_primal_create": (c_i32, [P(QCfg), P(c_vp)]),
        "mapfx_primal_destroy": (None, [c_vp]),
        "mapfx_primal_act": (c_i32, [c_vp, P(QState), c_vp, c_vp, c_i32, P(QOut), c_vp]),
        "mapfx_primal_act_timed": (c_i32, [c_vp, P(QState), c_vp, c_vp, c_i32, P(QOut), c_vp, c_vp, c_vp]),
        "mapfx_runner_begin": (c_i32, [P(RState), P(POut), P(ERows), c_vp]),
        "mapfx_runner_actions": (c_i32, [P(RState), c_vp, c_i32, c_i64, c_i32, P(ERows), c_vp]),
        "mapfx_runner_post": (c_i32, [P(RState), c_vp, P(POut), c_i32, c_vp, P(ERows), c_vp]),
        "mapfx_runner_step": (c_i32, [c_vp, P(PState), P(POut), P(RState), c_vp, c_i32, c_i64, c_i32,
                                      c_vp, P(ERows), c_vp]),
        "mapfx_host_ring_alloc": (c_i32, [c_i32, P(c_vp), P(c_vp)]),
        "mapfx_host_ring_free": (None, [c_vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mapfx_abi_version() != ABI_VERSION:
        raise ImportError("%s has ABI %d, the bindings expect %d: rebuild it"
                          % (LIB_PATH, lib.mapfx_abi_version(), ABI_VERSION))
    return lib


lib = _load()


def check(rc: int, what: str):
    if rc != 0:
        msg = lib.mapfx_last_error()
        raise MapfxError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))


def build_id() -> str:
    """mapfx_build_id(): "src=<sources sha256[:16]> git=<head>[+dirty]" of the loaded library."""
    return lib.mapfx_build_id().decode()


def last_kernel() -> str:
    """mapfx_last_kernel(): the rocprofv3 name of this thread's last env-kernel launch."""
    return lib.mapfx_last_kernel().decode()


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()
