"""Counter-based splitmix64 streams shared by the host (numpy) and the device.

The device versions live in csrc/mapfx.hip (`splitmix64`, `gen_action`); the
functions here are bit-identical numpy restatements used to build synthetic
instances on the host and to check the device action generator.  Every stream
is keyed by the GLOBAL env id, so an env's inputs do not depend on how envs are
sharded over ranks.
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
K_ENV = np.uint64(0xD1B54A32D192ED03)
K_T = np.uint64(0xABC98388FB8FAC03)
K_AGENT = np.uint64(0x8CB92BA72F3D8DD7)
K_CELL = np.uint64(0x9E6C63D0676A9A99)
K_STREAM = np.uint64(0xF1357AEA2E62A9C5)


def splitmix64(x):
    """Vectorised splitmix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def _mul(a, k):
    with np.errstate(over="ignore"):
        return np.asarray(a, dtype=np.uint64) * k


def gen_actions(seed, env_ids, t_ids, n_agents):
    """Actions in {0..4}: splitmix64(seed ^ env*K_ENV ^ t*K_T ^ agent*K_AGENT) % 5.

    Same formula as `gen_action` in csrc/mapfx.hip / `mapfx_action` in
    include/mapfx.h.  Returns int8 [len(t_ids), len(env_ids), n_agents].
    """
    env = np.asarray(env_ids, dtype=np.int64).astype(np.uint64)[None, :, None]
    t = (np.asarray(t_ids, dtype=np.int64) & 0xFFFFFFFF).astype(np.uint64)[:, None, None]
    ag = np.arange(n_agents, dtype=np.uint64)[None, None, :]
    k = np.uint64(seed) ^ _mul(env, K_ENV) ^ _mul(t, K_T) ^ _mul(ag, K_AGENT)
    return (splitmix64(k) % np.uint64(5)).astype(np.int8)


def cell_keys(seed, env_ids, n_cells, stream):
    """Per-(env, cell) uint64 keys of stream `stream` (obstacles, starts, goals)."""
    env = np.asarray(env_ids, dtype=np.int64).astype(np.uint64)[:, None]
    cell = np.arange(n_cells, dtype=np.uint64)[None, :]
    k = (np.uint64(seed) ^ _mul(env, K_ENV) ^ _mul(cell, K_CELL)
         ^ _mul(np.uint64(stream), K_STREAM))
    return splitmix64(k)
