"""Host-side map / scenario feeders for the batched step.

* MovingAI `.map` / `.scen` loaders with the reference's exact semantics
  (MARL-curve-main/src/envs/mapf_gridworld.py:421-449): 4 header lines, any
  char other than '.' is an obstacle, scen columns 4..7 = start x, start y,
  goal x, goal y used as (row, col) — the transposition the reference makes
  (SURVEY.md quirk 2).
* Synthetic instances for the benchmark configs: i.i.d.
  obstacles and distinct free starts/goals per env, all drawn from counter-based
  splitmix64 streams keyed by the global env id (mapfx.rng).
* Bitmap packing into the device layout of include/mapfx.h (bit r*W+c,
  LSB-first, mapfx_map_stride bytes per env).
"""
from __future__ import annotations

import io

import numpy as np

from . import rng

STREAM_OBST, STREAM_START, STREAM_GOAL = 1, 2, 3


def map_stride(h: int, w: int) -> int:
    """Bytes per env bitmap: ceil(H*W/8) rounded up to 16 (mapfx_map_stride)."""
    return ((h * w + 7) // 8 + 15) // 16 * 16


def parse_map_text(text: str) -> np.ndarray:
    """envs/mapf_gridworld.py:421-428 + :282-288 -> int8 grid (-1 obstacle, 0 free).

    Lines are split exactly as the reference's text-mode `f.readlines()` splits
    them (universal newlines: \\n, \\r\\n, \\r -- not \\v, \\f or \\u2028), then
    rstrip()ed; 4 header lines.  A row shorter than row 0 raises IndexError, as
    the reference's `_original_grid[i][j]` does; longer rows are cut at row 0's
    width (the reference never reads past it)."""
    rows = [row.rstrip() for row in io.StringIO(text, newline=None).readlines()][4:]
    if not rows or not rows[0]:
        raise AssertionError("empty map")
    w = len(rows[0])
    arr = np.full((len(rows), w), -1, dtype=np.int8)
    for i, row in enumerate(rows):
        if len(row) < w:
            raise IndexError("string index out of range (map row %d has %d of %d cells)"
                             % (i, len(row), w))
        for j, ch in enumerate(row[:w]):
            if ch == ".":
                arr[i, j] = 0
    return arr


def load_map(path: str) -> np.ndarray:
    with open(path, "r") as f:
        return parse_map_text(f.read())


def parse_scen_lines(lines):
    """Scenario lines -> list of ((sx, sy), (gx, gy)) as the reference reads them
    (envs/mapf_gridworld.py:442-445: `f_line.replace('\\t', ',').split(',')`)."""
    out = []
    for f_line in lines:
        parts = f_line.replace("\t", ",").split(",")
        out.append(((int(parts[4]), int(parts[5])), (int(parts[6]), int(parts[7]))))
    return out


def pack_bits(grids: np.ndarray) -> np.ndarray:
    """[E, H, W] (nonzero = obstacle) -> uint8 [E, map_stride(H, W)] device bitmaps."""
    grids = np.asarray(grids)
    if grids.ndim == 2:
        grids = grids[None]
    e, h, w = grids.shape
    flat = (grids.reshape(e, h * w) != 0)
    packed = np.packbits(flat, axis=1, bitorder="little")
    out = np.zeros((e, map_stride(h, w)), dtype=np.uint8)
    out[:, : packed.shape[1]] = packed
    return out


def unpack_bits(bits: np.ndarray, h: int, w: int) -> np.ndarray:
    """Inverse of pack_bits -> int8 [E, H, W] in {-1, 0}."""
    bits = np.asarray(bits, dtype=np.uint8)
    if bits.ndim == 1:
        bits = bits[None]
    flat = np.unpackbits(bits, axis=1, count=h * w, bitorder="little")
    return -(flat.reshape(-1, h, w).astype(np.int8))


def warehouse_grid(size: int = 64) -> np.ndarray:
    """Square synthetic warehouse (BASELINE configs[2]): obstacle
    border, an open staging zone on the left, 10x2 shelf blocks separated by
    1-cell aisles — the pattern of warehouse-10-20-10-2-1.map:5-16, squared
    because MAPF_GRID only runs square maps (quirk 5)."""
    g = np.zeros((size, size), dtype=np.int8)
    g[0, :] = g[-1, :] = -1
    g[:, 0] = g[:, -1] = -1
    left = max(2, size // 7)
    for r in range(1, size - 2):
        if (r - 1) % 3 == 0:
            continue  # aisle row
        for c in range(left, size - 1):
            if (c - left) % 11 < 10:
                g[r, c] = -1
    return g


def _pick_cells(keys: np.ndarray, free: np.ndarray, n: int) -> np.ndarray:
    """Per row, the n free cells with the smallest keys (distinct by construction)."""
    k = np.where(free, keys, np.uint64(0xFFFFFFFFFFFFFFFF))
    if np.any(free.sum(axis=1) < n):
        raise ValueError("an env has fewer than n_agents free cells")
    idx = np.argpartition(k, n - 1, axis=1)[:, :n]
    # order the chosen cells by key so agent order is deterministic
    kk = np.take_along_axis(k, idx, axis=1)
    order = np.argsort(kk, axis=1, kind="stable")
    return np.take_along_axis(idx, order, axis=1)


def synthetic_instances(n_envs: int, h: int, w: int, n_agents: int, p_obstacle: float = 0.10,
                        seed: int = 1, env_offset: int = 0, shared_grid: np.ndarray | None = None):
    """Random maps + distinct free starts / goals for envs [env_offset, env_offset+E).

    Returns dict(grid=int8 [E or 1, H, W], bits=uint8 [E or 1, stride],
    init_pos=int32 [E, N, 2], goals=int32 [E, N, 2]).
    """
    env_ids = np.arange(env_offset, env_offset + n_envs, dtype=np.int64)
    hw = h * w
    if shared_grid is not None:
        grid = np.asarray(shared_grid, dtype=np.int8).reshape(1, h, w)
        free = np.broadcast_to(grid.reshape(1, hw) == 0, (n_envs, hw))
    else:
        thr = np.uint64(min(int(p_obstacle * 2.0 ** 64), 0xFFFFFFFFFFFFFFFF))
        ob = rng.cell_keys(seed, env_ids, hw, STREAM_OBST) < thr
        grid = -(ob.reshape(n_envs, h, w).astype(np.int8))
        free = ~ob
    starts = _pick_cells(rng.cell_keys(seed, env_ids, hw, STREAM_START), free, n_agents)
    goals = _pick_cells(rng.cell_keys(seed, env_ids, hw, STREAM_GOAL), free, n_agents)
    to_rc = lambda idx: np.stack([idx // w, idx % w], axis=-1).astype(np.int32)
    return {"grid": grid, "bits": pack_bits(grid), "init_pos": to_rc(starts),
            "goals": to_rc(goals)}



# ---------------------------------------------------------------------------
# PRIMAL random worlds: MAPFEnv._setWorld without a given
# world (MARL-curve-main/src/envs/mapf_primal.py:248-341).  Host code, as in the
# reference; it draws from the same global generators (numpy's legacy
# np.random and the stdlib `random`) in the same order, so the same seeds give
# the same world.
# ---------------------------------------------------------------------------
def _primal_region(world, memo, x, y):
    """getConnectedRegion (:250-274): free cells 4-connected to (x, y), as a set
    built by the reference's stack order (list(set) order then matches too).
    Every agent cell met on the way is memoised to the same set object."""
    if (x, y) in memo:
        return memo[(x, y)]
    seen = set()
    h, w = world.shape
    stack = [(x, y)]
    while stack:
        i, j = stack.pop()
        if i < 0 or i >= h or j < 0 or j >= w or world[i, j] == -1:
            continue
        if world[i, j] > 0:
            memo[(i, j)] = seen
        if (i, j) in seen:
            continue
        seen.add((i, j))
        stack.extend(((i + 1, j), (i, j + 1), (i - 1, j), (i, j - 1)))
    memo[(x, y)] = seen
    return seen


def _primal_place(world, num_agents, np_random, py_random):
    """Agents on random free cells, then each agent's goal on a random free cell of
    its own connected region (:290-306 / :316-336).  `world` is modified in place
    (agent ids written at the starts); returns the goals array."""
    locs = []
    a = 1
    while a <= num_agents:
        x, y = np_random.randint(0, world.shape[0]), np_random.randint(0, world.shape[1])
        if world[x, y] == 0:
            world[x, y] = a
            locs.append((x, y))
            a += 1
    goals = np.zeros(world.shape).astype(int)
    memo = {}
    a = 1
    while a <= num_agents:
        sx, sy = locs[a - 1]
        x, y = py_random.choice(list(_primal_region(world, memo, sx, sy)))
        if goals[x, y] == 0 and world[x, y] != -1:
            goals[x, y] = a
            a += 1
    return goals


def primal_world(num_agents, SIZE=(10, 40), PROB=(0, .5), world0=None, blank_world=False,
                 np_random=None, py_random=None):
    """(world, goals) in PRIMAL's encoding (-1 obstacle, agent id at its start /
    goal cell), as MAPFEnv(num_agents, SIZE=SIZE, PROB=PROB, world0=world0,
    blank_world=blank_world) would set them up.

    * world0 None: random square world -- obstacle density triangular over PROB,
      side drawn from (SIZE[0], mean, SIZE[1]) with p (.5, .25, .25) (:316-318).
    * blank_world: agents and goals placed on the given world0 (:290-306).
    The generators default to the global np.random / random modules (the
    reference's), so seeding those reproduces the reference's draws."""
    import random as _random
    npr = np.random if np_random is None else np_random
    pyr = _random if py_random is None else py_random
    if world0 is not None:
        if not blank_world:
            raise ValueError("a given world0 carries its own agents; pass blank_world=True to place them")
        world = np.array(world0)
        return world, _primal_place(world, num_agents, npr, pyr)
    prob = npr.triangular(PROB[0], .33 * PROB[0] + .66 * PROB[1], PROB[1])
    size = npr.choice([SIZE[0], SIZE[0] * .5 + SIZE[1] * .5, SIZE[1]], p=[.5, .25, .25])
    world = -(npr.rand(int(size), int(size)) < prob).astype(int)
    return world, _primal_place(world, num_agents, npr, pyr)
