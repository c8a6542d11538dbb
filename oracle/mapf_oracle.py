"""CPU ORACLE — test infrastructure only, never product code.

Plain-Python restatement of the reference MAPF_GRID step / observation path
(DongmingShenDS/MAPF-MARL, `MARL-curve-main/src/envs/mapf_gridworld.py`), the
marl_partial observation window (`src/envs/marl_partial.py:323-342`) and the
PRIMAL window observation (`src/envs/mapf_primal.py:343-386`).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import this module, and only as the *checker*.  The product path (the HIP
library behind `include/mapfx.h`) never calls into `oracle/`.

Parity pin: this restatement is checked bit-for-bit against golden vectors that
`tests/golden/gen_fixtures.py` produced by importing and running the reference
Python env in the build container.  Every function
cites the reference file:line it restates; paths below are relative to
`MARL-curve-main/src/`.

Conventions (identical to the reference):
  * positions are (row, col) == the reference's (pos[0], pos[1]);
  * grid G[r][c] = -1 for any map char other than '.', else 0
    (envs/mapf_gridworld.py:282-288);
  * occ = G + number of agents on the cell (envs/mapf_gridworld.py:132-135,297-299);
  * action deltas: 0:(-1,0) 1:(+1,0) 2:(0,-1) 3:(0,+1) 4:(0,0)
    (envs/mapf_gridworld.py:323-332, ACTION_MEANING :483-489).
"""
from __future__ import annotations

import math

import numpy as np

# envs/mapf_gridworld.py:323-332
DELTAS = ((-1, 0), (1, 0), (0, -1), (0, 1), (0, 0))


def grid_from_map_text(text: str) -> np.ndarray:
    """MovingAI .map text -> G (H, W) int8 in {-1, 0}.

    envs/mapf_gridworld.py:421-428 (`__setup_grid`: drop 4 header lines, rstrip)
    and :282-288 (`__create_grid`: '.' -> 0, anything else -> -1).
    The reference indexes `_grid[i][j]` with i < shape[1], j < shape[0], so it
    only works for square maps (quirk 5); this restatement keeps H x W general.
    """
    rows = [row.rstrip() for row in text.splitlines()][4:]
    rows = [r for r in rows]
    h = len(rows)
    w = len(rows[0])
    g = np.zeros((h, w), dtype=np.int8)
    for i in range(h):
        for j in range(w):
            g[i, j] = 0 if rows[i][j] == '.' else -1
    return g


def occupancy(grid: np.ndarray, pos) -> np.ndarray:
    """occ = G + agent counts (envs/mapf_gridworld.py:132-135, 290-299)."""
    occ = grid.astype(np.int64).copy()
    for (r, c) in pos:
        occ[r, c] += 1
    return occ


def _in_bounds(shape, r, c):
    # envs/mapf_gridworld.py:270-272
    return 0 <= r < shape[0] and 0 <= c < shape[1]


def avail_actions(occ: np.ndarray, pos) -> list:
    """envs/mapf_gridworld.py:198-224: 1 iff in-bounds and occ != -1; stay always 1."""
    out = []
    for (r, c) in pos:
        v = [0, 0, 0, 0, 0]
        for d in range(4):
            nr, nc = r + DELTAS[d][0], c + DELTAS[d][1]
            if _in_bounds(occ.shape, nr, nc) and occ[nr, nc] != -1:
                v[d] = 1
        v[4] = 1
        out.append(v)
    return out


class GridEnvState:
    """State of one MAPF_GRID env, stepped exactly as the reference does.

    `step` restates envs/mapf_gridworld.py:85-141 (Appendix A of SURVEY.md).
    """

    def __init__(self, grid, init_pos, goals, episode_limit=10000,
                 step_reward=-0.01, collide_reward=-10):
        self.grid = np.asarray(grid, dtype=np.int8)
        self.init_pos = [tuple(int(v) for v in p) for p in init_pos]
        self.goals = [tuple(int(v) for v in p) for p in goals]
        self.n = len(self.init_pos)
        self.episode_limit = episode_limit
        self.step_reward = step_reward
        self.collide_reward = collide_reward
        self.reset()

    # envs/mapf_gridworld.py:70-83
    def reset(self):
        self.t = 0
        self.steps = [0] * self.n
        self.done = [False] * self.n
        self.node = [0] * self.n
        self.edge = [0] * self.n
        self.pos = list(self.init_pos)
        self.occ = occupancy(self.grid, self.pos)

    def step(self, actions):
        """Returns (R, done(list copy), node, edge, envc).  R keeps the
        reference's Python type: `sum()` of ints stays int (quirk 4)."""
        n = self.n
        actions = [int(a) for a in actions]
        assert len(actions) == n                       # :91
        assert all(a in (0, 1, 2, 3, 4) for a in actions)  # :92
        self.t += 1                                    # :93
        rewards = [0] * n                              # :94
        new = [self.pos[i] if self.done[i] else None for i in range(n)]  # :95
        envc = [False] * n
        for i, a in enumerate(actions):                # :99-118
            new_pos = self.pos[i]
            if not self.done[i]:
                self.steps[i] += 1                     # :102
                # __agent_step :319-342 (reads PRE-step occ, quirk 1)
                r, c = self.pos[i]
                if a == 4:
                    new_pos, flag = (r, c), False
                else:
                    nr, nc = r + DELTAS[a][0], c + DELTAS[a][1]
                    if not _in_bounds(self.occ.shape, nr, nc):
                        new_pos, flag = (r, c), True
                    elif self.occ[nr, nc] == -1:
                        new_pos, flag = (r, c), True
                    else:
                        new_pos, flag = (nr, nc), False
                new[i] = new_pos
                envc[i] = flag
                if flag:
                    rewards[i] += self.collide_reward  # :105-108
                rewards[i] += self.step_reward         # :110
            if new_pos == self.goals[i]:               # :112-114, 313-317
                self.done[i] = True
            if self.t >= self.episode_limit:           # :116-117
                self.done[i] = True
        # __count_node_collision :344-362 (includes done agents)
        groups = {}
        for i, p in enumerate(new):
            groups.setdefault(p, []).append(i)
        node = [0] * n
        for p, members in groups.items():
            if len(members) > 1:
                for i in members:
                    node[i] += 1
        # __count_edge_collision :364-383 with key(p) = H*p[1] + p[0] (:465-468)
        h = self.grid.shape[0]
        old_k = [h * p[1] + p[0] for p in self.pos]
        new_k = [h * p[1] + p[0] for p in new]
        edge = [0] * n
        for i in range(n):
            if old_k[i] == new_k[i]:
                continue
            for j in range(n):
                if old_k[j] != new_k[i] or j == i:
                    continue
                if new_k[j] == old_k[i] and new_k[j] != new_k[i]:
                    edge[i] += 1
        # :127-130 reward order: node then edge, per agent
        for i in range(n):
            rewards[i] += self.collide_reward * node[i]
            rewards[i] += self.collide_reward * edge[i]
        # :132-135 rebuild occupancy from new positions
        self.pos = list(new)
        self.occ = occupancy(self.grid, self.pos)
        self.node, self.edge = node, edge
        # :141 `sum(rewards)`: explicit left fold (CPython <= 3.11 semantics)
        total = 0
        for r in rewards:
            total = total + r
        return total, list(self.done), node, edge, envc

    def avail(self):
        return avail_actions(self.occ, self.pos)

    def full_obs(self):
        """envs/mapf_gridworld.py:143-183, 190-192: row-major occ, per agent."""
        return self.occ.reshape(-1).copy()


def window_obs(occ: np.ndarray, pos, window: int = 5) -> np.ndarray:
    """marl_partial window, envs/marl_partial.py:323-342 (flatten order :374).

    Returns (N, 2, W, W) int64: [obstacle_map, agents_map].
    """
    n = len(pos)
    out = np.zeros((n, 2, window, window), dtype=np.int64)
    half = window // 2
    for a, (r, c) in enumerate(pos):
        tr, tc = r - half, c - half
        for i in range(tr, tr + window):
            for j in range(tc, tc + window):
                if not _in_bounds(occ.shape, i, j):
                    out[a, 0, i - tr, j - tc] = 1
                    continue
                v = occ[i, j]
                if v == -1:
                    out[a, 0, i - tr, j - tc] = 1
                elif v > 0:
                    out[a, 1, i - tr, j - tc] = v
    return out


def primal_obs(grid: np.ndarray, pos, goals, size: int = 10, agents=None):
    """PRIMAL `_observe`, envs/mapf_primal.py:343-386, applied to a MAPF_GRID
    state.  PRIMAL's world holds one agent id per cell (an agent overrides the
    obstacle it stands on); with stacked agents every agent on a cell counts as
    visible.  Parity with the reference is pinned on distinct positions/goals.

    Returns maps (N, 4, s, s) uint8 [poss, goal, goals, obs] and vec (N, 3) f64;
    with `agents` (a list of indices) only those rows are filled.
    """
    n = len(pos)
    # Python ints, as PRIMAL's State holds them (mapf_primal.py:53-66): numpy
    # scalars would route `** .5` through numpy's sqrt fast path, not libm pow.
    pos = [(int(r), int(c)) for r, c in pos]
    goals = [(int(r), int(c)) for r, c in goals]
    h, w = grid.shape
    cnt = np.zeros((h, w), dtype=np.int64)
    for (r, c) in pos:
        cnt[r, c] += 1
    maps = np.zeros((n, 4, size, size), dtype=np.uint8)
    vec = np.zeros((n, 3), dtype=np.float64)
    half = size // 2
    for a in (range(n) if agents is None else agents):
        pr, pc = pos[a]
        tr, tc = pr - half, pc - half
        visible = []
        for i in range(tr, tr + size):
            for j in range(tc, tc + size):
                if i >= h or i < 0 or j >= w or j < 0:
                    maps[a, 3, i - tr, j - tc] = 1         # :356-359
                    continue
                if grid[i, j] == -1 and cnt[i, j] == 0:
                    maps[a, 3, i - tr, j - tc] = 1         # :360-362
                if cnt[i, j] > 0:
                    maps[a, 0, i - tr, j - tc] = 1         # :363-365, 369-372
                if (i, j) == tuple(goals[a]):
                    maps[a, 1, i - tr, j - tc] = 1         # :366-368
        for b in range(n):
            if b == a:
                continue
            br, bc = pos[b]
            if tr <= br < tr + size and tc <= bc < tc + size:
                visible.append(b)
        for b in visible:                                   # :374-378
            x, y = goals[b]
            mr = max(tr, min(tr + size - 1, x))
            mc = max(tc, min(tc + size - 1, y))
            maps[a, 2, mr - tr, mc - tc] = 1
        dx = goals[a][0] - pr                               # :380-386
        dy = goals[a][1] - pc
        mag = (dx ** 2 + dy ** 2) ** .5                     # libm pow (quirk 8)
        if mag != 0:
            dx = dx / mag
            dy = dy / mag
        vec[a] = (dx, dy, mag)
    return maps, vec


def goal_vectors(pos, goals):
    """envs/mapf_gridworld.py:451-463 (computed by get_obs, never emitted)."""
    out = []
    for (pr, pc), (gr, gc) in zip(pos, goals):
        d0, d1 = gr - pr, gc - pc
        norm = math.sqrt(d0 ** 2 + d1 ** 2)
        out.append(((0, 0) if norm == 0 else (d0 / norm, d1 / norm), norm))
    return out
