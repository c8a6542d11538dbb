"""CPU restatement of PRIMAL's sequential dynamics -- TEST
INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline may use it).

Follows MARL-curve-main/src/envs/mapf_primal.py (paths relative to it):
  State.moveAgent   :103-135  (status 1 reached/stayed on goal, 2 left goal, 0 moved,
                               -1 out of bounds, -2 wall, -3 robot)
  MAPFEnv._step     :549-637  reward table :579-596 (JOINT = False);
                               the stay-on-goal blocking term (:583, needs the
                               un-vendored od_mstar3) is defined as 0: parity unpinned
  State.done        :159-166
  _listNextValidActions :639-667 (opposite of the previous action removed)
  _observe          :343-386  via oracle.mapf_oracle.primal_obs
  DIAGONAL_MOVEMENT (:175): actions 5..8 (dirDict :28), agents_past (:55-66,
  :110-112, :129-131) and State.diagonalCollision (:77-99; integer coordinates,
  so np.isclose of the midpoints is equality of the coordinate sums)
Pinned by tests/golden/pd_*.npz (tests/golden/gen_primal_dyn_fixtures.py).
"""
from __future__ import annotations

import numpy as np

from .mapf_oracle import primal_obs

ACTION_COST, IDLE_COST, GOAL_REWARD, COLLISION_REWARD = -0.3, -.5, 0.0, -2.  # :25
DIRS = {0: (0, 0), 1: (0, 1), 2: (1, 0), 3: (0, -1), 4: (-1, 0),             # :28
        5: (1, 1), 6: (1, -1), 7: (-1, -1), 8: (-1, 1)}
OPPOSITE = {0: -1, 1: 3, 2: 4, 3: 1, 4: 2, 5: 7, 6: 8, 7: 5, 8: 6}             # :26


class PrimalWorld:
    def __init__(self, grid, starts, goals, size=10, diagonal=False, past=None):
        self.grid = np.asarray(grid, dtype=np.int64)
        self.h, self.w = self.grid.shape
        self.pos = [tuple(int(v) for v in p) for p in starts]
        self.goals = [tuple(int(v) for v in p) for p in goals]
        self.size = int(size)
        self.n = len(self.pos)
        self.diagonal = bool(diagonal)
        # agents_past (:55-66): equal to the positions in a fresh world
        self.past = list(self.pos) if past is None else [tuple(int(v) for v in p) for p in past]

    def diagonal_collision(self, aid, new):  # State.diagonalCollision :77-99 (aid 0-based)
        last = self.pos[aid]
        for b in range(self.n):
            if b == aid:
                continue
            pa, pr = self.past[b], self.pos[b]
            if pa[0] + pr[0] == last[0] + new[0] and pa[1] + pr[1] == last[1] + new[1]:
                return True
        return False

    def _occupant(self, cell):
        for b, p in enumerate(self.pos):
            if p == cell:
                return b
        return -1

    def move(self, aid, action):  # State.moveAgent :103-135 (aid 0-based)
        ax, ay = self.pos[aid]
        if action == 0:
            self.past[aid] = self.pos[aid]
            return 1 if self.goals[aid] == (ax, ay) else 0
        dx, dy = DIRS[action]
        nx, ny = ax + dx, ay + dy
        if nx >= self.h or nx < 0 or ny >= self.w or ny < 0:
            return -1
        if self._occupant((nx, ny)) >= 0:   # state > 0 (an agent id) takes precedence
            return -3
        if self.grid[nx, ny] < 0:
            return -2
        if self.diagonal and self.diagonal_collision(aid, (nx, ny)):
            return -3
        self.past[aid] = self.pos[aid]
        self.pos[aid] = (nx, ny)
        if self.goals[aid] == (nx, ny):
            return 1
        if self._goal_owner((nx, ny)) != aid and self._goal_owner((ax, ay)) == aid:
            return 2
        return 0

    def _goal_owner(self, cell):
        for b, g in enumerate(self.goals):
            if g == cell:
                return b
        return -1

    def done(self):  # :159-166
        return all(self.pos[b] == self.goals[b] for b in range(self.n))

    def next_mask(self, aid, prev_action):  # :639-667
        ax, ay = self.pos[aid]
        acts = [0]
        for a in range(1, 9 if self.diagonal else 5):
            dx, dy = DIRS[a]
            nx, ny = ax + dx, ay + dy
            if nx >= self.h or nx < 0 or ny >= self.w or ny < 0:
                continue
            if self._occupant((nx, ny)) >= 0 or self.grid[nx, ny] < 0:
                continue
            if self.diagonal and self.diagonal_collision(aid, (nx, ny)):
                continue
            acts.append(a)
        if OPPOSITE[prev_action] in acts:
            acts.remove(OPPOSITE[prev_action])
        m = 0
        for a in acts:
            m |= 1 << a
        return m

    def step(self, aid, action):
        """MAPFEnv._step((aid + 1, action)) -> (maps [4,s,s], vec [3], reward, done,
        next_mask, on_goal, blocking, valid)."""
        status = self.move(aid, action)
        if action == 0:
            reward = GOAL_REWARD + 0 if status == 1 else IDLE_COST
        else:
            if status == 1:
                reward = GOAL_REWARD
            elif status in (-1, -2, -3):
                reward = COLLISION_REWARD
            else:
                reward = ACTION_COST
        maps, vec = primal_obs(self._world_grid(), self.pos, self.goals, self.size, agents=[aid])
        return (maps[aid], vec[aid], float(reward), self.done(), self.next_mask(aid, action),
                self.pos[aid] == self.goals[aid], False, status >= 0)

    def _world_grid(self):
        return self.grid
