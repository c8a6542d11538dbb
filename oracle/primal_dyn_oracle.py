"""CPU restatement of PRIMAL's sequential dynamics -- TEST
INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline may use it).

Follows MARL-curve-main/src/envs/mapf_primal.py (paths relative to it):
  State.moveAgent   :103-135  (status 1 reached/stayed on goal, 2 left goal, 0 moved,
                               -1 out of bounds, -2 wall, -3 robot)
  MAPFEnv._step     :549-637  reward table :579-596 (JOINT = False, no diagonal moves);
                               the stay-on-goal blocking term (:583, needs the
                               un-vendored od_mstar3) is defined as 0: parity unpinned
  State.done        :159-166
  _listNextValidActions :639-667 (opposite of the previous action removed)
  _observe          :343-386  via oracle.mapf_oracle.primal_obs
Pinned by tests/golden/pd_*.npz (tests/golden/gen_primal_dyn_fixtures.py).
"""
from __future__ import annotations

import numpy as np

from .mapf_oracle import primal_obs

ACTION_COST, IDLE_COST, GOAL_REWARD, COLLISION_REWARD = -0.3, -.5, 0.0, -2.  # :25
DIRS = {0: (0, 0), 1: (0, 1), 2: (1, 0), 3: (0, -1), 4: (-1, 0)}             # :28
OPPOSITE = {0: -1, 1: 3, 2: 4, 3: 1, 4: 2}                                     # :26


class PrimalWorld:
    def __init__(self, grid, starts, goals, size=10):
        self.grid = np.asarray(grid, dtype=np.int64)
        self.h, self.w = self.grid.shape
        self.pos = [tuple(int(v) for v in p) for p in starts]
        self.goals = [tuple(int(v) for v in p) for p in goals]
        self.size = int(size)
        self.n = len(self.pos)

    def _occupant(self, cell):
        for b, p in enumerate(self.pos):
            if p == cell:
                return b
        return -1

    def move(self, aid, action):  # State.moveAgent :103-135 (aid 0-based)
        ax, ay = self.pos[aid]
        if action == 0:
            return 1 if self.goals[aid] == (ax, ay) else 0
        dx, dy = DIRS[action]
        nx, ny = ax + dx, ay + dy
        if nx >= self.h or nx < 0 or ny >= self.w or ny < 0:
            return -1
        if self._occupant((nx, ny)) >= 0:   # state > 0 (an agent id) takes precedence
            return -3
        if self.grid[nx, ny] < 0:
            return -2
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
        for a in range(1, 5):
            dx, dy = DIRS[a]
            nx, ny = ax + dx, ay + dy
            if nx >= self.h or nx < 0 or ny >= self.w or ny < 0:
                continue
            if self._occupant((nx, ny)) >= 0 or self.grid[nx, ny] < 0:
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
