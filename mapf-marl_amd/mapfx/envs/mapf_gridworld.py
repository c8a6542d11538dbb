"""MAPF_GRID drop-in: the reference env's plugin surface over the HIP step.

Same constructor, methods, return types, RNG draw order and error behaviour as
MARL-curve-main/src/envs/mapf_gridworld.py (`MAPF_GRID`, lines 18-469); the
transition, collisions, rewards, occupancy, observations and available actions
are computed by the HIP kernel (mapfx.batch.MapfGridBatch, E = 1) instead of
the reference's Python loops.  Rendering (PIL base image, cv2 window) is out of
scope and not reproduced.
"""
from __future__ import annotations

import math
import os.path
import random

import numpy as np
import torch

from ..batch import MapfGridBatch
from ..maps import load_map, parse_scen_lines
from .multiagentenv import MultiAgentEnv

ACTION_MEANING = {0: "LEFT", 1: "RIGHT", 2: "UP", 3: "DOWN", 4: "STAY"}  # :483-489
PRE_IDS = {"obs": -1, "ept": 0, "agent": ""}                               # :491-495


class MAPF_GRID(MultiAgentEnv):
    """MultiAgentEnv, the base of customized envs"""

    def __init__(self, grid_file_path, agents_path, n_agents=4, episode_limit: int = 10000,
                 seed=None, render="human", step_reward=-0.01, collide_reward=-10, debug=False,
                 device=None):
        assert os.path.exists(grid_file_path)                         # :34
        self._grid_file_path = grid_file_path
        self._agent_path = agents_path
        self._seed = random.randint(0, 9999)                         # :37 (RNG draw order)
        np.random.seed(self._seed)                                   # :38
        if seed:
            self._seed = seed
        self._render_mode = render
        self._debug_mode = debug
        self._n_agents = n_agents
        self.n_agents = n_agents
        self.agents = [a for a in range(self._n_agents)]
        self.episode_limit = episode_limit
        self._step_count = None
        self._agent_init_pos = {a: None for a in self.agents}
        self._agent_goal_pos = {a: None for a in self.agents}
        self._actions = [0, 1, 2, 3, 4]
        self.__setup_grid()                                          # :54
        self.__setup_agent()                                         # :55
        self._step_rew = step_reward
        self._collide_rew = collide_reward
        self.agent_positions = [(-1, -1) for _ in self.agents]
        self._total_episode_reward = None
        self._agent_step_count = None
        self._agent_dones = None
        self._curr_agents_count = None
        self._device = device
        self._batch = None

    # ---------------------------------------------------------------- setup
    def __setup_grid(self):
        """:421-428 + :282-288.  Non-square maps fail like the reference's
        __create_grid (IndexError, quirk 5)."""
        grid = load_map(self._grid_file_path)
        n_rows, n_cols = grid.shape
        assert n_rows > 0 and n_cols > 0
        if n_rows != n_cols:
            raise IndexError("list index out of range")
        self._grid_shape = (n_rows, n_cols)
        self._grid = grid

    def __setup_agent(self):
        """:430-449 — same draws: random.randint(1, 25) then random.sample."""
        random_scen_path = self._agent_path + str(random.randint(1, 25)) + ".scen"
        assert os.path.exists(random_scen_path)
        with open(random_scen_path, "r") as f:
            f_lines = [row.rstrip() for row in f.readlines()][1:]
        sampled_lines = random.sample(f_lines, self._n_agents)
        for a_index, (start, goal) in enumerate(parse_scen_lines(sampled_lines)):
            self._agent_init_pos[a_index] = start    # scen (x, y) used as (row, col)
            self._agent_goal_pos[a_index] = goal
        self.agent_starts = [self._agent_init_pos[i] for i in range(self._n_agents)]
        self.agent_goals = [self._agent_goal_pos[i] for i in range(self._n_agents)]

    def _make_batch(self):
        init = np.array([self._agent_init_pos[a] for a in self.agents], dtype=np.int32)[None]
        goals = np.array([self._agent_goal_pos[a] for a in self.agents], dtype=np.int32)[None]
        self._batch = MapfGridBatch(init, goals, grids=self._grid[None],
                                    episode_limit=self.episode_limit,
                                    step_reward=self._step_rew, collide_reward=self._collide_rew,
                                    obs=("full",), device=self._device, packed=True)
        self._built_from = (init.tobytes(), goals.tobytes())
        # one pinned host mirror of state + outputs (one D2H copy per step) and a
        # pinned action row -> device row (no pageable copies on the step path)
        self._host_flat, self._host = self._batch.host_mirror()
        self._act_host = torch.empty((1, self._n_agents), dtype=torch.int8, pin_memory=True)
        self._act_dev = torch.empty((1, self._n_agents), dtype=torch.int8,
                                    device=self._batch.device)

    # ---------------------------------------------------------------- plugin API
    def reset(self):
        """:70-83 — returns get_obs()."""
        init = np.array([self._agent_init_pos[a] for a in self.agents], dtype=np.int32)[None]
        goals = np.array([self._agent_goal_pos[a] for a in self.agents], dtype=np.int32)[None]
        if self._batch is None or self._built_from != (init.tobytes(), goals.tobytes()):
            self._make_batch()
        self._batch.reset()
        self._total_episode_reward = [0 for _ in range(self._n_agents)]
        self._step_count = 0
        self._agent_step_count = [0 for _ in range(self._n_agents)]
        self._agent_dones = [False for _ in range(self._n_agents)]
        self._node_collision_agents = [0 for _ in range(self._n_agents)]
        self._edge_collision_agents = [0 for _ in range(self._n_agents)]
        self._curr_agents_count = 0
        self.agent_positions = [self._agent_init_pos[a] for a in self.agents]
        self.dir_unit_vectors = [[0, 0] for _ in self.agents]
        self.norm_unit_vectors = [0 for _ in self.agents]
        self._pull()
        return self.get_obs()

    def _pull(self):
        """The step's state and outputs -> host: ONE copy + ONE stream sync."""
        self._batch.pull(self._host_flat)
        h = self._host
        self._occ = h["obs_full"][0].numpy().astype(np.int64)
        self._avail_mask = h["avail"][0].numpy()

    def step(self, agents_action):
        """:85-141 — returns (sum(rewards), self._agent_dones (aliased), info)."""
        if self._debug_mode:
            print("goals: ", self._agent_goal_pos)
        if isinstance(agents_action, torch.Tensor):
            agents_action = agents_action.detach().cpu().numpy()
        assert len(agents_action) == self._n_agents                              # :91
        assert all([action_i in ACTION_MEANING.keys() for action_i in agents_action])  # :92
        done_pre = list(self._agent_dones)
        self._act_host.numpy()[0] = [int(a) for a in agents_action]
        self._act_dev.copy_(self._act_host, non_blocking=True)
        b = self._batch
        b.step(self._act_dev)
        self._pull()
        h = self._host
        R = float(h["reward"][0])
        pos = h["pos"][0].numpy()
        done = h["done"][0].numpy()
        node = h["node"][0].numpy()
        edge = h["edge"][0].numpy()
        self._step_count += 1
        for i in self.agents:
            if not done_pre[i]:
                self._agent_step_count[i] += 1
            self.agent_positions[i] = (int(pos[i, 0]), int(pos[i, 1]))
            self._agent_dones[i] = bool(done[i])      # in place: the list stays aliased
        self._node_collision_agents = [int(v) for v in node]
        self._edge_collision_agents = [int(v) for v in edge]
        self._avail_actions = self.get_avail_actions()
        # Python type of `sum(rewards)` (quirk 4): an int iff no float was ever added
        if isinstance(self._collide_rew, int) and (isinstance(self._step_rew, int)
                                                   or all(done_pre)):
            R = int(R)
        info = {"_step_count": self._step_count}
        return R, self._agent_dones, info

    def get_obs(self):
        """:143-161 — (N, H*W) int64, one identical occupancy map per agent."""
        self.__update_goal_vectors()
        return np.array([self.get_obs_agent(agent_i) for agent_i in self.agents])

    def get_obs_agent(self, agent_id):
        """:163-183 — the row-major occupancy map."""
        return self._occ.reshape(-1).copy()

    def get_obs_size(self):
        return self._grid_shape[0] * self._grid_shape[1]

    def get_state(self):
        """:190-192."""
        return self._occ.reshape(-1).copy()

    def get_state_size(self):
        return self._grid_shape[0] * self._grid_shape[1]

    def get_avail_actions(self):
        """:198-201."""
        self._avail_actions = [self.get_avail_agent_actions(agent_i) for agent_i in self.agents]
        return self._avail_actions

    def get_avail_agent_actions(self, agent_id):
        """:203-224 from the kernel's 5-bit mask."""
        m = int(self._avail_mask[agent_id])
        return [(m >> d) & 1 for d in range(5)]

    def get_total_actions(self):
        return len(self._actions)

    def get_stats(self):
        # not in the reference (why it is unregistered there, parallel_runner.py:180,256)
        return {}

    def render(self):
        return None

    def close(self):
        pass

    def seed(self):
        pass

    def save_replay(self):
        pass

    def get_env_info(self):
        return {"state_shape": self.get_state_size(), "obs_shape": self.get_obs_size(),
                "n_actions": self.get_total_actions(), "n_agents": self._n_agents,
                "episode_limit": self.episode_limit}

    def episode_done(self):
        return sum(self._agent_dones) == self._n_agents

    def __update_goal_vectors(self):
        """:451-463 (computed, not emitted)."""
        for i in range(self._n_agents):
            pos, goal = self.agent_positions[i], self.agent_goals[i]
            distance = [goal[0] - pos[0], goal[1] - pos[1]]
            norm = math.sqrt(distance[0] ** 2 + distance[1] ** 2)
            self.dir_unit_vectors[i] = [0, 0] if norm == 0 else [distance[0] / norm,
                                                                 distance[1] / norm]
            self.norm_unit_vectors[i] = norm
