"""MARL_PARTIAL_ENV drop-in: the env the reference registers (src/envs/__init__.py:60).

Same constructor, plugin methods, return types and RNG draw order as
MARL-curve-main/src/envs/marl_partial.py (`MARL_PARTIAL_ENV`, lines 23-1000); the
goal-distance tables, transition, rewards, collisions, observations, state and
available actions come from the HIP kernels (mapfx.partial.MarlPartialBatch,
E = 1).  Observations are float32, the dtype PyMARL's EpisodeBatch stores them
in.  Not reproduced (out of scope): rendering / visual json export and the
`output=True` random collision repair (:262-275).
"""
from __future__ import annotations

import os.path
import random

import numpy as np
import torch

from ..maps import load_map
from ..partial import MarlPartialBatch
from .multiagentenv import MultiAgentEnv

ACTION_MEANING = {0: "LEFT", 1: "RIGHT", 2: "UP", 3: "DOWN", 4: "STAY"}  # :1076-1082


class MARL_PARTIAL_ENV(MultiAgentEnv):
    """MultiAgentEnv, the base of customized envs"""

    def __init__(self, grid_file_path, agents_path, n_agents=4, obs_window=5, obs_knn_agents=5,
                 episode_limit=100, seed=None, render='human', move_reward=-0.01, stay_reward=-0.02,
                 stay_goal_reward=0, node_collide_reward=-1, edge_collide_reward=-1,
                 env_collide_reward=-1, complete_reward=1000, complete_fac=1.5, debug=False,
                 visual=False, gamma=0.99, output=False, device=None):
        assert os.path.exists(grid_file_path)                                    # :54
        self._output_mode = bool(output)   # :58 (collision repair after the step, :262-275)
        self._grid_file_path = grid_file_path
        self._agent_path = agents_path
        self._render_mode = render
        self._debug_mode = debug
        self._n_agents = n_agents
        self._seed = random.randint(0, 9999)                                     # :61
        np.random.seed(self._seed)
        if seed:
            self._seed = seed
        self.agents = [a for a in range(self._n_agents)]
        self._n_features = 13
        self._actions = [0, 1, 2, 3, 4]
        self.episode_limit = episode_limit
        self._obs_window = obs_window
        self._obs_knn_agents = obs_knn_agents
        self._params = dict(obs_window=obs_window, obs_knn_agents=obs_knn_agents,
                            episode_limit=episode_limit, move_reward=move_reward,
                            stay_reward=stay_reward, stay_goal_reward=stay_goal_reward,
                            node_collide_reward=node_collide_reward,
                            edge_collide_reward=edge_collide_reward,
                            env_collide_reward=env_collide_reward, complete_reward=complete_reward,
                            complete_fac=complete_fac, gamma=gamma)
        self._device = device
        self._agent_init_pos = [(-1, -1) for _ in self.agents]
        self._agent_goal_pos = [(-1, -1) for _ in self.agents]
        self.__setup_grid()                                                      # :107
        self.__setup_agent()                                                     # :108
        self._batch = None
        self._step_count = None
        self._terminated = False

    # ---------------------------------------------------------------- setup
    def __setup_grid(self):
        """:862-894 (map only; the networkx graph is replaced by the BFS kernel)."""
        grid = load_map(self._grid_file_path)
        n_rows, n_cols = grid.shape
        assert n_rows > 0 and n_cols > 0
        if n_rows != n_cols:  # __create_grid indexes [col][row] (:514-522): square maps only
            raise IndexError("list index out of range")
        self._grid_shape = (n_rows, n_cols)
        self._grid = grid

    def __setup_agent(self):
        """:896-920: same draws (random.randint(1, 25), random.sample), scen
        fields 4..7 = start x(col), start y(row), goal x, goal y."""
        random_scen_path = self._agent_path + str(random.randint(1, 25)) + '.scen'
        assert os.path.exists(random_scen_path)
        with open(random_scen_path, "r") as f:
            f_lines = [row.rstrip() for row in f.readlines()][1:]
            assert len(f_lines) > self._n_agents
            rand_lines = random.sample(f_lines, self._n_agents)
            for a_index, f_line in enumerate(rand_lines):
                line_list = f_line.replace('\t', ',').split(",")
                s_col, s_row, f_col, f_row = (int(line_list[4]), int(line_list[5]),
                                              int(line_list[6]), int(line_list[7]))
                self._agent_init_pos[a_index] = (s_row, s_col)
                self._agent_goal_pos[a_index] = (f_row, f_col)

    def _load_instance(self):
        init = np.array([self._agent_init_pos], dtype=np.int32)
        goals = np.array([self._agent_goal_pos], dtype=np.int32)
        if self._batch is None:
            self._batch = MarlPartialBatch(init, goals, grids=self._grid[None],
                                           device=self._device, packed=True, **self._params)
            self._host_flat, self._host = self._batch.host_mirror()
            self._act_host = torch.empty((1, self._n_agents), dtype=torch.int8, pin_memory=True)
            self._act_dev = torch.empty((1, self._n_agents), dtype=torch.int8,
                                        device=self._batch.device)
        else:
            self._batch.set_agents(init, goals)

    # ---------------------------------------------------------------- plugin API
    def reset(self):
        """:125-163: re-samples the agents, resets, returns get_obs()."""
        self.__setup_agent()
        self._load_instance()
        self._batch.reset()
        self._step_count = 0
        self._terminated = False
        self._pull()
        return self.get_obs()

    def _pull(self):
        """The step's state and outputs -> host: ONE copy + ONE stream sync."""
        self._batch.pull(self._host_flat)
        h = self._host
        self._obs = h["obs"][0].numpy().copy()
        self._state = h["state"][0].numpy().copy()
        self._avail_mask = h["avail"][0].numpy().copy()
        self._agent_positions = [tuple(int(v) for v in p) for p in h["pos"][0].numpy()]

    def agent_pos(self, agent_id):
        assert -1 < agent_id < self._n_agents
        return self._agent_positions[agent_id]

    def step(self, agents_action):
        """:165-310 -- returns (sum(rewards), terminated, {'_step_count': t})."""
        if isinstance(agents_action, torch.Tensor):
            agents_action = agents_action.detach().cpu().numpy()
        assert len(agents_action) == self._n_agents                              # :173
        assert all([action_i in ACTION_MEANING.keys() for action_i in agents_action])  # :174
        old_pos = list(self._agent_positions)
        self._act_host.numpy()[0] = [int(a) for a in agents_action]
        self._act_dev.copy_(self._act_host, non_blocking=True)
        self._batch.step(self._act_dev)
        self._pull()
        h = self._host
        R = float(h["reward"][0])
        self._step_count += 1
        self._terminated = bool(h["terminated"][0])
        if self._output_mode:
            self._repair(old_pos, list(agents_action))
        return R, self._terminated, {'_step_count': self._step_count}

    # ------------------------------------------------- output mode (:262-275)
    def _repair(self, old_pos, actions):
        """Rewards, at-goal flags and collision totals stay those of the raw step;
        positions are made collision free like the reference's solvers; the node /
        edge vectors the observation reads are then those of the last check (all
        zero)."""
        new = list(self._agent_positions)
        n_node, node_vec = _check_node(new)                                      # :236
        n_edge, _, pairs = _check_edge(old_pos, new)                             # :238
        if n_node == 0 and n_edge == 0:
            return
        occ_old = self._grid.astype(np.int64).copy()    # the PRE-step _full_obs (:279-280)
        for p in old_pos:
            occ_old[p] += 1
        ctx = (self._grid.shape, occ_old, old_pos, actions)
        if n_node > 0:                                                           # :263-268
            while n_node > 0:
                new = _solve_node(ctx, new, node_vec)
                n_node, node_vec = _check_node(new)
        if n_edge > 0:                                                           # :269-275
            while n_edge > 0:
                new = _solve_edge(ctx, new, pairs)
                n_edge, _, _ = _check_edge(old_pos, new)
        b = self._batch
        b.pos[0].copy_(torch.tensor(new, dtype=torch.int32))
        b.node[0].zero_()
        b.edge[0].zero_()
        b.observe()
        self._pull()

    def get_obs(self):
        """:312-317 -- (N, 2W^2 + 13K), float32 values."""
        return self._obs.copy()

    def get_obs_agent(self, agent_id):
        return self._obs[agent_id].copy()

    def get_obs_size(self):
        return 2 * (self._obs_window ** 2) + self._obs_knn_agents * self._n_features

    def get_state(self):
        """:377-387 -- [total collisions, step count, sum(each goal cost)]."""
        return self._state.astype(np.int64)

    def get_state_size(self):
        return 3

    def get_avail_actions(self):
        return [self.get_avail_agent_actions(i) for i in self.agents]

    def get_avail_agent_actions(self, agent_id):
        m = int(self._avail_mask[agent_id])
        return [(m >> d) & 1 for d in range(5)]

    def get_total_actions(self):
        return len(self._actions)

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
        return bool(self._host["done"][0].all())


# ---------------------------------------------------------------------------
# output-mode collision repair, host side as in the reference (marl_partial.py):
# sequential, randomised (random.shuffle on the global stream), data-dependent.
# ---------------------------------------------------------------------------
def _check_node(pos):
    """__check_node_collisions (:747-770): (count, 0/1 vector)."""
    at = {}
    for i, p in enumerate(pos):
        at.setdefault(p, set()).add(i)
    vec = [0] * len(pos)
    count = 0
    for agents in at.values():
        if len(agents) > 1:
            count += len(agents)
            for i in agents:
                vec[i] += 1
    return count, vec


def _check_edge(old, new):
    """__check_edge_collisions (:823-857): (count, vector, set of sorted pairs)."""
    vec = [0] * len(new)
    count = 0
    pairs = set()
    for i, (io, inew) in enumerate(zip(old, new)):
        if io == inew:
            continue
        for j, jo in enumerate(old):
            if j != i and jo == inew and new[j] == io:
                count += 1
                vec[i] += 1
                pairs.add(tuple(sorted([i, j])))
    return count, vec, pairs


_DELTA = {0: (-1, 0), 1: (1, 0), 2: (0, -1), 3: (0, 1)}


def _free(ctx, p):
    """__is_valid and not __is_cell_obstacle on the pre-step occupancy (:504-522)."""
    (h, w), occ, _, _ = ctx
    return 0 <= p[0] < h and 0 <= p[1] < w and occ[p] != -1


def _agent_step(ctx, act, pos):
    """__agent_step (:617-643) -> (next_pos, env collision)."""
    if act == 4:
        return pos, False
    d = _DELTA[act]
    nxt = (pos[0] + d[0], pos[1] + d[1])
    return (nxt, False) if _free(ctx, nxt) else (pos, True)


def _solve_node(ctx, new, node_vec):
    """__solve_node_collisions (:645-712)."""
    _, _, old, acts = ctx
    n = len(new)
    col = [i for i in range(n) if node_vec[i] > 0]
    random.shuffle(col)
    cnt = {}
    for p in new:
        cnt[p] = cnt.get(p, 0) + 1
    for a in col:
        a_pos = new[a]
        if cnt[a_pos] <= 1:
            continue
        a_new = old[a]
        if cnt.get(a_new, 0) <= 0:
            cnt[a_pos] -= 1
            new[a] = a_new
            cnt[a_new] = cnt.get(a_new, 0) + 1
            continue
        these = [i for i in range(n) if old[a] == new[i]]
        random.shuffle(these)
        these_acts = [acts[i] for i in these]
        a_act = acts[a]
        solved = False
        for act in these_acts:
            if act == a_act:
                continue
            p, coll = _agent_step(ctx, act, old[a])
            if not coll and cnt.get(p, 0) <= 0:
                cnt[a_pos] -= 1
                new[a] = p
                cnt[p] = cnt.get(p, 0) + 1
                solved = True
                break
        if solved:
            continue
        tries = [0, 1, 2, 3]
        random.shuffle(tries)
        o = old[a]
        for act in tries:
            d = _DELTA[act]
            p = (o[0] + d[0], o[1] + d[1])
            if act == a_act or not _free(ctx, p):
                continue
            if cnt.get(p, 0) <= 0:
                cnt[o] -= 1   # the reference decrements the OLD cell here (:706)
                new[a] = p
                cnt[p] = cnt.get(p, 0) + 1
                break
    return new


def _solve_edge(ctx, new, pairs):
    """__solve_edge_collisions (:772-821)."""
    _, _, old, acts = ctx
    try_map = {0: [2, 3], 1: [3, 2], 2: [0, 1], 3: [1, 0]}
    back = {0: 1, 1: 0, 2: 3, 3: 2}
    pairs = list(pairs)
    random.shuffle(pairs)
    cnt = {}
    for p in new:
        cnt[p] = cnt.get(p, 0) + 1
    for pair in pairs:
        pair = list(pair)
        random.shuffle(pair)
        solved = False
        for a in pair:
            a_pos = new[a]
            broke = False
            o = old[a]
            for act in try_map[acts[a]]:
                d = _DELTA[act]
                p = (o[0] + d[0], o[1] + d[1])
                if not _free(ctx, p):
                    continue
                if cnt.get(p, 0) <= 0:
                    cnt[a_pos] -= 1
                    new[a] = p
                    cnt[p] = cnt.get(p, 0) + 1
                    broke = True
                    break
            if broke:
                solved = True
                break
        if solved:
            continue
        for a in pair:
            o = old[a]
            d = _DELTA[back[acts[a]]]
            p = (o[0] + d[0], o[1] + d[1])
            if not _free(ctx, p):
                continue
            if cnt.get(p, 0) <= 0:
                cnt[a_pos] -= 1   # a_pos as left by the loop above (:807)
                new[a] = p
                cnt[p] = cnt.get(p, 0) + 1
                solved = True
        if solved:
            continue
        for a in pair:
            new[a] = old[a]
    return new
