"""Env plugin registry, mirroring MARL-curve-main/src/envs/__init__.py:33-60.

`REGISTRY[name](**env_args)` builds an env exactly as the reference's runners do
(`env_REGISTRY[args.env](**args.env_args)`, runners/episode_runner.py:32).
"""
from functools import partial

from .multiagentenv import MultiAgentEnv
from .mapf_gridworld import MAPF_GRID
from .marl_partial import MARL_PARTIAL_ENV


def env_fn(env, **kwargs) -> MultiAgentEnv:
    return env(**kwargs)


REGISTRY = {}
# commented out in the reference (envs/__init__.py:23,59) only because MAPF_GRID
# lacks get_stats; the drop-in provides it.
REGISTRY["mapf_gridworld"] = partial(env_fn, env=MAPF_GRID)
REGISTRY["marl_partial"] = partial(env_fn, env=MARL_PARTIAL_ENV)  # envs/__init__.py:60

__all__ = ["REGISTRY", "env_fn", "MultiAgentEnv", "MAPF_GRID", "MARL_PARTIAL_ENV"]
