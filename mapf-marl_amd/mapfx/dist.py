"""Env sharding over the GPUs of a node.

Env instances never interact, so each rank owns a contiguous block of GLOBAL env
ids and steps it with no per-step communication; every synthetic input (maps,
starts/goals, generator actions) is keyed by the global env id, so a sharded run
is bit-identical, env for env, to a single-GPU run of all envs.

The only collective is the one the reference's runner architecture implies:
ParallelRunner collects every worker env's (obs, reward, done) in the parent
process (runners/parallel_runner.py:117-173).  Here that is a torch.distributed
gather (RCCL over xGMI with the "nccl" backend) of a rollout chunk's trajectory
tensors to rank 0, issued on a side stream so it overlaps the next chunk.
"""
from __future__ import annotations

import os

import torch


def env_info():
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(n_total: int, rank: int, world: int):
    """Contiguous block of global env ids owned by `rank`: (offset, count).
    The first n_total % world ranks get one extra env."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world %d/%d" % (rank, world))
    base, extra = divmod(n_total, world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def gather_to_root(tensors: dict, keys, dst: int = 0, group=None):
    """Gather tensors[k] (same shape on every rank) to `dst`.  Returns on dst a
    dict k -> list of per-rank tensors (rank order = global env order), else None."""
    import torch.distributed as dist
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    out = {} if rank == dst else None
    for k in keys:
        t = tensors[k].contiguous()
        lst = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
        dist.gather(t, gather_list=lst, dst=dst, group=group)
        if rank == dst:
            out[k] = lst
    return out


def concat_env_major(parts, env_dim: int):
    """Rank-ordered per-shard tensors -> one tensor over all global envs."""
    return torch.cat(parts, dim=env_dim)


class OverlappedGather:
    """Double-buffered trajectory chunks: chunk i is gathered to rank 0 on a side
    stream while chunk i+1 is being stepped on the compute stream."""

    def __init__(self, batch, T: int, keys=("obs_window", "reward", "traj_done"), outputs=None):
        import torch.distributed as dist
        self.dist = dist
        self.batch = batch
        self.T = T
        self.keys = tuple(keys)
        self.outputs = outputs
        self.bufs = [batch._alloc_out(T), batch._alloc_out(T)]
        self.side = torch.cuda.Stream(device=batch.device)
        self.done_ev = [None, None]
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.recv = None
        if self.rank == 0:
            self.recv = {k: [torch.empty_like(self.bufs[0][k]) for _ in range(self.world)]
                         for k in self.keys}
        self.i = 0

    def bytes_per_chunk(self):
        return sum(self.bufs[0][k].numel() * self.bufs[0][k].element_size() for k in self.keys)

    def step_chunk(self, actions=None, seed=0, t0=0):
        cur = self.i & 1
        if self.done_ev[cur] is not None:  # buffer reuse: its gather must be finished
            torch.cuda.current_stream().wait_event(self.done_ev[cur])
        traj = self.batch.rollout(self.T, actions=actions, seed=seed, t0=t0, traj=self.bufs[cur],
                                  outputs=self.outputs)
        ready = torch.cuda.Event()
        ready.record()
        with torch.cuda.stream(self.side):
            self.side.wait_event(ready)
            for k in self.keys:
                self.dist.gather(traj[k], gather_list=self.recv[k] if self.rank == 0 else None,
                                 dst=0)
            ev = torch.cuda.Event()
            ev.record(self.side)
            self.done_ev[cur] = ev
        self.i += 1
        return traj

    def synchronize(self):
        torch.cuda.synchronize(self.batch.device)
