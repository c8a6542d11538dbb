"""Env sharding over the GPUs of a node.

Env instances never interact, so each rank owns a contiguous block of GLOBAL env
ids and steps it with no per-step communication; every synthetic input (maps,
starts/goals, generator actions) is keyed by the global env id, so a sharded run
is bit-identical, env for env, to a single-GPU run of all envs.

The only collective is the one the reference's runner architecture implies:
ParallelRunner collects every worker env's (obs, reward, done) in the parent
process (runners/parallel_runner.py:117-173).  Here that is ONE torch.distributed
gather (RCCL over xGMI with the "nccl" backend) per rollout chunk: the chunk's
trajectory tensors live in one flat byte buffer (ChunkLayout) whose gathered
keys form a contiguous prefix, issued on a side stream so it overlaps the next
chunk.  Both the send buffers and rank 0's receive buffers are double-buffered.
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


def _nbytes(shape, dtype):
    n = torch.empty((), dtype=dtype).element_size()
    for s in shape:
        n *= int(s)
    return n


class ChunkLayout:
    """Several typed tensors carved out of ONE flat uint8 buffer.

    `spec` maps name -> (shape, dtype); names are laid out in `order` (the
    rest of `spec` after it), each at a 16-byte aligned offset, so the first k
    names form a contiguous prefix that one collective can move."""

    ALIGN = 16

    def __init__(self, spec: dict, order=()):
        names = [k for k in order if k in spec] + [k for k in spec if k not in order]
        missing = [k for k in order if k not in spec]
        if missing:
            raise KeyError("ChunkLayout: %s not in the output spec" % missing)
        self.spec = {k: (tuple(int(s) for s in spec[k][0]), spec[k][1]) for k in names}
        self.offsets = {}
        off = 0
        for k in names:
            self.offsets[k] = off
            off += -(-_nbytes(*self.spec[k]) // self.ALIGN) * self.ALIGN
        self.nbytes = off

    def end_of(self, keys):
        """Bytes of the prefix holding `keys` (which must be a prefix of the order)."""
        names = list(self.spec)
        if list(keys) != names[:len(keys)]:
            raise ValueError("keys %s are not a prefix of the layout %s" % (list(keys), names))
        if not keys:
            return 0
        k = keys[-1]
        return self.offsets[k] + _nbytes(*self.spec[k])

    def alloc(self, device):
        return torch.zeros(self.nbytes, dtype=torch.uint8, device=device)

    def views(self, flat, keys=None):
        """name -> typed view into `flat` ([nbytes] or [R, >=nbytes] uint8: then
        each view gets a leading R dimension)."""
        out = {}
        for k in (self.spec if keys is None else keys):
            shape, dt = self.spec[k]
            o, n = self.offsets[k], _nbytes(shape, dt)
            v = flat[..., o:o + n].view(dt)
            out[k] = v.unflatten(-1, shape) if shape else v.view(flat.shape[:-1])
        return out


COMPACT_KEYS = ("reward", "cell", "done_bits")


def compact_spec(T, E, N):
    """The compact gather payload of a T-step chunk of E envs of N agents: the env
    rewards (f64, the runner's reward row) and, per agent-step, the u16 cell index
    row * W + col (held in int16) and the done flag as one bit (the
    observations follow from the positions and the static maps, so rank 0 rebuilds
    the ones it needs with mapfx_observe -- unpack_compact)."""
    T, E, N = int(T), int(E), int(N)
    return {"reward": ((T, E), torch.float64), "cell": ((T, E, N), torch.int16),
            "done_bits": ((T, E, (N + 7) // 8), torch.uint8)}


COMPACT_MAX_CELLS = 65536   # cells travel as u16 row * W + col


def check_compact_grid(H, W):
    """The compact payload's u16 cell index needs H * W <= 65536 (mapfx_pack_compact
    refuses larger grids; a host-side cast would wrap silently)."""
    if int(H) * int(W) > COMPACT_MAX_CELLS:
        raise ValueError("compact gather payload: cells are u16, H * W = %d > %d"
                         % (int(H) * int(W), COMPACT_MAX_CELLS))


def pack_compact_host(traj_pos, traj_done, W, cell, done_bits, H=None):
    """mapfx_pack_compact for CPU tensors (the gloo tests' oracle stand-in batch;
    device batches use the HIP kernel)."""
    if H is not None:
        check_compact_grid(H, W)
    if traj_pos.numel() and int(traj_pos[..., 0].max()) * int(W) + int(W) > COMPACT_MAX_CELLS:
        raise ValueError("compact gather payload: a cell index exceeds u16 (W = %d)" % int(W))
    c = traj_pos[..., 0] * int(W) + traj_pos[..., 1]
    cell.copy_(c.to(torch.int32).to(torch.int16))
    N = traj_done.shape[-1]
    nb = done_bits.shape[-1]
    pad = torch.zeros(traj_done.shape[:-1] + (nb * 8,), dtype=torch.int32)
    pad[..., :N] = (traj_done != 0).to(torch.int32)
    w = torch.tensor([1 << k for k in range(8)], dtype=torch.int32)
    done_bits.copy_((pad.view(traj_done.shape[:-1] + (nb, 8)) * w).sum(-1).to(torch.uint8))


def unpack_compact(views, W, N):
    """Gathered compact views (key -> [..., T, E, ...]) -> {"reward", "pos" [..., N, 2]
    int32 (row, col), "done" [..., N] uint8}."""
    cell = views["cell"].to(torch.int32) & 0xFFFF
    pos = torch.stack((cell // int(W), cell % int(W)), dim=-1).to(torch.int32)
    db = views["done_bits"].to(torch.int32)
    bits = torch.arange(8, device=db.device, dtype=torch.int32)
    done = ((db.unsqueeze(-1) >> bits) & 1).flatten(-2)[..., :int(N)].to(torch.uint8)
    return {"reward": views["reward"], "pos": pos, "done": done}


class OverlappedGather:
    """Rollout chunks with ONE gather of each chunk's (obs, reward, done) to `dst`.

    Chunk i is stepped on the current stream into send buffer i % 2 and gathered
    on a side stream into receive buffer i % 2 while chunk i+1 steps.  Ordering:
      * the rollout into send buffer s waits for the previous gather out of s;
      * the gather into receive buffer s waits for everything enqueued on the
        current stream before step_chunk() was called, so a consumer's reads of
        chunk i (kernels on the current stream, or host copies) that come before
        step_chunk(i + 2) never race the overwrite;
      * result(i) makes the current stream wait for chunk i's gather (no host sync).
    On a CPU device (gloo) everything is synchronous on the calling thread.

    compact=True gathers COMPACT_KEYS instead of `keys`: the reward row plus every
    agent-step's u16 cell and done bit, packed by mapfx_pack_compact on the side
    stream (about a tenth of the occupancy-window payload).

    Uneven shards (mapfx.dist.shard of an env count the world does not divide): the
    ranks exchange their env counts once at construction; every rank sends the
    largest rank's prefix size (its own prefix, then whatever bytes follow it in its
    chunk buffer -- e.g. its other rollout outputs such as traj_pos; dst ignores them),
    so the collective's equal-size contract holds, and result(i) returns one dict of
    views per rank, each cut to that rank's env count, instead of [world, ...] views.

    Construction is COLLECTIVE unless `rank_envs` (every rank's env count, e.g. from
    mapfx.dist.shard) is given: it runs one all_reduce of the env counts, so every
    rank of the group must construct its OverlappedGather in the same order.
    """

    def __init__(self, batch, T: int, keys=("obs_window", "reward", "traj_done"), outputs=None,
                 dst: int = 0, group=None, compact=False, rank_envs=None):
        import torch.distributed as dist
        self.dist = dist
        self.batch = batch
        self.T = int(T)
        self.compact = bool(compact)
        spec = dict(batch.out_spec(self.T))
        if self.compact:   # the gathered prefix is COMPACT_KEYS, packed from the rollout
            check_compact_grid(batch.H, batch.W)
            keys = COMPACT_KEYS
            spec.update(compact_spec(self.T, batch.E, batch.N))
            if outputs is not None:
                outputs = tuple(outputs) + tuple(k for k in ("reward", "traj_pos", "traj_done")
                                                 if k not in outputs)
        self.keys = tuple(keys)
        self.outputs = outputs
        self.dst, self.group = dst, group
        self.layout = ChunkLayout(spec, order=self.keys)
        dev = batch.device
        self.cuda = torch.device(dev).type == "cuda"
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        # every rank's env count (given, or one small all-reduce at construction)
        if rank_envs is not None:
            self.rank_envs = [int(c) for c in rank_envs]
            if len(self.rank_envs) != self.world or self.rank_envs[self.rank] != int(batch.E):
                raise ValueError("rank_envs %r does not match world %d / this rank's %d envs"
                                 % (self.rank_envs, self.world, int(batch.E)))
        else:
            counts = torch.zeros(self.world, dtype=torch.int64, device=dev)
            counts[self.rank] = int(batch.E)
            dist.all_reduce(counts, group=group)
            self.rank_envs = [int(c) for c in counts.tolist()]
        self.even = len(set(self.rank_envs)) == 1
        # each rank's gathered prefix (its own layout: the env dimension of every
        # gathered [T, E, ...] tensor is that rank's count), whole 16-B units so every
        # typed view of a received row stays aligned
        self.rank_layouts = [self._layout_for(spec, e) for e in self.rank_envs]
        self.gbytes = max(-(-lay.end_of(self.keys) // ChunkLayout.ALIGN) * ChunkLayout.ALIGN
                          for lay in self.rank_layouts)
        nb = max(self.layout.nbytes, self.gbytes)
        self.flat = [torch.zeros(nb, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.bufs = [self.layout.views(f) for f in self.flat]
        self.recv = None
        if self.rank == dst:
            self.recv = [torch.empty((self.world, self.gbytes), dtype=torch.uint8, device=dev)
                         for _ in range(2)]
        self.side = torch.cuda.Stream(device=dev) if self.cuda else None
        self.gather_ev = [None, None]
        self.i = 0

    def bytes_per_chunk(self):
        """Bytes one rank sends per chunk (the gathered prefix)."""
        return self.gbytes

    def _gather(self, cur):
        lst = list(self.recv[cur].unbind(0)) if self.rank == self.dst else None
        self.dist.gather(self.flat[cur][:self.gbytes], gather_list=lst, dst=self.dst,
                         group=self.group)

    def step_chunk(self, actions=None, seed=0, t0=0):
        """Step one chunk and start its gather.  Returns the chunk index."""
        i, cur = self.i, self.i & 1
        if not self.cuda:
            self.batch.rollout(self.T, actions=actions, seed=seed, t0=t0, traj=self.bufs[cur],
                               outputs=self.outputs)
            if self.compact:
                b = self.bufs[cur]
                pack_compact_host(b["traj_pos"], b["traj_done"], self.batch.W, b["cell"],
                                  b["done_bits"], H=self.batch.H)
            self._gather(cur)
            self.i += 1
            return i
        cs = torch.cuda.current_stream(self.batch.device)
        if self.gather_ev[cur] is not None:      # send buffer reuse: its gather must be done
            cs.wait_event(self.gather_ev[cur])
        self.batch.rollout(self.T, actions=actions, seed=seed, t0=t0, traj=self.bufs[cur],
                           outputs=self.outputs)
        ready = torch.cuda.Event()
        ready.record(cs)
        with torch.cuda.stream(self.side):
            self.side.wait_event(ready)
            if self.compact:    # the pack runs beside the next chunk, like the gather
                b = self.bufs[cur]
                self.batch.pack_compact(b["traj_pos"], b["traj_done"], b["cell"], b["done_bits"])
            self._gather(cur)
            ev = torch.cuda.Event()
            ev.record(self.side)
            self.gather_ev[cur] = ev
        self.i += 1
        return i

    def local(self, i):
        """This rank's trajectory tensors of chunk i (valid until step_chunk(i + 2))."""
        self._check(i)
        return self.bufs[i & 1]

    def _layout_for(self, spec, envs):
        """The gathered keys' layout for a rank holding `envs` envs: every gathered
        tensor is [T, E, ...], so only its env dimension changes."""
        sub = {}
        for k in self.keys:
            shape, dt = spec[k]
            sub[k] = ((shape[0], int(envs)) + tuple(shape[2:]), dt)
        return ChunkLayout(sub, order=self.keys)

    def result(self, i):
        """On dst: chunk i's gathered tensors, key -> [world, T, E_rank, ...] (rank
        order = global env order); with uneven shards a list over ranks of
        key -> [T, E_r, ...].  Valid until step_chunk(i + 2) is called."""
        self._check(i)
        if self.rank != self.dst:
            return None
        cur = i & 1
        if self.cuda and self.gather_ev[cur] is not None:
            torch.cuda.current_stream(self.batch.device).wait_event(self.gather_ev[cur])
        if self.even:
            return self.layout.views(self.recv[cur], self.keys)
        return [lay.views(self.recv[cur][r], self.keys) for r, lay in enumerate(self.rank_layouts)]

    def _check(self, i):
        if not self.i - 2 <= i < self.i:
            raise IndexError("chunk %d is not resident (chunks %d..%d are)"
                             % (i, max(0, self.i - 2), self.i - 1))

    def synchronize(self):
        if self.cuda:
            torch.cuda.synchronize(self.batch.device)
