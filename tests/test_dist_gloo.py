"""world_size-2 CPU (gloo) test of the env-sharding + gather path.

Each rank builds only its shard of the global env ids (mapfx.dist.shard,
synthetic instances keyed by global env id), steps it (the C oracle stands in
for the device step on a CPU-only box), and rank 0 gathers (obs, reward, done)
with mapfx.dist.gather_to_root.  The gathered result must equal an unsharded
run of all envs, env for env.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_ROOT, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    import sys
    sys.path[:0] = [REPO, PKG_ROOT]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mapfx import dist as mdist
        from mapfx.maps import synthetic_instances
        from oracle import corc
        S, N, T, W = 16, 8, 12, 5
        off, cnt = mdist.shard(n_total, rank, world)
        inst = synthetic_instances(cnt, S, S, N, p_obstacle=0.15, seed=3, env_offset=off)
        ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], S, S, limit=9,
                              env_offset=off, nthreads=1)
        out = ob.rollout(T, seed=11, t0=0, window=W)
        # pad shards to equal size for gather (uneven n_total)
        m = n_total // world + (1 if n_total % world else 0)

        def pad(a):
            p = np.zeros((m,) + a.shape[1:], a.dtype)
            p[:a.shape[0]] = a
            return torch.from_numpy(p)
        t = {"reward": pad(out["reward"]), "done": pad(ob.done), "pos": pad(ob.pos),
             "obs": pad(out["obs_window"]), "count": torch.tensor([cnt])}
        g = mdist.gather_to_root(t, ("reward", "done", "pos", "obs", "count"))
        if rank == 0:
            counts = [int(c.item()) for c in g["count"]]
            res = {k: torch.cat([x[:c] for x, c in zip(g[k], counts)]).numpy()
                   for k in ("reward", "done", "pos", "obs")}
            q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [64, 37])
def test_sharded_rollout_gather_equals_unsharded(n_total):
    from mapfx import dist as mdist
    from mapfx.maps import synthetic_instances
    from oracle import corc
    world = 2
    assert sum(mdist.shard(n_total, r, world)[1] for r in range(world)) == n_total
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    S, N, T, W = 16, 8, 12, 5
    inst = synthetic_instances(n_total, S, S, N, p_obstacle=0.15, seed=3)
    ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], S, S, limit=9,
                          nthreads=2)
    out = ob.rollout(T, seed=11, t0=0, window=W)
    assert np.array_equal(res["reward"].view(np.uint64), out["reward"].view(np.uint64))
    assert np.array_equal(res["done"], ob.done)
    assert np.array_equal(res["pos"], ob.pos)
    assert np.array_equal(res["obs"], out["obs_window"])


def test_shard_bounds():
    from mapfx.dist import shard
    for n in (0, 1, 7, 4096, 32768, 32769):
        for w in (1, 2, 3, 8):
            spans = [shard(n, r, w) for r in range(w)]
            assert spans[0][0] == 0
            for (o1, c1), (o2, _) in zip(spans, spans[1:]):
                assert o1 + c1 == o2
            assert sum(c for _, c in spans) == n
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
