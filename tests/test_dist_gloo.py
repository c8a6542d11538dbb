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


# ---------------------------------------------------------------- launcher + packed gather
def _run_bench(*argv, timeout=180):
    import subprocess
    import sys
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + list(argv),
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                          timeout=timeout, env=env)


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launcher_spawns_ranks(world):
    """bench.py --gpus N with no torchrun environment starts N ranks itself
    (launch_ranks): the gloo rehearsal of the same path shards global env ids and
    gathers one packed buffer per rank to rank 0."""
    import json
    r = _run_bench("--gpus", str(world), "--dist-selftest")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout           # rank 0 prints, the others stay quiet
    assert lines[0]["dist_selftest"] == "ok"
    assert lines[0]["n_gpus"] == world and lines[0]["launcher"] == "bench.py launch_ranks"


def test_bench_refuses_more_gpus_than_visible():
    n = max(2, torch.cuda.device_count() + 1)
    r = _run_bench("--gpus", str(n), "--steps", "2", "--warmup", "0")
    assert r.returncode != 0
    assert "requested but only" in r.stderr
    assert not any(x.startswith("{") for x in r.stdout.splitlines())


def test_bench_rejects_world_mismatch():
    import subprocess
    import sys
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--dist-selftest"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_chunk_layout_prefix_and_views():
    from mapfx.dist import ChunkLayout
    spec = {"a": ((3, 5), torch.float64), "b": ((7,), torch.uint8), "c": ((2, 3), torch.int32),
            "d": ((), torch.int64)}
    lay = ChunkLayout(spec, order=("b", "a"))
    assert list(lay.spec) == ["b", "a", "c", "d"]
    assert all(o % 16 == 0 for o in lay.offsets.values())
    assert lay.end_of(("b",)) == 7 and lay.end_of(("b", "a")) == 16 + 120
    with pytest.raises(ValueError):
        lay.end_of(("a",))
    flat = lay.alloc("cpu")
    v = lay.views(flat)
    v["a"].copy_(torch.arange(15, dtype=torch.float64).view(3, 5))
    v["b"].fill_(9)
    v["c"].copy_(torch.tensor([[1, 2, 3], [4, 5, 6]], dtype=torch.int32))
    v["d"].fill_(-5)
    two = torch.stack([flat, flat.clone()])
    v2 = lay.views(two)
    assert v2["a"].shape == (2, 3, 5) and torch.equal(v2["a"][1], v["a"])
    assert torch.equal(v2["c"][0], v["c"]) and v2["d"].tolist() == [-5, -5]
    with pytest.raises(KeyError):
        ChunkLayout(spec, order=("zz",))


class _OracleTrajBatch:
    """Test stand-in for MapfGridBatch on a CPU rank: the C oracle steps the
    shard, and rollout() fills [T, ...] trajectory tensors like mapfx_rollout."""

    def __init__(self, inst, S, N, W, offset):
        from oracle import corc
        self.corc = corc
        self.E, self.N, self.win, self.offset = inst["init_pos"].shape[0], N, W, offset
        self.H = self.W = S   # grid size (MapfGridBatch.H / W), what the compact cells use
        self.device = torch.device("cpu")
        self.ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], S, S, limit=7,
                                   env_offset=offset, nthreads=1)

    def out_spec(self, T):
        E, N, W = self.E, self.N, self.win
        return {"obs_window": ((T, E, N, 2, W, W), torch.int8),
                "obs_window_occ": ((T, E, N, W, W), torch.int8), "reward": ((T, E), torch.float64),
                "traj_done": ((T, E, N), torch.uint8), "traj_pos": ((T, E, N, 2), torch.int32)}

    def rollout(self, T, actions=None, seed=0, t0=0, traj=None, outputs=None):
        lib = self.corc.lib()
        for k in range(T):
            a = np.array([[lib.orc_action(seed, self.offset + e, t0 + k, i) for i in range(self.N)]
                          for e in range(self.E)], dtype=np.int32)
            r = self.ob.step(a)
            o = self.ob.observe(window=self.win, full=False)
            traj["reward"][k].copy_(torch.from_numpy(r["reward"]))
            traj["obs_window"][k].copy_(torch.from_numpy(o["obs_window"]))
            ob_, ag_ = o["obs_window"][:, :, 0], o["obs_window"][:, :, 1]   # -> occ = agents - obst
            traj["obs_window_occ"][k].copy_(torch.from_numpy(np.where(ob_ == 1, -1, ag_)
                                                             .astype(np.int8)))
            traj["traj_done"][k].copy_(torch.from_numpy(self.ob.done))
            traj["traj_pos"][k].copy_(torch.from_numpy(self.ob.pos))
        return traj


_OG = dict(S=12, N=6, W=5, T=3, chunks=3, E=5)


def _og_worker(rank, world, port, q, keys):
    import sys
    sys.path[:0] = [REPO, PKG_ROOT]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mapfx.dist import OverlappedGather
        from mapfx.maps import synthetic_instances
        c = _OG
        inst = synthetic_instances(c["E"], c["S"], c["S"], c["N"], p_obstacle=0.1, seed=5,
                                   env_offset=rank * c["E"])
        fb = _OracleTrajBatch(inst, c["S"], c["N"], c["W"], rank * c["E"])
        og = OverlappedGather(fb, c["T"], keys=keys, compact=(keys == "compact"))
        assert og.bytes_per_chunk() % 16 == 0
        got = []
        for i in range(c["chunks"]):
            og.step_chunk(seed=9, t0=i * c["T"])
            res = og.result(i)
            if rank == 0:
                got.append({k: v.clone().numpy() for k, v in res.items()})
            with pytest.raises(IndexError):
                og.result(i - 2) if i >= 2 else og.result(i + 1)
        if rank == 0:
            q.put(got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("keys", [("obs_window", "reward", "traj_done"),
                                  ("obs_window_occ", "reward", "traj_done"),
                                  ("reward", "traj_done"), "compact"])
def test_overlapped_gather_packed_world2(keys):
    """OverlappedGather at world 2 (gloo): ONE gather per chunk of the packed
    (obs, reward, done) prefix, double-buffered receive side; rank 0's per-chunk
    result equals an unsharded run, env for env.  The payloads of bench.py
    --gather-payload: the two window planes, the occupancy window (half the bytes,
    the planes follow from it), or reward + done only."""
    from mapfx.maps import synthetic_instances
    world, c = 2, _OG
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_og_worker, args=(r, world, port, q, keys)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    inst = synthetic_instances(world * c["E"], c["S"], c["S"], c["N"], p_obstacle=0.1, seed=5)
    fb = _OracleTrajBatch(inst, c["S"], c["N"], c["W"], 0)
    for i in range(c["chunks"]):
        traj = {k: torch.zeros(s, dtype=d) for k, (s, d) in fb.out_spec(c["T"]).items()}
        fb.rollout(c["T"], seed=9, t0=i * c["T"], traj=traj)
        g = got[i]
        if keys == "compact":   # reward row + unpacked cells / done bits == the unsharded run
            from mapfx.dist import COMPACT_KEYS, unpack_compact
            assert tuple(g) == COMPACT_KEYS
            u = unpack_compact({k: torch.from_numpy(v) for k, v in g.items()}, c["S"], c["N"])
            for k, ref in (("reward", "reward"), ("pos", "traj_pos"), ("done", "traj_done")):
                merged = np.concatenate(list(u[k].numpy()), axis=1)
                assert np.array_equal(merged.view(np.uint8), traj[ref].numpy().view(np.uint8)), (i, k)
            continue
        assert set(g) == set(keys)
        for k in g:
            # [world, T, E_rank, ...] -> [T, world * E_rank, ...]
            merged = np.concatenate(list(g[k]), axis=1)
            assert np.array_equal(merged.view(np.uint8), traj[k].numpy().view(np.uint8)), (i, k)


def _og_uneven_worker(rank, world, port, q, n_total, compact):
    import sys
    sys.path[:0] = [REPO, PKG_ROOT]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mapfx.dist import OverlappedGather, shard
        from mapfx.maps import synthetic_instances
        c = _OG
        off, cnt = shard(n_total, rank, world)
        inst = synthetic_instances(cnt, c["S"], c["S"], c["N"], p_obstacle=0.1, seed=5, env_offset=off)
        fb = _OracleTrajBatch(inst, c["S"], c["N"], c["W"], off)
        keys = "compact" if compact else ("obs_window_occ", "reward", "traj_done")
        # compact: the counts handed in from shard() (no construction all_reduce);
        # otherwise exchanged by the constructor's collective
        given = [shard(n_total, r, world)[1] for r in range(world)] if compact else None
        og = OverlappedGather(fb, c["T"], keys=keys, compact=compact, rank_envs=given)
        assert not og.even and og.rank_envs == [shard(n_total, r, world)[1] for r in range(world)]
        got = []
        for i in range(c["chunks"]):
            og.step_chunk(seed=9, t0=i * c["T"])
            res = og.result(i)
            if rank == 0:
                got.append([{k: v.clone().numpy() for k, v in part.items()} for part in res])
        if rank == 0:
            q.put(got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("compact", [False, True])
def test_overlapped_gather_uneven_world3(compact):
    """World 3 over gloo with uneven shards (mapfx.dist.shard of 8 envs: 3 / 3 / 2):
    every rank sends the largest rank's prefix size, rank 0 gets one view dict per
    rank cut to that rank's env count, and the concatenation equals an unsharded run."""
    from mapfx.maps import synthetic_instances
    world, c, n_total = 3, _OG, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_og_uneven_worker, args=(r, world, port, q, n_total, compact))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    inst = synthetic_instances(n_total, c["S"], c["S"], c["N"], p_obstacle=0.1, seed=5)
    fb = _OracleTrajBatch(inst, c["S"], c["N"], c["W"], 0)
    for i in range(c["chunks"]):
        traj = {k: torch.zeros(s, dtype=d) for k, (s, d) in fb.out_spec(c["T"]).items()}
        fb.rollout(c["T"], seed=9, t0=i * c["T"], traj=traj)
        parts = got[i]
        assert [p_["reward"].shape[1] for p_ in parts] == [3, 3, 2]
        if compact:
            from mapfx.dist import unpack_compact
            us = [unpack_compact({k: torch.from_numpy(v) for k, v in p_.items()}, c["S"], c["N"])
                  for p_ in parts]
            for k, ref in (("reward", "reward"), ("pos", "traj_pos"), ("done", "traj_done")):
                merged = np.concatenate([u[k].numpy() for u in us], axis=1)
                assert np.array_equal(merged.view(np.uint8), traj[ref].numpy().view(np.uint8)), (i, k)
            continue
        for k in ("obs_window_occ", "reward", "traj_done"):
            merged = np.concatenate([p_[k] for p_ in parts], axis=1)
            assert np.array_equal(merged.view(np.uint8), traj[k].numpy().view(np.uint8)), (i, k)


def test_compact_refuses_large_grid():
    """The compact payload's cells are u16: a grid above 65536 cells is refused before
    anything is packed (the host pack would otherwise wrap silently)."""
    from mapfx.dist import check_compact_grid, pack_compact_host
    check_compact_grid(256, 256)
    with pytest.raises(ValueError):
        check_compact_grid(257, 256)
    pos = torch.zeros((1, 1, 1, 2), dtype=torch.int32)
    with pytest.raises(ValueError):
        pack_compact_host(pos, torch.zeros((1, 1, 1), dtype=torch.uint8), 300,
                          torch.zeros((1, 1, 1), dtype=torch.int16),
                          torch.zeros((1, 1, 1), dtype=torch.uint8), H=300)
