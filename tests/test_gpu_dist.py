"""Two ranks of real MapfGridBatch shards on the GPU (both on cuda:0, collectives
over gloo: the RCCL run itself needs one GPU per rank, the driver's 8-GPU node).
Each rank steps its shard of the global env ids with the HIP kernel (the
store-wave split writing obs_window_occ, the bench's gather payload) and
OverlappedGather moves each chunk's packed (obs_window_occ, reward, done) to rank
0; the gathered chunks must equal an unsharded single-batch run, env for env, bit
for bit (sharding by global env id is invisible in the results)."""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import PKG_ROOT, REPO

pytestmark = pytest.mark.gpu

C = dict(S=32, N=16, T=5, chunks=3, W=5, seed=17)
KEYS = ("obs_window_occ", "reward", "traj_done")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(mapfx, E, offset):
    from mapfx.maps import synthetic_instances
    inst = synthetic_instances(E, C["S"], C["S"], C["N"], p_obstacle=0.1, seed=4, env_offset=offset)
    b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(C["S"], C["S"]),
                            episode_limit=2000, obs=("window_occ",), window=C["W"], device="cuda:0",
                            env_offset=offset, track_steps=False)
    b.reset()
    return b


def _worker(rank, world, port, q, compact, n_total):
    import sys
    sys.path[:0] = [REPO, PKG_ROOT]
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mapfx
        from mapfx.dist import OverlappedGather, shard
        off, cnt = shard(n_total, rank, world)
        b = _batch(mapfx, cnt, off)
        outs = ("reward", "term", "node", "edge", "avail", "obs_window_occ", "traj_pos", "traj_done",
                "traj_t")
        og = OverlappedGather(b, C["T"], keys=KEYS, outputs=outs, compact=compact)
        got = []
        for i in range(C["chunks"]):
            og.step_chunk(seed=C["seed"], t0=i * C["T"])
            res = og.result(i)
            if rank == 0:
                parts = res        # uneven shards: one dict per rank already
                if og.even:        # [world, T, E, ...] -> one dict per rank
                    parts = [{k: v[r] for k, v in res.items()} for r in range(world)]
                got.append([{k: v.cpu().numpy().copy() for k, v in p_.items()} for p_ in parts])
        og.synchronize()
        if rank == 0:
            q.put(got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total,compact", [(2, 128, False), (2, 128, True),
                                                   (3, 160, True), (3, 160, False)])
def test_two_rank_shards_gather_equals_unsharded(world, n_total, compact):
    """compact=True: the gathered payload is the reward row + u16 cells + done bits
    (mapfx_pack_compact on the side stream); unpacked it equals the unsharded
    trajectory, and rank 0 rebuilds every step's window from the unpacked positions
    with mapfx_observe, bit for bit the window the rollout wrote.  World 3 shards
    160 envs unevenly (54 / 53 / 53, mapfx.dist.shard): every rank sends the largest
    prefix, rank 0 cuts each rank's part to its env count."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import mapfx
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, compact, n_total))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=100)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    full = _batch(mapfx, n_total, 0)
    obs_b = _batch(mapfx, n_total, 0)      # rank 0's observation rebuilder
    for i in range(C["chunks"]):
        traj = full.rollout(C["T"], seed=C["seed"], t0=i * C["T"])
        if compact:
            from mapfx.dist import COMPACT_KEYS, unpack_compact
            assert all(tuple(p_) == COMPACT_KEYS for p_ in got[i])
            us = [unpack_compact({k: torch.from_numpy(v) for k, v in p_.items()}, C["S"], C["N"])
                  for p_ in got[i]]
            for k, ref in (("reward", "reward"), ("pos", "traj_pos"), ("done", "traj_done")):
                merged = np.concatenate([u[k].numpy() for u in us], axis=1)
                assert np.array_equal(merged.view(np.uint8), traj[ref].cpu().numpy().view(np.uint8)), (i, k)
            pos = torch.cat([u["pos"] for u in us], dim=1)            # [T, n_total, N, 2]
            for k in range(C["T"]):
                obs_b.set_positions(pos[k])
                o = obs_b.observe()
                torch.cuda.synchronize()
                assert torch.equal(o["obs_window_occ"], traj["obs_window_occ"][k]), (i, k)
            continue
        for k in KEYS:
            merged = np.concatenate([p_[k] for p_ in got[i]], axis=1)   # -> [T, n_total, ...]
            ref = traj[k].cpu().numpy()
            assert np.array_equal(merged.view(np.uint8), ref.view(np.uint8)), (i, k)
