#!/usr/bin/env python3
"""Benchmark of the batched MAPF gridworld step (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 32x32 grids with
i.i.d. 10% obstacles per env, 16 agents, 4096 envs per GPU (weak scaling:
every rank owns 4096 envs with globally keyed seeds), marl_partial 5x5 window
observations, uniform random actions resident in HBM.

A "step" is one env step of every env of the batch: actions read from HBM,
moves + vertex/edge collisions + fp64 rewards + dones, and every per-step
output a PyMARL runner consumes written to HBM (positions, dones, t, reward,
term, node/edge collisions, avail mask, window obs).  The timed path is the
fused rollout kernel (`mapfx_rollout`, T steps per launch, state kept on
chip); the per-step drop-in path (`mapfx_step`, one launch per step, state
round-trips HBM) is measured too and reported under "per_step".

The timed K env steps run as launches of T = min(K, --chunk) fused steps (one
launch of T = 20 at the driver's --steps 20), every launch prepared before the
timed region so it holds only the foreign calls.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
With --gpus N > 1 and no torchrun environment, bench.py starts the N rank
processes itself (launch_ranks) and refuses to run when fewer than N HIP devices
are visible.  `--dist-selftest` rehearses that multi-rank path on CPU (gloo).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "mapf-marl_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)

CONFIGS = {
    # name: (H=W, N, envs per GPU, p_obstacle, shared warehouse map)
    "c2": (32, 16, 4096, 0.10, False),
    "c3": (64, 64, 2048, None, True),
    "c5": (128, 256, 1024, 0.10, False),
    "c1": (8, 2, 4096, 0.0, False),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=512)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--chunk", type=int, default=64, help="env steps per rollout launch")
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--per-step-steps", type=int, default=200)
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="target CPU work of the cpu_baseline sample (0 disables)")
    ap.add_argument("--no-gather", action="store_true",
                    help="N > 1: skip the RCCL gather leg (reported beside the compute-only value)")
    ap.add_argument("--gather-payload", default="compact",
                    choices=("occ", "planes", "reward_done", "compact"),
                    help="what each chunk gathers to rank 0: compact (default) = reward + u16 "
                         "cell + done bit per agent-step (rank 0 rebuilds observations with "
                         "mapfx_observe; the payload whose rank-0 ingress keeps up with the compute "
                         "at 8 ranks); occ = obs_window_occ (the window as one occupancy plane) + "
                         "reward + done; planes = obs_window + reward + done; reward_done = reward "
                         "+ done only (observations consumed on-rank)")
    ap.add_argument("--dist-selftest", action="store_true",
                    help="CPU/gloo rehearsal of the multi-rank launch + shard + packed gather")
    ap.add_argument("--selftest-envs", type=int, default=6)
    ap.add_argument("--rehearse-shared-gpu", action="store_true",
                    help="rehearsal of the N-rank path on a one-GPU box: every rank on cuda:0, "
                         "collectives over gloo (never a scaling number)")
    ap.add_argument("--pmc", default=None, help="PMC summary (default profiles/pmc_<config>.json)")
    ap.add_argument("--env", default="mapf_grid",
                    choices=("mapf_grid", "marl_partial", "runner", "primal"),
                    help="mapf_grid: the BASELINE.json metric (default); marl_partial: the "
                         "SURVEY §8(f) F1 env on its yaml config, one launch per step; runner: "
                         "F2 batched ParallelRunner episodes; primal: F3 sequential dynamics")
    ap.add_argument("--primal-envs", type=int, default=4096)
    ap.add_argument("--primal-calls", type=int, default=64, help="_step calls per world per launch")
    ap.add_argument("--partial-envs", type=int, default=4096)
    return ap.parse_args()


ACT_SEED = 2          # the device generator's action seed of every timed leg


def mapf_workload(config, window, device, offset=0):
    """One mapf_grid bench leg's batch and output set: what the timed launches run.
    tests/test_gpu_parity.py::test_bench_leg_matches_oracle builds its launches from
    this same function, so the instance a bench line times is the instance the test
    checks against the oracle."""
    import mapfx
    from mapfx.maps import synthetic_instances, warehouse_grid
    S, N, E, p, shared = CONFIGS[config]
    inst = synthetic_instances(E, S, S, N, p_obstacle=p or 0.0, seed=1, env_offset=offset,
                               shared_grid=warehouse_grid(S) if shared else None)
    limit = 2 ** 31 - 1
    # N > 127: agent counts need int16 cells; the window leaves as ONE int16 occupancy
    # plane (obs_window_occ: obstacle = -1, agents = max(v, 0)), 2 B per window cell,
    # instead of two int16 planes (the 0/1 obstacle plane would pay 2 B per cell)
    wkind = "window_occ" if N > 127 else "window"
    wkey = "obs_" + wkind
    b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                            episode_limit=limit, obs=(wkind,), window=window,
                            device=device, env_offset=offset, track_steps=False)
    outs = ("reward", "term", "node", "edge", "avail", wkey, "traj_pos", "traj_done", "traj_t")
    return {"S": S, "N": N, "E": E, "p": p, "shared": shared, "inst": inst, "batch": b,
            "wkind": wkind, "wkey": wkey, "outs": outs, "limit": limit}


def bench_traj(b, T):
    """The trajectory buffers of a timed launch: every rollout output but the f32 reward
    copy (the runner set: the kernel instance without it is the one timed)."""
    traj = b._alloc_out(T)
    traj.pop("reward_f32")
    return traj


def out_bytes_per_env_step(N, W):
    """Algorithmic HBM bytes of one env step of the fused rollout:
    actions N (read) + pos 8N + done N + t 4 + reward 8 + term 1 + node N + edge N
    + avail N + window obs 2*W*W*N (written)."""
    return N + 8 * N + N + 4 + 8 + 1 + N + N + N + 2 * W * W * N


def canonical_bytes_per_env_step(H, Wd, N, W):
    """SURVEY.md §8(d) D-4 canonical bytes of the per-step path (state round-trips
    HBM): reads N + 8N + 8N + N + 4 + H*W/8, writes 8N + N + 4 + 8 + 2N + N + obs."""
    return (N + 8 * N + 8 * N + N + 4 + (H * Wd) // 8) + (8 * N + N + 4 + 8 + 2 * N + N) \
        + 2 * W * W * N


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, need_gpus=True):
    """`bench.py --gpus N` without torchrun: start N rank processes of this script
    (one per GPU, torchrun's RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* environment)
    as children, wait for all of them and return the worst exit code.  The parent
    never touches the GPU (it only counts devices) and never exec()s."""
    import subprocess
    if need_gpus:
        have = torch.cuda.device_count()
        if have < n:
            print("bench.py: --gpus %d requested but only %d HIP device(s) visible; refusing "
                  "to report a %d-rank result" % (n, have, n), file=sys.stderr, flush=True)
            return 2
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0:
                rc = rc or (code if code > 0 else 1)
                for q in pending:          # a failed rank would leave the others blocked
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def dist_selftest(args, rank, world):
    """CPU (gloo) rehearsal of the multi-rank bench plumbing: each rank builds the
    weak-scaling shard bench.py would give it (global env ids [rank*E, (rank+1)*E)),
    packs its (obs-shaped, reward, done) inputs into one ChunkLayout buffer and rank 0
    gathers them with ONE gather.  Rank 0 checks the result against an unsharded
    build of all world*E envs and prints one JSON line."""
    import torch.distributed as dist
    from mapfx.dist import ChunkLayout
    from mapfx.maps import synthetic_instances
    dist.init_process_group("gloo")
    S, N, E = 16, 8, args.selftest_envs
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=1, env_offset=rank * E)
    spec = {"init_pos": ((E, N, 2), torch.int32), "goals": ((E, N, 2), torch.int32),
            "bits": (inst["bits"].shape, torch.uint8), "rank": ((1,), torch.int64)}
    lay = ChunkLayout(spec, order=("init_pos", "goals", "bits", "rank"))
    flat = lay.alloc("cpu")
    v = lay.views(flat)
    v["init_pos"].copy_(torch.from_numpy(inst["init_pos"]))
    v["goals"].copy_(torch.from_numpy(inst["goals"]))
    v["bits"].copy_(torch.from_numpy(inst["bits"]))
    v["rank"].fill_(rank)
    recv = torch.empty((world, lay.nbytes), dtype=torch.uint8) if rank == 0 else None
    dist.gather(flat, gather_list=list(recv.unbind(0)) if rank == 0 else None, dst=0)
    if rank == 0:
        g = lay.views(recv)
        full = synthetic_instances(world * E, S, S, N, p_obstacle=0.1, seed=1)
        ok = (g["rank"].view(-1).tolist() == list(range(world))
              and all(np.array_equal(g[k].reshape((world * E,) + g[k].shape[2:]).numpy(), full[k])
                      for k in ("init_pos", "goals", "bits")))
        print(json.dumps({"dist_selftest": "ok" if ok else "MISMATCH", "n_gpus": world,
                          "world": world, "envs_per_rank": E, "backend": "gloo",
                          "launcher": "torchrun env" if os.environ.get("TORCHELASTIC_RUN_ID")
                          else "bench.py launch_ranks"}), flush=True)
        rc = 0 if ok else 3
    else:
        rc = 0
    dist.barrier()
    dist.destroy_process_group()
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:],
                              need_gpus=not (args.dist_selftest or args.rehearse_shared_gpu)))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse_shared_gpu:
        local = 0
    if world != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus), file=sys.stderr)
        sys.exit(2)
    if args.dist_selftest:
        sys.exit(dist_selftest(args, rank, world))
    if torch.cuda.device_count() <= local:
        print("bench.py: rank %d needs HIP device %d, %d visible" % (rank, local,
              torch.cuda.device_count()), file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.rehearse_shared_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import mapfx
    from mapfx.maps import synthetic_instances, warehouse_grid

    if args.env == "marl_partial":
        return run_partial(args, dist, rank, world, local)
    if args.env == "runner":
        return run_runner(args, dist, rank, world, local)
    if args.env == "primal":
        return run_primal(args, dist, rank, world, local)
    S, N, E, p, shared = CONFIGS[args.config]
    W = args.window
    K, WU = args.steps, args.warmup
    T = max(1, min(K, args.chunk))          # env steps per rollout launch
    n_full, rem = divmod(K, T)              # K = n_full launches of T (+ one of rem)
    n_wu = -(-WU // T) if WU > 0 else 0     # warmup: whole launches of the timed shape
    offset = rank * E                 # weak scaling: rank r owns global envs [r*E, (r+1)*E)
    wl = mapf_workload(args.config, W, "cuda:%d" % local, offset)
    inst, b, wkind, wkey, outs, limit = (wl[k] for k in ("inst", "batch", "wkind", "wkey",
                                                         "outs", "limit"))
    b.reset()
    stream = torch.cuda.current_stream()
    acts = b.gen_actions(n_wu * T + K, seed=ACT_SEED)           # inputs resident in HBM
    traj = bench_traj(b, T)

    def plan(k0, t, events=None):
        tr = traj if t == T else {k: v[:t] for k, v in traj.items()}
        return b.rollout_plan(t, actions=acts[k0:k0 + t], traj=tr, outputs=outs, stream=stream,
                              events=events)

    # ---- warmup: whole launches of the timed shape (>= W env steps) ----
    for i in range(n_wu):
        plan(i * T, T)()
    torch.cuda.synchronize()
    # every timed launch prepared up front: the timed region is the ctypes calls only
    # (no event packets in it: an event record costs ~3 us of wall time at this size,
    # profiles/r02_wall_probe.json)
    k0 = n_wu * T
    nl = n_full + (1 if rem else 0)
    plans = [plan(k0 + i * T, T) for i in range(n_full)]
    if rem:
        plans.append(plan(k0 + n_full * T, rem))
    # the kernel's launch duration, measured live right after the timed region on the
    # same stream: the same launches again, each recording start / stop events at the
    # kernel's own begin / end (hipExtLaunchKernel, mapfx_rollout_timed) -- the
    # duration rocprofv3 reports for the kernel
    # (KREP passes of the K steps, at least 15 launches in all; the median pass is
    # reported, so one disturbed launch does not move the roofline, and a rocprofv3 trace
    # of the command averages enough launches to compare with it)
    KREP = max(5, -(-15 // nl))
    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for _ in range(nl)] for _ in range(KREP)]
    for rep_evs in evs:     # torch creates the HIP events at their first record()
        for a_, b_ in rep_evs:
            a_.record(stream)
            b_.record(stream)
    kplans = []
    for rep_evs in evs:
        kp = [plan(k0 + i * T, T, rep_evs[i]) for i in range(n_full)]
        if rem:
            kp.append(plan(k0 + n_full * T, rem, rep_evs[-1]))
        kplans.append(kp)
    # every replay pass starts from the state the timed region started from: the replays
    # then run the timed launches' exact work (a state hundreds of steps further on is a
    # different workload -- C3's done agents crowd the aisles: 175 -> 223 us per launch,
    # profiles/r05_c3_trace_gaps.json)
    state0 = [x.clone() for x in (b.pos, b.done, b.t)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()

    # ---- timed: exactly K env steps of all envs ----
    t0 = time.perf_counter()
    for pl in plans:
        pl()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    from mapfx import _abi
    kernel_name = _abi.last_kernel()    # the instance the timed launches ran
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    for kp in kplans:       # kernel timing passes (untimed wall clock)
        for x, x0 in zip((b.pos, b.done, b.t), state0):
            x.copy_(x0)
        for pl in kp:
            pl()
    torch.cuda.synchronize()
    kern_passes = sorted(sum(a_.elapsed_time(b_) for a_, b_ in rep_evs) for rep_evs in evs)
    kern_ms_total = kern_passes[KREP // 2]     # median pass; events on the launch stream
    kern_ms = kern_ms_total / len(plans)
    el = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    total_envs = E * world
    value = total_envs * N * K / elapsed           # agent-steps/s (agents x envs), whole job
    bpes = out_bytes_per_env_step(N, W)
    state_io = E * ((8 + 8 + 1) * N + 4 + inst["bits"].shape[1] * (0 if shared else 1)
                    + (8 + 1) * N + 4)             # per-launch state read + write-back
    timed_bytes = E * K * bpes + len(plans) * state_io
    launch_bytes = timed_bytes / len(plans)
    achieved = timed_bytes / (kern_ms_total * 1e-3) / 1e9

    # ---- per-step path (one mapfx_step launch per env step) ----
    # `ks` launches captured once as a HIP graph and replayed: kernels back to back,
    # no Python / ctypes launch overhead between them ("eager" = one Python call
    # per step, as the drop-in env does it, reported beside it).
    per_step = None
    if args.per_step_steps > 0:
        b2 = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                                 episode_limit=limit, obs=(wkind,), window=W,
                                 device="cuda:%d" % local, env_offset=offset, track_steps=False)
        b2.reset()
        ks = args.per_step_steps
        na = acts.shape[0]
        pouts = ("reward", "term", "node", "edge", "avail", wkey)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for k in range(ks):
                b2.step(acts[k % na], outputs=pouts)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for k in range(ks):
                b2.step(acts[k % na], outputs=pouts)
        graph.replay()
        torch.cuda.synchronize()
        step_kernel = _abi.last_kernel()
        pe0, pe1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        t1 = time.perf_counter()
        pe0.record(stream)
        for _ in range(reps):
            graph.replay()
        pe1.record(stream)
        torch.cuda.synchronize()
        pel = time.perf_counter() - t1
        pk_ms = pe0.elapsed_time(pe1) / (reps * ks)
        t2 = time.perf_counter()
        for k in range(ks):
            b2.step(acts[k % na], outputs=pouts)
        torch.cuda.synchronize()
        eager_ms = (time.perf_counter() - t2) / ks * 1e3
        cb = canonical_bytes_per_env_step(S, S, N, W)
        # HBM bytes per launch of the per-step kernel from its own PMC profile
        # (profiles/pmc_<config>_step.json, taken of this bench command)
        ptraffic, ptraffic_src = profile_traffic("%s_step" % args.config, kernel=step_kernel,
                                                 config=args.config + "_step", T=1, E=E)
        per_step = {
            "value": round(E * N * reps * ks / pel * world, 1),
            "ms_per_step": round(pel / (reps * ks) * 1e3, 5),
            "kernel_ms": round(pk_ms, 5),
            "eager_ms_per_step": round(eager_ms, 5),
            "launch": "HIP graph of %d mapfx_step launches, replayed" % ks,
            "kernel": step_kernel,
            "roofline": {"bound": "hbm", "achieved": round(E * cb / (pk_ms * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(E * cb / (pk_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": ptraffic, "traffic_source": ptraffic_src,
                         "bytes_per_env_step": cb, "bytes_per_launch": E * cb},
        }

    # ---- RCCL gather of (obs, reward, done) to rank 0 (N > 1: on by default) ----
    gather = None
    if dist and not args.no_gather:
        gb, gouts, gkeys = b, outs, (wkey, "reward", "traj_done")
        if args.gather_payload == "reward_done":
            gkeys = ("reward", "traj_done")
        elif args.gather_payload == "compact":
            from mapfx.dist import COMPACT_KEYS
            gkeys = COMPACT_KEYS
        elif args.gather_payload == "occ" and wkind != "window_occ":
            gb = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                                     episode_limit=limit, obs=("window_occ",), window=W,
                                     device="cuda:%d" % local, env_offset=offset, track_steps=False)
            gb.reset()
            gouts = tuple("obs_window_occ" if k == wkey else k for k in outs)
            gkeys = ("obs_window_occ", "reward", "traj_done")
        gather = time_gather(dist, gb, acts, gouts, T, n_wu * T, K, world, E, N, gkeys,
                             args.gather_payload)

    # ---- CPU baseline: the oracle's C restatement on this host (rank 0, N=1) ----
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(inst, S, N, E, W, args.cpu_seconds)

    traffic, traffic_src = profile_traffic(args.config, kernel=kernel_name, path=args.pmc,
                                           config=args.config, T=T, E=E)

    if rank == 0:
        line = {
            "metric": "env-steps/sec (agents×envs) at 32×32/16-agent, 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": WU,
            "ms_per_step": round(elapsed / K * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32+f64",
            "data": "synthetic (splitmix64 random maps p=%.2f, distinct free starts/goals, "
                    "uniform random actions in HBM)" % (p or 0.0),
            "config": {"workload": "%s: %dx%d %s, %d agents, %d envs/GPU, window %dx%d obs%s, "
                                   "fused rollout T=%d env-steps per launch (%d launch%s)"
                                   % (args.config, S, S, "square synthetic warehouse (shelf "
                                      "blocks, stands in for highway_layout_v19)" if shared
                                      else "grid", N, E, W, W,
                                      " (one int16 occupancy plane per agent)"
                                      if wkind == "window_occ" else "", T, len(plans),
                                      "" if len(plans) == 1 else "es"),
                       "envs_total": total_envs, "agents": N, "grid": [S, S], "chunk_T": T,
                       "parallelism": "env-shard x%d" % world
                       + (" (REHEARSAL: all ranks on cuda:0 over gloo)" if args.rehearse_shared_gpu
                          else "")},
            "env_steps_per_s": round(total_envs * K / elapsed, 1),
            "kernel_ms_per_launch": round(kern_ms, 5),
            "kernel": kernel_name,
            "build_id": _abi.build_id(),
            "timing": {"wall_ms": round(elapsed * 1e3, 4),
                       "kernel_ms_events": round(kern_ms_total, 4),
                       "kernel_timing": "per-launch start/stop events recorded at the "
                                        "kernel's begin/end (hipExtLaunchKernel) on %d replays "
                                        "of the same launches right after the timed region; "
                                        "median replay" % KREP,
                       "kernel_ms_replays": [round(x, 4) for x in kern_passes],
                       "launches": len(plans),
                       "wall_over_kernel": round(elapsed * 1e3 / kern_ms_total, 3)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "bytes_per_env_step": bpes, "bytes_per_launch": int(launch_bytes)},
            "per_step": per_step,
            "cpu_baseline": cpu,
        }
        if gather is not None:
            line["gather"] = gather
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


# rank 0's xGMI ingress: 7 peers x one ~153 GB/s link each
XGMI_LINK_GBS = 153.0
GATHER_MIN_CHUNKS = 3


def time_gather(dist, b, acts, outs, T, k0, K, world, E, N, keys, payload):
    """The same K env steps as rollout chunks of T, each chunk's gathered outputs
    (`keys`: window obs, reward, done) packed in one buffer and gathered to rank 0 with
    ONE RCCL gather on a side stream, overlapped with the next chunk
    (mapfx.dist.OverlappedGather).  Rank 0 orders a read of every chunk after its
    gather (stream wait, no sync).  The ingress bound: rank 0 receives (world - 1)
    chunks per chunk time over at most (world - 1) links."""
    from mapfx.dist import OverlappedGather
    og = OverlappedGather(b, T, keys=keys, outputs=outs, compact=(payload == "compact"))
    og.step_chunk(actions=acts[:T])                  # warm the communicator
    og.result(0)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    # at least GATHER_MIN_CHUNKS chunks whatever --steps is: with one chunk the
    # double-buffered overlap (chunk i + 1 computing while chunk i travels) would
    # never be what gets timed
    nch = max(GATHER_MIN_CHUNKS, K // T)
    if acts.shape[0] < k0 + nch * T:                 # more inputs, resident before timing
        acts = b.gen_actions(k0 + nch * T, seed=2)
        torch.cuda.synchronize()
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(nch):
        og.step_chunk(actions=acts[k0 + i * T:k0 + (i + 1) * T])
        og.result(og.i - 1)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    dist.barrier()
    t = torch.tensor([el], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    per_chunk = int(og.bytes_per_chunk())
    ingress = (world - 1) * per_chunk
    return {"value": round(world * E * N * nch * T / el, 1),
            "ingress_arithmetic": payload_arithmetic(T, E, N, b.window, world),
            "ms_per_step": round(el / (nch * T) * 1e3, 5),
            "steps": nch * T, "chunk_steps": T, "payload": payload, "keys": list(keys),
            "bytes_per_rank_per_chunk": per_chunk,
            "rank0_ingress_bytes_per_chunk": ingress,
            "ingress_bound_ms_per_chunk": round(ingress / (max(1, world - 1) * XGMI_LINK_GBS * 1e9)
                                                * 1e3, 5),
            "collective": "one torch.distributed.gather (%s) per chunk to rank 0 on a side "
                          "stream, packed %s buffer" % ("RCCL" if dist.get_backend() == "nccl"
                                                        else dist.get_backend(), "+".join(keys))}


def payload_arithmetic(T, E, N, W, world):
    """Bytes per rank per T-step chunk of each --gather-payload (16-B aligned fields, as
    mapfx.dist.ChunkLayout lays them out) and rank 0's xGMI ingress time at N ranks:
    (world - 1) chunks over (world - 1) links of XGMI_LINK_GBS each."""
    al = lambda n: -(-n // 16) * 16   # noqa: E731
    fields = {"compact": (8 * T * E, 2 * T * E * N, T * E * ((N + 7) // 8)),
              "occ": (T * E * N * W * W, 8 * T * E, T * E * N),
              "planes": (2 * T * E * N * W * W, 8 * T * E, T * E * N),
              "reward_done": (8 * T * E, T * E * N)}
    out = {}
    for k, f in fields.items():
        per = sum(al(x) for x in f)
        out[k] = {"bytes_per_rank_per_chunk": per,
                  "rank0_ingress_bytes_per_chunk": (world - 1) * per,
                  "ingress_bound_ms_per_chunk": round(per / (XGMI_LINK_GBS * 1e9) * 1e3, 5)
                  if world > 1 else 0.0}
    return out


PARTIAL_YAML = dict(  # MARL-curve-main/src/config/envs/marl_partial.yaml:3-23
    obs_window=5, obs_knn_agents=5, episode_limit=100, move_reward=0, stay_reward=-0.1,
    stay_goal_reward=1, node_collide_reward=-2000, edge_collide_reward=-2000,
    env_collide_reward=-2000, complete_reward=1000, complete_fac=1.5, gamma=0.99)


def kernel_instance(name):
    """The instance part of a demangled kernel name (tools/pmc_traffic.instance)."""
    i = name.find("<")
    j = name.find("(", i) if i >= 0 else -1
    return (name[:j] if j > 0 else name).strip()


def build_src(build_id):
    """The `src=<hash>` part of a build id ("src=<hash> git=<head>[+dirty] tu=..."), or None."""
    for part in (build_id or "").split():
        if part.startswith("src=") and part != "src=unknown":
            return part
    return None


def kernel_unit(kernel):
    """The translation unit (mapf-marl_amd/csrc/<unit>.hip) that defines a kernel."""
    base = kernel_instance(kernel or "").split("<")[0].split("::")[-1].strip()
    for pre, unit in (("partial_", "partial"), ("primal_", "primal"), ("runner_", "runner")):
        if base.startswith(pre):
            return unit
    return "mapfx"


def build_unit(build_id, unit):
    """The hash of one translation unit in a build id's `tu=` part, or None."""
    for part in (build_id or "").split():
        if part.startswith("tu="):
            for item in part[3:].split(","):
                name, _, h = item.partition(":")
                if name == unit and h:
                    return h
    return None


def profile_traffic(leg, kernel=None, path=None, **match):
    """(traffic bytes per launch, source) from profiles/pmc_<leg>.json, or (None, why).
    The file is written by tools/pmc_traffic.py from separate rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes (MI355X_MICROARCH.md corrections).  It is cited only when it was
    taken of THIS kernel code (the `src=` hash of its build_id -- the HIP sources,
    headers and compiler flags -- equals that of the loaded library, or the `tu=` hash
    of the translation unit that defines the kernel does: its source, the headers and
    its flags; the `git=` part records the commit it was built at and is reported, not
    compared: rebuilding the same sources at a later commit gives the same kernels), of
    the same kernel instance
    the bench just launched (`kernel`, mapfx_last_kernel) and of this workload (every
    `match` key equal); otherwise traffic is null and the reason is reported instead
    of a stale figure."""
    from mapfx import _abi
    path = path or os.path.join(REPO, "profiles", "pmc_%s.json" % leg)
    rel = os.path.relpath(path, REPO)
    try:
        with open(path) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return None, "no profile %s" % rel
    same_src = build_src(pm.get("build_id")) is not None and \
        build_src(pm.get("build_id")) == build_src(_abi.build_id())
    unit = kernel_unit(kernel or pm.get("kernel"))
    same_unit = build_unit(pm.get("build_id"), unit) is not None and \
        build_unit(pm.get("build_id"), unit) == build_unit(_abi.build_id(), unit)
    if not (same_src or same_unit):
        return None, "refused %s: taken of build %r, running %r" % (rel, pm.get("build_id"),
                                                                    _abi.build_id())
    if kernel is not None and kernel_instance(pm.get("kernel", "")) != kernel_instance(kernel):
        return None, "refused %s: profiled kernel %r, launched %r" % (rel, pm.get("kernel"), kernel)
    bad = [k for k, v in match.items() if pm.get(k) != v]
    if bad or not pm.get("traffic_bytes_per_launch"):
        return None, "refused %s: workload keys %s differ" % (rel, bad)
    return pm["traffic_bytes_per_launch"], "%s (build %s): %s" % (rel, pm.get("build_id"),
                                                                  pm.get("command", "rocprofv3 --pmc passes"))


def partial_bytes_per_env_step(N, D, HW, gd_bytes=2):
    """Algorithmic HBM bytes of one MARL_PARTIAL env step (state round-trips HBM):
    reads actions N + state 27N + 13 (pos 8, steps 4, at_goal 1, done 1, goal_cost 4,
    node 1, edge 4, carried goal distance 4 per agent) + goal/init 16N + one goal-distance
    entry per (moving) agent (gd_bytes: 1 for the u8 tables of maps up to 255 cells, 2
    for int16) + bitmap HW/8; writes obs 4DN + reward 8 + state 12 + avail N + state
    27N + 9."""
    return (N + 27 * N + 13 + 16 * N + gd_bytes * N + HW // 8) + (4 * D * N + 8 + 12 + N + 27 * N + 9)


def run_partial(args, dist, rank, world, local):
    """MARL_PARTIAL_ENV on the reference's yaml config: 8x8 empty
    map, 15 agents, window 5, K = 5, episode limit 100; E envs per GPU, one
    mapfx_partial_step launch per env step, every env reset each 100 steps."""
    import mapfx
    from mapfx.maps import synthetic_instances
    S, N, E = 8, 15, args.partial_envs
    limit = PARTIAL_YAML["episode_limit"]
    # whole episodes: round --steps / --warmup up to multiples of the episode limit
    K = -(-args.steps // limit) * limit
    WU = -(-args.warmup // limit) * limit
    offset = rank * E
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.0, seed=1, env_offset=offset)
    grids = np.zeros((1, S, S), dtype=np.int8)
    b = mapfx.MarlPartialBatch(inst["init_pos"], inst["goals"], grids=grids,
                               device="cuda:%d" % local, env_offset=offset, **PARTIAL_YAML)
    b.reset()
    ga = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                             obs=(), device="cuda:%d" % local, env_offset=offset,
                             track_steps=False)
    acts = ga.gen_actions(WU + K, seed=2)  # uniform actions from the device generator, in HBM
    del ga
    stream = torch.cuda.current_stream()

    # One episode (reset + `limit` steps, one kernel launch each) captured once as a
    # HIP graph and replayed: the per-step launches run back to back without the
    # Python / ctypes launch overhead of the drop-in path between them.
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        b.reset()
        for k in range(limit):           # eager warm-up of every launch before capture
            b.step(acts[k])
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    with torch.cuda.graph(graph):
        b.reset()
        for k in range(limit):
            b.step(acts[k])
    for _ in range(WU // limit):
        graph.replay()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)       # create the HIP events outside the timed region
    e1.record(stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(K // limit):
        graph.replay()
    e1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    kern_ms = e0.elapsed_time(e1) / K   # per env step, including the per-episode reset
    el = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    # the drop-in style (one Python call per step) for reference
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    b.reset()
    for k in range(limit):
        b.step(acts[k])
    torch.cuda.synchronize()
    eager_ms = (time.perf_counter() - t1) / limit * 1e3
    from mapfx import _abi
    kernel_name = _abi.last_kernel()     # the step instance the graph replays
    D = b.obs_dim
    bpes = partial_bytes_per_env_step(N, D, S * S, b.goal_dist.element_size())
    achieved = E * bpes / (kern_ms * 1e-3) / 1e9
    # traffic per launch (one env step of E envs) from the PMC profile of this workload
    traffic, traffic_src = profile_traffic("partial", kernel=kernel_name, E=E, N=N, S=S)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = partial_cpu_baseline(inst, S, N, args.cpu_seconds)
    if rank == 0:
        print(json.dumps({
            "metric": "MARL_PARTIAL env-steps/sec (agents x envs), yaml config 8x8/15 agents",
            "value": round(E * world * N * K / elapsed, 1), "unit": "agent-steps/s",
            "n_gpus": world, "steps": K, "warmup": WU, "ms_per_step": round(elapsed / K * 1e3, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32+f64+f32",
            "data": "synthetic (empty 8x8 map, distinct random starts/goals; one episode of "
                    "uniform random actions in HBM, replayed every episode)",
            "config": {"workload": "marl_partial yaml: 8x8 empty, 15 agents, window 5, K 5, "
                                   "limit 100, %d envs/GPU, one launch per step, episodes "
                                   "replayed as a HIP graph (reset + 100 steps)" % E,
                       "envs_total": E * world, "agents": N, "obs_dim": D,
                       "parallelism": "env-shard x%d" % world},
            "env_steps_per_s": round(E * world * K / elapsed, 1),
            "kernel_ms_per_step": round(kern_ms, 5),
            "eager_ms_per_step": round(eager_ms, 5),
            "kernel": kernel_name, "build_id": _abi.build_id(),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "bytes_per_env_step": bpes, "bytes_per_launch": E * bpes},
            "cpu_baseline": cpu}), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def primal_bytes_per_call(s):
    """Algorithmic HBM bytes of one PRIMAL `_step((agent_id, action))` call
    (SURVEY §8(f) F3): agent id + action read (8), reward f64 + done + next mask +
    on_goal + valid (12), the 4 x s x s observation maps (u8) and the f64 goal vector (24)."""
    return 8 + 12 + 4 * s * s + 24


def run_primal(args, dist, rank, world, local):
    """PRIMAL sequential dynamics (envs/mapf_primal.py:549-637): E
    worlds of 32 x 32 (10 % obstacles) with 16 agents and observation_size 10 per GPU;
    each launch makes `--primal-calls` single-agent `_step` calls per world, in order
    (agents round robin, random actions), every call's observation written."""
    import mapfx
    from mapfx.maps import synthetic_instances
    S, N, s_obs, E, KC = 32, 16, 10, args.primal_envs, args.primal_calls
    offset = rank * E
    inst = synthetic_instances(E, S, S, N, p_obstacle=0.10, seed=1, env_offset=offset)
    b = mapfx.PrimalBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                          observation_size=s_obs, device="cuda:%d" % local)
    rng = np.random.default_rng(7 + rank)
    ids = torch.from_numpy(np.tile((np.arange(KC) % N + 1).astype(np.int32), (E, 1))).cuda()
    acts = torch.from_numpy(rng.integers(0, 5, size=(E, KC)).astype(np.int32)).cuda()
    R = max(1, args.steps // KC)          # launches timed
    RW = max(1, args.warmup // KC)
    for _ in range(RW):
        b.act(ids, acts)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    e1.record(stream)
    pos0 = b.pos.clone()     # the event-timed launches below replay the timed ones from here
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(R):
        b.act(ids, acts)
    e1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    wall_kern_ms = e0.elapsed_time(e1) / R  # stream interval per launch, host launch gaps included
    # the kernel's own duration: the same launches again, each recording start / stop at
    # the kernel's begin / end (mapfx_primal_act_timed, hipExtLaunchKernel); median
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(R)]
    for a0, a1 in ev:
        a0.record(stream)   # creates the HIP events
        a1.record(stream)
    b.pos.copy_(pos0)
    for pr in ev:
        b.act(ids, acts, events=pr)
    torch.cuda.synchronize()
    from mapfx import _abi
    kernel_name = _abi.last_kernel()
    kern_list = sorted(a0.elapsed_time(a1) for a0, a1 in ev)
    kern_ms = kern_list[len(kern_list) // 2]
    el = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    b.check_err()
    calls = E * world * KC * R
    bpc = primal_bytes_per_call(s_obs)
    launch_bytes = E * (KC * bpc + (8 + 8 + 8) * N + inst["bits"].shape[1])  # + pos/goal in, pos out
    achieved = launch_bytes / (kern_ms * 1e-3) / 1e9
    # the profile is keyed by what tools/pmc_traffic.py records: config, calls per launch
    # (T) and worlds (E); the bench's fixed 32 x 32 / 16 agents / s = 10 shape is implied
    traffic, traffic_src = profile_traffic("primal", kernel=kernel_name, config="primal", E=E, T=KC)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        from oracle.primal_dyn_oracle import PrimalWorld
        ids_h, acts_h = ids.cpu().numpy(), acts.cpu().numpy()
        t_start, n, e = time.perf_counter(), 0, 0
        while time.perf_counter() - t_start < args.cpu_seconds:
            we = e % E
            w = PrimalWorld(inst["grid"][we % inst["grid"].shape[0]], inst["init_pos"][we],
                            inst["goals"][we], s_obs)
            for k in range(KC):
                w.step(int(ids_h[we, k]) - 1, int(acts_h[we, k]))
            n += KC
            e += 1
        el_c = time.perf_counter() - t_start
        cpu = {"value": round(n / el_c, 1), "unit": "agent-calls/s", "cores": 1, "kind": "port",
               "sample": "%d calls (%d worlds x %d) of the same workload: "
                         "oracle/primal_dyn_oracle.py PrimalWorld.step, %.1f s" % (n, e, KC, el_c)}
    if rank == 0:
        print(json.dumps({
            "metric": "PRIMAL _step calls/sec (sequential single-agent dynamics + observation)",
            "value": round(calls / elapsed, 1), "unit": "agent-calls/s",
            "n_gpus": world, "steps": KC * R, "warmup": KC * RW,
            "ms_per_step": round(elapsed / (KC * R) * 1e3, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32+f64+u8",
            "data": "synthetic (32x32 maps, 10% obstacles, distinct free starts/goals; agents "
                    "round robin, uniform random actions in HBM)",
            "config": {"workload": "primal: %d worlds/GPU of 32x32, %d agents, observation_size "
                                   "%d, %d _step calls per world per launch (%d launches)"
                                   % (E, N, s_obs, KC, R),
                       "envs_total": E * world, "agents": N, "parallelism": "env-shard x%d" % world},
            "kernel_ms_per_launch": round(kern_ms, 5),
            "kernel": kernel_name, "build_id": _abi.build_id(),
            "timing": {"kernel_ms_launches": [round(x, 5) for x in kern_list],
                       "stream_ms_per_launch": round(wall_kern_ms, 5),
                       "kernel_timing": "per-launch start/stop events recorded at the kernel's "
                                        "begin/end (hipExtLaunchKernel) on %d launches right after "
                                        "the timed region; median" % R},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "bytes_per_call": bpc, "bytes_per_launch": int(launch_bytes)},
            "cpu_baseline": cpu}), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


class RandomAvailMAC:
    """select_actions: uniform over each agent's available actions, on the device
    (the distribution of epsilon-greedy's random branch at epsilon = 1,
    action_selectors.py:65-69: Categorical over the avail mask), sampled as the
    argmax of uniform noise on the available actions (3 launches, no sync)."""

    def __init__(self, seed=0):
        self.gen = None
        self.seed = seed

    def init_hidden(self, batch_size):
        pass

    def select_actions(self, batch, t_ep, t_env, bs, test_mode=False):
        avail = batch["avail_actions"][bs, t_ep]
        if self.gen is None:
            self.gen = torch.Generator(device=avail.device)
            self.gen.manual_seed(self.seed)
        noise = torch.rand(avail.shape, generator=self.gen, device=avail.device)
        return torch.argmax(noise * avail, dim=-1)


def run_runner(args, dist, rank, world, local):
    """the batched ParallelRunner (mapfx/runners.py) collecting
    episodes of the marl_partial yaml config into device-resident EpisodeBatch
    storage, a random-available-action MAC choosing actions from the batch."""
    import tempfile
    import types
    from mapfx.episode import DeviceEpisodeBatch
    from mapfx.maps import synthetic_instances
    from mapfx.runners import ParallelRunner
    S, N, B = 8, 15, args.partial_envs
    inst = synthetic_instances(B, S, S, N, p_obstacle=0.0, seed=1, env_offset=rank * B)
    tmp = tempfile.mkdtemp(prefix="mapfx_runner_")
    mp = os.path.join(tmp, "empty-8-8.map")
    with open(mp, "w") as f:
        f.write("type octile\nheight 8\nwidth 8\nmap\n" + "\n".join(["." * 8] * 8) + "\n")
    ea = dict(PARTIAL_YAML, grid_file_path=mp, agents_path=os.path.join(tmp, "x-"), n_agents=N)
    rargs = types.SimpleNamespace(env="marl_partial", batch_size_run=B, device="cuda:%d" % local,
                                  env_args=ea, episode_batch_cls=DeviceEpisodeBatch,
                                  test_nepisode=B, runner_log_interval=1 << 62)
    runner = ParallelRunner(rargs, None, instance_fn=lambda ep: (inst["init_pos"], inst["goals"]))
    info = runner.get_env_info()
    scheme = {"state": {"vshape": info["state_shape"]},
              "obs": {"vshape": info["obs_shape"], "group": "agents"},
              "actions": {"vshape": (1,), "group": "agents", "dtype": torch.long},
              "avail_actions": {"vshape": (info["n_actions"],), "group": "agents",
                                "dtype": torch.int},
              "reward": {"vshape": (1,)}, "terminated": {"vshape": (1,), "dtype": torch.uint8}}
    from mapfx.episode import OneHot
    runner.setup(scheme, {"agents": N}, {"actions": ("actions_onehot", [OneHot(out_dim=5)])},
                 RandomAvailMAC(seed=rank))   # PyMARL's preprocess (run.py): one-hot actions
    runs = max(1, args.steps // info["episode_limit"])
    for _ in range(max(1, args.warmup // info["episode_limit"])):
        runner.run()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t_env0 = runner.t_env
    t0 = time.perf_counter()
    for _ in range(runs):
        runner.run()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    steps = runner.t_env - t_env0
    el = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.barrier()
    elapsed = float(el.item())
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = partial_cpu_baseline(inst, S, N, args.cpu_seconds)
    # roofline of the runner step on the wall clock (the MAC's torch kernels and the
    # launch gaps included): per env step, the env step's own bytes plus the
    # EpisodeBatch rows the runner writes (episode_buffer.py:100-134 layouts: obs f32,
    # state f32, avail_actions i32, actions i64, actions_onehot f32, reward f32,
    # terminated u8, filled i64) and the MAC's read of the avail row
    D = info["obs_shape"]
    row_bytes = 4 * N * D + 4 * 3 + 4 * 5 * N + 8 * N + 4 * 5 * N + 4 + 1 + 8 + 4 * 5 * N
    bpes = partial_bytes_per_env_step(N, D, S * S, runner.env.goal_dist.element_size()) + row_bytes
    achieved = steps * world * bpes / elapsed / 1e9
    if rank == 0:
        print(json.dumps({
            "metric": "ParallelRunner env-steps/sec (agents x envs) into EpisodeBatch, marl_partial yaml",
            "value": round(steps * world * N / elapsed, 1), "unit": "agent-steps/s", "n_gpus": world,
            "steps": runs * info["episode_limit"], "warmup": args.warmup,
            "ms_per_step": round(elapsed / max(1, runs * info["episode_limit"]) * 1e3, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32+f64+f32",
            "data": "synthetic (empty 8x8 map, distinct random starts/goals, random available actions "
                    "chosen on the device from the batch)",
            "config": {"workload": "batched ParallelRunner.run(): %d envs x 100-step episodes, "
                                   "mapfx.episode.DeviceEpisodeBatch storage" % B,
                       "envs_total": B * world, "agents": N, "parallelism": "env-shard x%d" % world},
            "env_steps_per_s": round(steps * world / elapsed, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved / world, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / world / HBM_PEAK_GBS, 4),
                         "traffic": None, "bytes_per_env_step": bpes, "episode_row_bytes": row_bytes,
                         "timing": "wall clock of run() per GPU: MAC torch kernels, launch gaps "
                                   "and the 2-step-late loop exit included"},
            "cpu_baseline": cpu}), flush=True)
    if dist:
        dist.destroy_process_group()


def partial_cpu_baseline(inst, S, N, seconds):
    """The Python restatement (oracle/partial_oracle.py, the reference's algorithm
    in plain Python, one core) on a bounded sample: as many env-steps of the same
    workload as fit in ~`seconds`."""
    from oracle.partial_oracle import PartialEnvState
    grid = np.zeros((S, S), dtype=np.int8)
    rng = np.random.default_rng(3)
    n_done, t0 = 0, time.perf_counter()
    e = 0
    while time.perf_counter() - t0 < seconds:
        env = PartialEnvState(grid, inst["init_pos"][e], inst["goals"][e], **PARTIAL_YAML)
        for _ in range(PARTIAL_YAML["episode_limit"]):
            env.step(rng.integers(0, 5, size=N))
            env.obs()
            env.avail()
            n_done += 1
        e += 1
    el = time.perf_counter() - t0
    return {"value": round(n_done * N / el, 1), "unit": "agent-steps/s", "cores": 1, "kind": "port",
            "sample": "%d env-steps (%d episodes of 100) of the same workload: "
                      "oracle/partial_oracle.py step + get_obs + avail, %.1f s" % (n_done, e, el)}


def cpu_baseline(inst, S, N, E, W, seconds):
    """Time the oracle's bit-identical C restatement (OpenMP over envs) on a bounded
    sample of the same workload: all envs of the shard, as many steps as fit in
    ~`seconds` of CPU work.  Test infrastructure used only as the baseline."""
    from oracle import corc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    ob = corc.OracleBatch(inst["bits"], inst["init_pos"], inst["goals"], S, S, limit=2 ** 31 - 1,
                          nthreads=threads)
    ob.rollout(2, seed=2, t0=0, window=W)         # thread-pool / page warm-up
    ob.reset()
    t0 = time.perf_counter()
    ob.rollout(64, seed=2, t0=0, window=W)
    probe = time.perf_counter() - t0
    steps = int(max(1, min(200000, seconds / max(probe / 64, 1e-6))))
    ob.reset()
    t0 = time.perf_counter()
    ob.rollout(steps, seed=2, t0=0, window=W)
    el = time.perf_counter() - t0
    return {"value": round(E * N * steps / el, 1), "unit": "agent-steps/s", "cores": threads,
            "kind": "port",
            "sample": "%d envs x %d steps (%.1f s) of the same workload: oracle/mapf_oracle.c "
                      "step + avail + window obs, OpenMP over envs" % (E, steps, el)}


if __name__ == "__main__":
    main()
