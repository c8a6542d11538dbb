#!/usr/bin/env python3
"""Host side of the driver's launch (bench.py --gpus 1 --steps 20 --warmup 5): how long
the prepared mapfx_rollout foreign call takes on the host (enqueue only), how long until
torch.cuda.synchronize() returns, and the floors beside them (a ctypes call of an empty
C function; a torch launch of a tiny kernel + sync).  Medians of --reps.
usage: python3 tools/launch_probe.py [--reps 50] [--sched 1]"""
import argparse
import ctypes
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--sched", type=int, default=-1,
                    help="hipSetDeviceFlags(value) before the device is touched (1 spin, 2 yield, 4 blocking)")
    a = ap.parse_args()
    if a.sched >= 0:
        hip = ctypes.CDLL("libamdhip64.so")
        print("hipSetDeviceFlags(%d) -> %d" % (a.sched, hip.hipSetDeviceFlags(ctypes.c_uint(a.sched))))
    import bench
    import mapfx
    from mapfx._abi import lib
    from mapfx.maps import synthetic_instances
    S, N, E, p, shared = bench.CONFIGS["c2"]
    inst = synthetic_instances(E, S, S, N, p_obstacle=p or 0.0, seed=1)
    b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                            episode_limit=2 ** 31 - 1, obs=("window",), window=5, track_steps=False)
    b.reset()
    T = 20
    acts = b.gen_actions(T, seed=2)
    outs = ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos", "traj_done", "traj_t")
    traj = b._alloc_out(T)
    traj.pop("reward_f32")
    plan = b.rollout_plan(T, actions=acts, traj=traj, outputs=outs)
    for _ in range(5):
        plan()
    torch.cuda.synchronize()
    enq, total = [], []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        plan()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append((t1 - t0) * 1e6)
        total.append((t2 - t0) * 1e6)
    ver = lib.mapfx_abi_version
    cc = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        ver()
        cc.append((time.perf_counter() - t0) * 1e6)
    x = torch.zeros(16, device="cuda")
    tiny = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x.fill_(1.0)
        torch.cuda.synchronize()
        tiny.append((time.perf_counter() - t0) * 1e6)
    med = statistics.median
    print("rollout T=20 plan call (enqueue)      %7.2f us" % med(enq))
    print("rollout T=20 plan call + sync         %7.2f us" % med(total))
    print("ctypes call of an empty C function    %7.2f us" % med(cc))
    print("torch tiny fill + sync                %7.2f us" % med(tiny))


if __name__ == "__main__":
    main()
