#!/usr/bin/env python3
"""C5 generic rollout (bench.py --config c5 shape, runner output set, T = 64): kernel time
with int8 actions read from HBM (one step ahead) against the same launch with actions
from the device generator (no action loads), event-timed, medians of 5.  A gap between
the two is the price of waiting on the action load -- which, with vmcnt counting loads
and stores in order, waits for every store issued after it."""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]
import torch  # noqa: E402


def main():
    import bench
    from mapfx import _abi
    wl = bench.mapf_workload(os.environ.get("PROBE_CONFIG", "c5"), 5, "cuda:0")
    b = wl["batch"]
    T = int(os.environ.get("PROBE_T", 64))
    b.reset()
    acts = b.gen_actions(T, seed=bench.ACT_SEED)
    traj = bench.bench_traj(b, T)
    state0 = [x.clone() for x in (b.pos, b.done, b.t)]
    res = {}
    for mode in ("hbm", "rng", "hbm", "rng"):
        ts = []
        for _ in range(5):
            for x, x0 in zip((b.pos, b.done, b.t), state0):
                x.copy_(x0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if mode == "hbm":
                b.rollout(T, actions=acts, traj=traj, outputs=wl["outs"])
            else:
                b.rollout(T, seed=bench.ACT_SEED, traj=traj, outputs=wl["outs"])
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        res.setdefault(mode, []).append(statistics.median(ts))
        print(mode, "%.4f ms" % statistics.median(ts), _abi.last_kernel()[28:90], flush=True)


if __name__ == "__main__":
    main()
