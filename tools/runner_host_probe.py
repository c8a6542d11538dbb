#!/usr/bin/env python3
"""Host-side cost of one batched ParallelRunner step (bench.py --env runner's shape):
the runner loop of mapfx/runners.py restated with perf_counter stamps around each
piece (ring wait, the MAC's select_actions, the action tensor checks, the
mapfx_runner_step foreign call, the ring event record), medians over a few
episodes.  When the sum is above the GPU time per step the loop is host-bound.
usage: python3 tools/runner_host_probe.py [--episodes 4]"""
import argparse
import ctypes
import os
import statistics
import sys
import tempfile
import time
import types

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=4)
    ap.add_argument("--envs", type=int, default=4096)
    args = ap.parse_args()
    import bench
    from mapfx._abi import lib
    from mapfx.episode import DeviceEpisodeBatch, OneHot
    from mapfx.maps import synthetic_instances
    from mapfx.runners import _ADT, _RING, ParallelRunner
    S, N, B = 8, 15, args.envs
    inst = synthetic_instances(B, S, S, N, p_obstacle=0.0, seed=1)
    tmp = tempfile.mkdtemp(prefix="mapfx_probe_")
    mp = os.path.join(tmp, "empty-8-8.map")
    with open(mp, "w") as f:
        f.write("type octile\nheight 8\nwidth 8\nmap\n" + "\n".join(["." * 8] * 8) + "\n")
    ea = dict(bench.PARTIAL_YAML, grid_file_path=mp, agents_path=os.path.join(tmp, "x-"), n_agents=N)
    rargs = types.SimpleNamespace(env="marl_partial", batch_size_run=B, device="cuda:0", env_args=ea,
                                  episode_batch_cls=DeviceEpisodeBatch, test_nepisode=B,
                                  runner_log_interval=1 << 62)
    runner = ParallelRunner(rargs, None, instance_fn=lambda ep: (inst["init_pos"], inst["goals"]))
    info = runner.get_env_info()
    scheme = {"state": {"vshape": info["state_shape"]},
              "obs": {"vshape": info["obs_shape"], "group": "agents"},
              "actions": {"vshape": (1,), "group": "agents", "dtype": torch.long},
              "avail_actions": {"vshape": (info["n_actions"],), "group": "agents", "dtype": torch.int},
              "reward": {"vshape": (1,)}, "terminated": {"vshape": (1,), "dtype": torch.uint8}}
    mac = bench.RandomAvailMAC(seed=0)
    runner.setup(scheme, {"agents": N}, {"actions": ("actions_onehot", [OneHot(out_dim=5)])}, mac)
    runner.run()  # warm
    torch.cuda.synchronize()
    names = ("ring_wait", "mac", "act_checks", "step_call", "ev_record", "loop_total")
    acc = {k: [] for k in names}
    for _ in range(args.episodes):
        runner.reset()
        r, rs, env = runner._erows, ctypes.byref(runner._rs), runner.env
        stream = torch.cuda.current_stream(runner.device)
        sh = stream.cuda_stream
        fixed = (env._h, ctypes.byref(env._state), ctypes.byref(env._out), rs)
        step = lib.mapfx_runner_step
        k = 0
        while k < int(r.max_t):   # (mapfx/runners.py run(): the batch's last row ends it)
            t0 = time.perf_counter()
            if k >= 2:
                ev, hc, _ = runner._ring[(k - 2) % _RING]
                ev.synchronize()
                if int(hc[1]) == 0:
                    break
            t1 = time.perf_counter()
            actions = mac.select_actions(runner.batch, t_ep=k, t_env=runner.t_env, bs=runner._bs)
            t2 = time.perf_counter()
            a = actions.reshape(-1, N)
            if a.device != runner.device:
                a = a.to(runner.device)
            if a.dtype not in _ADT:
                a = a.to(torch.int64)
            a = a.contiguous()
            ev, _, dslot = runner._ring[k % _RING]
            t3 = time.perf_counter()
            rc = step(*fixed, a.data_ptr(), _ADT[a.dtype], a.stride(0), k, dslot, ctypes.byref(r), sh)
            assert rc == 0
            t4 = time.perf_counter()
            ev.record(stream)
            t5 = time.perf_counter()
            if k >= 4:
                for n_, v in zip(names, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t5 - t0)):
                    acc[n_].append(v * 1e6)
            k += 1
        torch.cuda.synchronize()
    for n_ in names:
        print("%-11s median %7.2f us  mean %7.2f us" % (n_, statistics.median(acc[n_]), statistics.mean(acc[n_])))
    # whole run() calls, and the host time of the per-episode pieces around the loop
    spent = {}

    def timed(name, fn):
        def w(*a, **k):
            t0 = time.perf_counter()
            out = fn(*a, **k)
            spent.setdefault(name, []).append((time.perf_counter() - t0) * 1e6)
            return out
        return w
    runner.new_batch = timed("new_batch", runner.new_batch)
    runner._draw = timed("_draw", runner._draw)
    runner._rows = timed("_rows", runner._rows)
    runner.env.reset = timed("env.reset", runner.env.reset)
    runner.reset = timed("reset (all)", runner.reset)
    runner.env.check_err = timed("check_err", runner.env.check_err)
    torch.cuda.synchronize()
    walls, steps = [], []
    for _ in range(args.episodes):
        t0 = time.perf_counter()
        t_env0 = runner.t_env
        runner.run()
        walls.append((time.perf_counter() - t0) * 1e6)
        steps.append(runner.t_env - t_env0)
    torch.cuda.synchronize()
    print("run() wall median %.1f us for %d loop iterations (%.2f us / iteration)"
          % (statistics.median(walls), runner.t, statistics.median(walls) / runner.t))
    for n_, v in spent.items():
        print("per episode %-12s median %8.1f us" % (n_, statistics.median(v)))
    # the MAC stand-in's pieces (host time per call, queued without waiting)
    batch, bs = runner.batch, runner._bs
    gen = torch.Generator(device="cuda")
    avail = batch["avail_actions"][bs, 3]
    noise = torch.rand(avail.shape, generator=gen, device="cuda")
    pieces = {"batch[key]": lambda: batch["avail_actions"],
              "adv_index": lambda: batch["avail_actions"][bs, 3],
              "rand": lambda: torch.rand(avail.shape, generator=gen, device="cuda"),
              "mul": lambda: noise * avail,
              "argmax": lambda: torch.argmax(noise, dim=-1)}
    for n_, fn in pieces.items():
        ts = []
        for _ in range(300):
            t0 = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize()
        print("mac piece %-10s median %7.2f us" % (n_, statistics.median(ts)))


if __name__ == "__main__":
    main()
