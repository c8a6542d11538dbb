#!/usr/bin/env python3
"""Per-wave shader cycles and effective clock of the fused rollout loop
(diagnostic build libmapfx_clocks.so, -DMAPFX_CLOCKS):

  python tools/clocks.py [--envs 1024,4096,8192]
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MAPFX_LIB"] = os.path.join(REPO, "mapf-marl_amd", "mapfx", "libmapfx_clocks.so")
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", default="1024,4096,8192")
    ap.add_argument("--T", type=int, default=64)
    a = ap.parse_args()
    import mapfx
    from mapfx._abi import lib
    from mapfx.maps import synthetic_instances
    fn = lib.mapfx_debug_clocks
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p]
    S, N, T = 32, 16, a.T
    outs = ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos", "traj_done",
            "traj_t")
    for E in [int(x) for x in a.envs.split(",")]:
        inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=1)
        b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                                episode_limit=2 ** 31 - 1, obs=("window",), window=5,
                                track_steps=False)
        b.reset()
        acts = b.gen_actions(T * 3, seed=2)
        traj = b._alloc_out(T)
        for i in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            b.rollout(T, actions=acts[i * T:(i + 1) * T], traj=traj, outputs=outs)
            e1.record()
            torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        buf = (ctypes.c_ulonglong * (8 * 32768))()
        assert fn(ctypes.addressof(buf)) == 0
        c = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)[:E * N // 64].astype(np.float64)
        cyc = c[:, 1] - c[:, 0]
        rt = (c[:, 3] - c[:, 2]) / 100e6  # s_memrealtime: 100 MHz
        clk = cyc / rt / 1e9
        start = (c[:, 2] - c[:, 2].min()) / 100e6 * 1e6
        end = (c[:, 3] - c[:, 2].min()) / 100e6 * 1e6
        t0 = c[:, 4].min()
        pro = (c[:, 2] - c[:, 4]) / 100e6 * 1e6
        epi = (c[:, 5] - c[:, 3]) / 100e6 * 1e6
        print("E=%5d waves=%5d kernel %.1f us | loop cycles/step med %.0f min %.0f max %.0f | "
              "clock GHz med %.2f | loop us med %.1f | prologue us med %.1f max %.1f | "
              "epilogue us med %.1f max %.1f | first entry->last exit %.1f us | entry skew %.1f us"
              % (E, len(c), ms * 1e3, np.median(cyc) / T, cyc.min() / T, cyc.max() / T,
                 np.median(clk), np.median(rt) * 1e6, np.median(pro), pro.max(), np.median(epi),
                 epi.max(), (c[:, 5].max() - t0) / 100e6 * 1e6, (c[:, 4].max() - t0) / 100e6 * 1e6))
        del b, traj, acts


if __name__ == "__main__":
    main()
