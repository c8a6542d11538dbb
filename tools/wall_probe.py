"""Where the host-side time of bench.py's timed region goes (C2, T=20 rollout).
Each variant is repeated; median microseconds printed as JSON."""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mapf-marl_amd")]
import torch  # noqa: E402

import mapfx  # noqa: E402
from mapfx.maps import synthetic_instances  # noqa: E402

S, N, E, T, W = 32, 16, 4096, 20, 5
inst = synthetic_instances(E, S, S, N, p_obstacle=0.1, seed=1)
b = mapfx.MapfGridBatch(inst["init_pos"], inst["goals"], bits=inst["bits"], hw=(S, S),
                        episode_limit=2 ** 31 - 1, obs=("window",), window=W, device="cuda:0",
                        track_steps=False)
b.reset()
acts = b.gen_actions(T, seed=2)
traj = b._alloc_out(T)
traj.pop("reward_f32")
outs = ("reward", "term", "node", "edge", "avail", "obs_window", "traj_pos", "traj_done", "traj_t")
st = torch.cuda.current_stream()
plan = b.rollout_plan(T, actions=acts, traj=traj, outputs=outs, stream=st)
xev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
xev[0].record(st)
xev[1].record(st)
xplan = b.rollout_plan(T, actions=acts, traj=traj, outputs=outs, stream=st, events=xev)
tiny = torch.zeros(1, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(5):
    plan()
torch.cuda.synchronize()


def run(name, body, idle_s=0.0, reps=40):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        if idle_s:
            time.sleep(idle_s)
        t0 = time.perf_counter()
        body()
        ts.append((time.perf_counter() - t0) * 1e6)
    return name, round(statistics.median(ts), 2), round(min(ts), 2)


def ev_plan():
    e0.record(st)
    plan()
    e1.record(st)
    torch.cuda.synchronize()


def spin():
    e1.record(st)
    while not e1.query():
        pass
    torch.cuda.synchronize()


def ev_plan_spin():
    e0.record(st)
    plan()
    spin()


res = []
for idle in (0.0, 0.002):
    sfx = "" if not idle else "+idle2ms"
    res += [
        run("sync_only" + sfx, lambda: torch.cuda.synchronize(), idle),
        run("events_sync" + sfx, lambda: (e0.record(st), e1.record(st), torch.cuda.synchronize()), idle),
        run("tiny_fill_sync" + sfx, lambda: (tiny.fill_(1.0), torch.cuda.synchronize()), idle),
        run("plan_sync" + sfx, lambda: (plan(), torch.cuda.synchronize()), idle),
        run("plan_streamsync" + sfx, lambda: (plan(), st.synchronize()), idle),
        run("ev_plan_sync" + sfx, ev_plan, idle),
        run("plan_x2_sync" + sfx, lambda: (plan(), plan(), torch.cuda.synchronize()), idle),
        run("extplan_sync" + sfx, lambda: (xplan(), torch.cuda.synchronize()), idle),
        run("plan_spin" + sfx, lambda: (plan(), spin()), idle),
        run("ev_plan_spin" + sfx, ev_plan_spin, idle),
        run("tiny_spin" + sfx, lambda: (tiny.fill_(1.0), spin()), idle),
        run("spin_only" + sfx, spin, idle),
    ]
    e0.record(st); plan(); e1.record(st); torch.cuda.synchronize()
    res.append(("kernel_events" + sfx, round(e0.elapsed_time(e1) * 1e3, 2), None))
def hot_then(body, n_hot):
    def f():
        for _ in range(n_hot):
            plan()
        torch.cuda.synchronize()
        body()
    return f


def timed_after(prep, body, reps=20):
    ts = []
    for _ in range(reps):
        prep()
        t0 = time.perf_counter()
        body()
        ts.append((time.perf_counter() - t0) * 1e6)
    return round(statistics.median(ts), 2), round(min(ts), 2)


def busy(n):
    def f():
        for _ in range(n):
            plan()
        torch.cuda.synchronize()
    return f


for n in (0, 10):
    res.append(("ev_plan_sync_after_%d_launches" % n, *timed_after(busy(n), ev_plan)))
    res.append(("extplan_sync_after_%d_launches" % n, *timed_after(busy(n), lambda: (xplan(), torch.cuda.synchronize()))))
    res.append(("plan_sync_after_%d_launches" % n, *timed_after(busy(n), lambda: (plan(), torch.cuda.synchronize()))))
xplan()
torch.cuda.synchronize()
res.append(("extplan_kernel_us", round(xev[0].elapsed_time(xev[1]) * 1e3, 2), None))
print(json.dumps({k: [m, mn] for k, m, mn in res}, indent=0))
