#!/usr/bin/env python3
"""Back-to-back launch cost of a HIP graph on this box: 100 tiny kernels
(an in-place add on 64 floats) captured and replayed -- the floor under any
one-launch-per-step path."""
import torch

x = torch.zeros(64, device="cuda")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(100):
        x.add_(1.0)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(100):
        x.add_(1.0)
g.replay()
torch.cuda.synchronize()
best = 1e9
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1) * 10.0)
print("graph replay: %.2f us per tiny kernel" % best)
