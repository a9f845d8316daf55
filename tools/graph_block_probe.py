"""Does a hipGraph replay block the host?  Host time of graph.replay() calls with the GPU idle or busy,
for one graph exec replayed back to back and for two execs of the same work alternated (rollout design aid).
usage: python tools/graph_block_probe.py"""
import json
import time

import torch

dev = "cuda:0"
x = torch.randn(1 << 22, device=dev)  # 16 MB: ~10 us elementwise kernels
ys = [torch.empty_like(x) for _ in range(4)]


def body():
    for i in range(12):
        torch.mul(x, 1.0001, out=ys[i % 4])


def cap():
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    return g


ga, gb = cap(), cap()
for _ in range(5):
    ga.replay()
    gb.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
ga.replay()
e1.record()
torch.cuda.synchronize()
gpu_us = e0.elapsed_time(e1) * 1e3
res = {"graph_gpu_us": round(gpu_us, 1)}


def host_us(fn, n=20):
    torch.cuda.synchronize()
    t = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        t.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    return round(sorted(t)[n // 2], 1)


res["replay_same_exec_host_us"] = host_us(lambda: ga.replay())
res["replay_alternating_execs_host_us"] = host_us(lambda: (ga.replay(), gb.replay()))
res["eager_12_kernels_host_us"] = host_us(body)
# wall time of 50 back-to-back replays vs their GPU time
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    ga.replay()
torch.cuda.synchronize()
res["50_replays_wall_us_per"] = round((time.perf_counter() - t0) * 1e6 / 50, 1)
print(json.dumps(res))
