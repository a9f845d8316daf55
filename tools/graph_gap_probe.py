"""GPU-timeline cost of mixing eager launches with hipGraph replays (rollout design aid).

Each pattern runs N iterations queued back to back (one sync at the end) and reports the GPU time
per iteration from events around the loop:
  eager6        6 small eager kernels
  graph6        one replay of a graph holding the same 6 kernels
  e1+g5         1 eager kernel, then a 5-kernel graph     (the rollout today: noise eager, policy graph)
  e1+g5+e1      eager, graph, eager                         (+ the env step eager)
  g7            one 7-kernel graph (everything captured)
  g5+g2         two graphs back to back
"""
import json
import sys

import torch

dev = "cuda:0"
N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
x = torch.randn(1 << 20, device=dev)  # 4 MB: a few-us elementwise kernel
ys = [torch.empty_like(x) for _ in range(8)]


def k(i):
    torch.mul(x, 1.0001, out=ys[i % 8])


def capture(n):
    for i in range(n):
        k(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n):
            k(i)
    return g


g6, g5, g7, g2 = capture(6), capture(5), capture(7), capture(2)
pats = {
    "eager6": lambda: [k(i) for i in range(6)],
    "graph6": lambda: g6.replay(),
    "e1+g5": lambda: (k(0), g5.replay()),
    "e1+g5+e1": lambda: (k(0), g5.replay(), k(1)),
    "g7": lambda: g7.replay(),
    "g5+g2": lambda: (g5.replay(), g2.replay()),
}
res = {}
for name, fn in pats.items():
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(N):
        fn()
    b.record()
    torch.cuda.synchronize()
    res[name] = round(a.elapsed_time(b) * 1e3 / N, 2)
    print(f"{name:10s} {res[name]:8.2f} us per iteration", flush=True)
print(json.dumps(res))
