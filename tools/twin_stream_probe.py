"""The rollout's policy trunks at 4096 rows (PHCPolicy widths, f16 operands, bias + SiLU epilogues): the batched
twin chain (actor and critic as batch 2 of one launch per layer, as the rollout runs them) against the two trunks
as separate batch-1 chains, one after the other and on two streams at once (actor on the current stream, critic on
a side stream: the layout that would let the critic overlap the actor's tail and the env step).  HIP events over
REPS chains, replayed from captured graphs like the rollout.

usage: python tools/twin_stream_probe.py [rows]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd import _native as N  # noqa: E402

DIMS = [960, 2048, 1536, 1024, 1024, 512, 512]
REPS = 50


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    dev, dt = "cuda", torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s, sc=1.0: ((torch.rand(s, device=dev, generator=g) * 2 - 1) * sc).to(dt)  # noqa: E731
    x = rnd(M, DIMS[0])
    w = [rnd(2 * DIMS[1], DIMS[0], sc=DIMS[0] ** -0.5)] + [rnd(2, DIMS[l], DIMS[l - 1], sc=DIMS[l - 1] ** -0.5)
                                                          for l in range(2, 7)]
    b = [torch.randn(2 * DIMS[l], device=dev, generator=g) for l in range(1, 7)]
    # batched twins: L1 one [M, 4096] launch, then batch-2 launches
    zb = [torch.empty((2, M, DIMS[l]), dtype=dt if l < 6 else torch.float32, device=dev) for l in range(1, 7)]

    def batched():
        N.twin_gemm(x, w[0], N.EPI_BIAS_SILU, zb[0], (2, DIMS[1]), bias=b[0])
        for l in range(2, 7):
            epi = N.EPI_BIAS_SILU if l < 6 else N.EPI_BIAS
            N.twin_gemm(zb[l - 2], w[l - 1], epi, zb[l - 1], (2, DIMS[l]), bias=b[l - 1])

    # one trunk t as its own batch-1 chain
    zt = [[torch.empty((M, DIMS[l]), dtype=dt if l < 6 else torch.float32, device=dev) for l in range(1, 7)]
          for _ in range(2)]

    def trunk(t):
        n1 = DIMS[1]
        N.twin_gemm(x, w[0][t * n1:(t + 1) * n1], N.EPI_BIAS_SILU, zt[t][0], (1, n1), bias=b[0][t * n1:(t + 1) * n1])
        for l in range(2, 7):
            epi = N.EPI_BIAS_SILU if l < 6 else N.EPI_BIAS
            n = DIMS[l]
            N.twin_gemm(zt[t][l - 2], w[l - 1][t], epi, zt[t][l - 1], (1, n), bias=b[l - 1][t * n:(t + 1) * n])

    side = torch.cuda.Stream()

    def two_streams():
        side.wait_stream(torch.cuda.current_stream())
        trunk(0)
        with torch.cuda.stream(side):
            trunk(1)
        torch.cuda.current_stream().wait_stream(side)

    def sequential():
        trunk(0)
        trunk(1)

    res = {}
    for name, fn in (("batched twins", batched), ("two chains, one stream", sequential),
                     ("two chains, two streams", two_streams)):
        fn()
        torch.cuda.synchronize()
        s0 = torch.cuda.Stream()
        s0.wait_stream(torch.cuda.current_stream())
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s0), torch.cuda.graph(gr):
            for _ in range(REPS):
                fn()
        torch.cuda.current_stream().wait_stream(s0)
        torch.cuda.synchronize()
        for _ in range(2):
            gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / REPS * 1e3
    # the two layouts compute the same trunks: compare the critic's last layer
    batched()
    sequential()
    torch.cuda.synchronize()
    same = torch.equal(zb[5][1], zt[1][5]) and torch.equal(zb[5][0], zt[0][5])
    for k, v in res.items():
        print(f"{k:26s} {v:8.1f} us per forward ({M} rows)")
    print("batched == per-trunk outputs bit for bit:", same)


if __name__ == "__main__":
    main()
