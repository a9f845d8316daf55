"""Does running the input-gradient GEMMs and the weight-gradient GEMMs of one PPO minibatch on two
streams at once beat running them one after the other?  (32768 rows, the trunk shapes; HIP events.)

serial : dgrad L6..L2 (SiLU-grad epilogues) then the grouped weight gradient of layers 5..1
overlap: the grouped weight gradient of layers 5..2 on a side stream as soon as the main stream's
         dgrad L3 is done (its inputs exist then), dgrad L2 on the main stream meanwhile, then
         layer 1's weight gradient
usage: python tools/overlap_probe.py
"""
import sys

import torch

sys.path.insert(0, ".")
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd import _native as N  # noqa: E402

dev = "cuda:0"
dt = torch.float16
M = 32768
DIMS = [960, 2048, 1536, 1024, 1024, 512, 512]
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*shape, scale=1.0):
    return (torch.rand(shape, device=dev, generator=g) * 2 - 1).mul_(scale).to(dt)


# dgrad inputs: gs[l] = d loss / d out of layer l (l = 1..6, 1-based), pres = pre-activations
gs = {l: rnd(2, M, DIMS[l], scale=0.1) for l in range(2, 7)}
wts = {l: rnd(2, DIMS[l - 1], DIMS[l], scale=DIMS[l] ** -0.5) for l in range(2, 7)}
pres = {l: rnd(2, M, DIMS[l - 1]) for l in range(2, 7)}
outs = {l: torch.empty((2, M, DIMS[l - 1]), dtype=dt, device=dev) for l in range(2, 7)}
dbs = {l: torch.empty(2 * DIMS[l - 1], device=dev) for l in range(2, 7)}
zs = {l: rnd(2, M, DIMS[l - 1]) for l in range(2, 6)}  # layer inputs y_{l-1}
x0 = rnd(M, DIMS[0])
g1 = rnd(M, 2 * DIMS[1], scale=0.1)


def problem(l):
    nout, nin = DIMS[l], DIMS[l - 1]
    if l == 1:
        return (g1, x0, [torch.zeros((nout, 934), device=dev) for _ in range(2)], nout, 934)
    return (gs[l], zs[l], [torch.zeros((nout, nin), device=dev) for _ in range(2)], nout, nin)


probs = {l: problem(l) for l in range(1, 6)}


def dgrad(l):
    N.twin_gemm(gs[l], wts[l], N.EPI_SILU_GRAD, outs[l], (2, DIMS[l - 1]), aux=pres[l], bias_grad=dbs[l])


side = torch.cuda.Stream()


def serial():
    for l in range(6, 1, -1):
        dgrad(l)
    N.weight_grad_group([probs[l] for l in range(5, 0, -1)], accumulate=False)


def overlap():
    main = torch.cuda.current_stream()
    for l in range(6, 2, -1):
        dgrad(l)
    ev = torch.cuda.Event()
    ev.record(main)
    side.wait_event(ev)
    with torch.cuda.stream(side):
        N.weight_grad_group([probs[l] for l in range(5, 1, -1)], accumulate=False)
    dgrad(2)
    N.weight_grad_group([probs[1]], accumulate=False)
    main.wait_stream(side)


def overlap_split():
    """every layer's weight gradient on the side stream right after its input gradient exists,
    in two launches: layers 5..3 after dgrad L4, layer 2 + 1 after the last dgrad"""
    main = torch.cuda.current_stream()
    for l in range(6, 3, -1):
        dgrad(l)
    ev = torch.cuda.Event()
    ev.record(main)
    side.wait_event(ev)
    with torch.cuda.stream(side):
        N.weight_grad_group([probs[l] for l in range(5, 2, -1)], accumulate=False)
    dgrad(3)
    dgrad(2)
    N.weight_grad_group([probs[l] for l in (2, 1)], accumulate=False)
    main.wait_stream(side)


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for r in range(2):
    print(f"round {r}: serial {timeit(serial):8.1f} us   overlap {timeit(overlap):8.1f} us   "
          f"overlap_split {timeit(overlap_split):8.1f} us", flush=True)
