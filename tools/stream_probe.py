"""Does running the actor and critic trunks as two persistent half-GPU launch chains on two
streams, phase-shifted, hide the GEMM epilogue's store burst?  Times the forward chain L2..L5
(32768 rows, bias + SiLU epilogue) as (a) one batched launch per layer, (b) per-trunk launches on
two streams with max_workgroups = CUs / 2 and an initial offset on the second stream.

usage: python tools/stream_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, ".")
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd import _native as N  # noqa: E402

dev = "cuda:0"
dt = torch.float16
M = 32768
DIMS = [2048, 1536, 1024, 1024, 512]
REPS = int(os.environ.get("REPS", "20"))
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*shape, scale=1.0):
    return (torch.rand(shape, device=dev, generator=g) * 2 - 1).mul_(scale).to(dt)


x = rnd(2, M, DIMS[0])
W = [rnd(2, DIMS[l + 1], DIMS[l], scale=DIMS[l] ** -0.5) for l in range(len(DIMS) - 1)]
B = [torch.randn(2 * DIMS[l + 1], device=dev, generator=g) * 0.1 for l in range(len(DIMS) - 1)]
Z = [torch.empty((2, M, DIMS[l + 1]), dtype=dt, device=dev) for l in range(len(DIMS) - 1)]
P = [torch.empty((2, M, DIMS[l + 1]), dtype=dt, device=dev) for l in range(len(DIMS) - 1)]
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
cus = torch.cuda.get_device_properties(dev).multi_processor_count


def batched():
    a = x
    for l in range(len(W)):
        N.twin_gemm(a, W[l], N.EPI_BIAS_SILU, Z[l], (2, DIMS[l + 1]), bias=B[l], aux=P[l])
        a = Z[l]


def trunk(t, mwg):
    a = x[t]
    for l in range(len(W)):
        n = DIMS[l + 1]
        N.twin_gemm(a, W[l][t], N.EPI_BIAS_SILU, Z[l][t], (1, n), bias=B[l][t * n:(t + 1) * n], aux=P[l][t],
                    max_workgroups=mwg)
        a = Z[l][t]


def two_streams(mwg, offset):
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        trunk(0, mwg)
    with torch.cuda.stream(s2):
        if offset:
            torch.cuda._sleep(offset)
        trunk(1, mwg)
    cur.wait_stream(s1)
    cur.wait_stream(s2)


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / REPS * 1e3


def check():
    batched()
    ref = [z.clone() for z in Z] + [p.clone() for p in P]
    bad = False
    for name, fn in (("per trunk", lambda: (trunk(0, 0), trunk(1, 0))), ("persistent", lambda: (trunk(0, cus // 2), trunk(1, cus // 2))),
                     ("two streams", lambda: two_streams(cus // 2, 20000))):
        for z in Z + P:
            z.zero_()
        fn()
        torch.cuda.synchronize()
        for i, (r, z) in enumerate(zip(ref, Z + P)):
            if not torch.equal(r, z):
                d = (r.float() - z.float()).abs()
                print(f"{name}: tensor {i} differs: max {d.max().item():.3g} at {d.flatten().argmax().item()}, "
                      f"{(d > 0).sum().item()} elements; trunk0 {(d[0] > 0).sum().item()} trunk1 {(d[1] > 0).sum().item()}")
                bad = True
    assert not bad


if os.environ.get("CHECK_ONLY"):
    try:
        check()
        print("check ok", os.environ.get("PHC_HIP_LIB"))
    except AssertionError:
        print("check FAILED", os.environ.get("PHC_HIP_LIB"))
    sys.exit(0)
check()
fl = sum(2.0 * M * 2 * DIMS[l] * DIMS[l + 1] for l in range(len(W)))
rows = [("batched, one launch per layer", batched),
        ("per trunk, one stream", lambda: (trunk(0, 0), trunk(1, 0))),
        ("two streams, full grids", lambda: two_streams(0, 0)),
        ("two streams, persistent CUs/2, no offset", lambda: two_streams(cus // 2, 0))]
for off in (5000, 20000, 50000, 100000):
    rows.append((f"two streams, persistent CUs/2, offset {off}", lambda off=off: two_streams(cus // 2, off)))
for name, fn in rows:
    us = timeit(fn)
    print(f"{name:48s} {us:8.1f} us  {fl / us / 1e6:6.0f} TF/s", flush=True)
