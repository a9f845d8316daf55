"""Time every twin-trunk GEMM of one PPO minibatch (32768 rows) with its real epilogue on
phc_twin_gemm, plus the hipBLASLt weight-gradient GEMMs, and print TF/s per GEMM.

usage: [PHC_HIP_LIB=...] python tools/gemm_mb_probe.py [rows]
Several library builds are compared by running this once per PHC_HIP_LIB (tools/gemm_ab.sh).
"""
import os
import sys

import torch

sys.path.insert(0, ".")
import phc_amd_path  # noqa: E402

phc_amd_path.register()
from puffer_phc_amd import _native as N  # noqa: E402

dev = "cuda:0"
if os.environ.get("MAXWG"):  # persistent tile loop over this many workgroups
    import functools

    N.twin_gemm = functools.partial(N.twin_gemm, max_workgroups=int(os.environ["MAXWG"]))
dt = torch.float16
M = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
DIMS = [960, 2048, 1536, 1024, 1024, 512, 512]  # padded input width, then the six layer widths
REPS = int(os.environ.get("REPS", "20"))
PER_TRUNK = os.environ.get("PER_TRUNK", "0") == "1"  # one launch per trunk (batch 1) instead of batched twins
# YONLY=1: the forward GEMMs store the activation only, not the pre-activation (the upper bound of a
# y-only forward store whose consumers would recompute what they need)
AUX = os.environ.get("YONLY", "0") != "1"
# DERIV=1: the silu'-aux pair (forward PHC_EPI_BIAS_SILU_D, input gradients PHC_EPI_DSILU_GRAD), as the trunk runs it
DERIV = os.environ.get("DERIV", "0") == "1"


SUMS = []


def timeit(fn, out=None):
    for _ in range(3):
        fn()
    if out is not None:  # checksum of one output, to compare library builds / tile configurations
        torch.cuda.synchronize()
        SUMS.append(float(out.double().sum()))
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(REPS):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / REPS * 1e3  # us


def main():
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*shape, scale=1.0):
        return (torch.rand(shape, device=dev, generator=g) * 2 - 1).mul_(scale).to(dt)

    rows = []
    total_us, total_fl = 0.0, 0.0
    # forward: L1 from the [M, 960] input, SPLIT pre-activation, GROUPED output
    x = rnd(M, DIMS[0])
    w0 = rnd(2 * DIMS[1], DIMS[0], scale=DIMS[0] ** -0.5)
    b0 = torch.randn(2 * DIMS[1], device=dev, generator=g)
    z = torch.empty((2, M, DIMS[1]), dtype=dt, device=dev)
    pre = torch.empty((M, 2 * DIMS[1]), dtype=dt, device=dev)
    us = timeit(lambda: N.twin_gemm(x, w0, N.EPI_BIAS_SILU_D if DERIV else N.EPI_BIAS_SILU, z, (2, DIMS[1]), bias=b0, aux=pre if AUX else None,
                                    aux_layout=N.SPLIT, out_layout=N.GROUPED), z)
    rows.append(("fwd L1", M, 2 * DIMS[1], DIMS[0], 1, us))
    for l in range(2, 7):
        k, n = DIMS[l - 1], DIMS[l]
        a = rnd(2, M, k)
        w = rnd(2, n, k, scale=k ** -0.5)
        b = torch.randn(2 * n, device=dev, generator=g)
        if l < 6 and PER_TRUNK:
            o = torch.empty((2, M, n), dtype=dt, device=dev)
            p = torch.empty((2, M, n), dtype=dt, device=dev)
            us = timeit(lambda: [N.twin_gemm(a[t], w[t], N.EPI_BIAS_SILU, o[t], (1, n), bias=b[t * n:(t + 1) * n],
                                             aux=p[t] if AUX else None) for t in range(2)], o)
        elif l < 6:
            o = torch.empty((2, M, n), dtype=dt, device=dev)
            p = torch.empty((2, M, n), dtype=dt, device=dev)
            us = timeit(lambda: N.twin_gemm(a, w, N.EPI_BIAS_SILU_D if DERIV else N.EPI_BIAS_SILU, o, (2, n), bias=b, aux=p if AUX else None), o)
        else:
            o = torch.empty((2, M, n), dtype=torch.float32, device=dev)
            us = timeit(lambda: N.twin_gemm(a, w, N.EPI_BIAS, o, (2, n), bias=b), o)
        rows.append((f"fwd L{l}", M, n, k, 2, us))
    # backward input gradients L6..L2: g [2, M, n_out] x W^T -> [2, M, n_in], SiLU' epilogue
    for l in range(6, 1, -1):
        nout, nin = DIMS[l], DIMS[l - 1]
        gg = rnd(2, M, nout)
        wt = rnd(2, nin, nout, scale=nout ** -0.5)
        p = rnd(2, M, nin)
        db = torch.empty(2 * nin, device=dev)
        if l > 2 and PER_TRUNK:
            o = torch.empty((2, M, nin), dtype=dt, device=dev)
            us = timeit(lambda: [N.twin_gemm(gg[t], wt[t], N.EPI_SILU_GRAD, o[t], (1, nin), aux=p[t],
                                             bias_grad=db[t * nin:(t + 1) * nin]) for t in range(2)], o)
        elif l > 2:
            o = torch.empty((2, M, nin), dtype=dt, device=dev)
            us = timeit(lambda: N.twin_gemm(gg, wt, N.EPI_DSILU_GRAD if DERIV else N.EPI_SILU_GRAD, o, (2, nin), aux=p, bias_grad=db), o)
        else:
            o = torch.empty((M, 2 * nin), dtype=dt, device=dev)
            p = rnd(M, 2 * nin)
            us = timeit(lambda: N.twin_gemm(gg, wt, N.EPI_DSILU_GRAD if DERIV else N.EPI_SILU_GRAD, o, (2, nin), aux=p, aux_layout=N.SPLIT,
                                            out_layout=N.SPLIT, bias_grad=db), o)
        rows.append((f"dgrad L{l}", M, nin, nout, 2, us))
    # weight gradients (hipBLASLt, fp32 out): dW[b] = g[b]^T z[b]
    for l in (range(6, 0, -1) if os.environ.get("WGRAD", "0") == "1" else []):
        nout, nin = DIMS[l], DIMS[l - 1]
        bt = 1 if l == 1 else 2
        gg = rnd(bt, M, nout * (2 if l == 1 else 1))
        zz = rnd(bt, M, nin)
        us = timeit(lambda: torch.bmm(gg.transpose(1, 2), zz, out_dtype=torch.float32))
        rows.append((f"wgrad L{l}", nout * (2 if l == 1 else 1), nin, M, bt, us))
    if os.environ.get("WGRAD", "2") == "2":  # the grouped weight-gradient launch of layers 5..1
        probs = []
        for l in range(5, 0, -1):
            nout, nin = DIMS[l], DIMS[l - 1]
            if l == 1:
                gg = rnd(M, 2 * nout, scale=0.1)
                zz = rnd(M, nin)
                d = [torch.zeros((nout, 934), device=dev) for _ in range(2)]
                probs.append((gg, zz, d, nout, 934))
            else:
                gg = rnd(2, M, nout, scale=0.1)
                zz = rnd(2, M, nin)
                d = [torch.zeros((nout, nin), device=dev) for _ in range(2)]
                probs.append((gg, zz, d, nout, nin))
        us = timeit(lambda: N.weight_grad_group(probs, accumulate=False), probs[0][2][0])
        fl = sum(2.0 * M * p_[0].shape[-1] * p_[1].shape[-1] * (2 if p_[0].dim() == 3 else 1) for p_ in probs)
        rows.append(("wgrad grp", 1, 1, 1, 1, us))
        total_fl += fl - 2.0
    for name, m, n, k, b, us in rows:
        fl = 2.0 * m * n * k * b
        total_us += us
        total_fl += fl
        print(f"{name:10s} m={m:6d} n={n:5d} k={k:5d} b={b} {us:8.1f} us {fl / us / 1e6:7.0f} TF/s", flush=True)
    print("checksums", " ".join(f"{v:.6e}" for v in SUMS))
    print(f"TOTAL {total_us:.1f} us {total_fl / total_us / 1e6:.0f} TF/s  lib={os.environ.get('PHC_HIP_LIB', 'default')}")


if __name__ == "__main__":
    main()
