"""Probe: can kernels inside a captured hipGraph be timed by HIP events recorded during the capture?

(1) torch.cuda.Event(enable_timing=True).record() inside torch.cuda.graph capture, (2) hipEventRecord
through ctypes on the capturing stream (what libphc_hip would do), each around a known matmul; the
graph is replayed and the elapsed times compared with an eager event pair around the same matmul.
"""
import ctypes
import sys

import torch


def main():
    dev = "cuda"
    a = torch.randn(4096, 4096, device=dev, dtype=torch.float16)
    b = torch.randn(4096, 4096, device=dev, dtype=torch.float16)
    c = torch.empty(4096, 4096, device=dev, dtype=torch.float16)
    for _ in range(3):
        torch.mm(a, b, out=c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.mm(a, b, out=c)
    e1.record()
    torch.cuda.synchronize()
    print("eager mm ms", e0.elapsed_time(e1), flush=True)

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
    hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
    h0, h1 = ctypes.c_void_p(), ctypes.c_void_p()
    print("create", hip.hipEventCreate(ctypes.byref(h0)), hip.hipEventCreate(ctypes.byref(h1)), flush=True)

    g = torch.cuda.CUDAGraph()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            torch.mm(a, b, out=c)
            t0.record()
            torch.mm(a, b, out=c)
            t1.record()
            st = torch.cuda.current_stream().cuda_stream
            rc0 = hip.hipEventRecord(h0, ctypes.c_void_p(st))
            torch.mm(a, b, out=c)
            torch.mm(a, b, out=c)
            rc1 = hip.hipEventRecord(h1, ctypes.c_void_p(st))
    print("capture hipEventRecord rc", rc0, rc1, flush=True)
    for i in range(3):
        g.replay()
        torch.cuda.synchronize()
        try:
            print("replay", i, "torch event ms (1 mm)", t0.elapsed_time(t1), flush=True)
        except Exception as ex:  # noqa: BLE001
            print("torch event elapsed failed:", ex, flush=True)
        ms = ctypes.c_float()
        rc = hip.hipEventElapsedTime(ctypes.byref(ms), h0, h1)
        print("replay", i, "ctypes hip event rc", rc, "ms (2 mm)", ms.value, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
