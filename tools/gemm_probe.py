"""Probe policy-GEMM throughput/precision options on the box (fp32, tf32 flag, bf16)."""
import time, torch
torch.manual_seed(0)
dev = "cuda:0"
M, K, N = 32768, 2048, 1536
a = torch.randn(M, K, device=dev); b = torch.randn(K, N, device=dev) / K ** 0.5
ref = (a.double() @ b.double())
def bench(fn, n=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / n
for name, setup, fn in [
    ("fp32", lambda: setattr(torch.backends.cuda.matmul, "allow_tf32", False), lambda: a @ b),
    ("fp32 allow_tf32", lambda: setattr(torch.backends.cuda.matmul, "allow_tf32", True), lambda: a @ b),
    ("bf16", lambda: None, lambda: (a.bfloat16() @ b.bfloat16())),
]:
    setup()
    dt = bench(fn)
    out = fn().double()
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    print(f"{name:18s} {dt*1e3:7.3f} ms  {2*M*K*N/dt/1e12:7.1f} TFLOP/s  max rel err {err:.2e}")
ab, bb = a.bfloat16(), b.bfloat16()
dt = bench(lambda: ab @ bb)
print(f"bf16 (pre-cast)    {dt*1e3:7.3f} ms  {2*M*K*N/dt/1e12:7.1f} TFLOP/s")
