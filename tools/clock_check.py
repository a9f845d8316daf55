"""Kernel-timer check: per-launch durations stamped by the kernels (phc_timer_*) beside rocprofv3's for
the same launches.  Run under `rocprofv3 --kernel-trace`, then `clock_check.py compare <trace.csv>
<clock.json>`: every 2nd launch is timed, so the trace also shows whether a timed launch runs longer
than an untimed one.  Cases: the fused env step (4096 envs, eager), a PPO-sized trunk GEMM (eager), the
same GEMM inside a captured graph (replayed).

usage: python tools/clock_check.py run <clock.json>
       python tools/clock_check.py compare <run_kernel_trace.csv> <clock.json>
"""
import csv
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(out):
    import torch

    import phc_amd_path

    phc_amd_path.register()
    import bench
    from puffer_phc_amd import _native as N

    res = {}
    a = types.SimpleNamespace(envs=4096, min_len=60, max_len=300, physics="replay", amp=False)
    env, _, _ = bench.build_env(a, 0)
    act = torch.zeros((4096, 69), device="cuda")
    for _ in range(5):
        env.step(act)
    torch.cuda.synchronize()
    t = N.KernelTimer(capacity=256, period=2)
    env.env.kernel_timer = t
    for _ in range(40):
        env.step(act)
    torch.cuda.synchronize()
    env.env.kernel_timer = None
    res["env"] = t.durations_ms()

    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn((32768, 2048), device="cuda", generator=g).half()
    w = (torch.randn((2, 1536, 2048), device="cuda", generator=g) / 45.0).half()
    z = torch.empty((2, 32768, 1536), device="cuda", dtype=torch.float16)
    for _ in range(3):
        N.twin_gemm(x, w, N.EPI_STORE, z, (2, 1536))
    torch.cuda.synchronize()
    t = N.KernelTimer(capacity=256, period=2)
    N.gemm_set_timer(t)
    for _ in range(20):
        N.twin_gemm(x, w, N.EPI_STORE, z, (2, 1536))
    torch.cuda.synchronize()
    res["gemm"] = t.durations_ms()
    t2 = N.KernelTimer(capacity=256, period=2)
    N.gemm_set_timer(t2)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(graph):
        for _ in range(6):
            N.twin_gemm(x, w, N.EPI_STORE, z, (2, 1536))
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    for _ in range(4):
        graph.replay()
    torch.cuda.synchronize()
    t2.reset()
    graph.replay()
    torch.cuda.synchronize()
    N.gemm_set_timer(None)
    res["gemm_graph_last"] = t2.durations_ms()
    json.dump(res, open(out, "w"))
    print(json.dumps({k: [round(v * 1e3, 1) for v in vs] for k, vs in res.items()}))


def compare(trace, clock):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    res = json.load(open(clock))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
    env = [dur(r) for r in rows if ("k_env_step" in r["Kernel_Name"] or "k_env_replay" in r["Kernel_Name"])][-40:]
    gem = [dur(r) for r in rows if "k_twin_gemm" in r["Kernel_Name"]]
    gemm_eager, gemm_graph = gem[3:23], gem[-6:]
    out = {}
    for name, tr, ck in (("env", env, res["env"]), ("gemm", gemm_eager, res["gemm"]),
                         ("gemm_graph_last", gemm_graph, res["gemm_graph_last"])):
        timed, untimed = tr[0::2], tr[1::2]
        out[name] = {"trace_timed_us": sum(timed) / len(timed), "trace_untimed_us": sum(untimed) / len(untimed),
                     "clock_us": 1e3 * sum(ck) / max(len(ck), 1), "n_clock": len(ck),
                     "trace_timed": [round(v, 1) for v in timed], "clock": [round(v * 1e3, 1) for v in ck]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3])
