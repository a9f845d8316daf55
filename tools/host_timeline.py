"""Host-side timeline of one PPO iteration of `bench.py` (ppo mode): perf_counter stamps around the
calls between the rollout's last device read and the train graph's launch (where rocprofv3 shows the
GPU idle, tools/host_gaps.py), then a cProfile of a few iterations sorted by own time.

usage: python tools/host_timeline.py [bench.py args ...]
"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench

    sys.argv = ["bench.py", "--no-cpu-baseline"] + sys.argv[1:]
    args = bench.parse()
    env, _, env_cfg = bench.build_env(args, 0)
    runner = bench.Runner(args, env, env_cfg)
    from puffer_phc_amd.clean_pufferl import core
    from puffer_phc_amd._native import RowCompactor

    log = []

    def wrap(owner, name, label=None):
        fn = getattr(owner, name)

        def w(*a, **k):
            t0 = time.perf_counter()
            try:
                return fn(*a, **k)
            finally:
                log.append((label or name, t0, time.perf_counter()))

        setattr(owner, name, w)

    for name in ("_evaluate_graph", "_compute_advantages_train", "_train_minibatches_graphed", "_finish_train",
                 "_global_count"):
        wrap(core, name)
    wrap(core.RolloutStep, "run_block")
    wrap(core.RolloutStep, "run")
    wrap(RowCompactor, "state")
    pol = runner.policy.policy
    wrap(pol, "update_obs_rms")
    stats = runner.info.stats
    wrap(stats, "extend", "stats.extend")
    wrap(type(env), "recv", "vecenv.recv")
    for _ in range(4):
        runner.step()
    torch.cuda.synchronize()
    for it in range(3):
        log.clear()
        t0 = time.perf_counter()
        runner.step()
        t1 = time.perf_counter()
        agg = {}
        for name, a, b in log:
            n, s, first = agg.get(name, (0, 0.0, a))
            agg[name] = (n + 1, s + b - a, first)
        print(f"iteration {it}: host {1e3 * (t1 - t0):.2f} ms")
        for name, (n, s, first) in sorted(agg.items(), key=lambda kv: kv[1][2]):
            print(f"  {1e3 * (first - t0):8.3f} ms  {name:28s} x{n:4d}  {1e3 * s:8.3f} ms")
        # the stretch the GPU idles in: last state() read -> the train graph's launch
        ends = [b for name, a, b in log if name == "state"]
        starts = [a for name, a, b in log if name == "_train_minibatches_graphed"]
        if ends and starts:
            print(f"  last state() end -> train graph call: {1e3 * (starts[-1] - ends[-1]):.3f} ms")
    torch.cuda.synchronize()
    prof = cProfile.Profile()
    prof.enable()
    for _ in range(3):
        runner.step()
    torch.cuda.synchronize()
    prof.disable()
    pstats.Stats(prof).sort_stats("tottime").print_stats(40)


if __name__ == "__main__":
    main()
