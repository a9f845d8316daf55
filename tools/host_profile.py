"""Host-side profile of the PPO iteration (bench.py's Runner): cProfile over N iterations after a
warmup, to find the Python work that leaves the GPU idle (the train-phase gaps of the kernel trace).

usage: python tools/host_profile.py [iterations]
"""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
sys.argv = ["bench.py", "--no-cpu-baseline"]
import bench  # noqa: E402

args = bench.parse()
world, rank = bench.setup_dist()
torch.manual_seed(1234)
env, packed, env_cfg = bench.build_env(args, rank)
runner = bench.Runner(args, env, env_cfg)
for _ in range(3):
    runner.step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(n):
    runner.step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
st.sort_stats("cumulative").print_stats(45)
