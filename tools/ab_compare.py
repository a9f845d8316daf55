"""Bit-level A/B of two builds of libphc_hip.so on the same env trajectory.

    python tools/ab_compare.py --lib A.so --out a.npz      # one process per library
    python tools/ab_compare.py --compare a.npz b.npz

Runs PHCPufferEnv.step (actions->PD, replay physics, fused obs/reward/reset with auto reset)
for --steps steps on synthetic clips and records obs / rewards / dones of every step, so a
kernel rewrite that claims identical float32 results can be checked bit for bit.
"""

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(lib, out, envs, steps):
    os.environ["PHC_HIP_LIB"] = os.path.abspath(lib)
    import torch

    import phc_amd_path

    phc_amd_path.register()
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    torch.cuda.set_device(0)
    q, t, counts, fps = synthetic_clips(envs, 20, 120, seed=7, device="cuda:0")
    packed = PackedMotions.from_global_rotations(q, t, counts, fps)
    env = PHCPufferEnv(EnvConfig(num_envs=envs, device_id=0, seed=3), motion_data=packed)
    env.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(11)
    obs, rew, done = [], [], []
    for _ in range(steps):
        a = torch.rand((envs, 69), device="cuda:0", generator=g) * 2 - 1
        o, r, d, *_ = env.step(a)
        obs.append(o.cpu().numpy().copy())
        rew.append(r.cpu().numpy().copy())
        done.append(d.cpu().numpy().copy())
    np.savez(out, obs=np.stack(obs), rew=np.stack(rew), done=np.stack(done),
             frames=packed.frames.cpu().numpy())


def compare(a, b):
    A, B = np.load(a), np.load(b)
    ok = True
    for k in A.files:
        x, y = A[k], B[k]
        same = np.array_equal(x.view(np.uint8), y.view(np.uint8))
        msg = "bit-identical" if same else "DIFFERS"
        if not same and x.dtype.kind == "f":
            d = np.abs(x.astype(np.float64) - y.astype(np.float64))
            msg += f" (max abs {d.max():.3e}, {np.count_nonzero(d)} of {d.size} elements)"
        print(f"{k:8s} {str(x.shape):24s} {msg}")
        ok &= same
    return ok


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib")
    ap.add_argument("--out")
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        sys.exit(0 if compare(*a.compare) else 1)
    run(a.lib, a.out, a.envs, a.steps)
