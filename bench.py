"""Benchmark: whole-job env-steps/s of the PHC imitation env step on MI355X.

Contract: `python bench.py --gpus N --steps K --warmup W` (N>1 under torch.distributed.run,
one rank per GPU over RCCL).  Rank 0 prints ONE JSON line.

Workload (BASELINE.json metric: env-steps/s, 24-joint SMPL, 4096 envs per GPU): one step =
PHCPufferEnv.step on 4096 envs = actions->PD (phc_actions_to_pd) + the physics stand-in
(phc_physics_replay: replayed reference states + noise, BASELINE configs[1]) + the fused
obs/reward/reset/bookkeeping kernel (phc_env_step) + re-initialisation of terminated envs
(phc_reset_envs).  Motions: a synthetic library of 4096 clips, U{60..300} frames at 30 fps,
built on device by the HIP FK path (AMASS is not available offline).  Actions are a fixed
random batch (no policy inference in this step).  Envs shard across ranks with no data-path
collective (weak scaling); the only collectives are the timing barrier and the max-reduce.

Roofline: the dominant kernel is phc_env_step (HBM-bound); algorithmic bytes per env-step =
10,886 (7,122 read + 3,764 written), achieved = bytes x envs / average kernel
time measured with HIP events around every launch in the timed region.  `traffic` = HBM
bytes per launch from rocprofv3 PMC counters (FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction)
read from profiles/traffic_<envs>.json when present, else null.

cpu_baseline: the numpy oracle (oracle/phc_oracle.py) env step on the same 4096-env batch,
1 thread, bounded to ~10 s, rank 0 at N=1 only.
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import phc_amd_path  # noqa: E402

phc_amd_path.register()

BYTES_PER_ENV_STEP = 10886
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--min-len", type=int, default=60)
    ap.add_argument("--max-len", type=int, default=300)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--traffic-file", default=None)
    return ap.parse_args()


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def build_env(args, rank, device):
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, counts, fps = synthetic_clips(args.envs, args.min_len, args.max_len, seed=1000 + rank, device=device)
    packed = PackedMotions.from_global_rotations(q, t, counts, fps)
    del q, t
    cfg = EnvConfig(num_envs=args.envs, device_id=torch.cuda.current_device(), seed=rank)
    env = PHCPufferEnv(cfg, motion_data=packed)
    env.reset()
    return env, packed


def cpu_baseline(env, packed, seconds):
    """Oracle env step on the same batch (numpy, 1 thread)."""
    from oracle import phc_oracle as O

    fr = packed.frames.cpu().numpy()
    lib = O.MotionLib(fr[..., 0:3], fr[..., 3:7], packed.local_rot.cpu().numpy(), fr[..., 7:10], fr[..., 10:13],
                      packed.dof_vel.cpu().numpy(), packed.num_frames.cpu().numpy(),
                      (1.0 / packed.motion_dt.double()).cpu().numpy())
    e = env.env
    args = (e._sampled_motion_ids.cpu().numpy(), (e.progress_buf.cpu().numpy() + 1).astype(np.int16),
            e._motion_start_times.cpu().numpy(), e._motion_start_times_offset.cpu().numpy(),
            e._global_offset.cpu().numpy(), e._rigid_body_state.cpu().numpy(), e._dof_vel.cpu().numpy(),
            e.dof_force_tensor.cpu().numpy())
    n = len(args[0])
    O.env_step(lib, *args)  # warm
    t0 = time.perf_counter()
    steps = 0
    while True:
        O.env_step(lib, *args)
        steps += 1
        if time.perf_counter() - t0 > seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": n * steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"{steps} oracle env steps x {n} envs (motion state x2 + reward + reset + obs, numpy fp32, "
                      f"1 thread, {dt:.1f}s)"}


def main():
    args = parse()
    world, rank, local = setup_dist(args)
    device = f"cuda:{torch.cuda.current_device()}"
    torch.manual_seed(1234 + rank)
    env, packed = build_env(args, rank, device)
    actions = torch.rand((args.envs, 69), device=device) * 2 - 1

    for _ in range(args.warmup):
        env.step(actions)
    torch.cuda.synchronize()
    env.env.kernel_events = []
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        env.step(actions)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in env.env.kernel_events]
    env.env.kernel_events = None
    kern_s = float(np.mean(kern_ms)) * 1e-3
    t = torch.tensor([elapsed, kern_s], dtype=torch.float64, device=device)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    elapsed, kern_s = float(t[0]), float(t[1])

    # sanity: the env must be tracking (not resetting every step)
    resets = float(env.stats.sum(0)[7].item())

    if rank == 0:
        total_env_steps = args.envs * world * args.steps
        achieved = BYTES_PER_ENV_STEP * args.envs / kern_s / 1e9
        traffic = None
        tf = args.traffic_file or os.path.join(ROOT, "profiles", f"traffic_{args.envs}.json")
        if os.path.exists(tf):
            with open(tf) as f:
                traffic = json.load(f).get("bytes_per_launch")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(env, packed, args.cpu_seconds)
        out = {
            "metric": "env-steps/sec (whole node), 24-joint SMPL humanoid, 4096 envs per GPU",
            "value": total_env_steps / elapsed,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (device-generated SMPL clips U{%d..%d} frames @30fps; replayed physics)" % (
                args.min_len, args.max_len),
            "config": {"workload": "PHCPufferEnv.step: actions->PD + replay physics + fused obs/reward/reset + "
                                   "reset re-init (no policy)", "envs_per_gpu": args.envs,
                       "global_envs": args.envs * world, "motions_per_gpu": args.envs,
                       "parallelism": f"dp{world} (env shards)"},
            "roofline": {"bound": "hbm", "kernel": "phc_env_step", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel_us": kern_s * 1e6, "algorithmic_bytes_per_env_step": BYTES_PER_ENV_STEP},
            "cpu_baseline": cpu,
            "resets_in_timed_region": resets,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
