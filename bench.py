"""Benchmark: whole-job env-steps/s of the PHC imitation rollout + PPO step on MI355X.

Contract: `python bench.py --gpus N --steps K --warmup W`: N>1 runs one rank per GPU over RCCL,
either under the caller's torch.distributed.run or, without one, under a torch.distributed.run
this script starts as a child process (launch_ranks).  Rank 0 prints ONE JSON line.  Default workload (BASELINE.json
configs[2] at 4096 envs per GPU; the metric's config):

  --mode ppo (default): one step = one full PPO iteration of clean_pufferl exactly as
      scripts/train.py runs it: evaluate() until 131072 mask-true rows are collected
      (PHCPolicy inference + PHCPufferEnv.step on 4096 envs + on-device experience store),
      RunningNorm update over the batch, train() = GAE + 4 epochs x 4 minibatches of 32768
      (forward, PPO loss, backward, grad clip, Adam).  value = rows collected / wall time,
      the reference's SPS definition (clean_pufferl/structs.py:354).
  --mode rollout: one step = policy inference + PHCPufferEnv.step + experience store.
  --mode env: one step = PHCPufferEnv.step (actions->PD, physics stand-in, fused
      obs/reward/reset/re-init kernel) with a fixed random action batch.

Physics is the replay stand-in (BASELINE configs[1]); motions are a synthetic library of 4096
clips, U{60..300} frames at 30 fps, built on device by the HIP FK path (AMASS is not
available offline).  Policy weights are random-init (orthogonal, as the reference).  Envs
shard across ranks (weak scaling); the PPO update all-reduces gradients and advantage
statistics over RCCL.

Roofline: with the replay physics the whole env phase is ONE launch, phc_env_step_replay
(HBM-bound; R13 + the stand-in + the fused obs / reward / reset step): 11,714 algorithmic bytes per
env-step (BYTES_PER_ENV_STEP_FUSED); with articulated physics the env step is phc_env_step,
10,886 B (7,122 read + 3,764 written).  achieved = bytes x envs / average kernel
time, which the kernels stamp themselves (phc_timer_*: the first workgroup's start and the last
workgroup's end from the 100 MHz constant clock, plain per-workgroup stores into a slot of the
timer) for a uniform sample of the launches in the timed region: every ENV_TIMER_PERIOD-th env step
and every GEMM_TIMER_PERIOD-th trunk GEMM, launches replayed from captured hipGraphs included (HIP
events cannot be timed inside a graph on ROCm 7.2).  A stamped launch runs as fast as an untimed
one; rocprofv3's duration of the same launch is ~3 us (env step) / ~1 % (GEMM) longer: it also counts
the dispatch and the end-of-kernel release (profiles/r05_clock_vs_rocprof.json).  `traffic` = HBM bytes per launch from rocprofv3 PMC counters
(2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction) read from profiles/traffic[_fused]_<envs>.json
when present, else null.

cpu_baseline: the numpy oracle (oracle/phc_oracle.py) env step on the same 4096-env batch at
1 thread and over all available cores (forked env shards), plus the C restatement of the
reference's GAE, bounded to ~10 s, rank 0 at N=1 only.  An env-step-only comparison (the PPO
GEMMs have no CPU oracle); the line says so.
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

BYTES_PER_ENV_STEP = 10886  # phc_env_step (K1+K2) after a separate physics launch
# phc_env_step_replay (the default with replay physics): R13 + the stand-in + the env step in one
# launch.  Reads 5,874 B: 4 frame rows 4,992 + the 2 dof-vel frame rows at t 552 + actions 276 +
# scalars 54; writes 5,840 B: rigid bodies 1,248 + dof vel 276 + forces 276 + PD targets 276 + obs /
# reward / flags / progress 3,764
BYTES_PER_ENV_STEP_FUSED = 11714
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
MFMA_F16_PEAK_TFS = 2500.0  # dense f16 / bf16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense, no sparsity)
DEFAULTS = {"env": (200, 20), "rollout": (64, 8), "ppo": (10, 5)}  # ppo: the warmup covers every graph capture
# kernel-timer sampling (module docstring): every 4th env-step / physics launch, every 16th trunk GEMM
# (16 is coprime to a minibatch's 13 GEMM launches and divides an iteration's 16 x 13: each layer's
# launch exactly once per iteration)
ENV_TIMER_PERIOD = 4
GEMM_TIMER_PERIOD = 16
KERNEL_TIMING_NOTE = ("in-kernel stamps (first workgroup start -> last workgroup end, s_memrealtime); rocprofv3 "
                      "durations of the same launches run ~3 us (env) / ~1 % (GEMM) longer: dispatch + end-of-kernel "
                      "release (profiles/r05_clock_vs_rocprof.json)")
ENV_TIMING_NOTE = ("kernel_us / frac: dispatch-inclusive (the rocprofv3 basis) = the stamped mean over the timed region's "
                   "sampled launches + dispatch_us, the mean (HIP-event-bracketed duration - stamped duration) of "
                   "DISPATCH_PROBE_STEPS eager launches of the same kernel right after the timed region; "
                   "kernel_us_stamped / frac_stamped: the in-kernel stamps alone")
DISPATCH_PROBE_STEPS = 32


def env_dispatch_us(env, actions, steps=DISPATCH_PROBE_STEPS):
    """The env kernel's dispatch + end-of-kernel overhead that its own stamps do not see: `steps` eager
    HumanoidPHC.step launches (one kernel each with the replay physics), each bracketed by HIP events on
    the launching stream AND stamped by the kernel; returns mean(event duration - stamped duration) in
    microseconds (what rocprofv3 adds to the stamped time), or None."""
    from puffer_phc_amd._native import KernelTimer

    e = env.env
    # a slot holds 2 words per workgroup; the timer sizes its buffer for 1,024 workgroups per slot and the
    # replay kernel runs one workgroup per env pair
    per_slot = -(-((e.num_envs + 1) // 2) // 1024)
    timer = KernelTimer(capacity=(steps + 8) * per_slot, period=1)
    old = e.kernel_timer
    e.kernel_timer = timer
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in evs:  # materialise the events before the measured launches
        a.record()
        b.record()
    torch.cuda.synchronize()
    timer.reset()
    for a, b in evs:
        a.record()
        e.step(actions, auto_reset=True)
        b.record()
    torch.cuda.synchronize()
    e.kernel_timer = old
    stamped = timer.durations_ms()
    if len(stamped) != steps:
        return None
    ev = [a.elapsed_time(b) for a, b in evs]
    return float(np.mean(np.asarray(ev) - np.asarray(stamped)) * 1e3)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--mode", choices=["env", "rollout", "ppo"], default="ppo")
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--batch-size", type=int, default=131072, help="PPO rows per rank per iteration")
    ap.add_argument("--minibatch-size", type=int, default=32768)
    ap.add_argument("--min-len", type=int, default=60)
    ap.add_argument("--max-len", type=int, default=300)
    ap.add_argument("--precision", default="fp16", choices=["xf32", "fp16", "bf16"],
                    help="policy GEMM arithmetic (TrainConfig.precision)")
    ap.add_argument("--amp", action="store_true",
                    help="AMP discriminator obs + discriminator loss (BASELINE config C5, with --precision bf16)")
    ap.add_argument("--physics", choices=["replay", "articulated"], default="replay",
                    help="replay = BASELINE configs[1]'s physics stand-in (the headline); articulated = the N3 "
                         "articulated-body step (phc_physics_step) in its place")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--traffic-file", default=None)
    ap.add_argument("--dp-mode", choices=["grouped", "per_layer", "split"], default="grouped",
                    help="data-parallel weight-gradient / all-reduce schedule at N > 1 (twin_mlp.set_dp_mode)")
    ap.add_argument("--dist-1rank", action="store_true",
                    help="run the data-parallel path on ONE GPU: a 1-rank RCCL group (every gradient / advantage "
                         "all-reduce of an N-GPU rank, on one process), to time the DP path beside the headline")
    a = ap.parse_args()
    k, w = DEFAULTS[a.mode]
    a.steps = k if a.steps is None else a.steps
    a.warmup = w if a.warmup is None else a.warmup
    return a


def setup_dist(dist_1rank=False):
    from puffer_phc_amd import distributed as D

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # RCCL over xGMI; PHC_DIST_BACKEND=gloo rehearses several ranks on one GPU
        D.init_from_env(os.environ.get("PHC_DIST_BACKEND", "nccl"))
    elif dist_1rank:
        # a 1-rank RCCL group, initialised before any other GPU call (the rendezvous on the loopback)
        import socket

        if "MASTER_PORT" not in os.environ:
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")):
            os.environ.setdefault(k, v)
        D.init_from_env("nccl", force=True)
    else:
        torch.cuda.set_device(0)
    return D.world_size(), D.rank()


def build_env(args, rank):
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    device = f"cuda:{torch.cuda.current_device()}"
    q, t, counts, fps = synthetic_clips(args.envs, args.min_len, args.max_len, seed=1000 + rank, device=device)
    packed = PackedMotions.from_global_rotations(q, t, counts, fps)
    del q, t
    cfg = EnvConfig(num_envs=args.envs, device_id=torch.cuda.current_device(), seed=rank, use_amp_obs=args.amp,
                    physics=args.physics)
    env = PHCPufferEnv(cfg, motion_data=packed)
    env.reset()
    return env, packed, cfg


# wave-instructions/s: 256 CUs x 4 SIMD-32 units, a wave64 VALU instruction every 2 cycles per SIMD
# (MI355X_MICROARCH.md "Wave scheduling"), at 2.4 GHz
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2


def physics_roofline(args, kern_s, launches):
    """N3 physics kernel (phc_physics_step): VALU-issue bound.  achieved = the kernel's VALU
    wave-instructions per launch (SQ_INSTS_VALU from the committed PMC pass over this bench
    command's own launches, profiles/physics_valu_4096_bench.json — the count depends on the contact
    and self-collision state — else the standing probe's, profiles/physics_valu_4096.json; scaled by
    the wave count: one wave per 2 envs) / its mean launch duration timed live by the launch's own
    events; peak = VALU_ISSUE_PEAK."""
    f = os.path.join(ROOT, "profiles", "physics_valu_4096_bench.json")
    if not os.path.exists(f):
        f = os.path.join(ROOT, "profiles", "physics_valu_4096.json")
    instr = None
    if os.path.exists(f):
        with open(f) as fh:
            ref = json.load(fh)
        instr = ref["valu_instr_per_launch"] * ((args.envs + 1) // 2) / ref["waves_per_launch"]
    ach = instr / kern_s if instr and kern_s > 0 else None
    return {"bound": "valu-issue", "kernel": "phc_physics_step", "achieved": ach, "peak": VALU_ISSUE_PEAK,
            "unit": "wave-instr/s", "frac": ach / VALU_ISSUE_PEAK if ach else None, "kernel_us": kern_s * 1e6,
            "launches_timed": launches, "env_steps_per_s_kernel": args.envs / kern_s if kern_s > 0 else None,
            "valu_instr_per_launch": instr, "valu_count_file": os.path.basename(f) if instr else None}


def physics_cpu_baseline(seconds):
    """The float64 numpy restatement of the physics step (oracle/physics_oracle.py, test
    infrastructure) on this host, one thread, over a 64-env sample of standing humanoids."""
    import numpy as np

    from oracle import physics_oracle as PO

    m = PO.load_model()
    n = 64
    rb, dof = PO.rest_state(m, n, 0.0)
    tgt = np.random.default_rng(0).normal(0, 0.1, (n, PO.NUM_DOF))
    t0 = time.perf_counter()
    k = 0
    while True:
        rb, dof, _ = PO.step(m, rb, dof, tgt)
        k += 1
        if time.perf_counter() - t0 > seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": n * k / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"{k} physics steps x {n} envs (float64 numpy, vectorised over envs, 16 substeps each)"}


def _host_cpu():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model


def _host_workers():
    """Worker processes for the all-cores leg: the CPUs this process may run on, capped at the GPU's
    share of its host.  The measurement boxes lease one GPU of an 8-GPU host together with 16 of the
    host's CPUs (OMP_NUM_THREADS / MAX_JOBS are set to 16 there), while os.sched_getaffinity and
    nproc report every CPU of the machine, so the affinity set alone would time cores that belong
    to the other seven GPUs' jobs.  16 is therefore the fair all-cores figure per GPU; on a host
    whose affinity set is smaller, that set is used."""
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(avail, cap, 16))


_CPU_SHARD = None  # (lib, args) of one worker, inherited through fork


def _cpu_shard_run(job):
    """One worker of the all-cores leg: `steps` oracle env steps over its env shard."""
    from oracle import phc_oracle as O

    lo, hi, steps = job
    lib, args = _CPU_SHARD
    sub = tuple(a[lo:hi] for a in args)
    O.env_step(lib, *sub)  # warm
    t0 = time.perf_counter()
    for _ in range(steps):
        O.env_step(lib, *sub)
    return time.perf_counter() - t0


def cpu_baseline(env, packed, seconds):
    """BASELINE.md §3 / SURVEY §8d: the CPU restatement of the env step (motion state x2 + reward
    + reset + obs, the composition HumanoidPHC.step performs, physics excluded) on the same
    4096-env batch, timed on this host at 1 thread and at all available cores (env shards over
    forked worker processes, numpy fp32), plus the reference's GAE (oracle/gae.c, the Cython
    loop restated in C) over one 131072-row batch.  This is an ENV-STEP-ONLY comparison: it
    does not include policy inference or the PPO update that the headline value contains."""
    import multiprocessing as mp

    from oracle import c_oracle
    from oracle import phc_oracle as O

    global _CPU_SHARD
    fr = packed.frames.cpu().numpy()
    lib = O.MotionLib(fr[..., 0:3], fr[..., 3:7], packed.local_rot.cpu().numpy(), fr[..., 7:10], fr[..., 10:13],
                      packed.dof_vel.cpu().numpy(), packed.num_frames.cpu().numpy(),
                      packed.fps.cpu().numpy())
    e = env.env
    args = (e._sampled_motion_ids.cpu().numpy(), (e.progress_buf.cpu().numpy() + 1).astype(np.int16),
            e._motion_start_times.cpu().numpy(), e._motion_start_times_offset.cpu().numpy(),
            e._global_offset.cpu().numpy(), e._rigid_body_state.cpu().numpy(), e._dof_vel.cpu().numpy(),
            e.dof_force_tensor.cpu().numpy())
    n = len(args[0])
    half = seconds / 2
    # 1 thread (the reference's setting after load_motions, motion_lib.py:335)
    O.env_step(lib, *args)  # warm
    t0 = time.perf_counter()
    steps1 = 0
    while True:
        O.env_step(lib, *args)
        steps1 += 1
        if time.perf_counter() - t0 > half:
            break
    dt1 = time.perf_counter() - t0
    one = n * steps1 / dt1
    # all cores: the same batch split into `workers` env shards, each stepped by a forked process
    # (numpy only in the children: they never touch the GPU)
    workers = _host_workers()
    steps_all = max(2, int(round(half * one * workers * 0.75 / n)))  # ~half seconds at 75 % scaling
    bounds = np.linspace(0, n, workers + 1).astype(int)
    jobs = [(int(bounds[i]), int(bounds[i + 1]), steps_all) for i in range(workers)]
    _CPU_SHARD = (lib, args)
    try:
        with mp.get_context("fork").Pool(workers) as pool:
            pool.map(_cpu_shard_run, [(lo, min(hi, lo + 8), 1) for lo, hi, _ in jobs])  # fork + import warm-up
            t0 = time.perf_counter()
            per = pool.map(_cpu_shard_run, jobs)
            dta = time.perf_counter() - t0
    finally:
        _CPU_SHARD = None
    allc = n * steps_all / dta
    # GAE (c_gae.pyx restated in C) over one PPO batch of 131072 rows, 1 thread
    rng = np.random.default_rng(0)
    B = 131072
    d = (rng.random(B) < 0.01).astype(np.float32)
    v, r = rng.standard_normal(B).astype(np.float32), rng.standard_normal(B).astype(np.float32)
    c_oracle.compute_gae(d, v, r, 0.98, 0.2)
    reps, t0 = 0, time.perf_counter()
    while reps < 20 or time.perf_counter() - t0 < 0.5:
        c_oracle.compute_gae(d, v, r, 0.98, 0.2)
        reps += 1
    gae_ms = (time.perf_counter() - t0) / reps * 1e3
    # the port's speed relative to the reference's own torch-CPU composition, measured side by side on
    # one host (tools/ref_vs_port_cpu.py: the reference cannot travel to this box)
    calib = None
    cf = os.path.join(ROOT, "profiles", "r04_ref_vs_port_cpu.json")
    if os.path.exists(cf):
        with open(cf) as f:
            c = json.load(f)
        calib = {"port_over_reference_1_thread": c["port_over_reference"], "calibration_host": c["host_cpu_model"],
                 "reference_equivalent_value_1_thread": one / c["port_over_reference"],
                 "reference_equivalent_value_all_cores": allc / c["port_over_reference"],
                 "file": os.path.relpath(cf, ROOT)}
    return {"value": allc, "unit": "env-steps/s", "cores": workers, "kind": "port",
            "reference_calibration": calib,
            "comparison": "env step only (motion state x2 + reward + reset + obs); no policy inference or PPO "
                          "update, which the headline value includes",
            "value_1_thread": one, "value_all_cores": allc, "cores_all": workers,
            "cores_note": "all-cores leg = min(affinity set, OMP_NUM_THREADS, 16): the one-GPU lease's CPU share "
                          "(bench._host_workers)",
            "host_nproc": os.cpu_count(), "host_cpu_model": _host_cpu(),
            "gae_ms_131072_rows_1_thread": gae_ms,
            "sample": f"{n} envs: {steps1} oracle env steps at 1 thread ({dt1:.1f}s); {steps_all} steps over "
                      f"{workers} forked env shards ({dta:.1f}s, slowest shard {max(per):.1f}s); numpy fp32. "
                      f"GAE: oracle/gae.c over 131072 rows x {reps}"}


def whole_job_steps(counts, is_global, world):
    """Whole-job env-steps of the timed region from each rank's count.  ppo mode counts the
    reference's SPS numerator, `global_step` (clean_pufferl/core.py:135-138), which data-parallel
    evaluate() already sums over ranks (core._global_count): every rank holds the whole-job count
    and it is taken once.  env / rollout modes count each rank's own env steps: they are summed."""
    counts = [float(c) for c in counts]
    if len(counts) != world:
        raise ValueError(f"{len(counts)} rank counts for world size {world}")
    if is_global:
        if max(counts) != min(counts):
            raise ValueError(f"ranks disagree on the whole-job step count: {counts}")
        return counts[0]
    return sum(counts)


class Runner:
    """One benchmark 'step' per mode; returns the env-steps it processed (ppo mode: the
    whole-job count, see whole_job_steps)."""

    def __init__(self, args, env, env_cfg):
        self.args, self.env = args, env
        dev = env_cfg.device
        self.actions = torch.rand((args.envs, 69), device=dev) * 2 - 1
        if args.mode == "env":
            return
        from puffer_phc_amd import clean_pufferl
        from puffer_phc_amd.config import TrainConfig
        from puffer_phc_amd.policies import PHCPolicy, Policy

        self.cp = clean_pufferl
        self.policy = Policy(PHCPolicy(env)).to(dev)
        self.tcfg = TrainConfig(device_id=torch.cuda.current_device(), batch_size=args.batch_size,
                                minibatch_size=args.minibatch_size, checkpoint_interval=10 ** 9,
                                total_timesteps=10 ** 15, precision=args.precision)
        self.components, self.info, self.util = clean_pufferl.create("bench", self.tcfg, env_cfg, env, self.policy)
        self.obs = env.observations

    def phase_ms(self, steps):
        """Host wall time of evaluate / train per timed step (clean_pufferl Profile; ppo mode)."""
        if self.args.mode != "ppo":
            return None
        p = self.info.profile
        return {k: (getattr(p, k).elapsed - self._p0[k]) / steps * 1e3 for k in self._p0}

    def skipped(self):
        """Optimizer steps the fp16 loss scaler skipped so far (None outside fp16 PPO)."""
        c = getattr(self, "components", None)
        if c is None or c.skipped_steps is None:
            return None
        return int(c.skipped_steps)

    _gpu_phases = None

    def mark(self):
        self._skip0 = self.skipped()
        self._gpu_phases = [] if self.args.mode == "ppo" else None
        if self._gpu_phases is not None:
            # the phase events of every timed step, created (and their HIP events materialised by a
            # record) before the timed region: a torch Event creates its hipEvent at its first record
            self._event_pool = [self._phase_events() for _ in range(self.args.steps + 1)]
            for ev in self._event_pool:
                for e in ev:
                    e.record()
            torch.cuda.synchronize()
        if self.args.mode == "ppo":
            p = self.info.profile
            self._p0 = {k: getattr(p, k).elapsed for k in ("evaluate", "env", "eval_forward", "train",
                                                             "train_forward", "learn", "train_misc")}

    def step(self):
        a = self.args
        if a.mode == "env":
            self.env.step(self.actions)
            return a.envs
        if a.mode == "rollout":
            exp = self.components.experience
            if exp.full:
                exp.ptr = 0
            o, r, d, t, _, env_id, mask = self.env.recv()
            with torch.no_grad(), self.cp.core.autocast(self.tcfg):
                actions, logprob, _, value = self.policy(o)
            exp.store(o, None, value.flatten(), actions, logprob, r, d, t, env_id, mask, n_valid=a.envs)
            self.env.send(actions)
            return a.envs
        g0 = self.info.global_step
        ev = None
        if self._gpu_phases is not None:
            pool = getattr(self, "_event_pool", None)
            ev = pool.pop() if pool else self._phase_events()
        if ev:
            ev[0].record()
        self.cp.evaluate(self.components, self.info)
        if ev:
            ev[1].record()
        self.policy.policy.update_obs_rms(self.components.experience.obs)
        if self.args.amp:
            self.policy.policy.update_amp_obs_rms(self.components.experience.amp_obs)
        if ev:
            ev[2].record()
        self.cp.train(self.components, self.info, self.util)
        if ev:
            ev[3].record()
            self._gpu_phases.append(ev)
        return self.info.global_step - g0

    @staticmethod
    def _phase_events():
        return [torch.cuda.Event(enable_timing=True) for _ in range(4)]

    def gpu_phase_ms(self):
        """GPU-timeline time per timed step between events recorded on the stream at the phase
        boundaries (evaluate | obs-RMS update | train): what the GPU spent from the first launch
        of a phase to the last, idle gaps included — unlike the host timers, no phase absorbs
        another's GPU work through a synchronising call."""
        if not self._gpu_phases:
            return None
        n = len(self._gpu_phases)
        tot = {"evaluate": 0.0, "rms_update": 0.0, "train": 0.0}
        for e in self._gpu_phases:
            tot["evaluate"] += e[0].elapsed_time(e[1])
            tot["rms_update"] += e[1].elapsed_time(e[2])
            tot["train"] += e[2].elapsed_time(e[3])
        return {k: v / n for k, v in tot.items()}


DP_FIELDS = ("mode", "backend", "allreduce_exposed_ms_per_minibatch_rank0",
             "allreduce_exposed_ms_per_minibatch_max_rank", "minibatches_timed", "grad_bytes_per_minibatch",
             "train_graph", "dist_1rank", "note")


def dp_summary(mode, exp_ms, n_bw, grad_bytes, device, train_graph=False, dist_1rank=False):
    """config.dp at N > 1 (collective: every rank calls it): the exposed all-reduce wait per minibatch
    backward on this rank (rank 0's goes in the line) and on the slowest rank."""
    e = torch.tensor([exp_ms or 0.0], dtype=torch.float64, device=device)
    torch.distributed.all_reduce(e, op=torch.distributed.ReduceOp.MAX)
    return {"mode": mode, "backend": torch.distributed.get_backend(),
            "allreduce_exposed_ms_per_minibatch_rank0": exp_ms,
            "allreduce_exposed_ms_per_minibatch_max_rank": float(e[0]), "minibatches_timed": n_bw,
            "grad_bytes_per_minibatch": grad_bytes, "train_graph": bool(train_graph), "dist_1rank": bool(dist_1rank),
            "note": "CUDA events on rank's compute stream around the wait for the backward's all-reduces "
                    "(FlatGrads.overlap_finish): the stall after the last backward kernel"}


def launch_ranks(n):
    """`--gpus N` without a torch.distributed launcher around this process: start N ranks (one per
    GPU) under torch.distributed.run as CHILD processes and return their exit code.  This parent
    never touches the GPU (nothing before this point initialises HIP); rank 0 prints the JSON line
    on the inherited stdout."""
    import socket
    import subprocess

    with socket.socket() as s:  # a free rendezvous port on the loopback interface
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}: the launcher's world "
              "size is used", file=sys.stderr)
    if os.environ.get("PHC_WATCHDOG_S"):  # debugging aid: dump every thread's stack periodically
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["PHC_WATCHDOG_S"]), repeat=True)
    world, rank = setup_dist(args.dist_1rank)
    from puffer_phc_amd import distributed as D

    dp_on = D.is_dist()  # the data-parallel path runs (N > 1, or --dist-1rank)
    from puffer_phc_amd.policies import twin_mlp

    twin_mlp.set_dp_mode(args.dp_mode)
    device = f"cuda:{torch.cuda.current_device()}"
    torch.manual_seed(1234 + rank)
    env, packed, env_cfg = build_env(args, rank)
    runner = Runner(args, env, env_cfg)

    from puffer_phc_amd._native import KernelTimer, gemm_set_timer

    # the kernel timers are attached before the warmup, so launches captured into hipGraphs during it
    # (the train / rollout graphs) carry timer slots; reset() after the warmup keeps only what the
    # timed region stamps (a graph's slots: its last replay)
    # sized for every sampled launch at one slot per launch (2 words per workgroup; 1,024 workgroups per slot)
    per_slot = -(-((args.envs + 1) // 2) // 1024)
    timer = env.env.kernel_timer = KernelTimer(capacity=max(4096, 64 * args.steps) * per_slot, period=ENV_TIMER_PERIOD)
    # the PPO update's trunk GEMMs (phc_twin_gemm of more than 4,096 rows + the weight gradients), every
    # GEMM_TIMER_PERIOD-th stamped by the kernel itself, with its 2 m n k FLOPs
    gtimer = KernelTimer(capacity=max(4096, 256 * args.steps), period=GEMM_TIMER_PERIOD)
    gemm_set_timer(gtimer)
    ptimer = None
    if args.physics == "articulated":  # phc_physics_step launches, stamped by the kernel
        ptimer = env.env.physics.timer = KernelTimer(capacity=max(4096, 64 * args.steps), period=ENV_TIMER_PERIOD)
    for _ in range(args.warmup):
        runner.step()
    torch.cuda.synchronize()
    for tm in (timer, gtimer, ptimer):
        if tm is not None:
            tm.reset()
    flat = getattr(getattr(runner, "components", None), "flat_grads", None)
    if flat is not None and dp_on:
        flat.timing, flat.exposed = True, []
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    runner.mark()
    from puffer_phc_amd import _native as _N

    gemm_launch0, tick0 = _N.GEMM_LAUNCHES[0], env.tick
    t0 = time.perf_counter()
    processed = 0
    for _ in range(args.steps):
        processed += runner.step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    skipped = runner.skipped()
    skipped = None if skipped is None else skipped - runner._skip0
    env_steps = timer.count  # sampled env-step launches of the timed region, stamped by the kernel itself
    # launches the timed region ran (captured graphs replay launches the host does not offer again)
    env_offered, gemm_offered = env.tick - tick0, _N.GEMM_LAUNCHES[0] - gemm_launch0
    kern_s = timer.total_ms() / max(env_steps, 1) * 1e-3
    env.env.kernel_timer = None
    gemm_set_timer(None)
    gemm_launches, gemm_flops = gtimer.count, gtimer.work
    gemm_s = gtimer.total_ms() * 1e-3 if gemm_launches else 0.0
    phys_launches, phys_s = 0, 0.0
    if ptimer is not None:
        env.env.physics.timer = None
        phys_launches = ptimer.count
        phys_s = ptimer.total_ms() * 1e-3 / max(phys_launches, 1)
    # the env kernel's dispatch overhead (for the rocprof-basis roofline), measured on eager launches after
    # the timed region (replay physics: one launch per step)
    disp_us = env_dispatch_us(env, runner.actions) if args.physics == "replay" else None
    t = torch.tensor([elapsed, kern_s], dtype=torch.float64, device=device)
    counts = [float(processed)]
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        mine = torch.tensor([float(processed)], dtype=torch.float64, device=device)
        every = [torch.zeros_like(mine) for _ in range(world)]
        torch.distributed.all_gather(every, mine)
        counts = [float(c) for c in every]
    elapsed, kern_s = float(t[0]), float(t[1])
    processed_all = whole_job_steps(counts, args.mode == "ppo", world)
    dp = None
    if flat is not None and dp_on:
        exp_ms, n_bw = flat.exposed_ms()
        flat.timing = False
        st = getattr(runner.components, "_train_graph", None)
        dp = dp_summary(args.dp_mode, exp_ms, n_bw, flat.flat.numel() * 4, device,
                        train_graph=bool(st and st.get("graph") is not None and not st.get("failed")),
                        dist_1rank=args.dist_1rank)

    if rank == 0:
        fused = bool(getattr(env.env, "fused_env_step", False)) and args.physics == "replay"
        env_bytes = BYTES_PER_ENV_STEP_FUSED if fused else BYTES_PER_ENV_STEP
        # the rollout's fused RunningNorm operand (HumanoidPHC.set_obs_operand): the step also writes
        # the policy's [N, ld] half-precision first-GEMM operand row of every env
        opnd = getattr(env.env, "_obs_operand", None)
        opnd_bytes = int(opnd[0].shape[1] * opnd[0].element_size()) if opnd is not None else 0
        env_bytes += opnd_bytes
        achieved_st = env_bytes * args.envs / kern_s / 1e9 if kern_s > 0 else 0.0
        kern_rp = kern_s + (disp_us or 0.0) * 1e-6  # dispatch-inclusive (rocprofv3 basis)
        achieved = env_bytes * args.envs / kern_rp / 1e9 if kern_rp > 0 else 0.0
        traffic = None
        # HBM bytes of the env step from the committed PMC passes: the rollout-context launch (fused
        # operand written) has its own file (tools/gpu_pass.sh, stage pmc)
        kind = ("fused_ppo_" if opnd_bytes else "fused_") if fused else ""
        tf = args.traffic_file or os.path.join(ROOT, "profiles", f"traffic_{kind}{args.envs}.json")
        if os.path.exists(tf):
            with open(tf) as f:
                traffic = json.load(f).get("bytes_per_launch")
        cpu = None
        if world == 1 and not args.no_cpu_baseline and args.physics == "replay":
            cpu = cpu_baseline(env, packed, args.cpu_seconds)
        workloads = {
            "ppo": "clean_pufferl PPO iteration: evaluate %d rows (PHCPolicy %s inference + PHCPufferEnv.step) + "
                   "RMS update + train (GAE, 4 epochs x %d minibatches of %d, Adam)" % (
                       args.batch_size, args.precision, args.batch_size // args.minibatch_size, args.minibatch_size),
            "rollout": "PHCPolicy %s inference + PHCPufferEnv.step + on-device experience store" % args.precision,
            "env": "PHCPufferEnv.step: actions->PD + %s physics + fused obs/reward/reset + reset re-init "
                   "(fixed random actions, no policy)" % args.physics,
        }
        phys_note = ("replayed physics" if args.physics == "replay" else
                     "articulated-body physics (phc_physics_step, %d substeps per sim step)" % env_cfg.physics_substeps)
        out = {
            "metric": "env-steps/sec (whole node), 24-joint SMPL humanoid, 4096 envs per GPU",
            "value": processed_all / elapsed,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"xf32": "fp32", "fp16": "fp16", "bf16": "bf16"}[args.precision] if args.mode != "env"
            else "fp32",
            "data": "synthetic (device-generated SMPL clips U{%d..%d} frames @30fps; %s; "
                    "random-init policy)" % (args.min_len, args.max_len, phys_note),
            "config": {"workload": workloads[args.mode], "mode": args.mode, "envs_per_gpu": args.envs,
                       "global_envs": args.envs * world, "motions_per_gpu": args.envs,
                       "parallelism": f"dp{world} (env shards, RCCL grad all-reduce)",
                       "amp_obs": bool(args.amp), "physics": args.physics,
                       "policy_gemm": {"xf32": "fp32 storage, hipBLASLt xf32 (torch 'high', as the reference)",
                                       "fp16": "fp16 operands (TF32's 11-bit significand; the reference runs "
                                               "TF32) on hand-written MFMA GEMMs with fused bias/SiLU epilogues, "
                                               "fp32 accumulate + outputs, dynamic loss scaling",
                                       "bf16": "bf16 operands on hand-written MFMA GEMMs with fused epilogues, "
                                               "fp32 accumulate + outputs"}[args.precision]
                       if args.mode != "env" else None,
                       "optimizer_steps_skipped_by_loss_scaler": skipped,
                       "phase_gpu_ms_per_step": runner.gpu_phase_ms(),
                       "phase_host_wall_ms_per_step": runner.phase_ms(args.steps),
                       "phase_note": "phase_gpu_ms: GPU-timeline time between stream events at the phase "
                                     "boundaries; phase_host_wall_ms: clean_pufferl's host Profile timers, "
                                     "where train_misc includes host waits on GPU work launched by other "
                                     "phases (the per-epoch stat readback)" if args.mode == "ppo" else None},
            "cpu_baseline": cpu,
        }
        out["config"]["env_steps_timed"] = processed_all  # value = env_steps_timed / wall seconds
        if dp is not None:
            out["config"]["dp"] = dp
        if args.physics == "articulated":
            out["roofline_physics"] = physics_roofline(args, phys_s, phys_launches)
            if not args.no_cpu_baseline:
                out["cpu_baseline_physics"] = physics_cpu_baseline(args.cpu_seconds)
        env_roof = {"bound": "hbm",
                    "kernel": "phc_env_step_replay (action->PD + replay physics + env step, one launch: the whole "
                              "env phase)" if fused else "phc_env_step",
                    "achieved": achieved, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                    "kernel_us": kern_rp * 1e6, "kernel_us_stamped": kern_s * 1e6, "dispatch_us": disp_us,
                    "frac_stamped": achieved_st / HBM_PEAK_GBS,
                    "timing": ENV_TIMING_NOTE if disp_us is not None else KERNEL_TIMING_NOTE,
                    "launches_timed": env_steps, "launches_in_region": env_offered,
                    "algorithmic_bytes_per_env_step": env_bytes, "obs_operand_bytes_per_env_step": opnd_bytes}
        if gemm_launches:
            # the dominant kernel of the PPO / rollout modes: the trunk GEMMs (MFMA-bound)
            tfs = gemm_flops / gemm_s / 1e12
            gtraffic = None  # HBM bytes per launch of the same launches (rocprofv3 PMC, tools/gpu_pass.sh stage pmc)
            gf = os.path.join(ROOT, "profiles", f"traffic_gemm_{args.envs}.json")
            if os.path.exists(gf):
                with open(gf) as f:
                    gtraffic = json.load(f).get("bytes_per_launch")
            out["roofline"] = {"bound": "mfma",
                               "kernel": "PPO-update trunk GEMMs: phc_twin_gemm (forward / input-gradient, fused "
                                         "epilogues) + phc_weight_grad_group / phc_weight_grad (weight gradients)",
                               "achieved": tfs, "peak": MFMA_F16_PEAK_TFS, "unit": "TFLOP/s",
                               "frac": tfs / MFMA_F16_PEAK_TFS, "traffic": gtraffic, "traffic_unit": "bytes",
                               "kernel_us": gemm_s / gemm_launches * 1e6, "timing": KERNEL_TIMING_NOTE, "launches_timed": gemm_launches,
                               "launches_in_region": gemm_offered,
                               "algorithmic_flops_per_launch": gemm_flops / gemm_launches}
            out["roofline_env_step"] = env_roof
        else:
            out["roofline"] = env_roof
        print(json.dumps(out), flush=True)
    if dp_on:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
