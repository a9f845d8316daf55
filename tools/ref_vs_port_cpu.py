"""Calibrate cpu_baseline's port against the reference's own CPU path on ONE host (build container only:
it imports the reference from /root/reference, which never travels to the GPU box).

Times, at 1 thread on the same 4096-env batch:
  * the reference's own post-physics env-step composition — MotionLibSMPL.get_motion_state x2,
    common.compute_imitation_reward, compute_humanoid_im_reset, compute_humanoid_observations_smpl_max,
    compute_imitation_observations_v6 (puffer_phc/motion_lib.py:549-626, envs/common.py:23-364), as
    tests/golden/make_golden.py `_compose_step` composes them (humanoid_phc.py:136-146, 1228-1333);
  * oracle/phc_oracle.env_step — the numpy port bench.py's cpu_baseline times on the GPU box.
Checks that both give the same obs / reward (1e-5) and writes profiles/<tag>_ref_vs_port_cpu.json with
env-steps/s of each and the port/reference factor that carries cpu_baseline over to the reference.

usage: OMP_NUM_THREADS=1 python tools/ref_vs_port_cpu.py [num_envs] [tag]
"""
import json
import os
import platform
import sys
import time

os.environ.setdefault("OMP_NUM_THREADS", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as G  # noqa: E402  (installs the stubs, imports the reference)
from oracle import phc_oracle as O  # noqa: E402


def _lib(num_clips, seed=11):
    rng = np.random.default_rng(seed)
    import joblib
    import tempfile
    from types import SimpleNamespace

    sk = G.SkeletonTree.from_mjcf(os.path.join(G.REF, "puffer_phc/assets/smpl_humanoid.xml"))
    lengths = rng.integers(60, 300, size=num_clips)
    motions = {f"synth_{i:04d}": G.synth_motion(rng, int(n)) for i, n in enumerate(lengths)}
    path = os.path.join(tempfile.mkdtemp(), "clips.pkl")
    joblib.dump(motions, path)  # our own file
    cfg = SimpleNamespace(motion_file=path, device="cpu", fix_height=G.ml.FixHeightMode.no_fix, min_length=-1,
                          max_length=300, im_eval=False, num_thread=1, smpl_type="smpl", step_dt=G.DT,
                          is_deterministic=True)
    lib = G.ml.MotionLibSMPL(cfg)
    lib.mesh_parsers = None
    lib.load_motions(skeleton_trees=[sk] * num_clips, gender_betas=torch.zeros(num_clips, 17),
                     limb_weights=torch.zeros(num_clips, 10), random_sample=False, start_idx=0)
    return lib


def _inputs(lib, n, seed=12):
    rng = np.random.default_rng(seed)
    M = lib._num_motions
    mids = rng.integers(0, M, size=n).astype(np.int64)
    lens = lib._motion_lengths.numpy()[mids]
    start = (np.floor(rng.random(n) * lens / np.float32(1 / 30)) * np.float32(1 / 30)).astype(np.float32)
    room = np.maximum(1, np.floor((lens - start) * 30)).astype(np.int64)
    progress = (rng.random(n) * room).astype(np.int16)
    start_off = np.zeros(n, np.float32)
    go = np.zeros((n, 3), np.float32)
    t_eval = (progress.astype(np.float32) * np.float32(G.DT) + start + start_off).astype(np.float32)
    rb = G._noisy_states(rng, lib, mids, t_eval, go)
    dof_vel = rng.normal(size=(n, 69)).astype(np.float32)
    dof_force = (rng.normal(size=(n, 69)) * 50).astype(np.float32)
    return mids, progress, start, start_off, go, rb, dof_vel, dof_force


def _time(fn, min_s=5.0):
    fn()
    reps, t0 = 0, time.perf_counter()
    while True:
        out = fn()
        reps += 1
        el = time.perf_counter() - t0
        if el >= min_s:
            return el / reps, reps, out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    tag = sys.argv[2] if len(sys.argv) > 2 else "r04"
    torch.set_num_threads(1)
    lib = _lib(256)
    mids, prog, start, so, go, rb, dv, df = _inputs(lib, n)
    term = np.full(24, 0.25, np.float32)
    ids = np.arange(24, dtype=np.int64)
    ref_s, ref_reps, ref = _time(lambda: G._compose_step(lib, mids, prog, start, so, go, rb, dv, df, term, ids, False))
    olib = O.MotionLib(lib.gts.numpy(), lib.grs.numpy(), lib.lrs.numpy(), lib.gvs.numpy(), lib.gavs.numpy(),
                       lib.dvs.numpy(), lib._motion_num_frames.numpy().astype(np.int64), lib._motion_fps.numpy())
    port_s, port_reps, port = _time(lambda: O.env_step(olib, mids, prog, start, so, go, rb, dv, df))
    np.testing.assert_allclose(port["obs"], ref["obs"], atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(port["rew"], ref["rew"], atol=1e-5, rtol=1e-5)
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(line.split(":", 1)[1].strip() for line in f if line.startswith("model name"))
    except (OSError, StopIteration):
        pass
    res = {"num_envs": n, "threads": 1, "host_cpu_model": cpu, "host": platform.node(),
           "reference_env_steps_per_s": n / ref_s, "reference_reps": ref_reps,
           "port_env_steps_per_s": n / port_s, "port_reps": port_reps,
           "port_over_reference": ref_s / port_s,
           "what": "post-physics env step (motion state x2 + reward + reset + obs) on the same inputs; reference = "
                   "its own torch-CPU functions composed as tests/golden/make_golden.py _compose_step, port = "
                   "oracle/phc_oracle.env_step (bench.py cpu_baseline's kind 'port'); obs / reward agree to 1e-5"}
    out = os.path.join(ROOT, "profiles", f"{tag}_ref_vs_port_cpu.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
