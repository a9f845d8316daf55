"""HumanoidPHC.resample_motions() at C3 scale (BASELINE C3: 4,096 envs over the 11,313-clip AMASS
train set; humanoid_phc.py:1361-1377 -> motion_lib.py:257-429): a synthetic pool of 11,313 in-memory
clips, resampled for 4,096 envs.  Checks that the sampled ids are torch.multinomial's draw from the
library's sampling distribution under the same seed, that the HBM clip pool's packed library (crops,
heading draws, FK, velocities) equals the per-clip loop's (PHC_MOTION_POOL=0) bit for bit, and prints
both reload times (profiles/r05_resample.log).  Needs an MI355X."""

import random
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CLIPS, ENVS = 11313, 4096


@pytest.fixture(scope="module")
def env():
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.synthetic import synthetic_clips

    # lengths 30..360 frames: about a third of the clips are longer than max_episode_length (300)
    # and get a random crop window
    q, t, counts, fps = synthetic_clips(CLIPS, 30, 360, seed=7, device=DEV)
    qh, th = q.float().cpu().numpy(), t.float().cpu().numpy()
    cnt = counts.cpu().numpy()
    fh = fps.cpu().numpy()
    del q, t
    ends = np.cumsum(cnt)
    clips = {}
    for i in range(CLIPS):
        s, e = ends[i] - cnt[i], ends[i]
        clips[f"synth_{i:05d}"] = {"pose_quat_global": qh[s:e], "root_trans_offset": torch.from_numpy(th[s:e]),
                                   "pose_aa": np.zeros((e - s, 72), np.float32), "fps": float(fh[i])}
    cfg = EnvConfig(num_envs=ENVS, device_id=0, seed=0)
    e = PHCPufferEnv(cfg, motion_data=clips)
    e.reset()
    return e


def _resample(henv, pool, seeds=(5, 6, 7)):
    from puffer_phc_amd import motion_lib as ML

    saved = ML.MOTION_POOL
    ML.MOTION_POOL = pool
    try:
        torch.manual_seed(seeds[0])
        random.seed(seeds[1])
        np.random.seed(seeds[2])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        henv.resample_motions()
        torch.cuda.synchronize()
        return time.perf_counter() - t0
    finally:
        ML.MOTION_POOL = saved


def test_resample_ids_and_pool_parity(env):
    h = env.env
    lib = h._motion_lib
    assert lib._num_unique_motions == CLIPS
    _resample(h, True)  # warm: builds the pool once (its build time is not a reload's)
    t_pool = _resample(h, True)
    ids = lib._curr_motion_ids.clone()
    frames, lrs, dvs = lib.packed.frames.clone(), lib.packed.local_rot.clone(), lib.packed.dof_vel.clone()
    nf = lib._motion_num_frames.clone()
    # the ids: torch.multinomial over the sampling distribution, the reference's draw
    # (motion_lib.py:305-308), from the same generator state
    torch.manual_seed(5)
    want = torch.multinomial(lib._sampling_prob, num_samples=ENVS, replacement=True).to(DEV)
    assert torch.equal(ids, want)
    assert int(nf.max()) <= h.cfg.max_episode_length and bool((nf >= 30).all())
    lens = lib._pool.lens[ids.cpu().numpy()]
    assert (lens > h.cfg.max_episode_length).any()  # crops happened
    # the per-clip loop (the reference's structure) gives the same library, bit for bit
    t_loop = _resample(h, False)
    assert torch.equal(lib._curr_motion_ids, ids)
    assert torch.equal(lib._motion_num_frames, nf)
    assert torch.equal(lib.packed.frames, frames)
    assert torch.equal(lib.packed.local_rot, lrs)
    assert torch.equal(lib.packed.dof_vel, dvs)
    assert bool(torch.isfinite(h.obs_buf).all())
    print(f"\nresample_motions {ENVS} envs from {CLIPS} clips ({int(nf.sum())} frames): "
          f"HBM pool {1e3 * t_pool:.1f} ms, per-clip loop {1e3 * t_loop:.1f} ms")


def test_resample_then_step(env):
    """The env steps on the resampled library (the packed descriptor the kernels read was replaced)."""
    _resample(env.env, True, seeds=(8, 9, 10))
    act = torch.zeros((ENVS, 69), device=DEV)
    for _ in range(3):
        env.step(act)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(env.env.obs_buf).all())
