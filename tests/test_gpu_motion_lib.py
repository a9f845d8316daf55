"""R5 MotionLibSMPL.load_motions end to end (clip selection, crop, heading randomisation, FK and
velocities on the device, packing) vs the reference's own loader output (needs an MI355X).

tests/golden/motion_lib.npz holds the reference MotionLibSMPL.load_motions result for six
synthetic clips loaded into 8 envs (deterministic, start_idx 0) together with the input clips.
Tolerance: positions / velocities atol 2e-5 (float64 FK rounded to float32), rotations 1e-6,
scalars and indices exact.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _clips(g):
    n = int(g["num_input_motions"])
    out = {}
    for i in range(n):
        q, t = g[f"in_quat_{i}"], g[f"in_trans_{i}"]
        out[f"synth_{i:02d}"] = {"pose_quat_global": q, "root_trans_offset": torch.from_numpy(t),
                                 "pose_aa": np.zeros((q.shape[0], 72)), "fps": 30}
    return out


def _lib(clips, deterministic=True, max_length=300, num_envs=8, start_idx=0, random_sample=False):
    from types import SimpleNamespace

    from puffer_phc_amd.motion_lib import FixHeightMode, MotionLibSMPL
    from puffer_phc_amd.skeleton import SkeletonTree

    cfg = SimpleNamespace(motion_file=clips, device=DEV, fix_height=FixHeightMode.no_fix, min_length=-1,
                          max_length=max_length, im_eval=False, num_thread=1, smpl_type="smpl", step_dt=1 / 30,
                          is_deterministic=deterministic)
    lib = MotionLibSMPL(cfg)
    sk = SkeletonTree.smpl()
    lib.load_motions(skeleton_trees=[sk] * num_envs, gender_betas=torch.zeros(num_envs, 17),
                     limb_weights=torch.zeros(num_envs, 10), random_sample=random_sample, start_idx=start_idx)
    return lib


def test_load_motions_matches_reference_loader(golden):
    g = golden("motion_lib")
    lib = _lib(_clips(g))
    np.testing.assert_array_equal(lib._curr_motion_ids.cpu().numpy(), g["sample_idxes"])
    np.testing.assert_array_equal(lib.length_starts.cpu().numpy(), g["length_starts"])
    np.testing.assert_array_equal(lib._motion_num_frames.cpu().numpy(), g["motion_num_frames"])
    np.testing.assert_array_equal(lib._motion_lengths.cpu().numpy(), g["motion_lengths"])
    np.testing.assert_array_equal(lib._motion_dt.cpu().numpy(), g["motion_dt"])
    for k, tol in (("gts", 2e-5), ("gvs", 2e-5), ("gavs", 2e-5), ("dvs", 2e-5), ("grvs", 2e-5), ("gravs", 2e-5)):
        np.testing.assert_allclose(getattr(lib, k).cpu().numpy(), g[k], atol=tol, rtol=1e-5, err_msg=k)
    for k in ("grs", "lrs"):
        np.testing.assert_allclose(getattr(lib, k).cpu().numpy(), g[k], atol=1e-6, err_msg=k)


def test_load_motions_crop_and_sequential_sampling(golden):
    """max_length crop (deterministic: frames [0, max_length)) and start_idx wrap-around."""
    g = golden("motion_lib")
    full = _lib(_clips(g), num_envs=6)
    crop = _lib(_clips(g), max_length=40, num_envs=6, start_idx=2)
    ids = crop._curr_motion_ids.cpu().numpy()
    np.testing.assert_array_equal(ids, (np.arange(6) + 2) % 6)
    nf_full = full._motion_num_frames.cpu().numpy()
    nf_crop = crop._motion_num_frames.cpu().numpy()
    np.testing.assert_array_equal(nf_crop, np.where(nf_full[ids] < 40, nf_full[ids], 40))
    # the cropped clip's poses are the first 40 frames' poses of the full clip (grs = input quats)
    fs, cs = full.length_starts.cpu().numpy(), crop.length_starts.cpu().numpy()
    for j, m in enumerate(ids):
        n = nf_crop[j]
        np.testing.assert_allclose(crop.grs[cs[j]:cs[j] + n].cpu().numpy(), full.grs[fs[m]:fs[m] + n].cpu().numpy(),
                                   atol=1e-6)


def test_heading_randomisation_rotates_about_z(golden):
    """Non-deterministic loading rotates each clip by a random heading (motion_lib.py:790-800):
    positions and velocities are the deterministic ones rotated about z; heights unchanged."""
    g = golden("motion_lib")
    np.random.seed(3)
    base = _lib(_clips(g), num_envs=6)
    rnd = _lib(_clips(g), deterministic=False, num_envs=6, random_sample=False)
    fs = base.length_starts.cpu().numpy()
    nf = base._motion_num_frames.cpu().numpy()
    rs = rnd.length_starts.cpu().numpy()
    ids_r = rnd._curr_motion_ids.cpu().numpy()
    for j, m in enumerate(ids_r):
        n = nf[m]
        if n > 300:
            continue
        a = base.gts[fs[m]:fs[m] + n].cpu().numpy().astype(np.float64)
        b = rnd.gts[rs[j]:rs[j] + n].cpu().numpy().astype(np.float64)
        np.testing.assert_allclose(b[..., 2], a[..., 2], atol=2e-5)
        ax, ay, bx, by = a[..., 0], a[..., 1], b[..., 0], b[..., 1]
        th = np.arctan2((ax * by - ay * bx).sum(), (ax * bx + ay * by).sum())  # least-squares angle
        c, s = np.cos(th), np.sin(th)
        rot = np.stack([c * a[..., 0] - s * a[..., 1], s * a[..., 0] + c * a[..., 1]], -1)
        np.testing.assert_allclose(b[..., :2], rot, atol=1e-4)
