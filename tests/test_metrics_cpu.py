"""Eval metrics (metrics.py: the published compute_metrics_lite algorithm of smpl_sim, which the
reference calls at scripts/train.py:197-198).  Parity unpinned (smpl_sim is not in the
reference); checked here against closed-form answers."""

import numpy as np

from puffer_phc_amd.metrics import compute_error_accel, compute_error_vel, compute_metrics_lite, p_mpjpe


def _motion(rng, t=30, j=24):
    return rng.normal(size=(t, j, 3))


def test_identical_motion_has_zero_error():
    rng = np.random.default_rng(0)
    gt = _motion(rng)
    m = compute_metrics_lite([gt], [gt.copy()])
    for k, v in m.items():
        np.testing.assert_allclose(v, 0.0, atol=1e-9, err_msg=k)
    assert m["mpjpe_g"].shape == (30,) and m["vel_dist"].shape == (29,) and m["accel_dist"].shape == (28,)


def test_global_offset_counts_only_in_global_mpjpe():
    rng = np.random.default_rng(1)
    gt = _motion(rng)
    off = np.array([0.03, -0.04, 0.0])  # 50 mm
    m = compute_metrics_lite([gt + off], [gt])
    np.testing.assert_allclose(m["mpjpe_g"], 50.0, rtol=1e-9)
    for k in ("mpjpe_l", "mpjpe_pa", "vel_dist", "accel_dist"):
        np.testing.assert_allclose(m[k], 0.0, atol=1e-9, err_msg=k)


def test_procrustes_removes_rotation_and_scale():
    rng = np.random.default_rng(2)
    gt = _motion(rng, t=5)
    th = 0.7
    r = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]])
    pred = 1.3 * gt @ r.T + np.array([0.1, 0.2, 0.3])
    np.testing.assert_allclose(p_mpjpe(pred, gt), 0.0, atol=1e-9)
    assert np.all(np.linalg.norm(pred - gt, axis=2).mean(1) > 0.1)


def test_velocity_and_acceleration_errors():
    t = np.arange(10, dtype=np.float64)
    gt = np.zeros((10, 2, 3))
    pred = np.zeros((10, 2, 3))
    pred[:, :, 0] = 0.5 * t[:, None]          # constant velocity 0.5 / frame
    np.testing.assert_allclose(compute_error_vel(gt, pred), 0.5)
    np.testing.assert_allclose(compute_error_accel(gt, pred), 0.0, atol=1e-12)
    pred[:, :, 1] = 0.1 * t[:, None] ** 2     # constant acceleration 0.2 / frame^2
    np.testing.assert_allclose(compute_error_accel(gt, pred), 0.2, rtol=1e-9)


def test_hand_worked_vectors():
    """compute_metrics_lite's published definitions on a 3-frame, 2-joint motion worked out by hand
    (metres in, millimetres out; smpl_sim.smpllib.smpl_eval, called at scripts/train.py:197-198):
      gt   : joint 0 at the origin, joint 1 at (1, 0, 0) m in every frame;
      pred : joint 1 displaced by (0, 0.003, 0.004) m (5 mm) in frame 1 only.
    mpjpe_g per frame = mean over joints = (0, 2.5, 0) mm; root-relative (joint 0 is the root and
    undisplaced) the same; velocity error: frames 0->1 and 1->2 each move joint 1 by 5 mm ->
    mean over joints 2.5 mm; acceleration error: joint 1's second difference 2 x 5 mm = 10 mm ->
    mean over joints 5 mm."""
    gt = np.zeros((3, 2, 3))
    gt[:, 1, 0] = 1.0
    pred = gt.copy()
    pred[1, 1] += [0.0, 0.003, 0.004]
    m = compute_metrics_lite([pred], [gt])
    np.testing.assert_allclose(m["mpjpe_g"], [0.0, 2.5, 0.0], atol=1e-9)
    np.testing.assert_allclose(m["mpjpe_l"], [0.0, 2.5, 0.0], atol=1e-9)
    np.testing.assert_allclose(m["vel_dist"], [2.5, 2.5], atol=1e-9)
    np.testing.assert_allclose(m["accel_dist"], [5.0], atol=1e-9)
    # frames 0 and 2 are exact, so their Procrustes error is 0; frame 1 is a non-similar
    # distortion of a 2-point set, which a similarity transform of 2 points always absorbs
    np.testing.assert_allclose(m["mpjpe_pa"], 0.0, atol=1e-9)


def test_procrustes_does_not_reflect():
    """The published p_mpjpe corrects the SVD's rotation to det = +1 (sign_det): a mirrored pose
    is not aligned away (a reflection would give 0)."""
    rng = np.random.default_rng(3)
    gt = rng.normal(size=(4, 24, 3))
    mirrored = gt * np.array([-1.0, 1.0, 1.0])
    assert np.all(p_mpjpe(mirrored, gt) > 0.05)
    # a proper rotation of the same pose is aligned away
    c, s = np.cos(0.4), np.sin(0.4)
    rot = gt @ np.array([[1, 0, 0], [0, c, -s], [0, s, c]]).T
    np.testing.assert_allclose(p_mpjpe(rot, gt), 0.0, atol=1e-9)
