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
