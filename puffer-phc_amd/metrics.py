"""Imitation metrics of the eval path.

The reference calls `smpl_sim.smpllib.smpl_eval.compute_metrics_lite` (scripts/train.py:197-198),
an un-vendored dependency (smpl_sim, not in /root/reference).  This restates its published
algorithm: per motion, global MPJPE, root-relative MPJPE, Procrustes-aligned MPJPE (the
VideoPose3D p_mpjpe) and the VIBE velocity / acceleration errors, all in millimetres, one
value per frame.  Parity unpinned: no fixture of smpl_sim's output exists in the reference.
"""

from collections import defaultdict

import numpy as np


def compute_error_vel(joints_gt, joints_pred):
    """Mean over joints of ||Δpred - Δgt|| per frame pair ([T, J, 3] -> [T-1])."""
    vel_gt = joints_gt[1:] - joints_gt[:-1]
    vel_pred = joints_pred[1:] - joints_pred[:-1]
    return np.mean(np.linalg.norm(vel_pred - vel_gt, axis=2), axis=1)


def compute_error_accel(joints_gt, joints_pred):
    """Mean over joints of the second-difference error ([T, J, 3] -> [T-2])."""
    accel_gt = joints_gt[:-2] - 2 * joints_gt[1:-1] + joints_gt[2:]
    accel_pred = joints_pred[:-2] - 2 * joints_pred[1:-1] + joints_pred[2:]
    return np.mean(np.linalg.norm(accel_pred - accel_gt, axis=2), axis=1)


def p_mpjpe(predicted, target):
    """Per-frame MPJPE after the optimal similarity transform (rotation, scale, translation)."""
    mu_x = np.mean(target, axis=1, keepdims=True)
    mu_y = np.mean(predicted, axis=1, keepdims=True)
    x0 = target - mu_x
    y0 = predicted - mu_y
    norm_x = np.sqrt(np.sum(x0 ** 2, axis=(1, 2), keepdims=True))
    norm_y = np.sqrt(np.sum(y0 ** 2, axis=(1, 2), keepdims=True))
    x0 = x0 / norm_x
    y0 = y0 / norm_y
    h = np.matmul(x0.transpose(0, 2, 1), y0)
    u, s, vt = np.linalg.svd(h)
    v = vt.transpose(0, 2, 1)
    r = np.matmul(v, u.transpose(0, 2, 1))
    sign_det = np.sign(np.expand_dims(np.linalg.det(r), axis=1))
    v[:, :, -1] *= sign_det
    s[:, -1] *= sign_det.flatten()
    r = np.matmul(v, u.transpose(0, 2, 1))
    tr = np.expand_dims(np.sum(s, axis=1, keepdims=True), axis=2)
    a = tr * norm_x / norm_y
    t = mu_x - a * np.matmul(mu_y, r)
    aligned = a * np.matmul(predicted, r) + t
    return np.mean(np.linalg.norm(aligned - target, axis=2), axis=1)


def compute_metrics_lite(pred_pos_all, gt_pos_all, root_idx=0, concatenate=True):
    """{mpjpe_g, mpjpe_l, mpjpe_pa, accel_dist, vel_dist} (mm) over lists of [T, J, 3] motions."""
    metrics = defaultdict(list)
    for pred, gt in zip(pred_pos_all, gt_pos_all):
        jp = np.asarray(pred, np.float64).copy()
        jg = np.asarray(gt, np.float64).copy()
        metrics["mpjpe_g"].append(np.linalg.norm(jg - jp, axis=2).mean(axis=-1) * 1000)
        metrics["vel_dist"].append(compute_error_vel(jp, jg) * 1000)
        metrics["accel_dist"].append(compute_error_accel(jp, jg) * 1000)
        jp = jp - jp[:, [root_idx]]
        jg = jg - jg[:, [root_idx]]
        metrics["mpjpe_pa"].append(p_mpjpe(jp, jg) * 1000)
        metrics["mpjpe_l"].append(np.linalg.norm(jp - jg, axis=2).mean(axis=-1) * 1000)
    if concatenate:
        metrics = {k: np.concatenate(v) for k, v in metrics.items()}
    return metrics
