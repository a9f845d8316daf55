"""CPU oracle for the PHC imitation hot path — TEST INFRASTRUCTURE ONLY.

This module restates, in numpy float32 (float64 where the reference computes in float64),
the arithmetic of the reference's hot path (SURVEY.md §8a rows R1–R22).  It is the checker
the HIP path is compared against.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import it; the product package never does, and the
product path fails loudly when its HIP library is missing instead of falling back here.

Parity pinning: every function is checked against golden vectors produced by running the
reference's own modules in the build container (tests/golden/make_golden.py →
tests/golden/*.npz, tested in tests/test_oracle_golden.py).  Rows whose reference code
cannot be imported here (R13 action→PD: needs isaacgym) are restated from source and are
"parity unpinned"; DESIGN.md lists them.

Operation order follows the reference expression by expression so float32 rounding stays
within a few ulps of torch-CPU (transcendentals differ by libm ulps only).  Citations are
`path:line` relative to the reference root.
"""

import numpy as np

F32 = np.float32
DT = F32(2 * (1.0 / 60.0))  # IsaacGymBase.dt, puffer_phc/envs/isaacgym_env.py:41

NUM_BODIES = 24
NUM_DOF = 69
SELF_OBS = 358
TASK_OBS = 576
OBS = SELF_OBS + TASK_OBS

BODY_NAMES = (
    "Pelvis", "L_Hip", "L_Knee", "L_Ankle", "L_Toe", "R_Hip", "R_Knee", "R_Ankle", "R_Toe",
    "Torso", "Spine", "Chest", "Neck", "Head", "L_Thorax", "L_Shoulder", "L_Elbow", "L_Wrist",
    "L_Hand", "R_Thorax", "R_Shoulder", "R_Elbow", "R_Wrist", "R_Hand",
)  # puffer_phc/body_sets.py:11-36
DOF_NAMES = BODY_NAMES[1:]
REMOVE_NAMES = ("L_Hand", "R_Hand", "L_Toe", "R_Toe")
KEY_BODIES = ("R_Ankle", "L_Ankle", "R_Wrist", "L_Wrist")
EVAL_BODIES = tuple(n for n in BODY_NAMES if n not in REMOVE_NAMES)

REWARD = dict(k_pos=100.0, k_rot=10.0, k_vel=0.1, k_ang_vel=0.1,
              w_pos=0.5, w_rot=0.3, w_vel=0.1, w_ang_vel=0.1)  # puffer_phc/config.py:23-36


def f32(x):
    return np.asarray(x, dtype=np.float32)


# ------------------------------------------------------------------ R1 quats --
def quat_mul(a, b):
    """8-multiply form, puffer_phc/torch_utils.py:55-75."""
    x1, y1, z1, w1 = a[..., 0], a[..., 1], a[..., 2], a[..., 3]
    x2, y2, z2, w2 = b[..., 0], b[..., 1], b[..., 2], b[..., 3]
    ww = (z1 + x1) * (x2 + y2)
    yy = (w1 - y1) * (w2 + z2)
    zz = (w1 + y1) * (w2 - z2)
    xx = ww + yy + zz
    qq = 0.5 * (xx + (z1 - x1) * (x2 - y2))
    w = qq - ww + (z1 - y1) * (y2 - z2)
    x = qq - xx + (x1 + w1) * (x2 + w2)
    y = qq - yy + (w1 - x1) * (y2 + z2)
    z = qq - zz + (z1 + y1) * (w2 - x2)
    return np.stack([x, y, z, w], -1)


def quat_conjugate(a):
    """puffer_phc/torch_utils.py:79-82."""
    return np.concatenate([-a[..., :3], a[..., 3:]], -1)


def _norm(x):
    # torch.norm(p=2, dim=-1) over a short last dim: sequential sum of squares, then sqrt
    acc = x[..., 0] * x[..., 0]
    for i in range(1, x.shape[-1]):
        acc = acc + x[..., i] * x[..., i]
    return np.sqrt(acc)


def normalize(x, eps=1e-9):
    """puffer_phc/torch_utils.py:45-46."""
    return x / np.maximum(_norm(x), x.dtype.type(eps))[..., None]


def normalize_angle(x):
    """puffer_phc/torch_utils.py:50-51."""
    return np.arctan2(np.sin(x), np.cos(x))


def quat_unit(x):
    """puffer_phc/torch_utils.py:174-179."""
    return x / np.maximum(_norm(x), x.dtype.type(1e-9))[..., None]


def quat_pos(x):
    """puffer_phc/torch_utils.py:154-161: `(q[...,3:] < 0).float()` is float32 even for f64 q."""
    z = (x[..., 3:] < 0).astype(np.float32)
    return (1 - 2 * z) * x


def quat_normalize(q):
    """puffer_phc/torch_utils.py:190-195."""
    return quat_unit(quat_pos(q))


def quat_mul_norm(x, y):
    """puffer_phc/torch_utils.py:264-270."""
    return quat_normalize(quat_mul(x, y))


def quat_rotate(rot, vec):
    """Full-product rotation, puffer_phc/torch_utils.py:273-279."""
    other = np.concatenate([vec, np.zeros_like(vec[..., :1])], -1)
    return quat_mul(quat_mul(rot, other), quat_conjugate(rot))[..., :3]


def my_quat_rotate(q, v):
    """puffer_phc/torch_utils.py:283-291 (the bmm dot restated as a sequential dot)."""
    q_w = q[..., 3]
    q_vec = q[..., :3]
    a = v * (2.0 * (q_w * q_w) - 1.0)[..., None]
    cx = q_vec[..., 1] * v[..., 2] - q_vec[..., 2] * v[..., 1]
    cy = q_vec[..., 2] * v[..., 0] - q_vec[..., 0] * v[..., 2]
    cz = q_vec[..., 0] * v[..., 1] - q_vec[..., 1] * v[..., 0]
    b = np.stack([cx, cy, cz], -1) * q_w[..., None] * 2.0
    dot = q_vec[..., 0] * v[..., 0] + q_vec[..., 1] * v[..., 1] + q_vec[..., 2] * v[..., 2]
    c = q_vec * dot[..., None] * 2.0
    return a + b + c


def quat_to_tan_norm(q):
    """puffer_phc/torch_utils.py:294-307."""
    ref_tan = np.zeros_like(q[..., 0:3])
    ref_tan[..., 0] = 1
    ref_norm = np.zeros_like(q[..., 0:3])
    ref_norm[..., -1] = 1
    return np.concatenate([my_quat_rotate(q, ref_tan), my_quat_rotate(q, ref_norm)], -1)


def quat_to_angle_axis(q):
    """puffer_phc/torch_utils.py:86-106 (NaN lanes are masked exactly as torch.where does)."""
    with np.errstate(invalid="ignore", divide="ignore"):
        w = q[..., 3]
        sin_theta = np.sqrt(1 - w * w)
        angle = 2 * np.arccos(w)
        angle = normalize_angle(angle)
        axis = q[..., 0:3] / sin_theta[..., None]
    mask = np.abs(sin_theta) > 1e-5
    default = np.zeros_like(axis)
    default[..., -1] = 1
    angle = np.where(mask, angle, np.zeros_like(angle))
    axis = np.where(mask[..., None], axis, default)
    return angle, axis


def quat_to_exp_map(q):
    """puffer_phc/torch_utils.py:135-150."""
    angle, axis = quat_to_angle_axis(q)
    return angle[..., None] * axis


def slerp(q0, q1, t):
    """puffer_phc/torch_utils.py:110-131; `t` broadcasts against [..., 1]."""
    cos_half = q0[..., 0] * q1[..., 0] + q0[..., 1] * q1[..., 1] + q0[..., 2] * q1[..., 2] + q0[..., 3] * q1[..., 3]
    neg = cos_half < 0
    q1 = np.where(neg[..., None], -q1, q1)
    cos_half = np.abs(cos_half)[..., None]
    with np.errstate(invalid="ignore", divide="ignore"):
        half_theta = np.arccos(cos_half)
        sin_half = np.sqrt(1.0 - cos_half * cos_half)
        ratio_a = np.sin((1 - t) * half_theta) / sin_half
        ratio_b = np.sin(t * half_theta) / sin_half
        new_q = ratio_a * q0 + ratio_b * q1
    new_q = np.where(np.abs(sin_half) < 0.001, 0.5 * q0 + 0.5 * q1, new_q)
    new_q = np.where(np.abs(cos_half) >= 1, q0, new_q)
    return new_q


def quat_from_angle_axis(angle, axis):
    """puffer_phc/torch_utils.py:354-358."""
    theta = (angle / 2)[..., None]
    xyz = normalize(axis) * np.sin(theta)
    w = np.cos(theta)
    return quat_unit(np.concatenate([xyz, w], -1))


def exp_map_to_quat(exp_map):
    """puffer_phc/torch_utils.py:334-365."""
    with np.errstate(invalid="ignore", divide="ignore"):
        angle = _norm(exp_map)
        axis = exp_map / angle[..., None]
    angle = normalize_angle(angle)
    default = np.zeros_like(exp_map)
    default[..., -1] = 1
    mask = np.abs(angle) > 1e-5
    angle = np.where(mask, angle, np.zeros_like(angle))
    axis = np.where(mask[..., None], axis, default)
    return quat_from_angle_axis(angle, axis)


def calc_heading(q):
    """puffer_phc/torch_utils.py:369-381."""
    ref = np.zeros_like(q[..., 0:3])
    ref[..., 0] = 1
    rot_dir = my_quat_rotate(q, ref)
    return np.arctan2(rot_dir[..., 1], rot_dir[..., 0])


def _z_axis_like(q):
    axis = np.zeros_like(q[..., 0:3])
    axis[..., 2] = 1
    return axis


def calc_heading_quat(q):
    """puffer_phc/torch_utils.py:384-394."""
    return quat_from_angle_axis(calc_heading(q), _z_axis_like(q))


def calc_heading_quat_inv(q):
    """puffer_phc/torch_utils.py:397-408."""
    return quat_from_angle_axis(-calc_heading(q), _z_axis_like(q))


def quat_angle_axis(x):
    """puffer_phc/torch_utils.py:219-228 (angle in [0, pi], axis normalised)."""
    s = 2 * (x[..., 3] ** 2) - 1
    angle = np.arccos(np.clip(s, -1, 1))
    axis = x[..., :3] / np.maximum(_norm(x[..., :3]), x.dtype.type(1e-9))[..., None]
    return angle, axis


# ------------------------------------------------------ R2 skeleton (MJCF) --
def skeleton_from_mjcf(path):
    """DFS over <body> elements, puffer_phc/poselib_skeleton.py:275-320."""
    import xml.etree.ElementTree as ET

    root = ET.parse(path).getroot().find("worldbody").find("body")
    names, parents, offsets = [], [], []

    def visit(node, parent):
        idx = len(names)
        names.append(node.attrib.get("name"))
        parents.append(parent)
        offsets.append(np.array(node.attrib.get("pos", "0 0 0").split(), dtype=np.float64))
        for child in node.findall("body"):
            visit(child, idx)

    visit(root, -1)
    return names, np.array(parents, np.int64), np.stack(offsets).astype(np.float32)


# ------------------------------------------------- R3/R4 FK + velocities --
def gaussian_weights(sigma=2.0, truncate=4.0):
    """scipy.ndimage.gaussian_filter1d kernel (order 0), as used by
    puffer_phc/poselib_skeleton.py:1232-1249."""
    radius = int(truncate * float(sigma) + 0.5)
    x = np.arange(-radius, radius + 1)
    phi = np.exp((-0.5 / (sigma * sigma) * x) * x, dtype=np.float64)
    phi /= phi.sum()
    return phi


def gaussian_filter_time(x, sigma=2.0):
    """Correlate along axis 0 with mode='nearest', accumulating in float64 in scipy's
    symmetric order (far pairs first): w0*x[t] + sum_{j=r..1} (x[t-j] + x[t+j]) * w_j; cast
    back to x.dtype.  Bit-exact with scipy.ndimage.gaussian_filter1d."""
    w = gaussian_weights(sigma)
    r = (len(w) - 1) // 2
    T = x.shape[0]
    xd = x.astype(np.float64)
    idx = np.arange(T)
    out = xd * w[r]
    for j in range(r, 0, -1):
        out = out + (xd[np.maximum(idx - j, 0)] + xd[np.minimum(idx + j, T - 1)]) * w[r - j]
    return out.astype(x.dtype)


def fk_motion(parents, local_translation, quat_global, root_trans, fps=30):
    """One motion's load-time FK + velocities.
    local rotation:  puffer_phc/poselib_skeleton.py:574-593 (float64, stored float32)
    local transl.:   puffer_phc/poselib_skeleton.py:605-619 (root row = root translation, float32)
    global FK:       puffer_phc/poselib_skeleton.py:518-539 with transform_mul
                     puffer_phc/torch_utils.py:322-330 (float32)
    lin. velocity:   puffer_phc/poselib_skeleton.py:1230-1238 (np.gradient / dt + gaussian)
    ang. velocity:   puffer_phc/poselib_skeleton.py:1240-1251 (float64)
    dof velocity:    puffer_phc/motion_lib.py:119-140
    Returns dict of float32 arrays gts [T,24,3], grs/lrs [T,24,4], gvs/gavs [T,24,3], dvs [T,23,3]."""
    q = np.asarray(quat_global, np.float64)
    T, J, _ = q.shape
    lrs = np.zeros((T, J, 4), np.float32)
    for j in range(J):
        p = parents[j]
        if p == -1:
            lrs[:, j] = q[:, j]
        else:
            lrs[:, j] = quat_mul_norm(quat_conjugate(q[:, p]), q[:, j])
    lt = np.broadcast_to(np.asarray(local_translation, np.float32), (T, J, 3)).copy()
    lt[:, 0] = np.asarray(root_trans, np.float64)
    g_rot = [None] * J
    g_pos = [None] * J
    for j in range(J):
        p = parents[j]
        if p == -1:
            g_rot[j], g_pos[j] = lrs[:, j], lt[:, j]
        else:
            g_rot[j] = quat_mul_norm(g_rot[p], lrs[:, j])
            g_pos[j] = quat_rotate(g_rot[p], lt[:, j]) + g_pos[p]
    gts = np.stack(g_pos, 1).astype(np.float32)
    dt = 1.0 / fps
    if T >= 2:
        grad = np.gradient(gts, axis=-3)
    else:
        grad = np.zeros_like(gts)
    gvs = gaussian_filter_time(grad / dt)
    diff = np.zeros((T, J, 4), np.float64)
    diff[..., 3] = 1.0
    diff[:-1] = quat_mul_norm(q[1:], quat_conjugate(q[:-1]))
    ang, axis = quat_angle_axis(diff)
    gav = axis * ang[..., None] / dt
    gavs = gaussian_filter_time(gav).astype(np.float32)
    # dof velocities from local rotations (float32), root dropped, last frame duplicated
    dvs = np.zeros((T, J - 1, 3), np.float32)
    if T >= 2:
        d = quat_mul(quat_conjugate(lrs[:-1]), lrs[1:])
        a, ax = quat_to_angle_axis(d)
        dv = ax * a[..., None] / F32(dt)
        dvs[:-1] = dv[:, 1:]
        dvs[-1] = dvs[-2]
    return dict(gts=gts, grs=q.astype(np.float32), lrs=lrs, gvs=gvs.astype(np.float32), gavs=gavs, dvs=dvs)


# --------------------------------------------------- R5/R6/R7 motion state --
class MotionLib:
    """Flat packed motion tensors, puffer_phc/motion_lib.py:396-419."""

    def __init__(self, gts, grs, lrs, gvs, gavs, dvs, num_frames, fps):
        self.gts, self.grs, self.lrs = f32(gts), f32(grs), f32(lrs)
        self.gvs, self.gavs, self.dvs = f32(gvs), f32(gavs), f32(dvs)
        self.num_frames = np.asarray(num_frames, np.int64)
        fps = np.asarray(fps, np.float64)
        self.motion_dt = (1.0 / fps).astype(np.float32)
        self.motion_lengths = (1.0 / fps * (self.num_frames - 1)).astype(np.float32)
        ls = np.roll(self.num_frames, 1)
        ls[0] = 0
        self.length_starts = np.cumsum(ls)


def calc_frame_blend(time, length, num_frames, dt):
    """puffer_phc/motion_lib.py:655-665 (bit-exact frame indices)."""
    time = f32(time).copy()
    phase = time / length
    phase = np.clip(phase, F32(0.0), F32(1.0))
    time[time < 0] = 0
    f0 = (phase * (num_frames - 1).astype(np.float32)).astype(np.int64)
    f1 = np.minimum(f0 + 1, num_frames - 1)
    blend = np.clip((time - f0.astype(np.float32) * dt) / dt, F32(0.0), F32(1.0))
    return f0, f1, blend


def motion_state(lib, motion_ids, motion_times, offset=None):
    """get_motion_state, puffer_phc/motion_lib.py:549-626 (+ :670-673 dof_pos)."""
    ids = np.asarray(motion_ids, np.int64)
    f0, f1, blend = calc_frame_blend(motion_times, lib.motion_lengths[ids], lib.num_frames[ids], lib.motion_dt[ids])
    f0l = f0 + lib.length_starts[ids]
    f1l = f1 + lib.length_starts[ids]
    b = blend[:, None, None]
    one_b = F32(1.0) - b

    def lerp(a):
        return one_b * a[f0l] + b * a[f1l]

    rg_pos = lerp(lib.gts)
    if offset is not None:
        rg_pos = rg_pos + f32(offset)[:, None, :]
    body_vel = lerp(lib.gvs)
    body_ang_vel = lerp(lib.gavs)
    dof_vel = lerp(lib.dvs)
    local_rot = slerp(lib.lrs[f0l], lib.lrs[f1l], b)
    dof_pos = quat_to_exp_map(local_rot[:, 1:]).reshape(len(ids), -1)
    rb_rot = slerp(lib.grs[f0l], lib.grs[f1l], b)
    return dict(
        root_pos=rg_pos[:, 0].copy(), root_rot=rb_rot[:, 0].copy(), dof_pos=dof_pos,
        root_vel=body_vel[:, 0].copy(), root_ang_vel=body_ang_vel[:, 0].copy(),
        dof_vel=dof_vel.reshape(len(ids), -1), rg_pos=rg_pos, rb_rot=rb_rot,
        body_vel=body_vel, body_ang_vel=body_ang_vel, frame_idx0=f0, frame_idx1=f1, blend=blend,
    )


def sample_time_interval(phase, motion_len):
    """puffer_phc/motion_lib.py:526-535 given the uniform draw `phase`."""
    curr = F32(1 / 30)
    return ((f32(phase) * f32(motion_len)) / curr).astype(np.int64).astype(np.float32) * curr


# ---------------------------------------------------------- R9/R10 obs ------
def humanoid_obs(body_pos, body_rot, body_vel, body_ang_vel):
    """compute_humanoid_observations_smpl_max, puffer_phc/envs/common.py:23-103 with
    local_root_obs=True, root_height_obs=True, upright=True (humanoid_phc.py:990-1002)."""
    n = body_pos.shape[0]
    root_pos = body_pos[:, 0]
    root_rot = body_rot[:, 0]
    root_h = root_pos[:, 2:3]
    hinv = np.repeat(calc_heading_quat_inv(root_rot)[:, None], NUM_BODIES, 1)
    local_pos = my_quat_rotate(hinv, body_pos - root_pos[:, None]).reshape(n, -1)[:, 3:]
    local_rot = quat_to_tan_norm(quat_mul(hinv, body_rot)).reshape(n, -1)
    local_vel = my_quat_rotate(hinv, body_vel).reshape(n, -1)
    local_ang = my_quat_rotate(hinv, body_ang_vel).reshape(n, -1)
    return np.concatenate([root_h, local_pos, local_rot, local_vel, local_ang], -1)


def imitation_obs_v6(root_pos, root_rot, body_pos, body_rot, body_vel, body_ang_vel,
                     ref_pos, ref_rot, ref_vel, ref_ang_vel):
    """compute_imitation_observations_v6, puffer_phc/envs/common.py:107-176, time_steps=1,
    upright=True."""
    n = body_pos.shape[0]
    hinv = np.repeat(calc_heading_quat_inv(root_rot)[:, None], NUM_BODIES, 1)
    hrot = np.repeat(calc_heading_quat(root_rot)[:, None], NUM_BODIES, 1)
    d_pos = my_quat_rotate(hinv, ref_pos - body_pos)
    d_rot = quat_mul(quat_mul(hinv, quat_mul(ref_rot, quat_conjugate(body_rot))), hrot)
    d_vel = my_quat_rotate(hinv, ref_vel - body_vel)
    d_ang = my_quat_rotate(hinv, ref_ang_vel - body_ang_vel)
    l_ref_pos = my_quat_rotate(hinv, ref_pos - root_pos[:, None])
    l_ref_rot = quat_to_tan_norm(quat_mul(hinv, ref_rot))
    return np.concatenate([
        d_pos.reshape(n, -1), quat_to_tan_norm(d_rot).reshape(n, -1), d_vel.reshape(n, -1),
        d_ang.reshape(n, -1), l_ref_pos.reshape(n, -1), l_ref_rot.reshape(n, -1)], -1)


# ---------------------------------------------------------- R11/R12 ---------
def _mean_last(x):
    acc = x[..., 0].copy()
    for i in range(1, x.shape[-1]):
        acc = acc + x[..., i]
    return acc / F32(x.shape[-1])


def imitation_reward(body_pos, body_rot, body_vel, body_ang_vel, ref_pos, ref_rot, ref_vel, ref_ang_vel,
                     spec=REWARD):
    """compute_imitation_reward, puffer_phc/envs/common.py:271-322."""
    r_pos = np.exp(F32(-spec["k_pos"]) * _mean_last(_mean_last((ref_pos - body_pos) ** 2)))
    ang = quat_to_angle_axis(quat_mul(ref_rot, quat_conjugate(body_rot)))[0]
    r_rot = np.exp(F32(-spec["k_rot"]) * _mean_last(ang ** 2))
    r_vel = np.exp(F32(-spec["k_vel"]) * _mean_last(_mean_last((ref_vel - body_vel) ** 2)))
    r_ang = np.exp(F32(-spec["k_ang_vel"]) * _mean_last(_mean_last((ref_ang_vel - body_ang_vel) ** 2)))
    rew = F32(spec["w_pos"]) * r_pos + F32(spec["w_rot"]) * r_rot + F32(spec["w_vel"]) * r_vel + \
        F32(spec["w_ang_vel"]) * r_ang
    return rew, np.stack([r_pos, r_rot, r_vel, r_ang], -1)


def power_reward(dof_force, dof_vel, progress, coef=0.0005):
    """puffer_phc/envs/humanoid_phc.py:1295-1303."""
    power = np.abs(f32(dof_force) * f32(dof_vel)).sum(-1, dtype=np.float32)
    pr = F32(-coef) * power
    pr[np.asarray(progress) <= 3] = 0
    return pr


def im_reset(progress, body_pos, ref_pos, pass_time, term_dist, reset_body_ids, use_mean,
             enable_early_termination=True):
    """compute_humanoid_im_reset, puffer_phc/envs/common.py:326-364 + humanoid_phc.py:1311-1333.
    Returns (reset, terminate, per-body distances)."""
    ids = np.asarray(reset_body_ids)
    dist = _norm(body_pos[:, ids] - ref_pos[:, ids])
    td = f32(term_dist)[ids]
    terminated = np.zeros(len(progress), bool)
    if enable_early_termination:
        if use_mean:
            fallen = _mean_last(dist) > td[0]
        else:
            fallen = np.any(dist > td, -1)
        fallen = fallen & (np.asarray(progress) > 1)
        terminated = fallen
    reset = np.where(pass_time, True, terminated)
    return reset, terminated, dist


# --------------------------------------------------- R14 step composition ---
def env_step(lib, motion_ids, progress, start, start_offset, global_offset, rb_state, dof_vel, dof_force,
             term_dist=None, reset_body_ids=None, use_mean=False):
    """Post-physics part of HumanoidPHC.step (puffer_phc/envs/humanoid_phc.py:136-146):
    reward(t) -> reset(t) -> obs(t+dt), t = progress*dt + start + offset in float32.
    `progress` is the value after `progress_buf += 1`.  rb_state is [N,24,13]."""
    if term_dist is None:
        term_dist = np.full(NUM_BODIES, 0.25, np.float32)
    if reset_body_ids is None:
        reset_body_ids = np.arange(NUM_BODIES)
    rb = f32(rb_state)
    bp, br, bv, bav = rb[..., 0:3], rb[..., 3:7], rb[..., 7:10], rb[..., 10:13]
    prog = np.asarray(progress, np.int16)
    t = prog.astype(np.float32) * DT + f32(start) + f32(start_offset)
    ref = motion_state(lib, motion_ids, t, global_offset)
    rew, raw = imitation_reward(bp, br, bv, bav, ref["rg_pos"], ref["rb_rot"], ref["body_vel"], ref["body_ang_vel"])
    pr = power_reward(dof_force, dof_vel, prog)
    rew = rew + pr
    reward_raw = np.concatenate([raw, pr[:, None]], -1)
    pass_time = t >= lib.motion_lengths[np.asarray(motion_ids)]
    reset, term, dist = im_reset(prog, bp, ref["rg_pos"], pass_time, term_dist, reset_body_ids, use_mean)
    t1 = (prog.astype(np.float32) + F32(1)) * DT + f32(start) + f32(start_offset)
    ref1 = motion_state(lib, motion_ids, t1, global_offset)
    obs = np.concatenate([
        humanoid_obs(bp, br, bv, bav),
        imitation_obs_v6(bp[:, 0], br[:, 0], bp, br, bv, bav, ref1["rg_pos"], ref1["rb_rot"],
                         ref1["body_vel"], ref1["body_ang_vel"])], -1)
    return dict(rew=rew, reward_raw=reward_raw, reset=reset, terminate=term, obs=obs, time=t,
                time_next=t1, reset_dist=dist)


def reset_subset(lib, motion_ids, phase, global_offset_old):
    """Reset path for the envs in the subset (puffer_phc/envs/humanoid_phc.py:692-729, 843-873,
    899-929, 745-778, then _compute_observations(env_ids)).  Returns the new start times, the
    reference state written into the sim buffers and the subset's observation."""
    mids = np.asarray(motion_ids, np.int64)
    mt = sample_time_interval(phase, lib.motion_lengths[mids])
    ref = motion_state(lib, mids, mt, global_offset_old)
    rb = np.concatenate([ref["rg_pos"], ref["rb_rot"], ref["body_vel"], ref["body_ang_vel"]], -1)
    t1 = (F32(0) + F32(1)) * DT + mt + F32(0)
    ref1 = motion_state(lib, mids, t1, np.zeros((len(mids), 3), np.float32))
    bp, br, bv, bav = rb[..., 0:3], rb[..., 3:7], rb[..., 7:10], rb[..., 10:13]
    obs = np.concatenate([
        humanoid_obs(bp, br, bv, bav),
        imitation_obs_v6(bp[:, 0], br[:, 0], bp, br, bv, bav, ref1["rg_pos"], ref1["rb_rot"],
                         ref1["body_vel"], ref1["body_ang_vel"])], -1)
    return dict(motion_times=mt, ref=ref, rb_state=rb, obs=obs)


# --------------------------------------------------------------- R13 --------
def pd_action_scale():
    """_build_pd_action_offset_scale (puffer_phc/envs/humanoid_phc.py:385-456) for the SMPL
    MJCF (every 3-DoF joint limited to +-180 or +-720 deg): offset 0, scale min(1.2*max, pi)
    = pi, knee-y scale 5.  Parity unpinned (needs isaacgym's parsed limits)."""
    scale = np.full(NUM_DOF, np.float32(np.pi), np.float32)
    scale[DOF_NAMES.index("L_Knee") * 3 + 1] = 5
    scale[DOF_NAMES.index("R_Knee") * 3 + 1] = 5
    return np.zeros(NUM_DOF, np.float32), scale


FROZEN_DOFS = np.concatenate([np.arange(DOF_NAMES.index(n) * 3, DOF_NAMES.index(n) * 3 + 3)
                              for n in ("L_Hand", "R_Hand", "L_Toe", "R_Toe")])


def actions_to_pd(actions, clip=True):
    """puffer_phc/clean_pufferl/env.py:91-93 (np.clip only when cfg.clip_actions) + humanoid_phc.py:106-128,
    1216-1226."""
    a = np.clip(f32(actions), -1, 1) if clip else f32(actions)
    off, scale = pd_action_scale()
    pd = off + scale * a
    pd[:, FROZEN_DOFS] = 0
    return pd


# --------------------------------------------------------------- R16 AMP ----
def dof_subset():
    idx = [np.arange(i * 3, i * 3 + 3) for i, n in enumerate(DOF_NAMES) if n not in REMOVE_NAMES]
    return np.concatenate(idx)


def amp_obs(root_pos, root_rot, root_vel, root_ang_vel, dof_pos, dof_vel, key_body_pos):
    """build_amp_observations_smpl, puffer_phc/envs/common.py:180-267 (local root obs,
    root height, dof subset, no shape/limb params, upright)."""
    n = root_pos.shape[0]
    hinv = calc_heading_quat_inv(root_rot)
    root_rot_obs = quat_to_tan_norm(quat_mul(hinv, root_rot))
    lv = my_quat_rotate(hinv, root_vel)
    lav = my_quat_rotate(hinv, root_ang_vel)
    kb = my_quat_rotate(np.repeat(hinv[:, None], key_body_pos.shape[1], 1),
                        key_body_pos - root_pos[:, None]).reshape(n, -1)
    sub = dof_subset()
    dof_obs = quat_to_tan_norm(exp_map_to_quat(dof_pos[:, sub].reshape(-1, 3))).reshape(n, -1)
    return np.concatenate([root_pos[:, 2:3], root_rot_obs, lv, lav, dof_obs, dof_vel[:, sub], kb], -1)


KEY_BODY_IDS = np.array([BODY_NAMES.index(n) for n in KEY_BODIES])


def amp_obs_from_sim(rb_state, dof_pos, dof_vel):
    """_compute_amp_observations (humanoid_phc.py:1123-1160) from the sim buffers."""
    rb = f32(rb_state)
    return amp_obs(rb[:, 0, 0:3], rb[:, 0, 3:7], rb[:, 0, 7:10], rb[:, 0, 10:13], f32(dof_pos), f32(dof_vel),
                   rb[:, KEY_BODY_IDS, 0:3])


def amp_obs_from_motion(lib, motion_ids, motion_times):
    """_get_amp_obs (humanoid_phc.py:819-836): reference state without offset."""
    ms = motion_state(lib, motion_ids, motion_times)
    return amp_obs(ms["root_pos"], ms["root_rot"], ms["root_vel"], ms["root_ang_vel"], ms["dof_pos"],
                   ms["dof_vel"], ms["rg_pos"][:, KEY_BODY_IDS])


def amp_update(amp, demo, lib, rb_state, dof_pos, dof_vel, progress, motion_ids, start, dt, init_only):
    """AMP history update in place on amp / demo [N, S, 196].

    init_only=False: HumanoidPHC.step's _update_hist_amp_obs + _compute_amp_observations
    (humanoid_phc.py:154-157, 1339-1348) for every env, followed by the reset of the envs that
    were just re-initialised (progress == 0) — whose _init_amp_obs (:789-836) overwrites all
    frames: frame 0 from the sim state, frame k from the motion library at start - k*dt, and
    copies the window into amp_obs_demo.  init_only=True: only the reset part (reset(env_ids))."""
    n, steps = amp.shape[0], amp.shape[1]
    init = np.asarray(progress) == 0
    if not init_only:
        amp[:, 1:] = amp[:, :-1].copy()
        amp[:, 0] = amp_obs_from_sim(rb_state, dof_pos, dof_vel)
    ids = np.nonzero(init)[0]
    if len(ids):
        amp[ids, 0] = amp_obs_from_sim(rb_state[ids], dof_pos[ids], dof_vel[ids])
        ks = np.arange(1, steps)
        times = f32(start)[ids][:, None] + (-F32(dt)) * ks.astype(np.float32)[None, :]
        mids = np.repeat(np.asarray(motion_ids)[ids], steps - 1)
        hist = amp_obs_from_motion(lib, mids, times.reshape(-1))
        amp[ids, 1:] = hist.reshape(len(ids), steps - 1, -1)
        demo[ids] = amp[ids]
    return amp, demo


# --------------------------------------------------------------- R17 RMS ----
def rms_update(mean, var, count, x):
    """RunningNorm.update, puffer_phc/policies/running_norm.py:22-34 (float64 batch stats)."""
    xd = np.asarray(x, np.float64)
    bm = xd.mean(0, keepdims=True).astype(np.float32)
    bv = xd.var(0, keepdims=True).astype(np.float32)
    w = F32(1) / f32(count)
    return mean * (1 - w) + bm * w, var * (1 - w) + bv * w, count + 1


def rms_normalize(x, mean, var, eps=1e-5, clip=10.0):
    """RunningNorm.forward, puffer_phc/policies/running_norm.py:15-20."""
    return np.clip((f32(x) - mean) / np.sqrt(var + F32(eps)), -clip, clip)


# --------------------------------------------------------------- R20 GAE ----
def compute_gae(dones, values, rewards, gamma, lam):
    """Backward recurrence over the flat buffer, puffer_phc/c_gae.pyx:11-32 (float32)."""
    d, v, r = f32(dones), f32(values), f32(rewards)
    n = len(r)
    adv = np.zeros(n, np.float32)
    g, l = F32(gamma), F32(lam)
    last = F32(0)
    for t in range(n - 1):
        cur = n - 2 - t
        nxt = n - 1 - t
        nnt = F32(1) - d[nxt]
        delta = r[nxt] + g * v[nxt] * nnt - v[cur]
        last = delta + g * l * nnt * last
        adv[cur] = last
    return adv
