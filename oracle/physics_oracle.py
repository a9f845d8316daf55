"""CPU oracle for the articulated-body physics step — TEST INFRASTRUCTURE ONLY.

What it replaces: the reference's `gym.simulate(sim)` x `control_freq_inv` (puffer_phc/envs/
humanoid_phc.py:129-134) — PhysX articulations (TGS, 4 position iterations, 0 velocity iterations,
puffer_phc/envs/isaacgym_env.py:6-35) driving the SMPL humanoid (assets/smpl_humanoid.xml) with
position drives at the MJCF gains x kp_scale / kd_scale (humanoid_phc.py:274-281) on a ground plane
with friction 1, restitution 0 (:255-262).  PhysX is a closed binary and not in this image, so
**parity with PhysX is unpinned**: this module restates the algorithm the HIP kernel
(puffer-phc_amd/csrc/phc_physics.hip) implements — Featherstone's articulated-body algorithm over
the 24-body tree with a 6-DoF floating root and 23 three-DoF ball joints, implicit joint-space PD,
penalty ground contact with capped viscous friction, penalty self-collision between the filtered
capsule pairs, angular damping and the angular-velocity cap, semi-implicit Euler substeps — in float64 with
generic 6x6 spatial matrices, as the checker the kernel is compared against.  It is pinned by
physical laws instead (tests/test_physics_oracle.py): closed-form free fall, conservation of
spatial momentum and energy of the unforced free-floating tree, the PD limit, a standing humanoid.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module.

Conventions (shared with the kernel): quaternions x, y, z, w; body frames at the MJCF body origins;
spatial vectors [angular; linear] in body coordinates; a joint's generalized velocity is the child's
angular velocity relative to its parent in child coordinates; dof_pos is the exp map (rotation
vector) of the joint rotation; rigid-body records hold the body origin's position and the centre
of mass's linear velocity (PhysX's convention).
"""

import json
import os

import numpy as np

NUM_BODIES = 24
NUM_DOF = 69
MODEL_JSON = os.path.join(os.path.dirname(__file__), "..", "puffer-phc_amd", "assets", "smpl_body_model.json")

DEFAULT_PARAMS = dict(sim_dt=1.0 / 60.0, control_freq_inv=2, substeps=8, kp_scale=1.0, kd_scale=1.0,
                      contact_stiffness=5.0e4, contact_damping=1.0e3, friction=1.0, friction_damping=1.0e3,
                      gravity=-9.81, angular_damping=0.01, max_angular_velocity=100.0, self_collision=True)

# shape filters of the capsule humanoid (puffer_phc/envs/humanoid_phc.py:374): shapes whose words
# share a bit do not collide; PhysX never collides a link with its parent
FILTER = (0, 0, 7, 16, 12, 0, 56, 2, 33, 128, 0, 192, 0, 64, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)


# ------------------------------------------------------------------ model --
def load_model(path=MODEL_JSON):
    """Per-body arrays from the body-model JSON (tools/make_body_model.py).  Contact points: a sphere
    is its centre with its radius, a capsule its two end-sphere centres with its radius, a box its 8
    corners with radius 0."""
    with open(path) as f:
        d = json.load(f)
    bodies = d["bodies"]
    assert len(bodies) == NUM_BODIES
    m = dict(parent=np.array([b["parent"] for b in bodies]), offset=np.array([b["offset"] for b in bodies]),
             mass=np.array([b["mass"] for b in bodies]), com=np.array([b["com"] for b in bodies]),
             inertia=np.array([b["inertia"] for b in bodies]), kp=np.array([b["kp"] for b in bodies]),
             kd=np.array([b["kd"] for b in bodies]), armature=np.array([b["armature"] for b in bodies]))
    pts = []
    for b in bodies:
        s = b["shape"]
        if s["type"] == "sphere":
            p = [s["center"] + [s["radius"]]]
        elif s["type"] == "capsule":
            p = [s["p0"] + [s["radius"]], s["p1"] + [s["radius"]]]
        else:
            c, h = np.array(s["center"]), np.array(s["half"])
            p = [list(c + h * np.array([sx, sy, sz])) + [0.0] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]
        pts.append(np.array(p, dtype=np.float64))
    m["points"] = pts
    # self-collision capsules (p0, p1, radius): sphere = zero-length segment, box = segment on its
    # longest half-axis shortened by the radius = the smallest other half-extent
    seg = np.zeros((NUM_BODIES, 2, 3))
    rad = np.zeros(NUM_BODIES)
    for i, b in enumerate(bodies):
        s = b["shape"]
        if s["type"] == "sphere":
            seg[i] = [s["center"], s["center"]]
            rad[i] = s["radius"]
        elif s["type"] == "capsule":
            seg[i] = [s["p0"], s["p1"]]
            rad[i] = s["radius"]
        else:
            c, h = np.array(s["center"]), np.array(s["half"])
            k = int(np.argmax(h))
            rad[i] = min(h[(k + 1) % 3], h[(k + 2) % 3])
            d = np.zeros(3)
            d[k] = max(h[k] - rad[i], 0.0)
            seg[i] = [c - d, c + d]
    m["seg"], m["seg_r"] = seg, rad
    par = m["parent"]
    m["pairs"] = [(i, j) for i in range(NUM_BODIES) for j in range(NUM_BODIES)
                  if i != j and par[i] != j and par[j] != i and not (FILTER[i] & FILTER[j])]
    # spatial inertia about the body origin, body coordinates (Featherstone's mcI)
    I6 = np.zeros((NUM_BODIES, 6, 6))
    for i in range(NUM_BODIES):
        C = skew(m["com"][i])
        I6[i, :3, :3] = m["inertia"][i] + m["mass"][i] * C @ C.T
        I6[i, :3, 3:] = m["mass"][i] * C
        I6[i, 3:, :3] = m["mass"][i] * C.T
        I6[i, 3:, 3:] = m["mass"][i] * np.eye(3)
    m["I6"] = I6
    return m


# ------------------------------------------------------------- rotations --
def skew(v):
    v = np.asarray(v, dtype=np.float64)
    z = np.zeros(v.shape[:-1])
    return np.stack([np.stack([z, -v[..., 2], v[..., 1]], -1), np.stack([v[..., 2], z, -v[..., 0]], -1),
                     np.stack([-v[..., 1], v[..., 0], z], -1)], -2)


def quat_mul(a, b):
    ax, ay, az, aw = np.moveaxis(a, -1, 0)
    bx, by, bz, bw = np.moveaxis(b, -1, 0)
    return np.stack([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz], -1)


def quat_to_mat(q):
    x, y, z, w = np.moveaxis(q, -1, 0)
    return np.stack([np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
                     np.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
                     np.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], -2)


def quat_from_rotvec(e):
    th = np.linalg.norm(e, axis=-1, keepdims=True)
    s = np.where(th > 1e-8, np.sin(0.5 * th) / np.maximum(th, 1e-30), 0.5 - th * th / 48.0)
    return np.concatenate([e * s, np.cos(0.5 * th)], -1)


def quat_to_rotvec(q):
    q = np.where(q[..., 3:4] < 0, -q, q)
    v = q[..., :3]
    sn = np.linalg.norm(v, axis=-1, keepdims=True)
    th = 2.0 * np.arctan2(sn, q[..., 3:4])
    k = np.where(sn > 1e-8, th / np.maximum(sn, 1e-30), 2.0 / np.maximum(q[..., 3:4], 1e-30))
    return v * k


def normalize(q):
    return q / np.linalg.norm(q, axis=-1, keepdims=True)


# ---------------------------------------------------------- spatial algebra --
def motion_xform(E, r):
    """Parent -> child motion transform: child frame rotated by E (child axes in parent coordinates)
    at offset r (parent coordinates).  X = [[E^T, 0], [-E^T [r]x, E^T]]."""
    n = E.shape[0]
    X = np.zeros((n, 6, 6))
    Et = np.swapaxes(E, -1, -2)
    X[:, :3, :3] = Et
    X[:, 3:, 3:] = Et
    X[:, 3:, :3] = -Et @ skew(np.broadcast_to(r, (n, 3)))
    return X


def crm(V):
    """Spatial motion cross product matrix."""
    n = V.shape[0]
    M = np.zeros((n, 6, 6))
    W, Vl = skew(V[:, :3]), skew(V[:, 3:])
    M[:, :3, :3] = W
    M[:, 3:, 3:] = W
    M[:, 3:, :3] = Vl
    return M


def crf(V):
    return -np.swapaxes(crm(V), -1, -2)


def mv(A, x):
    return np.einsum("nij,nj->ni", A, x)


# ---------------------------------------------------------------- state --
class State:
    """root_pos, root_quat (world), root_vel, root_ang_vel (world), joint_quat [E, 24, 4] (index 0
    unused), joint_vel [E, 24, 3] (relative angular velocity, child coordinates)."""

    def __init__(self, root_pos, root_quat, root_vel, root_ang_vel, dof_pos, dof_vel, com0=None):
        n = root_pos.shape[0]
        self.p0 = np.array(root_pos, dtype=np.float64)
        self.q0 = normalize(np.array(root_quat, dtype=np.float64))
        R0 = quat_to_mat(self.q0)
        self.w0 = np.einsum("nji,nj->ni", R0, root_ang_vel)  # body coordinates
        # root_vel is the centre of mass's velocity (PhysX): the origin's is v_com - w x com
        self.v0 = np.einsum("nji,nj->ni", R0, root_vel)
        if com0 is not None:
            self.v0 = self.v0 - np.cross(self.w0, com0)
        self.r = np.zeros((n, NUM_BODIES, 4))
        self.r[..., 3] = 1.0
        self.r[:, 1:] = quat_from_rotvec(np.asarray(dof_pos, dtype=np.float64).reshape(n, NUM_BODIES - 1, 3))
        self.om = np.zeros((n, NUM_BODIES, 3))
        self.om[:, 1:] = np.asarray(dof_vel, dtype=np.float64).reshape(n, NUM_BODIES - 1, 3)


def forward_kinematics(model, st):
    """World quaternions Q, rotations R, origins P and body-coordinate twists V of every body."""
    n = st.p0.shape[0]
    Q = np.zeros((n, NUM_BODIES, 4))
    R = np.zeros((n, NUM_BODIES, 3, 3))
    P = np.zeros((n, NUM_BODIES, 3))
    V = np.zeros((n, NUM_BODIES, 6))
    Q[:, 0], P[:, 0] = st.q0, st.p0
    R[:, 0] = quat_to_mat(st.q0)
    V[:, 0, :3], V[:, 0, 3:] = st.w0, st.v0
    Xs = [None] * NUM_BODIES
    for i in range(1, NUM_BODIES):
        p = model["parent"][i]
        Q[:, i] = quat_mul(Q[:, p], st.r[:, i])
        R[:, i] = quat_to_mat(Q[:, i])
        P[:, i] = P[:, p] + np.einsum("nij,j->ni", R[:, p], model["offset"][i])
        Xs[i] = motion_xform(quat_to_mat(st.r[:, i]), model["offset"][i])
        V[:, i] = mv(Xs[i], V[:, p])
        V[:, i, :3] += st.om[:, i]
    return Q, R, P, V, Xs


def _dot(a, b):
    return np.einsum("...i,...i->...", a, b)


def closest_points(p0, d1, q0, d2):
    """Clamped closest-point parameters (s, t) of segments p0 + s d1 and q0 + t d2, s, t in [0, 1]
    (the clamped 2x2 solve, then t clamped and s re-solved); any leading batch shape."""
    r = p0 - q0
    a, e, f, c, b = _dot(d1, d1), _dot(d2, d2), _dot(d2, r), _dot(d1, r), _dot(d1, d2)
    den = a * e - b * b
    ga, ge = a > 1e-12, e > 1e-12
    a1, e1 = np.where(ga, a, 1.0), np.where(ge, e, 1.0)
    s = np.where(den > 1e-12, np.clip((b * f - c * e) / np.where(den > 1e-12, den, 1.0), 0, 1), 0.0)
    t = (b * s + f) / e1
    s = np.where(t < 0, np.clip(-c / a1, 0, 1), np.where(t > 1, np.clip((b - c) / a1, 0, 1), s))
    t = np.clip(t, 0, 1)
    both = ga & ge
    s = np.where(both, s, np.where(ga, np.clip(-c / a1, 0, 1), 0.0))
    t = np.where(both, t, np.where(ga, 0.0, np.clip(f / e1, 0, 1)))
    return s, t


def self_contacts(model, R, P, V, prm):
    """Penalty self-collision between the filtered body pairs, both bodies as capsules: per pair
    i < j one contact (the closest points of the two segments), normal force stiffness x depth +
    damping x approach rate (>= 0) at the middle of the overlap, pushing i away from j and j away
    from i (action = reaction); body-coordinate wrenches about each body's origin [E, 24, 6]."""
    n = P.shape[0]
    pi = np.array([p[0] for p in model["pairs"] if p[0] < p[1]])
    pj = np.array([p[1] for p in model["pairs"] if p[0] < p[1]])
    ends = P[:, :, None, :] + np.einsum("nbij,bkj->nbki", R, model["seg"])  # [E, 24, 2, 3] world
    W = np.einsum("nbij,nbj->nbi", R, V[..., :3])
    Vo = np.einsum("nbij,nbj->nbi", R, V[..., 3:])
    ri, rj = model["seg_r"][pi], model["seg_r"][pj]
    a0, b0 = ends[:, pi, 0], ends[:, pj, 0]  # [E, pairs, 3]
    d1, d2 = ends[:, pi, 1] - a0, ends[:, pj, 1] - b0
    s, t = closest_points(a0, d1, b0, d2)
    c1 = a0 + s[..., None] * d1
    dd = b0 + t[..., None] * d2 - c1
    dist = np.linalg.norm(dd, axis=-1)
    pen = ri + rj - dist
    nrm = np.where((dist > 1e-6)[..., None], dd / np.maximum(dist, 1e-30)[..., None], np.array([0.0, 0.0, 1.0]))
    x = c1 + nrm * (ri - 0.5 * pen)[..., None]
    vi = Vo[:, pi] + np.cross(W[:, pi], x - P[:, pi])
    vj = Vo[:, pj] + np.cross(W[:, pj], x - P[:, pj])
    vn = _dot(vi - vj, nrm)
    fm = np.where(pen > 0, np.maximum(0.0, prm["contact_stiffness"] * pen + prm["contact_damping"] * vn), 0.0)
    f = np.zeros((n, NUM_BODIES, 6))
    for idx, sign in ((pi, 1.0), (pj, -1.0)):
        Rt = np.swapaxes(R[:, idx], -1, -2)
        Fb = np.einsum("npij,npj->npi", Rt, -sign * fm[..., None] * nrm)
        wrench = np.concatenate([np.cross(np.einsum("npij,npj->npi", Rt, x - P[:, idx]), Fb), Fb], -1)
        np.add.at(f, (slice(None), idx), wrench)
    return f


def external_forces(model, R, P, V, prm):
    """Gravity, angular damping, penalty ground contact and self-collision as body-coordinate
    wrenches about each body origin."""
    n = P.shape[0]
    f = np.zeros((n, NUM_BODIES, 6))
    g = np.array([0.0, 0.0, prm["gravity"]])
    zhat = np.array([0.0, 0.0, 1.0])
    if prm["self_collision"]:
        f += self_contacts(model, R, P, V, prm)
    for i in range(NUM_BODIES):
        Rt = np.swapaxes(R[:, i], -1, -2)
        F = model["mass"][i] * np.einsum("nij,j->ni", Rt, g)
        f[:, i, :3] += np.cross(model["com"][i], F)
        f[:, i, 3:] += F
        # angular damping (humanoid_phc.py:212): a pure torque -d Ic w
        f[:, i, :3] -= prm["angular_damping"] * np.einsum("ij,nj->ni", model["inertia"][i], V[:, i, :3])
        for c in model["points"][i]:
            x = P[:, i] + np.einsum("nij,j->ni", R[:, i], c[:3])
            d = c[3] - x[:, 2]  # penetration depth
            a = c[:3][None, :] - c[3] * np.einsum("nij,j->ni", Rt, zhat)  # contact point, body coords
            vw = np.einsum("nij,nj->ni", R[:, i], V[:, i, 3:] + np.cross(V[:, i, :3], a))
            fn = np.maximum(0.0, prm["contact_stiffness"] * d - prm["contact_damping"] * vw[:, 2])
            vt = np.linalg.norm(vw[:, :2], axis=-1)
            kt = np.minimum(prm["friction_damping"], prm["friction"] * fn / np.maximum(vt, 1e-12))
            Fw = np.stack([-kt * vw[:, 0], -kt * vw[:, 1], fn], -1)
            Fw = np.where((d > 0)[:, None], Fw, 0.0)
            Fb = np.einsum("nij,nj->ni", Rt, Fw)
            f[:, i, :3] += np.cross(a, Fb)
            f[:, i, 3:] += Fb
    return f


def clamp_norm(x, m):
    """Rows of x scaled down to norm <= m (m <= 0: no cap)."""
    if m <= 0:
        return x
    nrm = np.linalg.norm(x, axis=-1, keepdims=True)
    return np.where(nrm > m, x * (m / np.maximum(nrm, 1e-30)), x)


def substep(model, st, target, prm, dt):
    """One semi-implicit Euler substep; returns the applied joint torques [E, 24, 3]."""
    n = st.p0.shape[0]
    _, R, P, V, Xs = forward_kinematics(model, st)
    fext = external_forces(model, R, P, V, prm)
    kp = model["kp"] * prm["kp_scale"]
    kd = model["kd"] * prm["kd_scale"]
    e = np.zeros((n, NUM_BODIES, 3))
    e[:, 1:] = quat_to_rotvec(st.r[:, 1:])
    tau = kp * (target - e) - (kd + dt * kp) * st.om  # implicit PD: the -dt*(kd+dt*kp)*qdd part via D
    IA = np.broadcast_to(model["I6"], (n, NUM_BODIES, 6, 6)).copy()
    pA = np.zeros((n, NUM_BODIES, 6))
    c = np.zeros((n, NUM_BODIES, 6))
    for i in range(NUM_BODIES):
        pA[:, i] = mv(crf(V[:, i]), mv(IA[:, i], V[:, i])) - fext[:, i]
        if i > 0:
            S_om = np.concatenate([st.om[:, i], np.zeros((n, 3))], -1)
            c[:, i] = mv(crm(V[:, i]), S_om)
    U = [None] * NUM_BODIES
    Dinv = [None] * NUM_BODIES
    u = [None] * NUM_BODIES
    for i in range(NUM_BODIES - 1, 0, -1):
        p = model["parent"][i]
        U[i] = IA[:, i, :, :3]
        D = IA[:, i, :3, :3] + np.diag(model["armature"][i] + dt * kd[i] + dt * dt * kp[i])
        Dinv[i] = np.linalg.inv(D)
        u[i] = tau[:, i] - pA[:, i, :3]
        Ia = IA[:, i] - U[i] @ Dinv[i] @ np.swapaxes(U[i], -1, -2)
        pa = pA[:, i] + mv(Ia, c[:, i]) + mv(U[i], mv(Dinv[i], u[i]))
        Xt = np.swapaxes(Xs[i], -1, -2)
        IA[:, p] += Xt @ Ia @ Xs[i]
        pA[:, p] += mv(Xt, pa)
    a = np.zeros((n, NUM_BODIES, 6))
    a[:, 0] = -np.linalg.solve(IA[:, 0], pA[:, 0][..., None])[..., 0]
    qdd = np.zeros((n, NUM_BODIES, 3))
    for i in range(1, NUM_BODIES):
        ap = mv(Xs[i], a[:, model["parent"][i]]) + c[:, i]
        qdd[:, i] = mv(Dinv[i], u[i] - np.einsum("nji,nj->ni", U[i], ap))
        a[:, i] = ap
        a[:, i, :3] += qdd[:, i]
    applied = tau - dt * (kd + dt * kp) * qdd
    # integrate: velocities first, then positions with the new velocities
    st.om[:, 1:] += dt * qdd[:, 1:]
    st.om = clamp_norm(st.om, prm["max_angular_velocity"])  # AssetOptions.max_angular_velocity, :213
    st.r[:, 1:] = normalize(quat_mul(st.r[:, 1:], quat_from_rotvec(dt * st.om[:, 1:])))
    st.w0 = clamp_norm(st.w0 + dt * a[:, 0, :3], prm["max_angular_velocity"])
    st.v0 = st.v0 + dt * a[:, 0, 3:]
    st.p0 = st.p0 + dt * np.einsum("nij,nj->ni", R[:, 0], st.v0)
    st.q0 = normalize(quat_mul(st.q0, quat_from_rotvec(dt * st.w0)))
    return applied


def body_states(model, st):
    """Isaac Gym rigid-body layout [E, 24, 13]: pos (body origin), quat (xyzw), linear velocity of the
    centre of mass (PhysX's), angular velocity; world frame."""
    Q, R, P, V, _ = forward_kinematics(model, st)
    vcom = V[..., 3:] + np.cross(V[..., :3], model["com"][None])
    return np.concatenate([P, Q, np.einsum("nbij,nbj->nbi", R, vcom), np.einsum("nbij,nbj->nbi", R, V[..., :3])], -1)


def step(model, rb, dof_state, pd_target, params=None):
    """One env step = control_freq_inv sim steps of `substeps` substeps each, from the env buffers
    (rigid_body_state [E, 24, 13]: the root record is the state; dof_state [E, 69, 2]) to new
    (rigid_body_state, dof_state, dof_force [E, 69])."""
    prm = dict(DEFAULT_PARAMS, **(params or {}))
    n = rb.shape[0]
    st = State(rb[:, 0, 0:3], rb[:, 0, 3:7], rb[:, 0, 7:10], rb[:, 0, 10:13], dof_state[..., 0], dof_state[..., 1],
               com0=model["com"][0])
    target = np.zeros((n, NUM_BODIES, 3))
    target[:, 1:] = np.asarray(pd_target, dtype=np.float64).reshape(n, NUM_BODIES - 1, 3)
    dt = prm["sim_dt"] / prm["substeps"]
    applied = None
    for _ in range(int(prm["control_freq_inv"]) * int(prm["substeps"])):
        applied = substep(model, st, target, prm, dt)
    rb_out = body_states(model, st)
    dof = np.stack([quat_to_rotvec(st.r[:, 1:]).reshape(n, NUM_DOF), st.om[:, 1:].reshape(n, NUM_DOF)], -1)
    return rb_out, dof, applied[:, 1:].reshape(n, NUM_DOF)


def rest_state(model, n, height_clearance=0.0):
    """Zero pose, zero velocity, root raised so the lowest contact point sits `height_clearance`
    above the ground: (rigid_body_state, dof_state)."""
    rb = np.zeros((n, NUM_BODIES, 13))
    rb[:, 0, 6] = 1.0
    dof = np.zeros((n, NUM_DOF, 2))
    st = State(rb[:, 0, 0:3], rb[:, 0, 3:7], rb[:, 0, 7:10], rb[:, 0, 10:13], dof[..., 0], dof[..., 1])
    _, R, P, _, _ = forward_kinematics(model, st)
    low = min(float((P[0, i] + R[0, i] @ c[:3])[2] - c[3]) for i in range(NUM_BODIES) for c in model["points"][i])
    rb[:, 0, 2] = -low + height_clearance
    return body_states(model, State(rb[:, 0, 0:3], rb[:, 0, 3:7], rb[:, 0, 7:10], rb[:, 0, 10:13], dof[..., 0],
                                    dof[..., 1])), dof
