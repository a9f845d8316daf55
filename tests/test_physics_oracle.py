"""N3 physics oracle (oracle/physics_oracle.py) pinned by physical laws — PhysX itself is closed and
cannot be a fixture, so parity with the reference's simulator is unpinned.  These
checks hold for any correct articulated-body solver with this integrator:
  * free fall: the semi-implicit Euler closed form, to rounding, with the pose unchanged;
  * the unforced free-floating tree: spatial momentum and kinetic energy drift only at first order
    in the substep (ratio ~4 when the substep shrinks 4x) — a wrong inertia, bias force or transform
    leaves an O(1) residual instead;
  * the PD drive: a joint settles at its target with gravity off;
  * self-collision: the filtered pairs, the closest-point solve, internal (action = reaction) forces;
  * angular damping dissipates, the velocity cap holds, records carry centre-of-mass velocities;
  * a standing humanoid on the ground neither sinks nor explodes;
and the body-model extraction and its device packing are checked against the MJCF's numbers."""

import json
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from oracle import physics_oracle as P  # noqa: E402

ROOT = os.path.join(os.path.dirname(__file__), "..")


@pytest.fixture(scope="module")
def model():
    return P.load_model()


def _momentum(model, rb):
    """World linear momentum, angular momentum about the world origin, kinetic energy."""
    n = rb.shape[0]
    lin, ang, ke = np.zeros((n, 3)), np.zeros((n, 3)), np.zeros(n)
    for i in range(P.NUM_BODIES):
        R = P.quat_to_mat(rb[:, i, 3:7])
        c = rb[:, i, 0:3] + np.einsum("nij,j->ni", R, model["com"][i])
        w = rb[:, i, 10:13]
        vc = rb[:, i, 7:10]  # the record's linear velocity is the centre of mass's
        Iw = np.einsum("nij,jk,nlk->nil", R, model["inertia"][i], R)
        m = model["mass"][i]
        lin += m * vc
        ang += np.cross(c, m * vc) + np.einsum("nij,nj->ni", Iw, w)
        ke += 0.5 * m * (vc * vc).sum(-1) + 0.5 * np.einsum("ni,nij,nj->n", w, Iw, w)
    return lin, ang, ke


def _random_state(model, n, seed, clearance):
    rng = np.random.default_rng(seed)
    rb, dof = P.rest_state(model, n, clearance)
    dof[..., 0] = rng.normal(0, 0.3, (n, P.NUM_DOF))
    dof[..., 1] = rng.normal(0, 1.0, (n, P.NUM_DOF))
    rb[:, 0, 7:13] = rng.normal(0, 0.5, (n, 6))
    st = P.State(rb[:, 0, 0:3], rb[:, 0, 3:7], rb[:, 0, 7:10], rb[:, 0, 10:13], dof[..., 0], dof[..., 1])
    return P.body_states(model, st), dof


def test_model_matches_mjcf(model):
    with open(P.MODEL_JSON) as f:
        d = json.load(f)
    names = [b["name"] for b in d["bodies"]]
    assert names[0] == "Pelvis" and len(names) == 24
    np.testing.assert_allclose(model["mass"].sum(), 74.0, atol=0.05)  # SMPL neutral, MJCF densities
    assert all(model["parent"][i] < i for i in range(1, 24))
    # MJCF joint gains (assets/smpl_humanoid.xml): hips / knees / ankles 800, torso chain 1000
    assert model["kp"][names.index("L_Knee")].tolist() == [800.0] * 3
    assert model["kp"][names.index("Spine")].tolist() == [1000.0] * 3
    np.testing.assert_allclose(model["kd"][1:], model["kp"][1:] / 10)
    for i in range(24):
        assert np.all(np.linalg.eigvalsh(model["I6"][i]) > 0)


def test_free_fall_closed_form(model):
    rb, dof = P.rest_state(model, 3, 1.0)
    z0 = rb[:, 0, 2].copy()
    rb1, dof1, force = P.step(model, rb, dof, np.zeros((3, P.NUM_DOF)))
    k, dt, g = 16, 1.0 / 480.0, 9.81
    np.testing.assert_allclose(rb1[:, :, 2] - rb[:, :, 2], -g * dt * dt * k * (k + 1) / 2, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(rb1[:, :, 9], -g * dt * k, rtol=1e-9)
    np.testing.assert_allclose(dof1, 0.0, atol=1e-12)
    np.testing.assert_allclose(force, 0.0, atol=1e-9)
    assert np.all(rb1[:, 0, 2] < z0)


def test_unforced_tree_conserves_momentum_first_order(model):
    """Gravity, gains and armature off, airborne: momentum / energy drift shrinks ~4x per 4x
    shorter substep."""
    rb, dof = _random_state(model, 2, 0, 5.0)
    free = dict(model, armature=model["armature"] * 0)
    prm = dict(gravity=0.0, kp_scale=0.0, kd_scale=0.0, angular_damping=0.0, max_angular_velocity=0.0,
               self_collision=False)
    l0, a0, k0 = _momentum(model, rb)
    errs = []
    for sub in (8, 32):
        r, d = rb.copy(), dof.copy()
        for _ in range(2):
            r, d, _f = P.step(free, r, d, np.zeros((2, P.NUM_DOF)), dict(prm, substeps=sub))
        l1, a1, k1 = _momentum(model, r)
        errs.append((np.abs(l1 - l0).max(), np.abs(a1 - a0).max(), np.abs(k1 - k0).max()))
    for coarse, fine in zip(*errs):
        assert 3.0 < coarse / fine < 5.0, errs
    assert errs[1][0] < 0.1 and errs[1][2] < 0.05 * k0.min()


def test_pd_drive_reaches_target(model):
    """Airborne, gravity off, from rest: a single joint driven to 0.3 rad settles there."""
    rb, dof = P.rest_state(model, 1, 5.0)
    target = np.zeros((1, P.NUM_DOF))
    j = 3 * (2 - 1)  # first dof of body 2 (L_Knee): dof_state rows 3 (b - 1) .. + 2
    target[0, j] = 0.3
    for _ in range(30):  # 1 s
        rb, dof, f = P.step(model, rb, dof, target, dict(gravity=0.0))
    np.testing.assert_allclose(dof[0, j, 0], 0.3, atol=2e-3)
    np.testing.assert_allclose(np.delete(dof[0, :, 0], j), 0.0, atol=2e-3)
    assert abs(dof[0, j, 1]) < 1e-2


def test_standing_humanoid_is_supported(model):
    rb, dof = P.rest_state(model, 1, 0.0)
    z0 = rb[0, 0, 2]
    for _ in range(30):  # 1 s with the PD drives holding the zero pose
        rb, dof, f = P.step(model, rb, dof, np.zeros((1, P.NUM_DOF)))
    assert np.all(np.isfinite(rb))
    assert abs(rb[0, 0, 2] - z0) < 0.02
    assert np.abs(dof[0, :, 0]).max() < 0.1
    low = min(float((rb[0, i, 0:3] + P.quat_to_mat(rb[0, i, 3:7]) @ c[:3])[2] - c[3])
              for i in range(24) for c in model["points"][i])
    assert -0.01 < low < 0.005  # feet on, not through, the ground


def test_rotvec_roundtrip():
    rng = np.random.default_rng(1)
    e = rng.normal(0, 1.0, (100, 3))
    e *= np.minimum(1.0, 3.0 / np.linalg.norm(e, axis=-1, keepdims=True))  # |e| < pi
    np.testing.assert_allclose(P.quat_to_rotvec(P.quat_from_rotvec(e)), e, atol=1e-12)


def test_device_table_layout(model):
    """physics.BodyModel's packed table (what phc_physics_step reads) against the oracle's model."""
    torch = pytest.importorskip("torch")  # noqa: F841
    from puffer_phc_amd.physics import BodyModel

    bm = BodyModel(device="cpu")
    t = bm.host
    assert bm.depth == 8 and t.shape == (24, 80)
    np.testing.assert_array_equal(t[1:, 0], model["parent"][1:])
    np.testing.assert_allclose(t[:, 9], model["mass"], rtol=1e-6)
    np.testing.assert_allclose(t[:, 6:9], model["offset"], atol=1e-7)
    for i in range(24):
        np.testing.assert_allclose(t[i, 13:16], np.diag(model["inertia"][i]), rtol=1e-5)
        k = int(t[i, 28])
        assert k == len(model["points"][i])
        np.testing.assert_allclose(t[i, 32:32 + 4 * k].reshape(k, 4), model["points"][i], atol=1e-7)
        kids = [j for j in range(24) if model["parent"][j] == i and j > 0]
        assert int(t[i, 2]) == len(kids) and t[i, 3:3 + len(kids)].tolist() == kids
        np.testing.assert_allclose(t[i, 64:70].reshape(2, 3), model["seg"][i], atol=1e-7)
        np.testing.assert_allclose(t[i, 70], model["seg_r"][i], rtol=1e-6)
        assert int(t[i, 71]) == sum(1 << j for (a, j) in model["pairs"] if a == i)


def test_self_collision_pairs_follow_the_filters(model):
    """humanoid_phc.py:374's filter words: shapes sharing a bit never collide, nor do a parent and
    its child; the pair set is symmetric and the zero pose has no overlapping pair."""
    pairs = set(model["pairs"])
    assert all((j, i) in pairs for i, j in pairs)
    names = json.load(open(P.MODEL_JSON))["bodies"]
    idx = {b["name"]: k for k, b in enumerate(names)}
    assert (idx["L_Knee"], idx["L_Toe"]) not in pairs  # filter 7 & 12 share bit 4
    assert (idx["L_Knee"], idx["R_Ankle"]) not in pairs  # 7 & 2
    assert (idx["L_Hand"], idx["Pelvis"]) in pairs and (idx["L_Hand"], idx["R_Hand"]) in pairs
    assert (idx["L_Elbow"], idx["L_Wrist"]) not in pairs  # joined
    assert len(pairs) == 2 * 245
    rb, dof = P.rest_state(model, 1, 0.0)
    st = P.State(rb[:, 0, 0:3], rb[:, 0, 3:7], rb[:, 0, 7:10], rb[:, 0, 10:13], dof[..., 0], dof[..., 1])
    _, R, Pp, V, _ = P.forward_kinematics(model, st)
    assert np.abs(P.self_contacts(model, R, Pp, V, P.DEFAULT_PARAMS)).max() == 0.0


def test_closest_points_against_brute_force():
    rng = np.random.default_rng(4)
    n = 200
    p0, q0 = rng.normal(0, 1, (n, 3)), rng.normal(0, 1, (n, 3))
    d1, d2 = rng.normal(0, 1, (n, 3)), rng.normal(0, 1, (n, 3))
    d1[:20] = 0.0  # a point against a segment
    d2[20:40] = 0.0
    d2[40:60] = 2.5 * d1[40:60]  # parallel segments
    s, t = P.closest_points(p0, d1, q0, d2)
    got = np.linalg.norm(p0 + s[:, None] * d1 - q0 - t[:, None] * d2, axis=-1)
    g = np.linspace(0, 1, 201)
    a = p0[:, None, None, :] + g[None, :, None, None] * d1[:, None, None, :]
    b = q0[:, None, None, :] + g[None, None, :, None] * d2[:, None, None, :]
    brute = np.linalg.norm(a - b, axis=-1).reshape(n, -1).min(-1)
    assert np.all(got <= brute + 1e-12) and np.all(brute - got < 2e-2 * (1 + brute))


def test_self_contact_forces_are_internal(model):
    """Strongly bent poses make limbs overlap: every contact acts on both bodies of its pair at one
    point with opposite forces, so the world net force and net torque of the self-contacts vanish."""
    rng = np.random.default_rng(8)
    n = 64
    rb, dof = P.rest_state(model, n, 1.0)
    dof[..., 0] = rng.normal(0, 1.2, (n, P.NUM_DOF))
    dof[..., 1] = rng.normal(0, 2.0, (n, P.NUM_DOF))
    st = P.State(rb[:, 0, 0:3], rb[:, 0, 3:7], rb[:, 0, 7:10], rb[:, 0, 10:13], dof[..., 0], dof[..., 1])
    _, R, Pp, V, _ = P.forward_kinematics(model, st)
    f = P.self_contacts(model, R, Pp, V, P.DEFAULT_PARAMS)
    Fw = np.einsum("nbij,nbj->nbi", R, f[..., 3:])
    Tw = np.einsum("nbij,nbj->nbi", R, f[..., :3]) + np.cross(Pp, Fw)  # about the world origin
    touching = np.abs(Fw).sum((1, 2)) > 1.0
    assert touching.sum() >= n // 4
    scale = np.abs(Fw).sum((1, 2)).max()
    assert np.abs(Fw.sum(1)).max() < 1e-9 * scale and np.abs(Tw.sum(1)).max() < 1e-8 * scale


def test_angular_damping_and_velocity_cap(model):
    """Airborne, gravity / gains off: angular damping only removes kinetic energy; a joint spun
    past max_angular_velocity leaves the step at the cap."""
    rb, dof = _random_state(model, 2, 5, 5.0)
    free = dict(model, armature=model["armature"] * 0)
    base = dict(gravity=0.0, kp_scale=0.0, kd_scale=0.0, self_collision=False, max_angular_velocity=0.0)
    _, _, k0 = _momentum(model, rb)
    ke = {}
    for d in (0.0, 2.0):
        r, q, _ = P.step(free, rb.copy(), dof.copy(), np.zeros((2, P.NUM_DOF)), dict(base, angular_damping=d, substeps=32))
        ke[d] = _momentum(model, r)[2]
    assert np.all(ke[2.0] < ke[0.0] - 1e-3 * k0)
    dof[0, 6, 1] = 400.0
    _, q, _ = P.step(free, rb, dof, np.zeros((2, P.NUM_DOF)), dict(base, max_angular_velocity=100.0))
    w = np.linalg.norm(q[:, :, 1].reshape(2, 23, 3), axis=-1)
    assert w.max() <= 100.0 + 1e-9 and abs(w[0, 2] - 100.0) < 1e-9


def test_record_velocity_is_the_centre_of_mass_velocity(model):
    """A spinning free body: each record's linear velocity is d/dt of its centre of mass."""
    rb, dof = _random_state(model, 1, 9, 5.0)
    prm = dict(gravity=0.0, kp_scale=0.0, kd_scale=0.0, self_collision=False, angular_damping=0.0,
               max_angular_velocity=0.0, control_freq_inv=1, substeps=64, sim_dt=1e-3)

    def coms(r):
        return r[0, :, 0:3] + np.einsum("bij,bj->bi", P.quat_to_mat(r[0, :, 3:7]), model["com"])

    r1, d1, _ = P.step(model, rb, dof, np.zeros((1, P.NUM_DOF)), prm)
    r2, _, _ = P.step(model, r1, d1, np.zeros((1, P.NUM_DOF)), prm)
    fd = (coms(r2) - coms(rb)) / 2e-3
    np.testing.assert_allclose(r1[0, :, 7:10], fd, atol=2e-3 * (1 + np.abs(fd).max()))


def test_product_rest_state_matches_oracle(model):
    """physics.rest_state (the product's standing start, used by tools/physics_probe.py) puts the
    root at the oracle's rest height."""
    pytest.importorskip("torch")
    from puffer_phc_amd.physics import BodyModel, rest_state

    bm = BodyModel(device="cpu")
    rb, dof = rest_state(bm, 3, 0.05, device="cpu")
    want, _ = P.rest_state(model, 1, 0.05)
    np.testing.assert_allclose(rb[:, 0, 2].numpy(), want[0, 0, 2], atol=1e-6)
    assert float(dof.abs().max()) == 0.0 and rb.shape == (3, 24, 13)


def test_standing_clips_match_the_rest_pose(model):
    """synthetic.standing_clips (the balance task of profiles/r03_train_articulated_*.log): without
    sway every frame is the upright zero pose at the body model's rest height (feet on the
    ground, not through it); with sway the rotations stay within the cone."""
    torch = pytest.importorskip("torch")
    from puffer_phc_amd.synthetic import standing_clips

    q, t, c, fps = standing_clips(3, frames=40, device="cpu")
    assert q.shape == (120, 24, 4) and t.shape == (120, 3) and c.tolist() == [40] * 3
    assert torch.equal(q[..., 3], torch.ones(120, 24, dtype=torch.float64)) and float(q[..., :3].abs().max()) == 0
    rb, _ = P.rest_state(model, 1, 0.0)
    assert 0.0 <= float(t[0, 2]) - rb[0, 0, 2] < 0.01
    q, t, _, _ = standing_clips(2, frames=90, sway=0.1, device="cpu")
    ang = 2 * torch.acos(q[..., 3].abs().clamp(max=1))
    assert 0.01 < float(ang.max()) < 0.6 and torch.equal(t[:, :2], torch.zeros(180, 2, dtype=torch.float64))
