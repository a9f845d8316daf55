"""N3 articulated-body step on the HIP path (phc_physics_step) against the CPU restatement
(oracle/physics_oracle.py, float64).  Tolerances: the kernel computes in fp32 over 16 substeps of
the contact / PD dynamics, so positions are held to 2e-4 m, orientations to 2e-4, velocities to
5e-3 (m/s, rad/s) and PD torques to 0.2 N m (looser where penalty contacts act: a 5e4 N/m spring
over 16 substeps amplifies fp32 rounding) (gains up to 1000 N m/rad) — about 100x the measured
fp32-vs-fp64 differences, far below any modelling error (a wrong term moves them by O(1)).  At the
full bench size (4096 envs) the checks are size-independent: the free-fall closed form, finiteness,
and per-env agreement of a sampled subset with the oracle."""

import numpy as np
import pytest
import torch

from oracle import physics_oracle as P

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def model():
    return P.load_model()


@pytest.fixture(scope="module")
def device_model():
    from puffer_phc_amd.physics import BodyModel

    return BodyModel(device=DEV)


def _gpu_step(device_model, rb, dof, target, steps=1, **cfg):
    from puffer_phc_amd import _native
    from puffer_phc_amd.physics import ArticulatedPhysics, PhysicsConfig

    phys = ArticulatedPhysics(PhysicsConfig(**cfg), model=device_model)
    n = rb.shape[0]
    rb_t = torch.tensor(rb, dtype=torch.float32, device=DEV).contiguous()
    dof_t = torch.tensor(dof, dtype=torch.float32, device=DEV).contiguous()
    force_t = torch.full((n, P.NUM_DOF), float("nan"), device=DEV)
    root_t = torch.zeros((n, 13), device=DEV)
    tgt_t = torch.tensor(target, dtype=torch.float32, device=DEV).contiguous()
    env_c = _native.physics_env_struct(rb_t, dof_t, force_t, root_t)
    for _ in range(steps):
        _native.physics_step(env_c, tgt_t, device_model.table, phys.params)
    torch.cuda.synchronize()
    return rb_t.cpu().numpy().astype(np.float64), dof_t.cpu().numpy().astype(np.float64), \
        force_t.cpu().numpy().astype(np.float64), root_t.cpu().numpy().astype(np.float64)


def _oracle_steps(model, rb, dof, target, steps=1, **cfg):
    f = None
    for _ in range(steps):
        rb, dof, f = P.step(model, rb, dof, target, cfg)
    return rb, dof, f


def _random_state(model, n, seed, clearance, pose=0.3, vel=1.0):
    rng = np.random.default_rng(seed)
    rb, dof = P.rest_state(model, n, clearance)
    dof[..., 0] = rng.normal(0, pose, (n, P.NUM_DOF))
    dof[..., 1] = rng.normal(0, vel, (n, P.NUM_DOF))
    rb[:, 0, 7:13] = rng.normal(0, 0.5 * vel, (n, 6))
    yaw = rng.uniform(-np.pi, np.pi, n)
    rb[:, 0, 3:7] = np.stack([np.zeros(n), np.zeros(n), np.sin(yaw / 2), np.cos(yaw / 2)], -1)
    rb[:, 0, 0:2] = rng.normal(0, 1.0, (n, 2))
    st = P.State(rb[:, 0, 0:3], rb[:, 0, 3:7], rb[:, 0, 7:10], rb[:, 0, 10:13], dof[..., 0], dof[..., 1])
    target = rng.normal(0, 0.3, (n, P.NUM_DOF))
    return P.body_states(model, st), dof, target


def _quat_close(a, b, atol):
    """Quaternions up to sign."""
    d = np.minimum(np.abs(a - b).max(-1), np.abs(a + b).max(-1))
    assert d.max() < atol, d.max()


def _compare(got, want, pos=2e-4, rot=2e-4, vel=5e-3, force=0.2):
    rb_g, dof_g, f_g, root_g = got
    rb_w, dof_w, f_w = want
    np.testing.assert_allclose(rb_g[..., 0:3], rb_w[..., 0:3], atol=pos)
    _quat_close(rb_g[..., 3:7], rb_w[..., 3:7], rot)
    np.testing.assert_allclose(rb_g[..., 7:13], rb_w[..., 7:13], atol=vel)
    np.testing.assert_allclose(dof_g[..., 0], dof_w[..., 0], atol=rot)
    np.testing.assert_allclose(dof_g[..., 1], dof_w[..., 1], atol=vel)
    np.testing.assert_allclose(f_g, f_w, atol=force)
    np.testing.assert_array_equal(root_g, rb_g[:, 0].astype(np.float32).astype(np.float64))


@pytest.mark.parametrize("n", [1, 13])
def test_airborne_pd_matches_oracle(model, device_model, n):
    """Random poses / velocities / targets well above the ground: ABA + implicit PD + gravity."""
    rb, dof, tgt = _random_state(model, n, 10 + n, 2.0)
    got = _gpu_step(device_model, rb, dof, tgt)
    _compare(got, _oracle_steps(model, rb, dof, tgt))


def test_ground_contact_matches_oracle(model, device_model):
    """Random poses dropped from 5 cm: contacts on feet / hands / pelvis, 3 env steps."""
    rb, dof, tgt = _random_state(model, 9, 3, 0.05, pose=0.2, vel=0.3)
    got = _gpu_step(device_model, rb, dof, tgt, steps=3)
    _compare(got, _oracle_steps(model, rb, dof, tgt, steps=3), pos=5e-4, rot=5e-4, vel=1e-2, force=0.5)


def test_standing_matches_oracle(model, device_model):
    rb, dof = P.rest_state(model, 8, 0.0)
    tgt = np.zeros((8, P.NUM_DOF))
    got = _gpu_step(device_model, rb, dof, tgt, steps=5)
    _compare(got, _oracle_steps(model, rb, dof, tgt, steps=5), pos=5e-4, rot=5e-4, vel=1e-2, force=0.5)


def test_self_collision_matches_oracle(model, device_model):
    """Strongly bent airborne poses: limbs overlap, the penalty self-contacts of the filtered pairs
    (humanoid_phc.py:374) act beside the PD drives, angular damping and the velocity cap."""
    rb, dof, tgt = _random_state(model, 16, 21, 2.0, pose=1.0, vel=0.5)
    st = P.State(rb[:, 0, 0:3], rb[:, 0, 3:7], rb[:, 0, 7:10], rb[:, 0, 10:13], dof[..., 0], dof[..., 1],
                 com0=model["com"][0])
    _, R, Pp, V, _ = P.forward_kinematics(model, st)
    assert (np.abs(P.self_contacts(model, R, Pp, V, P.DEFAULT_PARAMS)).sum((1, 2)) > 1.0).sum() >= 4
    got = _gpu_step(device_model, rb, dof, tgt)
    _compare(got, _oracle_steps(model, rb, dof, tgt), pos=5e-4, rot=5e-4, vel=2e-2, force=1.0)
    off = _gpu_step(device_model, rb, dof, tgt, self_collision=False)
    _compare(off, _oracle_steps(model, rb, dof, tgt, self_collision=False))
    assert np.abs(off[0] - got[0]).max() > 1e-3  # the contacts moved something


def test_velocity_cap_on_device(model, device_model):
    rb, dof, tgt = _random_state(model, 3, 4, 2.0)
    dof[:, 9, 1] = 500.0
    got = _gpu_step(device_model, rb, dof, tgt, max_angular_velocity=100.0)
    w = np.linalg.norm(got[1][:, :, 1].reshape(3, 23, 3), axis=-1)
    assert w.max() <= 100.0 * (1 + 1e-5)
    _compare(got, _oracle_steps(model, rb, dof, tgt, max_angular_velocity=100.0), vel=2e-2, force=1.0)


def test_gains_and_substeps_are_honoured(model, device_model):
    rb, dof, tgt = _random_state(model, 4, 7, 1.5)
    cfg = dict(substeps=4, kp_scale=0.5, kd_scale=2.0, friction=0.5)
    got = _gpu_step(device_model, rb, dof, tgt, **cfg)
    _compare(got, _oracle_steps(model, rb, dof, tgt, **cfg))


def test_free_fall_at_bench_size(device_model):
    """4096 envs in free fall: every body follows the semi-implicit Euler closed form."""
    n = 4096
    model = P.load_model()
    rb, dof = P.rest_state(model, 1, 1.0)
    rb = np.repeat(rb, n, 0)
    rb[:, :, 0] += np.arange(n)[:, None] * 0.01  # distinct envs, same physics
    dof = np.repeat(dof, n, 0)
    got_rb, got_dof, got_f, _ = _gpu_step(device_model, rb, dof, np.zeros((n, P.NUM_DOF)))
    k, dt, g = 16, 1.0 / 480.0, 9.81
    np.testing.assert_allclose(got_rb[..., 2] - rb[..., 2], -g * dt * dt * k * (k + 1) / 2, atol=2e-5)
    np.testing.assert_allclose(got_rb[..., 9], -g * dt * k, atol=1e-4)
    np.testing.assert_allclose(got_rb[..., 0], rb[..., 0], atol=1e-5)
    np.testing.assert_allclose(got_dof, 0.0, atol=1e-5)


def test_bench_size_sampled_envs_match_oracle(model, device_model):
    n = 4096
    rb, dof, tgt = _random_state(model, n, 11, 0.03, pose=0.2, vel=0.5)
    got = _gpu_step(device_model, rb, dof, tgt)
    assert all(np.all(np.isfinite(x)) for x in got)
    idx = np.array([0, 1, 7, 8, 1023, 2048, 4095])
    want = _oracle_steps(model, rb[idx], dof[idx], tgt[idx])
    _compare(tuple(x[idx] for x in got), want, pos=5e-4, rot=5e-4, vel=1e-2, force=0.5)


def test_rejects_bad_params(device_model):
    from puffer_phc_amd import _native

    n = 2
    rb = torch.zeros((n, 24, 13), device=DEV)
    dof = torch.zeros((n, 69, 2), device=DEV)
    f = torch.zeros((n, 69), device=DEV)
    env_c = _native.physics_env_struct(rb, dof, f)
    tgt = torch.zeros((n, 69), device=DEV)
    bad = _native.PhysicsParamsC(1 / 60, 2, 8, 0, 1.0, 1.0, 5e4, 1e3, 1.0, 1e3, -9.81, 0.0)
    with pytest.raises(RuntimeError, match="tree_depth"):
        _native.physics_step(env_c, tgt, device_model.table, bad)
    bad = _native.PhysicsParamsC(1 / 60, 2, 0, 8, 1.0, 1.0, 5e4, 1e3, 1.0, 1e3, -9.81, 0.0)
    with pytest.raises(RuntimeError, match="time stepping"):
        _native.physics_step(env_c, tgt, device_model.table, bad)
    bad = _native.PhysicsParamsC(1 / 60, 2, 8, 8, 1.0, 1.0, 5e4, 1e3, 1.0, 1e3, -9.81, -0.01, 100.0, 1)
    with pytest.raises(RuntimeError, match="damping"):
        _native.physics_step(env_c, tgt, device_model.table, bad)


def test_env_steps_with_articulated_physics():
    """PHCPufferEnv with cfg.physics = "articulated": resets from the motion library, PD targets
    from the actions, the physics step, then the fused obs / reward / reset kernel."""
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(16, 20, 60, seed=2, device=DEV)
    packed = PackedMotions.from_global_rotations(q, t, c, fps)
    env = PHCPufferEnv(EnvConfig(num_envs=32, seed=1, physics="articulated"), motion_data=packed)
    obs, _ = env.reset()
    rb0 = env.env._rigid_body_state.clone()
    gen = torch.Generator(device=DEV).manual_seed(0)
    for _ in range(5):
        act = torch.randn((32, 69), device=DEV, generator=gen) * 0.1
        obs, rew, term, trunc, info = env.step(act)
    torch.cuda.synchronize()
    assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
    assert torch.isfinite(env.env._rigid_body_state).all()
    assert not torch.equal(rb0, env.env._rigid_body_state)
    assert torch.isfinite(env.env.dof_force_tensor).all()


@pytest.mark.parametrize("self_collision", [False, True])
def test_env_honours_has_self_collision(self_collision):
    """RobotConfig.has_self_collision reaches the physics step (the reference's
    --disable_self_collision, humanoid_phc.py:338 / 370-381): an env built from the config runs bit for
    bit like one handed ArticulatedPhysics(PhysicsConfig(self_collision=...)) explicitly."""
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, RobotConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.physics import ArticulatedPhysics, PhysicsConfig
    from puffer_phc_amd.synthetic import synthetic_clips

    envs = []
    for explicit in (False, True):
        q, t, c, fps = synthetic_clips(8, 20, 60, seed=3, device=DEV)
        packed = PackedMotions.from_global_rotations(q, t, c, fps)
        cfg = EnvConfig(num_envs=16, seed=2, physics="articulated",
                        robot=RobotConfig(has_self_collision=self_collision))
        phys = ArticulatedPhysics(PhysicsConfig(self_collision=self_collision)) if explicit else None
        env = PHCPufferEnv(cfg, motion_data=packed, physics=phys)
        env.reset()
        envs.append(env)
    assert envs[0].env.physics.config.self_collision is self_collision
    gen = torch.Generator(device=DEV).manual_seed(1)
    for _ in range(4):
        act = torch.randn((16, 69), device=DEV, generator=gen) * 2.0
        for env in envs:
            env.step(act)
        assert torch.equal(envs[0].env._rigid_body_state, envs[1].env._rigid_body_state)
        assert torch.equal(envs[0].env.dof_force_tensor, envs[1].env.dof_force_tensor)


def test_ppo_iteration_with_articulated_physics():
    """One clean_pufferl iteration (graph rollout + PPO update) with the physics step in the env:
    the rollout's physics launches run inside evaluate(), the update trains on their outcome."""
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(64, 20, 90, seed=6, device=DEV)
    packed = PackedMotions.from_global_rotations(q, t, c, fps)
    env = PHCPufferEnv(EnvConfig(num_envs=64, seed=4, physics="articulated"), motion_data=packed)
    env.reset()
    torch.manual_seed(0)
    policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
    cfg = TrainConfig(batch_size=64 * 16, minibatch_size=256, bptt_horizon=8, checkpoint_interval=10 ** 9)
    comps, info, util = clean_pufferl.create("t", cfg, env.cfg, env, policy)
    before = {k: v.detach().clone() for k, v in policy.named_parameters()}
    clean_pufferl.evaluate(comps, info)
    exp = comps.experience
    assert info.global_step >= cfg.batch_size
    assert torch.isfinite(exp.obs).all() and torch.isfinite(exp.rewards).all()
    losses = clean_pufferl.train(comps, info, util)
    assert np.isfinite([losses.policy_loss, losses.value_loss, losses.approx_kl]).all()
    assert sum(not torch.equal(before[k], v) for k, v in policy.named_parameters() if v.requires_grad) > 0


def test_physics_step_actions_equals_separate_pd_launch(device_model):
    """phc_physics_step_actions (R13 folded into the physics launch) == phc_actions_to_pd +
    phc_physics_step, bit for bit, including the PD-target buffer it writes."""
    import torch

    from puffer_phc_amd import _native
    from puffer_phc_amd.physics import ArticulatedPhysics, rest_state

    phys = ArticulatedPhysics(model=device_model)
    n = 67
    g = torch.Generator(device="cuda").manual_seed(2)
    act = torch.randn((n, 69), device="cuda", generator=g) * 1.3
    off = torch.zeros(69, device="cuda")
    scale = torch.full((69,), 3.1415927, device="cuda")
    frozen = torch.zeros(69, dtype=torch.uint8, device="cuda")
    frozen[30:33] = 1
    outs = []
    for fused in (False, True):
        rb, dof = rest_state(device_model, n, 0.02)
        force = torch.zeros((n, 69), device="cuda")
        pd = torch.full((n, 69), float("nan"), device="cuda")
        env_c = _native.physics_env_struct(rb, dof, force)
        if fused:
            phys_pd = _native.pd_map(act, pd, off, scale, frozen)
            _native.physics_step_actions(env_c, phys_pd, device_model.table, phys.params)
        else:
            _native.actions_to_pd(act, pd, off, scale, frozen)
            _native.physics_step(env_c, pd, device_model.table, phys.params)
        torch.cuda.synchronize()
        outs.append((rb, dof, force, pd))
    for x, y in zip(*outs):
        assert torch.equal(x, y)
