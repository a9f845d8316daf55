"""R16 AMP observations on the HIP path vs the reference's golden vectors and the oracle
(needs an MI355X).  Tolerance: float32 within atol 1e-5, rtol 1e-5 (BASELINE north_star)."""

import numpy as np
import pytest
import torch

from oracle import phc_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = dict(atol=1e-5, rtol=1e-5)


def _oracle_lib(packed):
    fr = packed.frames.cpu().numpy()
    return O.MotionLib(fr[..., 0:3], fr[..., 3:7], packed.local_rot.cpu().numpy(), fr[..., 7:10], fr[..., 10:13],
                       packed.dof_vel.cpu().numpy(), packed.num_frames.cpu().numpy(), packed.fps.cpu().numpy())


def test_amp_frame_matches_reference_golden(golden):
    """Sim buffers set to the golden reference states (build_amp_observations_smpl inputs of
    HumanoidPHC._get_amp_obs): the kernel's current frame equals the reference's amp obs."""
    from puffer_phc_amd import _native as N

    g = golden("amp_obs")
    n = g["amp_obs"].shape[0]
    rb = np.concatenate([g["ref_rg_pos"], g["ref_rb_rot"], g["ref_body_vel"], g["ref_body_ang_vel"]], -1)
    dof = np.stack([g["ref_dof_pos"], g["ref_dof_vel"]], -1)
    f = lambda x, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(x)).to(DEV, dt)  # noqa: E731
    rb_t, dof_t = f(rb), f(dof)
    prog = torch.ones(n, dtype=torch.int16, device=DEV)  # not a reset env: shift + current frame
    ids = torch.zeros(n, dtype=torch.int64, device=DEV)
    st = torch.zeros(n, device=DEV)
    z3 = torch.zeros((n, 3), device=DEV)
    env_c = N.env_struct(n, rb_t, None, dof_t, torch.zeros((n, 69), device=DEV), prog, ids, st, st.clone(), z3,
                         torch.zeros((n, 934), device=DEV), torch.zeros(n, device=DEV), torch.zeros((n, 5), device=DEV),
                         torch.zeros(n, dtype=torch.bool, device=DEV), torch.zeros(n, dtype=torch.bool, device=DEV))
    m = golden("motion_lib")
    frames = f(np.concatenate([m["gts"], m["grs"], m["gvs"], m["gavs"]], -1))
    lrs, dvs = f(m["lrs"]), f(m["dvs"])
    mlen, mdt = f(m["motion_lengths"]), f(m["motion_dt"])
    nf, ls = f(m["motion_num_frames"], torch.int64), f(m["length_starts"], torch.int64)
    lib_c = N.motion_lib_struct(frames, lrs, dvs, mlen, mdt, nf, ls)
    amp = torch.full((n, 3, 196), 7.0, device=DEV)
    amp[:, 0] = 1.0
    amp[:, 1] = 2.0
    demo = torch.zeros_like(amp)
    N.amp_obs(env_c, lib_c, N.amp_struct(amp, demo), O.DT, N.AMP_STEP)
    out = amp.cpu().numpy()
    np.testing.assert_allclose(out[:, 0], g["amp_obs"], **TOL)
    assert (out[:, 1] == 1.0).all() and (out[:, 2] == 2.0).all()  # history shifted by one frame
    assert (demo.cpu().numpy() == 0).all()  # demo only written on init
    # the oracle restatement agrees with the same golden vector
    np.testing.assert_allclose(O.amp_obs_from_sim(rb, g["ref_dof_pos"], g["ref_dof_vel"]), g["amp_obs"], **TOL)


@pytest.fixture(scope="module")
def amp_env():
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(64, 20, 90, seed=9, device=DEV)
    packed = PackedMotions.from_global_rotations(q, t, c, fps)
    env = PHCPufferEnv(EnvConfig(num_envs=64, seed=4, use_amp_obs=True), motion_data=packed)
    env.reset()
    return env, packed


def _state(e):
    return dict(rb=e._rigid_body_state.cpu().numpy(), dp=e._dof_pos.cpu().numpy(), dv=e._dof_vel.cpu().numpy(),
                prog=e.progress_buf.cpu().numpy(), ids=e._sampled_motion_ids.cpu().numpy(),
                st=e._motion_start_times.cpu().numpy())


def test_amp_init_and_steps_match_oracle(amp_env):
    """After reset every env's 10-frame window (sim frame + 9 motion-library frames) and the
    demo buffer match the oracle; then 25 PHCPufferEnv steps (with in-launch resets) keep the
    shifted history equal to the oracle's _update_hist_amp_obs/_init_amp_obs composition."""
    env, packed = amp_env
    e = env.env
    lib = _oracle_lib(packed)
    assert env.amp_obs.shape == (64, 1960) and env.fetch_amp_obs_demo().shape == (64, 1960)
    s = _state(e)
    assert (s["prog"] == 0).all()
    amp = np.zeros((64, 10, 196), np.float32)
    demo = np.zeros_like(amp)
    O.amp_update(amp, demo, lib, s["rb"], s["dp"], s["dv"], s["prog"], s["ids"], s["st"], O.DT, init_only=True)
    np.testing.assert_allclose(e._amp_obs_buf.cpu().numpy(), amp, **TOL)
    np.testing.assert_allclose(e._amp_obs_demo_buf.cpu().numpy(), demo, **TOL)
    seen_reset = 0
    g = torch.Generator(device=DEV)
    g.manual_seed(0)
    for _ in range(25):
        env.step(torch.rand((64, 69), device=DEV, generator=g) * 2 - 1)
        s = _state(e)
        seen_reset += int((s["prog"] == 0).sum())
        O.amp_update(amp, demo, lib, s["rb"], s["dp"], s["dv"], s["prog"], s["ids"], s["st"], O.DT, init_only=False)
        np.testing.assert_allclose(e._amp_obs_buf.cpu().numpy(), amp, **TOL)
        np.testing.assert_allclose(e._amp_obs_demo_buf.cpu().numpy(), demo, **TOL)
        np.testing.assert_array_equal(env.amp_obs.cpu().numpy(), e._amp_obs_buf.cpu().numpy().reshape(64, -1))
    assert seen_reset > 0


def test_amp_ppo_iteration(amp_env):
    """use_amp_obs end to end: rollout stores amp obs, the discriminator reward enters GAE and
    the BCE discriminator loss trains (clean_pufferl/core.py:229-242, 319-333)."""
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.policies import PHCPolicy, Policy

    env, _ = amp_env
    torch.manual_seed(0)
    policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
    assert policy.policy.use_amp_obs
    cfg = TrainConfig(batch_size=64 * 16, minibatch_size=256, bptt_horizon=8, checkpoint_interval=10 ** 9)
    comps, info, util = clean_pufferl.create("t", cfg, env.cfg, env, policy)
    clean_pufferl.evaluate(comps, info)
    exp = comps.experience
    assert exp.amp_obs.abs().sum() > 0
    policy.policy.update_obs_rms(exp.obs)
    before = {k: v.detach().clone() for k, v in policy.named_parameters()}
    losses = clean_pufferl.train(comps, info, util)
    assert np.isfinite([losses.policy_loss, losses.value_loss, losses.disc_loss]).all() and losses.disc_loss > 0
    disc = [k for k in before if "disc" in k]
    assert disc and any(not torch.equal(before[k], dict(policy.named_parameters())[k]) for k in disc)
