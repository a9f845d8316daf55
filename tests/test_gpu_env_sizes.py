"""Env-step parity with the oracle at the BASELINE sizes (VERDICT r1 "parity at fixture sizes
only"): multi-step PHCPufferEnv.step at the kernel level with in-launch resets, compared with
oracle/phc_oracle.py env_step on the same pre-step state (needs an MI355X).

  * C2: 1024 envs on ONE shared clip — every env gathers the same frame rows;
  * C3: 4096 envs, 4096 clips;
  * ragged 1001 and 4095 envs: the last 8-env workgroup is partial (grid_envs tail).

Tolerances as north_star states them: obs / reward within 1e-5 (atol + rtol), reset and
terminate flags bit-exact (rows whose termination distance lies within 1e-6 of the threshold
excluded: a 1-ulp norm difference may flip them), progress / start times exact.
Reference: /root/reference/puffer_phc/envs/humanoid_phc.py:105-172, envs/common.py:23-364."""

import numpy as np
import pytest
import torch

from oracle import phc_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
STEPS = 16


def _oracle_lib(packed):
    fr = packed.frames.cpu().numpy()
    return O.MotionLib(fr[..., 0:3], fr[..., 3:7], packed.local_rot.cpu().numpy(), fr[..., 7:10], fr[..., 10:13],
                       packed.dof_vel.cpu().numpy(), packed.num_frames.cpu().numpy(), packed.fps.cpu().numpy())


def _make(num_envs, num_clips, seed):
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    # short clips (20..60 frames = 0.67..2 s) so pass_time resets occur within STEPS steps
    q, t, c, fps = synthetic_clips(num_clips, 20, 60, seed=seed, device=DEV)
    packed = PackedMotions.from_global_rotations(q, t, c, fps)
    env = PHCPufferEnv(EnvConfig(num_envs=num_envs, seed=seed), motion_data=packed)
    env.reset()
    return env, packed


@pytest.mark.parametrize("num_envs,num_clips", [(1024, 1), (4096, 4096), (1001, 64), (4095, 4095)],
                         ids=["c2_1024_shared_clip", "c3_4096", "ragged_1001", "ragged_4095"])
def test_env_step_parity_at_baseline_sizes(num_envs, num_clips):
    from puffer_phc_amd import _native as N

    env, packed = _make(num_envs, num_clips, seed=num_envs)
    e = env.env
    lib = _oracle_lib(packed)
    ids = e._sampled_motion_ids.cpu().numpy()
    if num_clips == 1:
        assert (ids == 0).all()  # every env reads the same clip's frame rows
    assert ids.max() < num_clips
    resets = 0
    for _ in range(STEPS):
        e.physics.step(e)
        pre = dict(progress=e.progress_buf.cpu().numpy().astype(np.int32), start=e._motion_start_times.cpu().numpy(),
                   off=e._motion_start_times_offset.cpu().numpy(), goff=e._global_offset.cpu().numpy(),
                   rb=e._rigid_body_state.cpu().numpy(), dv=e._dof_vel.cpu().numpy(),
                   df=e.dof_force_tensor.cpu().numpy())
        N.env_step(e._env_c, e._motion_lib.packed.c, e._step_params_auto)
        torch.cuda.synchronize()
        ref = O.env_step(lib, ids, (pre["progress"] + 1).astype(np.int16), pre["start"], pre["off"], pre["goff"],
                         pre["rb"], pre["dv"], pre["df"])
        np.testing.assert_allclose(env.rewards.cpu().numpy(), ref["rew"], atol=1e-5, rtol=1e-5)
        np.testing.assert_allclose(e.reward_raw.cpu().numpy(), ref["reward_raw"], atol=1e-5, rtol=1e-5)
        term, trunc = env.terminals.cpu().numpy(), env.truncations.cpu().numpy()
        ties = np.any(np.abs(ref["reset_dist"] - 0.25) < 1e-6, -1)
        np.testing.assert_array_equal(term[~ties], ref["terminate"][~ties])
        reset = term | trunc
        np.testing.assert_array_equal(reset[~ties], ref["reset"][~ties])
        np.testing.assert_array_equal(env.masks.cpu().numpy(), ~trunc)
        keep = ~reset
        np.testing.assert_allclose(env.observations.cpu().numpy()[keep], ref["obs"][keep], atol=1e-5, rtol=1e-5)
        prog = e.progress_buf.cpu().numpy()
        np.testing.assert_array_equal(prog[keep], pre["progress"][keep] + 1)
        np.testing.assert_array_equal(prog[reset], 0)
        if reset.any():
            resets += int(reset.sum())
            st = e._motion_start_times.cpu().numpy()[reset]
            np.testing.assert_allclose(st * 30, np.round(st * 30), atol=1e-3)
            ms = O.motion_state(lib, ids[reset], st, pre["goff"][reset])
            np.testing.assert_array_equal(e._rigid_body_state.cpu().numpy()[reset][..., 0:3], ms["rg_pos"])
    assert resets > 0


_FUSED_BUFS = ("_rigid_body_state", "_dof_state", "dof_force_tensor", "pd_target", "obs_buf", "rew_buf", "reward_raw",
               "progress_buf", "reset_buf", "_terminate_buf", "_motion_start_times", "_motion_start_times_offset",
               "_global_offset", "_sampled_motion_ids")


@pytest.mark.parametrize("num_envs,num_clips,amp", [(1024, 1, False), (4096, 4096, False), (4096, 4096, True)],
                         ids=["c2_1024_shared_clip", "c3_4096", "c3_4096_amp"])
def test_fused_replay_step_at_baseline_sizes(num_envs, num_clips, amp):
    """The kernel bench.py times (phc_env_step_replay = k_env_step<true, true>: R13 action -> PD map,
    the replay stand-in and the post-physics step in ONE launch) against the three-launch path
    (phc_actions_to_pd -> phc_physics_replay -> phc_env_step, oracle-pinned by the test above) at the
    sizes it is timed at: every buffer bit for bit over 16 PufferEnv steps with auto-resets and
    actions beyond [-1, 1].  The fused run's non-resetting rows are also checked against the oracle
    directly (obs / reward 1e-5, termination exact) from the state the fused launch wrote.
    Reference: /root/reference/puffer_phc/envs/humanoid_phc.py:105-172, clean_pufferl/env.py:90-164."""
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    envs = []
    for fused in (False, True):
        q, t, c, fps = synthetic_clips(num_clips, 20, 60, seed=num_envs + 1, device=DEV)
        packed = PackedMotions.from_global_rotations(q, t, c, fps)
        env = PHCPufferEnv(EnvConfig(num_envs=num_envs, seed=num_envs, use_amp_obs=amp, fused_env_step=fused),
                           motion_data=packed)
        env.reset()
        envs.append(env)
    a, b = envs
    assert a.env.fused_env_step is False and b.env.fused_env_step is True
    lib = _oracle_lib(packed)
    g = torch.Generator(device=DEV).manual_seed(num_envs)
    resets = 0
    for step in range(STEPS):
        eb = b.env
        pre = dict(progress=eb.progress_buf.cpu().numpy().astype(np.int32), start=eb._motion_start_times.cpu().numpy(),
                   off=eb._motion_start_times_offset.cpu().numpy(), goff=eb._global_offset.cpu().numpy(),
                   ids=eb._sampled_motion_ids.cpu().numpy())
        act = torch.randn((num_envs, 69), device=DEV, generator=g) * 1.5
        outs = [env.step(act) for env in envs]
        torch.cuda.synchronize()
        for name in _FUSED_BUFS:
            assert torch.equal(getattr(a.env, name), getattr(eb, name)), (step, name)
        for name in ("terminals", "truncations", "masks", "rewards", "observations"):
            assert torch.equal(getattr(a, name), getattr(b, name)), (step, name)
        if amp:
            assert torch.equal(a.env._amp_obs_buf, eb._amp_obs_buf), step
        assert torch.equal(outs[0][1], outs[1][1])
        # the fused launch against the oracle on the rows it did not re-initialise
        reset = (b.terminals | b.truncations).cpu().numpy()
        resets += int(reset.sum())
        keep = ~reset
        ref = O.env_step(lib, pre["ids"], (pre["progress"] + 1).astype(np.int16), pre["start"], pre["off"], pre["goff"],
                         eb._rigid_body_state.cpu().numpy(), eb._dof_vel.cpu().numpy(),
                         eb.dof_force_tensor.cpu().numpy())
        np.testing.assert_allclose(b.rewards.cpu().numpy()[keep], ref["rew"][keep], atol=1e-5, rtol=1e-5)
        np.testing.assert_allclose(b.observations.cpu().numpy()[keep], ref["obs"][keep], atol=1e-5, rtol=1e-5)
        ties = np.any(np.abs(ref["reset_dist"] - 0.25) < 1e-6, -1)
        np.testing.assert_array_equal(ref["terminate"][keep & ~ties], False)
        np.testing.assert_array_equal(ref["reset"][keep & ~ties], False)
    assert resets > 0
    np.testing.assert_array_equal(b.env.pd_target.cpu().numpy(), O.actions_to_pd(act.cpu().numpy()))


@pytest.mark.parametrize("num_envs,dtype,fused,physics", [(4096, torch.float16, True, "replay"),
                                                          (1001, torch.bfloat16, True, "replay"),
                                                          (1001, torch.float16, False, "replay"),
                                                          (64, torch.float16, True, "articulated")],
                         ids=["c3_f16", "ragged_bf16", "three_launch", "articulated"])
def test_step_writes_obs_operand(num_envs, dtype, fused, physics):
    """R17 fused into the step (HumanoidPHC.set_obs_operand): after every step the [N, 960] operand
    equals phc_obs_half(obs) bit for bit — in-launch auto-resets included — and a reset kernel
    marks it stale (obs_operand_fresh False)."""
    from puffer_phc_amd import _native as N
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(min(num_envs, 512), 20, 60, seed=5, device=DEV)
    env = PHCPufferEnv(EnvConfig(num_envs=num_envs, seed=3, fused_env_step=fused, physics=physics),
                       motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
    env.reset()
    g = torch.Generator(device=DEV).manual_seed(1)
    mean = torch.randn((1, 934), device=DEV, generator=g) * 0.3
    var = torch.rand((1, 934), device=DEV, generator=g) * 2 + 0.05
    opnd = torch.full((num_envs, 960), float("nan"), dtype=dtype, device=DEV)
    env.env.set_obs_operand(opnd, mean, var, 1e-5, 5.0)
    assert not env.env.obs_operand_fresh
    ref = torch.empty_like(opnd)
    resets = 0
    for _ in range(STEPS):
        env.step(torch.randn((num_envs, 69), device=DEV, generator=g) * 0.5)
        assert env.env.obs_operand_fresh
        N.obs_half(env.observations, mean, var, 1e-5, 5.0, ref)
        torch.cuda.synchronize()
        assert torch.equal(opnd.view(torch.int16), ref.view(torch.int16))
        resets += int((env.terminals | env.truncations).sum())
    assert resets > 0
    env.env.reset([0, 1])
    assert not env.env.obs_operand_fresh
