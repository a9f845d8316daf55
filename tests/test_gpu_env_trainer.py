"""End-to-end HIP path: motion-library build, multi-step env parity with the oracle (including
in-launch resets), and the on-device PPO trainer (needs an MI355X)."""

import numpy as np
import pytest
import torch

from oracle import phc_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _oracle_lib(packed):
    fr = packed.frames.cpu().numpy()
    return O.MotionLib(fr[..., 0:3], fr[..., 3:7], packed.local_rot.cpu().numpy(), fr[..., 7:10], fr[..., 10:13],
                       packed.dof_vel.cpu().numpy(), packed.num_frames.cpu().numpy(),
                       packed.fps.cpu().numpy())


@pytest.fixture(scope="module")
def small_env():
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(64, 20, 90, seed=5, device=DEV)
    packed = PackedMotions.from_global_rotations(q, t, c, fps)
    env = PHCPufferEnv(EnvConfig(num_envs=64, seed=3), motion_data=packed)
    env.reset()
    return env, packed, (q.cpu().numpy(), t.cpu().numpy(), c.cpu().numpy())


def test_fk_library_vs_oracle(small_env):
    from puffer_phc_amd.skeleton import SkeletonTree

    env, packed, (q, t, c) = small_env
    sk = SkeletonTree.smpl()
    starts = np.concatenate([[0], np.cumsum(c)[:-1]])
    fr = packed.frames.cpu().numpy()
    for m in (0, 17, 63):
        sl = slice(starts[m], starts[m] + c[m])
        out = O.fk_motion(sk.parent_indices.numpy(), sk.local_translation.numpy(), q[sl], t[sl], fps=30)
        np.testing.assert_allclose(fr[sl, :, 0:3], out["gts"], atol=2e-5, rtol=1e-5)
        np.testing.assert_allclose(fr[sl, :, 7:10], out["gvs"], atol=2e-5, rtol=1e-5)
        np.testing.assert_allclose(fr[sl, :, 10:13], out["gavs"], atol=2e-5, rtol=1e-5)
        np.testing.assert_allclose(packed.local_rot[sl].cpu().numpy(), out["lrs"], atol=1e-6)
        np.testing.assert_allclose(packed.dof_vel[sl].cpu().numpy(), out["dvs"], atol=2e-5, rtol=1e-5)


def test_multi_step_parity_with_resets(small_env):
    """20 steps of PHCPufferEnv.step at the kernel level: every env's reward/obs/flags match the
    oracle; envs that reset are re-initialised at a 1/30-snapped time with the old offset."""
    from puffer_phc_amd import _native as N

    env, packed, _ = small_env
    e = env.env
    lib = _oracle_lib(packed)
    ids = e._sampled_motion_ids.cpu().numpy()
    seen_reset = 0
    for step in range(20):
        e.physics.step(e)  # replay physics writes rigid bodies / dof state
        pre = dict(progress=e.progress_buf.cpu().numpy().astype(np.int32), start=e._motion_start_times.cpu().numpy(),
                   off=e._motion_start_times_offset.cpu().numpy(), goff=e._global_offset.cpu().numpy(),
                   rb=e._rigid_body_state.cpu().numpy(), dv=e._dof_vel.cpu().numpy(),
                   df=e.dof_force_tensor.cpu().numpy())
        N.env_step(e._env_c, e._motion_lib.packed.c, e._step_params_auto)
        torch.cuda.synchronize()
        ref = O.env_step(lib, ids, (pre["progress"] + 1).astype(np.int16), pre["start"], pre["off"], pre["goff"],
                         pre["rb"], pre["dv"], pre["df"])
        rew = env.rewards.cpu().numpy()
        np.testing.assert_allclose(rew, ref["rew"], atol=1e-5, rtol=1e-5)
        term = env.terminals.cpu().numpy()
        trunc = env.truncations.cpu().numpy()
        ties = np.any(np.abs(ref["reset_dist"] - 0.25) < 1e-6, -1)
        np.testing.assert_array_equal(term[~ties], ref["terminate"][~ties])
        np.testing.assert_array_equal((term | trunc)[~ties], ref["reset"][~ties])
        obs = env.observations.cpu().numpy()
        reset = term | trunc
        keep = ~reset
        np.testing.assert_allclose(obs[keep], ref["obs"][keep], atol=1e-5, rtol=1e-5)
        if reset.any():
            seen_reset += int(reset.sum())
            st = e._motion_start_times.cpu().numpy()[reset]
            lens = lib.motion_lengths[ids[reset]]
            assert np.all(st >= 0) and np.all(st <= lens + 1e-6)
            np.testing.assert_allclose(st * 30, np.round(st * 30), atol=1e-3)
            # re-initialised state = reference at the new start with the OLD global offset
            ms = O.motion_state(lib, ids[reset], st, pre["goff"][reset])
            rb = e._rigid_body_state.cpu().numpy()[reset]
            np.testing.assert_array_equal(rb[..., 0:3], ms["rg_pos"])
            np.testing.assert_allclose(rb[..., 3:7], ms["rb_rot"], atol=1e-6)
            # obs after reset: progress 0, offsets 0, reference at dt + start
            bp, br, bv, bav = ms["rg_pos"], ms["rb_rot"], ms["body_vel"], ms["body_ang_vel"]
            ms1 = O.motion_state(lib, ids[reset], (np.float32(1) * O.DT + st + np.float32(0)).astype(np.float32),
                                 np.zeros((reset.sum(), 3), np.float32))
            exp = np.concatenate([O.humanoid_obs(bp, br, bv, bav),
                                  O.imitation_obs_v6(bp[:, 0], br[:, 0], bp, br, bv, bav, ms1["rg_pos"], ms1["rb_rot"],
                                                     ms1["body_vel"], ms1["body_ang_vel"])], -1)
            np.testing.assert_allclose(obs[reset], exp, atol=1e-5, rtol=1e-5)
            assert (e.progress_buf[torch.from_numpy(reset).to(DEV)] == 0).all()
    assert seen_reset > 0  # short clips (20..90 frames) must reach pass_time within 20 steps


def test_vecenv_protocol_and_logging(small_env):
    env, _, _ = small_env
    env.async_reset(0)
    for _ in range(env.cfg.log_interval):
        o, r, d, t, info, ids, mask = env.recv()
        env.send(torch.zeros((64, 69), device=DEV))
    _, _, _, _, info, _, _ = env.recv()
    assert info and "rew_body_pos" in info[0] and 0.0 < info[0]["rew_body_pos"] <= 1.0
    assert o.shape == (64, 934) and mask.dtype == torch.bool


def test_ppo_iteration_trains(small_env):
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.policies import PHCPolicy, Policy

    env, _, _ = small_env
    torch.manual_seed(0)
    policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
    cfg = TrainConfig(batch_size=64 * 16, minibatch_size=256, bptt_horizon=8, checkpoint_interval=10 ** 9)
    comps, info, util = clean_pufferl.create("t", cfg, env.cfg, env, policy)
    before = {k: v.detach().clone() for k, v in policy.named_parameters()}
    clean_pufferl.evaluate(comps, info)
    exp = comps.experience
    assert info.global_step >= cfg.batch_size
    policy.policy.update_obs_rms(exp.obs)
    # GAE parity on the trainer's own sorted arrays
    adv = clean_pufferl.core.compute_advantages(comps, info)
    idx = torch.sort(exp.env_ids, stable=True).indices
    ref = O.compute_gae(exp.dones[idx].cpu().numpy(), exp.values[idx].cpu().numpy(),
                        exp.rewards[idx].cpu().numpy(), cfg.gamma, cfg.gae_lambda)
    np.testing.assert_allclose(adv.cpu().numpy(), ref, atol=1e-5, rtol=1e-5)
    env_sorted = exp.env_ids[idx].cpu().numpy()
    assert np.all(np.diff(env_sorted) >= 0)
    losses = clean_pufferl.train(comps, info, util)
    assert np.isfinite([losses.policy_loss, losses.value_loss, losses.approx_kl]).all()
    changed = sum(not torch.equal(before[k], v) for k, v in policy.named_parameters() if v.requires_grad)
    assert changed > 0
    assert float(policy.policy.obs_norm.count) == 2.0


@pytest.mark.parametrize("precision", ["fp16", "bf16", "xf32"])
def test_ppo_iteration_reduced_precision(small_env, precision):
    """TrainConfig.precision fp16 (default; dynamic loss scaling) / bf16 / xf32 (fp32 storage):
    one full PPO iteration stays finite, updates the weights and keeps fp32 master parameters."""
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.policies import PHCPolicy, Policy

    env, _, _ = small_env
    torch.manual_seed(0)
    policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
    cfg = TrainConfig(batch_size=64 * 16, minibatch_size=256, bptt_horizon=8, checkpoint_interval=10 ** 9,
                      precision=precision)
    comps, info, util = clean_pufferl.create("t", cfg, env.cfg, env, policy)
    assert (comps.scaler is not None) == (precision == "fp16")
    before = {k: v.detach().clone() for k, v in policy.named_parameters()}
    clean_pufferl.evaluate(comps, info)
    assert comps.experience.values.dtype == torch.float32
    policy.policy.update_obs_rms(comps.experience.obs)
    losses = clean_pufferl.train(comps, info, util)
    assert np.isfinite([losses.policy_loss, losses.value_loss, losses.approx_kl]).all()
    assert all(v.dtype == torch.float32 for v in policy.parameters())
    changed = sum(not torch.equal(before[k], v) for k, v in policy.named_parameters() if v.requires_grad)
    assert changed > 0
    if precision == "fp16":
        assert int(comps.skipped_steps) >= 0


@pytest.mark.parametrize("use_amp", [False, True])
def test_graph_rollout_matches_eager_loop(use_amp):
    """evaluate() with the captured rollout graph + device experience store fills the buffer
    exactly like the reference's eager loop (same obs / rewards / dones / env ids / values and
    the same global step count), including partial stores of masked (truncated) rows."""
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.synthetic import synthetic_clips

    runs = []
    for graph in (False, True):
        q, t, c, fps = synthetic_clips(64, 12, 40, seed=21, device=DEV)  # short clips: many truncations
        packed = PackedMotions.from_global_rotations(q, t, c, fps)
        env = PHCPufferEnv(EnvConfig(num_envs=64, seed=8, use_amp_obs=use_amp), motion_data=packed)
        torch.manual_seed(0)
        policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
        cfg = TrainConfig(batch_size=64 * 24, minibatch_size=64 * 8, bptt_horizon=8, checkpoint_interval=10 ** 9,
                          rollout_graph=graph)
        comps, info, _ = clean_pufferl.create("t", cfg, env.cfg, env, policy)
        clean_pufferl.evaluate(comps, info)
        steps1 = info.global_step
        clean_pufferl.evaluate(comps, info)  # second call: graph replays only
        e = comps.experience
        runs.append(dict(step=(steps1, info.global_step), obs=e.obs.clone(), rew=e.rewards.clone(),
                         done=e.dones.clone(), trunc=e.truncateds.clone(), ids=e.env_ids.clone(),
                         val=e.values.clone(), amp=e.amp_obs.clone() if use_amp else None,
                         logp=e.logprobs.clone()))
    a, b = runs
    assert a["step"] == b["step"] and a["step"][1] >= 64 * 24 * 2
    for k in ("obs", "rew", "done", "trunc", "ids"):
        assert torch.equal(a[k], b[k]), k
    torch.testing.assert_close(a["val"], b["val"], atol=1e-5, rtol=1e-5)
    if use_amp:
        assert torch.equal(a["amp"], b["amp"])
    assert torch.isfinite(b["logp"]).all()


@pytest.mark.parametrize("amp", [False, True])
def test_fused_replay_step_equals_three_launches(amp):
    """phc_env_step_replay (R13 + the physics stand-in + the env step in one launch) against
    phc_actions_to_pd -> phc_physics_replay -> phc_env_step on identical envs: every buffer bit for
    bit over 30 PufferEnv steps with auto-resets (short clips) and random actions beyond [-1, 1]."""
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    envs = []
    for fused in (False, True):
        q, t, c, fps = synthetic_clips(37, 12, 50, seed=4, device=DEV)
        env = PHCPufferEnv(EnvConfig(num_envs=301, seed=6, use_amp_obs=amp, fused_env_step=fused),
                           motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
        env.reset()
        envs.append(env)
    g = torch.Generator(device=DEV).manual_seed(0)
    resets = 0
    for step in range(30):
        act = torch.randn((301, 69), device=DEV, generator=g) * 1.5
        outs = [env.step(act) for env in envs]
        a, b = envs
        ea, eb = a.env, b.env
        for name in ("_rigid_body_state", "_dof_state", "dof_force_tensor", "pd_target", "obs_buf", "rew_buf",
                     "reward_raw", "progress_buf", "reset_buf", "_terminate_buf", "_motion_start_times"):
            assert torch.equal(getattr(ea, name), getattr(eb, name)), (step, name)
        for name in ("terminals", "truncations", "masks"):
            assert torch.equal(getattr(a, name), getattr(b, name)), (step, name)
        if amp:
            assert torch.equal(ea._amp_obs_buf, eb._amp_obs_buf), step
        resets += int(a.terminals.sum() + a.truncations.sum())
        assert torch.equal(outs[0][1], outs[1][1])
    assert resets > 0
    # the PD targets follow the reference's map (clip, scale, frozen hands / toes)
    ref = O.actions_to_pd(act.cpu().numpy())
    np.testing.assert_array_equal(envs[1].env.pd_target.cpu().numpy(), ref)


def test_rollout_env_written_operand_matches_obs_half():
    """The captured rollout reading the env step's fused RunningNorm operand (fused_obs_operand) vs a
    phc_obs_half launch per step: identical experience buffers over two evaluate() calls with an obs
    RunningNorm update between them (the operand is rebuilt at the start of each evaluate)."""
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.synthetic import synthetic_clips

    runs = []
    for fused_op in (False, True):
        q, t, c, fps = synthetic_clips(64, 12, 40, seed=21, device=DEV)
        env = PHCPufferEnv(EnvConfig(num_envs=128, seed=8), motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
        torch.manual_seed(0)
        policy = Policy(PHCPolicy(env, hidden_size=256, layer_sizes=(256, 256))).to(DEV)
        cfg = TrainConfig(batch_size=128 * 16, minibatch_size=128 * 8, bptt_horizon=8, checkpoint_interval=10 ** 9,
                          fused_obs_operand=fused_op)
        comps, info, _ = clean_pufferl.create("t", cfg, env.cfg, env, policy)
        out = []
        for _ in range(2):
            clean_pufferl.evaluate(comps, info)
            e = comps.experience
            out.append((e.obs.clone(), e.actions.clone(), e.logprobs.clone(), e.values.clone()))
            policy.policy.update_obs_rms(e.obs)
        assert (comps.rollout.opnd is not None) == fused_op
        runs.append(out)
    for (a, b) in zip(*runs):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


@pytest.mark.parametrize("amp", [False, True])
def test_block_rollout_matches_single_step_graphs(monkeypatch, amp):
    """evaluate() with its first min_steps steps replayed as ONE captured block (policy + store + fused
    env step per step, core.RolloutStep.run_block) against one graph per step with the env step eager:
    the same experience rows, the same tick, and the same mean_and_log infos — log points that fall
    inside a block included (log_interval 5 does not divide the 24-step rollouts).  amp: the AMP
    history launch of every step inside the block too, and the AMP rows stored."""
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.clean_pufferl import core
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.synthetic import synthetic_clips

    runs = []
    for block in (False, True):
        monkeypatch.setattr(core, "BLOCK_GRAPH", block)
        q, t, c, fps = synthetic_clips(64, 12, 40, seed=21, device=DEV)  # short clips: many resets
        env = PHCPufferEnv(EnvConfig(num_envs=64, seed=8, log_interval=5, use_amp_obs=amp),
                           motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
        torch.manual_seed(0)
        policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
        cfg = TrainConfig(batch_size=64 * 24, minibatch_size=64 * 8, bptt_horizon=8, checkpoint_interval=10 ** 9)
        comps, info, _ = clean_pufferl.create("t", cfg, env.cfg, env, policy)
        infos = []
        for it in range(4):
            torch.manual_seed(10 + it)
            _, env_infos = clean_pufferl.evaluate(comps, info)
            infos.append({k: [float(x) for x in v] for k, v in env_infos.items()})
        e = comps.experience
        runs.append(dict(step=info.global_step, tick=env.tick, obs=e.obs.clone(), rew=e.rewards.clone(),
                         done=e.dones.clone(), ids=e.env_ids.clone(), infos=infos,
                         amp=e.amp_obs.clone() if amp else e.obs[:0].clone(),
                         blocks=len(getattr(comps.rollout, "_blocks", {}))))
    a, b = runs
    assert a["blocks"] == 0 and b["blocks"] == 1
    assert a["step"] == b["step"] and a["tick"] == b["tick"]
    for k in ("obs", "rew", "done", "ids", "amp"):
        assert torch.equal(a[k], b[k]), k
    for ia, ib in zip(a["infos"], b["infos"]):
        assert ia.keys() == ib.keys()
        for k in ia:
            np.testing.assert_allclose(ia[k], ib[k], rtol=1e-9, atol=1e-12, err_msg=k)


@pytest.mark.parametrize("clip_len", [(12, 40), (400, 500)])
def test_speculative_step_after_block_matches_read_first(monkeypatch, clip_len):
    """core.SPECULATE_STEP: the step after the block is queued before the host reads whether the block
    filled the buffer.  Short clips: rows are masked, the step is needed and kept; long clips: no row
    is masked, the block fills the buffer and the queued step is taken back (mu, the noise buffer and
    the generator state restored, no env step sent).  Either way every experience row, the step and
    tick counts, mu and the generator's next draw equal the read-first loop's, over three evaluates."""
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.clean_pufferl import core
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.envs.state_init import StateInit
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.synthetic import synthetic_clips

    undo = {"n": 0}
    orig_undo = core.RolloutStep.speculate_undo

    def counting_undo(self, saved):
        undo["n"] += 1
        return orig_undo(self, saved)

    monkeypatch.setattr(core.RolloutStep, "speculate_undo", counting_undo)
    runs = []
    for spec in (False, True):
        monkeypatch.setattr(core, "SPECULATE_STEP", spec)
        q, t, c, fps = synthetic_clips(64, clip_len[0], clip_len[1], seed=21, device=DEV)
        init = StateInit.Start if clip_len[0] >= 400 else StateInit.Random  # Start: no clip ends in 72 steps
        env = PHCPufferEnv(EnvConfig(num_envs=64, seed=8, log_interval=5, max_episode_length=10 ** 6, state_init=init),
                           motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
        torch.manual_seed(0)
        policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
        cfg = TrainConfig(batch_size=64 * 24, minibatch_size=64 * 8, bptt_horizon=8, checkpoint_interval=10 ** 9)
        comps, info, _ = clean_pufferl.create("t", cfg, env.cfg, env, policy)
        out = []
        for it in range(3):
            torch.manual_seed(10 + it)
            clean_pufferl.evaluate(comps, info)
            e = comps.experience
            out.append(dict(step=info.global_step, tick=env.tick, obs=e.obs.clone(), act=e.actions.clone(),
                            logp=e.logprobs.clone(), val=e.values.clone(), mu=comps.rollout.mu.clone(),
                            draw=torch.randn(8, device=DEV)))
        runs.append(out)
    for ra, rb in zip(*runs):
        for k in ra:
            if isinstance(ra[k], torch.Tensor):
                assert torch.equal(ra[k], rb[k]), k
            else:
                assert ra[k] == rb[k], k
    assert (undo["n"] > 0) == (clip_len[0] >= 400)


def _dict_clips(n, lo, hi, seed):
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(n, lo, hi, seed=seed, device=DEV)
    qh, th, ch, fh = q.cpu().numpy(), t.cpu().numpy(), c.cpu().numpy(), fps.cpu().numpy()
    ends = np.cumsum(ch)
    return {f"clip_{i:04d}": {"pose_quat_global": qh[ends[i] - ch[i]:ends[i]],
                              "root_trans_offset": torch.from_numpy(th[ends[i] - ch[i]:ends[i]]),
                              "pose_aa": np.zeros((int(ch[i]), 72)), "fps": float(fh[i])} for i in range(n)}


def test_block_rollout_follows_resample(monkeypatch):
    """resample_motions() replaces the packed library the captured block's env-step launches hold by
    value: the block graphs are re-captured under the new library (HumanoidPHC.launch_key), and the
    rollout before and after the resample equals the per-step graphs' bit for bit."""
    import random

    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.clean_pufferl import core
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.policies import PHCPolicy, Policy

    clips = _dict_clips(200, 12, 60, seed=5)
    runs = []
    for block in (False, True):
        monkeypatch.setattr(core, "BLOCK_GRAPH", block)
        torch.manual_seed(1)  # the initial load's crops / headings: the same library in both runs
        random.seed(2)
        np.random.seed(3)
        env = PHCPufferEnv(EnvConfig(num_envs=64, seed=8, log_interval=5, max_episode_length=40), motion_data=clips)
        torch.manual_seed(0)
        policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
        cfg = TrainConfig(batch_size=64 * 24, minibatch_size=64 * 8, bptt_horizon=8, checkpoint_interval=10 ** 9)
        comps, info, _ = clean_pufferl.create("t", cfg, env.cfg, env, policy)
        obs, keys = [], []
        for it in range(5):
            if it == 3:
                torch.manual_seed(99)
                random.seed(98)
                np.random.seed(97)
                env.env.resample_motions()
                env.reset()
            torch.manual_seed(10 + it)
            clean_pufferl.evaluate(comps, info)
            obs.append(comps.experience.obs.clone())
            keys.append(getattr(comps.rollout, "_blocks_key", None))
        runs.append(dict(obs=obs, keys=keys, ids=env.env._motion_lib._curr_motion_ids.clone(), step=info.global_step))
    a, b = runs
    assert torch.equal(a["ids"], b["ids"]) and a["step"] == b["step"]
    assert b["keys"][2] is not None and b["keys"][3] != b["keys"][2] and b["keys"][4] == b["keys"][3]
    for x, y in zip(a["obs"], b["obs"]):
        assert torch.equal(x, y)
