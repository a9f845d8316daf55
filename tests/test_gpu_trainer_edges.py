"""clean_pufferl.train edge configurations (needs an MI355X).

* AMP with minibatch_size < num_envs: the reference gathers b_amp_obs[mb][:amp_mb] and
  b_amp_obs_replay[mb][:amp_mb] (puffer_phc/clean_pufferl/core.py:278-284), which then hold only
  minibatch_size rows each, and calls discriminate on them and on the demo rows separately
  (:337-344).  The agent / demo split of the one-pass logits must follow the rows gathered.
* l2_reg_coef > 0 (core.py:352-359): the L2-init term's gradient must reach the optimizer next
  to the fused minibatch's gradients.
* ragged discriminator row counts (num_envs not a multiple of 64) in the MFMA backward.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _env(num_envs, amp, seed=2):
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(64, 40, 120, seed=3, device=DEV)
    env = PHCPufferEnv(EnvConfig(num_envs=num_envs, seed=seed, use_amp_obs=amp),
                       motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
    env.reset()
    return env


def test_amp_minibatch_smaller_than_num_envs():
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.policies import PHCPolicy, Policy

    env = _env(256, True)
    torch.manual_seed(0)
    policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
    cfg = TrainConfig(batch_size=256 * 8, minibatch_size=128, bptt_horizon=8, precision="bf16",
                      checkpoint_interval=10 ** 9, update_epochs=1)
    comps, info, util = clean_pufferl.create("t", cfg, env.cfg, env, policy)
    clean_pufferl.evaluate(comps, info)
    losses = clean_pufferl.train(comps, info, util)
    # with the split at 2 * num_envs the demo slice was empty: BCE of nothing = NaN
    assert np.isfinite(losses.disc_loss) and losses.disc_loss > 0
    assert 0.0 <= losses.disc_demo_acc <= 1.0 and 0.0 <= losses.disc_agent_acc <= 1.0
    # the reference's two calls on the same rows, on the trained discriminator
    exp, pol = comps.experience, policy.policy
    demo = env.fetch_amp_obs_demo()
    mb = 0
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        rows = pol.discriminate_rows([(exp.amp_obs, exp.b_amp_idx[mb][:256]),
                                      (exp.amp_obs_replay, exp.b_amp_rep_idx[mb][:256]), (demo, None)]).float()
        agent = pol.discriminate(torch.cat([exp.amp_obs[exp.b_amp_idx[mb][:256]],
                                            exp.amp_obs_replay[exp.b_amp_rep_idx[mb][:256]]])).float()
        dem = pol.discriminate(demo).float()
    n_agent = agent.shape[0]
    assert n_agent == 2 * 128 and dem.shape[0] == 256
    torch.testing.assert_close(rows[:n_agent], agent, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(rows[n_agent:], dem, rtol=1e-5, atol=1e-5)


def _snapshot(policy, opt):
    return {k: v.detach().clone() for k, v in policy.state_dict().items()}, opt.state_dict()


def _restore(policy, opt, snap):
    policy.load_state_dict(snap[0])
    opt.load_state_dict(snap[1])


def test_l2_init_regulariser_gradient_reaches_the_update():
    """train() from the same state and the same collected batch, with l2_reg_coef 0 and > 0:
    the parameters must differ (the regulariser's gradient is nonzero once the parameters have
    left their initial values).  A fused backward that STORED its gradients would drop the
    regulariser's, leaving the runs bit-identical."""
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.policies import PHCPolicy, Policy

    env = _env(256, False)
    torch.manual_seed(0)
    policy = Policy(PHCPolicy(env, hidden_size=64, layer_sizes=(128, 64))).to(DEV)
    cfg = TrainConfig(batch_size=256 * 8, minibatch_size=512, bptt_horizon=8, checkpoint_interval=10 ** 9,
                      update_epochs=2, learning_rate=1e-3)
    comps, info, util = clean_pufferl.create("t", cfg, env.cfg, env, policy)
    clean_pufferl.evaluate(comps, info)
    policy.policy.update_obs_rms(comps.experience.obs)
    snap = _snapshot(policy, comps.optimizer)
    # one untracked train to move the parameters away from their initial values
    clean_pufferl.train(comps, info, util)
    moved = _snapshot(policy, comps.optimizer)
    finals = {}
    for coef in (0.0, 50.0, 100.0):
        _restore(policy, comps.optimizer, moved)
        cfg.l2_reg_coef = coef
        losses = clean_pufferl.train(comps, info, util)
        assert np.isfinite(losses.policy_loss)
        finals[coef] = torch.cat([p.detach().reshape(-1).clone() for p in policy.parameters() if p.requires_grad])
    cfg.l2_reg_coef = 0.0
    d1 = (finals[50.0] - finals[0.0]).norm()
    d2 = (finals[100.0] - finals[0.0]).norm()
    assert float(d1) > 0 and float(d2) > 0, "the L2-init gradient was dropped"
    assert not torch.equal(finals[50.0], finals[100.0])
    del snap


@pytest.mark.parametrize("rows", [1000, 1984])
def test_disc_ragged_rows_backward(rows):
    """MFMA discriminator backward with a row count that is not a multiple of 64: the weight
    gradients (zero-padded 64-row chunks) against fp32 autograd of the module path."""
    from puffer_phc_amd.envs.humanoid_phc import Box
    from puffer_phc_amd.policies import PHCPolicy

    class E:
        single_observation_space = Box(np.full(934, -np.inf), np.full(934, np.inf))
        single_action_space = Box(-np.ones(69), np.ones(69))
        amp_observation_space = Box(np.full(1960, -np.inf), np.full(1960, np.inf))

    torch.manual_seed(0)
    pol = PHCPolicy(E()).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn((rows, 1960), device=DEV, generator=g)
    lab = (torch.arange(rows, device=DEV) % 3 == 0).float()
    from puffer_phc_amd.policies import disc_mlp

    params = disc_mlp.disc_params(pol)

    def run(half):
        for p in params:
            p.grad = None
        ctx = torch.autocast("cuda", dtype=torch.float16) if half else torch.autocast("cuda", enabled=False)
        with ctx:
            lg = pol.discriminate_rows([(x, None)]).float().reshape(-1)
        torch.nn.functional.binary_cross_entropy_with_logits(lg, lab).backward()
        return [p.grad.detach().clone() for p in params]

    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        ref = run(False)
    finally:
        torch.set_float32_matmul_precision(prev)
    got = run(True)
    for a, b in zip(got, ref):
        rel = float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))
        assert rel < 3e-2, rel


def test_adversarial_reward_propagates_nan():
    """torch.maximum(1 - prob, 1e-4) keeps a NaN logit's NaN (reference core.py:237-239): the
    kernel must not clamp it to a finite reward."""
    from puffer_phc_amd import _native as N

    h = torch.ones((64, 512), dtype=torch.float16, device=DEV)
    w = torch.full((512,), 0.01, device=DEV)
    w[3] = float("nan")
    b = torch.zeros(1, device=DEV)
    reward = torch.empty(64, device=DEV)
    N.disc_head_fwd(h, w, b, reward=reward)
    assert torch.isnan(reward).all()


def test_deferred_loss_readback_matches_synchronous(monkeypatch):
    """train() returns PendingLossComponents (a non-blocking copy of the loss row into pinned memory
    plus its event).  The first read waits on that event only; its values must equal the row read
    after a full device synchronisation, field by field, and dataclasses.asdict must see them."""
    import dataclasses

    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.clean_pufferl import structs
    from puffer_phc_amd.clean_pufferl.core import _fill_losses
    from puffer_phc_amd.config import TrainConfig
    from puffer_phc_amd.policies import PHCPolicy, Policy

    hosts = []
    orig = structs.PendingLossComponents.__init__

    def spy(self, host, event, fill):
        hosts.append(host)
        orig(self, host, event, fill)

    monkeypatch.setattr(structs.PendingLossComponents, "__init__", spy)
    env = _env(256, False)
    torch.manual_seed(0)
    policy = Policy(PHCPolicy(env)).to(DEV)  # full widths: the fused f16 minibatch path
    cfg = TrainConfig(batch_size=256 * 32, minibatch_size=2048, bptt_horizon=8, checkpoint_interval=10 ** 9,
                      update_epochs=1)
    comps, info, util = clean_pufferl.create("t", cfg, env.cfg, env, policy)
    clean_pufferl.evaluate(comps, info)
    losses = clean_pufferl.train(comps, info, util)
    assert isinstance(losses, structs.PendingLossComponents) and len(hosts) == 1
    got = dataclasses.asdict(losses)  # first read: waits on the event alone
    torch.cuda.synchronize()
    ref = structs.LossComponents()
    _fill_losses(ref, hosts[0].numpy())
    exp = dataclasses.asdict(ref)
    for k, v in exp.items():
        np.testing.assert_equal(got[k], v, err_msg=k)
    assert np.isfinite([got["policy_loss"], got["value_loss"], got["entropy"]]).all()
    assert vars(losses)["approx_kl"] == exp["approx_kl"]
