"""train()'s minibatch loop replayed from one captured hipGraph (clean_pufferl.core
._train_minibatches_graphed) against the eager loop of the same launches: two trainers built from
the same seeds run the same iterations, one with the train graph (eager on first sight, captured on
the second eligible call, replayed after), one without.  Parameters, Adam moments, the loss-scaler
state and every logged loss must stay bit-identical, including across a learning-rate change between
replays (the graph reads the rate from the device state).  Reference: core.py:206-440."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _trainer(amp=False):
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(64, 20, 90, seed=7, device=DEV)
    env = PHCPufferEnv(EnvConfig(num_envs=64, seed=4, use_amp_obs=amp),
                       motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
    env.reset()
    torch.manual_seed(0)
    policy = Policy(PHCPolicy(env, hidden_size=512, layer_sizes=(256, 128))).to(DEV)
    cfg = TrainConfig(batch_size=64 * 16, minibatch_size=256, bptt_horizon=8, checkpoint_interval=10 ** 9)
    comps, info, _ = clean_pufferl.create("t", cfg, env.cfg, env, policy)
    return clean_pufferl, comps, info, policy


def _iterate(cp, comps, info, policy, seed):
    torch.manual_seed(seed)  # the rollout's action noise: the same draws for both trainers
    cp.evaluate(comps, info)
    policy.policy.update_obs_rms(comps.experience.obs)
    losses = cp.train(comps, info)
    torch.cuda.synchronize()
    return {k: float(getattr(losses, k)) for k in ("policy_loss", "value_loss", "entropy", "approx_kl", "clipfrac",
                                                   "before_clip_grad_norm", "l2_init_reg_loss", "mean_bound_loss",
                                                   "explained_variance", "disc_loss", "disc_agent_acc",
                                                   "disc_demo_acc")}


@pytest.mark.parametrize("amp", [False, True])
def test_graphed_train_matches_eager(monkeypatch, amp):
    """amp: the C5 configuration (AMP obs): the advantage pass with the adversarial reward and the
    replay buffer's counter-based refresh graphed, then the minibatch loop with the discriminator's
    agent / replay / demo rows, its BCE terms and the per-minibatch loss row (core.py:229-242,
    336-347, 394-395) — captured once that pass replays (the fourth call), replayed from the fifth."""
    from puffer_phc_amd.clean_pufferl import core

    eager = _trainer(amp)
    graphed = _trainer(amp)
    for it in range(8 if amp else 6):
        if it == 4:  # a schedule step between replays (scripts/train.py decays the rate each epoch)
            for tr in (eager, graphed):
                tr[1].optimizer.param_groups[0]["lr"] *= 0.5
        monkeypatch.setattr(core, "TRAIN_GRAPH", False)
        la = _iterate(*eager, seed=100 + it)
        monkeypatch.setattr(core, "TRAIN_GRAPH", True)
        lb = _iterate(*graphed, seed=100 + it)
        for k in la:
            assert (la[k] == lb[k]) or (la[k] != la[k] and lb[k] != lb[k]), (it, k, la[k], lb[k])
        pa = dict(eager[3].named_parameters())
        for n, p in graphed[3].named_parameters():
            assert torch.equal(p, pa[n]), (it, n)
        oa, ob = eager[1].optimizer, graphed[1].optimizer
        assert torch.equal(oa.exp_avg, ob.exp_avg) and torch.equal(oa.exp_avg_sq, ob.exp_avg_sq), it
        assert torch.equal(oa._state, ob._state), it
    st = graphed[1].__dict__.get("_train_graph")
    assert st is not None and st["graph"] is not None and not st["failed"]
    assert eager[1].__dict__.get("_train_graph") is None


def test_graphed_train_follows_parameter_writes_between_replays(monkeypatch):
    """A parameter write outside the captured Adam steps between two replays (here a policy
    load_state_dict of perturbed weights, as a checkpoint restore does; also a changed Adam eps and
    betas) must reach the replayed update: the graph's first minibatch reads the GEMM operand copies,
    which the replay path re-packs when they went stale, and the optimizer's by-value
    hyper-parameters are part of the graph key.  Bit-equal to the eager trainer after the write."""
    from puffer_phc_amd.clean_pufferl import core

    eager = _trainer()
    graphed = _trainer()
    for it in range(7):
        if it == 4:  # after the graph has been captured (call 2) and replayed (call 3)
            st = graphed[1].__dict__.get("_train_graph")
            assert st is not None and st["graph"] is not None
            g = torch.Generator(device=DEV).manual_seed(11)
            sd = {k: v.clone() for k, v in eager[3].state_dict().items()}
            for k, v in sd.items():
                if v.is_floating_point() and "running" not in k and "weight" in k:
                    v.add_(torch.randn(v.shape, generator=g, device=DEV) * 1e-3)
            for tr in (eager, graphed):
                tr[3].load_state_dict(sd)
        if it == 5:
            for tr in (eager, graphed):
                pg = tr[1].optimizer.param_groups[0]
                pg["eps"], pg["betas"] = 1e-6, (0.85, 0.99)
        monkeypatch.setattr(core, "TRAIN_GRAPH", False)
        la = _iterate(*eager, seed=200 + it)
        monkeypatch.setattr(core, "TRAIN_GRAPH", True)
        lb = _iterate(*graphed, seed=200 + it)
        for k in la:
            assert (la[k] == lb[k]) or (la[k] != la[k] and lb[k] != lb[k]), (it, k, la[k], lb[k])
        pa = dict(eager[3].named_parameters())
        for n, p in graphed[3].named_parameters():
            assert torch.equal(p, pa[n]), (it, n)
