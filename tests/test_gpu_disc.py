"""R22: the AMP discriminator on the hand-written MFMA path (policies/disc_mlp.py, phc_disc.hip,
phc_twin_gemm BIAS_RELU / RELU_GRAD) vs torch (needs an MI355X).

Reference: puffer_phc/policies/discriminator_policy.py:43-53, 72-79 (RunningNorm(1960) ->
Linear(1960, 1024) + ReLU -> Linear(1024, 512) + ReLU -> Linear(512, 1)) and
clean_pufferl/core.py:229-242 (adversarial reward), :336-347 (BCE discriminator loss).

Two references per check:
  * "emulated": float64 torch with the operands rounded exactly where the MFMA path rounds them
    (normalised input, weights, both ReLU outputs, the two input gradients) -- isolates the kernels'
    arithmetic (fp32 accumulation order only): rel. L2 <= 1e-4 / 5e-4 (fp16 / bf16) for the logits,
    5e-4 / 2e-3 for every gradient (an fp32-vs-float64 difference can flip the rounding of a stored
    f16 / bf16 activation or input gradient, each flip one operand ulp, and layers compound them);
  * "fp32": the unrounded reference math (the reference's own precision) -- bounds what the half
    operands cost: rel. L2 <= 3e-3 (fp16) / 3e-2 (bf16).
The adversarial reward is checked against the reference's formula applied to the same logits
(fp32, atol 1e-5 / rtol 1e-5), over logits from -16 to 16 so the 1e-4 clamp is exercised."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
REL_FP32 = {torch.float16: 3e-3, torch.bfloat16: 3e-2}
REL_EMU = {torch.float16: (1e-4, 5e-4), torch.bfloat16: (5e-4, 2e-3)}  # (logits, gradients)


class _Env:
    def __init__(self):
        from puffer_phc_amd.envs.humanoid_phc import Box

        self.single_observation_space = Box(np.full(934, -np.inf), np.full(934, np.inf))
        self.single_action_space = Box(-np.ones(69), np.ones(69))
        self.amp_observation_space = Box(np.full(1960, -np.inf), np.full(1960, np.inf))


def _policy(seed=0):
    from puffer_phc_amd.policies import PHCPolicy

    torch.manual_seed(seed)
    pol = PHCPolicy(_Env(), hidden_size=512).to(DEV)  # the reference's full widths
    g = torch.Generator(device=DEV).manual_seed(seed + 1)
    with torch.no_grad():
        n = pol.amp_obs_norm
        n.running_mean.copy_(0.3 * torch.randn(n.running_mean.shape, device=DEV, generator=g))
        n.running_var.copy_(0.5 + torch.rand(n.running_var.shape, device=DEV, generator=g))
        # biases away from zero so the ReLU masks are non-trivial on both sides
        for lin in (pol._disc_mlp[0], pol._disc_mlp[2], pol._disc_logits):
            lin.bias.copy_(0.05 * torch.randn(lin.bias.shape, device=DEV, generator=g))
    return pol


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _reference(pol, x, n_agent, dtype):
    """logits, BCE loss and parameter gradients in float64; dtype=None: unrounded (the fp32
    reference math), else operands rounded where the MFMA path rounds them (bias gradients from
    the unrounded products, as the epilogues sum them before rounding the operand they store)."""
    rd = (lambda t: t.to(dtype).double()) if dtype is not None else (lambda t: t)
    n = pol.amp_obs_norm
    if dtype is not None:  # the kernel normalises in fp32, then rounds
        xn = rd(torch.clamp((x - n.running_mean) / torch.sqrt(n.running_var + n.epsilon), -n.clip, n.clip))
    else:
        xn = torch.clamp((x.double() - n.running_mean.double()) / torch.sqrt(n.running_var.double() + n.epsilon),
                         -n.clip, n.clip)
    l1, l2, l3 = pol._disc_mlp[0], pol._disc_mlp[2], pol._disc_logits
    W1, W2 = rd(l1.weight.detach().double()), rd(l2.weight.detach().double())
    b1, b2 = l1.bias.detach().double(), l2.bias.detach().double()
    w3, b3 = l3.weight.detach().double().reshape(-1), l3.bias.detach().double()
    h1 = rd(torch.relu(xn @ W1.t() + b1))
    h2 = rd(torch.relu(h1 @ W2.t() + b2))
    logits = h2 @ w3 + b3
    la, ld = logits[:n_agent], logits[n_agent:]
    bce = torch.nn.functional.binary_cross_entropy_with_logits
    loss = 0.5 * (bce(la, torch.zeros_like(la)) + bce(ld, torch.ones_like(ld)))
    sg = torch.sigmoid(logits)
    gl = torch.cat([0.5 * sg[:n_agent] / n_agent, 0.5 * (sg[n_agent:] - 1) / ld.numel()])
    v2 = gl[:, None] * w3[None] * (h2 > 0)
    g2 = rd(v2)
    v1 = (g2 @ W2) * (h1 > 0)
    g1 = rd(v1)
    grads = [g1.t() @ xn[:, :W1.shape[1]], v1.sum(0), g2.t() @ h1, v2.sum(0), (gl @ h2)[None], gl.sum().reshape(1)]
    return logits, loss, grads


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_disc_logits_loss_grads(dtype):
    from puffer_phc_amd.policies import disc_mlp

    pol = _policy()
    g = torch.Generator(device=DEV).manual_seed(7)
    n_agent, n_demo = 2048, 1024  # (agent + replay rows, demo rows) as core.py:336-344 at 1024 envs
    src = torch.randn((3000, 1960), device=DEV, generator=g)
    idx = torch.randint(0, 3000, (n_agent,), device=DEV, generator=g)
    demo = torch.randn((n_demo, 1960), device=DEV, generator=g) * 1.5 + 0.2
    params = disc_mlp.disc_params(pol)
    for p in params:
        p.grad = None
    with torch.autocast("cuda", dtype=dtype):
        assert disc_mlp.mfma_disc_supported(pol, dtype)
        logits = pol.discriminate_rows([(src, idx), (demo, None)]).float().reshape(-1)
    bce = torch.nn.BCEWithLogitsLoss()
    loss = 0.5 * (bce(logits[:n_agent], torch.zeros(n_agent, device=DEV))
                  + bce(logits[n_agent:], torch.ones(n_demo, device=DEV)))
    loss.backward()
    got = [p.grad.clone() for p in params]

    x = torch.cat([src[idx], demo])
    lo_e, loss_e, gr_e = _reference(pol, x, n_agent, dtype)
    lo_f, loss_f, gr_f = _reference(pol, x, n_agent, None)
    names = ["w1", "b1", "w2", "b2", "w_logits", "b_logits"]
    tl, tg = REL_EMU[dtype]
    assert _rel(logits, lo_e) < tl, _rel(logits, lo_e)
    assert abs(float(loss.detach()) - float(loss_e)) < 1e-5 * max(1.0, float(loss_e))
    for nm, a, b in zip(names, got, gr_e):
        assert a.shape == b.shape, nm
        assert _rel(a, b) < tg, (nm, _rel(a, b))
    tol = REL_FP32[dtype]
    assert _rel(logits, lo_f) < tol, _rel(logits, lo_f)
    for nm, a, b in zip(names, got, gr_f):
        assert _rel(a, b) < 10 * tol, (nm, _rel(a, b))  # gradients: products of two rounded paths


def test_discriminate_matches_fp32_module_path():
    """discriminate() under autocast (MFMA path) vs the same call in fp32 (the nn.Linear modules,
    the reference's code path)."""
    pol = _policy(3)
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn((1000, 1960), device=DEV, generator=g)  # ragged row count (not a tile multiple)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        with torch.no_grad():
            ref = pol.discriminate(x).float()
            with torch.autocast("cuda", dtype=torch.float16):
                got = pol.discriminate(x).float()
    finally:
        torch.set_float32_matmul_precision(prev)
    assert got.shape == ref.shape == (1000, 1)
    assert _rel(got, ref) < REL_FP32[torch.float16]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_adversarial_reward_formula(dtype):
    """phc_disc_head_fwd's reward equals the reference's expression on the kernel's own logits,
    from deep negative to saturated positive logits (1 - sigmoid < 1e-4: the clamp)."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(11)
    R, H = 4096, 512
    h = torch.relu(torch.randn((R, H), device=DEV, generator=g)).to(dtype)
    w = torch.randn(H, device=DEV, generator=g) * 0.05
    base = (h.float() @ w)
    b = torch.zeros(1, device=DEV)
    logits = torch.empty(R, device=DEV)
    reward = torch.empty(R, device=DEV)
    N.disc_head_fwd(h, w, b, logits=logits, reward=reward)
    torch.testing.assert_close(logits, base, rtol=1e-5, atol=1e-4)
    b2 = torch.zeros(1, device=DEV)
    out_l = torch.empty(R, device=DEV)
    out_r = torch.empty(R, device=DEV)
    # one bias per call: walk a few shifts so both tails and the middle are covered
    for s in (-16.0, -4.0, 0.0, 4.0, 9.5, 16.0):
        b2.fill_(s)
        N.disc_head_fwd(h, w, b2, logits=out_l, reward=out_r)
        prob = 1 / (1 + torch.exp(-out_l))
        ref = -torch.log(torch.maximum(1 - prob, torch.tensor(0.0001, device=DEV)))
        torch.testing.assert_close(out_r, ref, rtol=1e-5, atol=1e-5)
    assert float(out_r.max()) == pytest.approx(-np.log(1e-4), rel=1e-6)  # clamp reached at +16


def test_adversarial_reward_matches_reference_loop():
    """DiscriminatorPolicy.adversarial_reward over index-gathered rows equals the reference's
    per-minibatch loop (core.py:229-242) run on the same policy under the same autocast."""
    pol = _policy(2)
    g = torch.Generator(device=DEV).manual_seed(9)
    amp = torch.randn((4096, 1960), device=DEV, generator=g)
    b_flat = torch.randperm(4096, device=DEV, generator=g).reshape(4, 1024)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        got = pol.adversarial_reward([(amp, b_flat.reshape(-1))]).view(4, 1024)
        ref = torch.zeros((4, 1024), device=DEV)
        for mb in range(4):
            lg = pol.discriminate(amp[b_flat[mb]]).squeeze().float()
            prob = 1 / (1 + torch.exp(-lg))
            ref[mb] = -torch.log(torch.maximum(1 - prob, torch.tensor(0.0001, device=DEV)))
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


def test_amp_bf16_ppo_iteration_full_widths():
    """C5 on one GPU: AMP obs + bf16 MFMA policy AND discriminator at the reference's full widths
    (hidden 512, trunk 2048-1536-1024-1024-512-512, disc 1024-512), one PPO iteration end to end."""
    from puffer_phc_amd import clean_pufferl
    from puffer_phc_amd.clean_pufferl.env import PHCPufferEnv
    from puffer_phc_amd.config import EnvConfig, TrainConfig
    from puffer_phc_amd.motion_lib import PackedMotions
    from puffer_phc_amd.policies import PHCPolicy, Policy
    from puffer_phc_amd.synthetic import synthetic_clips

    q, t, c, fps = synthetic_clips(64, 40, 120, seed=3, device=DEV)
    env = PHCPufferEnv(EnvConfig(num_envs=256, seed=2, use_amp_obs=True),
                       motion_data=PackedMotions.from_global_rotations(q, t, c, fps))
    env.reset()
    torch.manual_seed(0)
    policy = Policy(PHCPolicy(env)).to(DEV)
    pol = policy.policy
    assert pol.use_amp_obs and pol._disc_mlp[0].weight.shape == (1024, 1960)
    cfg = TrainConfig(batch_size=256 * 32, minibatch_size=2048, bptt_horizon=8, precision="bf16",
                      checkpoint_interval=10 ** 9)
    comps, info, util = clean_pufferl.create("t", cfg, env.cfg, env, policy)
    clean_pufferl.evaluate(comps, info)
    assert comps.experience.amp_obs.abs().sum() > 0
    before = {k: v.detach().clone() for k, v in policy.named_parameters()}
    losses = clean_pufferl.train(comps, info, util)
    assert np.isfinite([losses.policy_loss, losses.value_loss, losses.disc_loss]).all() and losses.disc_loss > 0
    assert 0.0 <= losses.disc_agent_acc <= 1.0 and 0.0 <= losses.disc_demo_acc <= 1.0
    after = dict(policy.named_parameters())
    for k in ("_disc_mlp.0.weight", "_disc_mlp.2.weight", "_disc_logits.weight"):
        kk = [n for n in before if n.endswith(k)]
        assert kk and not torch.equal(before[kk[0]], after[kk[0]]), k
