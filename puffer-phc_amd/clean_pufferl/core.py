"""clean_pufferl trainer API (puffer_phc/clean_pufferl/core.py:41-455): create / evaluate /
train / close, with the rollout buffer, GAE (phc_gae) and RMS statistics (phc_rms_*) on the
MI355X, and data parallelism over ranks (distributed.py).

Differences from the reference that do not change the math:
  * actions stay on the device (no .cpu().numpy() round trip per step);
  * GAE runs on the device over the same env-sorted flat arrays (the reference's Cython
    pass on the host, core.py:249);
  * per-parameter grad norms and loss scalars accumulate on the device and are read once
    per train() call instead of ~46 .item() syncs per minibatch;
  * with world_size > 1, gradients are averaged across ranks before clipping and the
    advantage normalisation uses global statistics (see distributed.py).
"""

import contextlib
import os
import time
import warnings
from collections import defaultdict

import numpy as np
import torch

from .. import _native
from .. import distributed as D
from ..optim import FlatAdam
from ..policies import weight_cache
from ..policies.fused_ppo import fused_ppo_loss, fused_ppo_supported
from ..policies.twin_mlp import half_input_width, refresh_twin
from .ppo_loss import ppo_coefs, ppo_objective
from .structs import Experience, LossComponents, PendingLossComponents, Profile, StatsData, TrainComponents, TrainInfo, Utilization
from .utils import count_params, save_checkpoint, seed_everything

# core.py:38 / structs.py:21: "high" float32 matmul precision.  On gfx950 hipBLASLt serves it
# with an xf32-style emulation (measured max rel err ~5e-6 vs float64 on 32768x2048x1536,
# 2x the plain-fp32 rate): at least as precise as the TF32 the reference gets on NVIDIA.
torch.set_float32_matmul_precision("high")


def _l2_init_reg(named_params, initial_params, need_grad):
    """sum_p mean((p - p0)^2) (core.py:352-359).  Logged every minibatch even at coef 0: then it
    is computed without autograd in a few multi-tensor kernels instead of 3 launches/param."""
    names = [n for n, _ in named_params if n in initial_params]
    params = [p for n, p in named_params if n in initial_params]
    inits = [initial_params[n] for n in names]
    if need_grad:
        l2 = torch.zeros((), device=params[0].device)
        for p, p0 in zip(params, inits):
            l2 = l2 + (p - p0).pow(2).mean()
        return l2
    with torch.no_grad():
        diffs = torch._foreach_sub([p.detach() for p in params], inits)
        norms = torch.stack(torch._foreach_norm(diffs))
        key = (params[0].device, len(params))
        if key not in _NUMEL_CACHE:
            _NUMEL_CACHE[key] = torch.tensor([float(p.numel()) for p in params], device=params[0].device)
        return (norms * norms / _NUMEL_CACHE[key]).sum()


_NUMEL_CACHE = {}
# fused minibatch backward stores every gradient (one writer per parameter) instead of adding it,
# so the flat gradient buffer is not zeroed per minibatch (PHC_STORE_GRADS=0: zero + accumulate)
STORE_GRADS = os.environ.get("PHC_STORE_GRADS", "1") == "1"

_AUTOCAST = {"fp16": torch.float16, "bf16": torch.bfloat16}


def autocast(cfg):
    """Policy-GEMM precision context for TrainConfig.precision (see config.py)."""
    if cfg.precision == "xf32":
        return contextlib.nullcontext()
    if cfg.precision not in _AUTOCAST:
        raise ValueError(f"unknown precision {cfg.precision!r} (xf32 | fp16 | bf16)")
    return torch.autocast("cuda", dtype=_AUTOCAST[cfg.precision])


def create(exp_id, train_cfg, env_cfg, vecenv, policy, optimizer=None, wandb=None):
    seed_everything(train_cfg.seed + D.rank(), train_cfg.torch_deterministic)
    profile = Profile()
    utilization = Utilization()
    msg = f"Model Size: {count_params(policy)} parameters"
    vecenv.async_reset(train_cfg.seed)
    obs_shape = vecenv.single_observation_space.shape
    atn_shape = vecenv.single_action_space.shape
    lstm = getattr(policy, "lstm", None)  # RecurrentPolicy: per-env (h, c) buffers (core.py:66-77)
    experience = Experience(train_cfg.batch_size, train_cfg.bptt_horizon, train_cfg.minibatch_size, obs_shape,
                            atn_shape=atn_shape, device=train_cfg.device, use_amp_obs=env_cfg.use_amp_obs,
                            amp_obs_size=getattr(vecenv.amp_observation_space, "shape", (1960,))[0]
                            if env_cfg.use_amp_obs else 1960, lstm=lstm,
                            lstm_total_agents=vecenv.num_agents if lstm is not None else 0)
    D.broadcast_params(policy)
    uncompiled_policy = policy
    if train_cfg.compile:
        policy = torch.compile(policy)
    autocast(train_cfg)  # validates the precision name
    inner = getattr(uncompiled_policy, "policy", uncompiled_policy)
    order = inner.grad_ready_order() if hasattr(inner, "grad_ready_order") else None
    flat_grads = D.FlatGrads(uncompiled_policy.parameters(), order=order)
    fp16 = train_cfg.precision == "fp16"
    if optimizer is None:
        if next(policy.parameters()).is_cuda:
            # flat parameter / gradient / moment buffers, the clip + loss-scale + Adam tail in one
            # HIP call (optim.FlatAdam); fp16 keeps TF32's mantissa but not its exponent range:
            # dynamic loss scaling (torch.amp.GradScaler's policy) for the gradients
            optimizer = FlatAdam(flat_grads, lr=train_cfg.learning_rate, eps=1e-5, use_loss_scale=fp16)
            if train_cfg.l2_reg_coef == 0:
                optimizer.track_init_distance()  # the logged L2-init term comes from the update pass
        else:
            optimizer = torch.optim.Adam(policy.parameters(), lr=train_cfg.learning_rate, eps=1e-5)
    initial_params = {name: p.detach().clone() for name, p in policy.named_parameters()}
    components = TrainComponents(vecenv=vecenv, policy=policy, uncompiled_policy=uncompiled_policy,
                                 experience=experience, optimizer=optimizer)
    if isinstance(optimizer, FlatAdam):
        components.scaler = optimizer if fp16 else None
        components.skipped_steps = optimizer.skipped_steps if fp16 else None
    elif fp16:
        components.scaler = torch.amp.GradScaler("cuda")
        components.skipped_steps = torch.zeros((), dtype=torch.int64, device=train_cfg.device)
    components.flat_grads = flat_grads
    components.gae = _native.GAE()
    info = TrainInfo(config=train_cfg, exp_id=exp_id, env_name=env_cfg.name, stats=StatsData(), msg=msg,
                     last_log_time=0, use_amp_obs=env_cfg.use_amp_obs, initial_params=initial_params,
                     profile=profile, wandb=wandb)
    return components, info, utilization


class RolloutStep:
    """Device part of one rollout step — policy inference on the env's observation buffer,
    staging of actions / logprob / value, and Experience.store of the mask-true rows
    (phc_compact_rows with a device cursor) — captured once as a hipGraph and replayed every
    step.  The env step (5 HIP launches) stays eager so its kernels keep their own timing.
    Inputs are the env's persistent buffers, so the graph is valid for the vecenv's lifetime;
    the twin-trunk weight cache is refreshed in place before every replay."""

    def __init__(self, components, info):
        env, exp = components.vecenv, components.experience
        self.env, self.exp, self.policy, self.cfg = env, exp, components.policy, info.config
        n = env.num_agents
        dev = env.observations.device
        self.value = torch.zeros(n, device=dev)
        # the sampled actions go straight into the env's own action buffer, so PHCPufferEnv.step
        # finds them in place (no per-step device copy)
        act = getattr(env, "actions", None)
        shape = (n, *env.single_action_space.shape)
        if (isinstance(act, torch.Tensor) and tuple(act.shape) == shape and act.dtype == torch.float32
                and act.device == torch.device(dev) and act.is_contiguous()):
            self.actions = act
        else:
            self.actions = torch.zeros(shape, device=dev)
        self.logprob = torch.zeros(n, device=dev)
        self.noise = torch.zeros((n, *env.single_action_space.shape), device=dev)
        # mu of the latest step: train() reads the reference's mean_bound_loss from it (the value
        # of the last rollout forward, core.py:225)
        self.mu = torch.zeros((n, *env.single_action_space.shape), device=dev)
        self.fused_act = getattr(info.config, "fused_act", True)
        pairs = [(env.observations, exp.obs), (self.value, exp.values), (self.actions, exp.actions),
                 (self.logprob, exp.logprobs), (env.rewards, exp.rewards), (env.terminals, exp.dones),
                 (env.truncations, exp.truncateds), (env.env_ids, exp.env_ids)]
        if info.use_amp_obs:
            pairs.append((env.amp_obs, exp.amp_obs))
        self.store = _native.RowCompactor(pairs, n, exp.batch_size, dev)
        self.graph = None
        self._blocks = {}  # captured multi-step blocks by length (run_block)
        self._blocks_key = None  # the env's launch_key() the blocks were captured under
        self.eager_steps = 0
        self._noise_ready = False
        pol = self.policy.policy if hasattr(self.policy, "policy") else self.policy
        self.twin = getattr(pol, "_twin", None)
        # R17 fused into the env step: the step kernel writes RunningNorm(obs) as the policy's first
        # GEMM operand (HumanoidPHC.set_obs_operand), so the captured graph starts at the trunks; the
        # operand is rebuilt eagerly (phc_obs_half) at the first step of every evaluate() — the
        # statistics change between iterations — and whenever a reset kernel wrote obs rows
        self.opnd, self.opnd_first = None, True
        henv = getattr(env, "env", None)
        width = half_input_width(self.twin, _compute_dtype(self.cfg)) if self.twin is not None else None
        if (self.fused_act and width is not None and hasattr(pol, "act_rollout") and hasattr(pol, "obs_norm")
                and henv is not None and hasattr(henv, "set_obs_operand") and
                getattr(info.config, "fused_obs_operand", True)):
            self.opnd = torch.zeros((n, width), dtype=_compute_dtype(self.cfg), device=dev)
            self._opnd_norm = None

    def begin(self):
        """Start of an evaluate() call: the RunningNorm statistics may have changed since the last."""
        self.opnd_first = True

    def _refresh_operand(self):
        pol = self.policy.policy if hasattr(self.policy, "policy") else self.policy
        nm = pol.obs_norm
        henv = self.env.env
        key = (nm.running_mean.data_ptr(), nm.running_var.data_ptr(), float(nm.epsilon), float(nm.clip))
        if key != self._opnd_norm:  # (re)point the step kernel at the statistics' buffers
            henv.set_obs_operand(self.opnd, nm.running_mean, nm.running_var, nm.epsilon, nm.clip)
            self._opnd_norm = key
        if self.opnd_first or not henv.obs_operand_fresh:
            _native.obs_half(self.env.observations, nm.running_mean, nm.running_var, nm.epsilon, nm.clip, self.opnd)
            self.opnd_first = False

    def _body(self, noise=None):
        pol = self.policy.policy if hasattr(self.policy, "policy") else self.policy
        with torch.no_grad(), autocast(self.cfg):
            fused = False
            if self.fused_act and hasattr(pol, "act_rollout"):
                # sample_logits' Normal draw (self.noise, drawn eagerly by run() before every step:
                # an RNG op inside the captured graph would add the generator's seed / offset
                # updates to every replay), then the fused policy tail writes the staging buffers
                fused = pol.act_rollout(self.env.observations, self.noise if noise is None else noise, self.actions,
                                        self.logprob, self.value, mu=self.mu, obs_half=self.opnd)
            if not fused:
                actions, logprob, _, value = self.policy(self.env.observations)
                self.value.copy_(value.flatten())
                self.actions.copy_(actions)
                self.logprob.copy_(logprob)
            self.fused = fused
        self.store(self.env.masks)

    def block_ok(self):
        """Whether whole blocks of steps (policy, store, env step) can replay from one graph."""
        return (BLOCK_GRAPH and self.fused_act and getattr(self.env, "block_steppable", False)
                and hasattr(self.env, "block_step"))

    def run_block(self, steps):
        """`steps` rollout steps from ONE captured graph (captured on first use of this length, after
        the single-step graph exists): per step the policy (its Normal draw from noise row k, all rows
        drawn by one launch before the replay), the experience store and the env step (the fused
        replay launch with its logging rows in row k: PHCPufferEnv.finish_block does the host's
        logging for the block).  Returns the block's infos."""
        if self.twin is not None:
            refresh_twin(self.twin, _compute_dtype(self.cfg))
        if self.opnd is not None:
            self._refresh_operand()
        shape = (steps,) + tuple(self.noise.shape)
        if getattr(self, "_noise_block", None) is None or self._noise_block.shape[0] < steps:
            self._noise_block = torch.zeros(shape, device=self.noise.device)
        noise = self._noise_block[:steps]
        noise.normal_()
        stats_buf = self.env.block_stats(steps)
        # the captured step launches hold the env / library / step-parameter structs by value: a
        # resample_motions() (a new packed library) or an eval toggle invalidates every block; so does a
        # reallocated noise or logging buffer (the graphs hold their addresses) and another kernel timer
        # (each captured env-step launch stamps into its timer's buffer)
        key = (self.env.env.launch_key(), self._noise_block.data_ptr(), stats_buf.data_ptr())
        if key != self._blocks_key:
            self._blocks.clear()
            self._blocks_key = key
        g = self._blocks.get(steps)
        if g is None:
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with _capture(g):
                for k in range(steps):
                    self._body(noise=noise[k])
                    self.env.block_step(self.actions, k)
            self._blocks[steps] = g
        g.replay()
        return self.env.finish_block(steps)

    def speculate(self, use_graph=True):
        """run() whose effects speculate_undo() can take back: the policy graph writes only staging
        buffers, the experience store (a no-op on a full buffer: the running sums it adds to are
        reset by the next evaluate) and mu; the generator state, the noise buffer and mu are saved."""
        if getattr(self, "_spec_mu", None) is None:
            self._spec_mu, self._spec_noise = torch.empty_like(self.mu), torch.empty_like(self.noise)
        self._spec_mu.copy_(self.mu)
        self._spec_noise.copy_(self.noise)
        saved = (torch.cuda.get_rng_state(self.noise.device), self._noise_ready)
        self.run(use_graph)
        return saved

    def speculate_undo(self, saved):
        self.mu.copy_(self._spec_mu)
        self.noise.copy_(self._spec_noise)
        torch.cuda.set_rng_state(saved[0], self.noise.device)
        self._noise_ready = saved[1]

    def run(self, use_graph=True):
        if self.twin is not None:
            refresh_twin(self.twin, _compute_dtype(self.cfg))  # in-place refresh after optimizer steps
        if self.opnd is not None:
            self._refresh_operand()
        ahead = self.fused_act and NOISE_AHEAD
        if self.fused_act and not (ahead and self._noise_ready):
            self.noise.normal_()
        if self.graph is not None:
            self.graph.replay()
        elif not use_graph or self.eager_steps == 0:
            self._body()  # first step eager: lazy library / allocator initialisation
            self.eager_steps += 1
        else:
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with _capture(g):
                self._body()
            self.graph = g
            g.replay()
        if ahead:
            # the next step's Normal draw, queued between this step's policy graph and its env step
            # (the buffer is read only by the next replay, stream-ordered after this draw)
            self.noise.normal_()
            self._noise_ready = True


def _capture(g):
    """torch.cuda.graph(g); under data parallelism in relaxed capture mode: RCCL's watchdog thread
    queries its (pre-capture) works' events while a capture runs, which the default global mode turns
    into hipErrorStreamCaptureUnsupported and an abort of the process.  (Thread-local mode does not
    serve: the backward's kernels are launched into the capturing stream by autograd's device thread.)
    Every capture here was validated in global mode, which rejects unsafe calls of any thread."""
    return torch.cuda.graph(g, capture_error_mode="relaxed" if D.is_dist() else "global")


def _global_count(n, device):
    """n summed over ranks (the identity without data parallelism)."""
    if not D.is_dist():
        return int(n)
    t = torch.tensor([int(n)], dtype=torch.int64, device=device)
    return int(D.allreduce_sum_(t).item())


def _global_mean(x):
    """Mean of a device scalar over ranks, as a Python float (the identity on one rank)."""
    t = torch.as_tensor(x, dtype=torch.float64).reshape(1).clone()
    if D.is_dist():
        D.allreduce_sum_(t)
        t /= D.world_size()
    return float(t.item())


def _rollout_bound_loss(components, pol):
    """The reference's mean_bound_loss as train() sees it: `getattr(policy, "mean_bound_loss")`
    read once at the start of train() (core.py:225), i.e. bound_loss(mu) of the LAST rollout
    forward (no_grad).  From the fused rollout's mu buffer, else the module's attribute."""
    rs = getattr(components, "rollout", None)
    if rs is not None and getattr(rs, "fused", False) and pol.training and hasattr(pol, "bound_loss"):
        with torch.no_grad():
            return pol.bound_loss(rs.mu)
    mbl = getattr(pol, "mean_bound_loss", None)
    return None if mbl is None else mbl.detach()


def _compute_dtype(cfg):
    return _AUTOCAST.get(cfg.precision, torch.float32)


def _evaluate_graph(components, info):
    train_cfg, profile, experience = info.config, info.profile, components.experience
    rs = getattr(components, "rollout", None)
    if rs is None or rs.exp is not experience or rs.env is not components.vecenv:
        rs = components.rollout = RolloutStep(components, info)
    env_infos = defaultdict(list)
    vecenv = components.vecenv
    with profile.evaluate:
        start = experience.ptr
        rs.store.reset(start)
        rs.begin()
        # a step stores at most num_agents rows, so the buffer cannot fill before `min_steps`:
        # those steps run without a host read; after them the device cursor is read once per
        # step (the reference's per-step mask.sum().item(), core.py:136, becomes the running
        # sums counts[2:4] read once per evaluate)
        n = max(1, rs.store.n)
        min_steps = max(1, -(-(experience.batch_size - start) // n))
        steps = 0
        step_infos = []  # read after the loop: a mean_and_log info resolves by waiting for its copy
        done = False
        if train_cfg.rollout_graph and rs.graph is not None and rs.block_ok() and min_steps >= 2:
            # the steps that cannot fill the buffer need no host read: one replayed block of them
            # (the single-step graph exists, so every lazy initialisation has happened)
            with profile.env:
                _, _, _, _, env_info, _, _ = vecenv.recv()  # the previous send's info
            step_infos.extend(env_info)
            with profile.eval_forward:
                step_infos.extend(rs.run_block(min_steps))
            vecenv._pending = (vecenv.observations, vecenv.rewards, vecenv.terminals, vecenv.truncations, [],
                               vecenv.env_ids, vecenv.masks)
            steps = min_steps
            with profile.eval_misc:
                rs.store.snapshot()  # the cursor after the block, read below without waiting for more
            spec = None
            if SPECULATE_STEP:
                with profile.env:
                    _, _, _, _, env_info, _, _ = vecenv.recv()
                with profile.eval_forward:
                    spec = rs.speculate(train_cfg.rollout_graph)
            with profile.eval_misc:
                cursor, n_valid, taken = rs.store.snapshot_read()
                done = cursor >= experience.batch_size
            if spec is not None:
                if done:  # the reference stops here: take the queued policy step back
                    rs.speculate_undo(spec)
                else:
                    step_infos.extend(env_info)
                    with profile.env:
                        vecenv.send(rs.actions)
                    steps += 1
                    if steps >= min_steps:
                        with profile.eval_misc:
                            cursor, n_valid, taken = rs.store.state()
                            done = cursor >= experience.batch_size
        while not done:
            with profile.env:
                _, _, _, _, env_info, _, _ = vecenv.recv()
            step_infos.extend(env_info)
            with profile.eval_forward:
                rs.run(train_cfg.rollout_graph)
            with profile.env:
                vecenv.send(rs.actions)
            steps += 1
            if steps >= min_steps:
                with profile.eval_misc:
                    cursor, n_valid, taken = rs.store.state()  # one read: the cursor and the running sums
                    if cursor >= experience.batch_size:
                        break
        with profile.eval_misc:
            for i in step_infos:
                for k, v in i.items():
                    env_infos[k].append(v)
            flush = getattr(vecenv, "flush", None)
            if flush is not None:  # infos a caller never reads still count their episodes now
                flush()
            # data parallel: every rank advances the same whole-job step count (its own mask-true
            # rows differ with the envs' truncation patterns), so loop exits agree across ranks
            info.global_step += _global_count(n_valid, rs.store.counts.device)
            experience.ptr = start + taken
            experience.step += steps
        for k, v in env_infos.items():
            info.stats.extend(k, list(np.atleast_1d(v)))
    experience.ptr = 0
    experience.step = 0
    return info.stats, env_infos


def evaluate(components, info):
    """Rollout until the buffer holds batch_size mask-true rows (core.py:120-203)."""
    train_cfg, profile, experience = info.config, info.profile, components.experience
    if train_cfg.rollout_graph and experience.lstm_h is None and \
            getattr(components.vecenv, "observations", None) is not None and components.vecenv.observations.is_cuda:
        return _evaluate_graph(components, info)
    policy = components.policy
    env_infos = defaultdict(list)
    local_steps = 0
    with profile.evaluate:
        while not experience.full:
            with profile.env:
                o, r, d, t, env_info, env_id, mask = components.vecenv.recv()
            with profile.eval_misc:
                n_valid = int(mask.sum().item())
                local_steps += n_valid
            if experience.lstm_h is not None:  # recurrent policies, in fp32 (core.py:149-160)
                with profile.eval_forward, torch.no_grad():
                    lstm_h, lstm_c = experience.lstm_h, experience.lstm_c
                    reset = torch.logical_or(d.bool(), t.bool())  # zero the state of envs that reset
                    if bool(reset.any()):
                        lstm_h[:, env_id[reset]] = 0
                        lstm_c[:, env_id[reset]] = 0
                    actions, logprob, _, value, (h, c) = policy(o, (lstm_h[:, env_id], lstm_c[:, env_id]))
                    lstm_h[:, env_id] = h
                    lstm_c[:, env_id] = c
            else:
                with profile.eval_forward, torch.no_grad(), autocast(train_cfg):
                    actions, logprob, _, value = policy(o)
            with profile.eval_misc:
                amp_obs = components.vecenv.amp_obs if info.use_amp_obs else None
                experience.store(o, amp_obs, value.flatten(), actions, logprob, r, d, t, env_id, mask, n_valid)
                for i in env_info:
                    for k, v in i.items():
                        env_infos[k].append(v)
            with profile.env:
                components.vecenv.send(actions)
        flush = getattr(components.vecenv, "flush", None)
        if flush is not None:
            flush()
        info.global_step += _global_count(local_steps, experience.obs.device)
        for k, v in env_infos.items():
            info.stats.extend(k, list(np.atleast_1d(v)))
    experience.ptr = 0
    experience.step = 0
    return info.stats, env_infos


def compute_advantages(components, info):
    """Sort to (env, step) order, adversarial reward, GAE, minibatch layout (core.py:212-260)."""
    cfg, experience = info.config, components.experience
    idxs = experience.sort_training_data()
    dones = experience.dones[idxs].contiguous()
    values = experience.values[idxs].contiguous()
    rewards = experience.rewards[idxs].contiguous()
    pol = components.policy.policy if hasattr(components.policy, "policy") else components.policy
    experience.b_obs_half = None
    if cfg.fused_obs and cfg.fused_loss and hasattr(pol, "obs_half_input") and experience.lstm_h is None:
        # RunningNorm + rounding into the first GEMM operand for the whole batch, in minibatch
        # order, once (the statistics are fixed during train(), scripts/train.py:337-346)
        with autocast(cfg):
            experience.b_obs_half = pol.obs_half_input(experience.obs, experience.b_idxs_obs.reshape(-1))
    experience.flatten_batch(skip_obs=experience.b_obs_half is not None)
    adv_rew = torch.zeros((experience.num_minibatches, cfg.minibatch_size), device=cfg.device)
    discriminate = getattr(components.policy.policy, "discriminate", None) if hasattr(components.policy, "policy") \
        else None
    if info.use_amp_obs and discriminate is not None:
        with torch.no_grad(), autocast(cfg):
            if hasattr(components.policy.policy, "adversarial_reward"):
                # every minibatch's rows in one pass (rows are independent; same values as the
                # reference's per-minibatch loop), gathered from the buffer by index
                adv_rew = components.policy.policy.adversarial_reward(
                    [(experience.amp_obs, experience.b_amp_idx.reshape(-1))]).view(adv_rew.shape)
            else:
                for mb in range(experience.num_minibatches):
                    logits = discriminate(experience.b_amp_obs[mb]).squeeze()
                    prob = 1 / (1 + torch.exp(-logits))
                    adv_rew[mb] = -torch.log(torch.clamp(1 - prob, min=0.0001))
    # the adversarial reward is indexed like the reference: flat ravel of [num_mb, mb_size]
    advantages = components.gae(dones, values, (rewards + adv_rew.reshape(-1)).contiguous(), cfg.gamma,
                                cfg.gae_lambda)
    experience.b_advantages = (advantages.reshape(experience.minibatch_rows, experience.num_minibatches,
                                                  experience.bptt_horizon)
                               .transpose(0, 1).reshape(experience.num_minibatches, experience.minibatch_size))
    experience.returns = advantages + values
    experience.sorted_values = values
    experience.b_returns = experience.b_advantages + experience.b_values
    # what train() needs from these fixed arrays, computed here so the graphed pass carries it:
    # the per-minibatch advantage (mean, std) of norm_adv (single process; data parallel reduces
    # over the ranks in train()) and the explained-variance pair logged at the end (core.py:397-399)
    experience.b_adv_ms = None if D.is_dist() else torch.stack(
        [experience.b_advantages.mean(1), experience.b_advantages.std(1)], 1).contiguous()
    var_y = torch.var(experience.returns, unbiased=False)
    ev_t = 1 - torch.var(experience.returns - values, unbiased=False) / var_y
    experience.ev_pair = torch.stack([var_y, ev_t]).double()
    return advantages


_ROW_INDEX = {}


def _row_index(device):
    """Device index tensors of the loss row's scatter (made once per device: an index given as a
    Python list is a host -> device copy and an index launch every iteration)."""
    key = str(device)
    if key not in _ROW_INDEX:
        mk = lambda v: torch.tensor(v, dtype=torch.long, device=device)  # noqa: E731
        _ROW_INDEX[key] = (mk([0, 1, 2, 3, 4, 5, 9]), mk([6, 7]), mk([0, 2]))
    return _ROW_INDEX[key]


class _PinnedRing:
    """Pinned host buffers for the loss row's non-blocking readback, reused round-robin (a pinned
    allocation per iteration cost ~0.1 ms of host time with the GPU idle).  A slot still owned by
    an unread PendingLossComponents is resolved (its copy long finished) before it is reused."""

    def __init__(self, n=4):
        self.n, self.slots, self.i = n, {}, 0

    def take(self, like, owner_of):
        key = (tuple(like.shape), like.dtype)
        ring = self.slots.setdefault(key, [])
        if len(ring) < self.n:
            ring.append([torch.empty(like.shape, dtype=like.dtype, pin_memory=True), None])
            slot = ring[-1]
        else:
            slot = ring[self.i % self.n]
            self.i += 1
            prev = slot[1]
            if prev is not None and object.__getattribute__(prev, "__dict__").get("_pending") is not None:
                prev.policy_loss  # noqa: B018  (resolves the earlier readback out of this buffer)
        slot[1] = owner_of
        return slot


_PINNED = _PinnedRing()


# train()'s advantage / minibatch-layout pass replayed from a captured hipGraph: ~20 small launches
# (sort, gathers, the operand build, GAE, reshapes) whose Python launch overhead left the GPU idle
# between the rollout and the first trunk GEMM.  The pass reads only device buffers that keep their
# addresses (the experience arrays, the RunningNorm statistics) and writes its outputs into the
# graph's own memory, which the experience attributes set during capture keep pointing at.
ADV_GRAPH = os.environ.get("PHC_ADV_GRAPH", "1") != "0"
# rollout: draw the next step's action noise right after the policy graph instead of before it
NOISE_AHEAD = os.environ.get("PHC_NOISE_AHEAD", "0") != "0"
# rollout: the steps that cannot fill the buffer (all but the last one or two) replay as ONE captured
# block of policy + store + env-step launches (RolloutStep.run_block); PHC_BLOCK_GRAPH=0: one graph per
# step with the env step eager
BLOCK_GRAPH = os.environ.get("PHC_BLOCK_GRAPH", "1") != "0"
# rollout: after the block, the next step's policy graph is queued BEFORE the host reads whether the
# block filled the buffer (the read waits for the block only), so the GPU runs it while the host
# decides; when the buffer turned out full, the step's visible effects (mu, the action-noise buffer
# and the generator state) are restored and its env step is not sent — the reference's loop would not
# have run it (core.py:129-181).  PHC_SPECULATE_STEP=0: read first, then launch.
SPECULATE_STEP = os.environ.get("PHC_SPECULATE_STEP", "1") != "0"


_ADV_ATTRS = ("b_idxs_obs", "b_idxs", "b_idxs_flat", "b_obs_half", "b_obs", "b_actions", "b_logprobs", "b_dones",
              "b_truncated", "b_values", "b_advantages", "returns", "sorted_values", "b_returns", "b_adv_ms",
              "ev_pair", "b_amp_idx", "b_amp_rep_idx")


def _adv_graph_key(components, info):
    exp, cfg = components.experience, info.config
    pol = components.policy.policy if hasattr(components.policy, "policy") else components.policy
    nm = getattr(pol, "obs_norm", None)
    ptrs = tuple(t.data_ptr() for t in (exp.obs, exp.actions, exp.logprobs, exp.values, exp.rewards, exp.dones,
                                         exp.truncateds, exp.env_ids))
    norm = (nm.running_mean.data_ptr(), nm.running_var.data_ptr(), float(nm.epsilon), float(nm.clip)) if nm else None
    # what decides which outputs compute_advantages produces: the half-precision operand build
    # (fused policy, its twin layout) and the single-process advantage statistics
    twin = getattr(pol, "_twin", None)
    width = half_input_width(twin, _compute_dtype(cfg)) if twin is not None else None
    amp = None
    if info.use_amp_obs:  # the AMP buffers, the replay's fill state and draw counter, the discriminator
        anm = getattr(pol, "amp_obs_norm", None)
        amp = (exp.amp_obs.data_ptr(), exp.amp_obs_replay.data_ptr(), exp.amp_obs_replay_filled,
               exp._amp_iter.data_ptr() if getattr(exp, "_amp_iter", None) is not None else None,
               float(exp.amp_obs_update_prob), id(getattr(pol, "_disc_ops", None)),
               (anm.running_mean.data_ptr(), anm.running_var.data_ptr()) if anm is not None else None,
               weight_cache.layout_key(None, list(pol.parameters())))
    return (ptrs, norm, exp.batch_size, exp.minibatch_size, exp.num_minibatches, exp.bptt_horizon,
            float(cfg.gamma), float(cfg.gae_lambda), cfg.fused_obs, cfg.fused_loss, cfg.precision,
            id(components.gae), bool(getattr(pol, "fused", False)), hasattr(pol, "obs_half_input"), width,
            D.is_dist(), amp)


def _compute_advantages_train(components, info):
    """compute_advantages for train(): eager on the first call, captured on the second, replayed
    after (re-captured when a key input changes; eager for recurrent policies or host tensors).  With
    AMP the pass holds the adversarial reward and the replay buffer's refresh (counter-based draws, a
    select: structs.Experience.flatten_batch)."""
    exp = components.experience
    if not (ADV_GRAPH and exp.obs.is_cuda and exp.lstm_h is None):
        return compute_advantages(components, info)
    st = getattr(components, "_adv_graph", None)
    if st is None:
        st = {"graph": None, "key": None, "out": None, "failed": False}
        components._adv_graph = st
    key = _adv_graph_key(components, info)
    st["replayed"] = False
    if st["graph"] is not None and st["key"] == key:
        st["graph"].replay()
        for k, v in st["attrs"].items():  # an eager call in between may have re-pointed them
            setattr(exp, k, v)
        st["replayed"] = True
        return st["out"]
    if st["failed"] or st["key"] != key:  # first sight of this key: eager (lazy initialisation)
        st["graph"], st["key"] = None, key
        return compute_advantages(components, info)
    try:
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with _capture(g):
            out = compute_advantages(components, info)
    except Exception:  # noqa: BLE001  (an op that cannot be captured: stay eager)
        st["failed"] = True
        torch.cuda.synchronize()
        return compute_advantages(components, info)
    st["graph"], st["out"] = g, out
    st["attrs"] = {k: getattr(exp, k) for k in _ADV_ATTRS if hasattr(exp, k)}
    g.replay()
    return out


def _adv_mean_std(experience):
    """Per-minibatch advantage (mean, std): the copy compute_advantages made (single process),
    else the all-rank reduction."""
    ms = getattr(experience, "b_adv_ms", None)
    return ms if ms is not None else D.global_mean_std_rows(experience.b_advantages)


def _fill_losses(losses, a):
    """The logged loss row (train's device accumulators, var_y, explained variance) into the
    LossComponents fields."""
    for i, k in enumerate(("policy_loss", "value_loss", "entropy", "old_approx_kl", "approx_kl", "clipfrac",
                           "before_clip_grad_norm", "l2_init_reg_loss", "disc_loss", "mean_bound_loss",
                           "disc_agent_acc", "disc_demo_acc")):
        setattr(losses, k, a[i])
    losses.explained_variance = float(a[13]) if a[12] != 0 else float("nan")


# train()'s minibatch loop (update_epochs x num_minibatches fused minibatches: trunks, tail, PPO
# objective, backward, clip + Adam) and the logged loss row replayed from ONE captured hipGraph: the
# ~40 launches per minibatch run back to back with no host in between.  Eligible: the fused path with
# FlatAdam and the reference's defaults (no AMP, no recurrent policy, no target-KL early stop, no
# L2-init loss, the bound term a no-grad constant), once train()'s advantage pass itself replays from
# its graph (fixed input addresses).  Data parallel (round 6): the graph holds the RCCL collectives too
# -- the per-train() advantage statistics all-reduce and every minibatch's gradient-span all-reduces,
# forked onto RCCL's stream by the backward's readiness hook and joined before the optimizer step
# (FlatGrads.overlap_begin / overlap_finish) -- so every rank replays the same collective sequence.
# PHC_TRAIN_GRAPH=0: eager; PHC_DP_TRAIN_GRAPH=0: eager under data parallelism only.
TRAIN_GRAPH = os.environ.get("PHC_TRAIN_GRAPH", "1") != "0"
DP_TRAIN_GRAPH = os.environ.get("PHC_DP_TRAIN_GRAPH", "1") != "0"


def _train_graph_eligible(components, info, pol):
    cfg, exp, opt = info.config, components.experience, components.optimizer
    adv = getattr(components, "_adv_graph", None)
    if not (TRAIN_GRAPH and exp.obs.is_cuda and exp.lstm_h is None
            and (not info.use_amp_obs or (hasattr(pol, "discriminate_rows") and hasattr(exp, "b_amp_rep_idx")))
            and (not D.is_dist() or (DP_TRAIN_GRAPH and D.backend() == "nccl"))
            and isinstance(opt, FlatAdam) and opt.param_init is not None and cfg.l2_reg_coef == 0
            and cfg.target_kl is None and not cfg.bound_loss_grad and STORE_GRADS and cfg.fused_loss
            and adv is not None and adv.get("replayed") and getattr(exp, "b_obs_half", None) is not None
            and hasattr(pol, "forward_train") and getattr(pol, "fused", False)):
        return False
    with autocast(cfg):
        return fused_ppo_supported(pol, exp.b_obs_half[:exp.minibatch_size])


_UNIT_MS = {}


def _amp_disc_terms(cfg, pol, exp, mb, amp_obs_demo, amp_mb, loss):
    """Minibatch mb's discriminator terms (core.py:336-347, 394-395): agent, replay and demo rows in one
    pass; returns (disc_loss, (agent acc, demo acc), loss + disc_coef * disc_loss)."""
    idx_agent = exp.b_amp_idx[mb][:amp_mb]
    idx_replay = exp.b_amp_rep_idx[mb][:amp_mb]
    with autocast(cfg):
        d_all = pol.discriminate_rows([(exp.amp_obs, idx_agent), (exp.amp_obs_replay, idx_replay),
                                       (amp_obs_demo, None)]).float()
    # a minibatch may hold fewer than amp_mb rows (minibatch_size < num_envs): split at the agent +
    # replay rows actually gathered, not at 2 * amp_mb
    n_agent = idx_agent.numel() + idx_replay.numel()
    d_agent, d_demo = d_all[:n_agent], d_all[n_agent:]
    bce = torch.nn.BCEWithLogitsLoss()
    disc_loss = 0.5 * (bce(d_agent, torch.zeros_like(d_agent)) + bce(d_demo, torch.ones_like(d_demo)))
    disc_acc = ((d_agent.detach() < 0).float().mean(), (d_demo.detach() > 0).float().mean())
    if cfg.disc_coef > 0:
        loss = loss + disc_loss * cfg.disc_coef
    return disc_loss, disc_acc, loss


def _fused_update(components, info, pol):
    """The minibatch loop of the eligible path (the same launches as train()'s general loop with
    fused_mb and opt_l2) and the loss row; returns the row (device float64 [14]).  Captured into the
    train graph, or run eagerly (first sight of a configuration)."""
    cfg, exp, opt = info.config, components.experience, components.optimizer
    flat = components.flat_grads
    dev = exp.obs.device
    acc_ppo = torch.zeros(7, dtype=torch.float64, device=dev)
    acc_opt = torch.zeros(3, dtype=torch.float64, device=dev)
    mbl_ref = _rollout_bound_loss(components, pol)
    total = exp.num_minibatches * cfg.update_epochs
    mbs = exp.minibatch_size
    coefs = ppo_coefs(cfg, pol.soft_bound)
    if cfg.norm_adv:
        adv_ms = _adv_mean_std(exp)
    else:
        key = str(dev)
        if key not in _UNIT_MS:
            _UNIT_MS[key] = torch.tensor([0.0, 1.0], dtype=torch.float32, device=dev)
        unit = _UNIT_MS[key]
    amp = info.use_amp_obs
    acc = torch.zeros(12, dtype=torch.float64, device=dev)
    if amp:  # the demo rows: the env's AMP demo buffer (a fixed address, refreshed by the rollout's steps)
        amp_obs_demo = components.vecenv.fetch_amp_obs_demo()
        amp_mb = amp_obs_demo.shape[0]
    for _epoch in range(cfg.update_epochs):
        for mb in range(exp.num_minibatches):
            obs = exp.b_obs_half[mb * mbs:(mb + 1) * mbs]
            atn = exp.b_actions[mb].reshape(-1, exp.b_actions.shape[-1])
            with autocast(cfg):  # the logged sums accumulate inside the objective / optimizer launches
                # AMP: the general loop's launches exactly (a second gradient source: no stored
                # gradients, the buffer zeroed; the loss row summed per minibatch as there)
                loss, st = fused_ppo_loss(pol, obs, atn, exp.b_logprobs[mb].reshape(-1), exp.b_advantages[mb],
                                          adv_ms[mb] if cfg.norm_adv else unit, exp.b_values[mb], exp.b_returns[mb],
                                          coefs, store_grads=not amp, stats_acc=None if amp else acc_ppo)
            if amp:
                disc_loss, disc_acc, loss = _amp_disc_terms(cfg, pol, exp, mb, amp_obs_demo, amp_mb, loss)
                flat.zero()
            flat.overlap_begin()  # data parallel: the gradient spans' all-reduces as the backward finishes them
            opt.backward(loss)
            flat.overlap_finish()
            if not amp:
                opt.fused_step(cfg.max_grad_norm, norm_acc=acc_opt)
                continue
            gnorm = opt.fused_step(cfg.max_grad_norm, norm_acc=None)[0]
            with torch.no_grad():
                pg_loss, v_loss, entropy_loss, old_approx_kl, approx_kl, clipfrac, _ = st.unbind(0)
                mbl = mbl_ref if mbl_ref is not None else torch.zeros((), device=dev)
                acc += torch.stack([pg_loss.detach(), v_loss.detach(), entropy_loss.detach(), old_approx_kl, approx_kl,
                                    clipfrac, gnorm, opt.norms[2].detach(), disc_loss.detach(), mbl.detach(),
                                    disc_acc[0], disc_acc[1]]).double() / total
    with torch.no_grad():
        i7, i67, i02 = _row_index(dev)
        acc.index_add_(0, i7, acc_ppo / total)
        acc.index_add_(0, i67, acc_opt.index_select(0, i02) / total)
        if mbl_ref is not None:
            acc[9] = mbl_ref.double()
        return torch.cat([acc, exp.ev_pair])


def _dp_mode_key():
    from ..policies import twin_mlp

    return twin_mlp.dp_mode()


def _train_graph_key(components, info, pol):
    cfg, exp = info.config, components.experience
    rs = getattr(components, "rollout", None)
    return (id(components._adv_graph.get("graph")), id(rs), rs.mu.data_ptr() if rs is not None else None,
            cfg.update_epochs, cfg.norm_adv, float(cfg.max_grad_norm), float(cfg.clip_coef), float(cfg.vf_clip_coef),
            float(cfg.vf_coef), float(cfg.ent_coef), float(cfg.bound_coef), bool(cfg.clip_vloss), cfg.precision,
            id(components.optimizer), components.optimizer.use_loss_scale, _native.gemm_timer_id(),
            weight_cache.layout_key(None, list(pol.parameters())), weight_cache.plans_version(),
            # the step kernel receives betas / eps / the hyper-parameter scales by value (lr is device state)
            tuple(components.optimizer.param_groups[0]["betas"]), float(components.optimizer.param_groups[0]["eps"]),
            tuple(components.optimizer._hp_scale),
            # data parallel: the collectives are captured too (the readiness schedule of the DP mode)
            D.is_dist(), D.world_size(), _dp_mode_key(),
            # AMP: the discriminator terms read the demo buffer and the buffers the advantage pass holds
            info.use_amp_obs, float(getattr(cfg, "disc_coef", 0.0)), _amp_demo_ptr(components, info))


def _amp_demo_ptr(components, info):
    if not info.use_amp_obs:
        return None
    demo = components.vecenv.fetch_amp_obs_demo()
    return None if demo is None else (demo.data_ptr(), tuple(demo.shape))


def _all_ranks_agree(flag, device):
    """True when `flag` holds on every rank (the identity without data parallelism).  The train graph holds
    collectives that every rank must replay in lockstep: a rank on another path would issue its own."""
    if not D.is_dist():
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int64, device=device)
    return int(D.allreduce_sum_(t).item()) == D.world_size()


def _train_minibatches_graphed(components, info, pol):
    """The loss row of this train() call from the train graph (captured on the second eligible call
    with an unchanged key, replayed after), or eagerly; None when not eligible.  Under data parallelism
    the capture's success is agreed over the ranks (eligibility follows from the configuration and the
    call count, the same on every rank)."""
    dev = components.experience.obs.device
    if not _train_graph_eligible(components, info, pol):
        return None
    opt = components.optimizer
    st = components.__dict__.setdefault("_train_graph", {"graph": None, "key": None, "row": None, "failed": False})
    key = _train_graph_key(components, info, pol)
    opt.sync_lr()
    if st["graph"] is not None and st["key"] == key:
        fresh = opt.fresh_operand_owners() if st["writes_operands"] else []
        if st["writes_operands"]:
            # the graph's first minibatch reads the GEMM operand copies as they are (its capture saw them
            # current, so it holds no refresh launch): re-pack any a parameter write outside the captured
            # Adam steps left stale (load_state_dict, a parameter broadcast, a manual copy)
            for o in opt._ops_owners:
                if not any(o is f for f in fresh):
                    o.plan.run()
                    weight_cache.mark_fresh(o)
                    fresh.append(o)
        st["graph"].replay()
        _native.GEMM_LAUNCHES[0] += st["gemm_launches"]
        # the replay rewrote the parameters behind every host-side cache key (FlatAdam.fused_step
        # bumps the generation when it runs on the host; a replay does not run it); the operand
        # caches its captured steps rewrote stay current
        opt.operands_written(fresh)
        return st["row"]
    if st["failed"] or st["key"] != key:  # first sight of this configuration: eager
        st["graph"], st["key"] = None, key
        return _fused_update(components, info, pol)
    ok = True
    try:
        torch.cuda.synchronize()
        if D.is_dist():
            # the capture makes RCCL's stream part of the capture; the process group's watchdog thread polls
            # its pending works' events every 100 ms, and on this HIP a query of an event recorded on a stream
            # that is capturing now fails (hipErrorCapturedEvent) and aborts the process.  Let the watchdog
            # retire every finished work first (once per capture)
            time.sleep(0.25)
        g = torch.cuda.CUDAGraph()
        launches0 = _native.GEMM_LAUNCHES[0]
        with _capture(g):
            row = _fused_update(components, info, pol)
        st["gemm_launches"] = _native.GEMM_LAUNCHES[0] - launches0
    except Exception as exc:  # noqa: BLE001  (an op that cannot be captured: stay eager)
        ok = False
        warnings.warn(f"train graph capture failed, the update stays eager: {exc!r}", RuntimeWarning, stacklevel=2)
    # a capture executes no collective, so the ranks can still agree after it: all replay, or all stay eager
    if not _all_ranks_agree(ok, dev):
        st["failed"] = True
        torch.cuda.synchronize()
        return _fused_update(components, info, pol)
    st["graph"], st["row"] = g, row
    # captured with the step writing the operand copies (FlatAdam's job table in use)
    st["writes_operands"] = opt._ops is not None and opt._ops_v == weight_cache.plans_version()
    fresh = opt.fresh_operand_owners() if st["writes_operands"] else []
    g.replay()
    opt.operands_written(fresh)
    return row


def train(components, info, utilization=None):
    """PPO update (core.py:206-440)."""
    cfg, profile = info.config, info.profile
    experience = components.experience
    pol = components.policy.policy if hasattr(components.policy, "policy") else components.policy
    flat = components.flat_grads
    acc = torch.zeros(12, dtype=torch.float64, device=cfg.device)  # device-side loss accumulators
    # fused path: the PPO kernel's 7 logged means and the optimizer's [norm sum, norm, l2]
    acc_ppo = torch.zeros(7, dtype=torch.float64, device=cfg.device)
    acc_opt = torch.zeros(3, dtype=torch.float64, device=cfg.device)
    opt_l2 = isinstance(components.optimizer, FlatAdam) and components.optimizer.param_init is not None \
        and cfg.l2_reg_coef == 0
    with profile.train:
        with profile.train_misc:
            _compute_advantages_train(components, info)
            row = _train_minibatches_graphed(components, info, pol)
        if row is not None:
            return _finish_train(components, info, row)
        with profile.train_misc:
            if info.use_amp_obs:
                amp_obs_demo = components.vecenv.fetch_amp_obs_demo()
                amp_mb = amp_obs_demo.shape[0]
            # the reference's bound term: a no-grad constant read once here (see config.py)
            mbl_ref = None if cfg.bound_loss_grad else _rollout_bound_loss(components, pol)
        total_minibatches = experience.num_minibatches * cfg.update_epochs
        adv_ms = None
        tail_coefs = None
        fused_loss = (cfg.fused_loss and hasattr(pol, "forward_train") and getattr(pol, "fused", False)
                      and experience.lstm_h is None)
        obs_dim = components.vecenv.single_observation_space.shape[0]
        recurrent = experience.lstm_h is not None
        for _epoch in range(cfg.update_epochs):
            lstm_state = None  # each epoch's minibatches carry (h, c) from one to the next (core.py:268)
            for mb in range(experience.num_minibatches):
                with profile.train_misc:
                    if experience.b_obs_half is not None:
                        mbs = experience.minibatch_size
                        obs = experience.b_obs_half[mb * mbs:(mb + 1) * mbs]
                    else:
                        obs = experience.b_obs[mb].reshape(-1, obs_dim)
                    atn = experience.b_actions[mb].reshape(-1, experience.b_actions.shape[-1])
                    log_probs = experience.b_logprobs[mb].reshape(-1)
                    val = experience.b_values[mb]
                    adv = experience.b_advantages[mb]
                    ret = experience.b_returns[mb]
                fused_obj = fused_loss and obs.is_cuda
                fused_mb = False
                with profile.train_forward, (contextlib.nullcontext() if recurrent else autocast(cfg)):
                    if recurrent:
                        # [minibatch_rows, bptt, obs] segments through the LSTM (core.py:287-289)
                        _, newlogprob, entropy, newvalue, lstm_state = components.policy(
                            experience.b_obs[mb], info=lstm_state, action=experience.b_actions[mb])
                        lstm_state = (lstm_state[0].detach(), lstm_state[1].detach())
                    elif fused_obj and fused_ppo_supported(pol, obs):
                        # the whole minibatch (trunks + LayerNorm/heads + PPO objective) as one
                        # autograd node (policies/fused_ppo.py)
                        fused_mb = True
                        if cfg.norm_adv:
                            if adv_ms is None:
                                adv_ms = _adv_mean_std(experience)
                            ms = adv_ms[mb]
                        else:
                            ms = torch.tensor([0.0, 1.0], dtype=torch.float32, device=obs.device)
                        if tail_coefs is None:
                            tail_coefs = ppo_coefs(cfg, pol.soft_bound)
                        # every gradient of this backward has one writer that stores it: the flat
                        # buffer need not be zeroed first.  Not with a second gradient source: AMP
                        # adds the discriminator's on top, and the L2-init term's AccumulateGrad
                        # nodes run BEFORE this node's backward (created later, higher sequence
                        # number), so a store would overwrite their gradient
                        store_grads = (STORE_GRADS and not info.use_amp_obs and cfg.l2_reg_coef == 0
                                       and isinstance(components.optimizer, FlatAdam))
                        in_kernel_acc = opt_l2 and not info.use_amp_obs
                        loss, st = fused_ppo_loss(pol, obs, atn, log_probs, adv, ms, val, ret, tail_coefs,
                                                  store_grads=store_grads,
                                                  stats_acc=acc_ppo if in_kernel_acc else None)
                    elif fused_obj:
                        mu, newvalue = pol.forward_train(obs)
                    else:
                        _, newlogprob, entropy, newvalue = components.policy(obs, action=atn)
                with profile.train_misc:
                    adv = adv.reshape(-1)
                    if fused_mb:
                        pg_loss, v_loss, entropy_loss, old_approx_kl, approx_kl, clipfrac, mbl_f = st.unbind(0)
                    elif fused_obj:
                        # PPO objective in two HIP kernels (clean_pufferl/ppo_loss.py); the
                        # per-minibatch advantage mean / std of every minibatch at once
                        if cfg.norm_adv:
                            if adv_ms is None:
                                adv_ms = _adv_mean_std(experience)
                            mean, std = adv_ms[mb], None
                        else:
                            mean, std = 0.0, 1.0
                        loss, st = ppo_objective(mu, newvalue, pol.sigma, atn, log_probs, adv, mean, std, val, ret,
                                                 cfg, pol.soft_bound)
                        pg_loss, v_loss, entropy_loss, old_approx_kl, approx_kl, clipfrac, mbl_f = st.unbind(0)
                    else:
                        logratio = newlogprob - log_probs
                        ratio = logratio.exp()
                        with torch.no_grad():
                            old_approx_kl = (-logratio).mean()
                            approx_kl = ((ratio - 1) - logratio).mean()
                            clipfrac = ((ratio - 1.0).abs() > cfg.clip_coef).float().mean()
                        if cfg.norm_adv:
                            mean, std = D.global_mean_std(adv)
                            adv = (adv - mean) / (std + 1e-8)
                        pg_loss1 = -adv * ratio
                        pg_loss2 = -adv * torch.clamp(ratio, 1 - cfg.clip_coef, 1 + cfg.clip_coef)
                        pg_loss = torch.max(pg_loss1, pg_loss2).mean()
                        newvalue = newvalue.view(-1)
                        if cfg.clip_vloss:
                            v_unclipped = (newvalue - ret) ** 2
                            v_clipped = val + torch.clamp(newvalue - val, -cfg.vf_clip_coef, cfg.vf_clip_coef)
                            v_loss = torch.max(v_unclipped, (v_clipped - ret) ** 2).mean()
                        else:
                            v_loss = ((newvalue - ret) ** 2).mean()
                        entropy_loss = entropy.mean()
                        loss = pg_loss - cfg.ent_coef * entropy_loss + v_loss * cfg.vf_coef
                    disc_loss = disc_acc = None  # zeros only where the logging row needs them (below)
                    if info.use_amp_obs:
                        # agent rows, replay rows and demo rows through the discriminator in one
                        # pass (core.py:336-344 calls it twice; rows are independent)
                        disc_loss, disc_acc, loss = _amp_disc_terms(cfg, pol, experience, mb, amp_obs_demo, amp_mb,
                                                                    loss)
                    if not cfg.bound_loss_grad:
                        mbl = mbl_ref  # constant: changes the loss value only, never a gradient
                        # (the loss value itself is not read: the logged bound term is mbl_ref, so
                        # the fused path skips the two scalar launches of the sum)
                        if cfg.bound_coef > 0 and mbl is not None and not fused_mb:
                            loss = loss + mbl * cfg.bound_coef
                    elif fused_obj:
                        mbl = mbl_f  # already inside `loss` (bound_coef term of the fused objective)
                    else:
                        mbl = getattr(pol, "mean_bound_loss", None)
                        if cfg.bound_coef > 0 and mbl is not None:
                            loss = loss + mbl * cfg.bound_coef
                    l2 = None if opt_l2 else _l2_init_reg(list(components.policy.named_parameters()),
                                                          info.initial_params, cfg.l2_reg_coef > 0)
                    if cfg.l2_reg_coef > 0:
                        loss = loss + l2 * cfg.l2_reg_coef
                with profile.learn:
                    if not (fused_mb and store_grads):
                        flat.zero()
                    opt, scaler = components.optimizer, components.scaler
                    if isinstance(opt, FlatAdam):
                        flat.overlap_begin()  # data parallel: per-layer all-reduces during the backward
                        opt.backward(loss)  # d(loss * S): S under fp16 loss scaling
                        flat.overlap_finish()
                        # unscale, clip, skip-on-inf, Adam (the logged norms summed in the same launch)
                        acc_in = fused_mb and opt_l2 and not info.use_amp_obs
                        gnorm = opt.fused_step(cfg.max_grad_norm, norm_acc=acc_opt if acc_in else None)[0]
                    elif scaler is None:
                        loss.backward()
                        flat.allreduce_mean()
                        gnorm = flat.clip_(cfg.max_grad_norm)  # clip_grad_norm_ (core.py:366-370)
                        opt.step()
                    else:
                        scaler.scale(loss).backward()
                        flat.allreduce_mean()
                        scaler.unscale_(opt)
                        gnorm = flat.clip_(cfg.max_grad_norm)
                        scaler.step(opt)  # skipped when a grad is inf/nan
                        for found in scaler._found_inf_per_device(opt).values():
                            components.skipped_steps += (found > 0).long()  # device-side count, no sync
                        scaler.update()
                with profile.train_misc, torch.no_grad():
                    if fused_obj and opt_l2 and not info.use_amp_obs:
                        if not fused_mb:  # (the fused minibatch's launches summed these already)
                            acc_ppo += st  # pg, v, ent, old_kl, kl, clipfrac, bound (ppo_loss.py)
                            acc_opt += components.optimizer.norms  # norm sum, total norm, l2
                        continue
                    if l2 is None:
                        l2 = components.optimizer.norms[2]
                    if disc_loss is None:
                        disc_loss = torch.zeros((), device=cfg.device)
                        disc_acc = (disc_loss, disc_loss)
                    acc += torch.stack([pg_loss.detach(), v_loss.detach(), entropy_loss.detach(), old_approx_kl,
                                        approx_kl, clipfrac, gnorm, l2.detach(), disc_loss.detach(),
                                        (mbl.detach() if mbl is not None else torch.zeros((), device=cfg.device)),
                                        disc_acc[0], disc_acc[1]]).double() / total_minibatches
            # ranks must agree on the early stop, or one would wait in the next minibatch's
            # gradient all-reduce: the test reads the ranks' mean approx_kl
            if cfg.target_kl is not None and _global_mean(approx_kl) > cfg.target_kl:
                break
        with profile.train_misc:
            if cfg.anneal_lr:  # core.py:405-408 (the caller's exp decay overrides it, as there)
                frac = 1.0 - info.global_step / cfg.total_timesteps
                components.optimizer.param_groups[0]["lr"] = frac * cfg.learning_rate
            i7, i67, i02 = _row_index(acc.device)
            acc.index_add_(0, i7, acc_ppo / total_minibatches)
            acc.index_add_(0, i67, acc_opt.index_select(0, i02) / total_minibatches)
            if mbl_ref is not None:
                acc[9] = mbl_ref.double()  # the reference logs the rollout's value (constant)
            elif not cfg.bound_loss_grad:
                acc[9] = 0.0
            # explained variance (core.py:397-399) in fp32 on the device; the loss row, var_y and
            # it come back in ONE device -> host copy, non-blocking into pinned memory: the values
            # are read (and waited for) only when the losses are first looked at
            ev_pair = getattr(experience, "ev_pair", None)
            if ev_pair is None:
                y_pred = experience.sorted_values
                y_true = experience.returns
                var_y = torch.var(y_true, unbiased=False)
                ev_t = 1 - torch.var(y_true - y_pred, unbiased=False) / var_y
                ev_pair = torch.stack([var_y, ev_t]).double()
            row = torch.cat([acc, ev_pair])
        return _finish_train(components, info, row, anneal=False)


def _finish_train(components, info, row, anneal=True):
    """train()'s host tail: the lr anneal, the loss row's non-blocking readback, logging and the
    checkpoint cadence (core.py:397-440).  Runs inside train()'s profile.train context."""
    cfg, profile = info.config, info.profile
    with profile.train_misc:
        if anneal and cfg.anneal_lr:  # core.py:405-408 (the caller's exp decay overrides it, as there)
            frac = 1.0 - info.global_step / cfg.total_timesteps
            components.optimizer.param_groups[0]["lr"] = frac * cfg.learning_rate
        if row.is_cuda:
            slot = _PINNED.take(row, None)
            host = slot[0]
            host.copy_(row, non_blocking=True)
            done = torch.cuda.Event()
            done.record()
            losses = PendingLossComponents(host, done, _fill_losses)
            slot[1] = losses
        else:
            losses = LossComponents()
            _fill_losses(losses, row.numpy())
        info.epoch += 1
        info.losses = losses
        done_training = info.global_step >= cfg.total_timesteps
        if done_training or profile.update(components, info):
            info.stats.mean_and_log(components, info, losses)
            info.stats.clear()
        if D.rank() == 0 and (info.epoch % cfg.checkpoint_interval == 0 or done_training):
            save_checkpoint(components.uncompiled_policy, components.optimizer, cfg, info.exp_id, info.epoch,
                            info.global_step)
            info.msg = f"Checkpoint saved at update {info.epoch}"
    return losses


def close(components, info, utilization=None):
    components.vecenv.close()
    if utilization is not None:
        utilization.stop()
    if info.wandb is not None:
        if D.rank() == 0:
            save_checkpoint(components.uncompiled_policy, components.optimizer, info.config, info.exp_id, info.epoch,
                            info.global_step)
        info.wandb.finish()
