"""PHCPolicy (puffer_phc/policies/phc_policy.py:10-61): 6-layer SiLU actor and critic with a
LayerNorm head, fixed-sigma Normal.  State-dict keys match the reference
(tests/golden/state_dict_keys.tsv)."""

from typing import Sequence

import torch
from torch import nn

from .discriminator_policy import DiscriminatorPolicy
from .pufferl_policy import Linear, layer_init
from .. import _native as N
from .twin_mlp import (TwinWeights, _use_mfma, half_input_width, head_linear, twin_ln_silu, twin_ln_silu_supported,
                       twin_trunks)


def mlp(layer_sizes, activation):
    layers = []
    for a, b in zip(layer_sizes[:-2], layer_sizes[1:-1]):
        layers.append(layer_init(Linear(a, b)))
        layers.append(activation())
    layers.append(layer_init(Linear(layer_sizes[-2], layer_sizes[-1])))
    return layers


class PHCPolicy(DiscriminatorPolicy):
    def __init__(self, env, hidden_size: int = 512, layer_sizes: Sequence[int] = (2048, 1536, 1024, 1024, 512)):
        super().__init__(env, hidden_size)
        self.actor_mlp = nn.Sequential(*mlp([self.input_size] + list(layer_sizes) + [hidden_size], nn.SiLU),
                                       nn.LayerNorm(hidden_size), nn.SiLU())
        self.critic_mlp = nn.Sequential(*mlp([self.input_size] + list(layer_sizes) + [hidden_size], nn.SiLU),
                                        nn.LayerNorm(hidden_size), nn.SiLU(),
                                        layer_init(Linear(hidden_size, 1), std=0.01))
        # both trunks' Linear layers, run as twin GEMMs + fused HIP epilogues on the device
        lin = [i for i, m in enumerate(self.actor_mlp) if isinstance(m, nn.Linear)]
        self._twin = TwinWeights([self.actor_mlp[i] for i in lin], [self.critic_mlp[i] for i in lin])
        self._head = len(lin) * 2 - 1  # index of the actor LayerNorm in the Sequential
        self.fused = True
        self.fused_ln = True  # LayerNorm + SiLU of both trunks in one kernel (False: torch modules)
        self._critic_trunk = None
        self._w_mu_aligned = None  # registered on the device by the first act_rollout

    def grad_ready_order(self):
        """Parameters in the order the fused minibatch backward finishes their gradients (the
        PPO tail, then the trunk layers from the last to the first): distributed.FlatGrads lays
        the flat gradient buffer out this way so its all-reduce overlaps the backward."""
        h = self._head
        la, lc = self.actor_mlp[h], self.critic_mlp[h]
        vh, mh = self.critic_mlp[h + 2], self.mu[0]
        order = [la.weight, la.bias, lc.weight, lc.bias, mh.weight, mh.bias, vh.weight, vh.bias]
        trunk = self._twin.params()
        for l in range(len(trunk) // 4 - 1, -1, -1):
            order += trunk[4 * l:4 * l + 4]
        return order

    def _compute_dtype(self):
        return torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else torch.float32

    def obs_half_input(self, obs, rows=None):
        """RunningNorm(obs[rows]) as the padded f16 / bf16 operand of the first trunk GEMM in one
        pass (phc_obs_half), or None when the current precision does not run the MFMA trunks.
        The trainer builds it once per train() call: the statistics only change between
        iterations (scripts/train.py:337-346)."""
        if not (self.fused and obs.is_cuda):
            return None
        dt = self._compute_dtype()
        width = half_input_width(self._twin, dt)
        if width is None:
            return None
        m = obs.shape[0] if rows is None else rows.shape[0]
        out = torch.empty((m, width), dtype=dt, device=obs.device)
        n = self.obs_norm
        return N.obs_half(obs, n.running_mean, n.running_var, n.epsilon, n.clip, out, rows)

    def act_rollout(self, obs, noise, actions, logprob, value, mu=None, obs_half=None):
        """Rollout inference (encode_observations + decode_actions + sample_logits) writing the
        sampled actions, their log-probability and the value into the given buffers: half input
        (phc_obs_half), MFMA trunks, then LayerNorm+SiLU, both heads, the Normal sample and
        log_prob in one kernel (phc_policy_act).  False when this precision / shape has no fused
        path (the caller then runs the module).  obs_half: the operand already built from obs (the
        env step's fused RunningNorm, HumanoidPHC.set_obs_operand)."""
        h = self._head
        if not (self.fused and self.fused_ln and twin_ln_silu_supported(self._twin.pairs[-1][0].weight.shape[0])):
            return False
        xc = obs_half if obs_half is not None else self.obs_half_input(obs)
        if xc is None:
            return False
        w = self.mu[0].weight
        if self._w_mu_aligned is None or self._w_mu_aligned.device != w.device:
            self._twin.extras = [e for e in self._twin.extras if e[0] is not w]
            # transposed [hidden, 72]: the tail's mu-head weight reads coalesce across the actions
            self._w_mu_aligned = self._twin.add_extra(w, transpose_ld=-(-w.shape[0] // 4) * 4)
        y = twin_trunks(xc, self._twin)  # refreshes the MFMA operands and the aligned mu weight
        la, lc = self.actor_mlp[h], self.critic_mlp[h]
        vh, mh = self.critic_mlp[h + 2], self.mu[0]
        # the mu weight's aligned copy, refreshed with the trunk operands by twin_trunks above (or
        # refresh_twin before a graph replay); the plain parameter on other paths
        w_mu_t = self._w_mu_aligned if _use_mfma(self._twin, xc.dtype) else None
        N.policy_act(y, (la.weight, la.bias), (lc.weight, lc.bias), la.eps, mh.weight, mh.bias, vh.weight, vh.bias,
                     self.sigma, noise, actions, logprob, value, mu=mu,
                     std_max=1e-6 if self._deterministic_action is True else float("inf"), w_mu_t=w_mu_t)
        return True

    def encode_observations(self, obs):
        if obs.dtype in (torch.float16, torch.bfloat16):
            self.obs_pointer = obs  # obs_half_input's output: normalised, padded GEMM operand
        else:
            self.obs_pointer = self.obs_norm(obs)
        if self.fused and obs.is_cuda:
            y = twin_trunks(self.obs_pointer, self._twin)  # [2, M, hidden]: actor, critic
            h = self._head
            if self.fused_ln and twin_ln_silu_supported(y.shape[2]):
                z = twin_ln_silu(y, self.actor_mlp[h], self.critic_mlp[h])  # LayerNorm + SiLU of both trunks
            else:
                z = [self.critic_mlp[h + 1](m[h](y[i])) if i else self.actor_mlp[h + 1](m[h](y[i]))
                     for i, m in enumerate((self.actor_mlp, self.critic_mlp))]
            self._critic_trunk = z[1]
            return z[0], None
        self._critic_trunk = None
        return self.actor_mlp(self.obs_pointer), None

    def forward_train(self, obs):
        """(mu [M, A], value [M, 1]) for the fused PPO objective (clean_pufferl/ppo_loss.py): the
        device path of encode_observations + decode_actions without the Normal distribution."""
        hidden, _ = self.encode_observations(obs)
        if self._critic_trunk is None:
            raise RuntimeError("forward_train needs the device (twin-trunk) path")
        mu = head_linear(hidden, self.mu[0]).float()
        value = head_linear(self._critic_trunk, self.critic_mlp[self._head + 2]).float()
        self._critic_trunk = None
        return mu, value

    def decode_actions(self, hidden, lookup=None):
        if self._critic_trunk is not None:  # device path: heads with split-K / chunked-sum gradients
            mu = head_linear(hidden, self.mu[0]).float()
        else:
            mu = self.mu(hidden).float()  # fp32 head under autocast
        std = torch.exp(self.sigma).expand_as(mu)
        if self._deterministic_action is True:
            std = torch.clamp(std, max=1e-6)
        probs = torch.distributions.Normal(mu, std, validate_args=False)  # no host-syncing checks
        if self.training:
            self.mean_bound_loss = self.bound_loss(mu)
        if self._critic_trunk is not None:
            value = head_linear(self._critic_trunk, self.critic_mlp[self._head + 2]).float()
            self._critic_trunk = None
        else:
            value = self.critic_mlp(self.obs_pointer).float()
        return probs, value
