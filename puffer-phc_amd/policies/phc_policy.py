"""PHCPolicy (puffer_phc/policies/phc_policy.py:10-61): 6-layer SiLU actor and critic with a
LayerNorm head, fixed-sigma Normal.  State-dict keys match the reference
(tests/golden/state_dict_keys.tsv)."""

from typing import Sequence

import torch
from torch import nn

from .discriminator_policy import DiscriminatorPolicy
from .pufferl_policy import Linear, layer_init
from .twin_mlp import TwinWeights, head_linear, twin_ln_silu, twin_ln_silu_supported, twin_trunks


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

    def encode_observations(self, obs):
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
