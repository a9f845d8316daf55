"""DiscriminatorPolicy (puffer_phc/policies/discriminator_policy.py:9-107)."""

import torch
from torch import nn

from . import disc_mlp
from .disc_mlp import mfma_disc_supported
from .pufferl_policy import Linear, layer_init
from .running_norm import RunningNorm
from .twin_mlp import _compute_dtype


class DiscriminatorPolicy(nn.Module):
    def __init__(self, env, hidden_size):
        super().__init__()
        self.is_continuous = True
        self._deterministic_action = False
        self.input_size = env.single_observation_space.shape[0]
        self.action_size = env.single_action_space.shape[0]
        self.soft_bound = 0.9 * float(env.single_action_space.high[0])
        self.obs_norm = RunningNorm(self.input_size)
        self.actor_mlp = None
        self.mu = nn.Sequential(layer_init(Linear(hidden_size, self.action_size), std=0.01))
        self.sigma = nn.Parameter(torch.zeros(self.action_size, dtype=torch.float32), requires_grad=False)
        nn.init.constant_(self.sigma, -2.9)
        self.critic_mlp = None
        self.use_amp_obs = getattr(env, "amp_observation_space", None) is not None
        self.amp_obs_norm = None
        if self.use_amp_obs:
            amp_obs_size = env.amp_observation_space.shape[0]
            self.amp_obs_norm = RunningNorm(amp_obs_size)
            self._disc_mlp = nn.Sequential(layer_init(Linear(amp_obs_size, 1024)), nn.ReLU(),
                                           layer_init(Linear(1024, hidden_size)), nn.ReLU())
            self._disc_logits = layer_init(Linear(hidden_size, 1))
        self.obs_pointer = None
        self.mean_bound_loss = None

    def forward(self, observations):
        hidden, lookup = self.encode_observations(observations)
        return self.decode_actions(hidden, lookup)

    def encode_observations(self, obs):
        raise NotImplementedError

    def decode_actions(self, hidden, lookup=None):
        raise NotImplementedError

    def set_deterministic_action(self, value):
        self._deterministic_action = value

    def discriminate(self, amp_obs):
        """Logits [rows, 1] (discriminator_policy.py:72-79); under f16 / bf16 autocast on the MFMA
        path (disc_mlp.py), otherwise the nn.Linear modules in fp32."""
        if not self.use_amp_obs:
            return None
        if mfma_disc_supported(self, _compute_dtype()):
            return disc_mlp.discriminate_rows(self, [(amp_obs.float().contiguous(), None)])
        return self._disc_logits(self._disc_mlp(self.amp_obs_norm(amp_obs)))

    def discriminate_rows(self, sources):
        """discriminate() of the concatenated rows of (amp_obs [*, D], row index [n] or None)
        sources, gathered inside the input kernel on the MFMA path (no copies of the rows)."""
        if mfma_disc_supported(self, _compute_dtype()):
            return disc_mlp.discriminate_rows(self, sources)
        return self.discriminate(torch.cat([src if idx is None else src[idx] for src, idx in sources]))

    @torch.no_grad()
    def adversarial_reward(self, sources):
        """-log(max(1 - sigmoid(logits), 1e-4)) [rows] of the concatenated sources
        (clean_pufferl/core.py:229-242)."""
        if mfma_disc_supported(self, _compute_dtype()):
            return disc_mlp.adversarial_reward(self, sources)
        logits = self.discriminate_rows(sources).float().reshape(-1)
        prob = 1 / (1 + torch.exp(-logits))
        return -torch.log(torch.maximum(1 - prob, torch.tensor(0.0001, device=logits.device)))

    def update_obs_rms(self, obs):
        self.obs_norm.update(obs)

    def update_amp_obs_rms(self, amp_obs):
        if self.use_amp_obs:
            self.amp_obs_norm.update(amp_obs)

    def bound_loss(self, mu):
        mu_loss = torch.zeros_like(mu)
        mu_loss = torch.where(mu > self.soft_bound, (mu - self.soft_bound) ** 2, mu_loss)
        mu_loss = torch.where(mu < -self.soft_bound, (mu + self.soft_bound) ** 2, mu_loss)
        return mu_loss.mean()
