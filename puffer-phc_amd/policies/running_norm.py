"""RunningNorm (puffer_phc/policies/running_norm.py:5-53) with HIP batch statistics.

forward: clamp((x - mean) / sqrt(var + eps), -clip, clip) (phc_rms_normalize on device,
differentiable w.r.t. nothing, like the reference's buffers-only module);
update: whole-batch mean / biased var folded in with weight 1/count (phc_rms_update).
Under torch.distributed the batch statistics are merged across ranks first so every replica
keeps identical stats.
"""

import torch
from torch import nn

from .. import _native


class RunningNorm(nn.Module):
    def __init__(self, shape: int, epsilon=1e-5, clip=10.0):
        super().__init__()
        self.register_buffer("running_mean", torch.zeros((1, shape), dtype=torch.float32))
        self.register_buffer("running_var", torch.ones((1, shape), dtype=torch.float32))
        self.register_buffer("count", torch.ones(1, dtype=torch.float32))
        self.epsilon = epsilon
        self.clip = clip
        self._ws = None

    def forward(self, x):
        if x.is_cuda and x.dtype == torch.float32 and x.dim() == 2:
            return _native.rms_normalize(x.contiguous(), self.running_mean, self.running_var, self.epsilon, self.clip)
        raise RuntimeError("RunningNorm runs on the HIP path only (float32 [rows, features] device tensor)")

    @torch.no_grad()
    def update(self, x):
        x = x.float()
        assert x.dim() == 2, "x must be 2D"
        if torch.distributed.is_available() and torch.distributed.is_initialized() and \
                torch.distributed.get_world_size() > 1:
            return self._update_distributed(x)
        self._ws = _native.rms_update(x.contiguous(), self.running_mean, self.running_var, self.count, self._ws)

    def _update_distributed(self, x):
        """Global batch mean / biased var over all ranks' rows via one all-reduce of
        (n, sum, sum of squares) in float64, then the reference's running update."""
        n = torch.tensor([x.shape[0]], dtype=torch.float64, device=x.device)
        s = x.double().sum(0)
        s2 = (x.double() ** 2).sum(0)
        buf = torch.cat([n, s, s2])
        torch.distributed.all_reduce(buf)
        F = x.shape[1]
        n_tot = buf[0]
        mean = buf[1:1 + F] / n_tot
        var = (buf[1 + F:] / n_tot - mean * mean).clamp_min(0.0)
        w = 1.0 / self.count
        self.running_mean.copy_(self.running_mean * (1 - w) + mean.float()[None] * w)
        self.running_var.copy_(self.running_var * (1 - w) + var.float()[None] * w)
        self.count += 1
