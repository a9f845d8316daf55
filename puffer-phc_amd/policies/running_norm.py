"""RunningNorm (puffer_phc/policies/running_norm.py:5-53) with HIP batch statistics.

forward: clamp((x - mean) / sqrt(var + eps), -clip, clip) (phc_rms_normalize on device,
differentiable w.r.t. nothing, like the reference's buffers-only module);
update: whole-batch mean / biased var folded in with weight 1/count (phc_rms_update).
Under torch.distributed the batch moments are merged across ranks first so every replica keeps
identical stats.
"""

import torch
from torch import nn

from .. import _native
from .. import distributed as D


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
        if not x.is_cuda:
            raise RuntimeError("RunningNorm runs on the HIP path only (float32 [rows, features] device tensor)")
        if D.is_dist():
            return self._update_distributed(x.contiguous())
        self._ws = _native.rms_update(x.contiguous(), self.running_mean, self.running_var, self.count, self._ws)

    def _update_distributed(self, x):
        """The global batch's mean / biased var over all ranks' rows: each rank's (mean, M2) per
        feature (phc_rms_moments, float64), one all-gather, the ranks' moments merged in rank
        order on every rank (phc_rms_apply: identical stats on every replica), then the
        reference's running update."""
        import torch.distributed as dist

        mom, self._ws = _native.rms_moments(x, self._ws)
        ws = D.world_size()
        moms = [torch.empty_like(mom) for _ in range(ws)]
        dist.all_gather(moms, mom)
        rows = torch.tensor([float(x.shape[0])], dtype=torch.float64, device=x.device)
        all_rows = [torch.empty_like(rows) for _ in range(ws)]
        dist.all_gather(all_rows, rows)
        _native.rms_apply(torch.stack(moms).contiguous(), torch.cat(all_rows).contiguous(), self.running_mean,
                          self.running_var, self.count)
