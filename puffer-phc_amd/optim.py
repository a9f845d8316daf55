"""Flat-buffer Adam for the PPO update (R21; reference: clean_pufferl/core.py:360-372).

The reference runs loss.backward(); clip_grad_norm_(parameters, max_grad_norm);
optimizer.step() with torch.optim.Adam(lr, eps=1e-5) — per-parameter tensors, so torch issues a
multi-tensor norm, a clip, (with fp16: a GradScaler unscale, inf check and update) and the fused
Adam, each over the ~17 M parameters.  Here parameters, gradients (distributed.FlatGrads) and
both Adam moments are single flat fp32 buffers whose per-parameter slices the modules and the
optimizer state see as views, and the whole tail is phc_opt_step (phc_optim.hip): three
launches, deterministic reductions, the clip coefficient / skip decision / Adam step count /
loss scale kept on the device.  The object is a torch.optim.Adam (param_groups, lr schedule,
state_dict round trip in torch's format) whose step() runs the fused kernel.
"""

import ctypes
import math

import torch

from . import _native as N
from .policies import weight_cache

_STATE_BYTES = ctypes.sizeof(N.OptStateC)


# the index space of FlatAdam.state_dict()'s "state" keys: the module's parameter order, as a
# torch.optim.Adam(policy.parameters()) checkpoint (marker written into "flat_adam")
INDEX_SPACE = "module"


class FlatAdam(torch.optim.Adam):
    """torch.optim.Adam over the FlatGrads parameter set with the fused clip / loss-scale /
    Adam step.  use_loss_scale follows torch.amp.GradScaler's defaults (init 2^16, growth 2 every
    2000 clean steps, backoff 0.5, the step skipped on inf / nan gradients)."""

    def __init__(self, flat_grads, lr, eps=1e-5, betas=(0.9, 0.999), use_loss_scale=False, init_scale=2.0 ** 16,
                 growth_factor=2.0, backoff_factor=0.5, growth_interval=2000):
        params = flat_grads.params
        dev = params[0].device
        super().__init__(params, lr=lr, eps=eps, betas=betas)
        self.flat_grads = flat_grads
        n = flat_grads.flat.numel()
        self.param_flat = torch.empty(n, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self._views = []
        off = 0
        chunk = int(N.lib().phc_opt_block_elems())
        ranges, seg_blk = [], [0]
        with torch.no_grad():
            for p in params:
                k = p.numel()
                view = self.param_flat[off:off + k].view_as(p)
                view.copy_(p)
                p.data = view
                self._views.append((off, k))
                for s in range(off, off + k, chunk):
                    ranges.append((s, min(s + chunk, off + k)))
                seg_blk.append(len(ranges))
                off += k
        self._blk = torch.tensor(ranges, dtype=torch.int64, device=dev)
        self._seg = torch.tensor(seg_blk, dtype=torch.int32, device=dev)
        self._ws = torch.empty(int(N.lib().phc_opt_workspace_bytes(len(ranges))), dtype=torch.uint8, device=dev)
        self._state = torch.zeros(_STATE_BYTES, dtype=torch.uint8, device=dev)
        self._f = self._state.view(torch.float32)
        self._i = self._state.view(torch.int32)
        self._f[0] = init_scale
        # [sum of per-param norms, total norm, L2-init regulariser]
        self.norms = torch.zeros(3, dtype=torch.float32, device=dev)
        self.param_init = None
        self.use_loss_scale = bool(use_loss_scale)
        self._hp_scale = (growth_factor, backoff_factor, growth_interval)
        self._bind_state()

    # -- torch.optim.Adam surface ---------------------------------------------------------
    def _bind_state(self):
        """Per-parameter state entries are views of the flat moments (torch's state format)."""
        for p, (off, k) in zip(self.flat_grads.params, self._views):
            st = self.state[p]
            st["exp_avg"] = self.exp_avg[off:off + k].view_as(p)
            st["exp_avg_sq"] = self.exp_avg_sq[off:off + k].view_as(p)
            st["step"] = self._i[2:3].view(())  # int32 device step counter shared by all slices

    def state_dict(self):
        """torch.optim.Adam's state dict as the REFERENCE's optimizer would write it
        (clean_pufferl/utils.py:18-42 saves torch.optim.Adam(policy.parameters()).state_dict()):
        parameter indices in the module's parameter order (frozen ones, e.g. sigma, included and
        without state), per-parameter exp_avg / exp_avg_sq / step.  The loss-scaler state rides
        in an extra "flat_adam" entry that torch's load_state_dict ignores."""
        sd = super().state_dict()
        order = self.flat_grads.module_params
        views = {id(p): v for p, v in zip(self.flat_grads.params, self._views)}
        step = torch.tensor(float(self._i[2]))
        state = {}
        for i, p in enumerate(order):
            if id(p) in views:
                off, k = views[id(p)]
                state[i] = {"step": step.clone(), "exp_avg": self.exp_avg[off:off + k].view_as(p).clone(),
                            "exp_avg_sq": self.exp_avg_sq[off:off + k].view_as(p).clone()}
        group = {k: v for k, v in sd["param_groups"][0].items() if k != "params"}
        group["params"] = list(range(len(order)))
        return {"state": state, "param_groups": [group],
                "flat_adam": {"loss_scale": float(self._f[0]), "growth_tracker": int(self._i[1]),
                              "skipped": int(self._i[3]), "index_space": INDEX_SPACE}}

    def load_state_dict(self, state_dict):
        """Loads a state dict in the module-parameter index space (what state_dict writes and what
        a torch.optim.Adam(policy.parameters()) checkpoint holds)."""
        extra = state_dict.get("flat_adam")
        if extra is not None and extra.get("index_space") != INDEX_SPACE:
            # FlatAdam before round 4 wrote its state in the flat, grad-ready order; the twin layers
            # share shapes, so such moments could load into the wrong parameters without any error
            raise ValueError("optimizer state dict written by an older FlatAdam (flat grad-ready index order, "
                             f"no flat_adam['index_space'] == {INDEX_SPACE!r}); it cannot be mapped to parameters")
        order = self.flat_grads.module_params
        groups = state_dict["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(order):
            raise ValueError(f"optimizer state dict has {sum(len(g['params']) for g in groups)} parameters in "
                             f"{len(groups)} groups; this policy has {len(order)} in one")
        views = {id(p): v for p, v in zip(self.flat_grads.params, self._views)}
        step = 0
        with torch.no_grad():
            for i, p in zip(groups[0]["params"], order):
                st = state_dict["state"].get(i)
                if st is None or id(p) not in views:
                    continue
                off, k = views[id(p)]
                if tuple(st["exp_avg"].shape) != tuple(p.shape) or tuple(st["exp_avg_sq"].shape) != tuple(p.shape):
                    raise ValueError(f"optimizer state {i}: moments of shape {tuple(st['exp_avg'].shape)} for a "
                                     f"parameter of shape {tuple(p.shape)}")
                self.exp_avg[off:off + k].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                step = int(float(st["step"]))
            self._i[2] = step
            if extra:
                self._f[0] = extra["loss_scale"]
                self._i[1] = extra["growth_tracker"]
                self._i[3] = extra["skipped"]
        for k, v in groups[0].items():
            if k != "params":
                self.param_groups[0][k] = v
        self._bind_state()
        weight_cache.bump()

    @torch.no_grad()
    def step(self, closure=None):
        """Adam step on the current gradients (no clipping)."""
        loss = closure() if closure is not None else None
        self.fused_step(math.inf)
        return loss

    # -- fused PPO update tail ------------------------------------------------------------
    def scale(self, loss):
        """loss * current loss scale (identity without loss scaling)."""
        return loss * self._f[0] if self.use_loss_scale else loss

    def backward(self, loss):
        """(loss * loss scale).backward() without the scalar kernels: the scale (a 0-dim view of
        the device state, or a cached 1) is handed to autograd as the loss's gradient, so no
        ones-fill, product or product-backward launches precede the policy's backward."""
        if self.use_loss_scale:
            seed = self._f[0]
        else:
            seed = getattr(self, "_one", None)
            if seed is None or seed.device != loss.device:
                seed = self._one = torch.ones((), device=loss.device)
        torch.autograd.backward(loss, grad_tensors=seed.to(loss.dtype) if loss.dtype != seed.dtype else seed)

    @property
    def loss_scale(self):
        return self._f[0:1]

    @property
    def skipped_steps(self):
        """Device int32: steps skipped for inf / nan gradients."""
        return self._i[3]

    def track_init_distance(self):
        """Keep a flat copy of the current parameters; every fused_step then also reports
        sum_p mean((p - p0)^2) over them (norms[2]), the L2-init regulariser the reference logs
        each minibatch (clean_pufferl/core.py:352-359), from the same pass over the buffers."""
        self.param_init = self.param_flat.detach().clone()

    def fused_step(self, max_norm):
        """clip_grad_norm_(max_norm) + Adam (+ loss-scale update); returns the device [3] tensor
        (sum of per-parameter gradient norms as the reference logs, global norm, L2-init
        distance of the parameters before the update when tracked)."""
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        gf, bf, gi = self._hp_scale
        hp = N.AdamParamsC(float(g["lr"]), b1, b2, float(g["eps"]), float(max_norm) if math.isfinite(max_norm)
                           else 3.0e38, int(self.use_loss_scale), gf, bf, gi, 0)
        n = self.param_flat.numel()
        N._check(N.lib().phc_opt_step(self.param_flat.data_ptr(), self.flat_grads.flat.data_ptr(),
                                      self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), n, self._blk.data_ptr(),
                                      self._blk.shape[0], self._seg.data_ptr(), self._seg.numel() - 1,
                                      ctypes.byref(hp), self._state.data_ptr(), self.norms.data_ptr(),
                                      self.param_init.data_ptr() if self.param_init is not None else None,
                                      self._ws.data_ptr(), N._stream()),
                 "phc_opt_step")
        # the parameters changed behind torch's version counters: every GEMM-operand cache of
        # them is stale now (policies/weight_cache.py)
        weight_cache.bump()
        return self.norms
