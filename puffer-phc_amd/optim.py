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
import os

import torch

from . import _native as N
from .policies import weight_cache

_STATE_BYTES = ctypes.sizeof(N.OptStateC)
# the step writes the registered GEMM-operand copies itself (PHC_OPERANDS_IN_STEP=0: the caches
# refresh them with their own phc_pack_weights launch)
OPERANDS_IN_STEP = os.environ.get("PHC_OPERANDS_IN_STEP", "1") != "0"


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
        # the gradient buffer's layout (64-B aligned parameter slices; the gaps are zeros here too)
        self.param_flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self._views = []
        chunk = int(N.lib().phc_opt_block_elems())
        ranges, seg_blk = [], [0]
        with torch.no_grad():
            for p in params:
                off, end = flat_grads._range[id(p)]
                k = end - off
                view = self.param_flat[off:off + k].view_as(p)
                view.copy_(p)
                p.data = view
                self._views.append((off, k))
                for s in range(off, off + k, chunk):
                    ranges.append((s, min(s + chunk, off + k)))
                seg_blk.append(len(ranges))
        self._blk = torch.tensor(ranges, dtype=torch.int64, device=dev)
        self._seg = torch.tensor(seg_blk, dtype=torch.int32, device=dev)
        self._ws = torch.empty(int(N.lib().phc_opt_workspace_bytes(len(ranges))), dtype=torch.uint8, device=dev)
        self._state = torch.zeros(_STATE_BYTES, dtype=torch.uint8, device=dev)
        self._f = self._state.view(torch.float32)
        self._i = self._state.view(torch.int32)
        self._f[0] = init_scale
        self._lr_dev = None  # the learning rate last written to the device state (phc_opt_state.lr)
        # GEMM-operand caches whose copies the step writes (phc_opt_step_operands): the device job
        # table, its job / workgroup counts, the caches it covers, the registry version it was built at
        self._ops, self._ops_owners, self._ops_v = None, [], -1
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
        self._lr_dev = None
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

    _LR_SLOT = 8  # phc_opt_state.lr as a float index of the state buffer

    def sync_lr(self):
        """Write param_groups[0]["lr"] into the device state the step kernel reads it from (when it
        changed): a captured hipGraph of the update then follows the schedule the trainer sets
        between replays (clean_pufferl's anneal, scripts/train.py's decay).  Stream-ordered."""
        lr = float(self.param_groups[0]["lr"])
        if lr != self._lr_dev:
            self._f[self._LR_SLOT].fill_(lr)
            self._lr_dev = lr

    def _operand_table(self):
        """(Re)build the job table of phc_opt_step_operands when the operand-cache registry changed:
        every registered cache whose copied parameters all live in the flat buffer gets one tile job
        per parameter (its copy destinations), flat jobs cover the rest of the buffer.  None (plain
        phc_opt_step + the caches' own refresh) when nothing is covered or two copies overlap."""
        v = weight_cache.plans_version()
        if v == self._ops_v:
            return self._ops
        if torch.cuda.is_current_stream_capturing():
            return None  # the table upload is a host copy: not inside a capture (the caches refresh)
        self._ops_v, self._ops, self._ops_owners = v, None, []
        base, n = self.param_flat.data_ptr(), self.param_flat.numel()
        tiles, owners = [], []
        for owner in weight_cache.plan_owners():
            js = []
            for src, dst, dst_t in owner.plan_jobs:
                s2 = src if src.dim() == 2 else src.reshape(1, -1)
                rows, cols = s2.shape
                off = src.data_ptr() - base
                if (src.dtype != torch.float32 or not src.is_contiguous() or off < 0 or off % 4
                        or off // 4 + rows * cols > n):
                    js = None
                    break
                ref = dst if dst is not None else dst_t
                dl = (dst if dst.dim() == 2 else dst.reshape(1, -1)).stride(0) if dst is not None else 0
                tl = (dst_t if dst_t.dim() == 2 else dst_t.reshape(-1, 1)).stride(0) if dst_t is not None else 0
                if (dst is not None and dst.dim() == 2 and dst.stride(1) != 1) or \
                        (dst_t is not None and dst_t.dim() == 2 and dst_t.stride(1) != 1):
                    js = None
                    break
                js.append((off // 4, rows, cols, dst, dst_t, dl if rows > 1 else cols, tl, N.DTYPE_CODE[ref.dtype]))
            if js:
                tiles += js
                owners.append(owner)
        if not tiles:
            return None
        tiles.sort(key=lambda j: j[0])
        jobs, pos = [], 0
        for j in tiles:
            if j[0] < pos:  # two copies of one parameter: leave the caches to their own refresh
                return None
            if j[0] > pos:
                jobs.append((pos, j[0] - pos, 0, None, None, 0, 0, 0, N.ADAM_FLAT))
            jobs.append(j + (N.ADAM_TILE,))
            pos = j[0] + j[1] * j[2]
        if pos < n:
            jobs.append((pos, n - pos, 0, None, None, 0, 0, 0, N.ADAM_FLAT))
        if len(jobs) > N.MAX_ADAM_JOBS:
            return None
        arr = (N.AdamJobC * len(jobs))()
        blocks = 0
        for q, (off, rows, cols, dst, dst_t, dl, tl, dt, kind) in enumerate(jobs):
            nb = int(N.lib().phc_adam_job_blocks(kind, rows, cols))
            arr[q] = N.AdamJobC(off, rows, cols, dst.data_ptr() if dst is not None else None,
                                dst_t.data_ptr() if dst_t is not None else None, dl, tl, blocks,
                                -(-cols // 64) if kind == N.ADAM_TILE else 0, dt, kind)
            blocks += nb
        host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        table = host.to(self.param_flat.device)
        self._ops = (table, len(jobs), blocks, [t[3:5] for t in tiles])  # keeps the destinations alive
        self._ops_owners = owners
        return self._ops

    def fresh_operand_owners(self):
        """The covered operand caches that are current now (a step keeps them current)."""
        return [o for o in self._ops_owners if weight_cache.is_fresh(o)] if self._ops is not None else []

    def operands_written(self, owners):
        """After steps that wrote the copies (phc_opt_step_operands, or a replayed graph of them):
        invalidate every other cache, keep the covered ones that were current before."""
        weight_cache.bump()
        for o in owners:
            weight_cache.mark_fresh(o)

    def fused_step(self, max_norm, norm_acc=None):
        """clip_grad_norm_(max_norm) + Adam (+ loss-scale update); returns the device [3] tensor
        (sum of per-parameter gradient norms as the reference logs, global norm, L2-init
        distance of the parameters before the update when tracked).  The learning rate comes from
        the device state (sync_lr); under graph capture the caller syncs it before each replay.
        norm_acc (device float64 [3], optional) += that tensor in the same launch."""
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        gf, bf, gi = self._hp_scale
        if not torch.cuda.is_current_stream_capturing():
            self.sync_lr()
        hp = N.AdamParamsC(float(g["lr"]), b1, b2, float(g["eps"]), float(max_norm) if math.isfinite(max_norm)
                           else 3.0e38, int(self.use_loss_scale), gf, bf, gi, 1)
        n = self.param_flat.numel()
        ops = self._operand_table() if OPERANDS_IN_STEP else None
        args = (self.param_flat.data_ptr(), self.flat_grads.flat.data_ptr(), self.exp_avg.data_ptr(),
                self.exp_avg_sq.data_ptr(), n, self._blk.data_ptr(), self._blk.shape[0], self._seg.data_ptr(),
                self._seg.numel() - 1, ctypes.byref(hp), self._state.data_ptr(), self.norms.data_ptr(),
                self.param_init.data_ptr() if self.param_init is not None else None, self._ws.data_ptr(),
                N._ptr(norm_acc, torch.float64, (3,), "norm_acc", nullable=True))
        if ops is None:
            N._check(N.lib().phc_opt_step(*args, N._stream()), "phc_opt_step")
            # the parameters changed behind torch's version counters: every GEMM-operand cache of
            # them is stale now (policies/weight_cache.py)
            weight_cache.bump()
        else:
            fresh = self.fresh_operand_owners()
            table, njobs, blocks, _ = ops
            N._check(N.lib().phc_opt_step_operands(*args, table.data_ptr(), njobs, blocks, N._stream()),
                     "phc_opt_step_operands")
            self.operands_written(fresh)
        return self.norms
