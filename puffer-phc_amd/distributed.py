"""Data parallelism over GPUs: one process per GPU, torch.distributed over RCCL (xGMI).

Envs shard across ranks (each rank steps its own envs and motion library: no data-path
collective in the rollout).  The PPO update needs exactly these collectives:
  (1) the gradient all-reduce of every minibatch — gradients live in ONE flat fp32 buffer
      (parameters' .grad are views into it), reduced in `bucket_bytes` slices so RCCL runs a
      few large ring all-reduces instead of one per parameter;
  (2) the advantage-normalisation statistics (sum, sum of squares, count) per minibatch;
  (3) the RunningNorm batch statistics (policies/running_norm.py);
  (4) scalar loss / SPS reductions for logging;
  (5) a broadcast of the initial parameters so replicas start identical.
With world_size 1 every helper is a no-op and the math is the reference's single-GPU math.
"""

import os

import torch
import torch.distributed as dist


def is_dist():
    """A process group is up: every collective below runs (a 1-rank group included, so the
    data-parallel path can be exercised on one GPU; without a group they are all no-ops)."""
    return dist.is_available() and dist.is_initialized()


def backend():
    """The process group's backend ("nccl" = RCCL on ROCm, "gloo"), None without a group."""
    return dist.get_backend() if is_dist() else None


def world_size():
    return dist.get_world_size() if is_dist() else 1


def rank():
    return dist.get_rank() if is_dist() else 0


def init_from_env(backend=None, force=False):
    """Initialise from torchrun's env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*); a single
    process only with force=True (a 1-rank group: the data-parallel path on one GPU)."""
    if (int(os.environ.get("WORLD_SIZE", "1")) <= 1 and not force) or dist.is_initialized():
        return rank(), world_size()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device("cuda", local))
    else:
        if torch.cuda.device_count() > 0:  # gloo over device tensors (rank rehearsal on one GPU)
            torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(backend)
    return rank(), world_size()


PARAM_ALIGN = 16  # elements: each parameter's slice of the flat buffers starts 64-B aligned


class FlatGrads:
    """Parameters' gradients as views into one flat buffer, all-reduced (averaged) in buckets.

    `order` (optional) lists parameters in the order the backward finishes their gradients
    (PHCPolicy.grad_ready_order: the PPO tail, then the trunk layers from the last to the first);
    the flat buffer is laid out in that order, so during an overlapped backward
    (overlap_begin / overlap_finish) each group the backward reports done is one contiguous
    slice whose all-reduce runs on RCCL's stream while the earlier layers' gradients are still
    being computed."""

    def __init__(self, params, bucket_bytes=32 << 20, order=None):
        # the module's own parameter order (requires_grad or not): the index space of a
        # torch.optim.Adam(module.parameters()) state dict (optim.FlatAdam.state_dict)
        self.module_params = list(params)
        params = [p for p in self.module_params if p.requires_grad]
        if order is not None:
            first = [p for p in order if p.requires_grad]
            ids = {id(p) for p in first}
            params = first + [p for p in params if id(p) not in ids]
        self.params = params
        # every parameter starts on a 64-B boundary (PARAM_ALIGN elements): the optimizer's per-tile
        # passes (phc_opt_step_operands) then read whole aligned float4s of any parameter; the gaps
        # stay zero (no gradient, no parameter, Adam keeps them at zero)
        offs, off = [], 0
        for p in self.params:
            off = -(-off // PARAM_ALIGN) * PARAM_ALIGN
            offs.append(off)
            off += p.numel()
        dev = self.params[0].device
        self.flat = torch.zeros(off, dtype=torch.float32, device=dev)
        self._range = {}
        for p, o in zip(self.params, offs):
            k = p.numel()
            p.grad = self.flat[o:o + k].view_as(p)
            self._range[id(p)] = (o, o + k)
        self.bucket = max(1, bucket_bytes // 4)
        self._works = None
        self._done = None
        # measurement aid (bench.py at N > 1): events on the compute stream around the wait for the
        # backward's all-reduces — the time the stream stalls on RCCL after its last backward kernel
        self.timing = False
        self.exposed = []

    def overlap_begin(self):
        """Install the gradient-ready hook for one backward (a no-op without data parallelism)."""
        if not is_dist():
            return
        from .policies import twin_mlp
        self._works, self._done = [], set()
        twin_mlp.GRAD_READY = self._on_ready

    def _on_ready(self, params):
        """All-reduce the (contiguous) slices of parameters whose gradients are final, async."""
        spans = sorted(self._range[id(p)] for p in params if id(p) in self._range and id(p) not in self._done)
        for p in params:
            self._done.add(id(p))
        s0 = e0 = None
        for s, e in spans + [(None, None)]:
            if s is not None and e0 is not None and 0 <= s - e0 < PARAM_ALIGN:  # adjacent (alignment gap)
                e0 = e
                continue
            if s0 is not None:
                self._works.append(dist.all_reduce(self.flat[s0:e0], async_op=True))
            s0, e0 = s, e

    def overlap_finish(self):
        """Reduce every gradient not reported during the backward, wait, average."""
        if not is_dist():
            return
        from .policies import twin_mlp
        twin_mlp.GRAD_READY = None
        rest = [p for p in self.params if id(p) not in self._done]
        if rest:
            self._on_ready(rest)
        ev = None
        # (timing events cannot be recorded inside a captured graph: a captured backward is not timed)
        if self.timing and self.flat.is_cuda and not torch.cuda.is_current_stream_capturing():
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        for w in self._works:
            w.wait()
        if ev is not None:
            ev[1].record()
            self.exposed.append(ev)
        self._works, self._done = None, None
        self.flat.div_(world_size())

    def exposed_ms(self):
        """Mean exposed all-reduce wait per backward (ms) over the timed backwards, and their count."""
        if not self.exposed:
            return None, 0
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self.exposed) / len(self.exposed), len(self.exposed)

    def zero(self):
        self.flat.zero_()

    def fill_grads_(self, value):
        """Fill every parameter's gradient view (the alignment gaps between them keep their zeros):
        tests pre-fill with NaN to prove a backward writes every gradient."""
        for p in self.params:
            p.grad.fill_(value)

    def allreduce_mean(self):
        if not is_dist():
            return
        ws = world_size()
        works = []
        for s in range(0, self.flat.numel(), self.bucket):
            works.append(dist.all_reduce(self.flat[s:s + self.bucket], async_op=True))
        for w in works:
            w.wait()
        self.flat.div_(ws)

    def norms_sum(self):
        """sum over parameters of ||grad_p|| (clean_pufferl/core.py:366-368), on device."""
        return torch.stack(torch._foreach_norm([p.grad for p in self.params])).sum()

    def clip_(self, max_norm):
        """torch.nn.utils.clip_grad_norm_ over the flat buffer (one multi-tensor norm, one scale
        kernel).  Returns the sum of per-parameter norms the reference logs."""
        norms = torch.stack(torch._foreach_norm([p.grad for p in self.params]))
        total = torch.linalg.vector_norm(norms)
        coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
        self.flat.mul_(coef)
        return norms.sum()


def broadcast_params(module, src=0):
    if not is_dist():
        return
    from .policies import weight_cache

    for t in list(module.parameters()) + list(module.buffers()):
        dist.broadcast(t.data, src)
    weight_cache.bump()  # written through .data: invisible to the version counters


def global_mean_std(x):
    """Mean and unbiased std over all ranks' elements of x (torch.std semantics)."""
    if not is_dist():
        return x.mean(), x.std()
    xd = x.double()
    buf = torch.stack([xd.sum(), (xd * xd).sum(),
                       torch.tensor(float(x.numel()), dtype=torch.float64, device=x.device)])
    dist.all_reduce(buf)
    n = buf[2]
    mean = buf[0] / n
    var = (buf[1] - n * mean * mean) / (n - 1)
    return mean.float(), var.clamp_min(0).sqrt().float()


def global_mean_std_rows(x):
    """[rows, 2] (mean, unbiased std) of each row of x over all ranks' copies of that row — the
    per-minibatch advantage statistics of a whole train() call in one reduction (and one
    all-reduce), instead of two reductions (and an all-reduce) per minibatch."""
    if not is_dist():
        return torch.stack([x.mean(1), x.std(1)], 1).contiguous()
    xd = x.double()
    buf = torch.stack([xd.sum(1), (xd * xd).sum(1),
                       torch.full((x.shape[0],), float(x.shape[1]), dtype=torch.float64, device=x.device)], 1)
    dist.all_reduce(buf)
    n = buf[:, 2]
    mean = buf[:, 0] / n
    var = (buf[:, 1] - n * mean * mean) / (n - 1)
    return torch.stack([mean, var.clamp_min(0).sqrt()], 1).float().contiguous()


def allreduce_sum_(t):
    if is_dist():
        dist.all_reduce(t)
    return t


def allreduce_max_(t):
    if is_dist():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t
