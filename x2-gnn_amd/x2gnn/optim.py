"""The reference trainer's parameter update on flat buffers (trainer.py:39-48, train_ema.py:45-48).

``FlatAdam`` re-homes every parameter as a view of ONE flat fp32 buffer (the gradient side is
``dist.GradBucket``'s flat buffer), so clip_grad_norm_ + Adam + the EMA of AveragedModel are
two launches of ``x2g_clip_adam_ema`` over contiguous memory instead of torch's per-tensor
foreach/capturable kernels.  Step count, norm and bias corrections live on the device, so the
update can sit inside a captured HIP graph.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import call, ptr, stream_ptr
from .dist import GradBucket, flat_layout

_LR, _B1, _B2, _EPS, _MAXN, _EMAD, _STEP, _NORM, _CLIP = range(9)
_WARMUP, _DECAY_STEPS, _DECAY_RATE, _BASE_LR, _STAIRCASE = range(11, 16)


class FlatAdam:
    """Adam(lr, betas, eps, amsgrad=False) + clip_grad_norm_(max_norm) + EMA(decay) over flat buffers.

    ``params`` must all be fp32 CUDA tensors; they become views of ``self.flat`` (values kept).
    ``ema`` (a flat buffer, same layout) holds the AveragedModel parameters; ``ema_params()``
    returns them shaped like the model's parameters."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, max_norm=100.0, ema_decay=0.95,
                 bucket: GradBucket | None = None):
        self.params = [p for p in params if p.requires_grad]
        dev = self.params[0].device
        self.offsets, n = flat_layout(self.params)  # same layout as GradBucket: 16-byte aligned views
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        for p, off in zip(self.params, self.offsets):
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
        self.bucket = bucket if bucket is not None else GradBucket(self.params)
        if self.bucket.offsets != self.offsets:
            raise ValueError("gradient bucket does not cover the same parameters")
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.ema = self.flat.clone() if ema_decay is not None else None
        sc = torch.zeros(16, dtype=torch.float32)
        sc[[_LR, _B1, _B2, _EPS, _MAXN, _EMAD]] = torch.tensor(
            [lr, betas[0], betas[1], eps, max_norm if max_norm else 0.0, ema_decay or 0.0], dtype=torch.float32)
        self.scalars = sc.to(dev)
        self.ws_bytes = int(_lib.load().x2g_optimizer_workspace(n))
        self.ws = torch.empty(max(self.ws_bytes, 4), dtype=torch.uint8, device=dev)

    def step(self, zero_grads=False):
        """One update; ``zero_grads``: also zero the gradient bucket as it is read (zero_grad()
        folded into the step's last kernel, so the next backward needs no fill)."""
        call("x2g_clip_adam_ema_ex", ptr(self.flat), ptr(self.bucket.flat), ptr(self.exp_avg), ptr(self.exp_avg_sq),
             ptr(self.ema), self.flat.numel(), ptr(self.scalars), 1 if zero_grads else 0, ptr(self.ws),
             self.ws_bytes, stream_ptr())

    def set_lr(self, lr):
        """A fixed learning rate from the next step on (clears a schedule; e.g. for a host-side
        ReduceLROnPlateau, train_ema.py:52-53)."""
        self.scalars[_WARMUP] = 0.0
        self.scalars[_LR] = lr

    def set_schedule(self, warmup_steps, decay_steps, decay_rate, staircase=False, base_lr=None):
        """LinearWarmupExponentialDecay (scheduler.py:4-31; train_ema.py:50-51) evaluated on the device
        from the step count at every update, so captured HIP graphs follow it: update t (0-based)
        uses base_lr * min(1/W + t/W, 1) * decay_rate^(t / decay_steps), as the reference's
        LambdaLR gives optimizer.step() when scheduler.step() follows every batch (trainer.py:47)."""
        if decay_rate > 1:
            raise ValueError("decay_rate must be <= 1 (scheduler.py:16)")
        base = float(self.scalars[_LR]) if base_lr is None and float(self.scalars[_WARMUP]) <= 0 else base_lr
        base = float(self.scalars[_BASE_LR]) if base is None else float(base)
        vals = torch.tensor([max(int(warmup_steps), 1), float(decay_steps), float(decay_rate), base,
                             1.0 if staircase else 0.0], dtype=torch.float32)
        self.scalars[_WARMUP:_STAIRCASE + 1] = vals.to(self.scalars.device)

    @property
    def lr(self):
        """The learning rate the last update used (device scalar)."""
        return self.scalars[_LR]

    @property
    def grad_norm(self):
        return self.scalars[_NORM]

    @property
    def steps(self):
        return self.scalars[_STEP]

    def ema_params(self):
        return [self.ema[off:off + p.numel()].view_as(p) for p, off in zip(self.params, self.offsets)]
