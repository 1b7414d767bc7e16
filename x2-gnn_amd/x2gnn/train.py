"""The reference trainer's per-batch step (trainer.py:37-48) on the device path, single- or
multi-rank (molecule-sharded data parallelism, x2gnn.dist).

``Trainer.step(batch)`` = forward (xgnn_poly.forward) + smooth-L1 loss (trainer.py:41) +
backward (trainer.py:42) into one flat gradient bucket + the gradient / loss all-reduce
(N > 1; §8(e) of SURVEY.md) + clip_grad_norm_(100) + Adam + EMA (trainer.py:44-48), with the
reference's per-batch LinearWarmupExponentialDecay (scheduler.py, trainer.py:47) when
``lr_schedule`` is given (evaluated on the device, so captured replays follow it).
``capture()`` records the step as two HIP graphs — forward+loss+backward, and the update — with
the all-reduce eager between them, so a replay enqueues the same kernels as an eager step
without the ~500 Python-side launches (the eager step is launch-bound).

Under data parallelism every rank owns a shard of the global batch (``dist.shard_by_triplets``:
balanced by triplet count, so shards hold unequal molecule counts).  The reference's loss is the
mean over the whole batch, so each rank's gradient of its own shard mean is weighted by
``local_count / global_count`` before the SUM all-reduce (``GradBucket.allreduce_mean``); the
shard's loss rides in the bucket's trailing slot, so the global mean loss comes out of the same
collective.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import ops
from .dist import GradBucket
from .optim import FlatAdam


def _world(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


class Trainer:
    """One training step over a resident batch with a flat gradient bucket.

    ``local_count`` / ``global_count``: molecules in this rank's shard / in the global batch
    (host ints from the sharding); None = every rank holds the same count (plain mean)."""

    def __init__(self, model, lr=1e-3, max_norm=100.0, ema_decay=0.95, local_count=None, global_count=None,
                 group=None, lr_schedule=None, exchange_chunks=1):
        """``lr_schedule``: None (constant ``lr``) or a dict of LinearWarmupExponentialDecay's
        arguments — warmup_steps, decay_steps, decay_rate[, staircase] (config.json: 3000, 3e6,
        0.01) — applied per step from base ``lr`` (FlatAdam.set_schedule).  ``exchange_chunks``: the
        gradient all-reduce as that many asynchronous collectives over contiguous bucket ranges
        (GradBucket.allreduce_mean(chunks=...)), joined before the optimizer."""
        self.model = model
        self.group = group
        self.multi = _world(group) > 1
        # one trailing float: the shard's loss, all-reduced together with the gradients
        self.bucket = GradBucket(model.parameters(), extra=1 if self.multi else 0)
        # clip_grad_norm_(100) + Adam(1e-3) + EMA(0.95) (config.json) in three launches over the
        # flat parameter / gradient buffers (x2gnn.optim.FlatAdam, csrc/optim.hip)
        self.opt = FlatAdam(model.parameters(), lr=lr, max_norm=max_norm, ema_decay=ema_decay, bucket=self.bucket)
        if lr_schedule is not None:
            self.opt.set_schedule(base_lr=lr, **lr_schedule)
        self.flat_launches = []  # [(rows, cols) per job] of the last backward's flat weight-gradient launches
        self.counts = (local_count, global_count)
        self.exchange_chunks = int(exchange_chunks)
        self.graphs = None
        self.loss = None
        self.grads_zeroed = False  # the bucket starts zeroed too; the first step zeroes it anyway
        # d loss / d loss, kept: autograd's per-step ones_like fill is skipped
        self.seed = torch.ones((), device=self.bucket.flat.device)

    def forward_backward(self, batch):
        """Forward + loss + backward into the bucket (no exchange, no update); returns the loss."""
        if not self.grads_zeroed:  # otherwise the previous update zeroed them (FlatAdam.step(zero_grads=True))
            self.bucket.zero()
        self.grads_zeroed = False
        self.model.train()  # trainer.py:30 (an Inference sharing the model may have left it in eval)
        res = self.model(batch)
        # trainer.py:41; the loss launch also writes d loss / d res for the seed (no backward launch)
        loss = ops.smooth_l1_loss(res, batch.y, unit_seed=self.seed)
        with ops.deferred_wgrad() as d:  # all layers' weight-gradient slab sums in one launch
            torch.autograd.backward(loss, self.seed)
        self.flat_launches = d.flat_launches
        if self.multi:
            self.bucket.extra_view.copy_(loss.detach().reshape(1))
        return loss

    def reduce(self):
        """The step's only exchange (N > 1): gradients + loss, count-weighted SUM all-reduce."""
        if not self.multi:
            return
        local, total = self.counts
        if local is None:
            self.bucket.allreduce_mean(group=self.group, chunks=self.exchange_chunks)
        else:
            self.bucket.allreduce_mean(group=self.group, local_count=local, global_count=total,
                                       chunks=self.exchange_chunks)

    def global_loss(self, local_loss):
        """The global-batch mean loss after ``reduce()`` (the shard's loss when single-rank)."""
        return self.bucket.extra_view[0] if self.multi else local_loss

    def update(self):
        self.opt.step(zero_grads=True)
        self.grads_zeroed = True

    def step(self, batch):
        """One step; returns the (global) loss as a device scalar.  After ``capture()`` it is the
        graph's own loss buffer — valid until the next step overwrites it (the CUDA / HIP graph output
        contract): read it (``float(loss)``) or ``clone()`` it to keep it.  (Copying it out on every step
        was a 4.6 µs launch of its own.)"""
        if self.graphs is None:
            loss = self.forward_backward(batch)
            self.reduce()
            self.update()
            return self.global_loss(loss)
        self.replay_forward_backward()
        self.reduce()
        self.graphs[1].replay()
        self.grads_zeroed = True
        return self.global_loss(self.loss)

    def replay_forward_backward(self):
        """Replay the captured forward+loss+backward (accumulates into the bucket: zeroed by the
        previous update, or by the caller); returns the captured loss tensor."""
        self.graphs[0].replay()
        self.grads_zeroed = False
        return self.loss

    def capture(self, batch, warm=3):
        """Record forward+backward and the update as two HIP graphs (warm-up passes on a side
        stream first: forward+backward+exchange only, the parameters are not updated)."""
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warm):
                self.forward_backward(batch)
                self.reduce()
        torch.cuda.current_stream().wait_stream(side)
        # the forward+backward graph accumulates into a zeroed bucket and does not zero it itself:
        # the update graph's last kernel does (FlatAdam.step(zero_grads=True)), so a replayed step
        # has no fill launch; a caller replaying g_fb alone zeroes the bucket first
        self.bucket.zero()
        self.grads_zeroed = True
        g_fb, g_up = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_fb):
            self.loss = self.forward_backward(batch)
        with torch.cuda.graph(g_up):
            self.update()
        self.graphs = (g_fb, g_up)
        self.grads_zeroed = True  # (nothing ran during capture: the bucket is still the zeroed one)


class Inference:
    """Config 5's step: the model forward on a resident batch (trainer.test's path without the
    MAE, trainer.py:52-58), captured in one HIP graph; ``step`` returns the energies' sum."""

    def __init__(self, model):
        self.model = model
        self.graph = None
        self.out = None

    def _fwd(self, batch):
        was = self.model.training  # eval for the forward (trainer.py:54), the caller's mode restored
        self.model.eval()
        try:
            with torch.no_grad():
                return self.model(batch).sum()
        finally:
            self.model.train(was)

    def step(self, batch):
        if self.graph is None:
            return self._fwd(batch)
        self.graph.replay()
        return self.out

    def capture(self, batch, warm=2):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warm):
                self._fwd(batch)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = self._fwd(batch)
