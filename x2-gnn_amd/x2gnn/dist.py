"""Molecule-sharded data parallelism (one process per GPU, torch.distributed over RCCL/xGMI).

The reference is single-device (train_ema.py:40); the build adds exactly one strategy:
molecules are independent (triplets, LayerNorm segments, readouts and pools never cross a
molecule), so each rank runs forward+backward on its own shard and the only exchange is one
all-reduce of a flat fp32 gradient bucket (1,158,795 parameters = 4.6 MB at config.json
widths) plus the scalar loss.  Shards are balanced by triplet count, the unit of work.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_by_triplets(triplet_counts, world: int):
    """Greedy longest-processing-time assignment of molecules to ``world`` ranks by triplet
    count; returns one sorted index array per rank (molecule order kept inside a shard)."""
    counts = np.asarray(triplet_counts, dtype=np.int64)
    order = np.argsort(-counts, kind="stable")
    load = np.zeros(world, dtype=np.int64)
    owner = np.empty(len(counts), dtype=np.int64)
    for m in order:
        r = int(np.argmin(load))
        owner[m] = r
        load[r] += counts[m]
    return [np.nonzero(owner == r)[0] for r in range(world)]


def collate_shard(mols, world: int, rank: int):
    """This rank's share of one global batch: (collated local Batch, local molecule count, global
    molecule count).  The shard is ``shard_by_triplets(...)[rank]``.

    The local batch also carries the GLOBAL batch's atomic numbers (``_x2g_count_z``): the
    embedding's max_norm renorm (rows present in the batch) and scale_grad_by_freq (gradient /
    per-element count) are per-batch rules (atom_embedding.py:14), so every rank evaluates them
    over the global batch -- the same rows renormalised on every rank (parameters never diverge)
    and the same divisor as the single-device step over the whole batch."""
    from .data import collate

    shards = shard_by_triplets([m["triplet_num"] for m in mols], world)
    mine = shards[rank]
    batch = collate([mols[i] for i in mine])
    batch._store["_x2g_count_z"] = torch.cat([torch.as_tensor(m["x"], dtype=torch.int64).reshape(-1) for m in mols])
    return batch, len(mine), len(mols)


def flat_layout(params, align=4):
    """Offsets of each parameter in a flat fp32 buffer, each rounded up to ``align`` floats
    (16 bytes) so views of the buffer keep the alignment the vectorised kernels want; returns
    (offsets, total)."""
    offs, off = [], 0
    for p in params:
        offs.append(off)
        off += (p.numel() + align - 1) // align * align
    return offs, off


class GradBucket:
    """All parameters' gradients as views of ONE flat buffer, so the per-step exchange is a
    single all-reduce (ring over xGMI) with no pack/unpack copies."""

    def __init__(self, params, extra=0):
        """``extra``: trailing floats after the gradients (x2gnn.train keeps the step's loss there so
        it is all-reduced by the same collective); ``extra_view`` is that slice."""
        self.params = [p for p in params if p.requires_grad]
        self.offsets, n = flat_layout(self.params)
        self.num_grad = n
        dev = self.params[0].device
        self.flat = torch.zeros(n + int(extra), dtype=torch.float32, device=dev)  # padding stays zero
        self.extra_view = self.flat[n:]
        for p, off in zip(self.params, self.offsets):
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            # the fused dense / attention backwards may sum weight gradients straight into this
            # buffer (ops.grad_sink) instead of returning them for autograd to add
            p._x2g_grad_sink = True

    def zero(self):
        self.flat.zero_()

    def chunk_bounds(self, chunks: int):
        """``chunks`` contiguous [lo, hi) ranges of the flat buffer that cover it, cut at parameter
        boundaries into near-equal byte shares, in REVERSE layout order: the last parameters (the
        readouts and the last conv layers, whose gradients a backward finishes first) lead.  The
        trailing ``extra`` floats (the loss slot) ride with the first range issued."""
        n = self.num_grad
        chunks = max(1, min(int(chunks), len(self.params)))
        cuts = [0]
        for k in range(1, chunks):
            target = k * n / chunks
            # the parameter boundary nearest the target, strictly increasing
            best = min(self.offsets, key=lambda o: abs(o - target))
            if best > cuts[-1]:
                cuts.append(best)
        cuts.append(self.flat.numel())
        ranges = [(cuts[i], cuts[i + 1]) for i in range(len(cuts) - 1)]
        return ranges[::-1]

    def allreduce_mean(self, group=None, local_count=None, global_count=None, chunks: int = 1):
        """Turn each rank's gradient of its own mean loss into the gradient of the global-batch
        mean loss (trainer.py:41, smooth_l1 with reduction='mean').

        Without counts every rank's shard is taken to hold the same number of molecules, and the
        per-rank gradients are averaged.  With ``local_count`` (molecules on this rank) and
        ``global_count`` (molecules over all ranks, known on the host from the sharding), each
        rank's gradient is weighted by local/global before the sum, which is what unequal shards
        (e.g. ``shard_by_triplets``) need.

        ``chunks`` > 1 issues the SUM as that many asynchronous collectives over the contiguous
        ranges of ``chunk_bounds`` (reverse layout order), all in flight together on the process
        group's own stream and joined to the current stream before returning — so the optimizer that
        follows waits for all of them, and RCCL pipelines one range's ring behind another's.  Each
        element is summed over the same ranks either way; with two ranks the result is bitwise equal
        to the single collective (tests/test_dist.py), with more the ring's per-element order may
        differ by chunk position (fp32 reassociation only)."""
        multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        if local_count is not None:
            if global_count is None or global_count <= 0:
                raise ValueError("weighted all-reduce needs the global molecule count")
            self.flat.mul_(float(local_count) / float(global_count))
            if multi:
                self._sum(group, chunks)
            return
        if multi:
            # SUM then one divide: ReduceOp.AVG would save the divide under RCCL, but it is the one
            # collective option the 1-GPU rehearsal (gloo) cannot exercise before the 8-GPU run
            self._sum(group, chunks)
            self.flat.div_(dist.get_world_size(group))

    def _sum(self, group, chunks):
        if chunks <= 1:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
            return
        works = [dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM, group=group, async_op=True)
                 for lo, hi in self.chunk_bounds(chunks)]
        for w in works:
            w.wait()
