"""Molecule-sharded data parallelism on CPU (gloo, world size 2): the N>1 path of bench.py.

Each rank runs the oracle model (same seeded weights) forward+backward on its own shard of
molecules, the flat gradient bucket is all-reduced (``GradBucket.allreduce_mean``), and the
result must equal the single-process gradient of the whole batch (loss = mean over molecules:
for equal shards the mean of the shard means, for unequal shards the count-weighted sum).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from x2gnn.data import collate
from x2gnn.dist import GradBucket, shard_by_triplets
from x2gnn.synth import synthetic_molecules

CFG = dict(conv_layers=1, sbf_dim=7, rbf_dim=6, in_channels=32, heads=4, embedding_size=32)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model():
    from oracle import ref_cpu

    torch.manual_seed(0)
    return ref_cpu.XGNN(**CFG)


def _grads(model, mols):
    from oracle import ref_cpu

    b = collate(mols)
    res = ref_cpu.run_batch(model, b)
    loss = torch.nn.functional.smooth_l1_loss(res, b.y)
    loss.backward()
    return loss.detach()


def _chunk_worker(rank, world, port, out_q):
    """One rank's gradient bucket all-reduced once whole and once as 3 asynchronous chunks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mols = synthetic_molecules(4, "S160", seed=7)
        model = _model()
        bucket = GradBucket(model.parameters(), extra=1)
        bucket.zero()
        loss = _grads(model, [mols[i] for i in range(rank, 4, world)])
        bucket.extra_view.copy_(loss.reshape(1))
        local = bucket.flat.clone()
        bucket.allreduce_mean(local_count=2, global_count=4)
        whole = bucket.flat.clone()
        bucket.flat.copy_(local)
        bucket.allreduce_mean(local_count=2, global_count=4, chunks=3)
        out_q.put((rank, whole.numpy(), bucket.flat.clone().numpy(), bucket.chunk_bounds(3), bucket.flat.numel()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_chunked_allreduce_equals_single_collective():
    """GradBucket.allreduce_mean(chunks=3): three asynchronous collectives over contiguous ranges cut at
    parameter boundaries (reverse layout order, the loss slot in the first) give the single
    collective's bucket bit for bit with two ranks."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chunk_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, whole, chunked, bounds, n = q.get(timeout=240)
        got[r] = (whole, chunked, bounds, n)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole, chunked, bounds, n = got[0]
    assert len(bounds) == 3 and bounds[0][1] == n and bounds[-1][0] == 0
    assert all(bounds[i][0] == bounds[i + 1][1] for i in range(len(bounds) - 1))  # contiguous, reversed
    np.testing.assert_array_equal(chunked, whole)
    np.testing.assert_array_equal(got[1][1], whole)


def _worker(rank, world, port, shards, out_q, weighted=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mols = synthetic_molecules(8, "S160", seed=5)
        model = _model()
        bucket = GradBucket(model.parameters())
        bucket.zero()
        loss = _grads(model, [mols[i] for i in shards[rank]])
        n_local = len(shards[rank])
        n_global = sum(len(s) for s in shards)
        if weighted:
            bucket.allreduce_mean(local_count=n_local, global_count=n_global)
            t = loss.clone() * n_local / n_global
            dist.all_reduce(t)
            out_q.put((rank, bucket.flat.clone().numpy(), float(t)))
        else:
            bucket.allreduce_mean()
            t = loss.clone()
            dist.all_reduce(t)
            out_q.put((rank, bucket.flat.clone().numpy(), float(t) / world))
    finally:
        dist.destroy_process_group()


def test_shard_by_triplets_partitions_and_balances():
    mols = synthetic_molecules(16, "S5A", seed=2)
    counts = [m["triplet_num"] for m in mols]
    shards = shard_by_triplets(counts, 4)
    allidx = np.sort(np.concatenate(shards))
    assert (allidx == np.arange(16)).all()
    loads = [sum(counts[i] for i in s) for s in shards]
    assert max(loads) - min(loads) <= max(counts)  # LPT bound


def test_gradbucket_views_and_zero():
    model = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.Linear(4, 2))
    bucket = GradBucket(model.parameters())
    model(torch.randn(5, 3)).sum().backward()
    assert bucket.flat.abs().sum() > 0
    for p in model.parameters():  # grads are views of the flat buffer
        assert p.grad.data_ptr() >= bucket.flat.data_ptr()
    bucket.zero()
    assert all(float(p.grad.abs().sum()) == 0 for p in model.parameters())


@pytest.mark.timeout(300)
@pytest.mark.parametrize("weighted", [False, True])
def test_two_rank_allreduce_equals_full_batch_gradient(weighted):
    """Equal shards with the plain mean; unequal shards (5 + 3 molecules, as shard_by_triplets
    produces) with the count-weighted all-reduce."""
    world = 2
    mols = synthetic_molecules(8, "S160", seed=5)
    if weighted:
        shards = [np.array([0, 2, 3, 5, 6]), np.array([1, 4, 7])]
    else:
        shards = [np.arange(0, 8, 2), np.arange(1, 8, 2)]  # equal sizes -> mean of means == mean
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shards, q, weighted)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict()
    for _ in range(world):
        r, flat, loss = q.get(timeout=240)
        got[r] = (flat, loss)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # both ranks hold identical, averaged gradients
    np.testing.assert_array_equal(got[0][0], got[1][0])

    model = _model()
    bucket = GradBucket(model.parameters())
    bucket.zero()
    loss = _grads(model, mols)
    ref = bucket.flat.numpy()
    scale = np.abs(ref).max()
    np.testing.assert_allclose(got[0][0], ref, rtol=0, atol=2e-5 * scale)
    assert abs(got[0][1] - float(loss)) <= 1e-5 * max(1.0, abs(float(loss)))


def _aid_worker(rank, world, port, idx, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from conftest import GOLDEN
        from oracle import ref_cpu
        from x2gnn.dist import collate_shard
        from x2gnn.synth import molecules_from_geometry_file

        mols = molecules_from_geometry_file(os.path.join(GOLDEN, "aid_geom.npz"), indices=idx)
        batch, n_local, n_global = collate_shard(mols, world, rank)
        model = _model()
        bucket = GradBucket(model.parameters())
        bucket.zero()
        res = ref_cpu.run_batch(model, batch)
        loss = torch.nn.functional.smooth_l1_loss(res, batch.y)
        loss.backward()
        local = bucket.flat.clone()
        bucket.allreduce_mean(local_count=n_local, global_count=n_global)
        whole = bucket.flat.clone()
        bucket.flat.copy_(local)
        bucket.allreduce_mean(local_count=n_local, global_count=n_global, chunks=4)
        # four ranks: the ring's per-element summation order may follow the chunk position
        np.testing.assert_allclose(bucket.flat.numpy(), whole.numpy(), rtol=1e-6, atol=1e-7 * float(whole.abs().max()))
        t = loss.detach().clone() * n_local / n_global
        dist.all_reduce(t)
        load = int(batch._meta["triplets"].sum())
        out_q.put((rank, whole.numpy(), float(t), n_local, load,
                   batch._store["_x2g_count_z"].numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
def test_four_rank_aid_mix_sharding_and_allreduce():
    """Config 4's sharding on an AID-sized mix (66-135-atom molecules, T from ~20k to ~120k each)
    over 4 gloo ranks: shard_by_triplets partitions the batch with unequal molecule counts and a
    load imbalance within the LPT bound (one molecule's T), collate_shard hands every rank the
    global batch's atomic numbers, and the count-weighted all-reduce of the shard gradients equals
    the single-process gradient of the whole batch (the embedding row excepted: the oracle
    evaluates scale_grad_by_freq per shard, the product's global-count rule is GPU-tested in
    tests/test_dist_gpu.py)."""
    from conftest import GOLDEN
    from oracle import ref_cpu
    from x2gnn.synth import molecules_from_geometry_file

    world = 4
    idx = [1, 3, 12, 0, 5, 16, 13, 2, 9, 17]  # 135, 79, 66, ... atoms: a ragged mix
    mols = molecules_from_geometry_file(os.path.join(GOLDEN, "aid_geom.npz"), indices=idx)
    counts = [m["triplet_num"] for m in mols]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_aid_worker, args=(r, world, port, idx, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, flat, loss, n_local, load, count_z = q.get(timeout=360)
        got[r] = (flat, loss, n_local, load, count_z)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sum(g[2] for g in got.values()) == len(mols) and len({g[2] for g in got.values()}) > 1
    loads = [g[3] for g in got.values()]
    assert sum(loads) == sum(counts) and max(loads) - min(loads) <= max(counts)
    all_z = np.concatenate([m["x"] for m in mols])
    for r in range(world):
        np.testing.assert_array_equal(got[r][4], all_z)
        np.testing.assert_array_equal(got[r][0], got[0][0])
    model = _model()
    bucket = GradBucket(model.parameters())
    bucket.zero()
    b = collate(mols)
    res = ref_cpu.run_batch(model, b)
    loss = torch.nn.functional.smooth_l1_loss(res, b.y)
    loss.backward()
    ref = bucket.flat.numpy().copy()
    emb = model.emb_block.embedding.weight
    e0 = (emb.grad.data_ptr() - bucket.flat.data_ptr()) // 4
    mask = np.ones_like(ref, dtype=bool)
    mask[e0:e0 + emb.numel()] = False
    scale = np.abs(ref).max()
    np.testing.assert_allclose(got[0][0][mask], ref[mask], rtol=0, atol=2e-5 * scale)
    lv = float(loss.detach())
    assert abs(got[0][1] - lv) <= 1e-5 * max(1.0, abs(lv))
