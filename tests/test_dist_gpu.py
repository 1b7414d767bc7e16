"""Config 4's path through the PRODUCT (BASELINE.json: batch 1024 molecule-sharded over 8 GPUs,
RCCL gradient all-reduce), rehearsed with two ranks on the one GPU of the test box.

Each rank is a fresh spawned process (nothing is exec'd from a GPU-initialised process) running
``x2gnn.xgnn_poly`` through ``x2gnn.train.Trainer`` on its shard of one global batch:
``dist.shard_by_triplets`` balances the shards by triplet count, so they hold UNEQUAL molecule
counts (``dist.collate_shard``: the embedding's per-batch renorm / scale_grad_by_freq counts are
taken over the global batch, as in the single-device step); the backward sums weight gradients straight into the flat ``GradBucket`` (grad sinks,
deferred slab sums, the one flat T-layout weight-gradient launch); ``reduce()`` weights each
rank's bucket by local/global molecule count and SUM-all-reduces it together with the shard's
loss.  The ranks use gloo (one GPU cannot host two RCCL ranks); the collective's arithmetic is
the same SUM.  The result must equal a single-process product gradient over the concatenated
global batch (2e-5 of the largest gradient; the row sums run in a different split), and the
captured HIP-graph step must reproduce the eager one bit for bit on every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(conv_layers=4, sbf_dim=7, rbf_dim=6, in_channels=128, heads=16, embedding_size=128)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _global_molecules():
    from x2gnn.synth import synthetic_molecules

    # mixed sizes (S5A ~4.4k triplets, S160 ~1.5k) so the triplet-balanced shards are unequal in count
    return synthetic_molecules(3, "S5A", seed=31) + synthetic_molecules(11, "S160", seed=32)


def _model(dev):
    import x2gnn

    torch.manual_seed(0)
    return x2gnn.xgnn_poly(device="cuda", **CFG).to(dev)


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from x2gnn.dist import collate_shard, shard_by_triplets
    from x2gnn.train import Trainer

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        mols = _global_molecules()
        mine = shard_by_triplets([m["triplet_num"] for m in mols], world)[rank]
        host, n_local, n_global = collate_shard(mols, world, rank)
        assert n_local == len(mine) and n_global == len(mols)
        batch = host.to(dev)
        # the exchange as 3 asynchronous collectives over contiguous bucket ranges (reverse layout order)
        tr = Trainer(_model(dev), local_count=n_local, global_count=n_global, exchange_chunks=3)
        # the captured step (what bench.py replays): capture (its 3 warm-up passes run eagerly),
        # zero, replay forward+backward, all-reduce
        tr.capture(batch)
        tr.bucket.zero()
        tr.replay_forward_backward()
        tr.reduce()
        torch.cuda.synchronize()
        graphed = tr.bucket.flat.detach().cpu().numpy().copy()
        # eager: forward + loss + backward into the bucket, then the weighted all-reduce.  (Both
        # after the same >= 4 forwards: each forward re-applies the embedding's max_norm renorm in
        # place, as torch does, and a renormalised row can be renormalised again by an ulp.)
        loss = tr.forward_backward(batch)
        local = tr.bucket.flat.clone()
        tr.reduce()
        eager = tr.bucket.flat.detach().cpu().numpy().copy()
        # the chunked exchange equals the single collective bit for bit (two ranks)
        tr.bucket.flat.copy_(local)
        tr.exchange_chunks = 1
        tr.reduce()
        torch.cuda.synchronize()
        assert np.array_equal(tr.bucket.flat.detach().cpu().numpy(), eager)
        eager_loss = float(tr.global_loss(loss))
        out_q.put((rank, [int(i) for i in mine], eager, eager_loss, graphed, tr.bucket.num_grad))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_two_rank_product_ddp_equals_single_process(cuda):
    from x2gnn import ops
    from x2gnn.data import collate
    from x2gnn.dist import GradBucket

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            r, mine, eager, eager_loss, graphed, ngrad = q.get(timeout=540)
            got[r] = (mine, eager, eager_loss, graphed, ngrad)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    sizes = [len(got[r][0]) for r in range(world)]
    assert sum(sizes) == 14 and sizes[0] != sizes[1], sizes  # unequal shards: the weighted path
    # every rank ends with the same all-reduced bucket (gradients + global loss), eager == graphed
    for r in range(world):
        np.testing.assert_array_equal(got[r][1], got[0][1])
        np.testing.assert_array_equal(got[r][3], got[r][1])
    ngrad = got[0][4]

    # single process, same weights, the whole global batch
    mols = _global_molecules()
    batch = collate(mols).to(cuda)
    model = _model(cuda)
    bucket = GradBucket(model.parameters())
    with torch.no_grad():
        for _ in range(4):  # the ranks' forwards so far (max_norm renorm state, see _worker)
            model(batch)
    bucket.zero()
    res = model(batch)
    loss = ops.smooth_l1_loss(res, batch.y)
    with ops.deferred_wgrad():
        loss.backward()
    ref = bucket.flat.detach().cpu().numpy()
    dp = got[0][1]
    scale = np.abs(ref).max()
    np.testing.assert_allclose(dp[:ngrad], ref[:ngrad], rtol=0, atol=2e-5 * scale)
    # per-parameter relative check as well (small gradients must not hide under the global scale)
    for p, off in zip(bucket.params, bucket.offsets):
        n = p.numel()
        a, b = dp[off:off + n], ref[off:off + n]
        assert np.abs(a - b).max() <= 1e-4 * np.abs(b).max() + 1e-7 * scale
    # the loss slot holds the global-batch mean loss
    loss = float(loss.detach())
    assert abs(float(dp[ngrad]) - loss) <= 1e-5 * max(1.0, abs(loss))
    assert abs(got[0][2] - loss) <= 1e-5 * max(1.0, abs(loss))


def _worker8(rank, world, port, out_q):
    """One rank of config 4: its triplet-balanced shard of the 1024-molecule global batch, the captured
    Trainer step (graph replay of forward + backward), the count-weighted SUM all-reduce."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import x2gnn
    from weights import load_seeded
    from x2gnn.dist import collate_shard, shard_by_triplets
    from x2gnn.synth import synthetic_molecules
    from x2gnn.train import Trainer

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        mols = synthetic_molecules(1024, "S160", seed=2000)
        tcount = [m["triplet_num"] for m in mols]
        mine = shard_by_triplets(tcount, world)[rank]
        host, n_local, n_global = collate_shard(mols, world, rank)
        assert n_local == len(mine) and n_global == 1024
        m = x2gnn.xgnn_poly(device="cuda", **CFG)
        load_seeded(m, 90)
        tr = Trainer(m.to(dev), local_count=n_local, global_count=n_global)
        tr.capture(host.to(dev))
        tr.bucket.zero()
        tr.replay_forward_backward()
        tr.reduce()
        torch.cuda.synchronize()
        out_q.put((rank, [int(i) for i in mine], int(sum(tcount[i] for i in mine)),
                   tr.bucket.flat.detach().cpu().numpy().copy(), tr.bucket.num_grad))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_config4_eight_ranks_1024_molecules_equals_single_process(cuda):
    """BASELINE config 4 at its own size through the product: 1024 S160 molecules sharded over 8 ranks by
    triplet count (8 spawned processes sharing the one GPU, gloo: one GPU cannot host 8 RCCL ranks; the
    collective's arithmetic is the same SUM), each replaying its captured Trainer step, then the
    count-weighted all-reduce.  Every rank ends with the same bucket, equal to a single-process B = 1024
    product step within 2e-5 of the largest gradient; the shards' sum-T imbalance (max / mean) is
    reported and bounded; and 8 molecules' energies from the B = 1024 forward match the oracle."""
    import x2gnn
    from weights import load_seeded
    from x2gnn import ops
    from x2gnn.data import collate
    from x2gnn.dist import GradBucket
    from x2gnn.synth import synthetic_molecules

    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker8, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            r, mine, tsum, bucket, ngrad = q.get(timeout=840)
            got[r] = (mine, tsum, bucket, ngrad)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    shards = [got[r][0] for r in range(world)]
    assert sorted(i for s in shards for i in s) == list(range(1024))
    tsums = np.array([got[r][1] for r in range(world)], dtype=np.float64)
    imbalance = float(tsums.max() / tsums.mean())
    print(f"config 4 shards: molecules {[len(s) for s in shards]}, sum-T {tsums.astype(int).tolist()}, "
          f"max/mean {imbalance:.5f}")
    assert imbalance < 1.01
    for r in range(world):
        np.testing.assert_array_equal(got[r][2], got[0][2])
    ngrad = got[0][3]

    mols = synthetic_molecules(1024, "S160", seed=2000)
    batch = collate(mols).to(cuda)
    model = x2gnn.xgnn_poly(device="cuda", **CFG)
    load_seeded(model, 90)
    model = model.to(cuda)
    bucket = GradBucket(model.parameters())
    with torch.no_grad():
        for _ in range(3):  # the ranks' warm-up forwards (max_norm renorm state)
            model(batch)
    bucket.zero()
    res = model(batch)
    loss = ops.smooth_l1_loss(res, batch.y)
    with ops.deferred_wgrad():
        loss.backward()
    ref = bucket.flat.detach().cpu().numpy()
    dp = got[0][2]
    scale = np.abs(ref[:ngrad]).max()
    np.testing.assert_allclose(dp[:ngrad], ref[:ngrad], rtol=0, atol=2e-5 * scale)
    for p, off in zip(bucket.params, bucket.offsets):
        n = p.numel()
        a, b = dp[off:off + n], ref[off:off + n]
        assert np.abs(a - b).max() <= 1e-4 * np.abs(b).max() + 1e-7 * scale
    # a sample of the molecules against the oracle (the same weights, the same renorm state)
    from oracle import ref_cpu

    sample = [0, 137, 255, 401, 512, 700, 888, 1023]
    orc = ref_cpu.XGNN(**CFG)
    load_seeded(orc, 90)
    with torch.no_grad():
        orc.emb_block.embedding.weight.copy_(model.emb_block.embedding.weight.detach().cpu())
        ref_e = ref_cpu.run_batch(orc, collate([mols[i] for i in sample])).numpy()
    got_e = res.detach().cpu().numpy()[sample]
    err = np.abs(got_e - ref_e) / np.maximum(np.abs(ref_e), 1e-3 * np.abs(ref_e).max())
    assert err.max() < 1e-4, err
