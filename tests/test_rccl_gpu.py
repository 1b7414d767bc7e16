"""The RCCL (torch.distributed backend "nccl") path on the one-GPU box: a spawned single-rank process
initialises the process group the way bench.py does for N > 1 (``init_process_group("nccl",
device_id=...)``), runs a SUM all-reduce of a GradBucket's flat buffer — whole and as the asynchronous
parameter-aligned chunks of ``allreduce_mean(chunks=k)`` issued on the process group's stream — a
barrier and the MAX all-reduce of the bench's timing, then tears the group down.  One rank cannot test
the ring's arithmetic (tests/test_dist*.py do, with gloo); this checks that the RCCL calls the 8-GPU
run makes execute on this image and leave the buffers as a one-rank sum must (unchanged, bit for bit).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch.distributed as dist

    from x2gnn.dist import GradBucket

    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        torch.cuda.set_device(0)
        model = torch.nn.Sequential(torch.nn.Linear(128, 128), torch.nn.SiLU(), torch.nn.Linear(128, 1)).cuda()
        bucket = GradBucket(model.parameters(), extra=1)
        g = torch.Generator(device="cuda").manual_seed(3)
        bucket.flat.copy_(torch.randn(bucket.flat.shape, device="cuda", generator=g))
        ref = bucket.flat.clone()
        dist.all_reduce(bucket.flat, op=dist.ReduceOp.SUM)
        whole = torch.equal(bucket.flat, ref)
        works = [dist.all_reduce(bucket.flat[lo:hi], op=dist.ReduceOp.SUM, async_op=True)
                 for lo, hi in bucket.chunk_bounds(3)]
        for w in works:
            w.wait()
        chunked = torch.equal(bucket.flat, ref)
        dist.barrier()
        t = torch.tensor([1.25], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        torch.cuda.synchronize()
        out_q.put((whole, chunked, float(t.item()), dist.get_backend()))
    except Exception as e:  # reported to the parent, which fails the test with it
        out_q.put(repr(e))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_single_rank_allreduce_paths(cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    try:
        res = q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert not isinstance(res, str), res
    whole, chunked, tmax, backend = res
    assert backend == "nccl" and whole and chunked and tmax == 1.25
    assert p.exitcode == 0
