"""world_size-2 gloo tests of the batch-sharded multi-GPU path.

On CPU the per-rank compute op is the CPU oracle (no GPU in this
container); the partition, per-rank independence and the root gather are the
code the GPU path runs unchanged (bench.py uses the same shard_range).  The
``gpu``-marked variant runs the same two ranks with the HIP library doing
each rank's shard (both ranks on cuda:0 of a one-GPU box; gloo carries the
gather) and checks the gathered result against the oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fhe_gpu.shard import gather_to_root, run_sharded, shard_range

P27 = 132120577


def test_shard_range_partitions():
    for total in (0, 1, 7, 64, 65536, 65537):
        for world in (1, 2, 3, 8):
            rs = [shard_range(total, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, n, q, out_path, use_gpu=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle

    x = oracle.splitmix_fill(3, q, total * n).reshape(total, n)
    y = oracle.splitmix_fill(4, q, total * n).reshape(total, n)
    if use_gpu:
        import fhe_gpu

        dev = rank % torch.cuda.device_count()
        torch.cuda.set_device(dev)
        ring = fhe_gpu.PolynomialRing(n, q, device=dev)

        def op(a, b):
            da = torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(f"cuda:{dev}")
            db = torch.from_numpy(np.ascontiguousarray(b).view(np.int64)).to(f"cuda:{dev}")
            return ring.multiply(da, db).cpu().numpy().view(np.uint64)
    else:
        t = oracle.NTT(n, q)

        def op(a, b):
            return t.polymul(a, b)
    local = run_sharded(op, [x, y], rank, world)
    lt = torch.from_numpy(local.view(np.int64).copy())
    full = gather_to_root(lt, total, rank, world)
    # barrier + max-over-ranks timing, as bench.py does
    dist.barrier()
    v = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    assert v.item() == world
    if rank == 0:
        np.save(out_path, full.numpy().view(np.uint64))
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [8, 9])
def test_gloo_sharded_polymul_gather(tmp_path, total):
    world, n, q = 2, 256, 7681
    out = str(tmp_path / "full.npy")
    mp.spawn(_worker, args=(world, _free_port(), total, n, q, out), nprocs=world, join=True)
    import oracle

    t = oracle.NTT(n, q)
    x = oracle.splitmix_fill(3, q, total * n).reshape(total, n)
    y = oracle.splitmix_fill(4, q, total * n).reshape(total, n)
    assert (np.load(out) == t.polymul(x, y)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("n,q,total", [(4096, P27, 9), (16384, 4611686018326724609, 4)])
def test_gloo_sharded_polymul_gather_on_gpu(tmp_path, n, q, total):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 2
    out = str(tmp_path / "full.npy")
    mp.spawn(_worker, args=(world, _free_port(), total, n, q, out, True), nprocs=world, join=True)
    import oracle

    t = oracle.NTT(n, q)
    x = oracle.splitmix_fill(3, q, total * n).reshape(total, n)
    y = oracle.splitmix_fill(4, q, total * n).reshape(total, n)
    assert (np.load(out) == t.polymul(x, y)).all()
