"""The multi-GPU sharding logic (ndnet.distributed) at world size 2 over gloo on
the CPU: contiguous disjoint shards, max-over-ranks timing and the rank-order
gather of per-rank outputs.  The per-rank "work" is the CPU
oracle on each rank's shard of clouds -- standing in for the GPU path here,
since the product has no CPU fallback -- and the gathered result must equal
the single-process run over the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_rows(cloud_ids, n, k):
    import oracle as O
    from ndnet.synthetic import uniform_cloud
    rows = []
    for i in cloud_ids:
        r = O.run(uniform_cloud(n, seed=i).astype(np.float64), k)
        rows.append(np.concatenate([np.asarray(r.out_pc), np.asarray(r.out_cov)], axis=1))
    return torch.from_numpy(np.stack(rows).astype(np.float32))


def _worker(rank, world, port, total, n, k, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (os.path.join(repo, "ndt-net_amd"), os.path.join(repo, "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from ndnet import distributed as D
    assert D.init("gloo")
    r, lr, w = D.world_from_env()
    assert (r, lr, w) == (rank, rank, world)
    start, count = D.shard(total, world, rank)
    out = _oracle_rows(range(start, start + count), n, k)
    D.barrier()
    t = D.max_over_ranks(float(rank + 1))
    s = D.sum_over_ranks(float(count))
    full = D.gather_shards(out)
    if rank == 0:
        q.put((t, s, full.numpy()))
    torch.distributed.destroy_process_group()


def test_shard_partition():
    from ndnet.distributed import shard
    for total in (1, 7, 16, 128):
        for world in (1, 2, 3, 8):
            got = [shard(total, world, r) for r in range(world)]
            assert sum(c for _, c in got) == total
            pos = 0
            for s, c in got:
                assert s == pos
                pos += c
            assert max(c for _, c in got) - min(c for _, c in got) <= 1
    with pytest.raises(ValueError):
        shard(4, 2, 2)


def test_gloo_world2_matches_single_process():
    total, n, k = 5, 2048, 64  # odd total: shards of 3 and 2 clouds
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, n, k, q)) for r in range(2)]
    for p in procs:
        p.start()
    t, s, full = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 2.0 and s == float(total)
    ref = _oracle_rows(range(total), n, k).numpy()
    assert full.shape == ref.shape
    np.testing.assert_array_equal(full, ref)
