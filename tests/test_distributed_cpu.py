"""The bench's multi-GPU logic on CPU: world_size-2 gloo processes.

bench.py shards DIB-R views contiguously across ranks (weak scaling), all-gathers the
per-shard losses (its only collective) and reports whole-job throughput from the max
over ranks of the timed region.  The HIP step itself needs a GPU; everything around it
is exercised here with the same helper functions, over gloo on 127.0.0.1.
"""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import bench
        per_rank = 4
        views = bench.views_for_rank(rank, world, per_rank)
        all_views = [None] * world
        dist.all_gather_object(all_views, views)
        # a per-shard "loss" that depends on the shard's views
        loss = torch.tensor(sum(math.cos(v) * (k + 1) for k, v in enumerate(views)), dtype=torch.float32)
        gathered = bench.gather_losses(loss, world)
        # ranks report different elapsed times; the job time is the max
        elapsed = bench.max_over_ranks(1.0 + 0.25 * rank, torch.device('cpu'), world)
        q.put((rank, all_views, gathered.tolist(), elapsed))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_bench_sharding_gather_and_timing(world):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    per_rank = 4
    views0 = res[0][1]
    flat = [v for vs in views0 for v in vs]
    # shards are disjoint, contiguous, and cover the job's views exactly once
    expect = [2 * math.pi * i / (per_rank * world) for i in range(per_rank * world)]
    assert flat == pytest.approx(expect)
    for rank, views, gathered, elapsed in res:
        assert views == views0
        # every rank sees every shard's loss, in rank order
        want = [sum(math.cos(v) * (k + 1) for k, v in enumerate(views0[r])) for r in range(world)]
        assert gathered == pytest.approx(want, rel=1e-6)
        assert elapsed == pytest.approx(1.0 + 0.25 * (world - 1))


def test_single_rank_is_identity():
    import bench
    assert bench.views_for_rank(0, 1, 4) == pytest.approx([0, math.pi / 2, math.pi, 3 * math.pi / 2])
    assert bench.max_over_ranks(2.5, torch.device('cpu'), 1) == 2.5
