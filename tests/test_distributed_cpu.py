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


# ------------------------------------------------------------------ launcher + point sharding
import json  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize('world', [2, 3])
def test_bench_launcher_spawns_ranks_and_shards_p2m(world):
    """bench.py --gpus N (no torchrun) starts N rank processes itself; over gloo the sharded
    point_to_mesh_distance (points split, faces replicated, outputs all-gathered, face gradient
    all-reduced) equals the unsharded op on every rank."""
    r = _run_bench(['--device', 'cpu', '--gpus', str(world), '--steps', '1'])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line['n_ranks'] == world
    assert line['p2m']['parity_all_ranks'] is True
    assert line['p2m']['points_per_rank'] == -(-203 // world)


def test_bench_refuses_world_size_mismatch():
    r = _run_bench(['--gpus', '2'], env_extra={'WORLD_SIZE': '3', 'RANK': '0'})
    assert r.returncode == 2
    assert 'refusing' in r.stderr


def test_shard_bounds_cover_in_order():
    from kaolin.distributed import shard_bounds
    for n in (0, 1, 7, 100, 101):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1
