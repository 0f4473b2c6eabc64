"""kaolin.distributed through RCCL on the GPU box (What's missing 1): a one-rank 'nccl'
process group on cuda:0 runs every device-tensor collective the sharded helpers use, and each
sharded result equals the unsharded op (tests/rccl_world1_worker.py, in a child process under its
own time limit so that a stuck rendezvous cannot hang the suite).  Two ranks cannot share one GPU
under RCCL; the multi-rank logic is covered by the gloo tests (test_distributed_cpu.py).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def test_sharded_ops_over_rccl_world1():
    env = dict(os.environ)
    env.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()), RANK='0', LOCAL_RANK='0', WORLD_SIZE='1')
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    r = subprocess.run([sys.executable, os.path.join(HERE, 'rccl_world1_worker.py')], env=env, capture_output=True,
                       text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res['backend'] == 'nccl' and res['world_size'] == 1
    failed = {k: v for k, v in res.items() if k not in ('backend', 'world_size', 'calls',
                                                         'collective_tensors_on_device') and v is not True}
    assert not failed, failed
    calls = res['calls']
    for op in ('all_gather', 'all_reduce', 'all_to_all_single', 'all_gather_into_tensor'):
        assert calls.get(op, 0) > 0, (op, calls)
    assert res['collective_tensors_on_device'] is True
