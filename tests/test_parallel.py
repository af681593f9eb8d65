"""Multi-process (gloo, world_size 2, CPU) tests of the RCCL data-parallel path
(m3d/parallel.py): bucketed flat-gradient all-reduce and rank-0 timing reduce."""
import os
import sys
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, q):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "3d-mask-r-cnn_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = fn(rank, world)
        q.put((rank, r.numpy().copy() if torch.is_tensor(r) else r))   # no shared-memory tensors
    finally:
        dist.destroy_process_group()


def run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return out


def _allreduce(rank, world):
    from m3d.parallel import allreduce_mean_
    g = torch.arange(10_000, dtype=torch.float32) * (rank + 1)
    allreduce_mean_(g, world, bucket=1024)       # 10 buckets, last one ragged
    return g


def test_bucketed_allreduce_mean():
    out = run(_allreduce)
    want = torch.arange(10_000, dtype=torch.float32) * 1.5
    for r in out.values():
        torch.testing.assert_close(torch.from_numpy(r), want)


def _max_time(rank, world):
    t = torch.tensor([1.0 + rank], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t)


def test_step_time_is_max_over_ranks():
    assert set(run(_max_time).values()) == {2.0}
