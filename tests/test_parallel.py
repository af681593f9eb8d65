"""Multi-process (gloo, world_size 2, CPU) tests of the RCCL data-parallel path
(m3d/parallel.py): bucketed flat-gradient all-reduce and rank-0 timing reduce."""
import os
import sys
import socket

import numpy as np
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


def _overlap(rank, world):
    """OverlappedAllReduce on a ParamStore-shaped flat buffer: layers report
    their gradients final in reverse order (as the backward does); buckets
    must launch tail-first during the 'backward' and the unregistered
    parameter's bucket only at finish; the result is the mean."""
    from m3d.params import ParamStore
    from m3d.parallel import OverlappedAllReduce
    st = ParamStore()
    sizes = [3000, 500, 7000, 2000, 4100, 900]          # padded to 1024-float chunks
    for i, n in enumerate(sizes):
        st.add(f"l{i}/kernel:0", (n,), "zeros", True)
    st.add("head/kernel:0", (1500,), "zeros", True)      # never registered (folded later)
    st.finalize("cpu")
    for i, p in enumerate(st.params):
        p.grad.copy_(torch.arange(p.numel, dtype=torch.float32) * (rank + 1) + i)
    h = OverlappedAllReduce(st, world, bucket=4096)
    for i in range(len(sizes)):
        h.use(f"l{i}", [st.params[i].grad])
    h.use("l2", [st.params[2].grad])                      # a shared layer used twice
    launched_before_finish = []
    for i in reversed(range(len(sizes))):
        h.done(f"l{i}")
        if i == 2:
            h.done("l2")
        launched_before_finish.append(list(h.order))
    early = list(h.order)
    h.finish()
    return {"early": early, "all": list(h.order), "nb": len(h.bounds),
            "grads": [p.grad.clone().numpy() for p in st.params]}


def test_overlapped_bucket_allreduce():
    out = run(_overlap)
    r = out[0]
    nb = r["nb"]
    # the head spans the last two buckets: they launch only at finish, every other
    # bucket during the 'backward', tail first (b3 as soon as l4 and l3 are final)
    assert sorted(r["all"]) == list(range(nb)) and nb == 6
    assert r["early"] == [3, 1, 2, 0]
    for i, g in enumerate(r["grads"]):
        n = g.size
        want = torch.arange(n, dtype=torch.float32) * 1.5 + i
        torch.testing.assert_close(torch.from_numpy(g), want)
    assert all(np.array_equal(a, b) for a, b in zip(out[0]["grads"], out[1]["grads"]))
