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


def _replicas(rank, world):
    """m3d.parallel.validate_replicas (bench.py's N > 1 self-check): tensors
    equal on every rank pass, one flipped bit on one rank fails exactly that
    tensor; the float loss comparison of the depth-slab check."""
    from m3d.parallel import rel_close, tensor_digest, validate_replicas
    g = torch.Generator().manual_seed(7)
    w = torch.randn(100_000, generator=g)
    rois = torch.rand((6000, 6), generator=g)
    bad = w.clone()
    if rank == world - 1:
        bad.view(torch.int32)[12345] ^= 1                 # one ulp on one rank
    ok = validate_replicas({"weights": w, "rpn_rois": rois})
    nok = validate_replicas({"weights": bad, "rpn_rois": rois})
    d1, d2 = tensor_digest(w), tensor_digest(bad)
    return {"ok": ok, "nok": nok, "digest_differs": bool(not torch.equal(d1, d2)),
            "close": rel_close(1.0, 1.0 + 5e-6, 1e-5), "far": rel_close(1.0, 1.0 + 5e-5, 1e-5)}


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float64, torch.float32, torch.int64,
                                   torch.bool])
def test_tensor_digest_is_bit_level_at_every_width(dtype):
    """tensor_digest reads each element's bytes as an integer of the element's
    width: a change in the last fraction bit of one bf16 / fp16 / fp64 element
    changes the digest (a value cast to int64 would truncate it away)."""
    from m3d.parallel import tensor_digest
    g = torch.Generator().manual_seed(3)
    w = (torch.rand(4096, generator=g) * 8).to(dtype) if dtype != torch.bool else torch.rand(4096, generator=g) > .5
    bad = w.clone()
    if dtype == torch.bool:
        bad[77] = ~bad[77]
    else:
        it = {2: torch.int16, 4: torch.int32, 8: torch.int64}[w.element_size()]
        bad.view(it)[77] ^= 1
    assert torch.equal(tensor_digest(w), tensor_digest(w.clone()))
    assert not torch.equal(tensor_digest(w), tensor_digest(bad))


@pytest.mark.parametrize("world", [2, 3])
def test_validate_replicas(world):
    out = run(_replicas, world)
    for rank, r in out.items():
        assert r["ok"] == {"ok": True, "identical": {"rpn_rois": True, "weights": True}}
        assert r["nok"] == {"ok": False, "identical": {"rpn_rois": True, "weights": False}}
        assert r["digest_differs"] == (rank == world - 1)
        assert r["close"] and not r["far"]


def test_init_from_env_timeout():
    """A gloo group from init_from_env with a 3 s timeout: rank 1 skips the
    all-reduce, rank 0's all_reduce raises within the timeout."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeout_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res[0][0] == "raised" and res[0][1] < 30, res
    assert res[1] == ("skipped", 0.0)


def _timeout_worker(rank, world, port, q):
    import time as _t
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "3d-mask-r-cnn_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      M3D_DIST_TIMEOUT="3")
    from m3d.parallel import init_from_env
    init_from_env(backend="gloo")
    if rank == 1:
        q.put((1, ("skipped", 0.0)))
        _t.sleep(8)
        return
    t0 = _t.time()
    try:
        dist.all_reduce(torch.ones(4))
        q.put((0, ("completed", _t.time() - t0)))
    except Exception:
        q.put((0, ("raised", _t.time() - t0)))
