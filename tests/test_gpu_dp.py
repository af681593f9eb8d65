"""Data-parallel RPN step on the GPU with the gradient buckets all-reduced
during the backward (m3d.parallel.OverlappedAllReduce), 2 ranks sharing the
box's one GPU over gloo: averaged gradients equal those of the
all-reduce-after-backward step within 1e-5 per tensor (the weight-gradient
kernels sum with fp32 atomics, so their last bits vary run to run either way),
parameters after SGD agree, gradients are identical on every rank, and all
but the last bucket launch before the backward ends."""
import json
import os

import pytest

from launch import torchrun

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_overlapped_dp_step_matches(cuda, tmp_path):
    world = 2
    r = torchrun(world, [os.path.join(ROOT, "tests", "dp_worker.py"), str(tmp_path)], ROOT, 300,
                 tmp_path / "torchrun.log")
    assert r.returncode == 0, r.log[-3000:]
    res = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(world)]
    for x in res:
        assert x["grads_close"] and x["grads_same_on_ranks"] and x["param_max_diff"] < 1e-6, x
        assert x["n_buckets"] > 8 and x["n_early"] >= x["n_buckets"] - 2, x


def test_overlapped_dp_step_rccl_device_path(cuda, tmp_path):
    """The RCCL device path of the data-parallel step (backend "nccl", one rank:
    RCCL refuses two ranks on one GPU): bucketed async all-reduces launched from
    the autograd thread under the weight-gradient side stream, waited on by the
    compute stream before SGD -- the same gradients and parameters as the step
    without collectives."""
    r = torchrun(1, [os.path.join(ROOT, "tests", "dp_worker.py"), str(tmp_path), "nccl"], ROOT, 300,
                 tmp_path / "torchrun.log", env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.log[-3000:]
    x = json.load(open(tmp_path / "rank0.json"))
    assert x["grads_close"] and x["grads_same_on_ranks"] and x["param_max_diff"] < 1e-6, x
    assert x["n_buckets"] > 8 and x["n_early"] >= x["n_buckets"] - 2, x
