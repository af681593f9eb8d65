"""Depth-slab sharded RPN on the GPU (m3d.parallel.SlabRPN), 2, 3 and 8 ranks
sharing the box's one GPU over gloo: the sharded forward (feature maps, RPN
logits / deltas, merged proposals) is bit-identical to the single-volume
forward, the loss equal and the SUM-all-reduced gradient equal up to fp32
summation order (1e-4 of the gradient scale, north-star tolerance)."""
import json
import os
import subprocess
import sys

import pytest

from launch import torchrun

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world,D", [(2, 16), (3, 16)])
def test_slab_rpn_matches_single_volume(cuda, tmp_path, world, D):
    r = torchrun(world, [os.path.join(ROOT, "tests", "slab_worker.py"), str(tmp_path), str(D)], ROOT, 300,
                 tmp_path / "torchrun.log")
    assert r.returncode == 0, r.log[-3000:]
    res = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(world)]
    for x in res:
        assert x["p2_bitexact"] and x["logits_bitexact"] and x["bbox_bitexact"], x
        assert x["rois_bitexact"], x
        assert abs(x["loss_slab"] - x["loss_full"]) <= 1e-5 * abs(x["loss_full"]), x
        assert x["grad_rel_err"] < 1e-4, x


def test_slab_rpn_256_eight_ranks(cuda, tmp_path):
    """BASELINE configs[4] geometry: ONE 256^3 volume in 8 depth slabs of 32
    planes (8 ranks sharing the box's GPU over gloo), against the unsharded
    256^3 step run beforehand in its own process and saved: P2..P6, RPN
    logits / deltas and the merged proposals (15000 -> 6000) bit-exact, the
    loss to 1e-5 and the SUM-all-reduced (overlapped) gradient to 1e-4 of its scale."""
    ref = tmp_path / "ref"
    ref.mkdir()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "slab_worker.py"), "ref", str(ref), "256", "256"],
                       cwd=ROOT, timeout=600)          # output streams into the (-s) log
    assert r.returncode == 0, r.returncode
    world = 8
    r = torchrun(world, [os.path.join(ROOT, "tests", "slab_worker.py"), "cmp", str(tmp_path), "256", "256",
                         str(ref)], ROOT, 900, tmp_path / "torchrun.log")
    assert r.returncode == 0, r.log[-3000:]
    res = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(world)]
    for x in res:
        print(x)
        assert x["z1"] - x["z0"] == 32, x
        for k in ("p2", "p3", "p4", "p5", "p6", "logits", "bbox", "rois"):
            assert x[f"{k}_bitexact"], (k, x)
        assert abs(x["loss_slab"] - x["loss_full"]) <= 1e-5 * abs(x["loss_full"]), x
        assert x["grad_rel_err"] < 1e-4, x


def test_slab_rpn_rccl_one_rank(cuda, tmp_path):
    """SlabRPN on the RCCL device path (backend "nccl", one rank: RCCL refuses
    two ranks on one GPU): the overlapped SUM all-reduce forced on
    (force_hook), the slab ProposalLayer on its side stream -- proposals
    bit-exact and the gradient equal to the plain step's up to the fp32
    atomics' order (1e-5 of its scale)."""
    r = torchrun(1, [os.path.join(ROOT, "tests", "slab_worker.py"), "nccl", str(tmp_path), "16"], ROOT, 300,
                 tmp_path / "torchrun.log", env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.log[-3000:]
    x = json.load(open(tmp_path / "rank0.json"))
    assert x["backend"] == "nccl" and x["hook_used"] and x["rois_bitexact"], x
    assert abs(x["loss_slab"] - x["loss_full"]) <= 1e-5 * abs(x["loss_full"]), x
    assert x["grad_rel_err"] < 1e-5, x
