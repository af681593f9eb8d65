"""Depth-slab sharded RPN on the GPU (m3d.parallel.SlabRPN), 2 and 3 ranks
sharing the box's one GPU over gloo: the sharded forward (feature maps, RPN
logits / deltas, merged proposals) is bit-identical to the single-volume
forward, the loss equal and the SUM-all-reduced gradient equal up to fp32
summation order (1e-4 of the gradient scale, north-star tolerance)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,D", [(2, 16), (3, 16)])
def test_slab_rpn_matches_single_volume(cuda, tmp_path, world, D):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "tests", "slab_worker.py"), str(tmp_path), str(D)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(world)]
    for x in res:
        assert x["p2_bitexact"] and x["logits_bitexact"] and x["bbox_bitexact"], x
        assert x["rois_bitexact"], x
        assert abs(x["loss_slab"] - x["loss_full"]) <= 1e-5 * abs(x["loss_full"]), x
        assert x["grad_rel_err"] < 1e-4, x
