"""Worker of tests/test_gpu_slab.py (launched by torch.distributed.run, gloo,
every rank on cuda:0 of a one-GPU box; halo planes staged through host memory).

Runs the RPN on a 64x64xD volume twice: unsharded (reference, on this rank)
and depth-slab sharded over the ranks (m3d.parallel.SlabRPN), then writes
per-rank comparisons to OUT_DIR/rank<r>.json."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def grads_of(model, out, targets):
    model.store.zero_grad()
    lc, lb = model.losses(out, targets)
    total = lc * 1.0 + lb * 1.5
    return total


def main():
    out_dir, D = sys.argv[1], int(sys.argv[2])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from m3d import slab
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume
    from m3d.parallel import SlabRPN

    cfg = synthetic_rpn_config(64, depth=D, PRE_NMS_LIMIT=3000, POST_NMS_ROIS_TRAINING=400)
    model = RPN(cfg, device=dev, seed=3)
    image = synthetic_volume(64, D, seed=0).to(dev)
    A = model.anchors.shape[1]
    match, bbox = synthetic_rpn_targets(A, 512, seed=2)

    # unsharded reference on this rank
    model.store.zero_grad()
    full = model.forward(image, proposals=True)
    lc, lb = model.losses(full, RPNTargets(match, bbox, dev))
    (lc * 1.0 + lb * 1.5).backward()
    model.rpn.finish_backward()
    g_full = model.store.grad_flat.detach().clone()
    loss_full = float(lc * 1.0 + lb * 1.5)

    # depth-slab sharded
    sg = slab.SlabGroup(D)
    srpn = SlabRPN(model, sg, match, bbox)
    model.store.zero_grad()
    out = srpn.forward(srpn.slice(image), proposals=True)
    lcs, lbs = model.losses(out, srpn.targets)
    tot = lcs * 1.0 + lbs * 1.5
    with slab.active(sg):
        tot.backward()
    model.rpn.finish_backward()
    sg.all_reduce_sum_(model.store.grad_flat)
    parts = torch.stack([tot.detach()])
    sg.all_reduce_sum_(parts)
    g = model.store.grad_flat.detach()
    gi = srpn.local_index
    res = {
        "rank": rank, "world": world, "z0": sg.z0, "z1": sg.z1,
        "logits_bitexact": bool(torch.equal(out["rpn_class_logits"], full["rpn_class_logits"][:, gi])),
        "bbox_bitexact": bool(torch.equal(out["rpn_bbox"], full["rpn_bbox"][:, gi])),
        "p2_bitexact": bool(torch.equal(out["feature_maps"][0],
                                        full["feature_maps"][0][:, :, :, sg.z0:sg.z1])),
        "rois_bitexact": bool(torch.equal(out["rpn_rois"], full["rpn_rois"])),
        "loss_full": loss_full, "loss_slab": float(parts[0]),
        "grad_rel_err": float((g - g_full).abs().max() / g_full.abs().max()),
        "grad_norm_rel": float((g - g_full).norm() / g_full.norm()),
    }
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
