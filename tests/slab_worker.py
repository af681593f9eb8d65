"""Worker of tests/test_gpu_slab.py (every rank on cuda:0 of a one-GPU box,
gloo with halo planes staged through host memory).

Modes:
  slab_worker.py OUT D              (torchrun) RPN on a 64x64xD volume, unsharded
                                    on every rank, then depth-slab sharded
                                    (m3d.parallel.SlabRPN); per-rank comparison
                                    to OUT/rank<r>.json.
  slab_worker.py ref OUT S D        (one process) the unsharded SxSxD step:
                                    P2..P6, logits, deltas, proposals, loss and
                                    the flat gradient saved as .npy under OUT.
  slab_worker.py cmp OUT S D REF    (torchrun) the sharded step compared with
                                    the saved unsharded one (memory-mapped).
  slab_worker.py nccl OUT D         (torchrun, 1 rank, RCCL) the slab step with
                                    the overlapped all-reduce forced on.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def setup(S, D, pre_nms, post_nms, n_train):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, synthetic_rpn_targets, synthetic_volume
    cfg = synthetic_rpn_config(S, depth=D, PRE_NMS_LIMIT=pre_nms, POST_NMS_ROIS_TRAINING=post_nms)
    model = RPN(cfg, device=dev, seed=3)
    image = synthetic_volume(S, D, seed=0).to(dev)
    match, bbox = synthetic_rpn_targets(model.anchors.shape[1], n_train, seed=2)
    return dev, model, image, match, bbox


def full_step(model, image, match, bbox, dev):
    from m3d.model import RPNTargets
    model.store.zero_grad()
    full = model.forward(image, proposals=True)
    lc, lb = model.losses(full, RPNTargets(match, bbox, dev))
    (lc * 1.0 + lb * 1.5).backward()
    model.rpn.finish_backward()
    return full, float((lc * 1.0 + lb * 1.5).detach()), model.store.grad_flat.detach().clone()


def slab_step(model, image, match, bbox, D):
    from m3d import slab
    from m3d.parallel import SlabRPN
    sg = slab.SlabGroup(D)
    srpn = SlabRPN(model, sg, match, bbox)
    r = srpn.train_step(srpn.slice(image), proposals=True, apply=False)
    return sg, srpn, r


def mode_inline(out_dir, D):
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev, model, image, match, bbox = setup(64, D, 3000, 400, 512)
    full, loss_full, g_full = full_step(model, image, match, bbox, dev)
    sg, srpn, r = slab_step(model, image, match, bbox, D)
    g = model.store.grad_flat.detach()
    gi = srpn.local_index
    out = r["outputs"]
    res = {
        "rank": rank, "world": world, "z0": sg.z0, "z1": sg.z1,
        "logits_bitexact": bool(torch.equal(out["rpn_class_logits"], full["rpn_class_logits"][:, gi])),
        "bbox_bitexact": bool(torch.equal(out["rpn_bbox"], full["rpn_bbox"][:, gi])),
        "p2_bitexact": bool(torch.equal(out["feature_maps"][0], full["feature_maps"][0][:, :, :, sg.z0:sg.z1])),
        "rois_bitexact": bool(torch.equal(r["rpn_rois"], full["rpn_rois"])),
        "loss_full": loss_full, "loss_slab": float(r["loss"]),
        "grad_rel_err": float((g - g_full).abs().max() / g_full.abs().max()),
        "grad_norm_rel": float((g - g_full).norm() / g_full.norm()),
    }
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


def mode_ref(out_dir, S, D):
    dev, model, image, match, bbox = setup(S, D, 15000, 6000, 1536)
    full, loss, g = full_step(model, image, match, bbox, dev)
    torch.cuda.synchronize()
    for i, p in enumerate(full["feature_maps"]):
        np.save(os.path.join(out_dir, f"p{i + 2}.npy"), p.detach().cpu().numpy())
    for k in ("rpn_class_logits", "rpn_bbox", "rpn_rois"):
        np.save(os.path.join(out_dir, f"{k}.npy"), full[k].detach().cpu().numpy())
    np.save(os.path.join(out_dir, "grad.npy"), g.cpu().numpy())
    with open(os.path.join(out_dir, "ref.json"), "w") as f:
        json.dump({"loss": loss, "peak_gb": torch.cuda.max_memory_allocated() / 1e9}, f)
    print(f"ref {S}x{S}x{D}: loss {loss:.6f}, peak {torch.cuda.max_memory_allocated() / 1e9:.1f} GB", flush=True)


def mode_cmp(out_dir, S, D, ref_dir):
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev, model, image, match, bbox = setup(S, D, 15000, 6000, 1536)
    sg, srpn, r = slab_step(model, image, match, bbox, D)
    torch.cuda.synchronize()
    out = r["outputs"]
    ld = lambda k: np.load(os.path.join(ref_dir, f"{k}.npy"), mmap_mode="r")  # noqa: E731
    gi = srpn.local_index.cpu().numpy()
    res = {"rank": rank, "world": world, "z0": sg.z0, "z1": sg.z1}
    for i, p in enumerate(out["feature_maps"]):
        res[f"p{i + 2}_bitexact"] = bool(np.array_equal(p.detach().cpu().numpy(), ld(f"p{i + 2}")[:, :, :, sg.z0:sg.z1]))
    res["logits_bitexact"] = bool(np.array_equal(out["rpn_class_logits"].detach().cpu().numpy(),
                                                 ld("rpn_class_logits")[:, gi]))
    res["bbox_bitexact"] = bool(np.array_equal(out["rpn_bbox"].detach().cpu().numpy(), ld("rpn_bbox")[:, gi]))
    res["rois_bitexact"] = bool(np.array_equal(r["rpn_rois"].cpu().numpy(), ld("rpn_rois")))
    g = model.store.grad_flat.detach().cpu().numpy().astype(np.float64)
    gref = np.asarray(ld("grad"), np.float64)
    res["grad_rel_err"] = float(np.abs(g - gref).max() / np.abs(gref).max())
    res["grad_norm_rel"] = float(np.linalg.norm(g - gref) / np.linalg.norm(gref))
    res["loss_slab"] = float(r["loss"])
    res["loss_full"] = json.load(open(os.path.join(ref_dir, "ref.json")))["loss"]
    res["peak_gb"] = torch.cuda.max_memory_allocated() / 1e9
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def mode_nccl(out_dir, D):
    """One rank on RCCL ("nccl"; RCCL refuses two ranks on one GPU): the slab
    step with the overlapped SUM all-reduce forced on (force_hook) and the
    slab ProposalLayer on its side stream, against the plain step."""
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    dev, model, image, match, bbox = setup(64, D, 3000, 400, 512)
    full, loss_full, g_full = full_step(model, image, match, bbox, dev)
    from m3d import slab
    from m3d.parallel import SlabRPN
    sg = slab.SlabGroup(D)
    srpn = SlabRPN(model, sg, match, bbox)
    r = srpn.train_step(srpn.slice(image), proposals=True, apply=False, force_hook=True)
    torch.cuda.synchronize()
    g = model.store.grad_flat.detach()
    res = {"backend": dist.get_backend(), "world": dist.get_world_size(),
           "hook_used": getattr(srpn, "_hook", None) is not None,
           "rois_bitexact": bool(torch.equal(r["rpn_rois"], full["rpn_rois"])),
           "loss_full": loss_full, "loss_slab": float(r["loss"]),
           "grad_rel_err": float((g - g_full).abs().max() / g_full.abs().max())}
    with open(os.path.join(out_dir, "rank0.json"), "w") as f:
        json.dump(res, f)
    print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    a = sys.argv[1:]
    if a[0] == "nccl":
        mode_nccl(a[1], int(a[2]))
    elif a[0] == "ref":
        mode_ref(a[1], int(a[2]), int(a[3]))
    elif a[0] == "cmp":
        mode_cmp(a[1], int(a[2]), int(a[3]), a[4])
    else:
        mode_inline(a[0], int(a[1]))
