"""Worker of tests/test_gpu_dp.py (torch.distributed.run, gloo with every rank
on cuda:0, or RCCL ("nccl") with one rank): one data-parallel RPN step with the all-reduce after the backward and
one with buckets all-reduced during the backward (OverlappedAllReduce) from
the same initial state; writes per-rank comparisons to OUT_DIR/rank<r>.json."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out_dir = sys.argv[1]
    backend = sys.argv[2] if len(sys.argv) > 2 else "gloo"
    dist.init_process_group(backend, device_id=torch.device("cuda", 0) if backend == "nccl" else None)
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from m3d import parallel
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume

    cfg = synthetic_rpn_config(64, depth=16, PRE_NMS_LIMIT=2000, POST_NMS_ROIS_TRAINING=300)
    res = {}
    for overlap in (False, True):
        model = RPN(cfg, device=dev, seed=3)
        image = synthetic_volume(64, 16, seed=10 + rank).to(dev)
        match, bbox = synthetic_rpn_targets(model.anchors.shape[1], 256, seed=20 + rank)
        # small buckets so several launch during the backward
        if overlap:
            model._dp_hook = parallel.OverlappedAllReduce(model.store, world, bucket=1 << 20)
        r = parallel.data_parallel_train_step(model, image, RPNTargets(match, bbox, dev), world,
                                              proposals=False, overlap=overlap, force_hook=overlap)
        torch.cuda.synchronize()
        res[overlap] = (model.store.flat.detach().clone(), model.store.grad_flat.clone(), float(r["loss"]),
                        getattr(getattr(model, "_dp_hook", None), "n_early", None),
                        len(getattr(getattr(model, "_dp_hook", None), "bounds", [])))
    (p0, g0, l0, _, _), (p1, g1, l1, early, nb) = res[False], res[True]
    allg = [torch.zeros_like(g1) for _ in range(world)]
    dist.all_gather(allg, g1)
    diff = []
    for p in model.store.params:
        a, b = g0[p.offset:p.offset + p.numel], g1[p.offset:p.offset + p.numel]
        if not torch.equal(a, b):
            diff.append((p.name, float((a - b).abs().max()), float(a.abs().max())))
    # conv_wgrad_kernel accumulates with fp32 atomics: summation order (and so the
    # last bits) varies run to run, overlap or not; compare within 1e-5 per tensor
    grad_ok = all(d <= 1e-5 * m for _, d, m in diff)
    pdiff = float((p0 - p1).abs().max())
    out = {"rank": rank, "grads_close": grad_ok, "param_max_diff": pdiff,
           "diff": diff[:12], "n_diff": len(diff),
           "grads_same_on_ranks": all(bool(torch.equal(allg[0], a)) for a in allg),
           "loss": l1, "n_early": early, "n_buckets": nb}
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
