"""One rank of tests/test_gpu_ddp.py::test_gloo_world2_native_backward (not collected by pytest).

Two ranks share the one GPU over a gloo group on CUDA tensors (RCCL refuses two ranks on one device).
Each rank builds the same f32-strict model twice: `ref` (no data parallelism) computes every rank's
micro-batch gradients locally; `m` runs with GradSync, so the native backward's bucket hooks all-reduce
the flat gradient while the backward is still running.  Rank r checks
  (1) one synced micro-batch on data (r, 0)            == mean_r g(r, 0)
  (2) no_sync micro-batch (r, 0) + synced (r, 1)       == mean_r [g(r, 0) + g(r, 1)]
and writes the per-check errors as JSON."""
import json
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, port, out = int(sys.argv[1]), sys.argv[2], sys.argv[3]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from s3od_amd.ddp import GradSync
    from s3od_amd.loss import LossModule, FOCAL_IOU
    from s3od_amd.model import DPTSegmentation
    dev = torch.device("cuda", 0)
    crit = LossModule(FOCAL_IOU, full_mask_lambda=0.1, decay_rate=0.2)

    def data(r, k):
        g = torch.Generator(device=dev).manual_seed(100 * r + k)
        x = torch.randn(2, 3, 128, 128, device=dev, generator=g)
        masks = (torch.rand(2, 128, 128, device=dev, generator=g) > 0.5).float()
        return x, masks

    def backward(model, r, k):
        x, masks = data(r, k)
        loss, _ = crit(model(x), {"masks": masks}, 0)
        loss.backward()
        torch.cuda.synchronize()

    def flat(model):
        return model._flat["buf"].detach().clone()

    ref = DPTSegmentation(compute_dtype="f32").to(dev).train()
    ref._rope_rescale = 1.0
    g = {}
    for r in range(2):
        for k in range(2):
            ref.zero_grad(set_to_none=False)
            backward(ref, r, k)
            g[r, k] = flat(ref)
    layout = ref._flat["layout"]
    del ref
    e1 = (g[0, 0] + g[1, 0]) / 2
    e2 = (g[0, 0] + g[0, 1] + g[1, 0] + g[1, 1]) / 2

    m = DPTSegmentation(compute_dtype="f32").to(dev).train()
    m._rope_rescale = 1.0
    sync = GradSync(m)
    m.zero_grad(set_to_none=False)
    backward(m, rank, 0)
    got1 = flat(m)
    issued = len(sync.works) == 0 and sync.stream is not None      # collectives were issued and joined
    m.zero_grad(set_to_none=False)
    with sync.no_sync():
        backward(m, rank, 0)
    local = flat(m)
    backward(m, rank, 1)
    got2 = flat(m)

    def errs(got, exp):
        tot = float((got - exp).norm()) / float(exp.norm())
        per = []
        for n, off, numel, _ in layout:
            if "resConfUnit" in n and (n.endswith("conv1.bias") or n.endswith("conv2.bias")):
                continue      # feeds a train-mode BN: the true gradient is 0, every run holds rounding noise
            a, b = got[off:off + numel], exp[off:off + numel]
            per.append((float((a - b).norm()) / max(float(b.norm()), 1e-30), n))
        return tot, max(per)

    res = {"rank": rank, "issued": issued,
           "synced": errs(got1, e1), "accumulated": errs(got2, e2),
           "no_sync_local": errs(local, g[rank, 0]),
           "ranks_differ": float((g[0, 0] - g[1, 0]).norm() / g[0, 0].norm())}
    json.dump(res, open(out, "w"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
