"""RCCL path on one GPU: a world-size-1 "nccl" (RCCL) process group with the collectives forced on
(S3OD_DDP_REHEARSE=1) runs the real bucketed all-reduce on the side HIP stream from inside the
native backward; the resulting gradients must equal a run without data parallelism up to the f32 atomic-order noise
(relative L2 <= 1e-4; the mean over one rank is the identity), which checks the bucket hooks, the stream/event ordering and finish()."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p


def test_rccl_grad_sync_world1(monkeypatch):
    from s3od_amd.ddp import GradSync
    from s3od_amd.loss import LossModule, FOCAL_IOU
    from s3od_amd.model import DPTSegmentation
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x = torch.randn(2, 3, 128, 128, device=dev)
    masks = (torch.rand(2, 128, 128, device=dev) > 0.5).float()
    crit = LossModule(FOCAL_IOU, full_mask_lambda=0.1, decay_rate=0.2)

    def grads(model):
        model._rope_rescale = 1.0
        out = model(x)
        loss, _ = crit(out, {"masks": masks}, 0)
        loss.backward()
        torch.cuda.synchronize()
        return {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}

    ref = grads(DPTSegmentation(compute_dtype="f32").to(dev).train())
    monkeypatch.setenv("S3OD_DDP_REHEARSE", "1")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        m = DPTSegmentation(compute_dtype="f32").to(dev).train()
        sync = GradSync(m)
        got = grads(m)
        assert sync.stream is not None, "no collective was issued"
    finally:
        dist.destroy_process_group()
    assert ref.keys() == got.keys()
    bad = []
    for n in ref:
        if "resConfUnit" in n and (n.endswith("conv1.bias") or n.endswith("conv2.bias")):
            continue     # feeds a train-mode BN: the true gradient is 0, both runs hold rounding noise
        err = float((ref[n] - got[n]).norm()) / max(float(ref[n].norm()), 1e-30)
        if err > 1e-4:
            bad.append((err, n))
    assert not bad, sorted(bad, reverse=True)[:12]
