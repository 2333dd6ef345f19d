"""Same-process A/B of the training step (configs[2]: bs 16, 1024^2, bf16, fwd + loss + bwd + AdamW) under two
settings of one per-call environment knob, alternating rounds (dev tool).

    python tools/ab_step.py S3OD_BWD_SIDE 0 1 [rounds] [steps]
    AB_MODE=infer AB_BATCH=8 AB_SIZE=1024 python tools/ab_step.py S3OD_POOL_PRE 0 1   # eval forward (C2 / C5)
"""
import os
os.environ.setdefault("S3OD_AB", "1")   # knobs toggled per call (csrc/common.hpp S3OD_KNOB)
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    knob, a, b = sys.argv[1:4]
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    from bench import synthetic_batch
    from s3od_amd.model import DPTSegmentation
    from s3od_amd.loss import LossModule, FOCAL_IOU
    from s3od_amd.optim import FusedAdamW, reference_param_groups
    dev = torch.device("cuda", 0)
    infer = os.environ.get("AB_MODE") == "infer"
    m = DPTSegmentation(compute_dtype="bf16").to(dev)
    m.eval() if infer else m.train()
    crit = LossModule(FOCAL_IOU, full_mask_lambda=0.1, decay_rate=0.2)
    opt = FusedAdamW(reference_param_groups(m, 1e-5), weight_decay=0.05)
    x, masks = synthetic_batch(int(os.environ.get("AB_BATCH", 8 if infer else 16)), int(os.environ.get("AB_SIZE", 1024)),
                               1000, dev)

    def step():
        if infer:
            with torch.no_grad():
                return m(x)["pred_iou"].sum()
        out = m(x)
        loss, _ = crit(out, {"images": x, "masks": masks}, 0)
        loss.backward()
        opt.step()
        m.zero_grad(set_to_none=False)
        return loss

    for v in (a, b):
        os.environ[knob] = v
        step(); step()
    res = {a: [], b: []}
    for r in range(rounds):
        for v in (a, b):
            os.environ[knob] = v
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                loss = step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps * 1e3
            res[v].append(dt)
            print(f"round {r} {knob}={v}: {dt:8.2f} ms/step  loss {float(loss):.5f}", flush=True)
    for v in (a, b):
        print(f"{knob}={v}: min {min(res[v]):.2f} median {sorted(res[v])[len(res[v]) // 2]:.2f} ms/step")


if __name__ == "__main__":
    main()
