"""S3OD MI355X benchmark (driver contract: one JSON line on rank 0).

Headline metric (BASELINE.json): "train images/sec (dinob 1024px bf16) at 1/2/4/8 GPU; infer masks/sec 1GPU".
Default workload = configs[2]: synth_sod train model=dinob, 1024x1024, bs=16 per GPU, bf16, forward +
focal_iou loss + backward + fused AdamW, synthetic on-device data.  --gpus N runs data-parallel over
RCCL (launched by torch.distributed.run, one rank per GPU), per-GPU batch fixed ("weak" scaling).
--mode infer measures configs[1] (bs=8 eval forward, masks/s).

`roofline`: the dominant kernel's ALGORITHMIC FLOPs per launch / its mean launch time measured with
HIP events around every launch inside the timed region.
`cpu_baseline`: the oracle (oracle/s3od_oracle.py, the reference's CPU fp32 path restated) timed on
this host's cores on a bounded sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PEAK_BF16 = 2.5e15      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32 = 157.3e12     # f32 MFMA


def synthetic_batch(B, S, seed, dev):
    g = torch.Generator(device=dev).manual_seed(seed)
    u8 = torch.randint(0, 256, (B, 3, S, S), generator=g, device=dev, dtype=torch.uint8)
    mean = torch.tensor([0.485, 0.456, 0.406], device=dev).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=dev).view(1, 3, 1, 1)
    x = ((u8.float() / 255.0) - mean) / std
    # 1-3 random filled ellipses per image
    yy = torch.arange(S, device=dev).view(1, S, 1).float()
    xx = torch.arange(S, device=dev).view(1, 1, S).float()
    masks = torch.zeros(B, S, S, device=dev)
    r = torch.rand(B, 3, 5, generator=g, device=dev)
    for k in range(3):
        cy, cx = (0.2 + 0.6 * r[:, k, 0]) * S, (0.2 + 0.6 * r[:, k, 1]) * S
        ry, rx = (0.08 + 0.22 * r[:, k, 2]) * S, (0.08 + 0.22 * r[:, k, 3]) * S
        inside = ((yy - cy.view(B, 1, 1)) / ry.view(B, 1, 1)) ** 2 + ((xx - cx.view(B, 1, 1)) / rx.view(B, 1, 1)) ** 2 <= 1
        use = (k == 0) | (r[:, k, 4] > 0.5)
        masks = torch.where(inside & use.view(B, 1, 1), torch.ones_like(masks), masks)
    return x.contiguous(), masks.contiguous()


def attn_flops(B, S):
    N = (S // 16) ** 2 + 5
    return 4.0 * B * 12 * N * N * 64           # QK^T + PV per layer launch


def cpu_baseline(S, mode, threads):
    """Oracle (reference CPU path restated in PyTorch fp32) on one image."""
    from oracle import s3od_oracle as O
    from s3od_amd.weights import synthetic_state_dict
    torch.set_num_threads(threads)
    sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(0).items()}
    x, masks = synthetic_batch(1, S, 123, "cpu")
    if mode == "train":
        params = {k: v.requires_grad_(True) for k, v in sd.items() if v.is_floating_point() and "running" not in k}

        def run():
            for p in params.values():
                p.grad = None
            out = O.forward(x, sd, train=True, rope_rescale=1.0)
            loss, *_ = O.multi_mask_loss(out, masks, 0)
            loss.backward()
    else:
        def run():
            with torch.no_grad():
                O.forward(x, sd)
    t0 = time.perf_counter()
    run()                        # warm-up (also counted into the budget)
    t1 = time.perf_counter()
    n = 1 if (t1 - t0) > 8 else 2
    t2 = time.perf_counter()
    for _ in range(n):
        run()
    dt = (time.perf_counter() - t2) / n
    return {"value": round(1.0 / dt, 4), "unit": "images/s" if mode == "train" else "masks/s", "cores": threads,
            "kind": "port", "sample": f"1 image {S}x{S}, {'fwd+focal_iou loss+bwd' if mode == 'train' else 'eval fwd'}, "
                                      f"fp32 oracle (oracle/s3od_oracle.py), {n} timed iter after 1 warm-up, {threads} threads"}


def infer_rate(model, B, S, steps, warmup, dev):
    """Eval-forward throughput (configs[1] / configs[4]): one selected mask per image -> masks/s."""
    x, _ = synthetic_batch(B, S, 7, dev)
    was_training = model.training
    model.eval()
    with torch.no_grad():
        for _ in range(warmup):
            model(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = model(x)["pred_masks"]
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    model.train(was_training)
    ok = bool(torch.isfinite(out).all().item())
    del out, x
    return {"value": round(B * steps / dt, 3), "unit": "masks/s", "ms_per_step": round(dt / steps * 1e3, 3),
            "batch": B, "image_size": S, "steps": steps, "warmup": warmup, "finite": ok}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/<tag>_pmc.json, written by tools/collect_profiles.py), or None."""
    files = sorted((ROOT / "profiles").glob("*_pmc.json"))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("kernel") == kernel:
            return {"bytes": d["traffic_bytes_per_launch"], "source": f"profiles/{f.name}"}
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=["train", "infer"], default="train")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 16 train / 8 infer)")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--dtype", choices=["bf16", "f32"], default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-infer", action="store_true", help="skip the secondary inference lines (train mode)")
    ap.add_argument("--ddp", action="store_true",
                    help="use the RCCL data-parallel path even at world size 1 (rehearsal on one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_dist = world > 1 or args.ddp
    if use_dist:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from s3od_amd.model import DPTSegmentation
    from s3od_amd.loss import LossModule, FOCAL_IOU
    from s3od_amd.optim import FusedAdamW, reference_param_groups
    from s3od_amd import _lib

    B = args.batch or (16 if args.mode == "train" else 8)
    S = args.size
    model = DPTSegmentation(compute_dtype=args.dtype).to(dev)
    sync = None
    if use_dist:
        from s3od_amd.ddp import GradSync, broadcast_parameters
        broadcast_parameters(model)
        sync = GradSync(model)
    x, masks = synthetic_batch(B, S, 1000 + rank, dev)

    if args.mode == "train":
        model.train()
        crit = LossModule(FOCAL_IOU, full_mask_lambda=0.1, decay_rate=0.2)
        opt = FusedAdamW(reference_param_groups(model, 1e-5), weight_decay=0.05)

        def step():
            out = model(x)
            loss, _ = crit(out, {"images": x, "masks": masks}, 0)
            loss.backward()
            opt.step()
            model.zero_grad(set_to_none=False)
            return loss
    else:
        model.eval()

        def step():
            with torch.no_grad():
                return model(x)["pred_masks"]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dom = "s3od_attn_fwd"
    lib = _lib.lib()
    lib.timers = {dom: []}
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        last = step()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if use_dist:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ev = lib.timers.pop(dom)
    lib.timers = {}
    kms = sum(a.elapsed_time(b) for a, b in ev) / max(len(ev), 1)
    ok = bool(torch.isfinite(last.float()).all().item())

    if rank == 0:
        total = B * world * args.steps
        value = total / el
        metric = ("train images/sec (dinob 1024px bf16) at 1/2/4/8 GPU; infer masks/sec 1GPU")
        unit = "images/s" if args.mode == "train" else "masks/s"
        peak = PEAK_BF16 if args.dtype == "bf16" else PEAK_F32
        achieved = attn_flops(B, S) / (kms * 1e-3) if kms > 0 else 0.0
        tr = pmc_traffic("attn_fwd_kernel") if (B == 16 and S == 1024 and args.dtype == "bf16") else None
        res = {
            "metric": metric, "value": round(value, 3), "unit": unit, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (seeded uint8 images, ImageNet-normalised; 1-3 ellipse masks), deterministic synthetic weights",
            "config": {"workload": ("synth_sod train model=dinob 1024px bs=16/GPU fwd+focal_iou loss+bwd+AdamW"
                                    if args.mode == "train" else "dinob inference bs=8 1024x1024 eval forward"),
                       "model": "dinob (DINOv3 ViT-B/16 + DPT + 3-mask head)", "global_batch": B * world,
                       "image_size": S, "parallelism": f"dp{world}"},
            "roofline": {"kernel": "attn_fwd_kernel (flash attention fwd, 1 launch per ViT layer)", "bound": "mfma",
                         "achieved": round(achieved / 1e12, 2), "peak": round(peak / 1e12, 1), "unit": "TFLOP/s",
                         "frac": round(achieved / peak, 4), "traffic": round(tr["bytes"]) if tr else None,
                         "traffic_unit": "bytes/launch (FETCH_SIZE*2 + WRITE_SIZE, gfx950-corrected)",
                         "traffic_source": tr["source"] if tr else None,
                         "flops_per_launch": attn_flops(B, S), "mean_launch_ms": round(kms, 4), "launches": len(ev)},
            "finite": ok,
        }
        if args.mode == "train" and world == 1 and not args.no_infer and args.dtype == "bf16":
            # the metric's second half ("infer masks/sec 1GPU"): configs[1] and configs[4]
            res["infer"] = dict(infer_rate(model, 8, 1024, 10, 3, dev),
                                config="dinob inference bs=8 1024x1024 eval forward (configs[1])")
            res["infer_2048"] = dict(infer_rate(model, 4, 2048, 4, 2, dev),
                                     config="high-res 2048x2048 eval forward bs=4 (configs[4])")
        if not args.no_cpu_baseline and world == 1:
            try:
                res["cpu_baseline"] = cpu_baseline(S, args.mode, args.cpu_threads)
            except Exception as e:  # reported, never fatal for the GPU number
                res["cpu_baseline"] = {"value": None, "error": repr(e)[:200]}
        print(json.dumps(res), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
