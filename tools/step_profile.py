"""Per-call profile of one training (or inference) step: every C-ABI call is bracketed by HIP
events on the current stream and attributed its algorithmic FLOPs, so each GEMM / conv /
attention launch shows its shape, time and TF/s (dev tool, GPU box only).

    python tools/step_profile.py [--mode train|infer] [--batch 16] [--size 1024]
"""
import argparse
import collections
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from s3od_amd import _lib  # noqa: E402
from bench import synthetic_batch  # noqa: E402


def flops(name, a):
    """Algorithmic FLOPs of one call from its scalar args (positions follow include/s3od_hip.h)."""
    if name == "s3od_linear_fwd":
        M, N, K = a[1:4]
        return 2.0 * M * N * K, f"M{M} N{N} K{K}"
    if name == "s3od_linear_dgrad":
        M, N, K = a[1:4]
        return 2.0 * M * N * K, f"M{M} N{N} K{K}"
    if name == "s3od_linear_wgrad":
        N, K, R = a[1:4]
        return 2.0 * N * K * R, f"N{N} K{K} rows{R}"
    if name == "s3od_qkv_rope_fwd":
        B, Nt, P, H = a[1:5]
        D = 64 * H
        return 2.0 * B * Nt * 3 * D * D, f"B{B} Nt{Nt} D{D}"
    if name in ("s3od_conv_fwd", "s3od_conv_dgrad", "s3od_conv_wgrad"):
        B, H, W, Cin, OH, OW, Cout, KH, KW, s, p = a[1:12]
        if name == "s3od_conv_dgrad" and s > 1 and OH > H:   # ConvT forward: Y-grid is the big one
            pass
        fl = 2.0 * B * OH * OW * Cout * Cin * KH * KW
        return fl, f"B{B} {H}x{W}x{Cin} -> {OH}x{OW}x{Cout} k{KH} s{s} p{p}"
    if name == "s3od_attn_fwd":
        B, H, N = a[6:9]
        return 4.0 * B * H * N * N * 64, f"B{B} H{H} N{N}"
    if name == "s3od_attn_bwd":
        B, H, N = a[11:14]
        return 10.0 * B * H * N * N * 64, f"B{B} H{H} N{N}"
    if name == "s3od_attn_bwd_qkv":
        B, H, N = a[15:18]
        return 10.0 * B * H * N * N * 64, f"B{B} H{H} N{N}"
    return 0.0, ""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="train")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--top", type=int, default=60)
    args = ap.parse_args()
    from s3od_amd.model import DPTSegmentation
    from s3od_amd.loss import LossModule, FOCAL_IOU
    from s3od_amd.optim import FusedAdamW, reference_param_groups
    dev = torch.device("cuda", 0)
    model = DPTSegmentation(compute_dtype="bf16").to(dev)
    x, masks = synthetic_batch(args.batch, args.size, 1, dev)
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
    else:
        model.eval()

        def step():
            with torch.no_grad():
                model(x)
    step(); step()
    torch.cuda.synchronize()
    L = _lib.lib()
    rec = []
    orig = _lib._Lib.__call__

    def timed(self, name, *a):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = orig(self, name, *a)
        e1.record()
        rec.append((name, a, e0, e1))
        return rc
    _lib._Lib.__call__ = timed
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    step()
    e1.record()
    torch.cuda.synchronize()
    _lib._Lib.__call__ = orig
    total = e0.elapsed_time(e1)
    rows = []
    for name, a, s, e in rec:
        ms = s.elapsed_time(e)
        fl, shape = flops(name, a)
        rows.append((ms, name, shape, fl))
    tot_native = sum(r[0] for r in rows)
    tot_fl = sum(r[3] for r in rows)
    print(f"step {total:.2f} ms; native calls {len(rows)} sum {tot_native:.2f} ms; algorithmic "
          f"{tot_fl / 1e12:.2f} TF -> {tot_fl / (total * 1e-3) / 1e12:.1f} TF/s over the step")
    agg = collections.OrderedDict()
    for ms, name, shape, fl in rows:
        k = (name, shape)
        c = agg.setdefault(k, [0, 0.0, 0.0])
        c[0] += 1; c[1] += ms; c[2] += fl
    print(f"{'ms':>8} {'calls':>5} {'TF/s':>7}  op  shape")
    for (name, shape), (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:args.top]:
        tf = fl / (ms * 1e-3) / 1e12 if fl else 0.0
        print(f"{ms:8.2f} {n:5d} {tf:7.1f}  {name[5:]}  {shape}")


if __name__ == "__main__":
    main()
