"""Time the per-step weight repack (engine.prepare(force=True): the s3od_repack_multi launches) on the GPU box (dev tool).

    python tools/repack_time.py
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd.model import DPTSegmentation  # noqa: E402


def main():
    model = DPTSegmentation(compute_dtype="bf16").cuda()
    eng = model.engine()
    for _ in range(3):
        eng.prepare(force=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        eng.prepare(force=True)
    e1.record()
    torch.cuda.synchronize()
    print(f"prepare (repack of every packed weight): {e0.elapsed_time(e1) / n * 1e3:.1f} us per call", flush=True)


if __name__ == "__main__":
    main()
