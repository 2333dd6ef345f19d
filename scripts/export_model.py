"""CLI of the reference's scripts/export_model.py:175-227 on this repo's checkpoint layer.

  python scripts/export_model.py --checkpoint best.ckpt --output s3od_checkpoint.ckpt

``--format checkpoint`` (the reference's recommended path, export_model.py:83-119) strips the
Lightning metadata to the ``{"state_dict": ...}`` file ``BackgroundRemoval`` loads
(s3od_amd.checkpoint.export_checkpoint; weights-only loading, no pickled objects).
``--format torchscript`` is out of scope: the native path is not traceable and the
reference itself marks TorchScript export legacy / device-specific.
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main(argv=None):
    ap = argparse.ArgumentParser(description="Export S3OD model for inference")
    ap.add_argument("--checkpoint", type=str, required=True, help="Path to model checkpoint (.ckpt file)")
    ap.add_argument("--output", type=str, required=True, help="Output path for exported model")
    ap.add_argument("--format", type=str, choices=["checkpoint", "torchscript"], default="checkpoint")
    ap.add_argument("--device", type=str, default="cpu", help="unused (TorchScript only in the reference)")
    ap.add_argument("--no-verify", action="store_true", help="unused (TorchScript only in the reference)")
    args = ap.parse_args(argv)
    if args.format == "torchscript":
        ap.error("TorchScript export is not supported by the MI355X build; use --format checkpoint")
    import torch
    from s3od_amd.checkpoint import export_checkpoint
    print(f"Loading checkpoint from: {args.checkpoint}")
    out = export_checkpoint(args.checkpoint, args.output)
    sd = torch.load(str(out), map_location="cpu", weights_only=True)
    size = Path(out).stat().st_size / (1024 * 1024)
    print(f"Checkpoint saved successfully! Size: {size:.2f} MB; contains {len(sd.get('state_dict', sd))} parameters")
    return 0


if __name__ == "__main__":
    sys.exit(main())
