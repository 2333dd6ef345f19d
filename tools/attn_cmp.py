"""Compare two attn_sweep.py output files bit for bit (dev tool)."""
import sys
import torch
a, b = torch.load(sys.argv[1], weights_only=True), torch.load(sys.argv[2], weights_only=True)
for n in a:
    for k in ("o", "dq", "dk", "dv"):
        x, y = a[n][k].float(), b[n][k].float()
        print(n, k, "identical" if torch.equal(x, y) else f"max diff {float((x - y).abs().max()):.3e} rel {float((x - y).norm() / y.norm()):.3e}")
