"""GPU: the production knob path.  tests/conftest.py sets S3OD_AB=1 for the whole suite, so every other GPU test runs
the per-call getenv branch of S3OD_KNOB; production reads each knob once into a function-local static
(csrc/common.hpp).  Here a fresh subprocess WITHOUT S3OD_AB runs two routed entries -- s3od_colsum (two-pass
workspace route) and s3od_conv_wgrad on an LDS-DMA shape (3x3, 64 -> 64, whole tiles) -- and its outputs must equal
this process's."""
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parent.parent

SCRIPT = r'''
import sys, torch
sys.path.insert(0, sys.argv[2])
from s3od_amd._lib import lib, stream, BF16
g = torch.Generator(device="cuda").manual_seed(5)
a = torch.randn(8192, 256, device="cuda", generator=g).bfloat16()
out = torch.zeros(256, device="cuda")
import ctypes
nb = ctypes.c_long(0)
lib()("s3od_colsum_ws", 8192, 256, ctypes.addressof(nb))
ws = torch.empty(max(nb.value, 4) // 4, device="cuda")
lib()("s3od_colsum", BF16, a, 256, 8192, 256, out, ws, nb.value, stream())
B, H, W, C = 2, 64, 64, 64
dy = torch.randn(B, H, W, C, device="cuda", generator=g).bfloat16()
x = torch.randn(B, H, W, C, device="cuda", generator=g).bfloat16()
dw = torch.zeros(C * 9 * C, device="cuda")
wsw = torch.zeros(C * 9 * C, device="cuda")
sb = ctypes.c_long(0)
lib()("s3od_conv_wgrad_ws", BF16, B, H, W, C, H, W, C, 3, 3, 1, 1, 0, ctypes.addressof(sb))
slab = torch.empty(max(sb.value, 4) // 4, device="cuda")
lib()("s3od_conv_wgrad", BF16, B, H, W, C, H, W, C, 3, 3, 1, 1, dy, x, 0, dw, wsw, 0, slab, sb.value, stream())
torch.cuda.synchronize()
assert int((wsw != 0).sum()) == 0
torch.save({"colsum": out.cpu(), "dw": dw.cpu(), "ws_bytes": (nb.value, sb.value)}, sys.argv[1])
'''


def test_read_once_knobs_match_per_call_knobs(tmp_path):
    out = tmp_path / "once.pt"
    env = {k: v for k, v in os.environ.items() if k != "S3OD_AB"}
    subprocess.run([sys.executable, "-c", SCRIPT, str(out), str(REPO)], env=env, check=True, timeout=240)
    once = torch.load(out, weights_only=True)
    mine = tmp_path / "ab.pt"
    assert os.environ.get("S3OD_AB") == "1"
    subprocess.run([sys.executable, "-c", SCRIPT, str(mine), str(REPO)], env=dict(os.environ), check=True, timeout=240)
    ab = torch.load(mine, weights_only=True)
    assert once["ws_bytes"] == ab["ws_bytes"]
    assert torch.equal(once["colsum"], ab["colsum"])                      # two fixed-order passes: deterministic
    d = (once["dw"] - ab["dw"]).abs().max() / ab["dw"].abs().max()
    assert float(d) <= 1e-5, float(d)
    # and the route is the production one: the DMA weight gradient needs no slab
    assert once["ws_bytes"][1] == 0
