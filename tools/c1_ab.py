"""C1 (BackgroundRemoval.remove_background on the fixture, end to end) timed per library build (dev tool, GPU box):
each build in its own subprocess (S3OD_HIP_LIB), alternating, 30 calls after 3 warm-up calls.

    python tools/c1_ab.py before_lib/libs3od_hip.so s3od_amd/libs3od_hip.so
"""
import os
import subprocess
import sys
from pathlib import Path

R = Path(__file__).resolve().parent.parent
CHILD = r'''
import sys, time, torch
sys.path.insert(0, sys.argv[1])
from PIL import Image
from s3od_amd.predictor import BackgroundRemoval
img = Image.open(sys.argv[1] + "/tests/fixture/image.jpg").convert("RGB")
br = BackgroundRemoval("synthetic", device="cuda")
for _ in range(3):
    br.remove_background(img)
torch.cuda.synchronize()
ts = []
for _ in range(30):
    t0 = time.perf_counter(); br.remove_background(img); ts.append(time.perf_counter() - t0)
ts.sort()
print(f"median {ts[15] * 1e3:.2f} ms  min {ts[0] * 1e3:.2f} ms  max {ts[-1] * 1e3:.2f} ms")
'''

if __name__ == "__main__":
    for rnd in range(2):
        for lib in sys.argv[1:]:
            env = dict(os.environ, S3OD_HIP_LIB=str((R / lib).resolve()))
            out = subprocess.run([sys.executable, "-c", CHILD, str(R)], env=env, capture_output=True, text=True, timeout=300)
            print(f"round {rnd} {lib}: {out.stdout.strip()} {out.stderr.strip()[-300:] if out.returncode else ''}", flush=True)
