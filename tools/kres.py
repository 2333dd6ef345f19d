"""Per-kernel register / spill / LDS summary of one HIP source (dev tool).

    python tools/kres.py s3od_amd/csrc/gemm_ops.hip [regex]
"""
import re
import subprocess
import sys

FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics", "-mllvm", "-amdgpu-mfma-vgpr-form=1"]


def main():
    src = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    extra = ["-fno-slp-vectorize"] if "attention" in src else []
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-c", src, "-o", "/tmp/kres.o",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    cur, rows = None, []
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?)(?: \[-Rpass.*)?$", line)
        if not m:
            continue
        s = m.group(1)
        if s.startswith("Function Name:"):
            cur = {"name": s.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in s:
            k, v = s.split(":", 1)
            cur[k.strip()] = v.strip()
    for d in rows:
        if pat and not pat.search(d["name"]):
            continue
        print(f"V{d.get('VGPRs', '?'):>4} A{d.get('AGPRs', '?'):>4} S{d.get('SGPRs', '?'):>4} "
              f"spillV {d.get('VGPRs Spill', '?'):>3} occ {d.get('Occupancy [waves/SIMD]', '?')} {d['name'][:150]}")
    if r.returncode:
        print(r.stderr[-3000:])


if __name__ == "__main__":
    main()
