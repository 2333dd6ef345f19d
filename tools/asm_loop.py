"""Instruction census of the largest loop of each kernel in a hipcc -S output (dev tool).

    hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S x.hip -o x.s
    python tools/asm_loop.py x.s [kernel-substring] [salu]   (salu: scalar ops in the census too)
"""
import re
import sys


def kernels(lines):
    starts = [(i, l.split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_Z\w+:", l)]
    for k, (i, name) in enumerate(starts):
        end = starts[k + 1][0] if k + 1 < len(starts) else len(lines)
        yield name, lines[i:end]


def classify(t):
    if "mfma" in t:
        return "mfma"
    if t.startswith("v_"):
        return "valu"
    if t.startswith("ds_"):
        return "ds"
    if t.startswith(("buffer_", "global_")):
        return "vmem"
    if t.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_setprio", "s_cbranch", "s_branch")):
        return t
    if t.startswith("s_"):
        return "salu"
    return t


def main():
    lines = open(sys.argv[1]).read().split("\n")
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, body in kernels(lines):
        if sub not in name:
            continue
        labels = {l.split(":")[0]: j for j, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
        best = None
        for j, l in enumerate(body):
            m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\d+_\d+)", l)
            if m and m.group(1) in labels and labels[m.group(1)] < j:
                a = labels[m.group(1)]
                span = sum("mfma" in x for x in body[a:j]) * 100000 + j - a   # the loop with the most MFMAs
                if best is None or span > best[0]:
                    best = (span, a, j)
        if best is None:
            continue
        _, a, b = best
        cnt, v = {}, {}
        for l in body[a:b + 1]:
            t = l.strip().split(" ")[0]
            if not t or t.startswith((";", ".")):
                continue
            c = classify(t)
            cnt[c] = cnt.get(c, 0) + 1
            if c == "valu" or (c == "salu" and len(sys.argv) > 3):
                v[t] = v.get(t, 0) + 1
        vg = re.search(r"\.vgpr_count:\s+(\d+)", "\n".join(body))
        print(name[:90], "| loop lines", b - a)
        print("   ", dict(sorted(cnt.items(), key=lambda x: -x[1])))
        print("    valu:", sorted(v.items(), key=lambda x: -x[1])[:24])


if __name__ == "__main__":
    main()
