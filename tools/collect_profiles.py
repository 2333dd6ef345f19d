"""Copy the judged rocprofv3 evidence of a round from gpurun_out/prof_<tag> (tools/profile_round.sh) into
profiles/.

Writes
  profiles/<tag>_kernel_stats.csv      rocprofv3 --stats of the training bench (verbatim)
  profiles/<tag>_summary.md            per-step kernel table + the roofline entry's PMC traffic
  profiles/<tag>_pmc.json              FETCH_SIZE / WRITE_SIZE per call of the roofline ENTRY (bench.py reads
                                       it: "entry" names the C-ABI function, its kernels are summed)
  profiles/<tag>_c5_kernel_stats.csv   rocprofv3 --stats of the 2048^2 bs=4 inference bench (configs[4])
  profiles/<tag>_c5_summary.md         per-kernel time + corrected HBM bytes + achieved GB/s for C5
  profiles/<tag>_bench_train.json / <tag>_bench_c5.json   the bench lines printed under the profiler

Counter correction per MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB and counts half the bytes of a wide
coalesced stream on gfx950 -> x2; WRITE_SIZE in KiB, exact.

    python tools/collect_profiles.py r02 [kernel-regex] [entry] [train-steps-traced]
"""
import csv
import json
import re
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
tag = sys.argv[1]
kre = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"attn_(bwd|delta)")
entry = sys.argv[3] if len(sys.argv) > 3 else "s3od_attn_bwd_qkv"
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 4       # 1 warm-up + 3 timed steps traced
src = ROOT / "gpurun_out" / f"prof_{tag}"
dst = ROOT / "profiles"
dst.mkdir(exist_ok=True)


def find(sub, name):
    hits = sorted((src / sub).rglob(name))
    if not hits:
        raise SystemExit(f"missing {src / sub}/**/{name}")
    return hits[0]


def stats(sub):
    f = find(sub, "run_kernel_stats.csv")
    return f, list(csv.DictReader(open(f)))


def counters(sub, c):
    """{kernel name: [value per dispatch]} of counter c."""
    out = defaultdict(list)
    for r in csv.DictReader(open(find(sub, "run_counter_collection.csv"))):
        if r["Counter_Name"] == c:
            out[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return out


def corrected(fetch_kib, write_kib):
    return fetch_kib * 1024 * 2, write_kib * 1024


# ---- training step: stats + roofline entry PMC ----
f, rows = stats("trace_train")
shutil.copy(f, dst / f"{tag}_kernel_stats.csv")
tot = sum(float(r["TotalDurationNs"]) for r in rows)
lines = [f"# rocprofv3 kernel stats, round tag {tag}", "",
         "Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline "
         "--no-infer --no-breakdown` (configs[2]: bf16, bs 16, 1024², training step)",
         f"Total kernel time {tot / 1e6:.1f} ms over {steps} steps = {tot / 1e6 / steps:.1f} ms/step.",
         "The backward's weight gradients run on a side stream beside the data-gradient chain (encoder since r04a, "
         "decoder since r04b), so kernels of the two streams overlap: each duration includes the CU sharing, and the "
         "sum exceeds the step's wall time (the bench line's ms_per_step).", "",
         "| ms/step | % | calls | avg us | kernel |", "|---:|---:|---:|---:|---|"]
for r in rows[:45]:
    lines.append(f"| {float(r['TotalDurationNs']) / 1e6 / steps:.2f} | {float(r['Percentage']):.2f} | {r['Calls']} | "
                 f"{float(r['AverageNs']) / 1e3:.1f} | `{r['Name'][:110]}` |")
fe, wr = counters("pmc_train_FETCH_SIZE", "FETCH_SIZE"), counters("pmc_train_WRITE_SIZE", "WRITE_SIZE")
per_kernel = {}
for k in sorted(set(fe) | set(wr)):
    if not kre.search(k):
        continue
    fb, wb = corrected(sum(fe[k]) / max(1, len(fe[k])), sum(wr[k]) / max(1, len(wr[k])))
    avg = [float(r["AverageNs"]) for r in rows if r["Name"] == k]
    per_kernel[k] = {"launches": len(fe[k]), "fetch_bytes_corrected": fb, "write_bytes": wb,
                     "trace_avg_ns": avg[0] if avg else None}
traffic = sum(v["fetch_bytes_corrected"] + v["write_bytes"] for v in per_kernel.values())
pmc = {"entry": entry, "kernel_regex": kre.pattern, "kernels": per_kernel, "traffic_bytes_per_launch": traffic,
       "trace_avg_ns_per_call": sum(v["trace_avg_ns"] or 0 for v in per_kernel.values()),
       "correction": "FETCH_SIZE[KiB]*1024*2 (gfx950 half-count of wide streaming reads) + WRITE_SIZE[KiB]*1024; "
                     "per call of the entry = sum over its kernels of the per-dispatch mean"}
json.dump(pmc, open(dst / f"{tag}_pmc.json", "w"), indent=1)
lines += ["", f"PMC (separate --pmc passes, kernels matching `{kre.pattern}` = one `{entry}` call):"]
for k, v in per_kernel.items():
    lines.append(f"- `{k[:90]}`: {v['launches']} dispatches, fetch {v['fetch_bytes_corrected'] / 1e9:.3f} GB + write "
                 f"{v['write_bytes'] / 1e9:.3f} GB per dispatch (corrected), avg {(v['trace_avg_ns'] or 0) / 1e3:.1f} us")
lines.append(f"- traffic per `{entry}` call: {traffic / 1e9:.3f} GB")
(dst / f"{tag}_summary.md").write_text("\n".join(lines) + "\n")

# ---- the single-stream training pass (S3OD_BWD_SIDE=0): kernel durations without the side stream's CU sharing ----
ss = src / "trace_train_ss"
if ss.exists():
    fs, rs = stats("trace_train_ss")
    shutil.copy(fs, dst / f"{tag}_ss_kernel_stats.csv")
    tots = sum(float(r["TotalDurationNs"]) for r in rs)
    ls = [f"# rocprofv3 kernel stats, SINGLE-STREAM pass, round tag {tag}", "",
          "Pass: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer "
          "--no-breakdown --single-stream` (configs[2]; the whole backward on one stream, S3OD_BWD_SIDE=0, so no two "
          "kernels share the CUs and each duration is the kernel's own).  The timed bench line runs the weight "
          "gradients on a side stream; its roofline.single_stream object is this pass's counterpart (HIP events).",
          f"Total kernel time {tots / 1e6:.1f} ms over {steps} steps = {tots / 1e6 / steps:.1f} ms/step.", "",
          "| ms/step | % | calls | avg us | kernel |", "|---:|---:|---:|---:|---|"]
    for r in rs[:45]:
        ls.append(f"| {float(r['TotalDurationNs']) / 1e6 / steps:.2f} | {float(r['Percentage']):.2f} | {r['Calls']} | "
                  f"{float(r['AverageNs']) / 1e3:.1f} | `{r['Name'][:110]}` |")
    ent = [r for r in rs if kre.search(r["Name"])]
    if ent:
        ls += ["", f"Kernels of one `{entry}` call (regex `{kre.pattern}`): " +
               ", ".join(f"`{r['Name'][:60]}` {float(r['AverageNs']) / 1e3:.1f} us" for r in ent) +
               f"; sum {sum(float(r['AverageNs']) for r in ent) / 1e3:.1f} us per call."]
    (dst / f"{tag}_ss_summary.md").write_text("\n".join(ls) + "\n")
    if (src / "bench_train_ss.json").exists():
        shutil.copy(src / "bench_train_ss.json", dst / f"{tag}_bench_train_ss.json")

# ---- C5 inference: stats + every kernel's HBM bytes ----
f5, rows5 = stats("trace_c5")
shutil.copy(f5, dst / f"{tag}_c5_kernel_stats.csv")
fe5, wr5 = counters("pmc_c5_FETCH_SIZE", "FETCH_SIZE"), counters("pmc_c5_WRITE_SIZE", "WRITE_SIZE")
tot5 = sum(float(r["TotalDurationNs"]) for r in rows5)
l5 = [f"# C5 (2048², bs 4, eval forward) kernel time and HBM traffic, round tag {tag}", "",
      "Trace: `rocprofv3 --kernel-trace --stats -- python3 bench.py --mode infer --batch 4 --size 2048 --steps 3 "
      "--warmup 1`; counters from separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes (1 warm-up + 1 step).",
      f"Total kernel time {tot5 / 1e6:.1f} ms over 4 forwards = {tot5 / 4e6:.1f} ms/forward.", "",
      "| ms/fwd | % | calls | avg us | HBM GB/dispatch (corr.) | GB/s | kernel |", "|---:|---:|---:|---:|---:|---:|---|"]
for r in rows5[:40]:
    k = r["Name"]
    gb = gbs = ""
    if k in fe5 and k in wr5:
        fb, wb = corrected(sum(fe5[k]) / len(fe5[k]), sum(wr5[k]) / len(wr5[k]))
        gb = f"{(fb + wb) / 1e9:.3f}"
        gbs = f"{(fb + wb) / float(r['AverageNs']):.0f}"
    l5.append(f"| {float(r['TotalDurationNs']) / 4e6:.2f} | {float(r['Percentage']):.2f} | {r['Calls']} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {gb} | {gbs} | `{k[:100]}` |")
(dst / f"{tag}_c5_summary.md").write_text("\n".join(l5) + "\n")
for n in ("bench_train.json", "bench_c5.json"):
    if (src / n).exists():
        shutil.copy(src / n, dst / f"{tag}_{n}")
print("\n".join(lines[-(len(per_kernel) + 2):]))
print("\n".join(l5[:16]))
