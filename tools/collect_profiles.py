"""Copy the judged rocprofv3 evidence of a round from gpurun_out/prof_<tag> into profiles/.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim), profiles/<tag>_summary.md
(per-step breakdown) and profiles/<tag>_pmc.json (FETCH_SIZE / WRITE_SIZE per launch of the
roofline kernel, corrected per MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB and reads half
the bytes of a wide coalesced stream on gfx950 -> x2; WRITE_SIZE exact)."""
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
tag = sys.argv[1]
kre = sys.argv[2] if len(sys.argv) > 2 else "attn_fwd_kernel"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 4      # 1 warm-up + 3 timed steps traced
src = ROOT / "gpurun_out" / f"prof_{tag}"
dst = ROOT / "profiles"
dst.mkdir(exist_ok=True)
shutil.copy(src / "trace" / "run_kernel_stats.csv", dst / f"{tag}_kernel_stats.csv")
rows = list(csv.DictReader(open(src / "trace" / "run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
lines = [f"# rocprofv3 kernel stats, round tag {tag}", "",
         f"Command: `rocprofv3 --kernel-trace --stats -- python bench.py --steps 3 --warmup 1` (bf16, bs 16, 1024², training step)",
         f"Total kernel time {tot / 1e6:.1f} ms over {steps} steps = {tot / 1e6 / steps:.1f} ms/step.", "",
         "| ms/step | % | calls | avg us | kernel |", "|---:|---:|---:|---:|---|"]
for r in rows[:40]:
    lines.append(f"| {float(r['TotalDurationNs']) / 1e6 / steps:.2f} | {float(r['Percentage']):.2f} | {r['Calls']} | "
                 f"{float(r['AverageNs']) / 1e3:.1f} | `{r['Name'][:110]}` |")
pmc = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = src / f"pmc_{c}" / "run_counter_collection.csv"
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if r["Counter_Name"] == c and kre in r["Kernel_Name"]]
    pmc[c] = sum(vals) / len(vals)
    pmc[c + "_launches"] = len(vals)
fetch_b = pmc["FETCH_SIZE"] * 1024 * 2
write_b = pmc["WRITE_SIZE"] * 1024
pmc.update(kernel=kre, fetch_bytes_corrected=fetch_b, write_bytes=write_b, traffic_bytes_per_launch=fetch_b + write_b,
           correction="FETCH_SIZE[KiB]*1024*2 (gfx950 half-count of wide streaming reads) + WRITE_SIZE[KiB]*1024")
avg = [r for r in rows if kre in r["Name"]]
if avg:
    pmc["trace_avg_ns"] = float(avg[0]["AverageNs"])
json.dump(pmc, open(dst / f"{tag}_pmc.json", "w"), indent=1)
lines += ["", f"PMC (separate passes, kernel `{kre}`): FETCH_SIZE {pmc['FETCH_SIZE']:.0f} KiB, WRITE_SIZE "
          f"{pmc['WRITE_SIZE']:.0f} KiB per launch -> traffic {(fetch_b + write_b) / 1e9:.3f} GB per launch (corrected)."]
(dst / f"{tag}_summary.md").write_text("\n".join(lines) + "\n")
print("\n".join(lines[:12]))
print(json.dumps(pmc, indent=1))
