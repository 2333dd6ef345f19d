"""Per-step launch census of a rocprofv3 kernel trace of the training bench (steps end at adamw_kernel):
native vs PyTorch / runtime (fill, copy, elementwise) launches per step.

    python tools/trace_steps.py gpurun_out/prof_<tag>/trace_train/run_kernel_trace.csv
"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
ends = [i for i, n in enumerate(names) if n.startswith("adamw_kernel")]
prev = 0
for k, i in enumerate(ends):
    step = names[prev:i + 1]
    other = collections.Counter(n.split("<")[0].split("(")[0][:60] for n in step if n.startswith(("void at::", "__amd")))
    print(f"step {k}{' (warm-up: first-step gradient views, optimizer state)' if k == 0 else ''}: {len(step)} launches, "
          f"{len(step) - sum(other.values())} native, {sum(other.values())} PyTorch/runtime: {dict(other)}")
    prev = i + 1
