"""Summarise tools/pmc_probe.sh output: mean counter value per kernel (short name)."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1])
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(d.glob("p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:60]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.4g}")
