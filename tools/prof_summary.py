"""Summarise a rocprofv3 kernel-trace .db: python tools/prof_summary.py <db> [n_steps] [top]"""
import sqlite3
import sys

db = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), sum(end-start), avg(end-start) from kernels group by name order by 3 desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"total kernel time {tot / 1e6:.2f} ms ({tot / 1e6 / steps:.2f} ms per step over {steps:g} steps)")
print(f"{'ms/step':>9} {'%':>6} {'calls':>6} {'avg us':>9}  kernel")
for name, n, s, a in rows[:top]:
    short = name.replace("_Z12igemm_kernelI", "igemm<").split("EvT2_")[0][:140]
    print(f"{s / 1e6 / steps:9.3f} {100 * s / tot:6.2f} {n:6d} {a / 1e3:9.1f}  {short}")
