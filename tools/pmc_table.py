"""Summarise a tools/pmc_gemm.sh (or pmc_*.sh) output directory: mean counter value per dispatch for every kernel
(short name), derived ratios (VALU / MFMA, MFMA busy, bytes), and the kernel-trace average durations.

    python tools/pmc_table.py gpurun_out/pmc_upfwd
"""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def short(n):
    return n.split("(")[0][:90]


def main():
    d = Path(sys.argv[1])
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(d.glob("p*/**/*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in sorted(d.glob("trace/**/*kernel_stats.csv")):
        print("kernel trace:", f.relative_to(d))
        for r in csv.DictReader(open(f)):
            print(f"   {float(r['AverageNs']) / 1e3:10.1f} us x {r['Calls']:>4}  {short(r['Name'])}")
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(k)
        for c, v in sorted(m.items()):
            print(f"   {c:28s} {v:16.5g}")
        if m.get("SQ_INSTS_MFMA"):
            print(f"   {'(VALU-MFMA)/MFMA':28s} {(m.get('SQ_INSTS_VALU', 0) - m['SQ_INSTS_MFMA']) / m['SQ_INSTS_MFMA']:16.3f}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    print(f"   {c + ' / WAVE_CYCLES':28s} {m[c] / wc:16.3f}")
            if m.get("GRBM_GUI_ACTIVE"):
                # SQ_WAVE_CYCLES is in quad-cycles summed over waves; GRBM_GUI_ACTIVE sums 8 XCDs
                print(f"   {'waves per SIMD (avg)':28s} {wc * 4 / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):16.3f}")
        if m.get("SQ_INSTS_MFMA") and m.get("SQ_INSTS_LDS"):
            print(f"   {'LDS insts / MFMA':28s} {m['SQ_INSTS_LDS'] / m['SQ_INSTS_MFMA']:16.3f}")
        if m.get("SQ_LDS_IDX_ACTIVE") and m.get("GRBM_GUI_ACTIVE"):
            print(f"   {'LDS busy / CU-cycle':28s} {m['SQ_LDS_IDX_ACTIVE'] / (m['GRBM_GUI_ACTIVE'] / 8 * 256):16.3f}")
        if m.get("SQ_BUSY_CYCLES") and m.get("SQ_VALU_MFMA_BUSY_CYCLES") and m.get("GRBM_GUI_ACTIVE"):
            # GRBM_GUI_ACTIVE sums the 8 XCDs; MFMA busy cycles sum 256 CUs x 4 SIMDs
            cyc = m["GRBM_GUI_ACTIVE"] / 8
            print(f"   {'MFMA busy / SIMD-cycle':28s} {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):16.3f}")
        if "FETCH_SIZE" in m:
            print(f"   {'fetch GB (x2 gfx950)':28s} {m['FETCH_SIZE'] * 2 * 1024 / 1e9:16.4f}")
        if "WRITE_SIZE" in m:
            print(f"   {'write GB':28s} {m['WRITE_SIZE'] * 1024 / 1e9:16.4f}")


if __name__ == "__main__":
    main()
