"""Per-kernel ratios from scripts/sq_passes.sh output (two rocprofv3 counter passes of one bench
command): MFMA pipe busy (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 128 SIMDs per XCD counter)),
VALU instructions per MFMA instruction, LDS bank-conflict cycles per LDS instruction, and the share of
wave cycles spent waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES), for the kernels with the most time.
    python scripts/sq_ratios.py gpurun_out/pmc_TAG [--top 20]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 20
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:90]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in sorted(glob.glob(os.path.join(d, "p*", "*kernel_trace.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:90]
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

    def m(k, c):
        v = vals[k].get(c)
        return sum(v) / len(v) if v else float("nan")

    rows = sorted(vals, key=lambda k: -sum(dur.get(k, [0])))[:top]
    print("| kernel | avg us | MFMA busy | VALU / MFMA | LDS conflict cyc / LDS instr | wait share |")
    print("|---|---:|---:|---:|---:|---:|")
    for k in rows:
        mf = m(k, "SQ_INSTS_MFMA")
        lds = m(k, "SQ_INSTS_LDS")
        busy = m(k, "SQ_VALU_MFMA_BUSY_CYCLES") / (m(k, "GRBM_GUI_ACTIVE") * 128)
        du = dur.get(k, [0])
        print("| `{}` | {:.1f} | {:.2f} | {} | {} | {:.2f} |".format(
            k, sum(du) / len(du), busy, "{:.1f}".format(m(k, "SQ_INSTS_VALU") / mf) if mf else "-",
            "{:.2f}".format(m(k, "SQ_LDS_BANK_CONFLICT") / lds) if lds else "-",
            m(k, "SQ_WAIT_ANY") / m(k, "SQ_WAVE_CYCLES")))


if __name__ == "__main__":
    main()
