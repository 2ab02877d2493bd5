"""The last kernels of a training step on every queue (rocprofv3 kernel trace): what the
optimizer step waits for.  python scripts/tail_timeline.py gpurun_out/prof_TAG [--us 400]"""
import csv
import glob
import os
import sys


def main():
    f = glob.glob(os.path.join(sys.argv[1], "*kernel_trace.csv"))[0]
    span = float(sys.argv[sys.argv.index("--us") + 1]) if "--us" in sys.argv else 400.0
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    sgd = [i for i, r in enumerate(rows) if "sgd_momentum" in r["Kernel_Name"]]
    end = int(rows[sgd[-1]]["Start_Timestamp"])
    t0 = end - span * 1e3
    for r in rows[sgd[-2] + 1:sgd[-1] + 1]:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if b >= t0:
            print(f"q{r['Queue_Id']}  {(a - end) / 1e3:8.1f} .. {(b - end) / 1e3:8.1f}  ({(b - a) / 1e3:6.1f})  "
                  f"{r['Kernel_Name'][:90]}")


if __name__ == "__main__":
    main()
