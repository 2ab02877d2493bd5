"""Main-stream idle gaps per training step from a rocprofv3 kernel trace: the last complete step
(delimited by the SGD-momentum kernel), gaps between consecutive kernels of the busiest queue,
split at the first backward kernel (the loss kernel).
    python scripts/gap_summary.py gpurun_out/prof_TAG
"""
import csv
import glob
import os
import statistics
import sys


def main():
    f = glob.glob(os.path.join(sys.argv[1], "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    sgd = [i for i, r in enumerate(rows) if "sgd_momentum" in r["Kernel_Name"]]
    seg = rows[sgd[-2] + 1:sgd[-1] + 1]
    q = max({r["Queue_Id"] for r in seg}, key=lambda k: sum(1 for r in seg if r["Queue_Id"] == k))
    main_q = [r for r in seg if r["Queue_Id"] == q]
    split = next((i for i, r in enumerate(main_q) if "softmax_xent" in r["Kernel_Name"]), len(main_q))
    for name, part in (("forward", main_q[:split + 1]), ("backward", main_q[split:])):
        gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(part, part[1:])]
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in part)
        print(f"{name}: {len(part)} kernels, busy {busy / 1e3:.1f} us, gaps {sum(gaps) / 1e3:.1f} us "
              f"(median {statistics.median(gaps) / 1e3:.2f} us, > 5 us: {sum(g > 5000 for g in gaps)})")
    t0, t1 = int(rows[sgd[-2]]["End_Timestamp"]), int(rows[sgd[-1]]["End_Timestamp"])
    print(f"step {(t1 - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
