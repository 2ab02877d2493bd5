"""Main-stream idle gaps per training step from a rocprofv3 kernel trace: the last complete step
(delimited by the SGD-momentum kernel), gaps between consecutive kernels of the busiest queue,
split at the first backward kernel (the loss kernel).
    python scripts/gap_summary.py gpurun_out/prof_TAG [--list]
--list: also the main queue's kernels grouped by name (busy time per step) and the ten largest
gaps with the kernel after which each opens, plus the other queues' busy time.
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
    split = next((i for i, r in enumerate(main_q) if "softmax_xent" in r["Kernel_Name"]),
                 next((i - 1 for i, r in enumerate(main_q) if "bwd" in r["Kernel_Name"]), len(main_q)))
    for name, part in (("forward", main_q[:split + 1]), ("backward", main_q[split:])):
        gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(part, part[1:])]
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in part)
        print(f"{name}: {len(part)} kernels, busy {busy / 1e3:.1f} us, gaps {sum(gaps) / 1e3:.1f} us "
              f"(median {statistics.median(gaps) / 1e3:.2f} us, > 5 us: {sum(g > 5000 for g in gaps)})")
    t0, t1 = int(rows[sgd[-2]]["End_Timestamp"]), int(rows[sgd[-1]]["End_Timestamp"])
    print(f"step {(t1 - t0) / 1e3:.1f} us")
    if "--list" not in sys.argv:
        return
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    by = {}
    for r in main_q:
        n = r["Kernel_Name"][:110]
        c, t = by.get(n, (0, 0))
        by[n] = (c + 1, t + dur(r))
    print("\nmain queue, by kernel (us per step):")
    for n, (c, t) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print(f"  {t / 1e3:8.1f}  x{c:3d}  {n}")
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"]), a["Kernel_Name"][:80], b["Kernel_Name"][:80])
            for a, b in zip(main_q, main_q[1:])]
    print("\nlargest main-queue gaps (us, after -> before):")
    for g, a, b in sorted(gaps, reverse=True)[:10]:
        print(f"  {g / 1e3:7.2f}  {a}  ->  {b}")
    for oq in sorted({r["Queue_Id"] for r in seg} - {q}):
        part = [r for r in seg if r["Queue_Id"] == oq]
        print(f"queue {oq}: {len(part)} kernels, busy {sum(dur(r) for r in part) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
