"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd .db or *_kernel_stats.csv)
into a markdown table: kernel, calls, total/avg duration, share.

    python scripts/prof_summary.py gpurun_out/prof_r01b [--steps 8] > profiles/r01_kernel_stats.md

With --steps N and a kernel trace (*_kernel_trace.csv) present, only the kernels of the last N
training steps are counted: a step ends at the SGD-momentum update kernel, so setup work (the
warm-up, the instrumented roofline step's event records, probes, the CPU baseline's transfers)
does not leak into the per-step numbers.
"""
import argparse
import csv
import glob
import os
import sqlite3


def rows_from_db(path):
    c = sqlite3.connect(path)
    return [(r[0], int(r[1]), float(r[2]), float(r[3]), float(r[4]))
            for r in c.execute("select name, total_calls, total_duration, average, percentage from top_kernels")]


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3,
                        float(r["Percentage"])))
    return out


def rows_from_trace(path, steps, marker="sgd_momentum"):
    """Per-kernel (name, calls, total us, avg us, pct) over the last `steps` step windows."""
    with open(path) as f:
        tr = list(csv.DictReader(f))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(tr) if marker in r["Kernel_Name"]]
    if len(ends) < steps + 1:
        return None
    lo, hi = ends[-steps - 1] + 1, ends[-1] + 1
    agg = {}
    for r in tr[lo:hi]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        a = agg.setdefault(r["Kernel_Name"], [0, 0.0])
        a[0] += 1
        a[1] += d
    tot = sum(v[1] for v in agg.values())
    return [(n, c, t, t / c, 100 * t / tot) for n, (c, t) in agg.items()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=0, help="training steps profiled (adds a per-step column)")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    dbs = glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True)
    traces = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = rows_from_trace(traces[0], a.steps) if (traces and a.steps) else None
    if rows is None:
        rows = rows_from_csv(csvs[0]) if csvs else rows_from_db(dbs[0])
    else:
        print("(last {} training steps of the kernel trace, delimited by the SGD-momentum kernel)\n".format(a.steps))
    rows.sort(key=lambda r: -r[2])
    total = sum(r[2] for r in rows)
    print("| kernel | calls | total us | avg us | % |" + (" us/step |" if a.steps else ""))
    print("|---|---:|---:|---:|---:|" + ("---:|" if a.steps else ""))
    for name, calls, tot, avg, pct in rows[:a.top]:
        short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        if len(short) > 110:
            short = short[:107] + "..."
        line = "| `{}` | {} | {:.1f} | {:.2f} | {:.2f} |".format(short, calls, tot, avg, 100 * tot / total)
        if a.steps:
            line += " {:.1f} |".format(tot / a.steps)
        print(line)
    print("\nTotal kernel time: {:.1f} us{}".format(total, " ({:.1f} us/step)".format(total / a.steps) if a.steps else ""))


if __name__ == "__main__":
    main()
