"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd .db or *_kernel_stats.csv)
into a markdown table: kernel, calls, total/avg duration, share.

    python scripts/prof_summary.py gpurun_out/prof_r01b [--steps 8] > profiles/r01_kernel_stats.md
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=0, help="training steps profiled (adds a per-step column)")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    dbs = glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True)
    rows = rows_from_csv(csvs[0]) if csvs else rows_from_db(dbs[0])
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
