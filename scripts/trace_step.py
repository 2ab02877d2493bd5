"""Print one training step of a rocprofv3 kernel trace in dispatch order: stream, kernel,
duration and the idle gap before it on its stream.

    python scripts/trace_step.py gpurun_out/prof_r02i/bench_kernel_trace.csv --step -2
"""
import argparse
import csv


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:120]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="dk::nchw_to_nhwc4_kernel", help="first kernel of a step")
    ap.add_argument("--step", type=int, default=-2)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(a.marker)]
    i0 = starts[a.step]
    i1 = starts[a.step + 1] if a.step + 1 < len(starts) and a.step != -1 else len(rows)
    last_end = {}
    t0 = int(rows[i0]["Start_Timestamp"])
    busy = 0
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r["Queue_Id"]
        gap = (s - last_end[q]) / 1e3 if q in last_end else 0.0
        last_end[q] = e
        busy += e - s
        print("{:9.1f} q{:>2} {:8.2f} us gap {:6.2f}  grid {:>7}x{:<3} {}".format(
            (s - t0) / 1e3, q, (e - s) / 1e3, gap, r["Grid_Size_X"], r["Grid_Size_Y"], short(r["Kernel_Name"])))
    print("step span {:.1f} us, kernel busy {:.1f} us, {} dispatches".format(
        (int(rows[i1 - 1]["End_Timestamp"]) - t0) / 1e3, busy / 1e3, i1 - i0))


if __name__ == "__main__":
    main()
