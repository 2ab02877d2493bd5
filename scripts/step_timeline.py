"""One training step's kernels from a rocprofv3 kernel trace, in start order: queue (numbered by first
appearance), start in us from the end of the previous SGD-momentum kernel, duration in us, kernel name.
The last complete step of the trace (delimited by the SGD-momentum kernel).
    python scripts/step_timeline.py gpurun_out/prof_TAG "config-3" > profiles/TAG_step_timeline.txt
"""
import csv
import glob
import os
import sys


def main():
    f = glob.glob(os.path.join(sys.argv[1], "*kernel_trace.csv"))[0]
    label = sys.argv[2] if len(sys.argv) > 2 else "config-3"
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    sgd = [i for i, r in enumerate(rows) if "sgd_momentum" in r["Kernel_Name"]]
    seg = rows[sgd[-2] + 1:sgd[-1] + 1]
    t0 = int(rows[sgd[-2]]["End_Timestamp"])
    qn = {}
    for r in seg:
        qn.setdefault(r["Queue_Id"], len(qn) + 1)
    tag = os.path.basename(os.path.normpath(sys.argv[1]))
    print(f"# one {label} training step (rocprofv3 kernel trace, {tag}): queue, start (us from the previous SGD), "
          "duration (us), kernel")
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].removeprefix("void ").replace("dk::", "")
        name = name[:name.index(">(") + 1] if ">(" in name else name.split("(")[0]
        print(f"q {qn[r['Queue_Id']]} {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {name[:80]}")


if __name__ == "__main__":
    main()
