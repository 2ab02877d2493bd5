"""Tabulate rocprofv3 counter passes (pmc_probe.sh output): mean counter value per kernel
and dispatch order group.  python scripts/pmc_table.py gpurun_out/pmc_TAG"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        k = k[:70] + " gx=" + r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(k)
    print("   " + "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))
