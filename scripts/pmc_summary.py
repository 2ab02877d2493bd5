"""Per-kernel HBM traffic from two rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d gpurun_out/pmc_fetch -o run -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d gpurun_out/pmc_write -o run -- python bench.py ...
    python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write --out profiles/<tag>_pmc.json

Corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so it is doubled.
Infinity-Cache hits are counted by these memory-side counters, not excluded.
"""
import argparse
import csv
import glob
import json
import os
import time
from collections import defaultdict


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != counter:
                    continue
                per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")


def index_add(path, config):
    """Append `path` (a summary under profiles/) to profiles/pmc_index.json as the newest entry for
    bench config `config`: bench.py takes the last matching entry, i.e. the order summaries were added."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    idx_path = os.path.join(root, "profiles", "pmc_index.json")
    with open(idx_path) as fh:
        idx = json.load(fh)
    rel = os.path.relpath(os.path.abspath(path), root)
    idx["entries"] = [e for e in idx["entries"] if e["file"] != rel]
    idx["entries"].append({"file": rel, "config": config, "commit": None, "added_unix": int(time.time())})
    with open(idx_path, "w") as fh:
        json.dump(idx, fh, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir", nargs="?")
    ap.add_argument("write_dir", nargs="?")
    ap.add_argument("--add", default=None, help="only register this existing summary in profiles/pmc_index.json")
    ap.add_argument("--out", default=None)
    ap.add_argument("--config", type=int, default=None,
                    help="append --out to profiles/pmc_index.json as the newest summary of this bench config")
    a = ap.parse_args()
    if a.add:
        if a.config is None:
            raise SystemExit("--add needs --config")
        return index_add(a.add, a.config)
    if not (a.fetch_dir and a.write_dir and a.out):
        raise SystemExit("fetch_dir, write_dir and --out are required")
    fetch = load(a.fetch_dir, "FETCH_SIZE")
    write = load(a.write_dir, "WRITE_SIZE")
    out = {"unit": "bytes per dispatch",
           "correction": "traffic = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes); gfx950 FETCH_SIZE halves wide reads",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        fv, wv = fetch.get(k, []), write.get(k, [])
        f = 1024.0 * sum(fv) / len(fv) if fv else None
        w = 1024.0 * sum(wv) / len(wv) if wv else None
        out["kernels"][short(k)] = {
            "dispatches": max(len(fv), len(wv)),
            "fetch_bytes_raw": f, "write_bytes": w,
            "traffic_bytes": (2 * f if f is not None else 0) + (w or 0),
        }
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    out["created_unix"] = int(time.time())
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    if a.config is not None:
        index_add(a.out, a.config)
    top = sorted(out["kernels"].items(), key=lambda kv: -kv[1]["traffic_bytes"] * kv[1]["dispatches"])[:15]
    for k, v in top:
        print(f"{k[:90]:90s} n={v['dispatches']:5d} traffic/dispatch={v['traffic_bytes'] / 1e6:9.2f} MB")


if __name__ == "__main__":
    main()
