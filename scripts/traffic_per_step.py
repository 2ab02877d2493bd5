"""HBM traffic per training step by kernel from scripts/pmc_summary.py --out files (FETCH_SIZE /
WRITE_SIZE passes over `bench.py --steps 3 --warmup 1`: 4 training steps per pass; traffic =
2 * FETCH_SIZE + WRITE_SIZE per dispatch, the gfx950 correction pmc_summary.py applies).
    python scripts/traffic_per_step.py LABEL PMC.json MS_PER_STEP [--steps 4] [--top 16]
"""
import json
import sys


def main():
    label, path, ms = sys.argv[1], sys.argv[2], float(sys.argv[3])
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 4
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 16
    ks = json.load(open(path))["kernels"]
    # whole-run totals; the setup's copies and the warm-up step are in the 4 steps' share too
    rows = sorted(((v["traffic_bytes"] * v["dispatches"] / steps, v["dispatches"] / steps, v["traffic_bytes"], k)
                   for k, v in ks.items()), reverse=True)
    total = sum(r[0] for r in rows)
    print(f"## {label}: {total / 1e9:.2f} GB per step; at {ms:.3f} ms per step that is "
          f"{total / (ms * 1e-3) / 1e12:.2f} TB/s averaged over the step")
    cum = 0.0
    for per, calls, per_call, k in rows[:top]:
        cum += per
        print(f"{k[:100]:<102} {calls:5.1f}/step {per_call / 1e6:10.2f} MB/call {per / 1e9:7.3f} GB/step  cum "
              f"{100 * cum / total:5.1f}%")


if __name__ == "__main__":
    main()
