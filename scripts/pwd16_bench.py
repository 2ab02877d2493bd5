"""bf16 deep pointwise layers of config 5 (batch 512): the weight-stationary kernels (pw_deep_bf16.hip,
knob 13 on) against the column-sliced ones (knob 13 off), forward with BN on load + statistics and
the BN-backward-on-load dgrad with dy write-through and the input BN's partials.  Median of 15 calls;
fraction of the HBM spec (8 TB/s) on the algorithmic bytes; outputs compared bitwise.
    python scripts/pwd16_bench.py [--only fwd|dgrad]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, stream_handle  # noqa: E402

B = 512
SHAPES = [(28, 128, 256), (14, 256, 256), (14, 256, 512), (7, 512, 512), (28, 128, 128)]  # HW, C, K


def timeit(fn, reps=15):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return 1e3 * t[len(t) // 2]


def main():
    st = stream_handle()
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    torch.manual_seed(0)
    bf = torch.bfloat16
    rnd = lambda n: torch.randn(n, device="cuda")
    for HW, C, K in SHAPES:
        M = B * HW * HW
        x, g, xo = rnd(M * C).to(bf), rnd(M * K).to(bf), rnd(M * K).to(bf)
        w = rnd(K * C) * 0.05
        pi = [rnd(C), rnd(C).abs() + 0.5, rnd(C), rnd(C)]
        po = [rnd(K), rnd(K).abs() + 0.5, rnd(K), rnd(K)]
        k12 = rnd(2 * K) * 0.1
        res, outs = [], {}
        for deep in (0, 1):
            lib.dk_debug_set_gemm_config(13, deep)
            y = torch.empty(M * K, dtype=bf, device="cuda")
            dy = torch.empty(M * K, dtype=bf, device="cuda")
            dx = torch.empty(M * C, dtype=bf, device="cuda")
            line = []
            if only in (None, "fwd"):
                rows = lib.dk_pwconv_fwd_bf16_stats_rows(B, HW, HW, K, C)
                part = torch.empty(rows * 2 * K, dtype=torch.float64, device="cuda")
                fa = (x.data_ptr(), B, HW, HW, C, w.data_ptr(), K, 1, 0, y.data_ptr(), HW, HW,
                      *(t.data_ptr() for t in pi), 1, part.data_ptr(), st)
                tf = timeit(lambda: lib.dk_pwconv_fwd_ex_bf16(*fa))
                byt = 2 * (M * C + M * K) + 4 * K * C
                line.append(f"fwd {tf:6.1f} us {byt / tf / 1e3 / 8000:4.2f}")
            if only in (None, "dgrad"):
                rows = lib.dk_pwconv_dgrad_bnbwd_bf16_stats_rows(B, HW, HW, K, C)
                partd = torch.empty(rows * 2 * C, dtype=torch.float64, device="cuda")
                da = (g.data_ptr(), xo.data_ptr(), B, HW, HW, K, *(t.data_ptr() for t in po), 1, k12.data_ptr(),
                      dy.data_ptr(), w.data_ptr(), C, dx.data_ptr(), 0, x.data_ptr(), *(t.data_ptr() for t in pi),
                      1, partd.data_ptr(), st)
                td = timeit(lambda: lib.dk_pwconv_dgrad_bnbwd_bf16(*da))
                byt = 2 * (3 * M * K + 2 * M * C) + 4 * K * C
                line.append(f"dgrad {td:6.1f} us {byt / td / 1e3 / 8000:4.2f}")
            torch.cuda.synchronize()
            outs[deep] = (y.clone(), dy.clone(), dx.clone())
            res.append(("ws " if deep else "cs ") + ", ".join(line))
        lib.dk_debug_set_gemm_config(13, -1)
        same = ["bitwise" if torch.equal(a, b) else "DIFF" for a, b in zip(outs[0], outs[1])]
        print(f"{B}x{HW}x{HW} C={C:3d} K={K:3d} | " + " | ".join(res) + " | y/dy/dx " + " ".join(same), flush=True)


if __name__ == "__main__":
    main()
