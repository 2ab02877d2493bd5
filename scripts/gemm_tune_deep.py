"""Tile configurations for the pointwise GEMMs that stay on the tiled engine (the 14 x 14 and 7 x 7
layers, K or C >= 256): every row configuration (knob 0) for the forward with BN on load +
statistics and for the BN-backward-on-load dgrad, every split-K configuration (knob 1) for the
weight gradient; median of 7 timed calls each.  fp32 at batch 256 (config 3) or, with --bf16,
bf16 at batch 512 (config 5).
    python scripts/gemm_tune_deep.py [--bf16]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, workspace  # noqa: E402

BF16 = torch.bfloat16
HALF = "--bf16" in sys.argv
B = 512 if HALF else 256
SHAPES = [(B, 14, 256, 256), (B, 14, 128, 256), (B, 7, 512, 512), (B, 7, 256, 512)]  # N, HW, C, K
DT = BF16 if HALF else torch.float32
SUF = "bf16" if HALF else "f32"


def timeit(fn, reps=7):
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
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(0)

    def rnd(*s, dt=torch.float32):
        return torch.randn(*s, device="cuda", generator=g).to(dt)

    nrow = lib.dk_debug_set_gemm_config(0, -1)
    nsplit = lib.dk_debug_set_gemm_config(1, -1)
    for N, HW, C, K in SHAPES:
        M = N * HW * HW
        x, y = rnd(M * C, dt=DT), torch.empty(M * K, dtype=DT, device="cuda")
        gy, xo = rnd(M * K, dt=DT), rnd(M * K, dt=DT)
        dy, dx = torch.empty(M * K, dtype=DT, device="cuda"), torch.empty(M * C, dtype=DT, device="cuda")
        w = rnd(K * C) * 0.05
        pi = [rnd(C), rnd(C).abs() + 0.5, rnd(C), rnd(C)]
        po = [rnd(K), rnd(K).abs() + 0.5, rnd(K), rnd(K)]
        k12 = rnd(2 * K) * 0.1
        dw = torch.empty(K * C, device="cuda")
        res = {}
        for cfg in list(range(nrow)) + [-1]:
            lib.dk_debug_set_gemm_config(0, cfg)
            rows = (lib.dk_pwconv_fwd_bf16_stats_rows if HALF else lib.dk_pwconv_fwd_stats_rows)(N, HW, HW, K, C)
            part = torch.empty(rows * 2 * K, dtype=torch.float64, device="cuda")
            fa = (x.data_ptr(), N, HW, HW, C, w.data_ptr(), K, 1, 0, y.data_ptr(), HW, HW,
                  *(t.data_ptr() for t in pi), 1, part.data_ptr(), st)
            tf = timeit(lambda: getattr(lib, "dk_pwconv_fwd_ex_" + SUF)(*fa))
            rows = (lib.dk_pwconv_dgrad_bnbwd_bf16_stats_rows if HALF else lib.dk_pwconv_dgrad_bnbwd_stats_rows)(N, HW, HW, K, C)
            partd = torch.empty(rows * 2 * C, dtype=torch.float64, device="cuda")
            da = (gy.data_ptr(), xo.data_ptr(), N, HW, HW, K, *(t.data_ptr() for t in po), 1, k12.data_ptr(),
                  dy.data_ptr(), w.data_ptr(), C, dx.data_ptr(), 0, x.data_ptr(), *(t.data_ptr() for t in pi), 1,
                  partd.data_ptr(), st)
            td = timeit(lambda: getattr(lib, "dk_pwconv_dgrad_bnbwd_" + SUF)(*da))
            res[cfg] = (tf, td)
            print(f"{N}x{HW}x{HW} C={C} K={K} row cfg {cfg:3d}: fwd {tf:7.1f} us  dgrad_bnbwd {td:7.1f} us", flush=True)
        lib.dk_debug_set_gemm_config(0, -1)
        for cfg in list(range(nsplit)) + [-1]:
            lib.dk_debug_set_gemm_config(1, cfg)
            nb = lib.dk_pwconv_wgrad_workspace_bytes(N, HW, HW, K, C)
            wa = (dy.data_ptr(), x.data_ptr(), N, HW, HW, C, K, 1, HW, HW, 0, 0.0, dw.data_ptr(), workspace.get(nb), nb,
                  *(t.data_ptr() for t in pi), 1, st)
            tw = timeit(lambda: getattr(lib, "dk_pwconv_wgrad_bnx_" + SUF)(*wa))
            print(f"{N}x{HW}x{HW} C={C} K={K} split cfg {cfg:3d}: wgrad {tw:7.1f} us", flush=True)
        lib.dk_debug_set_gemm_config(1, -1)
        del x, y, gy, xo, dy, dx


if __name__ == "__main__":
    main()
