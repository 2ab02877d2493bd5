"""fp32 deep pointwise layers of config 3 (batch 256): the deep streaming kernels (pw_deep.hip,
knob 11 on) against the previous path (knob 11 off: the tiled engine, or pw_stream.hip's K = C = 128
forward), forward with BN on load + statistics, the strided skip projections, the
BN-backward-on-load dgrad with dy write-through and the input BN's partials, and the BN-on-load
weight gradient (with its split reduce).  Median of 15 calls,
fraction of the fp32 MFMA peak (157.3 TF/s); outputs of the two paths compared bitwise.
    python scripts/pwd_bench.py [--only fwd|skip|dgrad|wgrad] [--shape HW,C,K] [--deep 0|1] [--fold]
(--fold: the forward also timed with the in-launch BatchNorm statistics fold armed, as in the network)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import fold_resources, lib, stream_handle  # noqa: E402

B = 256
PEAK = 157.3
SHAPES = [(28, 64, 128), (28, 128, 128), (14, 128, 256), (14, 256, 256), (7, 256, 512), (7, 512, 512)]
SKIPS = [(56, 64, 128), (28, 128, 256), (14, 256, 512)]  # input HW, C, K; stride 2


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


def rnd(n):
    return torch.randn(n, device="cuda")


def main():
    st = stream_handle()
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    shapes = SHAPES
    if "--shape" in sys.argv:
        shapes = [tuple(int(v) for v in sys.argv[sys.argv.index("--shape") + 1].split(","))]
    fold = "--fold" in sys.argv
    # 0: the tiled engine; 1: the deep kernels
    modes = (0, 1)
    if "--modes" in sys.argv:
        modes = tuple(int(v) for v in sys.argv[sys.argv.index("--modes") + 1].split(","))
    torch.manual_seed(0)
    for HW, C, K in shapes:
        M = B * HW * HW
        x, g, xo = rnd(M * C), rnd(M * K), rnd(M * K)
        w = rnd(K * C) * 0.05
        pi = [rnd(C), rnd(C).abs() + 0.5, rnd(C), rnd(C)]
        po = [rnd(K), rnd(K).abs() + 0.5, rnd(K), rnd(K)]
        k12 = rnd(2 * K) * 0.1
        flops = 2.0 * M * K * C
        res, outs, wout = [], {}, {}
        for deep in modes:
            lib.dk_debug_set_gemm_config(11, 1 if deep else 0)
            lib.dk_debug_set_gemm_config(14, 1 if deep else 0)
            y = torch.full((M * K,), float("nan"), device="cuda")
            dy = torch.full((M * K,), float("nan"), device="cuda")
            dx = torch.full((M * C,), float("nan"), device="cuda")
            line = []
            if only in (None, "fwd"):
                rows = lib.dk_pwconv_fwd_stats_rows(B, HW, HW, K, C)
                part = torch.empty(rows * 2 * K, dtype=torch.float64, device="cuda")
                fa = (x.data_ptr(), B, HW, HW, C, w.data_ptr(), K, 1, 0, y.data_ptr(), HW, HW,
                      *(t.data_ptr() for t in pi), 1, part.data_ptr(), st)
                tf = timeit(lambda: lib.dk_pwconv_fwd_ex_f32(*fa))
                line.append(f"fwd {tf:6.1f} us {flops / tf / 1e6 / PEAK:4.2f}")
                if fold:
                    # the network's call: the following BatchNorm's statistics folded in-launch
                    stats = [torch.empty(K, device="cuda") for _ in range(5)]
                    fr = fold_resources.get()

                    def armed():
                        lib.dk_bn_fold_arm_stats(part.data_ptr(), rows, K, float(M), 1e-5, 0.95, 0,
                                                 *(t.data_ptr() for t in stats), *fr)
                        lib.dk_pwconv_fwd_ex_f32(*fa)
                    tff = timeit(armed)
                    line.append(f"fwd+fold {tff:6.1f} us {flops / tff / 1e6 / PEAK:4.2f}")
            if only in (None, "dgrad"):
                rows = lib.dk_pwconv_dgrad_bnbwd_stats_rows(B, HW, HW, K, C)
                partd = torch.empty(rows * 2 * C, dtype=torch.float64, device="cuda")
                da = (g.data_ptr(), xo.data_ptr(), B, HW, HW, K, *(t.data_ptr() for t in po), 1, k12.data_ptr(),
                      dy.data_ptr(), w.data_ptr(), C, dx.data_ptr(), 0, x.data_ptr(), *(t.data_ptr() for t in pi),
                      1, partd.data_ptr(), st)
                td = timeit(lambda: lib.dk_pwconv_dgrad_bnbwd_f32(*da))
                line.append(f"dgrad {td:6.1f} us {flops / td / 1e6 / PEAK:4.2f}")
            if only in (None, "wgrad"):
                nb = lib.dk_pwconv_wgrad_workspace_bytes(B, HW, HW, K, C)
                ws = torch.empty(nb // 4 + 1, device="cuda")
                dw = torch.empty(K * C, device="cuda")
                wa = (g.data_ptr(), x.data_ptr(), B, HW, HW, C, K, 1, HW, HW, w.data_ptr(), 1e-4, dw.data_ptr(),
                      ws.data_ptr(), nb, *(t.data_ptr() for t in pi), 1, st)
                tw = timeit(lambda: lib.dk_pwconv_wgrad_bnx_f32(*wa))
                line.append(f"wgrad {tw:6.1f} us {flops / tw / 1e6 / PEAK:4.2f}")
                torch.cuda.synchronize()
                wout[deep] = dw.clone()
            if only in (None, "bwd") and deep and lib.dk_pwconv_bwd_fused_preferred(B, HW, HW, K, C):
                # the fused deep backward (knob 14): dgrad + weight gradient in one pass, dy not stored
                rows = lib.dk_pwconv_bwd_fused_rows(B, HW, HW, K, C)
                partb = torch.empty(rows * 2 * C, dtype=torch.float64, device="cuda")
                nbf = lib.dk_pwconv_bwd_fused_workspace_bytes(B, HW, HW, K, C)
                wsf = torch.empty(nbf // 4 + 1, device="cuda")
                dwf = torch.empty(K * C, device="cuda")
                ba = (g.data_ptr(), xo.data_ptr(), B, HW, HW, K, *(t.data_ptr() for t in po), 1, k12.data_ptr(),
                      w.data_ptr(), C, 1e-4, dwf.data_ptr(), dx.data_ptr(), 0, x.data_ptr(),
                      *(t.data_ptr() for t in pi), 1, partb.data_ptr(), wsf.data_ptr(), nbf, st)
                tb = timeit(lambda: lib.dk_pwconv_bwd_bnbwd_f32(*ba))
                line.append(f"fused bwd {tb:6.1f} us {2 * flops / tb / 1e6 / PEAK:4.2f}")
            torch.cuda.synchronize()
            outs[deep] = (y.clone(), dy.clone(), dx.clone())
            res.append(("old  ", "deep ")[deep] + ", ".join(line))
        for k in (11, 14):
            lib.dk_debug_set_gemm_config(k, -1)
        same = []
        ms = sorted(outs)
        for m0, m1 in zip(ms, ms[1:]):
            same.append("%d~%d " % (m0, m1) + " ".join(
                "bitwise" if torch.equal(a, b) else "DIFF(max %.2e)" % float((a - b).abs().nan_to_num(1e30).max())
                for a, b in zip(outs[m0], outs[m1])))
            if m0 in wout and m1 in wout:
                a, b = wout[m0].double(), wout[m1].double()
                same.append("dW rel %.1e" % float((a - b).norm() / a.norm()))
        print(f"{B}x{HW}x{HW} C={C:3d} K={K:3d} | " + " | ".join(res) + " | y/dy/dx " + " ".join(same), flush=True)
    if only in (None, "skip") and "--shape" not in sys.argv:
        for H, C, K in SKIPS:
            OH = H // 2
            M = B * OH * OH
            x, w = rnd(B * H * H * C), rnd(K * C) * 0.05
            flops = 2.0 * M * K * C
            line, outs = [], {}
            for deep in (0, 1):
                lib.dk_debug_set_gemm_config(11, deep)
                y = torch.full((M * K,), float("nan"), device="cuda")
                a = (x.data_ptr(), B, H, H, C, w.data_ptr(), K, 2, 0, y.data_ptr(), OH, OH, st)
                t = timeit(lambda: lib.dk_pwconv_fwd_f32(*a))
                torch.cuda.synchronize()
                outs[deep] = y.clone()
                line.append(f"{'deep' if deep else 'old '} {t:6.1f} us {flops / t / 1e6 / PEAK:4.2f}")
            lib.dk_debug_set_gemm_config(11, -1)
            print(f"skip {B}x{H}x{H} C={C:3d} K={K:3d} s2 | " + " | ".join(line) + " | " +
                  ("bitwise" if torch.equal(outs[0], outs[1]) else "DIFF"), flush=True)


if __name__ == "__main__":
    main()
