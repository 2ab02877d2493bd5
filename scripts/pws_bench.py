"""A/B timing of the streaming pointwise kernels (csrc/pw_stream.hip) against the tiled engine:
dk_pwconv_dgrad_bnbwd_f32 (the step's dominant entry point) at the K = C = 64 shapes of
ResNet-18-depsep, batch 256.  Prints us per call and GB/s of algorithmic bytes (perfmodel).

    python scripts/pws_bench.py [--batch 256]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib  # noqa: E402
from dorknet_amd import perfmodel  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return 1e3 * t[len(t) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    B = a.batch
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(0)

    def rnd(n):
        return torch.randn(n, device="cuda", generator=g)

    for name, H, K, C in (("res1 pw (56x56, 64->64)", 56, 64, 64), ("pw 28x28 64->64", 28, 64, 64)):
        P = B * H * H
        gg, xo, dy, xin = rnd(P * K), rnd(P * K), torch.empty(P * K, device="cuda"), rnd(P * C)
        dx = torch.empty(P * C, device="cuda")
        w = rnd(K * C) * 0.1
        po = [rnd(K), rnd(K).abs() + 0.5, rnd(K), rnd(K)]
        pi = [rnd(C), rnd(C).abs() + 0.5, rnd(C), rnd(C)]
        k12 = rnd(2 * K) * 0.1
        for res in (False, True):
            rr = rnd(P * C) if res else None
            line = []
            for mode in (0, 1):
                lib.dk_debug_set_gemm_config(3, mode)
                rows = lib.dk_pwconv_dgrad_bnbwd_stats_rows(B, H, H, K, C)
                part = torch.empty(rows * 2 * C, dtype=torch.float64, device="cuda")
                args = (gg.data_ptr(), xo.data_ptr(), B, H, H, K, *(t.data_ptr() for t in po), 1, k12.data_ptr(),
                        dy.data_ptr(), w.data_ptr(), C, dx.data_ptr(), rr.data_ptr() if res else 0, xin.data_ptr(),
                        *(t.data_ptr() for t in pi), 1, part.data_ptr(), st)
                us = timeit(lambda: lib.dk_pwconv_dgrad_bnbwd_f32(*args))
                f, by = perfmodel.work("dk_pwconv_dgrad_bnbwd_f32", args)
                line.append("{}: {:7.1f} us {:6.0f} GB/s ({} partial rows)".format(
                    "stream" if mode else "tiled ", us, by / us / 1e3, rows))
            lib.dk_debug_set_gemm_config(3, -1)
            print("{:28s} res={:d} | {}".format(name, res, " | ".join(line)), flush=True)
    # fused backward (dgrad + wgrad, dy never stored) vs the unfused pair at res1
    from dorknet_amd._hip import workspace
    K = C = 64
    H = 56
    P = B * H * H
    gg, xo, dy, xin = rnd(P * K), rnd(P * K), torch.empty(P * K, device="cuda"), rnd(P * C)
    dx = torch.empty(P * C, device="cuda")
    w = rnd(K * C) * 0.1
    dw = torch.empty(K * C, device="cuda")
    po = [rnd(K), rnd(K).abs() + 0.5, rnd(K), rnd(K)]
    pi = [rnd(C), rnd(C).abs() + 0.5, rnd(C), rnd(C)]
    k12 = rnd(2 * K) * 0.1
    rows = lib.dk_pwconv_dgrad_bnbwd_stats_rows(B, H, H, K, C)
    part = torch.empty(rows * 2 * C, dtype=torch.float64, device="cuda")
    nbw = lib.dk_pwconv_wgrad_workspace_bytes(B, H, H, K, C)
    wsw = workspace.get(nbw)

    def unfused():
        lib.dk_pwconv_dgrad_bnbwd_f32(gg.data_ptr(), xo.data_ptr(), B, H, H, K, *(t.data_ptr() for t in po), 1,
                                      k12.data_ptr(), dy.data_ptr(), w.data_ptr(), C, dx.data_ptr(), 0,
                                      xin.data_ptr(), *(t.data_ptr() for t in pi), 1, part.data_ptr(), st)
        lib.dk_pwconv_wgrad_bnx_f32(dy.data_ptr(), xin.data_ptr(), B, H, H, C, K, 1, H, H, w.data_ptr(), 1e-4,
                                    dw.data_ptr(), wsw, nbw, *(t.data_ptr() for t in pi), 1, st)
    us0 = timeit(unfused)
    rows1 = lib.dk_pwconv_bwd_fused_rows(B, H, H, K, C)
    part1 = torch.empty(rows1 * 2 * C, dtype=torch.float64, device="cuda")
    nbf = lib.dk_pwconv_bwd_fused_workspace_bytes(B, H, H, K, C)
    wsf = torch.empty(nbf, dtype=torch.uint8, device="cuda")
    fargs = (gg.data_ptr(), xo.data_ptr(), B, H, H, K, *(t.data_ptr() for t in po), 1, k12.data_ptr(), w.data_ptr(), C,
             1e-4, dw.data_ptr(), dx.data_ptr(), 0, xin.data_ptr(), *(t.data_ptr() for t in pi), 1, part1.data_ptr(),
             wsf.data_ptr(), nbf, st)
    us1 = timeit(lambda: lib.dk_pwconv_bwd_bnbwd_f32(*fargs))
    f, by = perfmodel.work("dk_pwconv_bwd_bnbwd_f32", fargs)
    print("bwd res1 (64->64, 56x56)     | unfused dgrad_bnbwd + wgrad_bnx: {:7.1f} us | fused: {:7.1f} us {:6.0f} GB/s "
          "({} blocks)".format(us0, us1, by / us1 / 1e3, rows1), flush=True)
    # forward with BN on load + output statistics (res1 pw; pw0: stride 2 from 112x112)
    for name, H, s in (("fwd_ex res1 pw (56x56)", 56, 1), ("fwd_ex pw0 (112->56, s2)", 112, 2)):
        K = C = 64
        OH = -(-H // s)
        x = rnd(B * H * H * C)
        y = torch.empty(B * OH * OH * K, device="cuda")
        w = rnd(K * C) * 0.1
        pi = [rnd(C), rnd(C).abs() + 0.5, rnd(C), rnd(C)]
        line = []
        for mode in (0, 1):
            lib.dk_debug_set_gemm_config(3, mode)
            rows = lib.dk_pwconv_fwd_stats_rows(B, OH, OH, K, C)
            part = torch.empty(rows * 2 * K, dtype=torch.float64, device="cuda")
            args = (x.data_ptr(), B, H, H, C, w.data_ptr(), K, s, 0, y.data_ptr(), OH, OH,
                    *(t.data_ptr() for t in pi), 1, part.data_ptr(), st)
            us = timeit(lambda: lib.dk_pwconv_fwd_ex_f32(*args))
            f, by = perfmodel.work("dk_pwconv_fwd_ex_f32", args)
            line.append("{}: {:7.1f} us {:6.0f} GB/s ({} rows)".format("stream" if mode else "tiled ", us,
                                                                       by / us / 1e3, rows))
        lib.dk_debug_set_gemm_config(3, -1)
        print("{:28s}       | {}".format(name, " | ".join(line)), flush=True)


if __name__ == "__main__":
    main()
