"""Per-shape timing of the memory-bound kernels of the ResNet-18-depsep step (bs=256):
depthwise fwd/dgrad/wgrad, BatchNorm stats/apply/backward, the pointwise GEMMs with and
without BN on load.  Prints time per call and achieved GB/s of compulsory traffic.

    python scripts/kbench.py [--batch 256] [--only dw,bn,pw]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, workspace  # noqa: E402
from dorknet_amd import perfmodel  # noqa: E402


def timeit(fn, reps=7):
    fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return 1e3 * t[len(t) // 2]


def report(tag, us, name, args):
    f, b = perfmodel.work(name, args)
    print(f"{tag:34s} {us:9.1f} us  {b / us / 1e3:7.0f} GB/s  {f / us / 1e6:6.1f} TF/s", flush=True)


DW = [("res1_dw", 56, 64, 1), ("res3_dw1", 56, 64, 2), ("res3_dw2", 28, 128, 1), ("res5_dw1", 28, 128, 2),
      ("res5_dw2", 14, 256, 1), ("res7_dw1", 14, 256, 2), ("res7_dw2", 7, 512, 1)]
BN = [("conv0_bn", 112, 64), ("res1_bn", 56, 64), ("res3_bn", 28, 128), ("res5_bn", 14, 256), ("res7_bn", 7, 512)]
PW = [("pw0", 112, 64, 64, 2), ("res1_pw", 56, 64, 64, 1), ("res3_dw2_pw", 28, 128, 128, 1),
      ("res5_dw2_pw", 14, 256, 256, 1), ("res7_dw2_pw", 7, 512, 512, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--only", default="dw,dwb,bn,pw")
    a = ap.parse_args()
    B = a.batch
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(0)
    only = set(a.only.split(","))

    def rnd(n):
        return torch.randn(n, device="cuda", generator=g)

    def bnp(C):
        return [rnd(C), rnd(C).abs() + 0.5, rnd(C), rnd(C)]

    if "dw" in only:
        for name, H, C, s in DW:
            R, pad = 3, 1
            OH = (H + 2 * pad - R) // s + 1
            x, dy = rnd(B * H * H * C), rnd(B * OH * OH * C)
            y, dx = torch.empty(B * OH * OH * C, device="cuda"), torch.empty(B * H * H * C, device="cuda")
            w = rnd(C * 9)
            wr = torch.empty(C * 9, device="cuda")
            lib.dk_dw_weight_rsc_f32(w.data_ptr(), C, 3, 3, wr.data_ptr(), st)
            p = bnp(C)
            fa = (x.data_ptr(), B, H, H, C, wr.data_ptr(), 3, 3, s, pad, 0, y.data_ptr(), OH, OH, st)
            report(name + " fwd", timeit(lambda: lib.dk_dwconv_fwd_f32(*fa)), "dk_dwconv_fwd_f32", fa)
            fb = fa[:-1] + tuple(t.data_ptr() for t in p) + (1, st)
            report(name + " fwd bnx", timeit(lambda: lib.dk_dwconv_fwd_bnx_f32(*fb)), "dk_dwconv_fwd_bnx_f32", fb)
            nb = lib.dk_dwconv_dgrad_workspace_bytes(C, 3, 3)
            da = (dy.data_ptr(), B, OH, OH, C, w.data_ptr(), 3, 3, s, pad, dx.data_ptr(), H, H, workspace.get(nb), nb,
                  st)
            report(name + " dgrad", timeit(lambda: lib.dk_dwconv_dgrad_f32(*da)), "dk_dwconv_dgrad_f32", da)
            nb = lib.dk_dwconv_wgrad_workspace_bytes(B, OH, OH, C, 3, 3)
            dw = torch.empty(C * 9, device="cuda")
            wa = (dy.data_ptr(), x.data_ptr(), B, H, H, C, 3, 3, s, pad, OH, OH, 0, 0.0, dw.data_ptr(),
                  workspace.get(nb), nb, st)
            report(name + " wgrad", timeit(lambda: lib.dk_dwconv_wgrad_f32(*wa)), "dk_dwconv_wgrad_f32", wa)
            wb = wa[:-1] + tuple(t.data_ptr() for t in p) + (1, st)
            report(name + " wgrad bnx", timeit(lambda: lib.dk_dwconv_wgrad_bnx_f32(*wb)), "dk_dwconv_wgrad_bnx_f32",
                   wb)
            del x, dy, y, dx
    if "dwb" in only:
        # stride-1 depthwise backward when the layer fed a BatchNorm: the unfused chain
        # (BN-backward apply -> dgrad_ex with the input BN's partials -> wgrad_bnx) vs one pass
        for name, H, C, s in DW:
            if s != 1:
                continue
            n = B * H * H * C
            gg, xo, xin = rnd(n), rnd(n), rnd(n)
            dy, dx = torch.empty(n, device="cuda"), torch.empty(n, device="cuda")
            w = rnd(C * 9)
            po, pi = bnp(C), bnp(C)
            k12 = rnd(2 * C) * 0.1
            rows = lib.dk_dwconv_dgrad_stats_rows(B, H, H, C, 1)
            part = torch.empty(rows * 2 * C, dtype=torch.float64, device="cuda")
            dw = torch.empty(C * 9, device="cuda")
            oa = tuple(t.data_ptr() for t in po) + (0, k12.data_ptr())
            ia = tuple(t.data_ptr() for t in pi) + (1,)
            ap = (xo.data_ptr(), gg.data_ptr(), n, C) + oa[:4] + (0, k12.data_ptr(), dy.data_ptr(), st)
            nbd = lib.dk_dwconv_dgrad_workspace_bytes(C, 3, 3)
            dga = (dy.data_ptr(), B, H, H, C, w.data_ptr(), 3, 3, 1, 1, dx.data_ptr(), H, H, workspace.get(nbd), nbd,
                   0, xin.data_ptr()) + ia + (part.data_ptr(), st)
            nbw = lib.dk_dwconv_wgrad_workspace_bytes(B, H, H, C, 3, 3)
            wga = (dy.data_ptr(), xin.data_ptr(), B, H, H, C, 3, 3, 1, 1, H, H, 0, 0.0, dw.data_ptr(),
                   workspace.get(nbw), nbw) + ia + (st,)

            def unfused():
                lib.dk_bn_bwd_apply_f32(*ap)
                lib.dk_dwconv_dgrad_ex_f32(*dga)
                lib.dk_dwconv_wgrad_bnx_f32(*wga)
            nbf = lib.dk_dwconv_bwd_bnbwd_workspace_bytes(B, H, H, C, 3, 3)
            fa = (gg.data_ptr(), xo.data_ptr(), B, H, H, C) + oa + (xin.data_ptr(), w.data_ptr(), 3, 3, 1, 0.0,
                                                                  dw.data_ptr(), dx.data_ptr(), 0) + ia + (
                part.data_ptr(), workspace.get(nbf), nbf, st)
            report(name + " bwd unfused", timeit(unfused), "dk_dwconv_bwd_bnbwd_f32", fa)
            report(name + " bwd fused", timeit(lambda: lib.dk_dwconv_bwd_bnbwd_f32(*fa)), "dk_dwconv_bwd_bnbwd_f32", fa)
            del gg, xo, xin, dy, dx
    if "bn" in only:
        for name, H, C in BN:
            P = B * H * H
            x, dy = rnd(P * C), rnd(P * C)
            y = torch.empty(P * C, device="cuda")
            p = bnp(C)
            mean, std, invstd, rm, rs = [torch.empty(C, device="cuda") for _ in range(5)]
            nb = lib.dk_bn_stats_workspace_bytes(P, C)
            sa = (x.data_ptr(), P, C, 1e-5, 0.95, 1, mean.data_ptr(), std.data_ptr(), invstd.data_ptr(), rm.data_ptr(),
                  rs.data_ptr(), workspace.get(nb), nb, st)
            report(name + " stats", timeit(lambda: lib.dk_bn_stats_f32(*sa)), "dk_bn_stats_f32", sa)
            aa = (x.data_ptr(), P * C, C, p[0].data_ptr(), p[1].data_ptr(), p[2].data_ptr(), p[3].data_ptr(), 1,
                  y.data_ptr(), 0, st)
            report(name + " apply", timeit(lambda: lib.dk_bn_apply_f32(*aa)), "dk_bn_apply_f32", aa)
            dg, db = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
            nb = lib.dk_bn_bwd_workspace_bytes(P, C)
            ba = (x.data_ptr(), dy.data_ptr(), P, C, p[0].data_ptr(), p[1].data_ptr(), p[2].data_ptr(),
                  p[3].data_ptr(), 1, dg.data_ptr(), db.data_ptr(), y.data_ptr(), workspace.get(nb), nb, st)
            report(name + " bwd", timeit(lambda: lib.dk_bn_bwd_f32(*ba)), "dk_bn_bwd_f32", ba)
            del x, dy, y
    if "pw" in only:
        for name, H, C, K, s in PW:
            OH = -(-H // s)
            x, dy = rnd(B * H * H * C), rnd(B * OH * OH * K)
            y = torch.empty(B * OH * OH * K, device="cuda")
            w = rnd(K * C) * 0.1
            p = bnp(C)
            fa = (x.data_ptr(), B, H, H, C, w.data_ptr(), K, s, 0, y.data_ptr(), OH, OH, st)
            report(name + " fwd", timeit(lambda: lib.dk_pwconv_fwd_f32(*fa)), "dk_pwconv_fwd_f32", fa)
            fb = fa[:-1] + tuple(t.data_ptr() for t in p) + (1, st)
            report(name + " fwd bnx", timeit(lambda: lib.dk_pwconv_fwd_bnx_f32(*fb)), "dk_pwconv_fwd_bnx_f32", fb)
            rows = lib.dk_pwconv_fwd_stats_rows(B, OH, OH, K, C)
            part = torch.empty(rows * 2 * K, dtype=torch.float64, device="cuda")
            fe = fa[:-1] + (0, 0, 0, 0, 0, part.data_ptr(), st)
            report(name + " fwd stats", timeit(lambda: lib.dk_pwconv_fwd_ex_f32(*fe)), "dk_pwconv_fwd_ex_f32", fe)
            fe2 = fa[:-1] + tuple(t.data_ptr() for t in p) + (1, part.data_ptr(), st)
            report(name + " fwd bnx+stats", timeit(lambda: lib.dk_pwconv_fwd_ex_f32(*fe2)), "dk_pwconv_fwd_ex_f32",
                   fe2)
            dw = torch.empty(K * C, device="cuda")
            nb = lib.dk_pwconv_wgrad_workspace_bytes(B, OH, OH, K, C)
            wa = (dy.data_ptr(), x.data_ptr(), B, H, H, C, K, s, OH, OH, 0, 0.0, dw.data_ptr(), workspace.get(nb), nb,
                  st)
            report(name + " wgrad", timeit(lambda: lib.dk_pwconv_wgrad_f32(*wa)), "dk_pwconv_wgrad_f32", wa)
            wb = wa[:-1] + tuple(t.data_ptr() for t in p) + (1, st)
            report(name + " wgrad bnx", timeit(lambda: lib.dk_pwconv_wgrad_bnx_f32(*wb)), "dk_pwconv_wgrad_bnx_f32",
                   wb)
            dx = torch.empty(B * OH * s * OH * s * C, device="cuda")
            ga = (dy.data_ptr(), B, OH, OH, K, w.data_ptr(), C, s, dx.data_ptr(), st)
            report(name + " dgrad", timeit(lambda: lib.dk_pwconv_dgrad_f32(*ga)), "dk_pwconv_dgrad_f32", ga)
            del x, dy, y, dx


if __name__ == "__main__":
    main()
