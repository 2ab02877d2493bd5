"""Sweep the GEMM tile configurations over every GEMM shape of the ResNet-18-depsep step
(bs=256) and BASELINE config 2; report per-call time, GB/s and TFLOP/s per config.

    python scripts/gemm_tune.py [--out gpurun_out/gemm_tune.json] [--batch 256]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, workspace  # noqa: E402
from dorknet_amd import perfmodel  # noqa: E402


def shapes(B):
    pw = [  # name, H (input), C, K, stride
        ("pw0", 112, 64, 64, 2), ("res1_pw", 56, 64, 64, 1), ("res3_dw1_pw", 28, 64, 128, 1),
        ("res3_skip", 56, 64, 128, 2), ("res3_dw2_pw", 28, 128, 128, 1), ("res5_dw1_pw", 14, 128, 256, 1),
        ("res5_skip", 28, 128, 256, 2), ("res5_dw2_pw", 14, 256, 256, 1), ("res7_dw1_pw", 7, 256, 512, 1),
        ("res7_skip", 14, 256, 512, 2), ("res7_dw2_pw", 7, 512, 512, 1)]
    out = [dict(kind="pw", name=n, N=B, H=h, C=c, K=k, st=s) for n, h, c, k, s in pw]
    out.append(dict(kind="conv", name="conv0", N=B, H=225, C=4, Creal=3, K=64, R=5, st=2, pad=1))
    out.append(dict(kind="conv", name="cfg2", N=B, H=56, C=64, Creal=64, K=64, R=3, st=1, pad=1))
    return out


def timeit(fn, reps=5):
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
    ap.add_argument("--out", default="gpurun_out/gemm_tune.json")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--fused-only", action="store_true", help="pw shapes: only the fused (ex / bnx) variants")
    ap.add_argument("--only", default=None, help="comma-separated shape names (e.g. conv0,res1_pw)")
    args = ap.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    nrow = lib.dk_debug_set_gemm_config(0, -1)
    nsplit = lib.dk_debug_set_gemm_config(1, -1)
    results = []
    g = torch.Generator(device="cuda").manual_seed(0)
    for sh in shapes(args.batch):
        if args.only and sh["name"] not in args.only.split(","):
            continue
        N, H, C, K = sh["N"], sh["H"], sh["C"], sh["K"]
        if sh["kind"] == "pw":
            s = sh["st"]
            OH = -(-H // s)
            x = torch.randn(N * H * H * C, device="cuda", generator=g)
            w = torch.randn(K * C, device="cuda", generator=g) * 0.1
            y = torch.empty(N * OH * OH * K, device="cuda")
            dy = torch.randn(N * OH * OH * K, device="cuda", generator=g)
            dx = torch.empty(N * OH * s * OH * s * C, device="cuda")
            dw = torch.empty(K * C, device="cuda")
            fwd = lambda: lib.dk_pwconv_fwd_f32(x.data_ptr(), N, H, H, C, w.data_ptr(), K, s, 0, y.data_ptr(), OH, OH, st)
            dgr = lambda: lib.dk_pwconv_dgrad_f32(dy.data_ptr(), N, OH, OH, K, w.data_ptr(), C, s, dx.data_ptr(), st)

            def wgr():
                nb = lib.dk_pwconv_wgrad_workspace_bytes(N, OH, OH, K, C)
                lib.dk_pwconv_wgrad_f32(dy.data_ptr(), x.data_ptr(), N, H, H, C, K, s, OH, OH, 0, 0.0, dw.data_ptr(),
                                        workspace.get(nb), nb, st)
            # the fused variants the training step runs: BN on load + output statistics (fwd),
            # BN-backward partials of the input BN (dgrad), BN on load (wgrad)
            bnp = [torch.randn(C, device="cuda", generator=g), torch.rand(C, device="cuda", generator=g) + 0.5,
                   torch.randn(C, device="cuda", generator=g), torch.randn(C, device="cuda", generator=g)]
            bna = tuple(t.data_ptr() for t in bnp) + (1,)
            part = torch.empty(max(lib.dk_pwconv_fwd_stats_rows(N, OH, OH, K, C) * 2 * K,
                                   lib.dk_pwconv_dgrad_stats_rows(N, OH, OH, K, C) * 2 * C), dtype=torch.float64,
                               device="cuda")
            fwdx = lambda: lib.dk_pwconv_fwd_ex_f32(x.data_ptr(), N, H, H, C, w.data_ptr(), K, s, 0, y.data_ptr(), OH,
                                                    OH, *bna, part.data_ptr(), st)

            def dgrx():
                if s != 1:
                    raise RuntimeError("strided: not fused")
                lib.dk_pwconv_dgrad_ex_f32(dy.data_ptr(), N, OH, OH, K, w.data_ptr(), C, s, dx.data_ptr(), 0,
                                           x.data_ptr(), *bna, part.data_ptr(), st)

            def wgrx():
                nb = lib.dk_pwconv_wgrad_workspace_bytes(N, OH, OH, K, C)
                lib.dk_pwconv_wgrad_bnx_f32(dy.data_ptr(), x.data_ptr(), N, H, H, C, K, s, OH, OH, 0, 0.0,
                                            dw.data_ptr(), workspace.get(nb), nb, *bna, st)
            work = {"fwd": perfmodel.work("dk_pwconv_fwd_f32", (0, N, H, H, C, 0, K, s, 0, 0, OH, OH, 0)),
                    "dgrad": perfmodel.work("dk_pwconv_dgrad_f32", (0, N, OH, OH, K, 0, C, s, 0, 0)),
                    "wgrad": perfmodel.work("dk_pwconv_wgrad_f32", (0, 0, N, H, H, C, K, s, OH, OH, 0, 0, 0, 0, 0, 0))}
            work["fwdx"], work["dgrx"], work["wgrx"] = work["fwd"], work["dgrad"], work["wgrad"]
            extra = [("fwdx", fwdx, 0), ("dgrx", dgrx, 0), ("wgrx", wgrx, 1)]
            if s == 1:
                # dgrad with the following BN's backward applied on load (+ dy write-through),
                # vs. the separate apply pass it replaces
                ox = torch.randn(N * OH * OH * K, device="cuda", generator=g)
                dyo = torch.empty_like(ox)
                obp = [torch.randn(K, device="cuda", generator=g), torch.rand(K, device="cuda", generator=g) + 0.5,
                       torch.randn(K, device="cuda", generator=g), torch.randn(K, device="cuda", generator=g)]
                k12 = torch.randn(2 * K, device="cuda", generator=g) * 0.1
                oba = tuple(t.data_ptr() for t in obp) + (0, k12.data_ptr())
                dgrb = lambda: lib.dk_pwconv_dgrad_bnbwd_f32(dy.data_ptr(), ox.data_ptr(), N, OH, OH, K, *oba,
                                                             dyo.data_ptr(), w.data_ptr(), C, dx.data_ptr(), 0,
                                                             x.data_ptr(), *bna, part.data_ptr(), st)
                bapp = lambda: lib.dk_bn_bwd_apply_f32(ox.data_ptr(), dy.data_ptr(), N * OH * OH * K, K, *oba[:5],
                                                       k12.data_ptr(), dyo.data_ptr(), st)
                work["dgrb"] = perfmodel.work("dk_pwconv_dgrad_bnbwd_f32", (0, 0, N, OH, OH, K) + (0,) * 6 + (
                    1, 0, C, 0, 0, 1) + (0,) * 7)
                work["bapp"] = perfmodel.work("dk_bn_bwd_apply_f32", (0, 0, N * OH * OH * K, K))
                extra += [("dgrb", dgrb, 0), ("bapp", bapp, 2)]
        else:
            R, s, pd, Cr = sh["R"], sh["st"], sh["pad"], sh["Creal"]
            OH = int((H + 2 * pd - R) / s + 1)
            x = torch.randn(N * H * H * C, device="cuda", generator=g)
            wk = torch.randn(K * R * R * C, device="cuda", generator=g) * 0.1
            wc = torch.randn(C * R * R * K, device="cuda", generator=g) * 0.1
            w = torch.randn(K * Cr * R * R, device="cuda", generator=g) * 0.1
            y = torch.empty(N * OH * OH * K, device="cuda")
            dy = torch.randn(N * OH * OH * K, device="cuda", generator=g)
            dx = torch.empty(N * H * H * C, device="cuda")
            dw = torch.empty(K * Cr * R * R, device="cuda")
            fwd = lambda: lib.dk_conv2d_fwd_f32(x.data_ptr(), N, H, H, C, wk.data_ptr(), K, R, R, s, pd, 0, y.data_ptr(),
                                                OH, OH, st)
            if s == 1:
                dgr = lambda: lib.dk_conv2d_dgrad_f32(dy.data_ptr(), N, OH, OH, K, wc.data_ptr(), C, R, R, pd,
                                                      dx.data_ptr(), H, H, st)
            else:
                def dgr():
                    nb = lib.dk_conv2d_dgrad_phase_workspace_bytes(K, Cr, R, R, s)
                    lib.dk_conv2d_dgrad_phase_f32(dy.data_ptr(), N, OH, OH, K, K, w.data_ptr(), Cr, R, R, s, pd,
                                                    dx.data_ptr(), H, H, workspace.get(nb), nb, st)

            def wgr():
                nb = lib.dk_conv2d_wgrad_workspace_bytes(N, OH, OH, K, C, R, R)
                lib.dk_conv2d_wgrad_f32(dy.data_ptr(), x.data_ptr(), N, H, H, C, Cr, K, R, R, s, pd, OH, OH, 0, 0.0,
                                        dw.data_ptr(), workspace.get(nb), nb, st)
            a = (0, N, H, H, C, 0, K, R, R, s, pd, 0, 0, OH, OH, 0)
            work = {"fwd": perfmodel.work("dk_conv2d_fwd_f32", a), "dgrad": perfmodel.work("dk_conv2d_fwd_f32", a),
                    "wgrad": perfmodel.work("dk_conv2d_fwd_f32", a)}
            extra = ()
        ops = [("fwd", fwd, 0), ("dgrad", dgr, 0), ("wgrad", wgr, 1)] + list(extra)
        if args.fused_only:
            ops = list(extra) or ops
        for op, fn, kind in ops:
            n = nrow if kind == 0 else (nsplit if kind == 1 else 0)
            row = {"shape": sh["name"], "op": op, "cfg": {}}
            for cfg in [-1] + list(range(n)):
                lib.dk_debug_set_gemm_config(min(kind, 1), cfg)
                try:
                    us = timeit(fn)
                except Exception as e:  # config not applicable
                    row["cfg"][str(cfg)] = str(e)[:60]
                    continue
                f, b = work[op]
                row["cfg"][str(cfg)] = {"us": round(us, 1), "GBs": round(b / us / 1e3, 1), "TFs": round(f / us / 1e6, 1)}
            lib.dk_debug_set_gemm_config(min(kind, 1), -1)
            if not isinstance(row["cfg"].get("-1"), dict):
                continue
            best = min(((v["us"], k) for k, v in row["cfg"].items() if isinstance(v, dict) and k != "-1"),
                       default=(row["cfg"]["-1"]["us"], "-1"))
            row["best"] = best[1]
            results.append(row)
            d = row["cfg"]["-1"]
            print("{:12s} {:5s} default {:8.1f} us ({:6.0f} GB/s {:5.1f} TF/s) | best cfg {} {:8.1f} us".format(
                sh["name"], op, d["us"], d["GBs"], d["TFs"], best[1], best[0]), flush=True)
        del x, y, dy, dx, dw
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
