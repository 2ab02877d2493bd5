"""Stem kernels at BASELINE config 3's size (256 x 3 x 225 x 225 -> 64 x 112 x 112): the narrow-input
forward / BN-backward weight gradient (conv_narrow.hip) vs the implicit-GEMM pair on the NHWC4 copy.
Prints us per call (median of 10, HIP events).  python scripts/stem_bench.py [--only narrow|gemm]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, workspace  # noqa: E402


def timeit(f, n=10):
    for _ in range(3):
        f()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        f()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[n // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    N, C, H, W, K, R, S, st, pad = a.batch, 3, 225, 225, 64, 5, 5, 2, 1
    OH = OW = (H + 2 * pad - R) // st + 1
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda", generator=g)
    w = torch.randn(K, C, R, R, device="cuda", generator=g) * 0.1
    y = torch.empty(N, OH, OW, K, device="cuda")
    gy = torch.randn(N, OH, OW, K, device="cuda", generator=g)
    par = [torch.rand(K, device="cuda") + 0.5 for _ in range(4)]
    k12 = torch.randn(2 * K, device="cuda") * 0.01
    dw = torch.empty(K, C, R, R, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    P = N * OH * OW
    fl = 2.0 * P * K * C * R * S
    out = []
    if a.only in (None, "narrow"):
        nb = lib.dk_conv2d_wgrad_narrow_workspace_bytes(N, C, H, W, K, R, S, st, pad, OH, OW)
        ws = workspace.get(nb)
        f = lambda: lib.dk_conv2d_fwd_narrow_f32(x.data_ptr(), N, C, H, W, w.data_ptr(), K, R, S, st, pad, 0,
                                                 y.data_ptr(), OH, OW, 0, s)
        t = timeit(f)
        out.append(("narrow fwd", t, fl / t / 1e6, (N * C * H * W + P * K) * 4 / t / 1e3))
        f = lambda: lib.dk_conv2d_wgrad_bnbwd_narrow_f32(gy.data_ptr(), y.data_ptr(), x.data_ptr(), N, C, H, W, K, R,
                                                         S, st, pad, OH, OW, *(p.data_ptr() for p in par), 1,
                                                         k12.data_ptr(), 1, w.data_ptr(), 1e-4, dw.data_ptr(), ws, nb, s)
        t = timeit(f)
        out.append(("narrow wgrad_bnbwd", t, fl / t / 1e6, (N * C * H * W + 2 * P * K) * 4 / t / 1e3))
    if a.only in (None, "gemm"):
        Cp = 4
        x4 = torch.zeros(N, H, W, Cp, device="cuda")
        x4[..., :3] = x.permute(0, 2, 3, 1)
        wk = torch.zeros(K, R, S, Cp, device="cuda")
        wk[..., :3] = w.permute(0, 2, 3, 1)
        f = lambda: lib.dk_conv2d_fwd_f32(x4.data_ptr(), N, H, W, Cp, wk.data_ptr(), K, R, S, st, pad, 0, y.data_ptr(),
                                          OH, OW, s)
        t = timeit(f)
        out.append(("gemm fwd (NHWC4)", t, fl / t / 1e6, (N * C * H * W + P * K) * 4 / t / 1e3))
        nb = lib.dk_conv2d_wgrad_workspace_bytes(N, OH, OW, K, Cp, R, S)
        ws = workspace.get(nb)
        f = lambda: lib.dk_conv2d_wgrad_bnbwd_f32(gy.data_ptr(), y.data_ptr(), x4.data_ptr(), N, H, W, Cp, C, K, R, S,
                                                  st, pad, OH, OW, *(p.data_ptr() for p in par), 1, k12.data_ptr(),
                                                  w.data_ptr(), 1e-4, dw.data_ptr(), ws, nb, 0, 0, 0, 0, 0, s)
        t = timeit(f)
        out.append(("gemm wgrad_bnbwd (NHWC4)", t, fl / t / 1e6, (N * C * H * W + 2 * P * K) * 4 / t / 1e3))
    for name, t, tf, gbs in out:
        print(f"{name:28s} {t:8.1f} us  {tf:6.1f} TF/s  {gbs:6.0f} GB/s (algorithmic)", flush=True)


if __name__ == "__main__":
    main()
