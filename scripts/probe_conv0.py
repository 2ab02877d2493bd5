"""Time the stem's fused weight gradient (dk_conv2d_wgrad_bnbwd_f32) under every split-K tile
configuration (ResNet-18-depsep conv0 at batch 256).  python scripts/probe_conv0.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, stream_handle, workspace  # noqa: E402


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


def main():
    N, H, W, Cp, C, K, R, s, pad = 256, 225, 225, 4, 3, 64, 5, 2, 1
    OH = OW = (H + 2 * pad - R) // s + 1
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(N * H * W * Cp, device="cuda", generator=g)
    go = torch.randn(N * OH * OW * K, device="cuda", generator=g)
    xo = torch.randn(N * OH * OW * K, device="cuda", generator=g)
    p = [torch.randn(K, device="cuda", generator=g) for _ in range(4)]
    k12 = torch.randn(2 * K, device="cuda", generator=g)
    dw = torch.empty(K * C * R * R, device="cuda")
    st = stream_handle()
    nsplit = lib.dk_debug_set_gemm_config(1, -1)
    for cfg in [-1] + list(range(nsplit)):
        lib.dk_debug_set_gemm_config(1, cfg)
        nb = lib.dk_conv2d_wgrad_workspace_bytes(N, OH, OW, K, Cp, R, R)
        a = (go.data_ptr(), xo.data_ptr(), x.data_ptr(), N, H, W, Cp, C, K, R, R, s, pad, OH, OW,
             *(t.data_ptr() for t in p), 1, k12.data_ptr(), 0, 0.0, dw.data_ptr(), workspace.get(nb), nb,
             0, 0, 0, 0, 0, st)
        us = timeit(lambda: lib.dk_conv2d_wgrad_bnbwd_f32(*a))
        nbytes = 4 * (2 * N * OH * OW * K + N * H * W * Cp)
        print("cfg {:2d}: {:8.1f} us  {:6.0f} GB/s".format(cfg, us, nbytes / us / 1e3), flush=True)
    lib.dk_debug_set_gemm_config(1, -1)


if __name__ == "__main__":
    main()
