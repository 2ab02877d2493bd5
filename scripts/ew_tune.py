"""Sweep dk_bn_bwd_apply_f32 launch variants (dk_debug_set_ew_variant) over the BatchNorm
shapes of the ResNet-18-depsep step (bs=256).  python scripts/ew_tune.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib  # noqa: E402

SHAPES = [("conv0_bn", 112, 64), ("res1_bn", 56, 64), ("res3_bn", 28, 128), ("res5_bn", 14, 256), ("res7_bn", 7, 512)]


def timeit(fn, reps=9):
    fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return 1e3 * t[len(t) // 2]


def main(B=256):
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(0)
    nvar = lib.dk_debug_set_ew_variant(-1)
    for name, H, C in SHAPES:
        P = B * H * H
        x, dy, dx = torch.randn(P * C, device="cuda", generator=g), torch.randn(P * C, device="cuda", generator=g), \
            torch.empty(P * C, device="cuda")
        prm = [torch.randn(C, device="cuda", generator=g) for _ in range(4)] + [torch.randn(2 * C, device="cuda")]
        args = (x.data_ptr(), dy.data_ptr(), P * C, C) + tuple(t.data_ptr() for t in prm[:4]) + (1, prm[4].data_ptr(),
                                                                                             dx.data_ptr(), st)
        res = []
        for v in [-1] + list(range(nvar)):  # -1 = the built-in default
            lib.dk_debug_set_ew_variant(v)
            us = timeit(lambda: lib.dk_bn_bwd_apply_f32(*args))
            res.append((us, v))
        lib.dk_debug_set_ew_variant(-1)
        base = res[0][0]
        best = sorted(res[1:])[:4]
        gbs = lambda us: 12 * P * C / us / 1e3  # noqa: E731
        print(f"{name:9s} default {base:7.1f} us {gbs(base):6.0f} GB/s | best " +
              "  ".join(f"v{v}:{us:.1f}us/{gbs(us):.0f}" for us, v in best), flush=True)
        del x, dy, dx


if __name__ == "__main__":
    main()
