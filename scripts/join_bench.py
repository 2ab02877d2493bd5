"""The residual join formed by the next depthwise forward (dk_dwconv_fwd_join_f32) against the join pass
(dk_bn_add_f32) + dk_dwconv_fwd_ex_f32, at ResNet-18-depsep's identity-block shapes (batch 256), with
the output statistics as in the network.  Median of 15 calls (HIP events), and HBM bytes per call.
    python scripts/join_bench.py [--stride 2]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, stream_handle  # noqa: E402

B = 256
SHAPES = [(56, 64), (28, 128), (14, 256), (7, 512)]


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
    stride = int(sys.argv[sys.argv.index("--stride") + 1]) if "--stride" in sys.argv else 1
    st = stream_handle()
    torch.manual_seed(0)
    for HW, C in SHAPES:
        if stride == 2:
            HW *= 2
            C //= 2
        n = B * HW * HW * C
        a, b = torch.randn(n, device="cuda"), torch.randn(n, device="cuda")
        pa = [torch.randn(C, device="cuda"), torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda"),
              torch.randn(C, device="cuda")]
        w = torch.randn(C * 9, device="cuda") * 0.3
        OH = (HW - 1) // stride + 1
        y = torch.empty(n, device="cuda")
        mask = torch.empty(n, dtype=torch.uint8, device="cuda")
        o = torch.empty(B * OH * OH * C, device="cuda")
        rows = lib.dk_dwconv_fwd_stats_rows(B, OH, OH, C, stride)
        part = torch.empty(rows * 2 * C, dtype=torch.float64, device="cuda")
        aa = (*(t.data_ptr() for t in pa), 0)

        def sep():
            lib.dk_bn_add_f32(a.data_ptr(), *aa, b.data_ptr(), 0, 0, 0, 0, 0, n, C, 1, y.data_ptr(), mask.data_ptr(), st)
            lib.dk_dwconv_fwd_ex_f32(y.data_ptr(), B, HW, HW, C, w.data_ptr(), 3, 3, stride, 1, 0, o.data_ptr(), OH, OH,
                                     0, 0, 0, 0, 0, part.data_ptr(), st)

        def add_only():
            lib.dk_bn_add_f32(a.data_ptr(), *aa, b.data_ptr(), 0, 0, 0, 0, 0, n, C, 1, y.data_ptr(), mask.data_ptr(), st)

        def fused(m=True):
            lib.dk_dwconv_fwd_join_f32(a.data_ptr(), *aa, b.data_ptr(), 0, 0, 0, 0, 0, y.data_ptr(),
                                       mask.data_ptr() if m else 0, B, HW, HW, C, w.data_ptr(), stride, 0, o.data_ptr(),
                                       OH, OH, part.data_ptr(), st)
        ts, ta, tf, tfm = timeit(sep), timeit(add_only), timeit(fused), timeit(lambda: fused(False))
        byt_sep = 4 * n * 3 + n + 4 * (n + B * OH * OH * C)
        byt_f = 4 * n * 3 + n + 4 * B * OH * OH * C
        print(f"{B}x{HW}x{HW}x{C} s{stride}: join pass + dw {ts:7.1f} us (join {ta:6.1f}, dw {ts - ta:6.1f}) "
              f"{byt_sep / ts / 1e6:5.2f} TB/s | fused {tf:7.1f} us {byt_f / tf / 1e6:5.2f} TB/s, "
              f"no mask {tfm:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
