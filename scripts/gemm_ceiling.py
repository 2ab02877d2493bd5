"""GEMM engine ceiling: TFLOP/s of the igemm_f32 engine per tile configuration on a large dense
problem and on the ResNet pointwise shapes at batch 256 and 2048 (small-problem effects vs the
inner loop).

    python scripts/gemm_ceiling.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib  # noqa: E402


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
    st = torch.cuda.current_stream().cuda_stream
    nrow = lib.dk_debug_set_gemm_config(0, -1)
    g = torch.Generator(device="cuda").manual_seed(0)
    cases = [("dense 16384x4096x4096", 16384, 4096, 4096)]
    for B in (256, 2048):
        for H, C in ((28, 128), (14, 256), (7, 512)):
            cases.append((f"pw {H}x{H}x{C} bs{B}", B * H * H, C, C))
    for name, M, IN, OUT in cases:
        x = torch.randn(M * IN, device="cuda", generator=g)
        w = torch.randn(IN * OUT, device="cuda", generator=g) * 0.05
        y = torch.empty(M * OUT, device="cuda")
        flops = 2.0 * M * IN * OUT
        res = []
        for cfg in [-1] + list(range(nrow)):
            lib.dk_debug_set_gemm_config(0, cfg)
            us = timeit(lambda: lib.dk_dense_fwd_f32(x.data_ptr(), M, IN, w.data_ptr(), OUT, 0, y.data_ptr(), st))
            res.append((cfg, us, flops / us / 1e6))
        lib.dk_debug_set_gemm_config(0, -1)
        best = max(res[1:], key=lambda r: r[2])
        print(f"{name:28s} default {res[0][1]:9.1f} us {res[0][2]:6.1f} TF/s | best cfg {best[0]:2d} "
              f"{best[1]:9.1f} us {best[2]:6.1f} TF/s | " + " ".join(f"{c}:{t:.0f}" for c, _, t in res[1:]),
              flush=True)


if __name__ == "__main__":
    main()
