"""bf16 deep pointwise layers of config 5 (batch 512): the column-sliced streaming kernels
(pw_stream_bf16.hip, knob 10 on) against the tiled engine (knob 10 off), forward with BN on load +
statistics and the BN-backward-on-load dgrad with dy write-through and the input BN's partials;
median of 9 calls, HBM rate of the algorithmic bytes.
    python scripts/pwsh_deep_bench.py [--no-bn]    (--no-bn: forward without the input BN)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, stream_handle  # noqa: E402

BF16 = torch.bfloat16
B = 512
SHAPES = [(14, 128, 256), (14, 256, 256), (7, 256, 512), (7, 512, 512)]  # HW, C (in), K (out)


def timeit(fn, reps=9):
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
    st = stream_handle()

    def rnd(n, dt=torch.float32):
        return torch.randn(n, device="cuda").to(dt)

    for HW, C, K in SHAPES:
        M = B * HW * HW
        x, y = rnd(M * C, BF16), torch.empty(M * K, dtype=BF16, device="cuda")
        g, xo, dy, dx = rnd(M * K, BF16), rnd(M * K, BF16), torch.empty(M * K, dtype=BF16, device="cuda"), \
            torch.empty(M * C, dtype=BF16, device="cuda")
        w = rnd(K * C) * 0.05
        pi = [rnd(C), rnd(C).abs() + 0.5, rnd(C), rnd(C)]
        po = [rnd(K), rnd(K).abs() + 0.5, rnd(K), rnd(K)]
        k12 = rnd(2 * K) * 0.1
        line = []
        for deep in (0, 1):
            lib.dk_debug_set_gemm_config(10, deep)
            rows = lib.dk_pwconv_fwd_bf16_stats_rows(B, HW, HW, K, C)
            part = torch.empty(rows * 2 * K, dtype=torch.float64, device="cuda")
            bn = (0, 0, 0, 0, 0) if "--no-bn" in sys.argv else (*(t.data_ptr() for t in pi), 1)
            fa = (x.data_ptr(), B, HW, HW, C, w.data_ptr(), K, 1, 0, y.data_ptr(), HW, HW, *bn, part.data_ptr(), st)
            tf = timeit(lambda: lib.dk_pwconv_fwd_ex_bf16(*fa))
            rows = lib.dk_pwconv_dgrad_bnbwd_bf16_stats_rows(B, HW, HW, K, C)
            partd = torch.empty(rows * 2 * C, dtype=torch.float64, device="cuda")
            da = (g.data_ptr(), xo.data_ptr(), B, HW, HW, K, *(t.data_ptr() for t in po), 1, k12.data_ptr(),
                  dy.data_ptr(), w.data_ptr(), C, dx.data_ptr(), 0, x.data_ptr(), *(t.data_ptr() for t in pi), 1,
                  partd.data_ptr(), st)
            td = timeit(lambda: lib.dk_pwconv_dgrad_bnbwd_bf16(*da))
            fb = 2 * M * (C + K)
            db = 2 * M * (3 * K + 2 * C)
            line.append(f"{'deep ' if deep else 'tiled'}: fwd {tf:6.1f} us {fb / tf / 1e6:4.2f} TB/s, "
                        f"dgrad {td:6.1f} us {db / td / 1e6:4.2f} TB/s")
        lib.dk_debug_set_gemm_config(10, -1)
        print(f"{B}x{HW}x{HW} C={C} K={K} | " + " | ".join(line), flush=True)


if __name__ == "__main__":
    main()
