"""The fused stride-1 depthwise backward (dk_dwconv_bwd_bnbwd_bf16 / _f32) at the depthwise-separable
stack's shapes: median of 15 calls (HIP events on the launch stream), HBM bytes per call (g, the BN
input, x read; dx written) and TB/s, per columns-per-thread setting (knob 21) for bf16.
    python scripts/dwb_bench.py [--batch 512] [--f32] [--hw 56] [--blocks 768,256,1536]
(--blocks: the fused backward's block target, knob 7, swept per shape)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, stream_handle  # noqa: E402

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
    f32 = "--f32" in sys.argv
    B = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else (256 if f32 else 512)
    dt = torch.float32 if f32 else torch.bfloat16
    esz = 4 if f32 else 2
    torch.manual_seed(0)
    only = int(sys.argv[sys.argv.index("--hw") + 1]) if "--hw" in sys.argv else None
    for HW, C in SHAPES:
        if only is not None and HW != only:
            continue
        n = B * HW * HW * C
        g, x1, x = (torch.randn(n, device="cuda").to(dt) for _ in range(3))
        dx = torch.empty(n, device="cuda", dtype=dt)
        p = [torch.randn(C, device="cuda"), torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda"),
             torch.randn(C, device="cuda")]
        k12 = torch.randn(2 * C, device="cuda") * 0.1
        w = torch.randn(C * 9, device="cuda") * 0.3
        dw = torch.empty(C * 9, device="cuda")
        line = f"{B}x{HW}x{HW}x{C} {'f32' if f32 else 'bf16'}:"
        blocks = [int(v) for v in sys.argv[sys.argv.index("--blocks") + 1].split(",")] if "--blocks" in sys.argv else [-1]
        for cols, nt, bt in [(c, 256, b) for c in (1, 2) for b in blocks]:
            lib.dk_debug_set_gemm_config(21, cols)
            lib.dk_debug_set_gemm_config(7, bt)
            rows_fn = lib.dk_dwconv_bwd_bnbwd_stats_rows if f32 else lib.dk_dwconv_bwd_bnbwd_bf16_stats_rows
            ws_fn = lib.dk_dwconv_bwd_bnbwd_workspace_bytes if f32 else lib.dk_dwconv_bwd_bnbwd_bf16_workspace_bytes
            rows = rows_fn(B, HW, HW, C)
            nb = ws_fn(B, HW, HW, C, 3, 3)
            ws = torch.empty(nb // 4 + 64, device="cuda")
            part = torch.empty(rows * 2 * C, dtype=torch.float64, device="cuda")
            fn = lib.dk_dwconv_bwd_bnbwd_f32 if f32 else lib.dk_dwconv_bwd_bnbwd_bf16

            def call():
                fn(g.data_ptr(), x1.data_ptr(), B, HW, HW, C, *(t.data_ptr() for t in p), 0, k12.data_ptr(),
                   x.data_ptr(), w.data_ptr(), 3, 3, 1, 0.0, dw.data_ptr(), dx.data_ptr(), 0,
                   *(t.data_ptr() for t in p), 1, part.data_ptr(), ws.data_ptr(), nb, stream_handle())
            t = timeit(call)
            byt = 4 * n * esz
            line += f"  cols {cols}{'' if bt < 0 else ' blk %d' % bt}: {t:7.1f} us {byt / t / 1e6:5.2f} TB/s ({rows} strips)"
        lib.dk_debug_set_gemm_config(21, -1)
        lib.dk_debug_set_gemm_config(7, -1)
        print(line, flush=True)


if __name__ == "__main__":
    main()
