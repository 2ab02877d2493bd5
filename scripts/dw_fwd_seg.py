"""Depthwise forward (BN on load + output statistics, the training forward) per shape against the
output rows per thread (knob 8): config 3's shapes (fp32, batch 256) or, with --bf16, config 5's
(bf16, batch 512); median of 9 timed calls, with the HBM rate of the algorithmic bytes.
    python scripts/dw_fwd_seg.py [--bf16]
DW_SEGS=-1,4,7 picks the segment lengths; DW_MODE = bn_stats (default) | bn | stats | plain drops the
BatchNorm on load and / or the statistics.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, stream_handle  # noqa: E402

HALF = "--bf16" in sys.argv
B = 512 if HALF else 256
DT = torch.bfloat16 if HALF else torch.float32
SHAPES = [(56, 64, 1), (56, 64, 2), (28, 128, 1), (28, 128, 2), (14, 256, 1), (14, 256, 2), (7, 512, 1)]
MODE = os.environ.get("DW_MODE", "bn_stats")
SEGS = [int(v) for v in os.environ.get("DW_SEGS", "-1,1,2,3,4,5,6,7,8,12,16").split(",")]


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
    fwd = lib.dk_dwconv_fwd_ex_bf16 if HALF else lib.dk_dwconv_fwd_ex_f32
    for H, C, stride in SHAPES:
        OH = (H + 2 - 3) // stride + 1
        x = torch.randn(B * H * H * C, device="cuda").to(DT)
        y = torch.empty(B * OH * OH * C, device="cuda", dtype=DT)
        w = torch.randn(C * 9, device="cuda") * 0.2
        p = [torch.randn(C, device="cuda"), torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda"),
             torch.randn(C, device="cuda")]
        nbytes = (x.numel() + y.numel()) * x.element_size()
        line = []
        for seg in SEGS:
            lib.dk_debug_set_gemm_config(8, seg)
            rows = lib.dk_dwconv_fwd_stats_rows(B, OH, OH, C, stride)
            part = torch.empty(rows * 2 * C, dtype=torch.float64, device="cuda")
            bn = (*(t.data_ptr() for t in p), 1) if "bn" in MODE else (0, 0, 0, 0, 0)
            args = (x.data_ptr(), B, H, H, C, w.data_ptr(), 3, 3, stride, 1, 0, y.data_ptr(), OH, OH,
                    *bn, part.data_ptr() if "stats" in MODE else 0, st)
            t = timeit(lambda: fwd(*args))
            line.append(f"{seg:3d}:{t:6.1f}us/{nbytes / t / 1e6:4.2f}TB/s")
        lib.dk_debug_set_gemm_config(8, -1)
        print(f"{MODE} {B}x{H}x{H}x{C} s{stride}  " + "  ".join(line), flush=True)


if __name__ == "__main__":
    main()
