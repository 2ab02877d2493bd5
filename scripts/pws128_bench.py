"""A/B timing of dk_pwconv_fwd_ex_f32 (BN + ReLU on load, output statistics) on the streaming
kernel vs the tiled engine at the K = C = 64 / 128 shapes of ResNet-18-depsep, batch 256.

    python scripts/pws128_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib  # noqa: E402
from scripts.pws_bench import timeit  # noqa: E402


def main(B=256):
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(0)
    for KC, H in ((64, 56), (128, 28)):
        M = B * H * H
        x = torch.randn(M * KC, device="cuda", generator=g)
        w = torch.randn(KC * KC, device="cuda", generator=g) * 0.1
        pm = [torch.rand(KC, device="cuda", generator=g) + 0.5 for _ in range(4)]
        y = torch.empty(M * KC, device="cuda")
        out = []
        for mode in (1, 0):
            lib.dk_debug_set_gemm_config(3, mode)
            try:
                rows = lib.dk_pwconv_fwd_stats_rows(B, H, H, KC, KC)
                part = torch.empty(rows * 2 * KC, dtype=torch.float64, device="cuda")
                f = lambda: lib.dk_pwconv_fwd_ex_f32(x.data_ptr(), B, H, H, KC, w.data_ptr(), KC, 1, 0, y.data_ptr(),
                                                     H, H, *(p.data_ptr() for p in pm), 1, part.data_ptr(), st)
                out.append(timeit(f))
            finally:
                lib.dk_debug_set_gemm_config(3, -1)
        fl, by = 2.0 * M * KC * KC, 2.0 * M * KC * 4
        print(f"K=C={KC:3d} {H}x{H}: stream {out[0]:7.1f} us ({fl / out[0] / 1e6:5.1f} TF/s, {by / out[0] / 1e3:5.0f} GB/s)"
              f"  tiled {out[1]:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
