"""Per-shape timing of the fused pointwise backward (dk_pwconv_bwd_bnbwd_f32) against the
unfused pair it replaces (dk_pwconv_dgrad_bnbwd_f32 + dk_pwconv_wgrad_bnx_f32), bs=256.

    DORKNET_PWF_PREFETCH=0|1 python scripts/pwf_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, workspace  # noqa: E402
from dorknet_amd import perfmodel  # noqa: E402
from scripts.kbench import timeit  # noqa: E402


def main(B=256):
    st = torch.cuda.current_stream().cuda_stream
    g0 = torch.Generator(device="cuda").manual_seed(0)
    for name, H, K, C in (("res1_pw", 56, 64, 64), ("res3_dw1_pw", 28, 128, 64), ("res3_dw2_pw", 28, 128, 128)):
        P = B * H * H
        r = lambda n: torch.randn(n, device="cuda", generator=g0)
        g, xo, x, res = r(P * K), r(P * K), r(P * C), r(P * C)
        w = r(K * C) * 0.1
        pp = lambda n: [r(n), torch.rand(n, device="cuda", generator=g0) + 0.5, r(n), r(n)]
        po, pi = pp(K), pp(C)
        k12 = r(2 * K) * 0.1
        dx, dy, dw = torch.empty(P * C, device="cuda"), torch.empty(P * K, device="cuda"), torch.empty(K * C, device="cuda")
        rows0 = lib.dk_pwconv_dgrad_bnbwd_stats_rows(B, H, H, K, C)
        part0 = torch.empty(rows0 * 2 * C, dtype=torch.float64, device="cuda")
        oa = tuple(t.data_ptr() for t in po) + (1, k12.data_ptr())
        ia = tuple(t.data_ptr() for t in pi) + (1,)

        def unfused():
            lib.dk_pwconv_dgrad_bnbwd_f32(g.data_ptr(), xo.data_ptr(), B, H, H, K, *oa, dy.data_ptr(), w.data_ptr(), C,
                                          dx.data_ptr(), res.data_ptr(), x.data_ptr(), *ia, part0.data_ptr(), st)
            nb = lib.dk_pwconv_wgrad_workspace_bytes(B, H, H, K, C)
            lib.dk_pwconv_wgrad_bnx_f32(dy.data_ptr(), x.data_ptr(), B, H, H, C, K, 1, H, H, w.data_ptr(), 1e-4,
                                        dw.data_ptr(), workspace.get(nb), nb, *ia, st)
        rows1 = lib.dk_pwconv_bwd_fused_rows(B, H, H, K, C)
        part1 = torch.empty(rows1 * 2 * C, dtype=torch.float64, device="cuda")

        def fused():
            nb = lib.dk_pwconv_bwd_fused_workspace_bytes(B, H, H, K, C)
            lib.dk_pwconv_bwd_bnbwd_f32(g.data_ptr(), xo.data_ptr(), B, H, H, K, *oa, w.data_ptr(), C, 1e-4,
                                        dw.data_ptr(), dx.data_ptr(), res.data_ptr(), x.data_ptr(), *ia,
                                        part1.data_ptr(), workspace.get(nb), nb, st)
        tu, tf = timeit(unfused), timeit(fused)
        f, b = perfmodel.work("dk_pwconv_bwd_bnbwd_f32", (0, 0, B, H, H, K) + (0,) * 6 + (0, C, 0.0, 0, 0, 1, 1) +
                              (0,) * 9)
        print(f"{name:12s} K={K:3d} C={C:3d} rows={rows1:5d}  unfused {tu:7.1f} us  fused {tf:7.1f} us  "
              f"({b / tf / 1e3:5.0f} GB/s, {f / tf / 1e6:5.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
