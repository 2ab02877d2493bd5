"""Run a few GEMM shapes of the ResNet step repeatedly (for rocprofv3 --pmc counter passes).

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY ... --kernel-trace -f csv -d OUT -o p -- python scripts/gemm_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, workspace  # noqa: E402


def main(reps=10, B=256):
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(0)
    for H, C, K in ((56, 64, 64), (14, 256, 256)):
        x = torch.randn(B * H * H * C, device="cuda", generator=g)
        dy = torch.randn(B * H * H * K, device="cuda", generator=g)
        w = torch.randn(K * C, device="cuda", generator=g) * 0.1
        y = torch.empty(B * H * H * K, device="cuda")
        dx = torch.empty(B * H * H * C, device="cuda")
        dw = torch.empty(K * C, device="cuda")
        nb = lib.dk_pwconv_wgrad_workspace_bytes(B, H, H, K, C)
        ws = workspace.get(nb)
        # the fused variants the training step runs: BN on load + output statistics (fwd), BN
        # backward on load + dy write-through + input-BN partials (dgrad), BN on load (wgrad)
        pi = [torch.randn(C, device="cuda", generator=g), torch.rand(C, device="cuda", generator=g) + 0.5,
              torch.randn(C, device="cuda", generator=g), torch.randn(C, device="cuda", generator=g)]
        po = [torch.randn(K, device="cuda", generator=g), torch.rand(K, device="cuda", generator=g) + 0.5,
              torch.randn(K, device="cuda", generator=g), torch.randn(K, device="cuda", generator=g)]
        k12 = torch.randn(2 * K, device="cuda", generator=g) * 0.1
        xo = torch.randn(B * H * H * K, device="cuda", generator=g)
        dyo = torch.empty_like(xo)
        ia = tuple(t.data_ptr() for t in pi) + (1,)
        oa = tuple(t.data_ptr() for t in po) + (1, k12.data_ptr())
        part = torch.empty(max(lib.dk_pwconv_fwd_stats_rows(B, H, H, K, C) * 2 * K,
                               lib.dk_pwconv_dgrad_stats_rows(B, H, H, K, C) * 2 * C), dtype=torch.float64,
                           device="cuda")
        for _ in range(reps):
            lib.dk_pwconv_fwd_f32(x.data_ptr(), B, H, H, C, w.data_ptr(), K, 1, 0, y.data_ptr(), H, H, st)
            lib.dk_pwconv_dgrad_f32(dy.data_ptr(), B, H, H, K, w.data_ptr(), C, 1, dx.data_ptr(), st)
            lib.dk_pwconv_wgrad_f32(dy.data_ptr(), x.data_ptr(), B, H, H, C, K, 1, H, H, 0, 0.0, dw.data_ptr(), ws, nb,
                                    st)
            lib.dk_pwconv_fwd_ex_f32(x.data_ptr(), B, H, H, C, w.data_ptr(), K, 1, 0, y.data_ptr(), H, H, *ia,
                                     part.data_ptr(), st)
            lib.dk_pwconv_dgrad_bnbwd_f32(dy.data_ptr(), xo.data_ptr(), B, H, H, K, *oa, dyo.data_ptr(), w.data_ptr(),
                                          C, dx.data_ptr(), 0, x.data_ptr(), *ia, part.data_ptr(), st)
            lib.dk_pwconv_wgrad_bnx_f32(dy.data_ptr(), x.data_ptr(), B, H, H, C, K, 1, H, H, 0, 0.0, dw.data_ptr(),
                                        ws, nb, *ia, st)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
