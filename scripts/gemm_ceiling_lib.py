"""Library ceiling for the deep pointwise GEMM shapes of the ResNet-18-depsep step (fp32): torch.mm
(hipBLASLt / rocBLAS) on the same M x N x K as the 14x14 and 7x7 layers' forward, next to
dk_pwconv_fwd_f32 (plain, no BN on load) on the same shape.  TF/s and fraction of the 157.3
TF/s fp32 MFMA peak.  python scripts/gemm_ceiling_lib.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    st = torch.cuda.current_stream().cuda_stream
    for (hw, C, K) in [(14, 256, 256), (7, 512, 512), (28, 128, 128), (14, 128, 256), (7, 256, 512)]:
        M = 256 * hw * hw
        x = torch.randn(M, C, device="cuda")
        w = torch.randn(K, C, device="cuda")
        y = torch.empty(M, K, device="cuda")
        fl = 2.0 * M * K * C
        t_mm = timeit(lambda: torch.mm(x, w.t(), out=y))
        t_dk = timeit(lambda: lib.dk_pwconv_fwd_f32(x.data_ptr(), 256, hw, hw, C, w.data_ptr(), K, 1, 0,
                                                    y.data_ptr(), hw, hw, st))
        print(f"M={M:6d} N={K:4d} K={C:4d}: torch.mm {t_mm:7.1f} us {fl / t_mm / 1e6:6.1f} TF/s "
              f"({fl / t_mm / 1e6 / 157.3:.3f})   dk_pwconv_fwd_f32 {t_dk:7.1f} us {fl / t_dk / 1e6:6.1f} TF/s "
              f"({fl / t_dk / 1e6 / 157.3:.3f})", flush=True)


if __name__ == "__main__":
    main()
