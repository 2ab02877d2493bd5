"""The skip projections' input gradient (dk_pwconv_dgrad_f32, stride 1 into the compact lattice) at
config 3's shapes: the deep kernels' plain form (knob 11 on) against the tiled engine (knob 11 off),
standalone, HIP-event timed, dx compared bitwise."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dorknet_amd._hip import lib, stream_handle  # noqa: E402

B = 256
SHAPES = [(14, 256, 128), (7, 512, 256), (28, 128, 64)]  # output HW, K (dy channels), C (dx channels)


def main():
    st = stream_handle()
    torch.manual_seed(0)
    for HW, K, C in SHAPES:
        M = B * HW * HW
        dy = torch.randn(M * K, device="cuda")
        w = torch.randn(K * C, device="cuda") * 0.05
        outs, line = {}, []
        for deep in (1, 0):
            lib.dk_debug_set_gemm_config(11, deep)
            dx = torch.full((M * C,), float("nan"), device="cuda")
            for _ in range(3):
                assert lib.dk_pwconv_dgrad_f32(dy.data_ptr(), B, HW, HW, K, w.data_ptr(), C, 1, dx.data_ptr(), st) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(20):
                lib.dk_pwconv_dgrad_f32(dy.data_ptr(), B, HW, HW, K, w.data_ptr(), C, 1, dx.data_ptr(), st)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            tf = 2.0 * M * K * C / us / 1e6
            line.append("%s %.1f us (%.1f TF/s)" % ("deep " if deep else "tiled", us, tf))
            outs[deep] = dx.clone()
        lib.dk_debug_set_gemm_config(11, -1)
        same = "bitwise" if torch.equal(outs[0], outs[1]) else "DIFF"
        print("HW %d K %d C %d: %s; %s" % (HW, K, C, ", ".join(line), same), flush=True)


if __name__ == "__main__":
    main()
