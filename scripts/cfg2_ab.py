"""A/B of the row-GEMM tile for BASELINE config 2 (3x3 conv fwd+dgrad+wgrad, 256x64x56x56): whole
passes timed with HIP events, configurations interleaved over rounds.
    python scripts/cfg2_ab.py [-1,6,14]        # row-tile configurations
    python scripts/cfg2_ab.py 6:0 6:3          # kind:value of dk_debug_set_gemm_config (knobs)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dorknet_amd._hip import lib  # noqa: E402
from dorknet_amd.layers.convolution import ConvLayer  # noqa: E402


def main():
    np.random.seed(0)
    conv = ConvLayer("c", filter_block_shape=(64, 64, 3, 3), stride=1, padding=1, with_bias=False)
    conv.to_gpu()
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn((256, 64, 56, 56), device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    dY = torch.randn((256, 64, 56, 56), device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    if len(sys.argv) > 1 and ":" in sys.argv[1]:
        cfgs = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]]
    else:
        cfgs = [(0, int(c)) for c in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["-1", "6", "14", "1"])]
    res = {c: [] for c in cfgs}
    for rnd in range(4):
        for c in cfgs:
            lib.dk_debug_set_gemm_config(*c)
            for _ in range(3):
                conv.forward(X)
                conv.backward(dY)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                conv.forward(X)
                conv.backward(dY)
            b.record()
            torch.cuda.synchronize()
            res[c].append(a.elapsed_time(b) / 20)
    for c in cfgs:
        lib.dk_debug_set_gemm_config(c[0], -1)
    flops = 3 * 2 * 256 * 56 * 56 * 64 * 64 * 9
    for c, t in res.items():
        m = float(np.median(t))
        print(f"knob {c[0]}:{c[1]:3d}: {m:.4f} ms/pass (rounds {' '.join(f'{x:.4f}' for x in t)}) "
              f"{flops / m / 1e9:.1f} TF/s = {flops / m / 1e9 / 157.3:.3f} of fp32 MFMA", flush=True)


if __name__ == "__main__":
    main()
