"""Achievable HBM rate for the traffic mixes of the step's kernels (dk_debug_stream_mix): reads
and writes of 205 MB fp32 streams (one res1 activation at batch 256), float4 per lane.  The
ceiling that the pointwise / depthwise kernels' roofline fractions are measured against in
practice (8 TB/s is the spec; MI355X_MICROARCH.md measures 6.29 TB/s for a float4 copy).

    python scripts/stream_ceiling.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib  # noqa: E402


def main():
    n = 256 * 56 * 56 * 64
    st = torch.cuda.current_stream().cuda_stream
    bufs = [torch.randn(n, device="cuda") for _ in range(5)]
    p = [b.data_ptr() for b in bufs]
    for nin, nout in ((1, 0), (1, 1), (2, 1), (1, 2), (2, 2), (3, 1), (3, 2), (1, 11), (2, 11), (3, 11), (2, 12),
                       (3, 12)):
        for blocks in (1024, 2048):
            f = lambda: lib.dk_debug_stream_mix(p[0], p[1], p[2], p[3], p[4], nin, nout, n, blocks, st)
            for _ in range(3):
                f()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
            for a, b in ev:
                a.record()
                f()
                b.record()
            torch.cuda.synchronize()
            t = sorted(a.elapsed_time(b) for a, b in ev)[5] * 1e-3
            gbs = (nin + nout % 10) * n * 4 / t / 1e9
            print("reads {} writes {}{} blocks {:5d}: {:7.1f} us  {:6.0f} GB/s".format(
                nin, nout % 10, " (nt)" if nout >= 10 else "", blocks, t * 1e6, gbs), flush=True)


if __name__ == "__main__":
    main()
