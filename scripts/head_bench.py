"""The network head's small kernels at config 3's shapes (batch 256): global average pooling forward /
backward over 7 x 7 x 512, softmax + cross-entropy forward / backward over 120 classes.  Median of 25
calls (HIP events).
    python scripts/head_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib, stream_handle  # noqa: E402


def timeit(fn, reps=25):
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
    B, HW, C, K = 256, 49, 512, 120
    torch.manual_seed(0)
    x = torch.rand(B * HW * C, device="cuda")
    g = torch.empty(B * C, device="cuda")
    dx = torch.empty(B * HW * C, device="cuda")
    g2 = torch.empty(B * HW * C, device="cuda")
    t = timeit(lambda: lib.dk_gap_fwd_f32(x.data_ptr(), B, HW, C, g.data_ptr(), st))
    print(f"gap_fwd  {B}x{HW}x{C}: {t:6.1f} us  {4 * (B * HW * C + B * C) / t / 1e6:5.2f} TB/s")
    t = timeit(lambda: lib.dk_gap_bwd_f32(g.data_ptr(), B, HW, C, dx.data_ptr(), st))
    print(f"gap_bwd  {B}x{HW}x{C}: {t:6.1f} us  {4 * (B * HW * C + B * C) / t / 1e6:5.2f} TB/s")
    P = B * HW
    mask = (torch.rand(B * HW * C, device="cuda") > 0.5).to(torch.uint8)
    bn = [torch.randn(C, device="cuda"), torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda"),
          torch.randn(C, device="cuda")]
    nb = lib.dk_bn_workspace_bytes(P, C)
    part = torch.empty(nb, dtype=torch.uint8, device="cuda")
    t = timeit(lambda: lib.dk_relu_bwd_bn_partial_f64(dx.data_ptr(), mask.data_ptr(), x.data_ptr(), P, C,
                                                      *(v.data_ptr() for v in bn), 1, g2.data_ptr(), part.data_ptr(),
                                                      nb, st))
    print(f"relu_bwd_bn_partial {P}x{C}: {t:6.1f} us  {(13 * P * C) / t / 1e6:5.2f} TB/s "
          f"({lib.dk_bn_partial_blocks(P, C)} partial rows)")
    logits = torch.randn(B, K, device="cuda")
    y = torch.nn.functional.one_hot(torch.randint(0, K, (B,), device="cuda"), K).float()
    p = torch.empty_like(logits)
    loss = torch.empty((), device="cuda")
    t = timeit(lambda: lib.dk_softmax_xent_fwd_f32(logits.data_ptr(), y.data_ptr(), B, K, p.data_ptr(),
                                                   loss.data_ptr(), st))
    print(f"softmax_xent_fwd {B}x{K}: {t:6.1f} us")
    d = torch.empty_like(p)
    t = timeit(lambda: lib.dk_softmax_xent_bwd_f32(p.data_ptr(), y.data_ptr(), B, K, d.data_ptr(), st))
    print(f"softmax_xent_bwd {B}x{K}: {t:6.1f} us")
    ref = torch.softmax(logits.double(), 1)
    print(f"  max |p - softmax| {float((p.double() - ref).abs().max()):.2e}, loss {float(loss):.6f} vs "
          f"{float(-(torch.log((ref * y).sum(1))).mean()):.6f}")


if __name__ == "__main__":
    main()
