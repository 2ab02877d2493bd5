"""Fused K = C = 64 pointwise backward (dk_pwconv_bwd_bnbwd_f32) at res1 (256 x 56 x 56): median time of
interleaved rounds, nontemporal dx stores off / on (knob 4).  DORKNET_HIP_LIB picks the build.
    python scripts/pws_ab.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dorknet_amd._hip import lib  # noqa: E402


def timeit(fn, reps=7):
    for _ in range(2):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return 1e3 * t[len(t) // 2]


def main():
    B, H, K, C = 256, 56, 64, 64
    st = torch.cuda.current_stream().cuda_stream
    P = B * H * H
    g = torch.Generator(device="cuda").manual_seed(0)

    def rnd(n):
        return torch.randn(n, device="cuda", generator=g)

    gg, xo, xin, dx = rnd(P * K), rnd(P * K), rnd(P * C), torch.empty(P * C, device="cuda")
    res = rnd(P * C)
    w, dw = rnd(K * C) * 0.1, torch.empty(K * C, device="cuda")
    po = [rnd(K), rnd(K).abs() + 0.5, rnd(K), rnd(K)]
    pi = [rnd(C), rnd(C).abs() + 0.5, rnd(C), rnd(C)]
    k12 = rnd(2 * K) * 0.1
    rows = lib.dk_pwconv_bwd_fused_rows(B, H, H, K, C)
    part = torch.empty(rows * 2 * C, dtype=torch.float64, device="cuda")
    nbf = lib.dk_pwconv_bwd_fused_workspace_bytes(B, H, H, K, C)
    ws = torch.empty(nbf, dtype=torch.uint8, device="cuda")
    out = {}
    for _ in range(5):
        for nt in (0, 1):
            for r in (0, 1):
                lib.dk_debug_set_gemm_config(4, nt << 3)  # bit 3: the fused pointwise backward
                args = (gg.data_ptr(), xo.data_ptr(), B, H, H, K, *(t.data_ptr() for t in po), 1, k12.data_ptr(),
                        w.data_ptr(), C, 1e-4, dw.data_ptr(), dx.data_ptr(), res.data_ptr() if r else 0,
                        xin.data_ptr(), *(t.data_ptr() for t in pi), 1, part.data_ptr(), ws.data_ptr(), nbf, st)
                out.setdefault((nt, r), []).append(timeit(lambda: lib.dk_pwconv_bwd_bnbwd_f32(*args)))
    lib.dk_debug_set_gemm_config(4, -1)
    for (nt, r), v in sorted(out.items()):
        v = sorted(v)
        print(f"nt={nt} residual={r}: min {v[0]:6.1f}  med {v[len(v) // 2]:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
