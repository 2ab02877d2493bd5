"""The bf16 streaming pointwise kernels (csrc/pw_stream_bf16.hip, and for the deep shapes also the
weight-stationary csrc/pw_deep_bf16.hip, BASELINE config 5) against the
tiled engine's bf16 MFMA mode they replace (knob 9 off): y, dy (written through) and dx bitwise
(same operand rounding, same MFMA k order, same fp32 epilogue), the BatchNorm partial sums to
fp64 rounding (one row per persistent block instead of one per 64-pixel tile).  Ragged pixel
counts, every (K, C) pair in {64, 128}, every epilogue option; outputs carved out of NaN-filled
buffers so that a store past the last row would show."""
import numpy as np
import pytest
import torch

from dorknet_amd._hip import lib, stream_handle

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


def padded(M, C, rng=None):
    """An [M][C] bf16 tensor (random, or NaN when rng is None) inside a buffer 7 rows longer that
    is NaN past it: (view, whole buffer)."""
    buf = torch.full(((M + 7) * C,), float("nan"), dtype=BF16, device="cuda")
    if rng is not None:
        buf[:M * C] = torch.as_tensor(rng.randn(M * C).astype(np.float32), device="cuda").to(BF16)
    return buf[:M * C], buf


def bn_params(C, rng):
    return [torch.as_tensor(v.astype(np.float32), device="cuda") for v in
            (rng.randn(C) * 0.3, rng.rand(C) + 0.5, 1 + 0.3 * rng.randn(C), 0.2 * rng.randn(C))]


def tail_is_nan(buf, M, C):
    return bool(torch.isnan(buf[M * C:].float()).all())


@pytest.mark.parametrize("K,C", [(64, 64), (128, 64), (64, 128), (128, 128)])
@pytest.mark.parametrize("bn,relu,stats,bias,N,H,W", [(True, 1, True, False, 3, 13, 11),
                                                    (True, 0, True, False, 2, 8, 8),
                                                    (False, 0, True, True, 2, 7, 5),
                                                    (True, 1, False, False, 1, 1, 5),
                                                    (True, 1, True, False, 16, 56, 56)])
def test_bf16_stream_fwd_matches_tiled_engine(K, C, bn, relu, stats, bias, N, H, W):
    rng = np.random.RandomState(K + C + 2 * bn + relu + 4 * stats + N)
    M = N * H * W
    x, _ = padded(M, C, rng)
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32) * 0.2, device="cuda")
    b = torch.as_tensor(rng.randn(K).astype(np.float32), device="cuda") if bias else None
    p = bn_params(C, rng)
    st = stream_handle()

    def run(stream_on):
        lib.dk_debug_set_gemm_config(9, 1 if stream_on else 0)
        try:
            y, ybuf = padded(M, K)
            rows = lib.dk_pwconv_fwd_bf16_stats_rows(N, H, W, K, C)
            part = torch.zeros((rows, 2, K), dtype=torch.float64, device="cuda") if stats else None
            bn_args = (*(t.data_ptr() for t in p), relu) if bn else (0, 0, 0, 0, 0)
            assert lib.dk_pwconv_fwd_ex_bf16(x.data_ptr(), N, H, W, C, w.data_ptr(), K, 1,
                                             b.data_ptr() if bias else 0, y.data_ptr(), H, W, *bn_args,
                                             part.data_ptr() if stats else 0, st) == 0
            torch.cuda.synchronize()
            return y, ybuf, rows, part
        finally:
            lib.dk_debug_set_gemm_config(9, -1)

    y0, _, rows0, part0 = run(False)
    y1, ybuf1, rows1, part1 = run(True)
    assert torch.equal(y0, y1)
    assert tail_is_nan(ybuf1, M, K)
    if stats:
        # at most one partial row per persistent block (a 32-pixel tile each at the least: the
        # weight-stationary kernels' walkers), against one per 64-pixel tile for the tiled engine
        assert rows1 <= max(rows0, -(-M // 32), 1)
        s0, s1 = part0.sum(0), part1.sum(0)
        assert float((s1 - s0).norm() / s0.norm()) < 1e-12


@pytest.mark.parametrize("K,C", [(64, 64), (128, 64), (64, 128), (128, 128)])
@pytest.mark.parametrize("relu,bn_in,resid,dyout,N,H,W", [(1, True, False, True, 3, 13, 11),
                                                        (0, True, False, True, 2, 8, 8),
                                                        (1, False, True, True, 3, 13, 11),
                                                        (1, True, True, False, 5, 7, 9),
                                                        (0, False, False, True, 1, 1, 3),
                                                        (1, True, False, True, 16, 56, 56)])
def test_bf16_stream_dgrad_bnbwd_matches_tiled_engine(K, C, relu, bn_in, resid, dyout, N, H, W):
    rng = np.random.RandomState(K + C + relu + 2 * bn_in + 4 * resid + N)
    M = N * H * W
    xo, _ = padded(M, K, rng)
    g, _ = padded(M, K, rng)
    po = bn_params(K, rng)
    k12 = torch.as_tensor(rng.randn(2 * K).astype(np.float32) * 0.1, device="cuda")
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32) * 0.2, device="cuda")
    xin, _ = padded(M, C, rng)
    pi = bn_params(C, rng)
    res = padded(M, C, rng)[0] if resid else None
    st = stream_handle()

    def run(stream_on):
        lib.dk_debug_set_gemm_config(9, 1 if stream_on else 0)
        try:
            dy, dybuf = padded(M, K)
            dx, dxbuf = padded(M, C)
            rows = lib.dk_pwconv_dgrad_bnbwd_bf16_stats_rows(N, H, W, K, C)
            part = torch.zeros((rows, 2, C), dtype=torch.float64, device="cuda")
            bn_args = (xin.data_ptr(), *(t.data_ptr() for t in pi), 1, part.data_ptr()) if bn_in else (0,) * 7
            assert lib.dk_pwconv_dgrad_bnbwd_bf16(g.data_ptr(), xo.data_ptr(), N, H, W, K,
                                                  *(t.data_ptr() for t in po), relu, k12.data_ptr(),
                                                  dy.data_ptr() if dyout else 0, w.data_ptr(), C, dx.data_ptr(),
                                                  res.data_ptr() if resid else 0, *bn_args, st) == 0
            torch.cuda.synchronize()
            return dy, dybuf, dx, dxbuf, part
        finally:
            lib.dk_debug_set_gemm_config(9, -1)

    dy0, _, dx0, _, part0 = run(False)
    dy1, dybuf1, dx1, dxbuf1, part1 = run(True)
    assert torch.equal(dx0, dx1)
    assert tail_is_nan(dxbuf1, M, C)
    if dyout:
        assert torch.equal(dy0, dy1)
        assert tail_is_nan(dybuf1, M, K)
    else:
        assert bool(torch.isnan(dybuf1.float()).all())
    if bn_in:
        s0, s1 = part0.sum(0), part1.sum(0)
        assert float((s1 - s0).norm() / s0.norm()) < 1e-12


# The deep shapes: K or C of 256 / 512 (config 5's 14 x 14 and 7 x 7 units), on the weight-stationary
# kernels of pw_deep_bf16.hip (the round-3 column-sliced kernels they superseded are deleted).
DEEP = [(256, 128), (256, 256), (512, 256), (512, 512), (128, 256)]


DEEP16_KNOB = 13  # 1: the weight-stationary kernels (pw_deep_bf16.hip, default); 0: the tiled engine


@pytest.fixture(params=[1], ids=["weight_stationary"])
def deep16(request):
    lib.dk_debug_set_gemm_config(DEEP16_KNOB, request.param)
    yield request.param
    lib.dk_debug_set_gemm_config(DEEP16_KNOB, -1)


@pytest.mark.parametrize("K,C", DEEP)
@pytest.mark.parametrize("bn,relu,stats,bias,N,H,W", [(True, 1, True, False, 3, 13, 11),
                                                    (False, 0, True, True, 2, 7, 5),
                                                    (True, 0, False, False, 1, 1, 5),
                                                    (True, 1, True, False, 16, 7, 7)])
def test_bf16_deep_fwd_matches_tiled_engine(K, C, bn, relu, stats, bias, N, H, W, deep16):
    test_bf16_stream_fwd_matches_tiled_engine(K, C, bn, relu, stats, bias, N, H, W)


@pytest.mark.parametrize("K,C", [(k, c) for c, k in DEEP])
@pytest.mark.parametrize("relu,bn_in,resid,dyout,N,H,W", [(1, True, False, True, 3, 13, 11),
                                                        (1, False, True, True, 3, 13, 11),
                                                        (1, True, True, False, 5, 7, 9),
                                                        (0, False, False, True, 1, 1, 3),
                                                        (1, True, False, True, 16, 7, 7)])
def test_bf16_deep_dgrad_bnbwd_matches_tiled_engine(K, C, relu, bn_in, resid, dyout, N, H, W, deep16):
    test_bf16_stream_dgrad_bnbwd_matches_tiled_engine(K, C, relu, bn_in, resid, dyout, N, H, W)


def test_bf16_deep_kernels_dispatch():
    """The deep shapes go to the streaming kernels: one partial row per walker block, not per tile."""
    M = 512 * 7 * 7
    lib.dk_debug_set_gemm_config(9, 0)
    try:
        tiled = lib.dk_pwconv_fwd_bf16_stats_rows(512, 7, 7, 512, 512)
    finally:
        lib.dk_debug_set_gemm_config(9, -1)
    streamed = lib.dk_pwconv_fwd_bf16_stats_rows(512, 7, 7, 512, 512)
    assert streamed != tiled and streamed <= 256 and tiled >= M // 256


@pytest.mark.parametrize("K,C", [(64, 64), (128, 128), (256, 128), (256, 256), (128, 256), (128, 64)])
@pytest.mark.parametrize("relu,bn_in,resid,N,H,W", [(1, True, False, 3, 13, 11), (0, True, False, 2, 8, 8),
                                                    (1, False, True, 3, 13, 11), (1, True, True, 5, 7, 9),
                                                    (0, False, False, 1, 1, 3), (1, True, False, 16, 56, 56)])
def test_bf16_fused_bwd_matches_dgrad_and_fp64(K, C, relu, bn_in, resid, N, H, W):
    """dk_pwconv_bwd_bnbwd_bf16 (dgrad and weight gradient in one pass, dy never stored: K = C = 64 on
    pw_stream_bf16.hip bwd_fused_kernel, K in {128, 256} on pw_deep_bf16.hip bwd_kernel, incl. K = 128 with
    C = 64, one column group) against the
    dgrad that stores dy: dx bitwise, the input BatchNorm's partial sums to fp64 rounding; and its
    weight gradient against fp64 dW = dy^T bf16(bn_relu(x)) + l2 w with dy the dgrad's stored bf16 dy
    (the MFMA operands the fused kernel forms), elementwise within 3e-5 of sum |dy| |xh|.
    Reference: pointwise_convolution.py:57-75."""
    assert lib.dk_pwconv_bwd_fused_bf16_rows(N, H, W, K, C) > 0
    rng = np.random.RandomState(5 + relu + 2 * bn_in + 4 * resid + N)
    M = N * H * W
    xo, _ = padded(M, K, rng)
    g, _ = padded(M, K, rng)
    po = bn_params(K, rng)
    k12 = torch.as_tensor(rng.randn(2 * K).astype(np.float32) * 0.1, device="cuda")
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32) * 0.2, device="cuda")
    xin, _ = padded(M, C, rng)
    pi = bn_params(C, rng)
    res = padded(M, C, rng)[0] if resid else None
    l2 = 1e-3
    st = stream_handle()
    # reference dgrad (stores dy)
    dy, _ = padded(M, K)
    dx0, _ = padded(M, C)
    rows0 = lib.dk_pwconv_dgrad_bnbwd_bf16_stats_rows(N, H, W, K, C)
    p0 = torch.zeros((rows0, 2, C), dtype=torch.float64, device="cuda")
    bn_args = (xin.data_ptr(), *(t.data_ptr() for t in pi), relu, p0.data_ptr()) if bn_in else (0,) * 7
    assert lib.dk_pwconv_dgrad_bnbwd_bf16(g.data_ptr(), xo.data_ptr(), N, H, W, K, *(t.data_ptr() for t in po), relu,
                                          k12.data_ptr(), dy.data_ptr(), w.data_ptr(), C, dx0.data_ptr(),
                                          res.data_ptr() if resid else 0, *bn_args, st) == 0
    # fused
    rows1 = lib.dk_pwconv_bwd_fused_bf16_rows(N, H, W, K, C)
    nb = lib.dk_pwconv_bwd_fused_bf16_workspace_bytes(N, H, W, K, C)
    ws = torch.empty(nb // 4 + 4, dtype=torch.float32, device="cuda")
    dx1, dx1buf = padded(M, C)
    dw = torch.full((K, C), float("nan"), device="cuda")
    p1 = torch.zeros((rows1, 2, C), dtype=torch.float64, device="cuda")
    bnb = (*(t.data_ptr() for t in pi), relu, p1.data_ptr()) if bn_in else (0,) * 6
    rc = lib.dk_pwconv_bwd_bnbwd_bf16(g.data_ptr(), xo.data_ptr(), N, H, W, K, *(t.data_ptr() for t in po), relu,
                                      k12.data_ptr(), w.data_ptr(), C, l2, dw.data_ptr(), dx1.data_ptr(),
                                      res.data_ptr() if resid else 0, xin.data_ptr(), *bnb, ws.data_ptr(), nb, st)
    assert rc in (0, 10100)
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)
    assert tail_is_nan(dx1buf, M, C)
    if bn_in:
        s0, s1 = p0.sum(0), p1.sum(0)
        assert float((s1 - s0).norm() / s0.norm()) < 1e-12
    dy64 = dy.view(M, K).double()
    xf = xin.view(M, C).float()
    if bn_in:
        xh = pi[2] * ((xf - pi[0]) * pi[1]) + pi[3]
        if relu:
            xh = torch.where(xh > 0, xh, torch.zeros_like(xh))
    else:
        xh = xf
    xh = xh.to(BF16).double()  # the bf16 MFMA operand
    ref = dy64.t() @ xh + l2 * w.double()
    bound = 3e-5 * (dy64.abs().t() @ xh.abs()) + 1e-6
    assert bool(torch.isfinite(dw).all())
    assert bool(((dw.double() - ref).abs() <= bound).all()), float(((dw.double() - ref).abs() / bound).max())
