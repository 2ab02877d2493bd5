"""The deep pointwise kernels (csrc/pw_deep.hip: reduction 64-512 with 128+ channels on a side)
against the tiled engine they replace (knob 11 off and the streaming kernels off):
dk_pwconv_fwd_ex_f32 y, dk_pwconv_fwd_f32 (the strided skip projections) y, and
dk_pwconv_dgrad_bnbwd_f32 dy / dx bitwise (the same MFMA k order), the output statistics and the
input BatchNorm's partial sums to fp64 rounding (one partial row per block and column group
instead of one per tile); ragged pixel counts, every epilogue option, a large grid (several tiles
per block), and nothing written past the outputs."""
import numpy as np
import pytest
import torch

from dorknet_amd._hip import lib, stream_handle

pytestmark = pytest.mark.gpu

STREAM_KNOB, DEEP_KNOB = 3, 11


def nhwc(a):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device="cuda").contiguous(
        memory_format=torch.channels_last)


def bn_params(C, rng):
    return [torch.as_tensor(v.astype(np.float32), device="cuda") for v in
            (rng.randn(C) * 0.3, rng.rand(C) + 0.5, 1 + 0.3 * rng.randn(C), 0.2 * rng.randn(C))]


def _modes(fn):
    """fn() under the tiled engine (streaming kernels off) and under the deep kernels."""
    out = []
    for knobs in (((STREAM_KNOB, 0),), ((DEEP_KNOB, 1),)):
        for k, v in knobs:
            lib.dk_debug_set_gemm_config(k, v)
        try:
            out.append(fn())
        finally:
            for k, _ in knobs:
                lib.dk_debug_set_gemm_config(k, -1)
    return out


def _close_sums(p0, p1):
    s0, s1 = p0.sum(0), p1.sum(0)
    return float((s1 - s0).norm() / max(float(s0.norm()), 1e-300)) < 1e-12


SHAPES = [(128, 64), (128, 128), (256, 128), (256, 256), (512, 256), (512, 512), (128, 512)]  # (K, C)


@pytest.mark.parametrize("K,C", SHAPES)
@pytest.mark.parametrize("bn,relu,stats,stride,bias,N,H,W", [(True, 1, True, 1, False, 3, 13, 11),
                                                           (True, 0, True, 2, False, 2, 13, 9),
                                                           (False, 0, True, 1, True, 2, 8, 8),
                                                           (True, 1, False, 1, False, 1, 1, 5),
                                                           (False, 0, False, 2, True, 3, 6, 7),
                                                           (True, 1, True, 1, False, 16, 14, 14)])
def test_deep_fwd_matches_tiled_engine(K, C, bn, relu, stats, stride, bias, N, H, W):
    rng = np.random.RandomState(K + C + int(bn) + 2 * relu + 4 * stats + 8 * stride + N)
    x = nhwc(rng.randn(N, C, H, W) * 2 + 0.3)
    w = torch.as_tensor((rng.randn(K, C) / np.sqrt(C)).astype(np.float32), device="cuda")
    b = torch.as_tensor(rng.randn(K).astype(np.float32), device="cuda") if bias else None
    pi = bn_params(C, rng)
    OH, OW = -(-H // stride), -(-W // stride)
    st = stream_handle()
    bn_args = (*(t.data_ptr() for t in pi), relu) if bn else (0, 0, 0, 0, 0)

    def run():
        rows = lib.dk_pwconv_fwd_stats_rows(N, OH, OW, K, C)
        part = torch.full((rows, 2, K), float("nan"), dtype=torch.float64, device="cuda") if stats else None
        y = torch.full((N, K, OH, OW), float("nan"), device="cuda").contiguous(memory_format=torch.channels_last)
        lib.dk_pwconv_fwd_ex_f32(x.data_ptr(), N, H, W, C, w.data_ptr(), K, stride, b.data_ptr() if bias else 0,
                                 y.data_ptr(), OH, OW, *bn_args, part.data_ptr() if stats else 0, st)
        torch.cuda.synchronize()
        return y, part
    (y0, p0), (y1, p1) = _modes(run)
    assert torch.equal(y0, y1)
    if stats:
        assert _close_sums(p0, p1)


@pytest.mark.parametrize("K,C,H", [(128, 64, 56), (256, 128, 28), (512, 256, 14), (128, 128, 9)])
def test_deep_strided_skip_projection(K, C, H):
    """dk_pwconv_fwd_f32 at stride 2 (the downsampling blocks' skip projections, no BN on load)."""
    N = 3
    rng = np.random.RandomState(K + H)
    x = nhwc(rng.randn(N, C, H, H))
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
    OH = -(-H // 2)
    st = stream_handle()

    def run():
        y = torch.full((N, K, OH, OH), float("nan"), device="cuda").contiguous(memory_format=torch.channels_last)
        lib.dk_pwconv_fwd_f32(x.data_ptr(), N, H, H, C, w.data_ptr(), K, 2, 0, y.data_ptr(), OH, OH, st)
        torch.cuda.synchronize()
        return y
    y0, y1 = _modes(run)
    assert torch.equal(y0, y1)


@pytest.mark.parametrize("K,C", SHAPES)
@pytest.mark.parametrize("relu,bn_in,resid,N,H,W", [(1, True, False, 3, 13, 11), (0, True, False, 2, 8, 8),
                                                    (1, False, True, 3, 13, 11), (1, True, True, 5, 7, 9),
                                                    (0, False, False, 1, 1, 3), (1, True, False, 16, 14, 14)])
def test_deep_dgrad_bnbwd_matches_tiled_engine(K, C, relu, bn_in, resid, N, H, W):
    rng = np.random.RandomState(K + C + relu + 2 * bn_in + 4 * resid + N)
    xo = nhwc(rng.randn(N, K, H, W))
    g = nhwc(rng.randn(N, K, H, W))
    po = bn_params(K, rng)
    k12 = torch.as_tensor(rng.randn(2 * K).astype(np.float32) * 0.1, device="cuda")
    w = torch.as_tensor((rng.randn(K, C) / np.sqrt(K)).astype(np.float32), device="cuda")
    xin = nhwc(rng.randn(N, C, H, W))
    pi = bn_params(C, rng)
    res = nhwc(rng.randn(N, C, H, W)) if resid else None
    st = stream_handle()

    def run():
        rows = lib.dk_pwconv_dgrad_bnbwd_stats_rows(N, H, W, K, C)
        dy = torch.full_like(g, float("nan"))
        dx = torch.full_like(xin, float("nan"))
        part = torch.full((rows, 2, C), float("nan"), dtype=torch.float64, device="cuda")
        bn_args = (xin.data_ptr(), *(t.data_ptr() for t in pi), 1, part.data_ptr()) if bn_in else (0,) * 7
        lib.dk_pwconv_dgrad_bnbwd_f32(g.data_ptr(), xo.data_ptr(), N, H, W, K, *(t.data_ptr() for t in po), relu,
                                      k12.data_ptr(), dy.data_ptr(), w.data_ptr(), C, dx.data_ptr(),
                                      res.data_ptr() if resid else 0, *bn_args, st)
        torch.cuda.synchronize()
        return dy, dx, part
    (dy0, dx0, p0), (dy1, dx1, p1) = _modes(run)
    assert torch.equal(dy0, dy1)
    assert torch.equal(dx0, dx1)
    if bn_in:
        assert _close_sums(p0, p1)


def test_deep_outputs_stay_in_bounds():
    """A ragged pixel count (M % 32 != 0) at a deep shape: nothing is written past y, dy or dx (their
    buffers are followed by a sentinel), and the deep path is the one taken."""
    from dorknet_amd._hip import lib as L
    N, H, W, K, C = 3, 7, 5, 256, 128
    M = N * H * W
    assert M % 32 and L.dk_pwconv_dgrad_bnbwd_stats_rows(N, H, W, K, C) > 0
    rng = np.random.RandomState(9)
    st = stream_handle()
    x = nhwc(rng.randn(N, C, H, W))
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
    pi = bn_params(C, rng)
    ybuf = torch.full((M * K + 4096,), 12345.0, device="cuda")
    rows = L.dk_pwconv_fwd_stats_rows(N, H, W, K, C)
    part = torch.zeros((rows, 2, K), dtype=torch.float64, device="cuda")
    L.dk_pwconv_fwd_ex_f32(x.data_ptr(), N, H, W, C, w.data_ptr(), K, 1, 0, ybuf.data_ptr(), H, W,
                           *(t.data_ptr() for t in pi), 1, part.data_ptr(), st)
    g = nhwc(rng.randn(N, K, H, W))
    xo = nhwc(rng.randn(N, K, H, W))
    po = bn_params(K, rng)
    k12 = torch.as_tensor(rng.randn(2 * K).astype(np.float32) * 0.1, device="cuda")
    dybuf = torch.full((M * K + 4096,), 12345.0, device="cuda")
    dxbuf = torch.full((M * C + 4096,), 12345.0, device="cuda")
    rows = L.dk_pwconv_dgrad_bnbwd_stats_rows(N, H, W, K, C)
    partd = torch.zeros((rows, 2, C), dtype=torch.float64, device="cuda")
    L.dk_pwconv_dgrad_bnbwd_f32(g.data_ptr(), xo.data_ptr(), N, H, W, K, *(t.data_ptr() for t in po), 1,
                                k12.data_ptr(), dybuf.data_ptr(), w.data_ptr(), C, dxbuf.data_ptr(), 0, x.data_ptr(),
                                *(t.data_ptr() for t in pi), 1, partd.data_ptr(), st)
    torch.cuda.synchronize()
    for buf, n in ((ybuf, M * K), (dybuf, M * K), (dxbuf, M * C)):
        assert bool((buf[n:] == 12345.0).all())
        assert bool(torch.isfinite(buf[:n]).all())
    assert bool(torch.isfinite(part).all()) and bool(torch.isfinite(partd).all())


WGRAD_SHAPES = [(128, 64), (128, 128), (256, 128), (256, 256), (512, 256), (512, 512)]  # (K, C)


@pytest.mark.parametrize("K,C", WGRAD_SHAPES)
@pytest.mark.parametrize("bn,relu,N,H,W", [(True, 1, 3, 13, 11), (True, 0, 2, 8, 8), (False, 0, 1, 1, 5),
                                           (True, 1, 16, 14, 14)])
def test_deep_wgrad_matches_fp64(K, C, bn, relu, N, H, W):
    """dk_pwconv_wgrad_bnx_f32 / dk_pwconv_wgrad_f32 (the tiled engine's split-K weight gradient, the
    deep layers' path where no fused backward takes them) against an fp64 dW = dy^T relu(bn(x)) + l2 w,
    elementwise within 3e-5 of sum |dy| |xh| (fp32 partial sums of a few hundred products each, then
    the fp64 reduce)."""
    rng = np.random.RandomState(K + 3 * C + N + int(bn) + 2 * relu)
    M = N * H * W
    dy = nhwc(rng.randn(N, K, H, W))
    x = nhwc(rng.randn(N, C, H, W) * 1.5 + 0.2)
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
    pi = bn_params(C, rng)
    l2 = 1e-3
    st = stream_handle()

    def run():
        # (the workspace size depends on the path the knobs select)
        nb = lib.dk_pwconv_wgrad_workspace_bytes(N, H, W, K, C)
        ws = torch.empty(max(nb, 4) // 4 + 1, dtype=torch.float32, device="cuda")
        dw = torch.full((K, C), float("nan"), device="cuda")
        if bn:
            rc = lib.dk_pwconv_wgrad_bnx_f32(dy.data_ptr(), x.data_ptr(), N, H, W, C, K, 1, H, W, w.data_ptr(), l2,
                                             dw.data_ptr(), ws.data_ptr(), nb, *(t.data_ptr() for t in pi), relu, st)
        else:
            rc = lib.dk_pwconv_wgrad_f32(dy.data_ptr(), x.data_ptr(), N, H, W, C, K, 1, H, W, w.data_ptr(), l2,
                                         dw.data_ptr(), ws.data_ptr(), nb, st)
        assert rc == 0
        torch.cuda.synchronize()
        return dw
    outs = [run()]
    dy64 = dy.permute(0, 2, 3, 1).reshape(M, K).double()
    x64 = x.permute(0, 2, 3, 1).reshape(M, C).double()
    if bn:
        # the kernels' fp32 bn_out (up to the fma's last bit), then exact products
        xf = x.permute(0, 2, 3, 1).reshape(M, C)
        xh = (pi[2] * ((xf - pi[0]) * pi[1]) + pi[3]).double()
        if relu:
            xh = xh.clamp_min(0.0)
    else:
        xh = x64
    ref = dy64.t() @ xh + l2 * w.double()
    bound = 3e-5 * (dy64.abs().t() @ xh.abs()) + 1e-6
    for dw in outs:
        assert bool(torch.isfinite(dw).all())
        assert bool(((dw.double() - ref).abs() <= bound).all()), float(((dw.double() - ref).abs() / bound).max())


@pytest.mark.parametrize("K,C,H", [(256, 128, 28), (512, 256, 14), (128, 128, 9), (256, 256, 13)])
def test_deep_wgrad_strided_skip(K, C, H):
    """dk_pwconv_wgrad_f32 at stride 2 (the downsampling blocks' skip projections: x read at (n, 2 oh, 2 ow))
    against fp64, the same elementwise bound as above."""
    N = 3
    rng = np.random.RandomState(K + C + H)
    OH = -(-H // 2)
    M = N * OH * OH
    dy = nhwc(rng.randn(N, K, OH, OH))
    x = nhwc(rng.randn(N, C, H, H))
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
    l2 = 1e-3
    st = stream_handle()
    nb = lib.dk_pwconv_wgrad_workspace_bytes(N, OH, OH, K, C)
    ws = torch.empty(max(nb, 4) // 4 + 1, dtype=torch.float32, device="cuda")
    dw = torch.full((K, C), float("nan"), device="cuda")
    assert lib.dk_pwconv_wgrad_f32(dy.data_ptr(), x.data_ptr(), N, H, H, C, K, 2, OH, OH, w.data_ptr(), l2,
                                   dw.data_ptr(), ws.data_ptr(), nb, st) == 0
    torch.cuda.synchronize()
    dy64 = dy.permute(0, 2, 3, 1).reshape(M, K).double()
    xs = x[:, :, ::2, ::2].permute(0, 2, 3, 1).reshape(M, C).double()
    ref = dy64.t() @ xs + l2 * w.double()
    bound = 3e-5 * (dy64.abs().t() @ xs.abs()) + 1e-6
    assert bool(torch.isfinite(dw).all())
    assert bool(((dw.double() - ref).abs() <= bound).all()), float(((dw.double() - ref).abs() / bound).max())


FUSED_KNOB = 14
FUSED_SHAPES = [(128, 128), (256, 128), (256, 256), (128, 256), (256, 512), (128, 64)]  # (K, C)


@pytest.mark.parametrize("K,C", FUSED_SHAPES)
@pytest.mark.parametrize("relu,bn_in,resid,N,H,W", [(1, True, False, 3, 13, 11), (0, True, False, 2, 8, 8),
                                                    (1, False, True, 3, 13, 11), (1, True, True, 5, 7, 9),
                                                    (0, False, False, 1, 1, 3), (1, True, False, 16, 14, 14),
                                                    (1, True, False, 64, 14, 14)])
def test_deep_fused_bwd_matches_unfused(K, C, relu, bn_in, resid, N, H, W):
    """dk_pwconv_bwd_bnbwd_f32 on the fused deep kernel (pw_deep.hip bwd_kernel: dgrad and weight
    gradient in one pass, dy never stored) against the deep dgrad (dk_pwconv_dgrad_bnbwd_f32): dx bitwise,
    the input BatchNorm's partial sums to fp64 rounding; and its weight gradient against fp64
    dW = dy^T relu(bn(x)) + l2 w (dy = the dgrad's stored dy, the values the fused kernel forms on load),
    elementwise within 3e-5 of sum |dy| |xh|.  Reference: pointwise_convolution.py:57-75."""
    assert lib.dk_pwconv_bwd_fused_preferred(N, H, W, K, C) == 1
    rng = np.random.RandomState(K + C + relu + 2 * bn_in + 4 * resid + N)
    M = N * H * W
    xo = nhwc(rng.randn(N, K, H, W))
    g = nhwc(rng.randn(N, K, H, W))
    po = bn_params(K, rng)
    k12 = torch.as_tensor(rng.randn(2 * K).astype(np.float32) * 0.1, device="cuda")
    w = torch.as_tensor((rng.randn(K, C) / np.sqrt(K)).astype(np.float32), device="cuda")
    xin = nhwc(rng.randn(N, C, H, W) * 1.5 + 0.2)
    pi = bn_params(C, rng)
    res = nhwc(rng.randn(N, C, H, W)) if resid else None
    l2 = 1e-3
    st = stream_handle()
    # the reference: deep dgrad (stores dy)
    rows = lib.dk_pwconv_dgrad_bnbwd_stats_rows(N, H, W, K, C)
    dy = torch.full_like(g, float("nan"))
    dx0 = torch.full_like(xin, float("nan"))
    p0 = torch.full((rows, 2, C), float("nan"), dtype=torch.float64, device="cuda")
    bn_args = (xin.data_ptr(), *(t.data_ptr() for t in pi), relu, p0.data_ptr()) if bn_in else (0,) * 7
    assert lib.dk_pwconv_dgrad_bnbwd_f32(g.data_ptr(), xo.data_ptr(), N, H, W, K, *(t.data_ptr() for t in po), relu,
                                         k12.data_ptr(), dy.data_ptr(), w.data_ptr(), C, dx0.data_ptr(),
                                         res.data_ptr() if resid else 0, *bn_args, st) in (0, 10100)
    # the fused kernel
    rows1 = lib.dk_pwconv_bwd_fused_rows(N, H, W, K, C)
    assert rows1 > 0
    nb = lib.dk_pwconv_bwd_fused_workspace_bytes(N, H, W, K, C)
    ws = torch.empty(nb // 4 + 4, dtype=torch.float32, device="cuda")
    dx1 = torch.full_like(xin, float("nan"))
    dw = torch.full((K, C), float("nan"), device="cuda")
    p1 = torch.full((rows1, 2, C), float("nan"), dtype=torch.float64, device="cuda")
    bnb = (*(t.data_ptr() for t in pi), relu, p1.data_ptr()) if bn_in else (0,) * 6
    rc = lib.dk_pwconv_bwd_bnbwd_f32(g.data_ptr(), xo.data_ptr(), N, H, W, K, *(t.data_ptr() for t in po), relu,
                                     k12.data_ptr(), w.data_ptr(), C, l2, dw.data_ptr(), dx1.data_ptr(),
                                     res.data_ptr() if resid else 0, xin.data_ptr(), *bnb, ws.data_ptr(), nb, st)
    assert rc in (0, 10100)
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)
    if bn_in:
        assert _close_sums(p0, p1)
    dy64 = dy.permute(0, 2, 3, 1).reshape(M, K).double()
    xf = xin.permute(0, 2, 3, 1).reshape(M, C)
    if bn_in:
        xh = (pi[2] * ((xf - pi[0]) * pi[1]) + pi[3]).double()
        if relu:
            xh = xh.clamp_min(0.0)
    else:
        xh = xf.double()
    ref = dy64.t() @ xh + l2 * w.double()
    bound = 3e-5 * (dy64.abs().t() @ xh.abs()) + 1e-6
    assert bool(torch.isfinite(dw).all())
    assert bool(((dw.double() - ref).abs() <= bound).all()), float(((dw.double() - ref).abs() / bound).max())


@pytest.mark.parametrize("K,C", [(256, 256), (128, 64)])
def test_deep_fused_bwd_deterministic_and_in_bounds(K, C):
    """The fused deep backward twice on the same inputs: dx and dW bitwise equal run to run (fixed-order
    reductions, no atomics); a ragged pixel count writes nothing past dx, the weight-gradient partial rows
    or the BatchNorm partial rows (sentinels; C = 64: the column group's idle half writes nothing)."""
    N, H, W = 3, 7, 5
    M = N * H * W
    rng = np.random.RandomState(5)
    st = stream_handle()
    xo, g = nhwc(rng.randn(N, K, H, W)), nhwc(rng.randn(N, K, H, W))
    po = bn_params(K, rng)
    k12 = torch.as_tensor(rng.randn(2 * K).astype(np.float32) * 0.1, device="cuda")
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
    xin = nhwc(rng.randn(N, C, H, W))
    pi = bn_params(C, rng)
    nb = lib.dk_pwconv_bwd_fused_workspace_bytes(N, H, W, K, C)
    rows = lib.dk_pwconv_bwd_fused_rows(N, H, W, K, C)
    outs = []
    for _ in range(2):
        ws = torch.full((nb // 4 + 4096,), 54321.0, dtype=torch.float32, device="cuda")
        dxbuf = torch.full((M * C + 4096,), 12345.0, device="cuda")
        dw = torch.empty((K, C), device="cuda")
        pbuf = torch.full((rows * 2 * C + 1024,), 777.0, dtype=torch.float64, device="cuda")
        part = pbuf[:rows * 2 * C].view(rows, 2, C)
        rc = lib.dk_pwconv_bwd_bnbwd_f32(g.data_ptr(), xo.data_ptr(), N, H, W, K, *(t.data_ptr() for t in po), 1,
                                         k12.data_ptr(), w.data_ptr(), C, 1e-4, dw.data_ptr(), dxbuf.data_ptr(), 0,
                                         xin.data_ptr(), *(t.data_ptr() for t in pi), 1, part.data_ptr(),
                                         ws.data_ptr(), nb, st)
        assert rc in (0, 10100)
        torch.cuda.synchronize()
        assert bool((dxbuf[M * C:] == 12345.0).all()) and bool(torch.isfinite(dxbuf[:M * C]).all())
        assert bool((ws[nb // 4:] == 54321.0).all()) and bool((pbuf[rows * 2 * C:] == 777.0).all())
        outs.append((dxbuf.clone(), dw.clone(), part.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][2], outs[1][2])


@pytest.mark.parametrize("K,C,N,H,W", [(256, 128, 3, 14, 14), (512, 256, 5, 7, 7), (128, 128, 2, 9, 13),
                                       (512, 512, 1, 3, 5)])
def test_deep_plain_dgrad_matches_tiled_engine(K, C, N, H, W):
    """dk_pwconv_dgrad_f32 at stride 1 (the skip projections' input gradient into the compact lattice) on
    the deep dgrad kernels' plain form (no BatchNorm around dy) against the tiled engine: dx bitwise (the
    same MFMA k order), ragged pixel counts, nothing written past dx."""
    rng = np.random.RandomState(K + C + N + H)
    M = N * H * W
    dy = nhwc(rng.randn(N, K, H, W))
    w = torch.as_tensor((rng.randn(K, C) / np.sqrt(K)).astype(np.float32), device="cuda")
    st = stream_handle()

    def run():
        buf = torch.full((M * C + 64,), 12345.0, device="cuda")
        assert lib.dk_pwconv_dgrad_f32(dy.data_ptr(), N, H, W, K, w.data_ptr(), C, 1, buf.data_ptr(), st) == 0
        torch.cuda.synchronize()
        assert bool((buf[M * C:] == 12345.0).all())
        return buf[:M * C].clone()
    d0, d1 = _modes(run)
    assert torch.equal(d0, d1)
    ref = dy.permute(0, 2, 3, 1).reshape(M, K).double() @ w.double()
    assert float((d1.double().reshape(M, C) - ref).norm() / ref.norm()) < 1e-5
