"""The streaming pointwise kernels (csrc/pw_stream.hip, K = C = 64) against the tiled engine
they replace: dk_pwconv_dgrad_bnbwd_f32 == dk_bn_bwd_apply_f32 -> dk_pwconv_dgrad_ex_f32
bitwise for dx and the written-through dy (same MFMA k order), the input BatchNorm's partial
sums to fp64 rounding (one partial row per persistent block instead of one per tile); ragged
pixel counts, every epilogue option, and a large grid (several tiles per wave)."""
import numpy as np
import pytest
import torch

from dorknet_amd._hip import lib, stream_handle

pytestmark = pytest.mark.gpu


def nhwc(a):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device="cuda").contiguous(
        memory_format=torch.channels_last)


def bn_params(C, rng):
    return [torch.as_tensor(v.astype(np.float32), device="cuda") for v in
            (rng.randn(C) * 0.3, rng.rand(C) + 0.5, 1 + 0.3 * rng.randn(C), 0.2 * rng.randn(C))]


@pytest.mark.parametrize("relu,bn_in,resid,N,H,W", [(1, True, False, 3, 13, 11), (0, True, False, 2, 8, 8),
                                                    (1, False, True, 3, 13, 11), (1, True, True, 5, 7, 9),
                                                    (0, False, False, 1, 1, 3), (1, True, False, 64, 56, 56)])
def test_stream_dgrad_bnbwd_matches_tiled_engine(relu, bn_in, resid, N, H, W):
    K = C = 64
    rng = np.random.RandomState(relu + 2 * bn_in + 4 * resid + N)
    xo = nhwc(rng.randn(N, K, H, W))
    g = nhwc(rng.randn(N, K, H, W))
    po = bn_params(K, rng)
    k12 = torch.as_tensor(rng.randn(2 * K).astype(np.float32) * 0.1, device="cuda")
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
    xin = nhwc(rng.randn(N, C, H, W))
    pi = bn_params(C, rng)
    res = nhwc(rng.randn(N, C, H, W)) if resid else None
    st = stream_handle()
    # reference: the tiled engine (streaming kernels off)
    lib.dk_debug_set_gemm_config(3, 0)
    try:
        dy0 = torch.empty_like(g)
        lib.dk_bn_bwd_apply_f32(xo.data_ptr(), g.data_ptr(), g.numel(), K, *(t.data_ptr() for t in po), relu,
                                k12.data_ptr(), dy0.data_ptr(), st)
        dx0 = torch.empty_like(xin)
        rows0 = lib.dk_pwconv_dgrad_stats_rows(N, H, W, K, C)
        part0 = torch.zeros((rows0, 2, C), dtype=torch.float64, device="cuda")
        bn_args = (xin.data_ptr(), *(t.data_ptr() for t in pi), 1, part0.data_ptr()) if bn_in else (0,) * 7
        assert lib.dk_pwconv_dgrad_ex_f32(dy0.data_ptr(), N, H, W, K, w.data_ptr(), C, 1, dx0.data_ptr(),
                                          res.data_ptr() if resid else 0, *bn_args, st) == 0
    finally:
        lib.dk_debug_set_gemm_config(3, -1)
    rows1 = lib.dk_pwconv_dgrad_bnbwd_stats_rows(N, H, W, K, C)
    dy1 = torch.full_like(g, float("nan"))
    dx1 = torch.full_like(xin, float("nan"))
    part1 = torch.full((rows1, 2, C), float("nan"), dtype=torch.float64, device="cuda")
    bn_args = (xin.data_ptr(), *(t.data_ptr() for t in pi), 1, part1.data_ptr()) if bn_in else (0,) * 7
    assert lib.dk_pwconv_dgrad_bnbwd_f32(g.data_ptr(), xo.data_ptr(), N, H, W, K, *(t.data_ptr() for t in po), relu,
                                         k12.data_ptr(), dy1.data_ptr(), w.data_ptr(), C, dx1.data_ptr(),
                                         res.data_ptr() if resid else 0, *bn_args, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(dy0, dy1)
    assert torch.equal(dx0, dx1)
    if bn_in:
        assert rows1 < max(rows0, 2) or N * H * W <= 128  # one row per persistent block
        s0, s1 = part0.sum(0), part1.sum(0)
        assert float((s1 - s0).norm() / s0.norm()) < 1e-12


@pytest.mark.parametrize("bn,relu,stats,stride,bias,N,H,W", [(True, 1, True, 1, False, 3, 13, 11),
                                                           (True, 0, True, 2, False, 2, 13, 9),
                                                           (False, 0, True, 1, True, 2, 8, 8),
                                                           (True, 1, False, 1, False, 1, 1, 5),
                                                           (False, 0, False, 2, True, 3, 6, 7),
                                                           (True, 1, True, 2, False, 32, 112, 112)])
@pytest.mark.parametrize("KC", [64, 128])
def test_stream_fwd_ex_matches_tiled_engine(bn, relu, stats, stride, bias, N, H, W, KC):
    """dk_pwconv_fwd_ex_f32 at K = C = 64 and 128: y bitwise equal to the tiled engine (BN + ReLU
    on load, bias, stride-2 subsampling), output statistics to fp64 rounding."""
    K = C = KC
    rng = np.random.RandomState(int(bn) + 2 * relu + 4 * stats + 8 * stride + N)
    x = nhwc(rng.randn(N, C, H, W) * 2 + 0.3)
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
    b = torch.as_tensor(rng.randn(K).astype(np.float32), device="cuda") if bias else None
    pi = bn_params(C, rng)
    OH, OW = -(-H // stride), -(-W // stride)
    st = stream_handle()
    bn_args = (*(t.data_ptr() for t in pi), relu) if bn else (0, 0, 0, 0, 0)
    outs = []
    for mode in (0, 1):
        lib.dk_debug_set_gemm_config(3, mode)
        try:
            rows = lib.dk_pwconv_fwd_stats_rows(N, OH, OW, K, C)
            part = torch.full((rows, 2, K), float("nan"), dtype=torch.float64, device="cuda") if stats else None
            y = torch.full((N, K, OH, OW), float("nan"), device="cuda").contiguous(memory_format=torch.channels_last)
            assert lib.dk_pwconv_fwd_ex_f32(x.data_ptr(), N, H, W, C, w.data_ptr(), K, stride,
                                            b.data_ptr() if bias else 0, y.data_ptr(), OH, OW, *bn_args,
                                            part.data_ptr() if stats else 0, st) == 0
            torch.cuda.synchronize()
            outs.append((y, part, rows))
        finally:
            lib.dk_debug_set_gemm_config(3, -1)
    (y0, p0, r0), (y1, p1, r1) = outs
    assert torch.equal(y0, y1)
    if stats:
        s0, s1 = p0.sum(0), p1.sum(0)
        assert float((s1 - s0).norm() / s0.norm()) < 1e-12


def carve(shape, rng, tail=4096, fill=None):
    """An NHWC tensor of `shape` (N, C, H, W) at the start of a larger buffer whose `tail` floats
    after it hold a sentinel: returns (view, whole buffer, number of leading floats)."""
    N, C, H, W = shape
    n = N * C * H * W
    buf = torch.full((n + tail,), float("nan") if fill is None else 0.0, device="cuda")
    if fill is not None:
        buf[:n] = torch.as_tensor(np.ascontiguousarray(fill(N, H, W, C), dtype=np.float32).ravel(), device="cuda")
    buf[n:] = 12345.0
    view = buf[:n].view(N, H, W, C).permute(0, 3, 1, 2)  # NCHW logical, NHWC bytes
    return view, buf, n


def tail_ok(buf, n):
    return bool((buf[n:] == 12345.0).all())


@pytest.mark.parametrize("N,H,W", [(3, 13, 11), (1, 5, 7), (2, 9, 9)])
def test_stream_kernels_ragged_tail_untouched(N, H, W):
    """M = N*H*W not a multiple of 32: the streaming kernels' ragged last tile must neither write
    past y / dx / dy nor let rows past M reach the results (row offsets live in the
    range-checked vector offset of every buffer access).  Operands are carved from the start of
    larger buffers whose tails hold a sentinel; outputs must match the exactly-sized run."""
    assert (N * H * W) % 32
    K = C = 64
    rng = np.random.RandomState(N * 100 + H)
    nh = lambda N_, H_, W_, C_: rng.randn(N_, H_, W_, C_)  # noqa: E731
    st = stream_handle()
    # forward (BN on load, statistics)
    x, xb, xn = carve((N, C, H, W), rng, fill=nh)
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
    pi = bn_params(C, rng)
    y, yb, yn = carve((N, K, H, W), rng)
    rows = lib.dk_pwconv_fwd_stats_rows(N, H, W, K, C)
    part = torch.zeros((rows, 2, K), dtype=torch.float64, device="cuda")
    assert lib.dk_pwconv_fwd_ex_f32(x.data_ptr(), N, H, W, C, w.data_ptr(), K, 1, 0, y.data_ptr(), H, W,
                                    *(t.data_ptr() for t in pi), 1, part.data_ptr(), st) == 0
    y_exact = torch.full((N, K, H, W), float("nan"), device="cuda").contiguous(memory_format=torch.channels_last)
    part2 = torch.zeros_like(part)
    xc = x.contiguous(memory_format=torch.channels_last)
    assert lib.dk_pwconv_fwd_ex_f32(xc.data_ptr(), N, H, W, C, w.data_ptr(), K, 1, 0, y_exact.data_ptr(), H, W,
                                    *(t.data_ptr() for t in pi), 1, part2.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert tail_ok(yb, yn)
    assert torch.equal(y, y_exact)
    assert torch.equal(part, part2)

    # dgrad with BN backward on load (dy written through, residual, input partials)
    xo, _, _ = carve((N, K, H, W), rng, fill=nh)
    g, _, _ = carve((N, K, H, W), rng, fill=nh)
    po = bn_params(K, rng)
    k12 = torch.as_tensor(rng.randn(2 * K).astype(np.float32) * 0.1, device="cuda")
    res, _, _ = carve((N, C, H, W), rng, fill=nh)
    dy, dyb, dyn = carve((N, K, H, W), rng)
    dx, dxb, dxn = carve((N, C, H, W), rng)
    rows = lib.dk_pwconv_dgrad_bnbwd_stats_rows(N, H, W, K, C)
    part = torch.zeros((rows, 2, C), dtype=torch.float64, device="cuda")
    assert lib.dk_pwconv_dgrad_bnbwd_f32(g.data_ptr(), xo.data_ptr(), N, H, W, K, *(t.data_ptr() for t in po), 1,
                                         k12.data_ptr(), dy.data_ptr(), w.data_ptr(), C, dx.data_ptr(),
                                         res.data_ptr(), x.data_ptr(), *(t.data_ptr() for t in pi), 1,
                                         part.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert tail_ok(dyb, dyn) and tail_ok(dxb, dxn)
    assert bool(torch.isfinite(dx).all()) and bool(torch.isfinite(part).all())

    # fused backward (dgrad + wgrad)
    dx2, dx2b, dx2n = carve((N, C, H, W), rng)
    dw = torch.full_like(w, float("nan"))
    rows = lib.dk_pwconv_bwd_fused_rows(N, H, W, K, C)
    part = torch.zeros((rows, 2, C), dtype=torch.float64, device="cuda")
    from dorknet_amd._hip import workspace
    nb = lib.dk_pwconv_bwd_fused_workspace_bytes(N, H, W, K, C)
    assert lib.dk_pwconv_bwd_bnbwd_f32(g.data_ptr(), xo.data_ptr(), N, H, W, K, *(t.data_ptr() for t in po), 1,
                                       k12.data_ptr(), w.data_ptr(), C, 0.0, dw.data_ptr(), dx2.data_ptr(),
                                       res.data_ptr(), x.data_ptr(), *(t.data_ptr() for t in pi), 1,
                                       part.data_ptr(), workspace.get(nb), nb, st) == 0
    torch.cuda.synchronize()
    assert tail_ok(dx2b, dx2n)
    assert torch.equal(dx, dx2)
    assert bool(torch.isfinite(dw).all())
