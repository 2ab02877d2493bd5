"""BN on load (dk_*_bnx_f32, dk_bn_add_f32): a consumer that applies the preceding
BatchNorm (+ReLU) as it loads its input must produce exactly -- bitwise -- what the
unfused sequence dk_bn_apply_f32 -> consumer produces (same bn_out arithmetic, padding 0).
Parity of the unfused sequence itself with the oracle is covered in test_gpu_layers.py."""
import numpy as np
import pytest
import torch

from dorknet_amd._hip import lib, stream_handle, tickets, workspace

pytestmark = pytest.mark.gpu


def nhwc(a):
    t = torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device="cuda")
    return t.contiguous(memory_format=torch.channels_last) if t.dim() == 4 else t


def bn_params(C, rng):
    mean = torch.as_tensor(rng.randn(C).astype(np.float32), device="cuda")
    invstd = torch.as_tensor((0.5 + rng.rand(C)).astype(np.float32), device="cuda")
    gamma = torch.as_tensor(rng.randn(C).astype(np.float32), device="cuda")
    beta = torch.as_tensor(rng.randn(C).astype(np.float32), device="cuda")
    return mean, invstd, gamma, beta


def args(p, relu):
    return (p[0].data_ptr(), p[1].data_ptr(), p[2].data_ptr(), p[3].data_ptr(), int(relu))


def apply(x, p, relu):
    y = torch.empty_like(x)
    lib.dk_bn_apply_f32(x.data_ptr(), x.numel(), x.shape[1], p[0].data_ptr(), p[1].data_ptr(), p[2].data_ptr(),
                        p[3].data_ptr(), int(relu), y.data_ptr(), 0, stream_handle())
    return y


def same(a, b):
    torch.cuda.synchronize()
    assert torch.equal(a, b), float((a - b).abs().max())


@pytest.mark.parametrize("stride,relu", [(1, 0), (1, 1), (2, 1), (2, 0)])
def test_pointwise_bnx_bitwise(stride, relu):
    rng = np.random.RandomState(stride * 10 + relu)
    N, C, H, W, K = 3, 24, 13, 11, 40
    x = nhwc(rng.randn(N, C, H, W))
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
    p = bn_params(C, rng)
    OH, OW = -(-H // stride), -(-W // stride)
    st = stream_handle()
    y0 = torch.empty((N, K, OH, OW), device="cuda").contiguous(memory_format=torch.channels_last)
    y1 = torch.empty_like(y0)
    xa = apply(x, p, relu)
    lib.dk_pwconv_fwd_f32(xa.data_ptr(), N, H, W, C, w.data_ptr(), K, stride, 0, y0.data_ptr(), OH, OW, st)
    lib.dk_pwconv_fwd_bnx_f32(x.data_ptr(), N, H, W, C, w.data_ptr(), K, stride, 0, y1.data_ptr(), OH, OW,
                              *args(p, relu), st)
    same(y0, y1)
    dy = nhwc(rng.randn(N, K, OH, OW))
    nb = lib.dk_pwconv_wgrad_workspace_bytes(N, OH, OW, K, C)
    g0 = torch.empty((K, C), device="cuda")
    g1 = torch.empty_like(g0)
    lib.dk_pwconv_wgrad_f32(dy.data_ptr(), xa.data_ptr(), N, H, W, C, K, stride, OH, OW, 0, 0.0, g0.data_ptr(),
                            workspace.get(nb), nb, st)
    lib.dk_pwconv_wgrad_bnx_f32(dy.data_ptr(), x.data_ptr(), N, H, W, C, K, stride, OH, OW, 0, 0.0, g1.data_ptr(),
                                workspace.get(nb), nb, *args(p, relu), st)
    same(g0, g1)


@pytest.mark.parametrize("stride,relu", [(1, 1), (2, 1), (1, 0)])
def test_depthwise_bnx_bitwise(stride, relu):
    rng = np.random.RandomState(7 + stride + relu)
    N, C, H, W, R = 2, 36, 15, 14, 3
    pad = 1
    x = nhwc(rng.randn(N, C, H, W))
    w = torch.as_tensor(rng.randn(C, R, R).astype(np.float32), device="cuda")
    p = bn_params(C, rng)
    OH, OW = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - R) // stride + 1
    st = stream_handle()
    w_rsc = torch.empty((R, R, C), device="cuda")
    lib.dk_dw_weight_rsc_f32(w.data_ptr(), C, R, R, w_rsc.data_ptr(), st)
    y0 = torch.empty((N, C, OH, OW), device="cuda").contiguous(memory_format=torch.channels_last)
    y1 = torch.empty_like(y0)
    xa = apply(x, p, relu)
    lib.dk_dwconv_fwd_f32(xa.data_ptr(), N, H, W, C, w_rsc.data_ptr(), R, R, stride, pad, 0, y0.data_ptr(), OH, OW,
                          st)
    lib.dk_dwconv_fwd_bnx_f32(x.data_ptr(), N, H, W, C, w_rsc.data_ptr(), R, R, stride, pad, 0, y1.data_ptr(), OH, OW,
                              *args(p, relu), st)
    same(y0, y1)
    dy = nhwc(rng.randn(N, C, OH, OW))
    nb = lib.dk_dwconv_wgrad_workspace_bytes(N, OH, OW, C, R, R)
    g0 = torch.empty((C, R, R), device="cuda")
    g1 = torch.empty_like(g0)
    lib.dk_dwconv_wgrad_f32(dy.data_ptr(), xa.data_ptr(), N, H, W, C, R, R, stride, pad, OH, OW, 0, 0.0,
                            g0.data_ptr(), workspace.get(nb), nb, st)
    lib.dk_dwconv_wgrad_bnx_f32(dy.data_ptr(), x.data_ptr(), N, H, W, C, R, R, stride, pad, OH, OW, 0, 0.0,
                                g1.data_ptr(), workspace.get(nb), nb, *args(p, relu), st)
    same(g0, g1)


def test_conv_bnx_bitwise():
    rng = np.random.RandomState(3)
    N, C, H, W, K, R, pad, stride = 2, 12, 10, 9, 20, 3, 1, 1
    x = nhwc(rng.randn(N, C, H, W))
    w = torch.as_tensor(rng.randn(K, C, R, R).astype(np.float32), device="cuda")
    p = bn_params(C, rng)
    OH, OW = H, W
    st = stream_handle()
    w_krsc = torch.empty((K, R, R, C), device="cuda")
    lib.dk_conv_weight_krsc_f32(w.data_ptr(), K, C, R, R, C, w_krsc.data_ptr(), st)
    y0 = torch.empty((N, K, OH, OW), device="cuda").contiguous(memory_format=torch.channels_last)
    y1 = torch.empty_like(y0)
    xa = apply(x, p, 1)
    lib.dk_conv2d_fwd_f32(xa.data_ptr(), N, H, W, C, w_krsc.data_ptr(), K, R, R, stride, pad, 0, y0.data_ptr(), OH,
                          OW, st)
    lib.dk_conv2d_fwd_bnx_f32(x.data_ptr(), N, H, W, C, w_krsc.data_ptr(), K, R, R, stride, pad, 0, y1.data_ptr(),
                              OH, OW, *args(p, 1), st)
    same(y0, y1)
    dy = nhwc(rng.randn(N, K, OH, OW))
    nb = lib.dk_conv2d_wgrad_workspace_bytes(N, OH, OW, K, C, R, R)
    g0 = torch.empty((K, C, R, R), device="cuda")
    g1 = torch.empty_like(g0)
    lib.dk_conv2d_wgrad_f32(dy.data_ptr(), xa.data_ptr(), N, H, W, C, C, K, R, R, stride, pad, OH, OW, 0, 0.0,
                            g0.data_ptr(), workspace.get(nb), nb, st)
    lib.dk_conv2d_wgrad_bnx_f32(dy.data_ptr(), x.data_ptr(), N, H, W, C, C, K, R, R, stride, pad, OH, OW, 0, 0.0,
                                g1.data_ptr(), workspace.get(nb), nb, *args(p, 1), st)
    same(g0, g1)


@pytest.mark.parametrize("bn_a,bn_b", [(True, False), (True, True), (False, True)])
def test_bn_add_bitwise(bn_a, bn_b):
    rng = np.random.RandomState(int(bn_a) * 2 + int(bn_b))
    N, C, H, W = 2, 20, 7, 9
    a = nhwc(rng.randn(N, C, H, W))
    b = nhwc(rng.randn(N, C, H, W))
    pa, pb = bn_params(C, rng), bn_params(C, rng)
    st = stream_handle()
    a0 = apply(a, pa, 0) if bn_a else a
    b0 = apply(b, pb, 1) if bn_b else b
    n = a.numel()
    y0 = torch.empty_like(a)
    m0 = torch.empty(a.shape, dtype=torch.uint8, device="cuda").contiguous(memory_format=torch.channels_last)
    lib.dk_add_f32(a0.data_ptr(), b0.data_ptr(), n, 1, y0.data_ptr(), m0.data_ptr(), st)
    y1 = torch.empty_like(a)
    m1 = torch.empty_like(m0)
    none = (0, 0, 0, 0, 0)
    lib.dk_bn_add_f32(a.data_ptr(), *(args(pa, 0) if bn_a else none), b.data_ptr(), *(args(pb, 1) if bn_b else none),
                      n, C, 1, y1.data_ptr(), m1.data_ptr(), st)
    same(y0, y1)
    same(m0, m1)


def _stats_pair(y, part, rows, C):
    """(mean, std) from the producer's partials and from a separate pass over y."""
    st = stream_handle()
    P = y.numel() // C
    out = []
    for use_part in (True, False):
        mean, std, invstd, rm, rs = [torch.empty(C, device="cuda") for _ in range(5)]
        if use_part:
            nb = lib.dk_bn_partials_workspace_bytes(rows, C)
            lib.dk_bn_stats_from_partials_f32(part.data_ptr(), rows, C, float(P), 1e-5, 0.95, 1, mean.data_ptr(),
                                              std.data_ptr(), invstd.data_ptr(), rm.data_ptr(), rs.data_ptr(),
                                              workspace.get(nb), nb, 0, st)
        else:
            nb = lib.dk_bn_stats_workspace_bytes(P, C)
            lib.dk_bn_stats_f32(y.data_ptr(), P, C, 1e-5, 0.95, 1, mean.data_ptr(), std.data_ptr(),
                                invstd.data_ptr(), rm.data_ptr(), rs.data_ptr(), workspace.get(nb), nb, st)
        out.append((mean, std))
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("kind,bn_in", [("pw", False), ("pw", True), ("conv", True), ("dw", False), ("dw", True)])
def test_producer_statistics(kind, bn_in):
    """*_fwd_ex_f32 with stats: y bit-identical to the plain forward, and mean/std from the
    epilogue partial sums equal to a separate statistics pass over y (to fp32 rounding)."""
    rng = np.random.RandomState(11)
    N, C, H, W = 3, 16, 37, 29   # ragged tiles: M = 3*37*29 is not a multiple of any tile
    K = 48
    x = nhwc(rng.randn(N, C, H, W) + 0.5)
    p = bn_params(C, rng)
    bargs = args(p, 1) if bn_in else (0, 0, 0, 0, 0)
    st = stream_handle()
    if kind == "pw":
        w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
        OH, OW = H, W
        rows = lib.dk_pwconv_fwd_stats_rows(N, OH, OW, K, C)
        Cout = K
        run = lambda yy, part: lib.dk_pwconv_fwd_ex_f32(x.data_ptr(), N, H, W, C, w.data_ptr(), K, 1, 0,  # noqa
                                                        yy.data_ptr(), OH, OW, *bargs, part, st)
    elif kind == "conv":
        w = torch.as_tensor(rng.randn(K, C, 3, 3).astype(np.float32), device="cuda")
        wk = torch.empty((K, 3, 3, C), device="cuda")
        lib.dk_conv_weight_krsc_f32(w.data_ptr(), K, C, 3, 3, C, wk.data_ptr(), st)
        OH, OW = H, W
        rows = lib.dk_conv2d_fwd_stats_rows(N, OH, OW, K, C, 3, 3)
        Cout = K
        run = lambda yy, part: lib.dk_conv2d_fwd_ex_f32(x.data_ptr(), N, H, W, C, wk.data_ptr(), K, 3, 3, 1, 1,  # noqa
                                                        0, yy.data_ptr(), OH, OW, *bargs, part, st)
    else:
        w = torch.as_tensor(rng.randn(C, 3, 3).astype(np.float32), device="cuda")
        wr = torch.empty((3, 3, C), device="cuda")
        lib.dk_dw_weight_rsc_f32(w.data_ptr(), C, 3, 3, wr.data_ptr(), st)
        OH, OW = H, W
        rows = lib.dk_dwconv_fwd_stats_rows(N, OH, OW, C, 1)
        Cout = C
        run = lambda yy, part: lib.dk_dwconv_fwd_ex_f32(x.data_ptr(), N, H, W, C, wr.data_ptr(), 3, 3, 1, 1, 0,  # noqa
                                                        yy.data_ptr(), OH, OW, *bargs, part, st)
    assert rows > 0
    y0 = torch.empty((N, Cout, OH, OW), device="cuda").contiguous(memory_format=torch.channels_last)
    y1 = torch.empty_like(y0)
    part = torch.empty((rows, 2, Cout), dtype=torch.float64, device="cuda")
    run(y0, 0)
    run(y1, part.data_ptr())
    same(y0, y1)
    (m1, s1), (m0, s0) = _stats_pair(y1, part, rows, Cout)
    assert torch.allclose(m1, m0, rtol=1e-6, atol=1e-6) and torch.allclose(s1, s0, rtol=1e-6, atol=0)


def _bwd_finalize(part, rows, C, P):
    st = stream_handle()
    dg, db, k12 = torch.empty(C, device="cuda"), torch.empty(C, device="cuda"), torch.empty(2 * C, device="cuda")
    nb = lib.dk_bn_partials_workspace_bytes(rows, C)
    lib.dk_bn_bwd_from_partials_f32(part.data_ptr(), rows, C, float(P), dg.data_ptr(), db.data_ptr(), k12.data_ptr(),
                                    workspace.get(nb), nb, 0, st)
    return dg, db, k12


def _bwd_reference(xbn, g, p, relu):
    """Stage 1 + 2 by the standalone passes (dk_bn_bwd_partial_f64 over xbn, g)."""
    st = stream_handle()
    C = xbn.shape[1]
    P = xbn.numel() // C
    nb = lib.dk_bn_workspace_bytes(P, C)
    part = torch.empty(nb // 8, dtype=torch.float64, device="cuda")
    lib.dk_bn_bwd_partial_f64(xbn.data_ptr(), g.data_ptr(), P, C, *args(p, relu)[:4], relu, part.data_ptr(), nb, st)
    return _bwd_finalize(part, lib.dk_bn_partial_blocks(P, C), C, P)


def _close(a, b):
    torch.cuda.synchronize()
    for u, v in zip(a, b):
        assert torch.allclose(u, v, rtol=1e-5, atol=1e-6 * float(v.abs().max()) + 1e-12), float((u - v).abs().max())


@pytest.mark.parametrize("stride,relu", [(1, 0), (2, 1)])
def test_pointwise_dgrad_bn_partials(stride, relu):
    """dgrad_ex: dx bit-identical to the plain dgrad, and the BN-backward sums of its
    epilogue equal the standalone reduction over (bn_x, dx)."""
    rng = np.random.RandomState(21 + stride)
    N, C, K, OH, OW = 3, 24, 40, 9, 7
    H, W = OH * stride, OW * stride
    dy = nhwc(rng.randn(N, K, OH, OW))
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
    xbn = nhwc(rng.randn(N, C, H, W))
    p = bn_params(C, rng)
    st = stream_handle()
    dx0 = torch.empty((N, C, H, W), device="cuda").contiguous(memory_format=torch.channels_last)
    dx1 = torch.empty_like(dx0)
    lib.dk_pwconv_dgrad_f32(dy.data_ptr(), N, OH, OW, K, w.data_ptr(), C, stride, dx0.data_ptr(), st)
    rows = lib.dk_pwconv_dgrad_stats_rows(N, OH, OW, K, C)
    part = torch.empty((rows, 2, C), dtype=torch.float64, device="cuda")
    lib.dk_pwconv_dgrad_ex_f32(dy.data_ptr(), N, OH, OW, K, w.data_ptr(), C, stride, dx1.data_ptr(), 0,
                               xbn.data_ptr(), *args(p, relu), part.data_ptr(), st)
    same(dx0, dx1)
    _close(_bwd_finalize(part, rows, C, N * H * W), _bwd_reference(xbn, dx0, p, relu))


def test_depthwise_dgrad_bn_partials():
    rng = np.random.RandomState(31)
    N, C, H, W = 2, 32, 11, 13
    dy = nhwc(rng.randn(N, C, H, W))
    w = torch.as_tensor(rng.randn(C, 3, 3).astype(np.float32), device="cuda")
    xbn = nhwc(rng.randn(N, C, H, W))
    p = bn_params(C, rng)
    st = stream_handle()
    nb = lib.dk_dwconv_dgrad_workspace_bytes(C, 3, 3)
    dx0 = torch.empty_like(dy)
    dx1 = torch.empty_like(dy)
    lib.dk_dwconv_dgrad_f32(dy.data_ptr(), N, H, W, C, w.data_ptr(), 3, 3, 1, 1, dx0.data_ptr(), H, W,
                            workspace.get(nb), nb, st)
    rows = lib.dk_dwconv_dgrad_stats_rows(N, H, W, C, 1)
    part = torch.empty((rows, 2, C), dtype=torch.float64, device="cuda")
    lib.dk_dwconv_dgrad_ex_f32(dy.data_ptr(), N, H, W, C, w.data_ptr(), 3, 3, 1, 1, dx1.data_ptr(), H, W,
                               workspace.get(nb), nb, 0, xbn.data_ptr(), *args(p, 1), part.data_ptr(), st)
    same(dx0, dx1)
    _close(_bwd_finalize(part, rows, C, N * H * W), _bwd_reference(xbn, dx0, p, 1))


@pytest.mark.parametrize("relu,C,H,W,R,pad", [(1, 32, 11, 13, 3, 1), (0, 64, 14, 14, 3, 1), (1, 16, 9, 10, 5, 2),
                                               (1, 128, 7, 7, 1, 0)])
def test_depthwise_strided_dgrad_bn_partials(relu, C, H, W, R, pad):
    """Stride 2 (the sub-pixel dgrad): dx bit-identical to the plain strided dgrad, and the input
    BatchNorm's stage-1 sums of its store (ReLU mask recomputed from the BN's raw input) equal
    the standalone reduction over (bn_x, dx)."""
    rng = np.random.RandomState(33 + C + R)
    N, st_ = 3, 2
    OH, OW = (H + 2 * pad - R) // st_ + 1, (W + 2 * pad - R) // st_ + 1
    dy = nhwc(rng.randn(N, C, OH, OW))
    w = torch.as_tensor(rng.randn(C, R, R).astype(np.float32), device="cuda")
    xbn = nhwc(rng.randn(N, C, H, W))
    p = bn_params(C, rng)
    st = stream_handle()
    nb = lib.dk_dwconv_dgrad_workspace_bytes(C, R, R)
    dx0 = torch.empty_like(xbn)
    dx1 = torch.full_like(xbn, float("nan"))
    lib.dk_dwconv_dgrad_f32(dy.data_ptr(), N, OH, OW, C, w.data_ptr(), R, R, st_, pad, dx0.data_ptr(), H, W,
                            workspace.get(nb), nb, st)
    rows = lib.dk_dwconv_dgrad_join_rows(N, H, W, C, R, R, st_, pad)
    assert rows > 0
    part = torch.empty((rows, 2, C), dtype=torch.float64, device="cuda")
    lib.dk_dwconv_dgrad_ex_f32(dy.data_ptr(), N, OH, OW, C, w.data_ptr(), R, R, st_, pad, dx1.data_ptr(), H, W,
                               workspace.get(nb), nb, 0, xbn.data_ptr(), *args(p, relu), part.data_ptr(), st)
    same(dx0, dx1)
    _close(_bwd_finalize(part, rows, C, N * H * W), _bwd_reference(xbn, dx0, p, relu))


def test_depthwise_strided_dgrad_bn_partials_bf16():
    """The same for bf16 storage: dx equal to the plain bf16 strided dgrad, the partials over the
    stored (rounded) dx against the standalone reduction on the widened tensors."""
    rng = np.random.RandomState(77)
    N, C, H, W, R, pad, st_ = 4, 64, 14, 14, 3, 1, 2
    OH, OW = 7, 7
    bf = torch.bfloat16
    dy = nhwc(rng.randn(N, C, OH, OW)).to(bf).contiguous(memory_format=torch.channels_last)
    w = torch.as_tensor(rng.randn(C, R, R).astype(np.float32), device="cuda")
    xbn = nhwc(rng.randn(N, C, H, W)).to(bf).contiguous(memory_format=torch.channels_last)
    p = bn_params(C, rng)
    st = stream_handle()
    nb = lib.dk_dwconv_dgrad_workspace_bytes(C, R, R)
    dx0 = torch.empty_like(xbn)
    dx1 = torch.full_like(xbn, float("nan"))
    lib.dk_dwconv_dgrad_ex_bf16(dy.data_ptr(), N, OH, OW, C, w.data_ptr(), R, R, st_, pad, dx0.data_ptr(), H, W,
                                workspace.get(nb), nb, 0, 0, 0, 0, 0, 0, 0, 0, st)
    rows = lib.dk_dwconv_dgrad_join_rows(N, H, W, C, R, R, st_, pad)
    part = torch.empty((rows, 2, C), dtype=torch.float64, device="cuda")
    lib.dk_dwconv_dgrad_ex_bf16(dy.data_ptr(), N, OH, OW, C, w.data_ptr(), R, R, st_, pad, dx1.data_ptr(), H, W,
                                workspace.get(nb), nb, 0, xbn.data_ptr(), *args(p, 1), part.data_ptr(), st)
    same(dx0, dx1)
    _close(_bwd_finalize(part, rows, C, N * H * W),
           _bwd_reference(xbn.float().contiguous(memory_format=torch.channels_last),
                          dx0.float().contiguous(memory_format=torch.channels_last), p, 1))


def test_relu_bwd_bn_partials():
    rng = np.random.RandomState(41)
    N, C, H, W = 2, 48, 9, 10
    dy = nhwc(rng.randn(N, C, H, W))
    xbn = nhwc(rng.randn(N, C, H, W))
    mask = torch.as_tensor((rng.rand(N, C, H, W) > 0.4).astype(np.uint8), device="cuda").contiguous(
        memory_format=torch.channels_last)
    p = bn_params(C, rng)
    st = stream_handle()
    n = dy.numel()
    P = n // C
    dx0 = torch.empty_like(dy)
    dx1 = torch.empty_like(dy)
    lib.dk_relu_bwd_f32(dy.data_ptr(), mask.data_ptr(), n, dx0.data_ptr(), st)
    nb = lib.dk_bn_workspace_bytes(P, C)
    part = torch.empty(nb // 8, dtype=torch.float64, device="cuda")
    lib.dk_relu_bwd_bn_partial_f64(dy.data_ptr(), mask.data_ptr(), xbn.data_ptr(), P, C, *args(p, 0),
                                   dx1.data_ptr(), part.data_ptr(), nb, st)
    same(dx0, dx1)
    _close(_bwd_finalize(part, lib.dk_bn_partial_blocks(P, C), C, P), _bwd_reference(xbn, dx0, p, 0))


@pytest.mark.parametrize("kind,stride", [("pw", 1), ("pw", 2), ("dw", 1), ("dw", 2)])
def test_dgrad_residual_bitwise(kind, stride):
    """dgrad_ex with a residual addend == plain dgrad followed by dk_add_f32, bitwise."""
    rng = np.random.RandomState(50 + stride)
    st = stream_handle()
    N, C = 2, 32
    if kind == "pw":
        K, OH, OW = 24, 7, 6
        H, W = OH * stride, OW * stride
        dy = nhwc(rng.randn(N, K, OH, OW))
        w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
        r = nhwc(rng.randn(N, C, H, W))
        dx0 = torch.empty_like(r)
        dx1 = torch.empty_like(r)
        lib.dk_pwconv_dgrad_f32(dy.data_ptr(), N, OH, OW, K, w.data_ptr(), C, stride, dx0.data_ptr(), st)
        lib.dk_pwconv_dgrad_ex_f32(dy.data_ptr(), N, OH, OW, K, w.data_ptr(), C, stride, dx1.data_ptr(), r.data_ptr(),
                                   0, 0, 0, 0, 0, 0, 0, st)
    else:
        H, W = 13, 12
        OH, OW = (H + 2 - 3) // stride + 1, (W + 2 - 3) // stride + 1
        dy = nhwc(rng.randn(N, C, OH, OW))
        w = torch.as_tensor(rng.randn(C, 3, 3).astype(np.float32), device="cuda")
        r = nhwc(rng.randn(N, C, H, W))
        dx0 = torch.empty_like(r)
        dx1 = torch.empty_like(r)
        nb = lib.dk_dwconv_dgrad_workspace_bytes(C, 3, 3)
        lib.dk_dwconv_dgrad_f32(dy.data_ptr(), N, OH, OW, C, w.data_ptr(), 3, 3, stride, 1, dx0.data_ptr(), H, W,
                                workspace.get(nb), nb, st)
        lib.dk_dwconv_dgrad_ex_f32(dy.data_ptr(), N, OH, OW, C, w.data_ptr(), 3, 3, stride, 1, dx1.data_ptr(), H, W,
                                   workspace.get(nb), nb, r.data_ptr(), 0, 0, 0, 0, 0, 0, 0, st)
    ref = torch.empty_like(r)
    lib.dk_add_f32(dx0.data_ptr(), r.data_ptr(), r.numel(), 0, ref.data_ptr(), 0, st)
    same(ref, dx1)


@pytest.mark.parametrize("rows,C", [(300, 16), (1000, 64), (12544, 64), (40000, 200), (65536, 48)])
def test_one_launch_fold(rows, C):
    """With tickets, a fold of > 256 partial rows runs in one launch (the last block to arrive
    folds the level-2 rows): bit-identical to the launch-per-level fold, twice in a row (the
    tickets are left zeroed), for statistics and backward coefficients."""
    rng = np.random.RandomState(rows % 97)
    part = torch.as_tensor(rng.randn(rows, 2, C) * 100 + 1000, dtype=torch.float64, device="cuda")
    part[:, 1, :] = part[:, 1, :].abs() * 1000
    st = stream_handle()
    nb = lib.dk_bn_partials_workspace_bytes(rows, C)
    tk = tickets.get(lib.dk_bn_fold_tickets_count(C))
    res = []
    for t in (0, tk, tk):
        o = [torch.full((C,), 3.0, device="cuda") for _ in range(5)]
        lib.dk_bn_stats_from_partials_f32(part.data_ptr(), rows, C, float(rows * 64), 1e-5, 0.95, 0,
                                          *[v.data_ptr() for v in o], workspace.get(nb), nb, t, st)
        b = [torch.empty(C, device="cuda"), torch.empty(C, device="cuda"), torch.empty(2 * C, device="cuda")]
        lib.dk_bn_bwd_from_partials_f32(part.data_ptr(), rows, C, float(rows * 64), *[v.data_ptr() for v in b],
                                        workspace.get(nb), nb, t, st)
        res.append(o + b)
    torch.cuda.synchronize()
    for r in res[1:]:
        for u, v in zip(res[0], r):
            same(u, v)


def _k12(C, rng):
    return torch.as_tensor(rng.randn(2 * C).astype(np.float32) * 0.1, device="cuda")


def bwd_apply(xo, g, p, relu, k12):
    out = torch.empty_like(g)
    lib.dk_bn_bwd_apply_f32(xo.data_ptr(), g.data_ptr(), g.numel(), g.shape[1], *args(p, relu)[:4], int(relu),
                            k12.data_ptr(), out.data_ptr(), stream_handle())
    return out


@pytest.mark.parametrize("relu,bn_in,resid,K", [(1, True, False, 40), (0, False, False, 64), (1, False, True, 200),
                                                 (1, True, True, 16)])
def test_pointwise_dgrad_bnbwd_bitwise(relu, bn_in, resid, K):
    """dk_pwconv_dgrad_bnbwd_f32 == dk_bn_bwd_apply_f32 -> dk_pwconv_dgrad_ex_f32, bitwise, for
    dx and the written-through dy; the input BN's partial sums to fp64 rounding (other tiles)."""
    rng = np.random.RandomState(relu + 2 * bn_in + 4 * resid + K)
    N, C, H, W = 3, 24, 13, 11
    xo = nhwc(rng.randn(N, K, H, W))        # this layer's output = the following BN's input
    g = nhwc(rng.randn(N, K, H, W))         # gradient w.r.t. that BN's (+ReLU) output
    po = bn_params(K, rng)
    k12 = _k12(K, rng)
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32), device="cuda")
    xin = nhwc(rng.randn(N, C, H, W))       # this layer's input BN's raw input
    pi = bn_params(C, rng)
    res = nhwc(rng.randn(N, C, H, W)) if resid else None
    st = stream_handle()
    rows = lib.dk_pwconv_dgrad_stats_rows(N, H, W, K, C)
    dy0 = bwd_apply(xo, g, po, relu, k12)
    dx0 = torch.empty_like(xin)
    part0 = torch.zeros((rows, 2, C), dtype=torch.float64, device="cuda")
    bn_args = (xin.data_ptr(), *args(pi, 1), part0.data_ptr()) if bn_in else (0, 0, 0, 0, 0, 0, 0)
    assert lib.dk_pwconv_dgrad_ex_f32(dy0.data_ptr(), N, H, W, K, w.data_ptr(), C, 1, dx0.data_ptr(),
                                      res.data_ptr() if resid else 0, *bn_args, st) == 0
    dy1 = torch.full_like(g, float("nan"))
    dx1 = torch.empty_like(xin)
    part1 = torch.zeros((lib.dk_pwconv_dgrad_bnbwd_stats_rows(N, H, W, K, C), 2, C), dtype=torch.float64,
                        device="cuda")
    bn_args = (xin.data_ptr(), *args(pi, 1), part1.data_ptr()) if bn_in else (0, 0, 0, 0, 0, 0, 0)
    assert lib.dk_pwconv_dgrad_bnbwd_f32(g.data_ptr(), xo.data_ptr(), N, H, W, K, *args(po, relu), k12.data_ptr(),
                                         dy1.data_ptr(), w.data_ptr(), C, dx1.data_ptr(),
                                         res.data_ptr() if resid else 0, *bn_args, st) == 0
    same(dy0, dy1)
    same(dx0, dx1)
    if bn_in:
        # its own column-tile width (row count): the per-tile partials fold to the same sums
        s0, s1 = part0.sum(0), part1.sum(0)
        assert float((s1 - s0).norm() / s0.norm()) < 1e-12


@pytest.mark.parametrize("relu,bn_in,resid,C,need_dx,runs", [(0, True, False, 64, True, -1),
                                                              (0, True, True, 32, True, -1),
                                                              (1, False, False, 16, True, -1),
                                                              (0, False, True, 128, True, -1),
                                                              (0, True, False, 8, False, -1),
                                                              (1, True, True, 256, True, -1),
                                                              (0, True, True, 64, True, 2),
                                                              (1, True, False, 256, True, 5)])
def test_depthwise_bwd_bnbwd(relu, bn_in, resid, C, need_dx, runs):
    """dk_dwconv_bwd_bnbwd_f32 (BN-backward apply + dgrad + wgrad in one pass) against the unfused
    sequence dk_bn_bwd_apply_f32 -> dk_dwconv_dgrad_ex_f32 + dk_dwconv_wgrad_bnx_f32: dx bitwise;
    the input BN's partial sums and the weight gradient (other summation orders) to fp32
    rounding.  runs > 0: the kernel's block target (knob 7) forces blocks that walk runs of
    several images (uneven: 3 images over 2 runs), as the full-size small-image layers do."""
    lib.dk_debug_set_gemm_config(7, runs)
    try:
        _depthwise_bwd_bnbwd(relu, bn_in, resid, C, need_dx)
    finally:
        lib.dk_debug_set_gemm_config(7, -1)


def _depthwise_bwd_bnbwd(relu, bn_in, resid, C, need_dx):
    rng = np.random.RandomState(relu + 2 * bn_in + 4 * resid + C + 8 * need_dx)
    N, H, W, R = 3, 13, 11, 3
    xo = nhwc(rng.randn(N, C, H, W))        # this layer's output = the following BN's input
    g = nhwc(rng.randn(N, C, H, W))         # gradient w.r.t. that BN's (+ReLU) output
    po = bn_params(C, rng)
    k12 = _k12(C, rng)
    w = torch.as_tensor(rng.randn(C, R, R).astype(np.float32), device="cuda")
    xin = nhwc(rng.randn(N, C, H, W))       # this layer's stored input (raw input of its input BN)
    pi = bn_params(C, rng)
    res = nhwc(rng.randn(N, C, H, W)) if resid else None
    st = stream_handle()
    rows = lib.dk_dwconv_dgrad_stats_rows(N, H, W, C, 1)
    dy0 = bwd_apply(xo, g, po, relu, k12)
    dx0 = torch.empty_like(xin)
    part0 = torch.zeros((rows, 2, C), dtype=torch.float64, device="cuda")
    nb = lib.dk_dwconv_dgrad_workspace_bytes(C, R, R)
    bnd = (xin.data_ptr(), *args(pi, 1), part0.data_ptr()) if bn_in else (0, 0, 0, 0, 0, 0, 0)
    assert lib.dk_dwconv_dgrad_ex_f32(dy0.data_ptr(), N, H, W, C, w.data_ptr(), R, R, 1, 1, dx0.data_ptr(), H, W,
                                      workspace.get(nb), nb, res.data_ptr() if resid else 0, *bnd, st) == 0
    dw0 = torch.empty_like(w)
    nb = lib.dk_dwconv_wgrad_workspace_bytes(N, H, W, C, R, R)
    wa = (dy0.data_ptr(), xin.data_ptr(), N, H, W, C, R, R, 1, 1, H, W, 0, 0.0, dw0.data_ptr(), workspace.get(nb), nb)
    if bn_in:
        assert lib.dk_dwconv_wgrad_bnx_f32(*wa, *args(pi, 1), st) == 0
    else:
        assert lib.dk_dwconv_wgrad_f32(*wa, st) == 0
    dx1 = torch.full_like(xin, float("nan")) if need_dx else None
    rows1 = lib.dk_dwconv_bwd_bnbwd_stats_rows(N, H, W, C)
    part1 = torch.zeros((rows1, 2, C), dtype=torch.float64, device="cuda") if (bn_in and need_dx) else None
    dw1 = torch.full_like(w, float("nan"))
    nb = lib.dk_dwconv_bwd_bnbwd_workspace_bytes(N, H, W, C, R, R)
    assert lib.dk_dwconv_bwd_bnbwd_f32(g.data_ptr(), xo.data_ptr(), N, H, W, C, *args(po, relu), k12.data_ptr(),
                                       xin.data_ptr(), w.data_ptr(), R, R, 1, 0.0, dw1.data_ptr(),
                                       dx1.data_ptr() if need_dx else 0, res.data_ptr() if (resid and need_dx) else 0,
                                       *(args(pi, 1) if bn_in else (0, 0, 0, 0, 0)),
                                       part1.data_ptr() if part1 is not None else 0, workspace.get(nb), nb, st) == 0
    torch.cuda.synchronize()
    if need_dx:
        same(dx0, dx1)
        if bn_in:
            s0, s1 = part0.sum(0), part1.sum(0)
            assert float((s1 - s0).norm() / s0.norm()) < 1e-12
    err = float((dw1 - dw0).norm() / dw0.norm())
    assert err < 1e-6, err


@pytest.mark.parametrize("relu,bn_in,Cp,K,R,stride", [(1, False, 4, 64, 5, 2), (0, True, 8, 16, 3, 1),
                                                        (1, True, 12, 32, 3, 2)])
def test_conv_wgrad_bnbwd_bitwise(relu, bn_in, Cp, K, R, stride):
    """dk_conv2d_wgrad_bnbwd_f32 == dk_bn_bwd_apply_f32 -> dk_conv2d_wgrad[_bnx]_f32, bitwise (dy is
    formed as it is loaded; the GEMM, its split and its reduction are unchanged)."""
    rng = np.random.RandomState(relu + 2 * bn_in + Cp + K + R)
    N, H, W, pad = 3, 17, 15, 1
    OH, OW = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - R) // stride + 1
    x = nhwc(rng.randn(N, Cp, H, W))
    xo = nhwc(rng.randn(N, K, OH, OW))
    g = nhwc(rng.randn(N, K, OH, OW))
    po = bn_params(K, rng)
    pi = bn_params(Cp, rng)
    k12 = _k12(K, rng)
    st = stream_handle()
    nb = lib.dk_conv2d_wgrad_workspace_bytes(N, OH, OW, K, Cp, R, R)
    dy = bwd_apply(xo, g, po, relu, k12)
    dw0 = torch.empty((K, Cp, R, R), device="cuda")
    a = (dy.data_ptr(), x.data_ptr(), N, H, W, Cp, Cp, K, R, R, stride, pad, OH, OW, 0, 0.0, dw0.data_ptr(),
         workspace.get(nb), nb)
    if bn_in:
        assert lib.dk_conv2d_wgrad_bnx_f32(*a, *args(pi, 1), st) == 0
    else:
        assert lib.dk_conv2d_wgrad_f32(*a, st) == 0
    dw1 = torch.full_like(dw0, float("nan"))
    assert lib.dk_conv2d_wgrad_bnbwd_f32(g.data_ptr(), xo.data_ptr(), x.data_ptr(), N, H, W, Cp, Cp, K, R, R, stride,
                                         pad, OH, OW, *args(po, relu), k12.data_ptr(), 0, 0.0, dw1.data_ptr(),
                                         workspace.get(nb), nb, *(args(pi, 1) if bn_in else (0, 0, 0, 0, 0)),
                                         st) == 0
    same(dw0, dw1)


@pytest.mark.parametrize("relu,C,K,R,stride,N,H,W", [(1, 3, 64, 5, 2, 3, 17, 15), (0, 1, 32, 3, 1, 2, 28, 28),
                                                       (1, 3, 16, 7, 2, 2, 30, 21)])
def test_conv_wgrad_bnbwd_narrow_bitwise(relu, C, K, R, stride, N, H, W):
    """dk_conv2d_wgrad_bnbwd_narrow_f32 == dk_bn_bwd_apply_f32 -> dk_conv2d_wgrad_narrow_f32, bitwise
    (dy is formed as it is staged; the row loop and the reduction are unchanged)."""
    rng = np.random.RandomState(relu + C + K + R)
    pad = 1
    OH, OW = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - R) // stride + 1
    x = torch.from_numpy(rng.randn(N, C, H, W).astype(np.float32)).cuda()  # NCHW
    xo = nhwc(rng.randn(N, K, OH, OW))
    g = nhwc(rng.randn(N, K, OH, OW))
    po = bn_params(K, rng)
    k12 = _k12(K, rng)
    w = torch.as_tensor(rng.randn(K, C, R, R).astype(np.float32), device="cuda")
    st = stream_handle()
    assert lib.dk_conv2d_narrow_preferred(N, C, H, W, K, R, R, stride, pad, OH, OW) == 1
    nb = lib.dk_conv2d_wgrad_narrow_workspace_bytes(N, C, H, W, K, R, R, stride, pad, OH, OW)
    dy = bwd_apply(xo, g, po, relu, k12)
    dw0 = torch.empty((K, C, R, R), device="cuda")
    assert lib.dk_conv2d_wgrad_narrow_f32(dy.data_ptr(), x.data_ptr(), N, C, H, W, K, R, R, stride, pad, OH, OW,
                                          w.data_ptr(), 1e-3, dw0.data_ptr(), workspace.get(nb), nb, st) == 0
    dw1 = torch.full_like(dw0, float("nan"))
    assert lib.dk_conv2d_wgrad_bnbwd_narrow_f32(g.data_ptr(), xo.data_ptr(), x.data_ptr(), N, C, H, W, K, R, R,
                                                stride, pad, OH, OW, *args(po, relu), k12.data_ptr(), 1, w.data_ptr(),
                                                1e-3, dw1.data_ptr(), workspace.get(nb), nb, st) == 0
    same(dw0, dw1)
    # g on the stride-2 lattice only (compact): the same weight gradient as the widened g, bitwise
    gc = nhwc(rng.randn(N, K, (OH + 1) // 2, (OW + 1) // 2))
    gw = torch.zeros((N, K, OH, OW), device="cuda").contiguous(memory_format=torch.channels_last)
    gw[:, :, ::2, ::2] = gc
    dw2 = torch.full_like(dw0, float("nan"))
    dw3 = torch.full_like(dw0, float("nan"))
    for gg, lat, out in ((gw, 1, dw2), (gc, 2, dw3)):
        assert lib.dk_conv2d_wgrad_bnbwd_narrow_f32(gg.data_ptr(), xo.data_ptr(), x.data_ptr(), N, C, H, W, K, R, R,
                                                    stride, pad, OH, OW, *args(po, relu), k12.data_ptr(), lat,
                                                    w.data_ptr(), 1e-3, out.data_ptr(), workspace.get(nb), nb,
                                                    st) == 0
    same(dw2, dw3)
    # and the weight gradient itself against a float64 torch reference
    ref = torch.nn.grad.conv2d_weight(x.double(), (K, C, R, R), dy.double().contiguous(), stride=stride,
                                      padding=pad) + 1e-3 * w.double()
    err = float((dw0.double() - ref).norm() / ref.norm())
    assert err < 1e-5, err


def test_network_bn_grad_deferral(monkeypatch):
    """pw -> BN -> ReLU -> dw -> BN -> pw -> BN -> ReLU: the fused backward (the apply of each BN
    that follows a pw layer runs in that layer's dgrad loader, the one after the dw layer in its
    one-pass backward) equals the layer-by-layer backward."""
    from dorknet_amd.layers.activations import ReLu
    from dorknet_amd.layers.batch_norm import BatchNormLayer
    from dorknet_amd.layers.depthwise_convolution import DepthwiseConvLayer
    from dorknet_amd.layers.pointwise_convolution import PointwiseConvLayer
    from dorknet_amd.layers._chain import chain_backward, chain_forward
    rng = np.random.RandomState(5)

    def build():
        r = np.random.RandomState(11)
        ls = [PointwiseConvLayer("p1", 1, (32, 16), with_bias=False), BatchNormLayer("b1", incoming_chans=32), ReLu("r1"),
              DepthwiseConvLayer("d1", filter_block_shape=(32, 3, 3), stride=1, padding=1, with_bias=False),
              BatchNormLayer("bd", incoming_chans=32),
              PointwiseConvLayer("p2", 1, (48, 32), with_bias=False), BatchNormLayer("b2", incoming_chans=48), ReLu("r2")]
        for l in ls:
            for k in list(l.learned_params or {}):
                l.learned_params[k] = r.randn(*l.learned_params[k].shape).astype(np.float32)
            l.to_gpu()
        return ls

    x = rng.randn(4, 16, 9, 10).astype(np.float32)
    dy = rng.randn(4, 48, 9, 10).astype(np.float32)
    outs = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("DORKNET_FUSE", fuse)
        ls = build()
        _, steps = chain_forward(ls, nhwc(x))
        dx = chain_backward(steps, nhwc(dy))
        torch.cuda.synchronize()
        outs.append([dx.float().cpu()] + [torch.as_tensor(l.grads[k]).float().cpu() if not torch.is_tensor(l.grads[k])
                                          else l.grads[k].float().cpu() for l in ls for k in sorted(l.grads or {})])
    names = ["dx"] + ["{}.{}".format(l.layer_name, k) for l in build() for k in sorted(l.grads or {})]
    for n, a, b in zip(names, *outs):
        # the fused depthwise backward (dk_dwconv_bwd_bnbwd_f32) sums its weight gradient and the
        # input BatchNorm's backward partials in other orders than the layer-by-layer kernels, so
        # everything upstream of d1 agrees to fp32 rounding rather than bitwise
        assert float((a - b).norm() / b.norm()) < 1e-5, n
