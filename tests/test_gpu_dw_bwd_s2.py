"""The fused stride-2 depthwise backward (dk_dwconv_bwd_s2_bnbwd_f32 / _bf16: the following
BatchNorm's backward apply, the sub-pixel dgrad, the weight gradient and the input BatchNorm's
stage-1 partials in one pass, dy never stored) against the unfused sequence the network ran before:
dk_bn_bwd_apply (writes dy) -> dk_dwconv_dgrad_ex (stride 2, input-BN partials on the store) and
dk_dwconv_wgrad_bnx on that dy.
  * fp32: dx bit-identical (same dy values, same tap order), the partial sums to fp64 rounding, the
    weight gradient to fp32 rounding (per-block sums grouped differently);
  * bf16: the same kernel on bf16 storage keeps dy in fp32, so its dx is exactly the bf16 rounding of
    the fp32 kernel's dx on the same (bf16-valued) inputs, and its weight gradient is bit-identical.
Reference: depthwise_convolution.py:198-221 (backward_cp), batch_norm.py:125-174."""
import numpy as np
import pytest
import torch

from dorknet_amd._hip import lib, stream_handle, workspace

pytestmark = pytest.mark.gpu

BF16 = torch.bfloat16


def _t(rng, shape, dt=torch.float32):
    a = torch.as_tensor(rng.randn(*shape).astype(np.float32), device="cuda").to(BF16).to(dt)  # bf16 values
    return a.contiguous(memory_format=torch.channels_last)


def _bn(C, rng):
    return [torch.as_tensor(v.astype(np.float32), device="cuda") for v in
            (rng.randn(C) * 0.3, rng.rand(C) + 0.5, 1 + 0.3 * rng.randn(C), 0.2 * rng.randn(C))]


def _fused(dt, g, x1, x, po, relu, k12, wd, pi, bn_relu, res, with_dx, l2):
    N, C, H, W = x.shape
    OH, OW = x1.shape[2], x1.shape[3]
    rows = lib.dk_dwconv_bwd_s2_stats_rows(N, H, W, C)
    assert rows > 0
    nb = lib.dk_dwconv_bwd_s2_workspace_bytes(N, H, W, C)
    part = torch.full((rows, 2, C), float("nan"), dtype=torch.float64, device="cuda") if pi is not None else None
    dx = torch.full_like(x, float("nan")) if with_dx else None
    dw = torch.full_like(wd, float("nan"))
    fn = lib.dk_dwconv_bwd_s2_bnbwd_bf16 if dt == BF16 else lib.dk_dwconv_bwd_s2_bnbwd_f32
    bn = (*(t.data_ptr() for t in pi), bn_relu) if pi is not None else (0,) * 5
    rc = fn(g.data_ptr(), x1.data_ptr(), N, H, W, C, OH, OW, *(t.data_ptr() for t in po), relu, k12.data_ptr(),
            x.data_ptr(), wd.data_ptr(), l2, dw.data_ptr(), dx.data_ptr() if with_dx else 0,
            res.data_ptr() if res is not None else 0, *bn, part.data_ptr() if part is not None else 0,
            workspace.get(nb), nb, stream_handle())
    torch.cuda.synchronize()
    assert rc in (0, 10100), rc
    return dx, dw, part


@pytest.mark.parametrize("N,H,W,C", [(2, 56, 56, 64), (3, 28, 28, 128), (2, 14, 14, 256), (2, 13, 11, 64),
                                     (1, 9, 10, 512), (3, 7, 7, 32)])
@pytest.mark.parametrize("relu,bn_in,bn_relu,resid", [(1, True, 1, False), (0, True, 0, False), (1, False, 0, True),
                                                      (0, False, 0, False)])
def test_s2_fused_matches_unfused_f32(N, H, W, C, relu, bn_in, bn_relu, resid):
    rng = np.random.RandomState(N + H + 3 * W + C + 5 * relu + 7 * bn_in + 11 * resid)
    OH, OW = (H + 1) // 2, (W + 1) // 2
    g, x1 = _t(rng, (N, C, OH, OW)), _t(rng, (N, C, OH, OW))
    x = _t(rng, (N, C, H, W))
    res = _t(rng, (N, C, H, W)) if resid else None
    po, pi = _bn(C, rng), (_bn(C, rng) if bn_in else None)
    k12 = torch.as_tensor(rng.randn(2 * C).astype(np.float32) * 0.1, device="cuda")
    wd = torch.as_tensor(rng.randn(C, 3, 3).astype(np.float32) * 0.3, device="cuda")
    l2 = 1e-3
    st = stream_handle()
    # unfused: the BN backward apply writes dy, then the strided dgrad and the weight gradient on it
    dy = torch.empty_like(g)
    lib.dk_bn_bwd_apply_f32(x1.data_ptr(), g.data_ptr(), g.numel(), C, *(t.data_ptr() for t in po), relu,
                            k12.data_ptr(), dy.data_ptr(), st)
    dx0 = torch.empty_like(x)
    nbd = lib.dk_dwconv_dgrad_workspace_bytes(C, 3, 3)
    rows0 = lib.dk_dwconv_dgrad_join_rows(N, H, W, C, 3, 3, 2, 1)
    p0 = torch.zeros((rows0, 2, C), dtype=torch.float64, device="cuda") if bn_in else None
    bnd = (x.data_ptr(), *(t.data_ptr() for t in pi), bn_relu, p0.data_ptr()) if bn_in else (0,) * 7
    assert lib.dk_dwconv_dgrad_ex_f32(dy.data_ptr(), N, OH, OW, C, wd.data_ptr(), 3, 3, 2, 1, dx0.data_ptr(), H, W,
                                      workspace.get(nbd), nbd, res.data_ptr() if resid else 0, *bnd, st) in (0, 10100)
    dw0 = torch.empty_like(wd)
    nbw = lib.dk_dwconv_wgrad_workspace_bytes(N, OH, OW, C, 3, 3)
    wargs = (dy.data_ptr(), x.data_ptr(), N, H, W, C, 3, 3, 2, 1, OH, OW, wd.data_ptr(), l2, dw0.data_ptr(),
             workspace.get(nbw), nbw)
    if bn_in:
        lib.dk_dwconv_wgrad_bnx_f32(*wargs, *(t.data_ptr() for t in pi), bn_relu, st)
    else:
        lib.dk_dwconv_wgrad_f32(*wargs, st)
    torch.cuda.synchronize()
    dx1, dw1, p1 = _fused(torch.float32, g, x1, x, po, relu, k12, wd, pi, bn_relu, res, True, l2)
    assert torch.equal(dx0, dx1)
    err = float((dw1 - dw0).norm() / dw0.norm())
    assert err < 2e-6, err
    if bn_in:
        s0, s1 = p0.sum(0), p1.sum(0)
        assert float((s1 - s0).norm() / s0.norm()) < 1e-12
    # weight gradient only (dx NULL): the same weight gradient
    _, dw2, _ = _fused(torch.float32, g, x1, x, po, relu, k12, wd, pi, bn_relu, None, False, l2)
    assert torch.equal(dw1, dw2)


@pytest.mark.parametrize("N,H,W,C", [(4, 56, 56, 64), (4, 28, 28, 128), (4, 14, 14, 256), (2, 13, 11, 64)])
@pytest.mark.parametrize("relu,bn_relu", [(1, 1), (0, 0)])
def test_s2_fused_bf16_is_rounded_f32(N, H, W, C, relu, bn_relu):
    rng = np.random.RandomState(3 * N + H + W + C + relu)
    OH, OW = (H + 1) // 2, (W + 1) // 2
    g, x1 = _t(rng, (N, C, OH, OW), BF16), _t(rng, (N, C, OH, OW), BF16)
    x = _t(rng, (N, C, H, W), BF16)
    po, pi = _bn(C, rng), _bn(C, rng)
    k12 = torch.as_tensor(rng.randn(2 * C).astype(np.float32) * 0.1, device="cuda")
    wd = torch.as_tensor(rng.randn(C, 3, 3).astype(np.float32) * 0.3, device="cuda")
    f32 = [t.float().contiguous(memory_format=torch.channels_last) for t in (g, x1, x)]
    dxh, dwh, ph = _fused(BF16, g, x1, x, po, relu, k12, wd, pi, bn_relu, None, True, 0.0)
    dxf, dwf, pf = _fused(torch.float32, *f32, po, relu, k12, wd, pi, bn_relu, None, True, 0.0)
    assert torch.equal(dxh, dxf.to(BF16))
    assert torch.equal(dwh, dwf)
    s0, s1 = pf.sum(0), ph.sum(0)  # partials over the stored (rounded) dx: bf16 rounding apart
    assert float((s1 - s0).norm() / s0.norm()) < 1e-2


def test_s2_rejects_other_shapes():
    assert lib.dk_dwconv_bwd_s2_stats_rows(2, 14, 14, 6) == 0       # C % 4
    assert lib.dk_dwconv_bwd_s2_stats_rows(2, 14, 14, 1024 + 4) == 0  # C / 4 does not divide 256
    assert lib.dk_dwconv_bwd_s2_stats_rows(2, 14, 14, 64) > 0


@pytest.mark.parametrize("N,H,W,C", [(2, 56, 56, 64), (3, 28, 28, 128), (2, 14, 14, 256), (2, 13, 11, 64)])
@pytest.mark.parametrize("relu,lattice", [(1, 2), (0, 0), (1, None)])
def test_s2_join_matches_unfused_f32(N, H, W, C, relu, lattice):
    """The join form (dk_dwconv_bwd_s2_bnbwd_join_f32: the layer input is a residual block's output y,
    dx masked by y > 0, stage 1 of bn_j's backward on the store) against dk_bn_bwd_apply ->
    dk_dwconv_dgrad_join_f32 (stored mask) + dk_dwconv_wgrad_f32: dx bitwise, partials to fp64
    rounding, dW to fp32 rounding.  lattice: 2 = compact stride-2 residual, 0 = dense, None = none."""
    rng = np.random.RandomState(2 * N + H + W + C + relu + (lattice or 0))
    OH, OW = (H + 1) // 2, (W + 1) // 2
    g, x1 = _t(rng, (N, C, OH, OW)), _t(rng, (N, C, OH, OW))
    y = torch.relu(_t(rng, (N, C, H, W)))
    mask = (y > 0).to(torch.uint8).contiguous(memory_format=torch.channels_last)
    jx = _t(rng, (N, C, H, W))
    jm = torch.as_tensor((rng.randn(C) * 0.3).astype(np.float32), device="cuda")
    ji = torch.as_tensor((rng.rand(C) + 0.5).astype(np.float32), device="cuda")
    res = None if lattice is None else _t(rng, (N, C, OH, OW) if lattice == 2 else (N, C, H, W))
    po = _bn(C, rng)
    k12 = torch.as_tensor(rng.randn(2 * C).astype(np.float32) * 0.1, device="cuda")
    wd = torch.as_tensor(rng.randn(C, 3, 3).astype(np.float32) * 0.3, device="cuda")
    l2 = 1e-3
    st = stream_handle()
    dy = torch.empty_like(g)
    lib.dk_bn_bwd_apply_f32(x1.data_ptr(), g.data_ptr(), g.numel(), C, *(t.data_ptr() for t in po), relu,
                            k12.data_ptr(), dy.data_ptr(), st)
    dx0 = torch.empty_like(y)
    nbd = lib.dk_dwconv_dgrad_workspace_bytes(C, 3, 3)
    rows0 = lib.dk_dwconv_dgrad_join_rows(N, H, W, C, 3, 3, 2, 1)
    p0 = torch.zeros((rows0, 2, C), dtype=torch.float64, device="cuda")
    assert lib.dk_dwconv_dgrad_join_f32(dy.data_ptr(), N, OH, OW, C, wd.data_ptr(), 3, 3, 2, 1, dx0.data_ptr(), H, W,
                                        workspace.get(nbd), nbd, res.data_ptr() if res is not None else 0,
                                        lattice or 0, mask.data_ptr(), jx.data_ptr(), jm.data_ptr(), ji.data_ptr(),
                                        p0.data_ptr(), st) in (0, 10100)
    dw0 = torch.empty_like(wd)
    nbw = lib.dk_dwconv_wgrad_workspace_bytes(N, OH, OW, C, 3, 3)
    lib.dk_dwconv_wgrad_f32(dy.data_ptr(), y.data_ptr(), N, H, W, C, 3, 3, 2, 1, OH, OW, wd.data_ptr(), l2,
                            dw0.data_ptr(), workspace.get(nbw), nbw, st)
    torch.cuda.synchronize()
    rows = lib.dk_dwconv_bwd_s2_stats_rows(N, H, W, C)
    nb = lib.dk_dwconv_bwd_s2_workspace_bytes(N, H, W, C)
    p1 = torch.full((rows, 2, C), float("nan"), dtype=torch.float64, device="cuda")
    dx1, dw1 = torch.full_like(y, float("nan")), torch.full_like(wd, float("nan"))
    rc = lib.dk_dwconv_bwd_s2_bnbwd_join_f32(g.data_ptr(), x1.data_ptr(), N, H, W, C, OH, OW,
                                             *(t.data_ptr() for t in po), relu, k12.data_ptr(), y.data_ptr(),
                                             wd.data_ptr(), l2, dw1.data_ptr(), dx1.data_ptr(),
                                             res.data_ptr() if res is not None else 0, lattice or 0, jx.data_ptr(),
                                             jm.data_ptr(), ji.data_ptr(), p1.data_ptr(), workspace.get(nb), nb, st)
    torch.cuda.synchronize()
    assert rc in (0, 10100), rc
    assert torch.equal(dx0, dx1)
    err = float((dw1 - dw0).norm() / dw0.norm())
    assert err < 2e-6, err
    s0, s1 = p0.sum(0), p1.sum(0)
    assert float((s1 - s0).norm() / s0.norm()) < 1e-12
