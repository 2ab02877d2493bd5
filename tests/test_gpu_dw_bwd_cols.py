"""The fused stride-1 depthwise backward with two output columns per thread
(dk_dwconv_bwd_bnbwd_bf16 / _f32, knob 21 = 2, the default where W >= 12) against the one-column form
(knob 21 = 1): dx bit-identical (same dy values, same tap order), the input BatchNorm's backward
partial sums to fp64 rounding and the weight gradient to fp32 rounding (a thread now sums two
pixels before the block reduction).  The one-column form's parity with the unfused sequence is
test_gpu_bf16.py's; the network's with the oracle test_gpu_bf16_fullsize.py's.
Reference: depthwise_convolution.py:198-221 (backward_cp), batch_norm.py:125-174."""
import numpy as np
import pytest
import torch

from dorknet_amd._hip import lib, stream_handle, workspace

pytestmark = pytest.mark.gpu

BF16 = torch.bfloat16
COLS_KNOB = 21


def _h(rng, N, C, H, W, dt=BF16):
    a = torch.as_tensor(rng.randn(N, C, H, W).astype(np.float32), device="cuda").to(dt)
    return a.contiguous(memory_format=torch.channels_last)


def _bn(C, rng):
    return [torch.as_tensor(v.astype(np.float32), device="cuda") for v in
            (rng.randn(C) * 0.3, rng.rand(C) + 0.5, 1 + 0.3 * rng.randn(C), 0.2 * rng.randn(C))]


def _run(cols, g, x1, x, wd, po, k12, relu, pi, bn_relu, res, with_dx, with_part):
    N, C, H, W = x.shape
    lib.dk_debug_set_gemm_config(COLS_KNOB, cols)
    bf = x.dtype == BF16
    try:
        rows = (lib.dk_dwconv_bwd_bnbwd_bf16_stats_rows if bf else lib.dk_dwconv_bwd_bnbwd_stats_rows)(N, H, W, C)
        nb = (lib.dk_dwconv_bwd_bnbwd_bf16_workspace_bytes if bf else lib.dk_dwconv_bwd_bnbwd_workspace_bytes)(
            N, H, W, C, 3, 3)
        ws = torch.empty(nb // 4 + 64, dtype=torch.float32, device="cuda")
        part = torch.full((rows, 2, C), float("nan"), dtype=torch.float64, device="cuda") if with_part else None
        dx = torch.full_like(x, float("nan")) if with_dx else None
        dw = torch.full_like(wd, float("nan"))
        bn = (*(t.data_ptr() for t in pi), bn_relu) if pi is not None else (0,) * 5
        rc = (lib.dk_dwconv_bwd_bnbwd_bf16 if bf else lib.dk_dwconv_bwd_bnbwd_f32)(g.data_ptr(), x1.data_ptr(), N, H, W, C, *(t.data_ptr() for t in po), relu,
                                          k12.data_ptr(), x.data_ptr(), wd.data_ptr(), 3, 3, 1, 1e-3, dw.data_ptr(),
                                          dx.data_ptr() if with_dx else 0, res.data_ptr() if res is not None else 0,
                                          *bn, part.data_ptr() if with_part else 0, ws.data_ptr(), nb, stream_handle())
        torch.cuda.synchronize()
    finally:
        lib.dk_debug_set_gemm_config(COLS_KNOB, -1)
    assert rc in (0, 10100), rc
    return rows, dx, dw, part


@pytest.mark.parametrize("N,H,W,C", [(2, 56, 56, 64), (3, 28, 28, 128), (4, 14, 14, 256), (2, 13, 19, 64),
                                     (2, 9, 12, 128), (1, 5, 40, 256)])
@pytest.mark.parametrize("relu,bn_in,stats,resid,with_dx", [(0, True, True, False, True), (1, True, True, True, True),
                                                            (1, True, False, False, True),
                                                            (0, False, False, True, True),
                                                            (1, False, False, False, False)])
@pytest.mark.parametrize("dt", [BF16, torch.float32], ids=["bf16", "f32"])
def test_two_columns_match_one(N, H, W, C, relu, bn_in, stats, resid, with_dx, dt):
    rng = np.random.RandomState(N * 7 + H + W + C + 2 * relu + 3 * bn_in + 5 * resid)
    g, x1, x = _h(rng, N, C, H, W, dt), _h(rng, N, C, H, W, dt), _h(rng, N, C, H, W, dt)
    res = _h(rng, N, C, H, W, dt) if resid else None
    po = _bn(C, rng)
    pi = _bn(C, rng) if bn_in else None
    k12 = torch.as_tensor(rng.randn(2 * C).astype(np.float32) * 0.1, device="cuda")
    wd = torch.as_tensor(rng.randn(C, 3, 3).astype(np.float32) * 0.3, device="cuda")
    args = (g, x1, x, wd, po, k12, relu, pi, 1, res, with_dx, stats)
    rows1, dx1, dw1, p1 = _run(1, *args)
    rows2, dx2, dw2, p2 = _run(2, *args)
    assert rows2 <= rows1  # two columns per thread: at most as many strips
    if with_dx:
        assert torch.equal(dx1, dx2)
    assert bool(torch.isfinite(dw2).all())
    err = float((dw2 - dw1).norm() / dw1.norm())
    assert err < 2e-6, err
    if stats:
        s1, s2 = p1.sum(0), p2.sum(0)
        assert float((s2 - s1).norm() / s1.norm()) < 1e-12


def test_geometry():
    """Two columns per thread where the width allows (W >= 12, C / 4 a multiple of 16), with the
    strip width that pads the row least; one column otherwise."""
    lib.dk_debug_set_gemm_config(COLS_KNOB, 1)
    try:
        one = {s: lib.dk_dwconv_bwd_bnbwd_bf16_stats_rows(*s) for s in [(64, 56, 56, 64), (64, 14, 14, 256),
                                                                       (64, 7, 7, 512)]}
    finally:
        lib.dk_debug_set_gemm_config(COLS_KNOB, -1)
    assert lib.dk_dwconv_bwd_bnbwd_bf16_stats_rows(64, 7, 7, 512) == one[(64, 7, 7, 512)]
    assert lib.dk_dwconv_bwd_bnbwd_bf16_stats_rows(64, 56, 56, 64) < one[(64, 56, 56, 64)]
    # the fp32 entries (and the join entry) have the same geometry
    assert lib.dk_dwconv_bwd_bnbwd_stats_rows(64, 56, 56, 64) == lib.dk_dwconv_bwd_bnbwd_bf16_stats_rows(64, 56, 56, 64)
