"""The tiled GEMM engine's launcher guards (gemm_engine.h: launch_occupancy / launch_igemm).

A launch whose static + dynamic LDS exceeds the CU's 160 KB makes the runtime abort the queue
(HSA_STATUS_ERROR_INVALID_ALLOCATION, seen once in round 3 with a 168 KB request); the launcher
refuses it with DK_ERR_ARGS instead.  The case: the BN-backward-on-load dgrad
(dk_pwconv_dgrad_bnbwd_f32) with a 1,024-channel BatchNorm table (2 float4 per channel = 32 KB of
dynamic LDS) forced onto row tile 9 (256 x 128 x 16, 4 x 2 waves: 136 KB of static LDS), 168 KB in
all.  The refused call must leave the stream usable: the next launch with the default tile runs
and agrees bitwise with another valid tile (the k order of the engine does not depend on the tile
shape), and the occupancy cached per dynamic-LDS size serves both sizes on one instantiation.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROW_KNOB, STREAM_KNOB = 0, 3
OVERSIZED_TILE, OTHER_TILE = 9, 16


def _dgrad(K, C, M, cfg, seed=5):
    from dorknet_amd._hip import lib, stream_handle
    g = torch.Generator(device="cuda").manual_seed(seed)
    dev = dict(device="cuda", dtype=torch.float32)
    gr = torch.randn((M, K), generator=g, **dev)
    x = torch.randn((M, K), generator=g, **dev)
    mean = 0.1 * torch.randn(K, generator=g, **dev)
    invstd = 1.0 + 0.1 * torch.rand(K, generator=g, **dev)
    gamma = 1.0 + 0.2 * torch.randn(K, generator=g, **dev)
    beta = 0.1 * torch.randn(K, generator=g, **dev)
    k12 = 0.01 * torch.randn(2 * K, generator=g, **dev)
    w = torch.randn((K, C), generator=g, **dev) / K ** 0.5
    dx = torch.full((M, C), float("nan"), **dev)
    lib.dk_debug_set_gemm_config(STREAM_KNOB, 0)
    lib.dk_debug_set_gemm_config(ROW_KNOB, cfg)
    try:
        lib.dk_pwconv_dgrad_bnbwd_f32(gr.data_ptr(), x.data_ptr(), 1, M, 1, K, mean.data_ptr(), invstd.data_ptr(),
                                      gamma.data_ptr(), beta.data_ptr(), 1, k12.data_ptr(), 0, w.data_ptr(), C,
                                      dx.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0, stream_handle())
    finally:
        lib.dk_debug_set_gemm_config(ROW_KNOB, -1)
        lib.dk_debug_set_gemm_config(STREAM_KNOB, -1)
    return dx


def test_oversized_lds_refused_and_stream_survives():
    from dorknet_amd._hip import DK_ERR_ARGS, HipError
    K, C, M = 1024, 128, 4096
    with pytest.raises(HipError) as e:
        _dgrad(K, C, M, OVERSIZED_TILE)
    assert "status {}".format(DK_ERR_ARGS) in str(e.value)
    # the same stream, right after: the default tile and another valid tile
    a = _dgrad(K, C, M, -1)
    b = _dgrad(K, C, M, OTHER_TILE)
    torch.cuda.synchronize()
    assert torch.isfinite(a).all()
    assert torch.equal(a, b)
    # the oversized tile at a table that fits (512 channels: 16 KB + 136 KB) still launches: the
    # guard is per dynamic size on one instantiation, not a cached verdict
    c = _dgrad(512, C, M, OVERSIZED_TILE)
    d = _dgrad(512, C, M, OTHER_TILE)
    torch.cuda.synchronize()
    assert torch.equal(c, d)
