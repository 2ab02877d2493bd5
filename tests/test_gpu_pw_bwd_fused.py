"""dk_pwconv_bwd_bnbwd_f32 (pointwise dgrad + wgrad + the following BN's backward apply + the
input BN's backward partials in one pass) against the unfused sequence the network ran before:
dk_pwconv_dgrad_bnbwd_f32 (which forms and stores dy) and dk_pwconv_wgrad_bnx_f32 on that dy.
dx is bit-identical (same dy values, same k-ordered MFMA chain, same residual add); the weight
gradient and the input BN's partial sums are fixed-order reductions grouped differently, so
they agree to fp32 / fp64 rounding.  Parity of the unfused sequence with the fp64 oracle is
covered in test_gpu_layers.py / test_gpu_network.py."""
import numpy as np
import pytest
import torch

from dorknet_amd._hip import lib, stream_handle, workspace

from .test_gpu_bn_on_load import _k12, args, bn_params, nhwc, same

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,C,relu,bn_in,resid,shape", [
    (64, 64, 1, True, False, (3, 13, 11)),      # ragged last 64-pixel tile
    (64, 64, 0, True, True, (4, 56, 56)),       # the res1 layer's per-image shape
    (64, 64, 1, True, False, (64, 56, 56)),     # streaming kernel: many tiles per wave
    (128, 64, 1, True, True, (2, 28, 28)),
    (64, 128, 0, False, False, (3, 9, 7)),
    (128, 128, 1, True, False, (5, 28, 28)),
    (128, 128, 0, False, True, (1, 1, 5)),      # a single partial tile
])
def test_pointwise_bwd_fused(K, C, relu, bn_in, resid, shape):
    rng = np.random.RandomState(K + C + relu + 2 * bn_in + 4 * resid + shape[1])
    N, H, W = shape
    xo = nhwc(rng.randn(N, K, H, W))        # this layer's output = the following BN's raw input
    g = nhwc(rng.randn(N, K, H, W))         # gradient w.r.t. that BN's (+ReLU) output
    po = bn_params(K, rng)
    k12 = _k12(K, rng)
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32) * 0.1, device="cuda")
    xin = nhwc(rng.randn(N, C, H, W))       # this layer's stored input (its input BN's raw input)
    pi = bn_params(C, rng)
    res = nhwc(rng.randn(N, C, H, W)) if resid else None
    l2 = 0.25
    st = stream_handle()

    # unfused: dgrad with BN-backward on load (writes dy) + the weight gradient on that dy
    dy0 = torch.empty_like(g)
    dx0 = torch.empty_like(xin)
    rows0 = lib.dk_pwconv_dgrad_bnbwd_stats_rows(N, H, W, K, C)
    part0 = torch.zeros((rows0, 2, C), dtype=torch.float64, device="cuda")
    bnd = (xin.data_ptr(), *args(pi, 1), part0.data_ptr()) if bn_in else (0, 0, 0, 0, 0, 0, 0)
    assert lib.dk_pwconv_dgrad_bnbwd_f32(g.data_ptr(), xo.data_ptr(), N, H, W, K, *args(po, relu), k12.data_ptr(),
                                         dy0.data_ptr(), w.data_ptr(), C, dx0.data_ptr(),
                                         res.data_ptr() if resid else 0, *bnd, st) == 0
    dw0 = torch.empty_like(w)
    nb = lib.dk_pwconv_wgrad_workspace_bytes(N, H, W, K, C)
    wa = (dy0.data_ptr(), xin.data_ptr(), N, H, W, C, K, 1, H, W, w.data_ptr(), l2, dw0.data_ptr(),
          workspace.get(nb), nb)
    if bn_in:
        assert lib.dk_pwconv_wgrad_bnx_f32(*wa, *args(pi, 1), st) == 0
    else:
        assert lib.dk_pwconv_wgrad_f32(*wa, st) == 0

    # fused
    rows1 = lib.dk_pwconv_bwd_fused_rows(N, H, W, K, C)
    assert rows1 > 0
    dx1 = torch.full_like(xin, float("nan"))
    dw1 = torch.full_like(w, float("nan"))
    part1 = torch.zeros((rows1, 2, C), dtype=torch.float64, device="cuda") if bn_in else None
    nb = lib.dk_pwconv_bwd_fused_workspace_bytes(N, H, W, K, C)
    assert lib.dk_pwconv_bwd_bnbwd_f32(g.data_ptr(), xo.data_ptr(), N, H, W, K, *args(po, relu), k12.data_ptr(),
                                       w.data_ptr(), C, l2, dw1.data_ptr(), dx1.data_ptr(),
                                       res.data_ptr() if resid else 0, xin.data_ptr(),
                                       *(args(pi, 1) if bn_in else (0, 0, 0, 0, 0)),
                                       part1.data_ptr() if bn_in else 0, workspace.get(nb), nb, st) == 0
    torch.cuda.synchronize()
    same(dx0, dx1)
    err = float((dw1 - dw0).norm() / dw0.norm())
    assert err < 2e-6, err
    if bn_in:
        s0, s1 = part0.sum(0), part1.sum(0)
        assert float((s1 - s0).norm() / s0.norm()) < 1e-12


def test_network_step_with_fused_pw_backward(monkeypatch):
    """The layer path (DORKNET_PW_FUSED_BWD=1) in a full ResNet training step: every parameter
    gradient matches the default (unfused) path to fp32 rounding."""
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    from dorknet_amd._tensor import as_device
    grads = []
    for flag in ("0", "1"):
        monkeypatch.setenv("DORKNET_PW_FUSED_BWD", flag)
        np.random.seed(0)
        net = ResNet18("r")
        net.to_gpu()
        X, _, onehot = synthetic_batch(4, seed=2, size=97)
        net.forward(as_device(X), as_device(onehot))
        net.backward()
        torch.cuda.synchronize()
        from tests._convert import all_layers
        grads.append({(l.layer_name, k): v.clone() for l in all_layers(net.layers) for k, v in (l.grads or {}).items()
                      if isinstance(v, torch.Tensor)})
    assert grads[0].keys() == grads[1].keys()
    for k in grads[0]:
        a, b = grads[0][k], grads[1][k]
        err = float((a - b).norm() / max(float(a.norm()), 1e-30))
        assert err < 1e-4, (k, err)


def test_pointwise_bwd_fused_rejects_other_shapes():
    # K = 512 (beyond the fused deep kernel's K in {128, 256}) and channel counts no kernel takes
    assert lib.dk_pwconv_bwd_fused_rows(2, 7, 7, 512, 512) == 0
    assert lib.dk_pwconv_bwd_fused_rows(2, 7, 7, 64, 48) == 0
    assert lib.dk_pwconv_bwd_fused_rows(2, 7, 7, 256, 64) == 0
    # K = C = 256: the fused deep kernel (pw_deep.hip bwd_kernel)
    assert lib.dk_pwconv_bwd_fused_rows(2, 7, 7, 256, 256) > 0


def test_bf16_pointwise_bwd_fused_shapes():
    # bf16: K = C = 64 (streaming form) and K in {128, 256} with C a multiple of 128 or K = 128 with
    # C = 64 (deep form, one column group)
    for K, C in [(64, 64), (128, 128), (256, 128), (256, 256), (128, 512), (128, 64)]:
        assert lib.dk_pwconv_bwd_fused_bf16_rows(2, 7, 7, K, C) > 0, (K, C)
    for K, C in [(512, 512), (256, 64), (64, 128), (256, 192)]:
        assert lib.dk_pwconv_bwd_fused_bf16_rows(2, 7, 7, K, C) == 0, (K, C)
