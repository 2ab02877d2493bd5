"""Config 3's size-dependent kernel paths at the real batch-256 shapes, through the layer API with
the network's fusions, against the torch fp64 twin (tests/_torch_twin.py, cross-checked against
the numpy oracle in tests/test_torch_twin.py).

The small-batch network tests cannot reach these paths' large-size behaviour: split-K grids
sized to one round of resident blocks, the XCD block remap on grids of thousands of tiles, BN
partial-row folds of thousands of rows (one-launch ticketed folds), the pointwise entries at
P = 802,816 pixels, the fused depthwise backward at res1's 256 x 64 x 56 x 56, and the stem
weight gradient with conv0_bn's backward on load at 256 x 3 x 225 x 225.  Each test also
records which C-ABI entry points ran, so it fails if a fusion stops being taken.

Tolerance: normwise relative 1e-4 for outputs, input and weight gradients, or
FP32_SLACK = 3x the error of the same maths evaluated in fp32 (the twin in float32, an
independent fp32 pipeline) where that is larger (tests/_convert.slack_bound).  At batch 256 the fp32 error itself reaches ~6e-4 on some
gradients: tens of millions of BN outputs per layer put a few within an ulp of the ReLU
threshold, and their masks flip between any two fp32 pipelines (measured: scripts/diag_fullsize.py,
profiles/r02_fullsize_conditioning.txt; at batch 16 every gradient agrees to ~1e-6).  A
BatchNorm whose output feeds a pointwise layer and another BatchNorm has dbeta = 0 in exact
arithmetic (the later BN's backward sums to zero); such sums are bounded by 1e-6 of their l1
scale sum|g| (fp64 partials on the GPU: far below fp32 summation error).
"""
import numpy as np
import pytest
import torch

from tests._convert import all_layers, log_slack, rel_err, slack_bound
from tests._torch_twin import TorchTwin

pytestmark = pytest.mark.gpu
TOL = 1e-4


class Calls:
    """Records the dk_* entry points called (wrapping dorknet_amd._hip.lib attributes)."""

    def __init__(self, monkeypatch, names):
        from dorknet_amd import _hip
        self.seen = set()
        for n in names:
            orig = getattr(_hip.lib, n)

            def w(*a, _o=orig, _n=n):
                self.seen.add(_n)
                return _o(*a)
            monkeypatch.setattr(_hip.lib, n, w)


def _perturb_bn(layers, rng):
    for l in TorchTwin._all(layers):
        if type(l).__name__ == "BatchNormLayer":
            C = l.incoming_chans
            l.learned_params["gamma"] = (1 + 0.2 * rng.standard_normal((1, C, 1, 1))).astype(np.float32)
            l.learned_params["beta"] = (0.1 * rng.standard_normal((1, C, 1, 1))).astype(np.float32)


def _run(layers, X, dY, input_grad, onehot=None, nhwc_input=False):
    """The layers as a FeedForwardNetwork on the GPU and the fp64 / fp32 twins.  With `onehot`
    the network ends in the reference's loss layer (SoftmaxWithCrossEntropy): Y = the
    probabilities, backward from the loss, and the losses are returned as twin.loss / twin32.loss
    / net._dk_loss."""
    from dorknet_amd.layers.losses import SoftmaxWithCrossEntropy
    from dorknet_amd.network.feed_forward_network import FeedForwardNetwork
    twin = TorchTwin(layers)                       # numpy parameters, before to_gpu
    net = FeedForwardNetwork("fullsize")
    for l in layers:
        net.add_layer(l)
    if onehot is not None:
        net.set_loss_layer(SoftmaxWithCrossEntropy("softmax1"))
    net.to_gpu()
    Xd = torch.as_tensor(X, device="cuda")
    if nhwc_input:  # as a previous block hands it over (channels-last storage)
        Xd = Xd.contiguous(memory_format=torch.channels_last)
    if onehot is None:
        dYd = torch.as_tensor(dY, device="cuda")
        _, Y = net.forward(Xd, None)
        dX = net.backward(dYd, input_grad=input_grad)
    else:
        dYd = None
        loss, Y = net.forward(Xd, torch.as_tensor(onehot, device="cuda"))
        dX = net.backward(input_grad=input_grad)
        net._dk_loss = float(loss)
    torch.cuda.synchronize()
    Yg = Y.float().cpu().numpy()
    dXg = dX.float().cpu().numpy() if input_grad else None
    grads = {(l.layer_name, k): l.grads[k].float().cpu().numpy()
             for l in all_layers(layers) for k in (l.grads or {})}
    del Xd, dYd, Y, dX
    Yt, dXt, gt = twin.run(X, dY, input_grad=input_grad, onehot=onehot)
    twin32 = TorchTwin(layers, np.float32)
    Y32, dX32, g32 = twin32.run(X, dY, input_grad=input_grad, onehot=onehot)
    if onehot is not None:
        twin.loss32 = twin32.loss
    return (Yg, dXg, grads), (Yt, dXt, gt), (Y32, dX32, g32), twin, net


def _bound(w, w32, extra=0.0):
    w = np.asarray(w, np.float64)
    return max(TOL * np.linalg.norm(w.ravel()), slack_bound(w, w32, 0.0), extra)


def _check(got, want, fp32, twin, layers):
    (Yg, dXg, gg), (Yt, dXt, gt), (Y32, dX32, g32) = got, want, fp32
    errs = {}
    e = np.linalg.norm((Yg - Yt).ravel())
    assert e <= _bound(Yt, Y32), ("Y", rel_err(Yg, Yt), rel_err(Y32, Yt))
    errs["Y"] = (rel_err(Yg, Yt), rel_err(Y32, Yt))
    if dXg is not None:
        e = np.linalg.norm((dXg - dXt).ravel())
        assert e <= _bound(dXt, dX32), ("dX", rel_err(dXg, dXt), rel_err(dX32, dXt))
        errs["dX"] = (rel_err(dXg, dXt), rel_err(dX32, dXt))
    bad = []
    for (name, k), w in gt.items():
        g = gg[(name, k)].reshape(w.shape).astype(np.float64)
        err = np.linalg.norm((g - w).ravel())
        extra = 1e-6 * float(torch.linalg.norm(twin.bn_l1[name])) if name in twin.bn_l1 else 0.0
        bound = _bound(w, g32[(name, k)].reshape(w.shape), extra)
        log_slack("fullsize {} {}".format(name, k), err, w, g32[(name, k)].reshape(w.shape))
        errs[(name, k)] = (rel_err(g, w), rel_err(g32[(name, k)].reshape(w.shape), w))
        if err > bound:
            bad.append((name, k, err, bound, rel_err(g, w)))
    print("errors (GPU vs fp64 twin, fp32 twin vs fp64 twin):")
    for k, (a, b) in errs.items():
        print("  {:40s} {:.3e} {:.3e}".format(str(k), a, b))
    assert not bad, bad
    # running statistics (first batch: running mean = batch mean, running std = batch std)
    for l in TorchTwin._all(layers):
        if l.layer_name in twin.bn_stats:
            m, s = twin.bn_stats[l.layer_name]
            assert rel_err(l.non_learned_params["running_mean"].cpu().numpy().ravel(), m.numpy()) <= 1e-6
            assert rel_err(l.non_learned_params["running_std"].cpu().numpy().ravel(), s.numpy()) <= 1e-6


FUSED = ["dk_pwconv_fwd_ex_f32", "dk_pwconv_dgrad_bnbwd_f32", "dk_pwconv_wgrad_bnx_f32", "dk_dwconv_bwd_bnbwd_f32",
         "dk_dwconv_fwd_ex_f32", "dk_bn_add_f32", "dk_relu_bwd_bn_partial_f64", "dk_conv2d_wgrad_bnbwd_f32",
         "dk_conv2d_fwd_ex_f32", "dk_bn_stats_from_partials_f32", "dk_bn_bwd_from_partials_f32",
         "dk_pwconv_bwd_bnbwd_f32", "dk_conv2d_fwd_narrow_f32", "dk_conv2d_wgrad_bnbwd_narrow_f32"]


@pytest.mark.parametrize("pw_fused_bwd", ["0", "1"])
def test_res1_full_size(monkeypatch, pw_fused_bwd):
    """pw0_bn + ReLU (applied on load by res1) and residual block res1 at 256 x 64 x 56 x 56:
    P = 802,816 pixels per pointwise GEMM, the fused stride-1 depthwise backward, BN folds of
    12,544 partial rows; the pointwise backward both as separate dgrad / wgrad launches and as
    the fused single pass."""
    from dorknet_amd._hip import lib
    monkeypatch.setenv("DORKNET_PW_FUSED_BWD", pw_fused_bwd)
    from examples.resnet18_depsep import ResNet18
    np.random.seed(31)
    layers = ResNet18("r18").layers[4:7]
    rng = np.random.default_rng(32)
    _perturb_bn(layers, rng)
    assert lib.dk_pwconv_fwd_stats_rows(256, 56, 56, 64, 64) > 256
    X = (0.5 + 2.0 * rng.standard_normal((256, 64, 56, 56), dtype=np.float32))
    dY = rng.standard_normal((256, 64, 56, 56), dtype=np.float32)
    calls = Calls(monkeypatch, FUSED)
    got, want, f32, twin, _ = _run(layers, X, dY, input_grad=True)
    pw_bwd = {"dk_pwconv_bwd_bnbwd_f32"} if pw_fused_bwd == "1" else {"dk_pwconv_dgrad_bnbwd_f32",
                                                                       "dk_pwconv_wgrad_bnx_f32"}
    assert pw_bwd | {"dk_pwconv_fwd_ex_f32", "dk_dwconv_bwd_bnbwd_f32", "dk_dwconv_fwd_ex_f32", "dk_bn_add_f32",
                     "dk_relu_bwd_bn_partial_f64"} <= calls.seen, calls.seen
    _check(got, want, f32, twin, layers)


@pytest.mark.parametrize("s2_fused", ["1", "0"])
def test_joins_full_size(monkeypatch, s2_fused):
    """res1 -> res2 -> res3 at batch 256: both residual-join fusions at full size -- res1's join
    backward in res2's fused stride-1 depthwise backward and res2's in res3's strided depthwise
    backward (dk_dwconv_bwd_bnbwd_join_f32; stride 2: the fused one-pass backward
    dk_dwconv_bwd_s2_bnbwd_join_f32, or with DORKNET_DW_S2_FUSED=0 the sub-pixel dgrad
    dk_dwconv_dgrad_join_f32: the join ReLU mask and the join BatchNorm's stage-1 partials on the
    dgrad store)."""
    monkeypatch.setenv("DORKNET_DW_S2_FUSED", s2_fused)
    from examples.resnet18_depsep import ResNet18
    np.random.seed(37)
    layers = ResNet18("r18").layers[6:9]
    rng = np.random.default_rng(38)
    _perturb_bn(layers, rng)
    X = np.abs(rng.standard_normal((256, 64, 56, 56), dtype=np.float32))   # a ReLU output
    dY = rng.standard_normal((256, 128, 28, 28), dtype=np.float32)
    calls = Calls(monkeypatch, FUSED + ["dk_dwconv_bwd_bnbwd_join_f32", "dk_dwconv_dgrad_join_f32",
                                        "dk_dwconv_bwd_s2_bnbwd_join_f32", "dk_dwconv_fwd_join_f32"])
    got, want, f32, twin, _ = _run(layers, X, dY, input_grad=True)
    s2 = "dk_dwconv_bwd_s2_bnbwd_join_f32" if s2_fused == "1" else "dk_dwconv_dgrad_join_f32"
    # both joins are formed by the next block's depthwise forward (res3's the stride-2 one, its skip
    # projection reading the written y)
    assert {"dk_dwconv_bwd_bnbwd_join_f32", s2, "dk_dwconv_fwd_join_f32"} <= calls.seen, calls.seen
    _check(got, want, f32, twin, layers)


def test_res7_res8_full_size(monkeypatch):
    """res7 (stride-2 depthwise, 256 -> 512 pointwise, stride-2 skip projection with the fused
    widen) and res8 (512 -> 512 pointwise at 7 x 7, P = 12,544) at batch 256."""
    from examples.resnet18_depsep import ResNet18
    np.random.seed(33)
    layers = ResNet18("r18").layers[12:14]
    rng = np.random.default_rng(34)
    _perturb_bn(layers, rng)
    X = np.abs(rng.standard_normal((256, 256, 14, 14), dtype=np.float32))   # a ReLU output
    dY = rng.standard_normal((256, 512, 7, 7), dtype=np.float32)
    calls = Calls(monkeypatch, FUSED)
    got, want, f32, twin, _ = _run(layers, X, dY, input_grad=True)
    assert {"dk_pwconv_fwd_ex_f32", "dk_pwconv_dgrad_bnbwd_f32", "dk_pwconv_wgrad_bnx_f32"} <= calls.seen
    _check(got, want, f32, twin, layers)


@pytest.mark.parametrize("narrow", ["1", "0"])
def test_stem_full_size(monkeypatch, narrow):
    """conv0 (64 x 3 x 5 x 5, stride 2) + conv0_bn + ReLU + pw0 (stride 2) + pw0_bn + ReLU on
    256 x 3 x 225 x 225: the stem weight gradient with conv0_bn's backward applied on load
    (the image gradient is not computed, as in the network's backward), conv0_bn's statistics
    folded in the forward launch -- through the narrow-input kernels on the NCHW image
    (dk_conv2d_*_narrow_f32, one partial row per block) and through the implicit GEMM on the
    NHWC4 copy (DORKNET_NARROW=0: dk_conv2d_wgrad_bnbwd_f32, 25,088 partial rows)."""
    monkeypatch.setenv("DORKNET_NARROW", narrow)
    from examples.resnet18_depsep import ResNet18
    np.random.seed(35)
    layers = ResNet18("r18").layers[0:6]
    rng = np.random.default_rng(36)
    _perturb_bn(layers, rng)
    X = rng.uniform(-128, 128, size=(256, 3, 225, 225)).astype(np.float32)
    dY = rng.standard_normal((256, 64, 56, 56), dtype=np.float32)
    calls = Calls(monkeypatch, FUSED)
    got, want, f32, twin, _ = _run(layers, X, dY, input_grad=False)
    expect = ({"dk_conv2d_wgrad_bnbwd_narrow_f32", "dk_conv2d_fwd_narrow_f32"} if narrow == "1" else
              {"dk_conv2d_wgrad_bnbwd_f32", "dk_conv2d_fwd_ex_f32"})
    assert expect <= calls.seen, calls.seen
    _check(got, want, f32, twin, layers)


@pytest.mark.parametrize("deep_bwd", [1, 0])
def test_res4_res6_full_size(monkeypatch, deep_bwd):
    """res4 (28 x 28 x 128), res5 (the stride-2 128 -> 256 block: strided depthwise, 128 -> 256
    pointwise, stride-2 skip projection) and res6 (14 x 14 x 256) at batch 256 through the fused
    network path (the middle blocks had no full-size check); the pointwise backward both
    as the fused deep pass (dgrad + weight gradient, dy never stored: dk_pwconv_bwd_bnbwd_f32 on
    pw_deep.hip's bwd_kernel, knob 14) and as the dgrad / side-stream weight-gradient pair."""
    from dorknet_amd._hip import lib
    from examples.resnet18_depsep import ResNet18
    lib.dk_debug_set_gemm_config(14, deep_bwd)
    np.random.seed(41)
    layers = ResNet18("r18").layers[9:12]
    assert [l.layer_name for l in layers] == ["res4", "res5", "res6"]
    rng = np.random.default_rng(42)
    _perturb_bn(layers, rng)
    X = np.abs(rng.standard_normal((256, 128, 28, 28), dtype=np.float32))   # res3's ReLU output
    dY = rng.standard_normal((256, 256, 14, 14), dtype=np.float32)
    calls = Calls(monkeypatch, FUSED + ["dk_dwconv_bwd_bnbwd_join_f32", "dk_dwconv_dgrad_join_f32",
                                        "dk_dwconv_bwd_s2_bnbwd_join_f32"])
    try:
        got, want, f32, twin, _ = _run(layers, X, dY, input_grad=True)
    finally:
        lib.dk_debug_set_gemm_config(14, -1)
    pw_bwd = {"dk_pwconv_bwd_bnbwd_f32"} if deep_bwd else {"dk_pwconv_dgrad_bnbwd_f32", "dk_pwconv_wgrad_bnx_f32"}
    assert pw_bwd | {"dk_pwconv_fwd_ex_f32", "dk_dwconv_fwd_ex_f32", "dk_bn_add_f32", "dk_dwconv_bwd_bnbwd_join_f32",
                     "dk_dwconv_bwd_s2_bnbwd_join_f32"} <= calls.seen, calls.seen
    if deep_bwd:
        assert "dk_pwconv_dgrad_bnbwd_f32" not in calls.seen, calls.seen
    _check(got, want, f32, twin, layers)


def test_res8_head_full_size(monkeypatch):
    """res8 (7 x 7 x 512) -> global average pooling -> dense 512 -> 120 -> softmax + cross-entropy
    at batch 256, backward from the loss ((p - y) / N, layers/losses.py:29-34): the network's
    head at the configuration's batch, loss with the l2 terms
    (feed_forward_network.py:54-60) against the twins'."""
    from examples.resnet18_depsep import ResNet18
    np.random.seed(43)
    layers = ResNet18("r18").layers[13:16]
    assert [l.layer_name for l in layers] == ["res8", "global_pool1", "dense1"]
    rng = np.random.default_rng(44)
    _perturb_bn(layers, rng)
    X = np.abs(rng.standard_normal((256, 512, 7, 7), dtype=np.float32))     # res7's ReLU output
    onehot = np.eye(120, dtype=np.float32)[rng.integers(0, 120, 256)]
    calls = Calls(monkeypatch, FUSED + ["dk_gap_join_fwd_f32", "dk_gap_bwd_f32", "dk_dense_fwd_f32", "dk_dense_dgrad_f32",
                                        "dk_dense_wgrad_f32", "dk_softmax_xent_fwd_f32", "dk_softmax_xent_bwd_f32"])
    got, want, f32, twin, net = _run(layers, X, None, input_grad=True, onehot=onehot, nhwc_input=True)
    # res8's join is pooled as it is formed (dk_gap_join_fwd_f32): no join pass, y never stored
    assert "dk_bn_add_f32" not in calls.seen, calls.seen
    assert {"dk_pwconv_fwd_ex_f32", "dk_pwconv_dgrad_bnbwd_f32", "dk_gap_join_fwd_f32", "dk_gap_bwd_f32", "dk_dense_fwd_f32",
            "dk_dense_dgrad_f32", "dk_dense_wgrad_f32", "dk_softmax_xent_fwd_f32",
            "dk_softmax_xent_bwd_f32"} <= calls.seen, calls.seen
    assert abs(net._dk_loss - twin.loss) <= max(TOL * abs(twin.loss), 3.0 * abs(twin.loss32 - twin.loss)), \
        (net._dk_loss, twin.loss, twin.loss32)
    _check(got, want, f32, twin, layers)
