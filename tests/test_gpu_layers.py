"""HIP path vs the oracle (fp64 restatement of the reference), layer by layer.

Tolerance: normwise relative error <= 1e-4 for fp32 outputs, input
gradients and weight gradients against the fp64-accumulated restatement.
"""
import numpy as np
import pytest
import torch

from oracle import ref
from oracle import net as O
from tests._convert import layer_to_oracle, log_slack, rel_err, slack_bound

pytestmark = pytest.mark.gpu
TOL = 1e-4


def dev(a):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device="cuda")


def host(t):
    return t.detach().float().cpu().numpy()


def check(name, got, want, tol=TOL, want32=None):
    """||got - want|| <= max(tol * ||want||, FP32_SLACK * ||want32 - want||): within 1e-4 of the
    fp64 restatement, or (for quantities that are ~0 in exact arithmetic, e.g. the shift
    gradient of a BN followed by another BN) no worse than 3x the reference's own fp32
    pipeline error (tests/_convert.py FP32_SLACK)."""
    got = host(got) if isinstance(got, torch.Tensor) else np.asarray(got)
    want = np.asarray(want, dtype=np.float64)
    assert got.shape == want.shape, f"{name}: shape {got.shape} != {want.shape}"
    err = np.linalg.norm((got.astype(np.float64) - want).ravel())
    bound = tol * np.linalg.norm(want.ravel())
    if want32 is not None:
        bound = max(bound, slack_bound(want, want32, 0.0))
        log_slack(name, err, want, want32)
    assert err <= bound or err == 0, f"{name}: err {err:.3e} > bound {bound:.3e} (rel {rel_err(got, want):.3e})"


def run_layer(layer, X, dY=None, rng=None, test_mode=False):
    """Forward (+ backward) through a dorknet_amd layer and its oracle twins (fp64 and the
    reference-faithful fp32)."""
    olayer = layer_to_oracle(layer)  # before to_gpu: same numpy weights
    o32 = layer_to_oracle(layer, np.float32)
    layer.to_gpu()
    Y = layer.forward(dev(X), test_mode=test_mode)
    Yo = olayer.forward(X.astype(np.float64), test_mode)
    check(f"{layer.layer_name} forward", Y, Yo, want32=o32.forward(X, test_mode))
    if dY is None:
        return layer, olayer
    dX = layer.backward(dev(dY))
    dXo = olayer.backward(dY.astype(np.float64))
    check(f"{layer.layer_name} dX", dX, dXo, want32=o32.backward(dY))
    for k in olayer.grads:
        check(f"{layer.layer_name} d{k}", layer.grads[k], olayer.grads[k], want32=o32.grads[k])
    return layer, olayer


CONV_CASES = [
    # K, C, R, S, stride, pad, N, H, W, bias, l2
    (8, 3, 5, 5, 2, 1, 2, 17, 17, False, 1e-4),     # conv0-like: C=3 (channel pad), strided dgrad
    (16, 16, 3, 3, 1, 1, 2, 9, 11, True, 0.0),      # non-square input, bias
    (32, 8, 4, 4, 2, 1, 3, 14, 14, False, 1e-4),    # MNIST conv_3-like
    (64, 64, 3, 3, 1, 1, 2, 14, 14, False, 0.0),    # BASELINE config 2 shape, small batch
    (40, 12, 3, 3, 1, 0, 2, 10, 10, True, 0.0),     # K not a multiple of 32, no padding
    (32, 1, 3, 3, 1, 1, 2, 28, 28, False, 1e-4),    # MNIST conv_1 (C=1)
    (130, 68, 3, 3, 1, 1, 1, 6, 5, False, 1e-4),    # K > 128 tile, ragged M
    (70, 5, 3, 3, 2, 1, 2, 33, 150, False, 0.0),    # sub-pixel dgrad: K % 4 != 0, 2 channel groups, 2 column tiles
    (8, 3, 7, 7, 2, 3, 1, 20, 19, True, 0.0),       # sub-pixel dgrad, 7x7 stem geometry
    (6, 20, 3, 3, 2, 1, 2, 9, 9, False, 0.0),       # strided, C > 16, K % 4 != 0: phase dgrad (dy padded)
    (128, 64, 3, 3, 2, 1, 2, 56, 56, False, 1e-4),  # the non-depthwise ResNet block's strided conv: phase dgrad
    (12, 24, 1, 1, 2, 0, 2, 10, 9, True, 0.0),      # 1x1 stride 2: phases without taps write zeros
    (6, 8, 3, 3, 1, 1, 2, 9, 9, False, 0.0),        # stride 1, K % 4 != 0: one phase, dy padded
    (16, 20, 4, 4, 3, 2, 1, 17, 13, False, 0.0),    # stride 3, even filter, ragged phases
    (64, 3, 5, 5, 2, 1, 2, 45, 61, False, 1e-4),    # the stem's filters, ragged 16-pixel row tiles (narrow path)
    (48, 1, 3, 3, 1, 2, 2, 9, 40, True, 0.0),       # narrow path: stride 1, pad 2, K not a multiple of 16
]


@pytest.mark.parametrize("narrow", ["1", "0"])
def test_conv_stem_paths(narrow, monkeypatch):
    """The stem shape through the narrow-input kernels and through the implicit GEMM."""
    monkeypatch.setenv("DORKNET_NARROW", narrow)
    test_conv_layer((64, 3, 5, 5, 2, 1, 2, 33, 35, False, 1e-4))


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_layer(case):
    from dorknet_amd.layers.convolution import ConvLayer
    from dorknet_amd.regularisers.l2 import l2
    K, C, R, S, st, pd, N, H, W, bias, s = case
    rng = np.random.RandomState(1)
    np.random.seed(2)
    layer = ConvLayer("c", (K, C, R, S), stride=st, padding=pd, with_bias=bias,
                      weight_regulariser=l2(s) if s else None)
    if bias:
        layer.learned_params["bias"] = rng.randn(K).astype(np.float32)
    X = rng.randn(N, C, H, W).astype(np.float32)
    OH = int((H + 2 * pd - R) / st + 1)
    OW = int((W + 2 * pd - S) / st + 1)
    dY = rng.randn(N, K, OH, OW).astype(np.float32)
    run_layer(layer, X, dY)


DW_CASES = [
    # C, R, S, stride, pad, N, H, W, bias
    (16, 3, 3, 1, 1, 2, 9, 9, False),
    (32, 3, 3, 2, 1, 2, 14, 14, False),   # stride-2 dw of res3/5/7 (58 -> 28.5 -> 28)
    (8, 3, 3, 2, 1, 2, 15, 15, True),
    (64, 3, 3, 1, 1, 3, 8, 8, False),
    (12, 5, 5, 1, 2, 2, 11, 11, True),
    (512, 3, 3, 1, 1, 2, 7, 7, False),    # res8 shape
    (8, 5, 5, 2, 2, 2, 13, 12, False),    # 5x5 stride-2 sub-pixel dgrad
    (4, 1, 1, 2, 0, 2, 9, 8, True),       # 1x1 stride-2
    (24, 3, 3, 2, 0, 1, 10, 11, False),   # stride 2 without a sub-pixel kernel (gather path)
]


@pytest.mark.parametrize("case", DW_CASES)
def test_depthwise_layer(case):
    from dorknet_amd.layers.depthwise_convolution import DepthwiseConvLayer
    C, R, S, st, pd, N, H, W, bias = case
    rng = np.random.RandomState(3)
    np.random.seed(4)
    layer = DepthwiseConvLayer("dw", (C, R, S), stride=st, padding=pd, with_bias=bias)
    if bias:
        layer.learned_params["bias"] = rng.randn(C).astype(np.float32)
    X = rng.randn(N, C, H, W).astype(np.float32)
    OH = int((H + 2 * pd - R) / st + 1)
    OW = int((W + 2 * pd - S) / st + 1)
    dY = rng.randn(N, C, OH, OW).astype(np.float32)
    run_layer(layer, X, dY)


PW_CASES = [
    # K, C, stride, N, H, W, bias, l2
    (64, 64, 2, 2, 12, 12, False, 1e-4),    # pw0 / skip projection (stride 2 + widen)
    (128, 64, 1, 2, 7, 7, False, 1e-4),
    (24, 40, 1, 3, 5, 6, True, 0.0),
    (512, 256, 2, 2, 14, 14, False, 1e-4),  # res7 skip
    (512, 512, 1, 4, 7, 7, False, 1e-4),    # res8 pw
    (16, 3, 1, 2, 9, 7, True, 1e-4),        # C % 4 != 0: zero-padded channels (the reference takes any C)
    (8, 6, 2, 3, 10, 10, False, 1e-4),      # C % 4 != 0 with stride 2 + widen
]


@pytest.mark.parametrize("case", PW_CASES)
def test_pointwise_layer(case):
    from dorknet_amd.layers.pointwise_convolution import PointwiseConvLayer
    from dorknet_amd.regularisers.l2 import l2
    K, C, st, N, H, W, bias, s = case
    rng = np.random.RandomState(5)
    np.random.seed(6)
    layer = PointwiseConvLayer("pw", stride=st, filter_block_shape=(K, C), with_bias=bias,
                               weight_regulariser=l2(s) if s else None)
    if bias:
        layer.learned_params["bias"] = rng.randn(K).astype(np.float32)
    X = rng.randn(N, C, H, W).astype(np.float32)
    dY = rng.randn(N, K, -(-H // st), -(-W // st)).astype(np.float32)
    run_layer(layer, X, dY)


@pytest.mark.parametrize("case", [(4, 512, 120, True, 1e-4), (7, 128, 10, True, 5e-4), (3, 20, 33, False, 0.0),
                                  (256, 512, 120, True, 1e-4)])
def test_dense_layer(case):
    from dorknet_amd.layers.dense_layer import DenseLayer
    from dorknet_amd.regularisers.l2 import l2
    B, IN, OUT, bias, s = case
    rng = np.random.RandomState(7)
    np.random.seed(8)
    layer = DenseLayer("d", IN, OUT, with_bias=bias, weight_regulariser=l2(s) if s else None)
    if bias:
        layer.learned_params["bias"] = rng.randn(OUT).astype(np.float32)
    run_layer(layer, rng.randn(B, IN).astype(np.float32), rng.randn(B, OUT).astype(np.float32))


@pytest.mark.parametrize("shape", [(3, 16, 5, 7), (2, 64, 9, 9), (4, 6, 3, 3), (5, 24)])
def test_batchnorm_layer(shape):
    from dorknet_amd.layers.batch_norm import BatchNormLayer
    rng = np.random.RandomState(9)
    C = shape[1]
    layer = BatchNormLayer("bn", input_dimension=len(shape), incoming_chans=C)
    pshape = (1, C, 1, 1) if len(shape) == 4 else (C,)
    layer.learned_params["gamma"] = (1 + 0.3 * rng.randn(*pshape)).astype(np.float32)
    layer.learned_params["beta"] = (0.2 * rng.randn(*pshape)).astype(np.float32)
    olayer = layer_to_oracle(layer)
    layer.to_gpu()
    for it in range(3):  # running stats: first call copies, later calls blend (batch_norm.py:76-89)
        X = (3.0 + 2.5 * rng.randn(*shape)).astype(np.float32)
        dY = rng.randn(*shape).astype(np.float32)
        check("bn fwd", layer.forward(dev(X)), olayer.forward(X.astype(np.float64)))
        check("bn dX", layer.backward(dev(dY)), olayer.backward(dY.astype(np.float64)))
        check("bn dgamma", layer.grads["gamma"], olayer.grads["gamma"])
        check("bn dbeta", layer.grads["beta"], olayer.grads["beta"])
        check("bn running_mean", layer.non_learned_params["running_mean"],
              olayer.non_learned_params["running_mean"])
        check("bn running_std", layer.non_learned_params["running_std"], olayer.non_learned_params["running_std"])
        check("bn std", layer.std, olayer.cache["std"])
    X = rng.randn(*shape).astype(np.float32)
    check("bn test-mode", layer.forward(dev(X), test_mode=True), olayer.forward(X.astype(np.float64), True))


def test_bn_relu_fused_matches_sequence():
    from dorknet_amd.layers.activations import ReLu
    from dorknet_amd.layers.batch_norm import BatchNormLayer
    rng = np.random.RandomState(10)
    bn = BatchNormLayer("bn", incoming_chans=32)
    bn.learned_params["beta"] = (0.3 * rng.randn(1, 32, 1, 1)).astype(np.float32)
    relu = ReLu("r")
    obn, orelu = layer_to_oracle(bn), O.OReLU("r")
    bn.to_gpu()
    relu.to_gpu()
    X = rng.randn(3, 32, 6, 6).astype(np.float32)
    dY = rng.randn(3, 32, 6, 6).astype(np.float32)
    Y = bn.forward_bn_relu(dev(X), relu)
    Yo = orelu.forward(obn.forward(X.astype(np.float64)))
    check("bn+relu fwd", Y, Yo)
    check("positive_locs", relu.positive_locs, (Yo > 0).astype(np.float64))
    dX = bn.backward_bn_relu(dev(dY), relu)
    dXo = obn.backward(orelu.backward(dY.astype(np.float64)))
    check("bn+relu dX", dX, dXo)
    check("bn+relu dgamma", bn.grads["gamma"], obn.grads["gamma"])


def test_relu_gap_softmax():
    from dorknet_amd.layers.activations import ReLu
    from dorknet_amd.layers.losses import SoftmaxWithCrossEntropy
    from dorknet_amd.layers.pooling import GlobalAveragePoolingLayer
    rng = np.random.RandomState(11)
    relu = ReLu("r")
    relu.to_gpu()
    X = rng.randn(2, 8, 5, 5).astype(np.float32)
    Y = relu.forward(dev(X))
    Yo, mask = ref.relu_forward(X.astype(np.float64))
    check("relu fwd", Y, Yo, 0)
    check("relu mask", relu.positive_locs, mask, 0)
    dY = rng.randn(*X.shape).astype(np.float32)
    check("relu bwd", relu.backward(dev(dY)), ref.relu_backward(dY, mask), 0)

    gap = GlobalAveragePoolingLayer("g")
    gap.to_gpu()
    check("gap fwd", gap.forward(dev(X)), ref.gap_forward(X.astype(np.float64)))
    dG = rng.randn(2, 8).astype(np.float32)
    check("gap bwd", gap.backward(dev(dG)), ref.gap_backward(dG.astype(np.float64), (5, 5)))

    sm = SoftmaxWithCrossEntropy("s")
    logits = rng.randn(6, 120).astype(np.float32)
    y = np.eye(120, dtype=np.float32)[rng.randint(0, 120, 6)]
    loss, P = sm.forward(dev(logits), dev(y))
    lo, Po = ref.softmax_xent_forward(logits.astype(np.float64), y.astype(np.float64))
    check("softmax P", P, Po)
    assert abs(float(loss) - lo) <= 1e-5 * max(1.0, abs(lo))
    check("softmax bwd", sm.backward(), ref.softmax_xent_backward(Po, y.astype(np.float64)))
    _, Pt = sm.forward(dev(logits), None, test_mode=True)
    check("softmax test-mode", Pt, Po)


@pytest.mark.parametrize("B,K", [(6, 120), (300, 12), (257, 10), (3, 130), (256, 128), (1, 4)])
def test_softmax_xent_shapes(B, K):
    """The head's softmax + cross-entropy forward on each of its paths: float4 rows (K % 4 == 0,
    K <= 128), scalar columns (K % 4 != 0), one wave per row (K > 128), and more than one 256-row
    pass (B > 256), against the oracle (losses.py:13-34)."""
    from dorknet_amd.layers.losses import SoftmaxWithCrossEntropy
    rng = np.random.RandomState(B + K)
    sm = SoftmaxWithCrossEntropy("s")
    logits = (2.0 * rng.randn(B, K)).astype(np.float32)
    y = np.eye(K, dtype=np.float32)[rng.randint(0, K, B)]
    loss, P = sm.forward(dev(logits), dev(y))
    lo, Po = ref.softmax_xent_forward(logits.astype(np.float64), y.astype(np.float64))
    check("softmax P", P, Po)
    assert abs(float(loss) - lo) <= 1e-5 * max(1.0, abs(lo)), (float(loss), lo)
    check("softmax bwd", sm.backward(), ref.softmax_xent_backward(Po, y.astype(np.float64)))


@pytest.mark.parametrize("N,C,H", [(2, 8, 5), (3, 6, 7), (4, 512, 7), (2, 64, 3)])
def test_gap_shapes(N, C, H):
    """Global average pooling forward (loads issued eight at a time, HW = 9 / 25 / 49 with a remainder)
    and backward (float4 for C % 4 == 0, scalar otherwise) against the oracle (pooling.py:23-36)."""
    from dorknet_amd.layers.pooling import GlobalAveragePoolingLayer
    rng = np.random.RandomState(N * C + H)
    X = rng.randn(N, C, H, H).astype(np.float32)
    gap = GlobalAveragePoolingLayer("g")
    gap.to_gpu()
    check("gap fwd", gap.forward(dev(X)), ref.gap_forward(X.astype(np.float64)))
    dG = rng.randn(N, C).astype(np.float32)
    check("gap bwd", gap.backward(dev(dG)), ref.gap_backward(dG.astype(np.float64), (H, H)))


def test_residual_block_and_sgd():
    """A downsampling depthwise-separable residual block + the optimiser, vs the oracle."""
    from dorknet_amd.layers.residual_block import ResidualBlock
    from examples.resnet18_depsep import ResNet18
    from dorknet_amd.optimisers.SGDMomentum import SGDMomentum
    from dorknet_amd.network.feed_forward_network import FeedForwardNetwork
    np.random.seed(12)
    shell = ResNet18("shell", load_layers=False)
    shell.add_res_block("rb", (32, 16, 3, 3), downsample=True, depthwise_sep=True)
    block = shell.layers[0]
    assert isinstance(block, ResidualBlock)
    oblock = layer_to_oracle(block)
    o32 = layer_to_oracle(block, np.float32)
    net = FeedForwardNetwork("n")
    net.add_layer(block)
    net.to_gpu()
    rng = np.random.RandomState(13)
    X = rng.randn(2, 16, 10, 10).astype(np.float32)
    dY = rng.randn(2, 32, 5, 5).astype(np.float32)
    check("resblock fwd", block.forward(dev(X)), oblock.forward(X.astype(np.float64)), want32=o32.forward(X))
    check("resblock dX", block.backward(dev(dY)), oblock.backward(dY.astype(np.float64)), want32=o32.backward(dY))
    from tests._convert import all_layers
    for l, ol, o3 in zip(all_layers([block]), all_layers([oblock]), all_layers([o32])):
        for k in (ol.grads or {}):
            check(f"{l.layer_name} d{k}", l.grads[k], ol.grads[k], want32=o3.grads[k])
    sgd = SGDMomentum(net, 0.1, 0.9)
    osgd = O.OSGDMomentum(O.ONetwork([oblock], None), 0.1, 0.9)
    osgd32 = O.OSGDMomentum(O.ONetwork([o32], None), 0.1, 0.9)
    for _ in range(2):
        sgd.update_weights()
        osgd.update_weights()
        osgd32.update_weights()
    for l, ol, o3 in zip(all_layers([block]), all_layers([oblock]), all_layers([o32])):
        for k in (ol.learned_params or {}):
            check(f"{l.layer_name} {k} after sgd", l.learned_params[k], ol.learned_params[k],
                  want32=o3.learned_params[k])
    # the skip projection is not updated (SGDMomentum.py:7-14)
    assert sgd.learnable_layers and block.skip_projection not in sgd.learnable_layers


def test_l2_regulariser():
    from dorknet_amd.regularisers.l2 import l2
    rng = np.random.RandomState(14)
    W = rng.randn(64, 3, 5, 5).astype(np.float32)
    r = l2(1e-4)
    want = ref.l2_forward(W.astype(np.float64), 1e-4)
    assert abs(float(r.forward(dev(W))) - want) <= 1e-6 * want
    check("l2 bwd", r.backward(dev(W)), ref.l2_backward(W.astype(np.float64), 1e-4), 1e-7)
