"""Host-side behaviour of the drop-in boundary (no GPU): constructors, initialisation,
__repr__ text, model structure, optimiser parameter discovery, module aliases, errors."""
import json

import numpy as np
import pytest

import dorknet_amd
from dorknet_amd.layers.activations import ReLu
from dorknet_amd.layers.batch_norm import BatchNormLayer
from dorknet_amd.layers.convolution import ConvLayer
from dorknet_amd.layers.dense_layer import DenseLayer
from dorknet_amd.layers.depthwise_convolution import DepthwiseConvLayer
from dorknet_amd.layers.losses import SoftmaxWithCrossEntropy
from dorknet_amd.layers.pointwise_convolution import PointwiseConvLayer
from dorknet_amd.layers.pooling import GlobalAveragePoolingLayer
from dorknet_amd.optimisers.SGDMomentum import SGDMomentum
from dorknet_amd.regularisers.l2 import l2
from examples.resnet18_depsep import ResNet18


def test_repr_matches_reference_format():
    # format strings of convolution.py:40-51, depthwise_convolution.py:41-51,
    # pointwise_convolution.py:35-44, dense_layer.py:38-44, batch_norm.py:48-51, ...
    assert repr(ConvLayer("conv0", (64, 3, 5, 5), stride=2, padding=1, with_bias=False,
                          weight_regulariser=l2(0.0001))) == \
        "ConvLayer(conv0, filter_block_shape=(64,3,5,5), stride=2, padding=1, with_bias=False, " \
        "weight_regulariser=l2(strength=0.0001))"
    assert repr(PointwiseConvLayer("pw0", filter_block_shape=(64, 64), with_bias=False, stride=2,
                                   weight_regulariser=l2(0.0001))) == \
        "PointwiseConvLayer(pw0, filter_block_shape=(64, 64), stride=2, with_bias=False, " \
        "weight_regulariser=l2(strength=0.0001), is_on_gpu=False)"
    assert repr(DepthwiseConvLayer("d", (64, 3, 3), with_bias=False)) == \
        "DepthwiseConvLayer(d, filter_block_shape=(64, 3, 3), stride=1, padding=1, with_bias=False, " \
        "weight_regulariser=None)"
    assert repr(DenseLayer("dense1", 512, 120, weight_regulariser=l2(0.0001))) == \
        "DenseLayer(dense1, incoming_chans=512, output_dim=120, weight_regulariser=l2(strength=0.0001))"
    assert repr(BatchNormLayer("bn", incoming_chans=64)) == \
        "BatchNormLayer(bn, input_dimension=4, incoming_chans=64, run_momentum=0.95)"
    assert repr(ReLu("r")) == "ReLu(r)"
    assert repr(GlobalAveragePoolingLayer("g")) == "GlobalAveragePoolingLayer(g)"
    assert repr(SoftmaxWithCrossEntropy("s")) == "SoftmaxWithCrossEntropy(s)"


def test_initialisation_follows_numpy_global_rng():
    np.random.seed(123)
    c = ConvLayer("c", (8, 3, 5, 5))
    d = DepthwiseConvLayer("d", (8, 3, 3), weight_initialiser="glorot_uniform")
    np.random.seed(123)
    w1 = 0.01 * np.random.randn(8, 3, 5, 5).astype(np.float32)
    lim = np.sqrt(6.0 / 16)
    w2 = np.random.uniform(low=-lim, high=lim, size=(8, 3, 3)).astype(np.float32)
    assert np.array_equal(c.learned_params["weights"], w1)
    assert np.array_equal(d.learned_params["weights"], w2)
    assert c.learned_params["bias"].shape == (8,) and not c.learned_params["bias"].any()
    bn = BatchNormLayer("bn", incoming_chans=5)
    assert bn.learned_params["gamma"].shape == (1, 5, 1, 1)
    assert BatchNormLayer("bn2", input_dimension=2, incoming_chans=5).learned_params["beta"].shape == (5,)
    with pytest.raises(ValueError):
        BatchNormLayer("bad", input_dimension=3)


def _all(layers):
    out = []
    for l in layers:
        out.append(l)
        if hasattr(l, "layer_list"):
            out += _all(l.layer_list)
            if l.skip_projection is not None:
                out.append(l.skip_projection)
    return out


def test_resnet18_depsep_structure():
    np.random.seed(0)
    net = ResNet18("r18")
    layers = _all(net.layers)
    n_params = sum(v.size for l in layers if l.learned_params for v in l.learned_params.values())
    skip = sum(l.learned_params["weights"].size for l in layers if l.layer_name.endswith("_pw_skip"))
    assert n_params == 1508344 and skip == 172032
    assert len([l for l in layers if isinstance(l, BatchNormLayer)]) == 34
    assert len([l for l in layers if isinstance(l, DepthwiseConvLayer)]) == 16
    assert len([l for l in layers if isinstance(l, PointwiseConvLayer)]) == 20
    assert [l.layer_name for l in net.layers[:6]] == ["conv0", "conv0_bn", "conv0_relu", "pw0", "pw0_bn",
                                                        "pw0_relu"]
    assert [l.layer_name for l in net.layers[6].layer_list] == [
        "res1_dw1_dw", "res1_dw1_dw_bn", "res1_dw1_pw", "res1_dw1_pw_bn", "res1_dw1pw_relu",
        "res1_dw2_dw", "res1_dw2_dw_bn", "res1_dw2_pw", "res1_dw2_pw_bn"]


def test_sgd_discovery_excludes_skip_projections():
    np.random.seed(0)
    net = ResNet18("r18")
    sgd = SGDMomentum(net, 0.064, 0.9)
    names = {l.layer_name for l in sgd.learnable_layers}
    assert not any(n.endswith("_pw_skip") for n in names)      # SGDMomentum.py:7-14 quirk
    ntens = sum(len(l.learned_params) for l in sgd.learnable_layers)
    nparam = sum(v.size for l in sgd.learnable_layers for v in l.learned_params.values())
    assert ntens == 104 and nparam == 1336312


def test_sgd_update_skip_projections_flag():
    """The quirk as an explicit flag: True also updates every
    ResidualBlock's skip projection (3 more tensors, the 172,032 skip parameters)."""
    np.random.seed(0)
    net = ResNet18("r18")
    sgd = SGDMomentum(net, 0.064, 0.9, update_skip_projections=True)
    names = [l.layer_name for l in sgd.learnable_layers]
    assert sum(n.endswith("_pw_skip") for n in names) == 3
    ntens = sum(len(l.learned_params) for l in sgd.learnable_layers)
    nparam = sum(v.size for l in sgd.learnable_layers for v in l.learned_params.values())
    assert ntens == 107 and nparam == 1336312 + 172032


def test_compute_requires_gpu():
    layer = ConvLayer("c", (4, 4, 3, 3))
    with pytest.raises(RuntimeError, match="to_gpu"):
        layer.forward(np.zeros((1, 4, 5, 5), np.float32))


def test_reference_module_aliases():
    dorknet_amd.install_reference_aliases()
    from layers.convolution import ConvLayer as C2            # the reference's import lines
    from network.feed_forward_network import FeedForwardNetwork
    from optimisers.SGDMomentum import SGDMomentum as S2
    from regularisers.l2 import l2 as L2
    assert C2 is ConvLayer and S2 is SGDMomentum and L2 is l2
    assert FeedForwardNetwork.__module__.startswith("dorknet_amd")


def test_structure_json(tmp_path):
    np.random.seed(0)
    net = ResNet18("DogsImageNet225ResNet18DepSep")
    p = tmp_path / "s.json"
    net.save_layer_structure_to_json(str(p))
    d = json.loads(p.read_text())
    assert d["name"] == "DogsImageNet225ResNet18DepSep"
    assert list(d)[1:4] == ["conv0", "conv0_bn", "conv0_relu"] and "softmax1" in d
    assert d["dense1"] == repr(net.layers[-1])


def test_perf_model_config2():
    from dorknet_amd import perfmodel
    f, b = perfmodel.work("dk_conv2d_fwd_f32", (0, 256, 56, 56, 64, 0, 64, 3, 3, 1, 1, 0, 0, 56, 56, 0))
    assert f == 2 * 256 * 56 * 56 * 64 * 64 * 9            # 59.19 GFLOP
    assert b == 4 * (2 * 256 * 56 * 56 * 64 + 64 * 64 * 9)


def test_perf_model_covers_header_signatures():
    """Every modelled entry point is declared in include/dorknet_hip.h and its formula takes
    exactly the declared arguments (the bench's roofline accounting cannot drift)."""
    from dorknet_amd import perfmodel
    from dorknet_amd._hip import parse_header
    decls = parse_header()
    for name in perfmodel.MODEL:
        assert name in decls, name
        args = tuple(1 for _ in decls[name][1])
        f, b = perfmodel.work(name, args)
        assert f >= 0 and b >= 0, name


def test_bn_fusion_plan_resnet():
    """The executor's plan for ResNet-18-depsep: every BatchNorm is applied by its consumer
    (pointwise / depthwise convolutions, residual blocks and joins) -- none is written."""
    from dorknet_amd.layers._chain import plan_group
    from dorknet_amd.layers.batch_norm import BatchNormLayer
    from dorknet_amd.layers.residual_block import ResidualBlock
    from examples.resnet18_depsep import ResNet18
    net = ResNet18("r18")
    modes = []
    i = 0
    while i < len(net.layers):
        group, mode = plan_group(net.layers, i, True)
        modes.append((group[0].layer_name, mode))
        i += len(group)
    assert ("conv0_bn", "defer") in modes and ("pw0_bn", "defer") in modes
    for layer in net.layers:
        if isinstance(layer, ResidualBlock):
            ll, j, inner = layer.layer_list, 0, []
            while j < len(ll):
                group, mode = plan_group(ll, j, True, out_accepts=True)
                if isinstance(group[0], BatchNormLayer):
                    inner.append(mode)
                j += len(group)
            assert inner == ["defer"] * 4, (layer.layer_name, inner)


def test_bn_fusion_plan_keeps_terminal_output():
    from dorknet_amd.layers._chain import plan_group
    from examples.resnet18_depsep import ResNet18
    net = ResNet18("r18")
    group, mode = plan_group(net.layers, 1, True, keep=("conv0_relu",))
    assert mode == "pair"
    group, mode = plan_group(net.layers, 1, False)
    assert mode == "single"


def test_env_switches_follow_runtime_changes(monkeypatch):
    """dorknet_amd._env.getenv reads os.environ's backing dict: a switch set, changed or removed at
    run time (as the tests' monkeypatch does) is seen on the next call, like os.environ.get."""
    from dorknet_amd._env import enabled, getenv
    monkeypatch.delenv("DORKNET_TEST_SWITCH", raising=False)
    assert getenv("DORKNET_TEST_SWITCH") is None and getenv("DORKNET_TEST_SWITCH", "d") == "d"
    assert enabled("DORKNET_TEST_SWITCH")
    monkeypatch.setenv("DORKNET_TEST_SWITCH", "0")
    assert getenv("DORKNET_TEST_SWITCH") == "0" and not enabled("DORKNET_TEST_SWITCH")
    monkeypatch.setenv("DORKNET_TEST_SWITCH", "1")
    assert enabled("DORKNET_TEST_SWITCH")
    monkeypatch.delenv("DORKNET_TEST_SWITCH")
    assert getenv("DORKNET_TEST_SWITCH") is None


def test_bnout_refuses_stale_statistics():
    """A BNOut aliases its BatchNormLayer's per-layer mean / invstd buffers: after that layer's next
    training forward (generation counter) using it raises instead of reading the newer batch's
    statistics (layers/_bn_input.py); a test-mode forward rewrites neither and keeps it valid."""
    import torch
    from dorknet_amd.layers._bn_input import BNOut
    bn = BatchNormLayer("bn_t", incoming_chans=4)
    bn._dk_gen = 3
    t = [torch.zeros(4) for _ in range(5)]
    out = BNOut(t[0], t[1], t[2], t[3], t[4], True, owner=bn)
    assert len(out.bn_args()) == 5
    bn._dk_gen += 1  # what _normalisation does on a training forward
    with pytest.raises(RuntimeError, match="bn_t"):
        out.bn_args()
    with pytest.raises(RuntimeError):
        out.materialize()
    assert BNOut(t[0], t[1], t[2], t[3], t[4], False, owner=None).bn_args()[-1] == 0


def test_stats_fold_arming_marks_records_stale(monkeypatch):
    """Arming a producer's in-launch statistics fold (batch_norm.py arm_stats_fold) means that launch
    rewrites the layer's mean / invstd before its forward runs: records of the previous forward go
    stale at the arming, not only at the forward."""
    import torch
    from dorknet_amd.layers import batch_norm
    from dorknet_amd.layers._bn_input import BNOut
    bn = BatchNormLayer("bn_f", incoming_chans=4)
    bn._dk_gen = 7
    t = [torch.zeros(4) for _ in range(5)]
    out = BNOut(t[0], t[1], t[2], t[3], t[4], True, owner=bn)
    monkeypatch.setattr(bn, "_stats_outputs", lambda C, dev: (t[0], t[1], t[2], t[3], t[4], False))
    monkeypatch.setattr(batch_norm.fold_resources, "get", lambda: (0, 0, 0, 0))

    class _Lib:
        def dk_bn_fold_arm_stats(self, *a):
            return 0
    monkeypatch.setattr(batch_norm, "lib", _Lib())
    assert bn.arm_stats_fold(torch.zeros((3, 2, 4), dtype=torch.float64), 12) is not None
    with pytest.raises(RuntimeError, match="bn_f"):
        out.bn_args()


def test_wgrad_flush_last_setting(monkeypatch):
    """DORKNET_WGRAD_FLUSH_LAST: the network's backward flushes the recorded reduces before each of
    its last this-many steps; 1 by default or when unparsable, never negative."""
    from dorknet_amd._hip import early_flush_steps
    monkeypatch.delenv("DORKNET_WGRAD_FLUSH_LAST", raising=False)
    assert early_flush_steps() == 1
    for v, want in (("0", 0), ("3", 3), ("-2", 0), ("x", 1)):
        monkeypatch.setenv("DORKNET_WGRAD_FLUSH_LAST", v)
        assert early_flush_steps() == want
