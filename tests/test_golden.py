"""Committed golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle reproduces every fixture (guards the restatement against drift).
GPU: the HIP path reproduces every fixture within the parity bound of test_gpu_layers.check.
"""
import glob
import os

import numpy as np
import pytest

from tests._convert import slack_bound
from tests.golden import make_golden

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(glob.glob(os.path.join(HERE, "*.npz")))


def load(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_fixtures_present():
    assert len(FILES) == len(make_golden.CASES)


@pytest.mark.parametrize("make", make_golden.CASES, ids=lambda f: f()[0])
def test_oracle_reproduces_fixture(make):
    name, inputs, o64, o32, meta = make()
    fx = load(os.path.join(HERE, name + ".npz"))
    for k, v in inputs.items():
        assert np.array_equal(fx["in_" + k], v), k
    for k, v in o64.items():
        ref = fx[k + "_f64"]
        assert np.linalg.norm((np.asarray(v) - ref).ravel()) <= 1e-10 * max(np.linalg.norm(ref.ravel()), 1e-30), k
    for k, v in o32.items():
        ref = fx[k + "_f32"].astype(np.float64)
        assert np.linalg.norm((np.asarray(v, np.float64) - ref).ravel()) <= 1e-5 * max(np.linalg.norm(ref.ravel()),
                                                                                       1e-30), k


# ------------------------------------------ GPU ------------------------------------------

def _gpu_outputs(fx):
    import torch
    from dorknet_amd.layers.batch_norm import BatchNormLayer
    from dorknet_amd.layers.convolution import ConvLayer
    from dorknet_amd.layers.dense_layer import DenseLayer
    from dorknet_amd.layers.depthwise_convolution import DepthwiseConvLayer
    from dorknet_amd.layers.pointwise_convolution import PointwiseConvLayer
    from dorknet_amd.regularisers.l2 import l2

    def dev(a):
        return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device="cuda")

    kind = str(fx["meta_kind"])
    reg = l2(float(fx["meta_l2"])) if "meta_l2" in fx and float(fx["meta_l2"]) else None
    bias = bool(int(fx["meta_bias"])) if "meta_bias" in fx else False
    out = {}
    if kind in ("conv", "dw", "pw", "dense"):
        W = fx["in_W"]
        if kind == "conv":
            layer = ConvLayer("g", W.shape, stride=int(fx["meta_stride"]), padding=int(fx["meta_padding"]),
                              with_bias=bias, weight_regulariser=reg)
        elif kind == "dw":
            layer = DepthwiseConvLayer("g", W.shape, stride=int(fx["meta_stride"]), padding=int(fx["meta_padding"]),
                                       with_bias=False)
        elif kind == "pw":
            layer = PointwiseConvLayer("g", stride=int(fx["meta_stride"]), filter_block_shape=W.shape,
                                       with_bias=False, weight_regulariser=reg)
        else:
            layer = DenseLayer("g", W.shape[0], W.shape[1], with_bias=True, weight_regulariser=reg)
        layer.learned_params["weights"] = W
        if bias:
            layer.learned_params["bias"] = fx["in_b"]
        layer.to_gpu()
        out["Y"] = layer.forward(dev(fx["in_X"]))
        out["dX"] = layer.backward(dev(fx["in_dY"]))
        out["dW"] = layer.grads["weights"]
        if bias:
            out["db"] = layer.grads["bias"]
    elif kind == "bn":
        shape = fx["in_X1"].shape
        layer = BatchNormLayer("g", input_dimension=len(shape), incoming_chans=shape[1])
        layer.learned_params["gamma"], layer.learned_params["beta"] = fx["in_gamma"], fx["in_beta"]
        layer.to_gpu()
        out["Y1"] = layer.forward(dev(fx["in_X1"]))
        out["Y2"] = layer.forward(dev(fx["in_X2"]))
        out["dX2"] = layer.backward(dev(fx["in_dY"]))
        out["dgamma"], out["dbeta"] = layer.grads["gamma"], layer.grads["beta"]
        out["running_mean"] = layer.non_learned_params["running_mean"]
        out["running_std"] = layer.non_learned_params["running_std"]
        out["Ytest"] = layer.forward(dev(fx["in_Xt"]), test_mode=True)
    elif kind == "head":
        from dorknet_amd.layers.activations import ReLu
        from dorknet_amd.layers.losses import SoftmaxWithCrossEntropy
        from dorknet_amd.layers.pooling import GlobalAveragePoolingLayer
        r, g, s = ReLu("r"), GlobalAveragePoolingLayer("p"), SoftmaxWithCrossEntropy("s")
        r.to_gpu()
        g.to_gpu()
        out["relu"] = r.forward(dev(fx["in_A"]))
        out["mask"] = r.positive_locs
        out["gap"] = g.forward(dev(fx["in_A"]))
        loss, out["P"] = s.forward(dev(fx["in_logits"]), dev(fx["in_y"]))
        out["loss"] = loss
        out["dlogits"] = s.backward()
    return {k: v.detach().float().cpu().numpy() for k, v in out.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p)[:-4])
def test_hip_matches_fixture(path):
    fx = load(path)
    got = _gpu_outputs(fx)
    assert got
    for k, v in got.items():
        want = fx[k + "_f64"]
        want32 = fx[k + "_f32"].astype(np.float64)
        assert v.shape == want.shape, k
        err = np.linalg.norm((v.astype(np.float64) - want).ravel())
        bound = slack_bound(want, want32, 1e-4)  # max(1e-4 ||want||, FP32_SLACK ||want32 - want||)
        assert err <= bound or err == 0, (os.path.basename(path), k, err, bound)
