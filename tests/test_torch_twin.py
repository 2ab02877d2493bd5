"""The torch fp64 twin (tests/_torch_twin.py, the full-size parity checker) against the numpy
oracle (the reference restated) on small shapes of the ResNet-18-depsep stem and blocks."""
import numpy as np

from tests._convert import layer_to_oracle
from tests._torch_twin import TorchTwin


def _perturb_bn(layers, rng):
    from tests._torch_twin import TorchTwin as T
    for l in T._all(layers):
        if type(l).__name__ == "BatchNormLayer":
            C = l.incoming_chans
            l.learned_params["gamma"] = (1 + 0.2 * rng.standard_normal((1, C, 1, 1))).astype(np.float32)
            l.learned_params["beta"] = (0.1 * rng.standard_normal((1, C, 1, 1))).astype(np.float32)


def _check(layers, X, dY):
    twin = TorchTwin(layers)
    Y, dX, grads = twin.run(X, dY)
    ol = [layer_to_oracle(l) for l in layers]
    h = X.astype(np.float64)
    for l in ol:
        h = l.forward(h, False)
    g = dY.astype(np.float64)
    for l in reversed(ol):
        g = l.backward(g)
    assert np.allclose(Y, h, rtol=1e-10, atol=1e-10)
    assert np.allclose(dX, g, rtol=1e-9, atol=1e-12)

    def walk(o):
        yield o
        for c in getattr(o, "layer_list", []) or []:
            yield from walk(c)
        if getattr(o, "skip_projection", None) is not None:
            yield o.skip_projection
    n = 0
    for o in ol:
        for oo in walk(o):
            for k, v in (oo.grads or {}).items():
                assert np.allclose(grads[(oo.layer_name, k)], v, rtol=1e-9, atol=1e-12), (oo.layer_name, k)
                n += 1
    return n


def test_twin_matches_oracle_blocks():
    from examples.resnet18_depsep import ResNet18
    np.random.seed(3)
    net = ResNet18("r18")
    rng = np.random.default_rng(4)
    layers = net.layers[4:9]          # pw0_bn, pw0_relu, res1, res2, res3 (stride 2 + skip)
    _perturb_bn(layers, rng)
    X = (0.5 + 2.0 * rng.standard_normal((2, 64, 10, 10))).astype(np.float32)
    dY = rng.standard_normal((2, 128, 5, 5)).astype(np.float32)
    assert _check(layers, X, dY) > 20


def test_twin_matches_oracle_stem():
    from examples.resnet18_depsep import ResNet18
    np.random.seed(5)
    net = ResNet18("r18")
    rng = np.random.default_rng(6)
    layers = net.layers[0:6]          # conv0 5x5/2, conv0_bn, relu, pw0 1x1/2, pw0_bn, relu
    _perturb_bn(layers, rng)
    X = rng.uniform(-128, 128, size=(2, 3, 21, 21)).astype(np.float32)
    dY = rng.standard_normal((2, 64, 5, 5)).astype(np.float32)
    assert _check(layers, X, dY) == 6
