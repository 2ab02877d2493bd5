"""The reference's CPU path restated (oracle/cpu_path.py: C/OpenMP versions of the Cython
kernels + numpy BLAS) agrees with the numpy restatement of the GPU branch, layer by layer
and for a whole MNISTNet training step (BASELINE config 1, the reference's CPU plumbing)."""
import numpy as np
import pytest

from oracle import cpu_path, models
from oracle import net as O
from oracle.net import OSGDMomentum


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-30)


@pytest.mark.parametrize("case", [(2, 3, 17, 8, 5, 2, 1), (2, 8, 9, 16, 3, 1, 1), (3, 4, 14, 8, 4, 2, 1)])
def test_cy_conv_matches_numpy(case):
    N, C, H, K, R, st, pd = case
    rng = np.random.default_rng(0)
    X = rng.standard_normal((N, C, H, H)).astype(np.float32)
    W = rng.standard_normal((K, C, R, R)).astype(np.float32)
    a, b = cpu_path.CyConv("c", W, None, st, pd, 1e-4), O.OConv("c", W.astype(np.float64), None, st, pd, 1e-4)
    Y, Yo = a.forward(X), b.forward(X.astype(np.float64))
    assert rel(Y, Yo) < 1e-5
    dY = rng.standard_normal(Y.shape).astype(np.float32)
    assert rel(a.backward(dY), b.backward(dY.astype(np.float64))) < 1e-5
    assert rel(a.grads["weights"], b.grads["weights"]) < 1e-5


@pytest.mark.parametrize("st", [1, 2])
def test_cy_depthwise_matches_numpy(st):
    rng = np.random.default_rng(1)
    X = rng.standard_normal((2, 8, 14, 14)).astype(np.float32)
    W = rng.standard_normal((8, 3, 3)).astype(np.float32)
    a, b = cpu_path.CyDepthwise("d", W, None, st, 1), O.ODepthwise("d", W.astype(np.float64), None, st, 1)
    Y, Yo = a.forward(X), b.forward(X.astype(np.float64))
    assert rel(Y, Yo) < 1e-5
    dY = rng.standard_normal(Y.shape).astype(np.float32)
    assert rel(a.backward(dY), b.backward(dY.astype(np.float64))) < 1e-5
    assert rel(a.grads["weights"], b.grads["weights"]) < 1e-5


def test_cy_bn_relu_match_numpy():
    rng = np.random.default_rng(2)
    X = (2 + rng.standard_normal((4, 6, 5, 5))).astype(np.float32)
    g = np.ones((1, 6, 1, 1), np.float32)
    b = np.zeros((1, 6, 1, 1), np.float32)
    a, o = cpu_path.CyBatchNorm("bn", g, b), O.OBatchNorm("bn", g.astype(np.float64), b.astype(np.float64))
    assert rel(a.forward(X), o.forward(X.astype(np.float64))) < 1e-5
    dY = rng.standard_normal(X.shape).astype(np.float32)
    assert rel(a.backward(dY), o.backward(dY.astype(np.float64))) < 1e-4
    r, ro = cpu_path.CyReLU("r"), O.OReLU("r")
    assert np.array_equal(r.forward(X - 2), ro.forward(X - 2))
    assert np.array_equal(r.mask, ro.mask)


def test_mnist_config1_step_cpu_path():
    """BASELINE config 1: MNISTNet, batch 64, reference CPU path vs numpy restatement."""
    rng = np.random.default_rng(3)
    cy = models.mnist_net("cy", rng=np.random.RandomState(0))
    npn = models.mnist_net("np", rng=np.random.RandomState(0), dtype=np.float64)
    X = rng.uniform(0, 1, (64, 1, 28, 28)).astype(np.float32)
    y = np.eye(10, dtype=np.float32)[rng.integers(0, 10, 64)]
    sgd, sgdo = OSGDMomentum(cy, 0.01, 0.9), OSGDMomentum(npn, 0.01, 0.9)
    for _ in range(2):
        l1, P1 = cy.forward(X, y)
        l2, P2 = npn.forward(X.astype(np.float64), y.astype(np.float64))
        assert abs(l1 - l2) < 1e-4 * abs(l2) and rel(P1, P2) < 1e-4
        cy.backward()
        npn.backward()
        sgd.update_weights()
        sgdo.update_weights()
    assert rel(cy.layers[0].learned_params["weights"], npn.layers[0].learned_params["weights"]) < 1e-4
