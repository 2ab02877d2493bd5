"""Pin the oracle (CPU restatement of the reference) against an independent second oracle
-- torch CPU F.conv2d / F.batch_norm / autograd in fp64 -- and analytic known answers.
(The reference ships no fixtures and could not be run: SURVEY.md 8c, DESIGN.md.)"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ref

TOL = 1e-10  # both sides fp64


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    d = np.linalg.norm(b.ravel())
    return np.linalg.norm((a - b).ravel()) / (d if d else 1.0)


def t(a, grad=False):
    return torch.tensor(np.asarray(a, np.float64), requires_grad=grad)


CONV = [  # N, C, H, W, K, R, S, stride, pad, bias
    (2, 3, 17, 17, 8, 5, 5, 2, 1, False),
    (2, 4, 9, 11, 6, 3, 3, 1, 1, True),
    (3, 2, 14, 14, 5, 4, 4, 2, 1, False),
    (1, 1, 28, 28, 4, 3, 3, 1, 1, False),
    (2, 5, 10, 10, 3, 3, 3, 1, 0, True),
    (2, 3, 8, 7, 4, 2, 3, 1, 1, False),   # non-square filter and input
]


@pytest.mark.parametrize("case", CONV)
def test_conv_vs_torch(case):
    N, C, H, W, K, R, S, st, pd, bias = case
    rng = np.random.default_rng(0)
    X = rng.standard_normal((N, C, H, W))
    Wt = rng.standard_normal((K, C, R, S))
    b = rng.standard_normal(K) if bias else None
    Y, cache = ref.conv_forward(X, Wt, b, st, pd)
    xt, wt = t(X, True), t(Wt, True)
    bt = t(b, True) if bias else None
    yt = F.conv2d(xt, wt, bt, stride=st, padding=pd)
    assert Y.shape == tuple(yt.shape)
    assert rel(Y, yt.detach().numpy()) < TOL
    dY = rng.standard_normal(Y.shape)
    yt.backward(t(dY))
    dX, dW, db = ref.conv_backward(dY, Wt, cache, st, pd, bias)
    assert rel(dX, xt.grad.numpy()) < TOL and dX.shape == X.shape
    assert rel(dW, wt.grad.numpy()) < TOL
    if bias:
        assert rel(db, bt.grad.numpy()) < TOL


@pytest.mark.parametrize("case", [(2, 6, 9, 9, 3, 1, 1, False), (2, 4, 14, 14, 3, 2, 1, True),
                                  (1, 8, 15, 15, 3, 2, 1, False), (2, 3, 11, 11, 5, 1, 2, True)])
def test_depthwise_vs_torch(case):
    N, C, H, W, R, st, pd, bias = case
    rng = np.random.default_rng(1)
    X = rng.standard_normal((N, C, H, W))
    Wt = rng.standard_normal((C, R, R))
    b = rng.standard_normal(C) if bias else None
    Y, cache = ref.depthwise_forward(X, Wt, b, st, pd)
    xt, wt = t(X, True), t(Wt[:, None], True)
    bt = t(b, True) if bias else None
    yt = F.conv2d(xt, wt, bt, stride=st, padding=pd, groups=C)
    assert rel(Y, yt.detach().numpy()) < TOL
    dY = rng.standard_normal(Y.shape)
    yt.backward(t(dY))
    dX, dW, db = ref.depthwise_backward(dY, Wt, cache, st, pd, bias)
    assert rel(dX, xt.grad.numpy()) < TOL
    assert rel(dW, wt.grad.numpy()[:, 0]) < TOL
    if bias:
        assert rel(db, bt.grad.numpy()) < TOL


@pytest.mark.parametrize("case", [(2, 8, 6, 6, 5, 1, False), (2, 8, 12, 12, 4, 2, True), (1, 3, 7, 8, 2, 1, True)])
def test_pointwise_vs_torch(case):
    N, C, H, W, K, st, bias = case
    rng = np.random.default_rng(2)
    X = rng.standard_normal((N, C, H, W))
    Wt = rng.standard_normal((K, C))
    b = rng.standard_normal(K) if bias else None
    Y, cache = ref.pointwise_forward(X, Wt, b, st)
    xt, wt = t(X, True), t(Wt[:, :, None, None], True)
    bt = t(b, True) if bias else None
    yt = F.conv2d(xt, wt, bt, stride=st)
    assert rel(Y, yt.detach().numpy()) < TOL
    dY = rng.standard_normal(Y.shape)
    yt.backward(t(dY))
    dX, dW, db = ref.pointwise_backward(dY, Wt, cache, st, bias)
    # the reference widens to (s*OH, s*OW) (pointwise_convolution.py:68-72) == input size for even H
    assert dX.shape == (N, C, Y.shape[2] * st, Y.shape[3] * st)
    assert rel(dX[:, :, :H, :W], xt.grad.numpy()) < TOL
    assert rel(dW, wt.grad.numpy()[:, :, 0, 0]) < TOL


def test_dense_vs_torch():
    rng = np.random.default_rng(3)
    X, Wt, b = rng.standard_normal((5, 7)), rng.standard_normal((7, 3)), rng.standard_normal(3)
    Y = ref.dense_forward(X, Wt, b)
    xt, wt, bt = t(X, True), t(Wt, True), t(b, True)
    yt = xt @ wt + bt
    assert rel(Y, yt.detach().numpy()) < TOL
    dY = rng.standard_normal(Y.shape)
    yt.backward(t(dY))
    dX, dW, db = ref.dense_backward(dY, X, Wt, True, l2_strength=0.1)
    assert rel(dX, xt.grad.numpy()) < TOL
    assert rel(dW, wt.grad.numpy() + 0.1 * Wt) < TOL
    assert rel(db, bt.grad.numpy()) < TOL


@pytest.mark.parametrize("shape", [(3, 4, 5, 6), (7, 5)])
def test_batchnorm_vs_torch(shape):
    rng = np.random.default_rng(4)
    X = 2.0 + 3.0 * rng.standard_normal(shape)
    C = shape[1]
    pshape = (1, C, 1, 1) if len(shape) == 4 else (C,)
    g = 1 + 0.2 * rng.standard_normal(pshape)
    b = 0.3 * rng.standard_normal(pshape)
    Y, cache, rm, rs = ref.bn_forward_train(X, g, b, None, None)
    xt, gt, bt = t(X, True), t(g.reshape(C), True), t(b.reshape(C), True)
    yt = F.batch_norm(xt, None, None, gt, bt, training=True, eps=1e-5)
    assert rel(Y, yt.detach().numpy()) < TOL
    # running buffers: first call copies the batch mean / std (batch_norm.py:76-89)
    axis = (0, 2, 3) if len(shape) == 4 else 0
    assert rel(rm.ravel(), X.mean(axis=axis)) < TOL
    assert rel(rs.ravel(), np.sqrt(X.var(axis=axis) + 1e-5)) < TOL
    dY = rng.standard_normal(shape)
    yt.backward(t(dY))
    dX, dg, db = ref.bn_backward(dY, g, cache)
    assert rel(dX, xt.grad.numpy()) < 1e-9
    assert rel(np.ravel(dg), gt.grad.numpy()) < TOL and rel(np.ravel(db), bt.grad.numpy()) < TOL
    # second call blends with momentum 0.95, std not var
    X2 = rng.standard_normal(shape)
    _, _, rm2, rs2 = ref.bn_forward_train(X2, g, b, rm, rs)
    assert rel(rm2.ravel(), 0.95 * rm.ravel() + 0.05 * X2.mean(axis=axis)) < TOL
    assert rel(rs2.ravel(), 0.95 * rs.ravel() + 0.05 * np.sqrt(X2.var(axis=axis) + 1e-5)) < TOL


def test_softmax_xent_relu_gap_vs_torch():
    rng = np.random.default_rng(5)
    X = rng.standard_normal((6, 10))
    y = np.eye(10)[rng.integers(0, 10, 6)]
    loss, P = ref.softmax_xent_forward(X, y)
    xt = t(X, True)
    lt = F.cross_entropy(xt, torch.tensor(y.argmax(1)))
    assert abs(loss - lt.item()) < 1e-12
    lt.backward()
    assert rel(ref.softmax_xent_backward(P, y), xt.grad.numpy()) < TOL
    A = rng.standard_normal((2, 3, 4, 5))
    out, mask = ref.relu_forward(A)
    assert np.array_equal(out, np.maximum(A, 0)) and np.array_equal(mask, (A > 0).astype(float))
    at = t(A, True)
    gt = at.mean(dim=(2, 3))
    assert rel(ref.gap_forward(A), gt.detach().numpy()) < TOL
    dG = rng.standard_normal((2, 3))
    gt.backward(t(dG))
    assert rel(ref.gap_backward(dG, (4, 5)), at.grad.numpy()) < TOL


def test_relu_decision_replay():
    """OReLU.replay (tests/_ties.py): the replayed mask decides one training forward and its
    backward; the next forward decides on out > 0 again; test mode ignores it."""
    from oracle.net import OReLU
    rng = np.random.default_rng(6)
    A = rng.standard_normal((2, 3, 4, 5))
    m = A > 0
    m[0, 1, 2, 3] = not m[0, 1, 2, 3]           # one flipped decision, as at a tie
    r = OReLU("r")
    r.replay = m
    assert np.array_equal(r.forward(A, test_mode=True), np.maximum(A, 0)) and r.replay is not None
    y = r.forward(A)
    assert np.array_equal(y, A * m) and r.replay is None and r.pre is A
    dY = rng.standard_normal(A.shape)
    assert np.array_equal(r.backward(dY), dY * m)
    assert np.array_equal(r.forward(A), np.maximum(A, 0))
    r.replay = m[:1]
    with pytest.raises(ValueError):
        r.forward(A)


# ------------------------------- known-answer tests -------------------------------------

def test_kat_identity_and_delta_filters():
    X = np.arange(2 * 3 * 5 * 5, dtype=np.float64).reshape(2, 3, 5, 5)
    Wid = np.zeros((3, 3, 3, 3))
    for c in range(3):
        Wid[c, c, 1, 1] = 1.0
    Y, _ = ref.conv_forward(X, Wid, None, 1, 1)       # identity 3x3 filter, pad 1
    assert np.array_equal(Y, X)
    Y2, _ = ref.pointwise_forward(X, np.eye(3), None, 2)   # stride-2 1x1 == subsampling
    assert np.array_equal(Y2, X[:, :, ::2, ::2])
    D = np.zeros((1, 1, 5, 5))
    D[0, 0, 2, 2] = 1.0                                  # delta input -> flipped? no: correlation
    Wk = np.arange(9, dtype=np.float64).reshape(1, 1, 3, 3)
    Yd, _ = ref.conv_forward(D, Wk, None, 1, 1)
    assert np.array_equal(Yd[0, 0, 1:4, 1:4], Wk[0, 0, ::-1, ::-1])


def test_kat_batchnorm_constant_channel():
    X = np.full((4, 2, 3, 3), 7.0)
    g = np.full((1, 2, 1, 1), 1.5)
    b = np.array([0.25, -0.5]).reshape(1, 2, 1, 1)
    Y, cache, _, _ = ref.bn_forward_train(X, g, b, None, None)
    assert np.allclose(Y, np.broadcast_to(b, X.shape))       # constant channel -> beta
    dY = np.random.default_rng(0).standard_normal(X.shape)
    dX, dg, db = ref.bn_backward(dY, g, cache)
    # x_hat == 0, so dgamma == 0 and dx = gamma / sqrt(eps) * (dy - mean(dy))
    assert np.allclose(dg, 0.0)
    assert np.allclose(dX, g / np.sqrt(1e-5) * (dY - dY.mean(axis=(0, 2, 3), keepdims=True)))


def test_kat_sgd_momentum_and_l2():
    W = np.array([1.0, -2.0])
    v = np.array([0.5, 0.0])
    g = np.array([0.1, 0.2])
    W2, v2 = ref.sgd_momentum_update(W, g, v, 0.1, 0.9)
    assert np.allclose(v2, -0.1 * g + 0.9 * v) and np.allclose(W2, W + v2)
    assert ref.l2_forward(W, 0.2) == pytest.approx(0.5 * 0.2 * 5.0)
    assert np.allclose(ref.l2_backward(W, 0.2), 0.2 * W)


def test_output_size_float_then_int():
    # convolution.py:67-68 -- (Hp - f)/s + 1 in float, truncated: 58 -> 28.5 -> 28
    assert ref.out_size(58, 3, 2) == (28.5, 28)
    assert ref.out_size(227, 5, 2) == (112.0, 112)
