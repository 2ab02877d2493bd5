"""CPU restatement of the reference's hot-path maths (numpy).  TEST INFRASTRUCTURE ONLY.

Each function restates one reference function (file:line under WJGiles/Dorknet) on numpy
arrays, in the dtype of its inputs: fp32 inputs reproduce the reference's fp32 pipeline,
fp64 inputs give a "truth" to measure fp32 error against.  The GPU-branch semantics
(CuPy path) are followed where the CPU (Cython) branch differs only in how; where the
reference's CUDA kernels are wrong (non-square outputs / non-square filters, SURVEY.md
7.3), the intended maths is restated.

PARITY UNPINNED: the reference ships no tests, golden vectors or fixtures, and running
the reference itself was denied, so this restatement is pinned by an
independent second oracle (torch CPU: F.conv2d, F.batch_norm, autograd), analytic
known-answer tests and committed fixtures (tests/golden) instead -- see DESIGN.md.

Nothing in the product package imports this module.
"""
from __future__ import annotations

import numpy as np


# ---------------------------------------------------------------------------------------
# convolution (layers/convolution.py)
# ---------------------------------------------------------------------------------------

def pad_input(X, padding):
    """convolution.py:144-151 (also depthwise_convolution.py:57-64)."""
    if padding <= 0:
        return X
    return np.pad(X, ((0, 0), (0, 0), (padding, padding), (padding, padding)), "constant")


def out_size(Hp, f, stride):
    """The float-then-int patch count (convolution.py:67-68)."""
    full = ((Hp - f) / stride) + 1
    return full, int(full)


def im2col(Xp, R, S, stride, OH, OW):
    """patches[N*OH*OW, C*R*S], row b*P + oh*OW + ow, column c*R*S + r*S + s
    (CUDA im2col convolution.py:187-203; im2col_cy im2col.pyx:14-36)."""
    N, C = Xp.shape[:2]
    win = np.lib.stride_tricks.sliding_window_view(Xp, (R, S), axis=(2, 3))  # N,C,Hp-R+1,Wp-S+1,R,S
    win = win[:, :, ::stride, ::stride][:, :, :OH, :OW]                      # N,C,OH,OW,R,S
    return np.ascontiguousarray(win.transpose(0, 2, 3, 1, 4, 5)).reshape(N * OH * OW, C * R * S)


def row2im(dx_rows, N, C, Hpd, Wpd, R, S, stride, OH, OW):
    """Scatter-add of dx_rows[N*OH*OW, C*R*S] into a padded (N, C, Hpd, Wpd) gradient
    (CUDA row2im convolution.py:205-222; row2im_cy im2col.pyx:207-234)."""
    out = np.zeros((N, C, Hpd, Wpd), dtype=dx_rows.dtype)
    t = dx_rows.reshape(N, OH, OW, C, R, S)
    for r in range(R):
        for s in range(S):
            out[:, :, r:r + stride * OH:stride, s:s + stride * OW:stride] += t[:, :, :, :, r, s].transpose(0, 3, 1, 2)
    return out


def conv_forward(X, W, b, stride, padding):
    """ConvLayer.forward GPU branch (convolution.py:58-87).  Returns (Y, cache)."""
    K, C, R, S = W.shape
    Xp = pad_input(X, padding)
    OHf, OH = out_size(Xp.shape[2], R, stride)
    OWf, OW = out_size(Xp.shape[3], S, stride)
    patches = im2col(Xp, R, S, stride, OH, OW)
    out = patches @ W.reshape(K, -1).T
    if b is not None:
        out = out + b.reshape(1, -1)
    N = X.shape[0]
    Y = out.reshape(N, OH, OW, K).transpose(0, 3, 1, 2)
    cache = dict(patches=patches, input_shape=X.shape, OHf=OHf, OWf=OWf, OH=OH, OW=OW)
    return Y, cache


def conv_backward(dY, W, cache, stride, padding, with_bias, l2_strength=0.0):
    """ConvLayer.backward GPU branch (convolution.py:90-117).  Returns (dX, dW, db)."""
    K, C, R, S = W.shape
    db = dY.sum(axis=(0, 2, 3)) if with_bias else None
    up = dY.transpose(0, 2, 3, 1).reshape(cache["patches"].shape[0], -1)
    dW = (up.T @ cache["patches"]).reshape(W.shape)
    if l2_strength:
        dW = dW + l2_backward(W, l2_strength)
    dx_rows = up @ W.reshape(K, -1)
    N, _, H, Wd = cache["input_shape"]
    Hpd = int(stride * (cache["OHf"] - 1) + R)
    Wpd = int(stride * (cache["OWf"] - 1) + S)
    padded = row2im(dx_rows, N, C, Hpd, Wpd, R, S, stride, cache["OH"], cache["OW"])
    if padding > 0:
        return padded[:, :, padding:-padding, padding:-padding], dW, db
    return padded, dW, db


# ---------------------------------------------------------------------------------------
# depthwise convolution (layers/depthwise_convolution.py)
# ---------------------------------------------------------------------------------------

def depthwise_forward(X, W, b, stride, padding):
    """forward_cp + CUDA forward_conv (depthwise_convolution.py:85-121): per output, a
    sequential sum over taps i_f = r*S + s starting from 0."""
    C, R, S = W.shape
    Xp = pad_input(X, padding)
    OHf, OH = out_size(Xp.shape[2], R, stride)
    OWf, OW = out_size(Xp.shape[3], S, stride)
    out = np.zeros((X.shape[0], C, OH, OW), dtype=X.dtype)
    for r in range(R):
        for s in range(S):
            out += W[:, r, s][None, :, None, None] * Xp[:, :, r:r + stride * OH:stride, s:s + stride * OW:stride]
    if b is not None:
        out = out + b[None, :, None, None]
    return out, dict(Xp=Xp, OH=OH, OW=OW, OHf=OHf, OWf=OWf)


def depthwise_backward(dY, W, cache, stride, padding, with_bias, l2_strength=0.0):
    """backward_cp + CUDA backward_conv (depthwise_convolution.py:198-221, :122-140)."""
    C, R, S = W.shape
    Xp = cache["Xp"]
    OH, OW = cache["OH"], cache["OW"]
    db = dY.sum(axis=(0, 2, 3)) if with_bias else None
    dW = np.zeros_like(W)
    dXp = np.zeros_like(Xp)
    for r in range(R):
        for s in range(S):
            xs = Xp[:, :, r:r + stride * OH:stride, s:s + stride * OW:stride]
            dW[:, r, s] = (dY * xs).sum(axis=(0, 2, 3))
            dXp[:, :, r:r + stride * OH:stride, s:s + stride * OW:stride] += dY * W[:, r, s][None, :, None, None]
    if l2_strength:
        dW = dW + l2_backward(W, l2_strength)
    if padding > 0:
        return dXp[:, :, padding:-padding, padding:-padding], dW, db
    return dXp, dW, db


# ---------------------------------------------------------------------------------------
# pointwise convolution (layers/pointwise_convolution.py)
# ---------------------------------------------------------------------------------------

def pointwise_forward(X, W, b, stride):
    """pointwise_convolution.py:46-55."""
    if stride > 1:
        X = X[:, :, ::stride, ::stride]
    patches = X.transpose(0, 2, 3, 1).reshape(-1, W.shape[1])
    out = patches @ W.T
    if b is not None:
        out = out + b.reshape(1, -1)
    N, _, OH, OW = X.shape
    return out.reshape(N, OH, OW, W.shape[0]).transpose(0, 3, 1, 2), dict(patches=patches)


def pointwise_backward(dY, W, cache, stride, with_bias, l2_strength=0.0):
    """pointwise_convolution.py:57-75."""
    db = dY.sum(axis=(0, 2, 3)) if with_bias else None
    up = dY.transpose(0, 2, 3, 1).reshape(cache["patches"].shape[0], -1)
    dW = (up.T @ cache["patches"]).reshape(W.shape)
    if l2_strength:
        dW = dW + l2_backward(W, l2_strength)
    dx_rows = up @ W
    dx = dx_rows.reshape(dY.shape[0], dY.shape[2], dY.shape[3], W.shape[1]).transpose(0, 3, 1, 2)
    if stride > 1:
        wide = np.zeros((dx.shape[0], dx.shape[1], dx.shape[2] * stride, dx.shape[3] * stride), dtype=dx.dtype)
        wide[:, :, ::stride, ::stride] = dx
        return wide, dW, db
    return dx, dW, db


# ---------------------------------------------------------------------------------------
# dense (layers/dense_layer.py)
# ---------------------------------------------------------------------------------------

def dense_forward(X, W, b):
    """dense_layer.py:46-55."""
    out = X @ W
    if b is not None:
        out = out + b[None, :]
    return out


def dense_backward(dY, X, W, with_bias, l2_strength=0.0):
    """dense_layer.py:57-67."""
    db = dY.sum(axis=0) if with_bias else None
    dW = X.T @ dY
    if l2_strength:
        dW = dW + l2_backward(W, l2_strength)
    return dY @ W.T, dW, db


# ---------------------------------------------------------------------------------------
# batch norm (layers/batch_norm.py, GPU branch)
# ---------------------------------------------------------------------------------------

def bn_forward_train(X, gamma, beta, running_mean, running_std, eps=1e-5, momentum=0.95):
    """batch_norm.py:54-100.  Returns (Y, cache, running_mean, running_std)."""
    axis = (0, 2, 3) if X.ndim == 4 else 0
    mean = X.mean(axis=axis)
    var = X.var(axis=axis)
    std = np.sqrt(var + X.dtype.type(eps))
    if X.ndim == 4:
        std = std[None, :, None, None]
        mean = mean[None, :, None, None]
    X_demean = X - mean
    X_hat = X_demean / std
    if running_mean is not None:
        running_mean = momentum * running_mean + (1 - momentum) * mean
    else:
        running_mean = mean
    if running_std is not None:
        running_std = momentum * running_std + (1 - momentum) * std
    else:
        running_std = std
    out = gamma * X_hat + beta
    return out, dict(X_demean=X_demean, X_hat=X_hat, std=std, shape=X.shape), running_mean, running_std


def bn_forward_test(X, gamma, beta, running_mean, running_std):
    """batch_norm.py:101-115."""
    X_hat = (X - running_mean) / running_std
    return gamma * X_hat + beta


def bn_backward(dY, gamma, cache):
    """batch_norm.py:118-174.  Returns (dX, dgamma, dbeta)."""
    four = dY.ndim == 4
    axis = (0, 2, 3) if four else 0
    shape = cache["shape"]
    dgamma = (dY * cache["X_hat"]).sum(axis=axis)
    dbeta = dY.sum(axis=axis)
    upstream_mean = dY.mean(axis=axis)
    std_recip = 1.0 / cache["std"]
    if four:
        upstream_mean = upstream_mean[None, :, None, None]
        dgamma = dgamma[None, :, None, None]
        dbeta = dbeta[None, :, None, None]
    M = float(shape[0] * shape[2] * shape[3]) if four else float(shape[0])
    factor = gamma * std_recip
    other = (1.0 / M) * (cache["X_demean"] * (std_recip ** 2))
    dot_sum = (dY * cache["X_demean"]).sum(axis=axis)
    if four:
        dot_sum = dot_sum[None, :, None, None]
    dx = factor * (dY - upstream_mean - other * dot_sum)
    return dx.astype(dY.dtype), dgamma, dbeta


# ---------------------------------------------------------------------------------------
# activations, pooling head, loss, regulariser, optimiser
# ---------------------------------------------------------------------------------------

def relu_forward(X):
    """activations.py:37-42 (mask = out > 0)."""
    out = np.maximum(X.dtype.type(0), X)
    return out, (out > 0).astype(X.dtype)


def relu_backward(dY, mask):
    """activations.py:44-47."""
    return dY * mask


def gap_forward(X):
    """pooling.py:23-27."""
    return X.mean(axis=(2, 3))


def gap_backward(dY, spatial_shape):
    """pooling.py:29-36."""
    hw = float(np.prod(spatial_shape))
    return (1.0 / hw) * dY[:, :, None, None] * np.ones((dY.shape[0], dY.shape[1]) + tuple(spatial_shape),
                                                       dtype=dY.dtype)


def softmax_xent_forward(X, y_one_hot):
    """losses.py:13-27: no max shift; P = (1/sum e) * e; loss = mean(-log(P . y))."""
    e = np.exp(X)
    P = (1.0 / e.sum(axis=1)).reshape(-1, 1).astype(X.dtype) * e
    if y_one_hot is None:
        return 0, P
    picked = np.einsum("bij,bjk->b", P.reshape(P.shape[0], 1, P.shape[1]),
                       y_one_hot.reshape(P.shape[0], y_one_hot.shape[1], 1))
    loss = (1 / float(P.shape[0])) * np.sum(-np.log(picked))
    return loss, P


def softmax_xent_backward(P, y_one_hot):
    """losses.py:29-34."""
    return (1 / float(P.shape[0])) * (P - y_one_hot)


def l2_forward(W, strength):
    """regularisers/l2.py:12-14."""
    return 0.5 * strength * np.sum(np.power(W, 2))


def l2_backward(W, strength):
    """regularisers/l2.py:16-17."""
    return strength * W


def sgd_momentum_update(W, g, v, lr, momentum):
    """SGDMomentum.update_weights (SGDMomentum.py:33-39) for one tensor; returns (W, v)."""
    dx = -lr * g + momentum * v
    return W + dx, dx
