"""The reference's CPU path (is_on_gpu == False) restated.  TEST INFRASTRUCTURE ONLY.

Cython kernels -> C/OpenMP (csrc/dorknet_oracle.c), np.dot -> numpy BLAS, elementwise ->
numpy, exactly the structure of the reference's CPU branches:
  ConvLayer ............. convolution.py:76-83 (im2col_cy + dot), :119-126 (dot + row2im_cy)
  DepthwiseConvLayer .... depthwise_convolution.py:72-83 (depthwise_conv_cy),
                          :186-196 (depthwise_backward_direct_cy + sum over batch)
  BatchNormLayer ........ batch_norm.py:64-65 (channelwise_mean_and_var_4d), :145, :162 (einsum)
  ReLu .................. activations.py:18-27 (relu_cy)
Used as bench.py's cpu_baseline (kind "port") and to run BASELINE config 1 (MNISTNet).
"""
from __future__ import annotations

import numpy as np

from . import ref
from ._clib import lib, p
from .net import OBatchNorm, OConv, ODepthwise, OReLU


def _f32c(a):
    return np.ascontiguousarray(a, dtype=np.float32)


class CyConv(OConv):
    def forward(self, X, test_mode=False):
        W = self.learned_params["weights"]
        K, C, R, S = W.shape
        self.input_shape = X.shape
        Xp = _f32c(ref.pad_input(X, self.padding))
        N, _, Hp, Wp = Xp.shape
        self.OHf, OH = ref.out_size(Hp, R, self.stride)
        self.OWf, OW = ref.out_size(Wp, S, self.stride)
        self.OH, self.OW = OH, OW
        patches = np.empty((N * OH * OW, C * R * S), dtype=np.float32)
        lib().oracle_im2col(p(Xp), N, C, Hp, Wp, R, S, self.stride, OH, OW, p(patches))
        self.patches = patches
        out = np.dot(patches, W.reshape(K, -1).T)
        if "bias" in self.learned_params:
            out += self.learned_params["bias"].reshape(1, -1)
        return out.reshape(N, OH, OW, K).transpose(0, 3, 1, 2)

    def backward(self, dY):
        W = self.learned_params["weights"]
        K, C, R, S = W.shape
        if "bias" in self.learned_params:
            self.grads["bias"] = np.sum(dY, axis=(0, 2, 3))
        up = dY.transpose(0, 2, 3, 1).reshape(self.patches.shape[0], -1)
        dW = np.dot(up.T, self.patches).reshape(W.shape)
        if self.l2:
            dW += ref.l2_backward(W, self.l2)
        self.grads["weights"] = dW
        dx_rows = _f32c(np.dot(up, W.reshape(K, -1)))
        N = self.input_shape[0]
        Hpd = int(self.stride * (self.OHf - 1) + R)
        Wpd = int(self.stride * (self.OWf - 1) + S)
        padded = np.empty((N, C, Hpd, Wpd), dtype=np.float32)
        lib().oracle_row2im(p(dx_rows), N, C, Hpd, Wpd, R, S, self.stride, self.OH, self.OW, p(padded))
        pd = self.padding
        return padded[:, :, pd:-pd, pd:-pd].copy() if pd > 0 else padded


class CyDepthwise(ODepthwise):
    def forward(self, X, test_mode=False):
        W = _f32c(self.learned_params["weights"])
        C, R, S = W.shape
        Xp = _f32c(ref.pad_input(X, self.padding))
        N, _, Hp, Wp = Xp.shape
        self.OHf, OH = ref.out_size(Hp, R, self.stride)
        self.OWf, OW = ref.out_size(Wp, S, self.stride)
        self.Xp, self.OH, self.OW = Xp, OH, OW
        out = np.empty((N, C, OH, OW), dtype=np.float32)
        lib().oracle_depthwise_conv(p(Xp), p(W), N, C, Hp, Wp, R, S, self.stride, OH, OW, p(out))
        if "bias" in self.learned_params:
            out += self.learned_params["bias"][None, :, None, None]
        return out

    def backward(self, dY):
        W = _f32c(self.learned_params["weights"])
        C, R, S = W.shape
        dY = _f32c(dY)
        N, _, Hp, Wp = self.Xp.shape
        if "bias" in self.learned_params:
            self.grads["bias"] = np.sum(dY, axis=(0, 2, 3))
        Hpd = int(self.stride * (self.OHf - 1) + R)
        Wpd = int(self.stride * (self.OWf - 1) + S)
        padded = np.empty((N, C, Hpd, Wpd), dtype=np.float32)
        dw = np.empty((N, C, R, S), dtype=np.float32)
        lib().oracle_depthwise_backward(p(dY), p(self.Xp), p(W), N, C, Hp, Wp, R, S, self.stride, self.OH, self.OW,
                                        Hpd, Wpd, p(padded), p(dw))
        dWs = np.sum(dw, axis=0)
        if self.l2:
            dWs += ref.l2_backward(W, self.l2)
        self.grads["weights"] = dWs
        pd = self.padding
        return padded[:, :, pd:-pd, pd:-pd].copy() if pd > 0 else padded


class CyBatchNorm(OBatchNorm):
    def forward(self, X, test_mode=False):
        if test_mode or X.ndim != 4:
            return super().forward(X, test_mode)
        X = _f32c(X)
        N, C, H, W = X.shape
        mean = np.empty(C, dtype=np.float32)
        var = np.empty(C, dtype=np.float32)
        lib().oracle_bn_stats(p(X), N, C, H, W, p(mean), p(var))
        std = np.sqrt(var + self.eps)[None, :, None, None]
        mean = mean[None, :, None, None]
        X_demean = X - mean
        X_hat = X_demean / std
        nlp = self.non_learned_params
        nlp["running_mean"] = mean if nlp["running_mean"] is None else \
            self.momentum * nlp["running_mean"] + (1 - self.momentum) * mean
        nlp["running_std"] = std if nlp["running_std"] is None else \
            self.momentum * nlp["running_std"] + (1 - self.momentum) * std
        self.cache = dict(X_demean=X_demean, X_hat=X_hat, std=std, shape=X.shape)
        return self.learned_params["gamma"] * X_hat + self.learned_params["beta"]

    def backward(self, dY):
        if dY.ndim != 4:
            return super().backward(dY)
        c = self.cache
        N, C, H, W = c["shape"]
        gamma = self.learned_params["gamma"]
        self.grads["gamma"] = np.einsum("ijkl,ijkl->j", dY, c["X_hat"])[None, :, None, None]
        self.grads["beta"] = dY.sum(axis=(0, 2, 3))[None, :, None, None]
        upstream_mean = dY.mean(axis=(0, 2, 3))[None, :, None, None]
        std_recip = 1.0 / c["std"]
        factor = gamma * std_recip
        other = (1.0 / float(N * H * W)) * (c["X_demean"] * (std_recip ** 2))
        dot_sum = np.einsum("ijkl,ijkl->j", dY, c["X_demean"])[None, :, None, None]
        return (factor * (dY - upstream_mean - other * dot_sum)).astype(np.float32)


class CyReLU(OReLU):
    def forward(self, X, test_mode=False):
        X = _f32c(X)
        out = np.empty_like(X)
        mask = np.empty_like(X)
        lib().oracle_relu_forward_train(p(X), X.size, p(out), p(mask))
        if not test_mode:
            self.mask = mask
        return out
