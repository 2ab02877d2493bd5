"""An independent fp64 checker for full-size parity tests: a torch (CPU, float64, autograd) twin
of a dorknet_amd layer list, built from the layers' numpy parameters.  TEST INFRASTRUCTURE.

It restates the training-mode maths of the reference's layers in torch ops, not the reference's
code structure:
  ConvLayer            F.conv2d (cross-correlation, zero padding; layers/convolution.py:58-87)
  DepthwiseConvLayer   sum over taps of shifted slices of the zero-padded input
                       (layers/depthwise_convolution.py:85-121)
  PointwiseConvLayer   X[:, :, ::s, ::s] then a 1x1 contraction (layers/pointwise_convolution.py:46-55)
  BatchNormLayer       batch mean / population variance, eps 1e-5 (layers/batch_norm.py:54-100)
  ReLu                 max(0, x), gradient 0 at 0 (layers/activations.py:37-47)
  ResidualBlock        relu(chain(X) + skip(X)) (layers/residual_block.py:65-97)
  GlobalAveragePooling mean over H, W (layers/pooling.py:23-27)
  DenseLayer           X @ W + b, W stored (in, out) (layers/dense_layer.py:46-55)
  SoftmaxWithCrossEntropy (run(..., onehot=...)): p = exp(z) / sum exp(z) without a max shift,
                       loss = mean(-log(p . y)); autograd of that loss w.r.t. z is the reference's
                       (p - y) / N for one-hot y (layers/losses.py:13-34)
  l2                   + strength * W in each weight gradient (regularisers/l2.py:16-17); with a
                       loss, 0.5 * strength * sum W^2 of every layer but the skip projections in
                       the loss (feed_forward_network.py:54-60, residual_block.py:78-84)
Cross-checked against the numpy oracle at small sizes by tests/test_torch_twin.py.

Every BatchNorm output's incoming gradient is also summarised per channel as sum|g| (the l1
scale of the sums dbeta = sum g and dgamma = sum g*x_hat): a BN followed by a pointwise layer
and another BN has dbeta = 0 in exact arithmetic, so its error is bounded by that scale.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def _np(v, dtype=np.float64):
    if isinstance(v, torch.Tensor):
        v = v.detach().cpu().numpy()
    return np.asarray(v, dtype=dtype)


class TorchTwin:
    """dtype float64: the checker; float32: the same maths in fp32, whose distance from the
    fp64 twin measures the problem's own fp32 conditioning (at batch 256, ReLU masks of
    elements within an ulp of the threshold flip between any two fp32 pipelines)."""

    def __init__(self, layers, dtype=np.float64):
        self.layers = layers
        self.dtype = dtype
        self.params = {}      # (layer_name, key) -> leaf float64 tensor
        self.l2 = {}          # layer_name -> strength
        self.bn_l1 = {}       # bn layer_name -> per-channel sum |dL/dy|
        self.bn_stats = {}    # bn layer_name -> (mean, std)
        for l in self._all(layers):
            for k, v in (l.learned_params or {}).items():
                self.params[(l.layer_name, k)] = torch.tensor(_np(v, dtype), requires_grad=True)
            reg = getattr(l, "weight_regulariser", None)
            if reg is not None:
                self.l2[l.layer_name] = float(reg.strength)

    @staticmethod
    def _all(layers):
        out = []
        for l in layers:
            out.append(l)
            if hasattr(l, "layer_list"):
                out += TorchTwin._all(l.layer_list)
                if getattr(l, "skip_projection", None) is not None:
                    out.append(l.skip_projection)
        return out

    def _p(self, l, k):
        return self.params[(l.layer_name, k)]

    def _layer(self, l, x):
        from dorknet_amd.layers.activations import ReLu
        from dorknet_amd.layers.batch_norm import BatchNormLayer
        from dorknet_amd.layers.convolution import ConvLayer
        from dorknet_amd.layers.dense_layer import DenseLayer
        from dorknet_amd.layers.depthwise_convolution import DepthwiseConvLayer
        from dorknet_amd.layers.pointwise_convolution import PointwiseConvLayer
        from dorknet_amd.layers.pooling import GlobalAveragePoolingLayer
        from dorknet_amd.layers.residual_block import ResidualBlock
        has_b = "bias" in (l.learned_params or {})
        if isinstance(l, ConvLayer):
            return F.conv2d(x, self._p(l, "weights"), self._p(l, "bias") if has_b else None,
                            stride=l.stride, padding=l.padding)
        if isinstance(l, DepthwiseConvLayer):
            w = self._p(l, "weights")
            C, R, S = w.shape
            s, p = l.stride, l.padding
            xp = F.pad(x, (p, p, p, p))
            OH = (x.shape[2] + 2 * p - R) // s + 1
            OW = (x.shape[3] + 2 * p - S) // s + 1
            y = 0
            for r in range(R):
                for c in range(S):
                    tap = xp[:, :, r:r + s * (OH - 1) + 1:s, c:c + s * (OW - 1) + 1:s]
                    y = y + tap * w[:, r, c].view(1, C, 1, 1)
            if has_b:
                y = y + self._p(l, "bias").view(1, C, 1, 1)
            return y
        if isinstance(l, PointwiseConvLayer):
            xs = x[:, :, ::l.stride, ::l.stride]
            y = torch.einsum("nchw,kc->nkhw", xs, self._p(l, "weights"))
            if has_b:
                y = y + self._p(l, "bias").view(1, -1, 1, 1)
            return y
        if isinstance(l, BatchNormLayer):
            mean = x.mean(dim=(0, 2, 3), keepdim=True)
            var = x.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
            std = torch.sqrt(var + l.eps)
            self.bn_stats[l.layer_name] = (mean.detach().view(-1), std.detach().view(-1))
            y = (x - mean) / std * self._p(l, "gamma") + self._p(l, "beta")
            if y.requires_grad:
                name = l.layer_name

                def hook(g, name=name):
                    self.bn_l1[name] = g.abs().sum(dim=(0, 2, 3)).detach()
                y.register_hook(hook)
            return y
        if isinstance(l, ReLu):
            return torch.relu(x)
        if isinstance(l, GlobalAveragePoolingLayer):
            return x.mean(dim=(2, 3))
        if isinstance(l, DenseLayer):
            y = x @ self._p(l, "weights")
            return y + self._p(l, "bias").view(1, -1) if has_b else y
        if isinstance(l, ResidualBlock):
            h = x
            for c in l.layer_list:
                h = self._layer(c, h)
            skip = self._layer(l.skip_projection, x) if l.skip_projection is not None else x
            return self._layer(l.post_skip_activation, h + skip)
        raise TypeError(type(l))

    def _l2_loss(self):
        """0.5 * strength * sum W^2 over the layers whose regulariser enters the loss: every layer
        with one except the skip projections (their l2 is in the gradient only)."""
        tot = 0
        def walk(layers):
            nonlocal tot
            for l in layers:
                if l.layer_name in self.l2:
                    tot = tot + 0.5 * self.l2[l.layer_name] * (self._p(l, "weights") ** 2).sum()
                if hasattr(l, "layer_list"):
                    walk(l.layer_list)
        walk(self.layers)
        return tot

    def run(self, X, dY, input_grad=True, onehot=None):
        """Forward on X (numpy/tensor), backward of dY; returns (Y, dX or None, grads) with
        grads[(layer_name, key)] including the l2 term.  With `onehot` the layers end in the
        softmax + cross-entropy loss: Y = the probabilities, the backward starts from the loss
        (dY unused), and self.loss holds the loss (l2 terms included)."""
        x = torch.tensor(_np(X, self.dtype), requires_grad=input_grad)
        h = x
        for l in self.layers:
            h = self._layer(l, h)
        if onehot is None:
            h.backward(torch.as_tensor(_np(dY, self.dtype)))
        else:
            e = torch.exp(h)
            p = e / e.sum(dim=1, keepdim=True)
            y = torch.as_tensor(_np(onehot, self.dtype))
            loss = (-torch.log((p * y).sum(dim=1))).mean()
            self.loss = float((loss + self._l2_loss()).detach())
            loss.backward()
            h = p
        grads = {}
        for (name, k), p in self.params.items():
            g = p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p)
            if k == "weights" and name in self.l2:
                g = g + self.l2[name] * p.detach()
            grads[(name, k)] = g.numpy().astype(np.float64)
        return (h.detach().numpy().astype(np.float64), (x.grad.numpy().astype(np.float64) if input_grad else None),
                grads)
