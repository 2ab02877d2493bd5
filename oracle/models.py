"""The reference's example models as oracle networks.  TEST INFRASTRUCTURE ONLY.

  resnet18_depsep ... examples/imagenet_dogs_225_resnet_18_depsep.py:34-160
  mnist_net ......... examples/MNIST_basic_convnet.py:15-69

``backend="np"`` builds from oracle/net.py (numpy restatement of the GPU branch);
``backend="cy"`` builds the reference's CPU path (oracle/cpu_path.py: C/OpenMP kernels +
numpy BLAS).  Weights: ``params[layer_name]`` if given, else 0.01 * randn from `rng`
(the reference's "normal" initialiser); BN gamma = 1, beta = 0.
"""
from __future__ import annotations

import numpy as np

from . import cpu_path
from .net import (OBatchNorm, OConv, ODense, ODepthwise, OGAP, ONetwork, OPointwise, OReLU, OResidual,
                  OSoftmaxXent)


class _Builder:
    def __init__(self, backend, params, rng, dtype):
        self.cy = backend == "cy"
        self.params = params or {}
        self.rng = rng if rng is not None else np.random.RandomState(0)
        self.dtype = dtype

    def _w(self, name, shape):
        if name in self.params:
            return np.asarray(self.params[name]["weights"], dtype=self.dtype)
        return (0.01 * self.rng.randn(*shape)).astype(self.dtype)

    def _b(self, name, n, with_bias):
        if not with_bias:
            return None
        if name in self.params and "bias" in self.params[name]:
            return np.asarray(self.params[name]["bias"], dtype=self.dtype)
        return np.zeros(n, dtype=self.dtype)

    def conv(self, name, shape, stride, padding, with_bias, l2):
        cls = cpu_path.CyConv if self.cy else OConv
        return cls(name, self._w(name, shape), self._b(name, shape[0], with_bias), stride, padding, l2)

    def dw(self, name, shape, stride, padding, l2=0.0):
        cls = cpu_path.CyDepthwise if self.cy else ODepthwise
        return cls(name, self._w(name, shape), None, stride, padding, l2)

    def pw(self, name, shape, stride, l2):
        return OPointwise(name, self._w(name, shape), None, stride, l2)

    def dense(self, name, fin, fout, l2):
        return ODense(name, self._w(name, (fin, fout)), self._b(name, fout, True), l2)

    def bn(self, name, c, four=True):
        cls = cpu_path.CyBatchNorm if self.cy else OBatchNorm
        shape = (1, c, 1, 1) if four else (c,)
        p = self.params.get(name, {})
        g = np.asarray(p.get("gamma", np.ones(shape)), dtype=self.dtype).reshape(shape)
        b = np.asarray(p.get("beta", np.zeros(shape)), dtype=self.dtype).reshape(shape)
        return cls(name, g, b)

    def relu(self, name):
        return cpu_path.CyReLU(name) if self.cy else OReLU(name)


def resnet18_depsep(backend="np", params=None, rng=None, dtype=np.float32, num_classes=120):
    b = _Builder(backend, params, rng, dtype)

    def dsep(name, inc, fbs, stride, final_relu):
        out = [b.dw(name + "_dw", (inc, fbs[-2], fbs[-1]), stride, 1),
               b.bn(name + "_dw_bn", inc),
               b.pw(name + "_pw", (fbs[0], inc), 1, 1e-4),
               b.bn(name + "_pw_bn", fbs[0])]
        if final_relu:
            out.append(b.relu(name + "pw_relu"))
        return out

    def res_block(name, shape, downsample=False):
        nf, inc, fr, fc = shape
        ll = dsep(name + "_dw1", inc, shape, 2 if downsample else 1, True)
        ll += dsep(name + "_dw2", nf, (nf, nf, fr, fc), 1, False)
        skip = b.pw(name + "_pw_skip", (nf, inc), 2, 1e-4) if downsample else None
        return OResidual(name, ll, skip, b.relu(name + "_relu2"))

    layers = [b.conv("conv0", (64, 3, 5, 5), 2, 1, False, 1e-4), b.bn("conv0_bn", 64), b.relu("conv0_relu"),
              b.pw("pw0", (64, 64), 2, 1e-4), b.bn("pw0_bn", 64), b.relu("pw0_relu"),
              res_block("res1", (64, 64, 3, 3)), res_block("res2", (64, 64, 3, 3)),
              res_block("res3", (128, 64, 3, 3), True), res_block("res4", (128, 128, 3, 3)),
              res_block("res5", (256, 128, 3, 3), True), res_block("res6", (256, 256, 3, 3)),
              res_block("res7", (512, 256, 3, 3), True), res_block("res8", (512, 512, 3, 3)),
              OGAP("global_pool1"), b.dense("dense1", 512, num_classes, 1e-4)]
    return ONetwork(layers, OSoftmaxXent("softmax1"))


def mnist_net(backend="cy", params=None, rng=None, dtype=np.float32):
    b = _Builder(backend, params, rng, dtype)
    L = []
    for i, (shape, stride) in enumerate([((32, 1, 3, 3), 1), ((32, 32, 3, 3), 1), ((64, 32, 4, 4), 2),
                                         ((64, 64, 3, 3), 1), ((128, 64, 4, 4), 2)], start=1):
        L += [b.conv("conv_%d" % i, shape, stride, 1, False, 1e-4), b.bn("bn_%d" % i, shape[0]),
              b.relu("relu_%d" % min(i, 4))]
    L += [OGAP("global_pool"), b.dense("dense_1", 128, 10, 5e-4)]
    return ONetwork(L, OSoftmaxXent("softmax"))
