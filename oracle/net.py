"""CPU restatement of the reference's layer objects, network and optimiser (numpy).
TEST INFRASTRUCTURE ONLY -- see oracle/ref.py for the parity status ("parity unpinned").

Mirrors the reference's object model closely enough to run whole training steps:
  layers ......... layers/*.py (forward / backward / learned_params / grads)
  residual block . layers/residual_block.py:65-97
  network ........ network/feed_forward_network.py:47-70
  optimiser ...... optimisers/SGDMomentum.py:4-39 (skip projections are not updated)
Parameters are passed in explicitly (copied from the product network under test), so
both sides start from identical weights.
"""
from __future__ import annotations

import numpy as np

from . import ref


class OLayer:
    def __init__(self, name):
        self.layer_name = name
        self.learned_params = None
        self.grads = None
        self.l2 = 0.0

    def regulariser_forward(self):
        if self.l2 and self.learned_params is not None:
            return ref.l2_forward(self.learned_params["weights"], self.l2)
        return 0.0


class OConv(OLayer):
    def __init__(self, name, W, b, stride, padding, l2=0.0):
        super().__init__(name)
        self.learned_params = {"weights": W} if b is None else {"weights": W, "bias": b}
        self.grads = {k: np.zeros_like(v) for k, v in self.learned_params.items()}
        self.stride, self.padding, self.l2 = stride, padding, l2

    def forward(self, X, test_mode=False):
        Y, self.cache = ref.conv_forward(X, self.learned_params["weights"], self.learned_params.get("bias"),
                                         self.stride, self.padding)
        return Y

    def backward(self, dY):
        dX, dW, db = ref.conv_backward(dY, self.learned_params["weights"], self.cache, self.stride, self.padding,
                                       "bias" in self.learned_params, self.l2)
        self.grads["weights"] = dW
        if db is not None:
            self.grads["bias"] = db
        return dX


class ODepthwise(OLayer):
    def __init__(self, name, W, b, stride, padding, l2=0.0):
        super().__init__(name)
        self.learned_params = {"weights": W} if b is None else {"weights": W, "bias": b}
        self.grads = {k: np.zeros_like(v) for k, v in self.learned_params.items()}
        self.stride, self.padding, self.l2 = stride, padding, l2

    def forward(self, X, test_mode=False):
        Y, self.cache = ref.depthwise_forward(X, self.learned_params["weights"], self.learned_params.get("bias"),
                                              self.stride, self.padding)
        return Y

    def backward(self, dY):
        dX, dW, db = ref.depthwise_backward(dY, self.learned_params["weights"], self.cache, self.stride,
                                            self.padding, "bias" in self.learned_params, self.l2)
        self.grads["weights"] = dW
        if db is not None:
            self.grads["bias"] = db
        return dX


class OPointwise(OLayer):
    def __init__(self, name, W, b, stride, l2=0.0):
        super().__init__(name)
        self.learned_params = {"weights": W} if b is None else {"weights": W, "bias": b}
        self.grads = {k: np.zeros_like(v) for k, v in self.learned_params.items()}
        self.stride, self.l2 = stride, l2

    def forward(self, X, test_mode=False):
        Y, self.cache = ref.pointwise_forward(X, self.learned_params["weights"], self.learned_params.get("bias"),
                                              self.stride)
        return Y

    def backward(self, dY):
        dX, dW, db = ref.pointwise_backward(dY, self.learned_params["weights"], self.cache, self.stride,
                                            "bias" in self.learned_params, self.l2)
        self.grads["weights"] = dW
        if db is not None:
            self.grads["bias"] = db
        return dX


class ODense(OLayer):
    def __init__(self, name, W, b, l2=0.0):
        super().__init__(name)
        self.learned_params = {"weights": W} if b is None else {"weights": W, "bias": b}
        self.grads = {k: np.zeros_like(v) for k, v in self.learned_params.items()}
        self.l2 = l2

    def forward(self, X, test_mode=False):
        self.X = X
        return ref.dense_forward(X, self.learned_params["weights"], self.learned_params.get("bias"))

    def backward(self, dY):
        dX, dW, db = ref.dense_backward(dY, self.X, self.learned_params["weights"], "bias" in self.learned_params,
                                        self.l2)
        self.grads["weights"] = dW
        if db is not None:
            self.grads["bias"] = db
        return dX


class OBatchNorm(OLayer):
    def __init__(self, name, gamma, beta, eps=1e-5, momentum=0.95):
        super().__init__(name)
        self.learned_params = {"gamma": gamma, "beta": beta}
        self.grads = {k: np.zeros_like(v) for k, v in self.learned_params.items()}
        self.non_learned_params = {"running_mean": None, "running_std": None}
        self.eps, self.momentum = eps, momentum

    def forward(self, X, test_mode=False):
        g, b = self.learned_params["gamma"], self.learned_params["beta"]
        if test_mode:
            return ref.bn_forward_test(X, g, b, self.non_learned_params["running_mean"],
                                       self.non_learned_params["running_std"])
        Y, self.cache, rm, rs = ref.bn_forward_train(X, g, b, self.non_learned_params["running_mean"],
                                                     self.non_learned_params["running_std"], self.eps,
                                                     self.momentum)
        self.non_learned_params["running_mean"], self.non_learned_params["running_std"] = rm, rs
        return Y

    def backward(self, dY):
        dX, dg, db = ref.bn_backward(dY, self.learned_params["gamma"], self.cache)
        self.grads["gamma"], self.grads["beta"] = dg, db
        return dX


class OReLU(OLayer):
    """activations.py:37-47.  `replay`: a bool mask that decides the next training forward instead
    of out > 0 (the tests hand in the GPU's own decisions, so that an fp32 tie -- an input within
    rounding of zero -- takes the same side in both; tests/_ties.py).  The pre-activation of that
    forward is kept in `pre` for the tie analysis."""
    replay = None

    def forward(self, X, test_mode=False):
        if self.replay is not None and not test_mode:
            m = np.asarray(self.replay, dtype=bool)
            if m.shape != X.shape:
                raise ValueError("replayed mask shape {} != input {}".format(m.shape, X.shape))
            self.replay, self.pre = None, X
            self.mask = m.astype(X.dtype)
            return X * self.mask
        Y, mask = ref.relu_forward(X)
        if not test_mode:
            self.mask, self.pre = mask, X
        return Y

    def backward(self, dY):
        return ref.relu_backward(dY, self.mask)


class OGAP(OLayer):
    def forward(self, X, test_mode=False):
        self.spatial = X.shape[-2:]
        return ref.gap_forward(X)

    def backward(self, dY):
        return ref.gap_backward(dY, self.spatial)


class OResidual(OLayer):
    def __init__(self, name, layer_list, skip=None, post=None):
        super().__init__(name)
        self.layer_list, self.skip_projection = layer_list, skip
        self.post_skip_activation = post if post is not None else OReLU(name + "_post")

    def forward(self, X, test_mode=False):
        t = X
        for l in self.layer_list:
            t = l.forward(t, test_mode)
        s = self.skip_projection.forward(X, test_mode) if self.skip_projection is not None else X
        return self.post_skip_activation.forward(t + s, test_mode)

    def regulariser_forward(self):
        return sum(l.regulariser_forward() for l in self.layer_list)

    def backward(self, dY):
        j = self.post_skip_activation.backward(dY)
        dx = j
        for l in reversed(self.layer_list):
            dx = l.backward(dx)
        if self.skip_projection is not None:
            return dx + self.skip_projection.backward(j)
        return dx + j


class OSoftmaxXent(OLayer):
    def forward(self, X, y_one_hot=None, test_mode=False):
        loss, P = ref.softmax_xent_forward(X, None if test_mode else y_one_hot)
        if not test_mode:
            self.P, self.y = P, y_one_hot
        return loss, P

    def backward(self, dY=None):
        return ref.softmax_xent_backward(self.P, self.y)


class ONetwork:
    def __init__(self, layers, loss_layer):
        self.layers, self.loss_layer = layers, loss_layer

    def forward(self, X, y_one_hot, test_mode=False):
        reg = []
        for l in self.layers:
            X = l.forward(X, test_mode)
            if not test_mode:
                reg.append(l.regulariser_forward())
        loss, P = self.loss_layer.forward(X, y_one_hot, test_mode)
        return loss + sum(reg), P

    def backward(self):
        dy = self.loss_layer.backward()
        for l in reversed(self.layers):
            dy = l.backward(dy)
        return dy


class OSGDMomentum:
    """SGDMomentum.py:4-39 including the top-level + one-level-of-layer_list discovery."""

    def __init__(self, net, lr, momentum, update_skip_projections=False):
        self.lr, self.momentum = lr, momentum
        self.learnable = []
        for l in net.layers:
            if l.learned_params is not None:
                self.learnable.append(l)
            if hasattr(l, "layer_list"):
                for c in l.layer_list:
                    if c.learned_params is not None:
                        self.learnable.append(c)
                # the build's update_skip_projections extension (default False = the reference)
                skip = getattr(l, "skip_projection", None)
                if update_skip_projections and skip is not None and skip.learned_params:
                    self.learnable.append(skip)
        self.cache = {id(l): {k: np.zeros_like(v) for k, v in l.grads.items()} for l in self.learnable}

    def update_weights(self):
        for l in self.learnable:
            for k in l.learned_params:
                w, v = ref.sgd_momentum_update(l.learned_params[k], l.grads[k], self.cache[id(l)][k], self.lr,
                                               self.momentum)
                l.learned_params[k] = w
                self.cache[id(l)][k] = v
