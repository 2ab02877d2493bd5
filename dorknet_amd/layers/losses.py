"""Softmax + cross-entropy (reference: layers/losses.py).

Same maths as the reference, including its quirks: no max-subtraction before exp
(:15-16), probabilities formed as (1/sum(e)) * e, loss = mean(-log(p . y_one_hot))
(:23-26), gradient (p - y)/N (:34).  ``forward`` returns (loss, probabilities); the loss
is a 0-d device tensor (the reference returns a 0-d cupy array).
"""
from __future__ import annotations

import torch

from .._hip import lib, stream_handle
from .._tensor import rows
from .layer import Layer


class SoftmaxWithCrossEntropy(Layer):

    def __init__(self, layer_name):
        super().__init__(layer_name)

    def __repr__(self):
        return "SoftmaxWithCrossEntropy({})".format(self.layer_name)

    def forward(self, X, y_one_hot=None, test_mode=False):
        x = rows(X)
        if x.device.type != "cuda":
            raise RuntimeError("SoftmaxWithCrossEntropy runs on the MI355X only")
        B, K = x.shape
        p = torch.empty_like(x)
        st = stream_handle()
        if test_mode:
            lib.dk_softmax_xent_fwd_f32(x.data_ptr(), 0, B, K, p.data_ptr(), 0, st)
            return 0, p
        y = rows(y_one_hot)
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        lib.dk_softmax_xent_fwd_f32(x.data_ptr(), y.data_ptr(), B, K, p.data_ptr(), loss.data_ptr(), st)
        self.y_one_hot = y
        self.downstream_x = p
        return loss, p

    def backward(self, upstream_dx=None):
        """upstream_dx is not used"""
        p, y = self.downstream_x, self.y_one_hot
        B, K = p.shape
        dx = torch.empty_like(p)
        lib.dk_softmax_xent_bwd_f32(p.data_ptr(), y.data_ptr(), B, K, dx.data_ptr(), stream_handle())
        return dx

    def save_to_h5(self, open_f, save_grads=True):
        from ..network.checkpoint import save_layer
        save_layer(self, open_f, save_grads)

    def load_from_h5(self, open_f, load_grads=True):
        pass
