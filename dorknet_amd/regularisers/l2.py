"""L2 weight regulariser (reference: regularisers/l2.py:4-17).

``forward(W) = 0.5 * strength * sum(W**2)`` (a 0-d device tensor) and
``backward(W) = strength * W``.  Inside the conv / pointwise / dense backward passes the
``+ strength * W`` term is folded into the weight-gradient reduction instead of being a
separate pass (convolution.py:99-100 adds it afterwards).
"""
from __future__ import annotations

import torch

from .._hip import lib, stream_handle
from .._tensor import as_device


class l2:
    def __init__(self, strength=0.005):
        self.type = "l2"
        self.strength = strength

    def __repr__(self):
        return "l2(strength={})".format(self.strength)

    def forward(self, X):
        X = as_device(X).contiguous()
        out = torch.empty((), dtype=torch.float32, device=X.device)
        lib.dk_l2_loss_f32(X.data_ptr(), X.numel(), float(self.strength), 0, out.data_ptr(), stream_handle())
        return out

    def backward(self, X):
        X = as_device(X).contiguous()
        out = torch.empty_like(X)
        lib.dk_scale_f32(X.data_ptr(), X.numel(), float(self.strength), out.data_ptr(), stream_handle())
        return out
