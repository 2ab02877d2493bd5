"""Global average pooling (reference: layers/pooling.py:10-43).

``forward``: mean over (H, W) -> (N, C); ``backward``: (1/(H*W)) * dy broadcast back.
(MaxPoolLayer, pooling.py:45-77, is CPU-only in the reference and used by no example:
out of scope, see DESIGN.md.)
"""
from __future__ import annotations

import torch

from .._hip import lib, stream_handle
from .._tensor import empty_nhwc, rows, to_nhwc
from .layer import Layer


class GlobalAveragePoolingLayer(Layer):
    """
    Takes the mean over spatial dimensions, reducing to one feature per channel per image
    """

    def __init__(self, layer_name):
        super().__init__(layer_name)

    def __repr__(self):
        return "GlobalAveragePoolingLayer({})".format(self.layer_name)

    def forward(self, X, test_mode=False):
        self._require_on_gpu()
        x = to_nhwc(X)
        N, C, H, W = x.shape
        self.spatial_shape = (H, W)
        out = torch.empty((N, C), dtype=torch.float32, device=x.device)
        lib.dk_gap_fwd_f32(x.data_ptr(), N, H * W, C, out.data_ptr(), stream_handle())
        return out

    def backward(self, upstream_dx):
        self._require_on_gpu()
        dy = rows(upstream_dx)
        N, C = dy.shape
        H, W = self.spatial_shape
        dx = empty_nhwc(N, C, H, W)
        lib.dk_gap_bwd_f32(dy.data_ptr(), N, H * W, C, dx.data_ptr(), stream_handle())
        return dx

    def save_to_h5(self, open_f, save_grads=True):
        from ..network.checkpoint import save_layer
        save_layer(self, open_f, save_grads)

    def load_from_h5(self, open_f, load_grads=True):
        pass
