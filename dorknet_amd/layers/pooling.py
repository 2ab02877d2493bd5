"""Global average pooling (reference: layers/pooling.py:10-43).

``forward``: mean over (H, W) -> (N, C); ``backward``: (1/(H*W)) * dy broadcast back.
(MaxPoolLayer, pooling.py:45-77, is CPU-only in the reference and used by no example:
out of scope, see DESIGN.md.)
"""
from __future__ import annotations

import torch

from .._env import getenv
from .._hip import lib, stream_handle
from .._tensor import empty_nhwc, rows, to_nhwc
from ._bn_input import JoinOut
from .layer import Layer


class GlobalAveragePoolingLayer(Layer):
    """
    Takes the mean over spatial dimensions, reducing to one feature per channel per image
    """

    def __init__(self, layer_name):
        super().__init__(layer_name)

    def __repr__(self):
        return "GlobalAveragePoolingLayer({})".format(self.layer_name)

    def takes_join_input(self):
        """forward(JoinOut): the last residual block's output is pooled as it is formed
        (dk_gap_join_fwd_f32, bit-identical to the join pass + the pooling) and never stored."""
        from ._chain import fusion_enabled
        return fusion_enabled() and getenv("DORKNET_FUSE_JOIN_FWD") != "0"

    def forward(self, X, test_mode=False):
        self._require_on_gpu()
        if isinstance(X, JoinOut):
            if not X.written and X.dim() == 4 and X.dtype == torch.float32:
                return self._forward_join(X, test_mode)
            X = X.materialize()
        x = to_nhwc(X)
        N, C, H, W = x.shape
        self.spatial_shape = (H, W)
        out = torch.empty((N, C), dtype=torch.float32, device=x.device)
        lib.dk_gap_fwd_f32(x.data_ptr(), N, H * W, C, out.data_ptr(), stream_handle())
        return out

    def _forward_join(self, J, test_mode):
        N, C, H, W = J.shape
        self.spatial_shape = (H, W)
        out = torch.empty((N, C), dtype=torch.float32, device=J.device)
        if not test_mode and J.mask is None:
            # the join's ReLU backward takes its mask (y itself is never stored)
            J.mask = torch.empty((N, C, H, W), dtype=torch.uint8, device=J.device, memory_format=torch.channels_last)
        a, b = J.join_args()[:6], J.join_args()[6:12]
        lib.dk_gap_join_fwd_f32(*a, *b, N, H * W, C, 0 if J.mask is None else J.mask.data_ptr(), out.data_ptr(),
                                stream_handle())
        J.mark_pooled()
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
