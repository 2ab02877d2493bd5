"""Fully connected layer (reference: layers/dense_layer.py).

``Y = X . W + b`` with W stored (in, out) exactly as the reference (:20-25); forward,
dgrad and wgrad (+ l2) run on the same MFMA GEMM engine as the convolutions
(dk_dense_fwd_f32 / _dgrad_f32 / _wgrad_f32).
"""
from __future__ import annotations

from .._hip import lib, stream_handle, weight_grad_stream, workspace
from .._tensor import ptr, rows
from ._common import add_regulariser_grad, grad_buffer, init_weights, l2_strength
from .layer import Layer

import torch


class DenseLayer(Layer):

    def __init__(self, layer_name, incoming_chans=None, output_dim=None, with_bias=True,
                 weight_regulariser=None, weight_initialiser="normal"):
        super().__init__(layer_name)
        self.incoming_chans = incoming_chans
        self.output_dim = output_dim
        self.with_bias = with_bias
        self.weight_regulariser = weight_regulariser
        self.downstream_X = None
        self.weight_initialiser = weight_initialiser
        if incoming_chans is not None and output_dim is not None:
            weights = init_weights((incoming_chans, output_dim), weight_initialiser, incoming_chans + output_dim)
            self.learned_params = {"weights": weights}
            self.grads = {"weights": weights * 0}
            if with_bias:
                bias = (weights[0, :] * 0).copy()
                self.learned_params["bias"] = bias
                self.grads["bias"] = bias * 0
        else:
            self.learned_params = {}
            self.grads = {}

    def __repr__(self):
        return "DenseLayer({}, incoming_chans={}, output_dim={}, weight_regulariser={})".format(
            self.layer_name, self.incoming_chans, self.output_dim, repr(self.weight_regulariser))

    def forward(self, X, test_mode=False):
        self._require_on_gpu()
        st = stream_handle()
        x = rows(X)
        B, IN = x.shape
        w = self.learned_params["weights"]
        OUT = w.shape[1]
        if not test_mode:
            self.downstream_X = x
        y = torch.empty((B, OUT), dtype=torch.float32, device=x.device)
        bias = self.learned_params["bias"] if self.with_bias else None
        lib.dk_dense_fwd_f32(x.data_ptr(), B, IN, w.data_ptr(), OUT, ptr(bias), y.data_ptr(), st)
        return y

    def backward(self, upstream_dx):
        self._require_on_gpu()
        st = stream_handle()
        dy = rows(upstream_dx)
        x = self.downstream_X
        B, IN = x.shape
        w = self.learned_params["weights"]
        OUT = w.shape[1]
        # the parameter gradients on the side stream (_hip.weight_grad_stream), beside the dgrad
        with weight_grad_stream(dy, x):
            sst = stream_handle()
            if self.with_bias:
                gb = grad_buffer(self, "bias", (OUT,))
                nb = lib.dk_colsum_workspace_bytes(B, OUT)
                lib.dk_colsum_f32(dy.data_ptr(), B, OUT, gb.data_ptr(), workspace.get(nb), nb, sst)
            gw = grad_buffer(self, "weights", (IN, OUT))
            s = l2_strength(self.weight_regulariser)
            nb = lib.dk_dense_wgrad_workspace_bytes(B, IN, OUT)
            lib.dk_dense_wgrad_f32(x.data_ptr(), dy.data_ptr(), B, IN, OUT, w.data_ptr() if s else 0, s or 0.0,
                                   gw.data_ptr(), workspace.get(nb), nb, sst)
            if s is None:
                add_regulariser_grad(gw, w, self.weight_regulariser)
        dx = torch.empty((B, IN), dtype=torch.float32, device=x.device)
        lib.dk_dense_dgrad_f32(dy.data_ptr(), B, OUT, w.data_ptr(), IN, dx.data_ptr(), st)
        return dx

    def save_to_h5(self, open_f, save_grads=True):
        from ..network.checkpoint import save_layer
        save_layer(self, open_f, save_grads)

    def load_from_h5(self, open_f, load_grads=True):
        from ..network.checkpoint import load_layer
        load_layer(self, open_f, load_grads)
