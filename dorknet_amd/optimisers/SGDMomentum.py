"""SGD with momentum (reference: optimisers/SGDMomentum.py).

Parameter discovery is the reference's (:7-14): every top-level layer with
``learned_params`` plus one level of ``layer_list`` -- so ResidualBlock skip
projections are *not* updated (a reference quirk, kept as the default).
``update_skip_projections=True`` (an extension, not in the reference) also updates each
ResidualBlock's ``skip_projection``; pass the same flag to ``parallel.DataParallel`` so
their gradients are all-reduced.  ``update_weights`` computes,
per parameter tensor, ``d = -lr * g + momentum * v;  W += d;  v = d`` (:31-39) -- as one
multi-tensor HIP launch over all tensors instead of ~4 CuPy kernels per tensor.
"""
from __future__ import annotations

import numpy as np
import torch

from .._hip import lib, stream_handle


class SGDMomentum:
    def __init__(self, network, learning_rate, momentum, update_skip_projections=False):
        self.network = network
        self.update_skip_projections = update_skip_projections
        # a data-parallel wrapper must all-reduce exactly the gradients this optimiser applies
        # (parallel.DataParallel checks the same pair from its side)
        dp_flag = getattr(network, "_dp_update_skip_projections", None)
        if dp_flag is not None and dp_flag != update_skip_projections:
            raise ValueError("SGDMomentum(update_skip_projections={}) disagrees with DataParallel's "
                             "update_skip_projections={}: skip-projection gradients would be applied "
                             "un-averaged".format(update_skip_projections, dp_flag))
        try:
            network._opt_update_skip_projections = update_skip_projections
        except AttributeError:
            pass
        self.learnable_layers = []
        for layer in network.layers:
            if layer.learned_params is not None:
                self.learnable_layers.append(layer)
            if hasattr(layer, "layer_list"):  # For composite layers like ResidualBlock
                for l in layer.layer_list:
                    if l.learned_params is not None:
                        self.learnable_layers.append(l)
                skip = getattr(layer, "skip_projection", None)
                if update_skip_projections and skip is not None and skip.learned_params:
                    self.learnable_layers.append(skip)
        self.learning_rate = learning_rate
        self.momentum = momentum
        self.grad_cache = {}
        for layer in self.learnable_layers:
            layer_d = {}
            for k, v in layer.grads.items():
                layer_d[k] = torch.zeros_like(v) if isinstance(v, torch.Tensor) else np.zeros_like(v)
            self.grad_cache[layer] = layer_d
        self._table = None
        self._table_sig = None
        self._total_blocks = 0

    def set_learning_rate(self, new_lr):
        self.learning_rate = new_lr

    def multiply_learning_rate(self, multiplier):
        self.learning_rate *= multiplier

    def _entries(self):
        out = []
        for layer in self.learnable_layers:
            for param in layer.learned_params.keys():
                w = layer.learned_params[param]
                g = layer.grads[param]
                v = self.grad_cache[layer][param]
                out.append((w, g, v))
        return out

    def _build_table(self, entries):
        rows = []
        block0 = 0
        for w, g, v in entries:
            for t in (w, g, v):
                if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32
                        and t.is_contiguous()):
                    raise RuntimeError("SGDMomentum: parameters, grads and velocities must be contiguous fp32 "
                                       "device tensors (build the optimiser after network.to_gpu())")
            n = w.numel()
            if g.numel() != n or v.numel() != n:
                raise ValueError("SGDMomentum: grad / velocity size mismatch")
            rows.append((w.data_ptr(), g.data_ptr(), v.data_ptr(), n, block0))
            block0 += -(-n // 256)
        table = np.array(rows, dtype=np.int64).reshape(-1, 5)
        self._table = torch.as_tensor(table, device="cuda")
        self._total_blocks = block0

    def update_weights(self):
        entries = self._entries()
        sig = tuple((w.data_ptr(), g.data_ptr(), v.data_ptr(), w.numel()) for w, g, v in entries)
        if sig != self._table_sig:
            self._build_table(entries)
            self._table_sig = sig
        lib.dk_sgd_momentum_multi_f32(self._table.data_ptr(), len(entries), self._total_blocks,
                                      float(self.learning_rate), float(self.momentum), 1.0, stream_handle())
