"""Sequential network container (reference: network/feed_forward_network.py).

Same API: ``add_layer``, ``set_loss_layer``, ``to_gpu``, ``forward(X, y_one_hot,
test_mode=False, terminal_layer_name=None) -> (loss, X)``, ``backward()``, ``test``,
``save_weights_to_h5``, ``save_layer_structure_to_json``,
``load_network_from_json_and_h5``.  The forward pass runs (BatchNormLayer, ReLu) pairs
fused (layers/_chain.py) and remembers the steps it took for ``backward``.
"""
from __future__ import annotations

import json

import numpy as np

from ..layers._bn_input import materialize
from ..layers._chain import chain_backward, execute
from ..layers.activations import ReLu  # noqa: F401  (re-exported names used by loaders)
from ..layers.batch_norm import BatchNormLayer  # noqa: F401
from ..layers.convolution import ConvLayer  # noqa: F401
from ..layers.dense_layer import DenseLayer  # noqa: F401
from ..layers.depthwise_convolution import DepthwiseConvLayer  # noqa: F401
from ..layers.losses import SoftmaxWithCrossEntropy  # noqa: F401
from ..layers.pointwise_convolution import PointwiseConvLayer  # noqa: F401
from ..layers.pooling import GlobalAveragePoolingLayer  # noqa: F401
from ..layers.residual_block import ResidualBlock  # noqa: F401
from .._hip import async_weight_grads
from .._tensor import as_device


class FeedForwardNetwork:
    def __init__(self, name):
        self.name = name
        self.is_on_gpu = False
        self.layers = []
        self.loss_layer = None
        self._steps = None

    def __repr__(self):
        out = "{}: \n".format(self.name)
        for l in self.layers:
            out += "\t" + l.__repr__() + "\n"
        return out

    def add_layer(self, layer):
        self.layers.append(layer)

    def set_loss_layer(self, loss_layer):
        self.loss_layer = loss_layer

    def to_gpu(self):
        if self.is_on_gpu:
            print("Model already on GPU, ignoring request")
            return
        layer = None
        try:
            for layer in self.layers:
                layer.to_gpu()
            if self.loss_layer is not None:
                self.loss_layer.is_on_gpu = True
            self.is_on_gpu = True
        except Exception as e:
            print("Error putting layer {} on GPU, error was: {}".format(layer, e))
            raise e

    def _l2_plan(self):
        """If every regularisation term the forward pass would add is a plain l2 on a
        layer's weights, return the (weights, strength) list (in the order
        feed_forward_network.py:55-60 and residual_block.py:78-84 visit them) so all terms
        are computed in one multi-tensor launch; None otherwise (per-layer fallback)."""
        from ..layers.layer import Layer
        from ..layers.residual_block import ResidualBlock
        from ..layers._common import l2_strength
        plan = []

        def visit(layer):
            rf = type(layer).regulariser_forward
            if rf is ResidualBlock.regulariser_forward:
                for l in layer.layer_list:
                    if hasattr(l, "regulariser_forward") and not visit(l):
                        return False
                return True
            if rf is not Layer.regulariser_forward:
                return False
            reg = layer.weight_regulariser
            if not reg:
                return True
            s = l2_strength(reg)
            w = layer.learned_params["weights"] if layer.learned_params else None
            if s is None or not (hasattr(w, "is_cuda") and w.is_cuda and w.is_contiguous()):
                return False
            plan.append((w, s))
            return True

        for layer in self.layers:
            if hasattr(layer, "regulariser_forward") and not visit(layer):
                return None
        return plan

    def _l2_total(self, plan, loss_tensor):
        """loss_tensor + sum of 0.5*s*sum(W^2) over `plan` (dk_l2_loss_multi_f32)."""
        import torch
        from .._hip import lib, stream_handle, workspace
        sig = tuple((w.data_ptr(), w.numel(), s) for w, s in plan)
        if getattr(self, "_l2_sig", None) != sig:
            rows, block0 = [], 0
            for w, s in plan:
                f = np.array([s, 0.0], dtype=np.float32).view(np.int64)[0]
                rows.append((w.data_ptr(), w.numel(), block0, int(f)))
                block0 += -(-w.numel() // 2048)
            self._l2_table = torch.as_tensor(np.array(rows, dtype=np.int64).reshape(-1, 4), device="cuda")
            self._l2_blocks = block0
            self._l2_sig = sig
        out = torch.empty((), dtype=torch.float32, device=loss_tensor.device)
        nb = lib.dk_l2_multi_workspace_bytes(self._l2_blocks)
        lib.dk_l2_loss_multi_f32(self._l2_table.data_ptr(), len(plan), self._l2_blocks, loss_tensor.data_ptr(),
                                 out.data_ptr(), workspace.get(nb), nb, stream_handle())
        return out

    def forward(self, X, y_one_hot, test_mode=False, terminal_layer_name=None):
        loss = 0
        regularisation_terms = []
        steps = []
        self._steps = steps
        plan = None
        if not test_mode and self.loss_layer is not None and terminal_layer_name is None:
            plan = self._l2_plan()
            if plan is not None and not plan:
                plan = None
        keep = () if terminal_layer_name is None else (terminal_layer_name,)

        def visit(group, X):
            for l in group:
                if l.layer_name == terminal_layer_name:
                    return True
                if not test_mode and plan is None and hasattr(l, "regulariser_forward"):
                    regularisation_terms.append(l.regulariser_forward())
            return False

        X, steps, stopped = execute(self.layers, X, test_mode, keep=keep, visit=visit)
        self._steps = steps
        if stopped:
            return loss, materialize(X)
        if self.loss_layer is not None:
            this_loss, X = self.loss_layer.forward(X, y_one_hot, test_mode=test_mode)
            if plan is not None:
                return self._l2_total(plan, this_loss), X
            loss += this_loss
            loss += sum(regularisation_terms)
        return loss, X  # NB if test_mode=True, you get softmax scores ("logits")

    def backward(self, upstream_dx=None, input_grad=False):
        """Reference behaviour (feed_forward_network.py:62-70): backward from the loss layer.
        Extension: an explicit output gradient for a network without a loss layer (BASELINE
        config 5's stack is driven this way).  Like the reference this returns nothing, so the
        gradient w.r.t. the network input (which the reference computes and drops) is not
        computed; input_grad=True computes and returns it."""
        if upstream_dx is not None:
            pass
        elif self.loss_layer is not None:
            upstream_dx = self.loss_layer.backward()
        else:
            raise ValueError("Network doesn't have a loss, can't run backward pass.")
        with async_weight_grads():  # weight gradients on the side stream, joined on exit
            dx = chain_backward(self._steps, upstream_dx, need_input_grad=input_grad)
        return dx if input_grad else None

    def test(self, data_loader, batch_size, test_set_size):
        from tqdm import tqdm
        test_correct_total = 0
        for X_test_batch, y_test_batch, _ in tqdm(data_loader, total=test_set_size / batch_size):
            X_test_batch = as_device(X_test_batch)
            _, batch_scores = self.forward(X_test_batch, y_one_hot=None, test_mode=True)
            test_correct_total += np.sum(np.asarray(y_test_batch) ==
                                         np.argmax(batch_scores.cpu().numpy(), axis=1))
        return float(test_correct_total) / test_set_size

    def save_weights_to_h5(self, fname):
        from .checkpoint import open_h5
        with open_h5(fname, "w") as f:
            for layer in self.layers:
                layer.save_to_h5(f)
            if self.loss_layer is not None:
                self.loss_layer.save_to_h5(f)

    def save_layer_structure_to_json(self, fname):
        structure_dict = {"name": self.name}
        for layer in self.layers:
            structure_dict[layer.layer_name] = repr(layer)
        if self.loss_layer is not None:
            structure_dict[self.loss_layer.layer_name] = repr(self.loss_layer)
        with open(fname, "w") as f:
            json.dump(structure_dict, f, indent=4)

    def load_network_from_json_and_h5(self, json_fname, h5_fname):
        from .checkpoint import load_network
        load_network(self, json_fname, h5_fname)
