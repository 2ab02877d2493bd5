"""The Layer protocol -- the drop-in boundary (reference: layers/layer.py:3-46).

Same attributes and methods as the reference: ``layer_name``, ``is_on_gpu``,
``learned_params`` / ``non_learned_params`` / ``grads`` dicts, ``weight_regulariser``,
``to_gpu()``, ``forward(X, test_mode=False)``, ``backward(upstream_dx)``,
``regulariser_forward()``.  ``to_gpu()`` moves the numpy parameters onto the MI355X as
fp32 torch tensors (the reference uses cp.asarray); compute only runs on the GPU.
"""
from __future__ import annotations

from .._hip import require_gpu
from .._tensor import to_param


class Layer:

    def __init__(self, layer_name, *args, **kwargs):
        self.layer_name = layer_name
        self.is_on_gpu = False
        self.learned_params = None
        self.non_learned_params = None
        self.grads = None
        self.weight_regulariser = None
        self._bn_in = None  # BNOut consumed by forward (layers/_bn_input.py), if any

    def __repr__(self):
        return "Layer of type {} didn't implement __repr__".format(self.__class__.__name__)

    def to_gpu(self):
        if self.is_on_gpu:
            print("Layer {} is already on GPU, ignoring request".format(self.layer_name))
            return
        require_gpu()
        for d in (self.learned_params, self.non_learned_params, self.grads):
            if d is None:
                continue
            for k, v in d.items():
                if v is not None:
                    d[k] = to_param(v)
        self.is_on_gpu = True

    def _bn_tensors(self):
        """Device tensors of the BNOut this layer's forward consumed (kept alive for work on
        the weight-gradient side stream)."""
        b = self._bn_in
        return () if b is None else (b.x, b.mean, b.invstd, b.gamma, b.beta)

    def _require_on_gpu(self):
        if not self.is_on_gpu:
            raise RuntimeError(
                "{}({}): dorknet_amd computes on the MI355X only; call to_gpu() (or "
                "network.to_gpu()) before forward/backward".format(type(self).__name__, self.layer_name))

    def forward(self, X, *args, test_mode=False, **kwargs):
        pass

    def backward(self, upstream_dx, *args, **kwargs):
        pass

    def regulariser_forward(self):
        out = 0
        if self.weight_regulariser:
            out += self.weight_regulariser.forward(self.learned_params["weights"])
        return out
