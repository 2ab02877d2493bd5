"""Mirror a dorknet_amd network (or layer) into an oracle network with identical weights."""
from __future__ import annotations

import numpy as np
import torch

from oracle import net as O


def _np(v, dtype):
    if isinstance(v, torch.Tensor):
        v = v.detach().cpu().numpy()
    return np.array(v, dtype=dtype)


def _l2(layer):
    r = getattr(layer, "weight_regulariser", None)
    return float(r.strength) if r is not None else 0.0


def layer_to_oracle(l, dtype=np.float64):
    from dorknet_amd.layers.activations import ReLu
    from dorknet_amd.layers.batch_norm import BatchNormLayer
    from dorknet_amd.layers.convolution import ConvLayer
    from dorknet_amd.layers.dense_layer import DenseLayer
    from dorknet_amd.layers.depthwise_convolution import DepthwiseConvLayer
    from dorknet_amd.layers.losses import SoftmaxWithCrossEntropy
    from dorknet_amd.layers.pointwise_convolution import PointwiseConvLayer
    from dorknet_amd.layers.pooling import GlobalAveragePoolingLayer
    from dorknet_amd.layers.residual_block import ResidualBlock
    lp = l.learned_params or {}
    W = _np(lp["weights"], dtype) if "weights" in lp else None
    b = _np(lp["bias"], dtype) if "bias" in lp else None
    if isinstance(l, ConvLayer):
        return O.OConv(l.layer_name, W, b, l.stride, l.padding, _l2(l))
    if isinstance(l, DepthwiseConvLayer):
        return O.ODepthwise(l.layer_name, W, b, l.stride, l.padding, _l2(l))
    if isinstance(l, PointwiseConvLayer):
        return O.OPointwise(l.layer_name, W, b, l.stride, _l2(l))
    if isinstance(l, DenseLayer):
        return O.ODense(l.layer_name, W, b, _l2(l))
    if isinstance(l, BatchNormLayer):
        bn = O.OBatchNorm(l.layer_name, _np(lp["gamma"], dtype), _np(lp["beta"], dtype), l.eps, l.run_momentum)
        nlp = l.non_learned_params
        if nlp["running_mean"] is not None:
            bn.non_learned_params = {k: _np(v, dtype) for k, v in nlp.items()}
        return bn
    if isinstance(l, ReLu):
        return O.OReLU(l.layer_name)
    if isinstance(l, GlobalAveragePoolingLayer):
        return O.OGAP(l.layer_name)
    if isinstance(l, SoftmaxWithCrossEntropy):
        return O.OSoftmaxXent(l.layer_name)
    if isinstance(l, ResidualBlock):
        return O.OResidual(l.layer_name, [layer_to_oracle(c, dtype) for c in l.layer_list],
                           layer_to_oracle(l.skip_projection, dtype) if l.skip_projection is not None else None,
                           layer_to_oracle(l.post_skip_activation, dtype))
    raise TypeError(type(l))


def network_to_oracle(net, dtype=np.float64):
    return O.ONetwork([layer_to_oracle(l, dtype) for l in net.layers], layer_to_oracle(net.loss_layer, dtype))


def all_layers(layers):
    out = []
    for l in layers:
        out.append(l)
        if hasattr(l, "layer_list"):
            out += all_layers(l.layer_list)
            if getattr(l, "skip_projection", None) is not None:
                out.append(l.skip_projection)
    return out


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.linalg.norm(b.ravel())
    num = np.linalg.norm((a - b).ravel())
    return num / den if den > 0 else num
