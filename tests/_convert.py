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


# Slack over the reference-faithful fp32 pipeline's own error (the restated reference in fp32 vs
# the fp64 oracle): a GPU result may be at most FP32_SLACK times as far from the fp64 oracle as
# that pipeline is.  Measured at full size the GPU is within ~2x of it
# (profiles/r02_fullsize_conditioning.txt), so 3x still catches a kernel whose error doubles.
FP32_SLACK = 3.0


def slack_bound(want64, want32, tol):
    """max(tol * ||want64||, FP32_SLACK * ||want32 - want64||)."""
    want64 = np.asarray(want64, dtype=np.float64)
    return max(tol * np.linalg.norm(want64.ravel()),
               FP32_SLACK * np.linalg.norm((np.asarray(want32, dtype=np.float64) - want64).ravel()))


def log_slack(name, err, want64, want32):
    """With DORKNET_SLACK_LOG=<file>: append err / ||want32 - want64|| (the ratio FP32_SLACK
    bounds) so a GPU run leaves the measured ratios behind."""
    import os
    path = os.environ.get("DORKNET_SLACK_LOG")
    if not path or want32 is None:
        return
    ref = np.linalg.norm((np.asarray(want32, np.float64) - np.asarray(want64, np.float64)).ravel())
    rel = np.linalg.norm(np.asarray(want64, np.float64).ravel())
    with open(path, "a") as f:
        f.write("{}\t{:.3e}\t{:.3e}\t{}\n".format(name, err / max(rel, 1e-300), ref / max(rel, 1e-300),
                                                  "inf" if ref == 0 else "{:.3f}".format(err / ref)))

