"""Sequential execution of a layer list with BatchNorm fusion.

Used by FeedForwardNetwork (network/feed_forward_network.py:47-70 in the reference) and
ResidualBlock (layers/residual_block.py:65-97).  Each layer keeps its own
forward/backward; the executor only decides how a BatchNormLayer (optionally followed by a
ReLu) runs, records the groups it ran, and replays them in reverse for backward:

  * "defer"  -- the next layer applies the normalisation (+ReLU) on load
                (``accepts_bn_input``; layers/_bn_input.py), so the BN output is never
                written: BatchNormLayer.forward_deferred hands over a BNOut;
  * "pair"   -- BN + ReLU in one apply pass (BatchNormLayer.forward_bn_relu);
  * "single" -- the layer on its own.

Backward is the same for all three: BatchNormLayer.backward[_bn_relu] recomputes what it
needs from the BN's raw input.  Set DORKNET_FUSE=0 to run every layer on its own (used by
the per-layer parity tests; results are bit-identical either way).
"""
from __future__ import annotations

import os

from ._bn_input import accepts_bn_input


def fusion_enabled() -> bool:
    return os.environ.get("DORKNET_FUSE", "1") != "0"


def fusable_pair(layer, nxt) -> bool:
    from .activations import ReLu
    from .batch_norm import BatchNormLayer
    return type(layer) is BatchNormLayer and type(nxt) is ReLu


def plan_group(layers, i, fuse, out_accepts=False, keep=()):
    """How to run layers[i:]: returns (group, mode).  `out_accepts`: whether whatever consumes
    the end of the list takes a BNOut; `keep`: layer names whose output must be materialised
    (e.g. a terminal layer)."""
    from .activations import ReLu
    from .batch_norm import BatchNormLayer
    layer = layers[i]
    if fuse and type(layer) is BatchNormLayer:
        relu = layers[i + 1] if i + 1 < len(layers) and type(layers[i + 1]) is ReLu else None
        group = (layer, relu) if relu is not None else (layer,)
        j = i + len(group)
        consumer_ok = accepts_bn_input(layers[j]) if j < len(layers) else out_accepts
        if consumer_ok and not any(l.layer_name in keep for l in group):
            return group, "defer"
        if relu is not None:
            return group, "pair"
    return (layer,), "single"


def run_group(group, mode, X, test_mode=False):
    if mode == "defer":
        return group[0].forward_deferred(X, group[1] if len(group) == 2 else None, test_mode=test_mode)
    if mode == "pair":
        return group[0].forward_bn_relu(X, group[1], test_mode=test_mode)
    return group[0].forward(X, test_mode=test_mode)


def chain_forward(layers, X, test_mode=False, out_accepts=False):
    """Run `layers` in order; returns (output, steps).  The output is a BNOut when the list
    ends in a BatchNormLayer [+ ReLu] and `out_accepts`."""
    steps = []
    fuse = fusion_enabled()
    i = 0
    while i < len(layers):
        group, mode = plan_group(layers, i, fuse, out_accepts)
        X = run_group(group, mode, X, test_mode)
        steps.append(group)
        i += len(group)
    return X, steps


def chain_backward(steps, dy):
    for step in reversed(steps):
        if len(step) == 2:
            dy = step[0].backward_bn_relu(dy, step[1])
        else:
            dy = step[0].backward(dy)
    return dy
