"""Sequential execution of a layer list with BN+ReLU fusion.

Used by FeedForwardNetwork (network/feed_forward_network.py:47-70 in the reference) and
ResidualBlock (layers/residual_block.py:65-97).  Each layer keeps its own
forward/backward; the executor only decides to run a (BatchNormLayer, ReLu) pair as one
fused pass, records the steps it took, and replays them in reverse for backward.
Set DORKNET_FUSE=0 to run every layer on its own (used by the per-layer parity tests).
"""
from __future__ import annotations

import os


def fusion_enabled() -> bool:
    return os.environ.get("DORKNET_FUSE", "1") != "0"


def fusable_pair(layer, nxt) -> bool:
    from .activations import ReLu
    from .batch_norm import BatchNormLayer
    return type(layer) is BatchNormLayer and type(nxt) is ReLu


def chain_forward(layers, X, test_mode=False):
    """Run `layers` in order; returns (output, steps)."""
    steps = []
    fuse = fusion_enabled()
    i = 0
    while i < len(layers):
        layer = layers[i]
        nxt = layers[i + 1] if i + 1 < len(layers) else None
        if fuse and nxt is not None and fusable_pair(layer, nxt):
            X = layer.forward_bn_relu(X, nxt, test_mode=test_mode)
            steps.append((layer, nxt))
            i += 2
        else:
            X = layer.forward(X, test_mode=test_mode)
            steps.append((layer,))
            i += 1
    return X, steps


def chain_backward(steps, dy):
    for step in reversed(steps):
        if len(step) == 2:
            dy = step[0].backward_bn_relu(dy, step[1])
        else:
            dy = step[0].backward(dy)
    return dy
