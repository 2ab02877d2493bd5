"""dorknet_amd -- Dorknet's convolution training hot path, MI355X-native.

Drop-in for the reference's `layers`, `network`, `optimisers` and `regularisers`
packages (WJGiles/Dorknet): same classes, signatures and semantics, with all compute in
hand-written HIP kernels for gfx950 (libdorknet_hip.so, C ABI in include/dorknet_hip.h).

    import dorknet_amd
    dorknet_amd.install_reference_aliases()   # `from layers.convolution import ConvLayer` now works
"""
from __future__ import annotations

import importlib
import sys

__version__ = "0.1.0"

_ALIASES = [
    "layers", "layers.layer", "layers.convolution", "layers.depthwise_convolution",
    "layers.pointwise_convolution", "layers.dense_layer", "layers.batch_norm", "layers.activations",
    "layers.residual_block", "layers.pooling", "layers.losses",
    "network", "network.feed_forward_network",
    "optimisers", "optimisers.SGDMomentum",
    "regularisers", "regularisers.l2",
]


def install_reference_aliases() -> None:
    """Register this package's modules under the reference's top-level module names so
    reference model code (e.g. examples/imagenet_dogs_225_resnet_18_depsep.py:1-18)
    imports unchanged.  Module objects are shared, so classes keep one identity."""
    for name in _ALIASES:
        mod = importlib.import_module(__name__ + "." + name)
        sys.modules.setdefault(name, mod)
