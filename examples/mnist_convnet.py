"""MNISTNet (reference: examples/MNIST_basic_convnet.py:15-69) on dorknet_amd -- BASELINE
config 1's model.  Five 3x3 / 4x4-stride-2 convolutions with BN + ReLU, GAP, dense 128->10.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dorknet_amd.layers.activations import ReLu  # noqa: E402
from dorknet_amd.layers.batch_norm import BatchNormLayer  # noqa: E402
from dorknet_amd.layers.convolution import ConvLayer  # noqa: E402
from dorknet_amd.layers.dense_layer import DenseLayer  # noqa: E402
from dorknet_amd.layers.losses import SoftmaxWithCrossEntropy  # noqa: E402
from dorknet_amd.layers.pooling import GlobalAveragePoolingLayer  # noqa: E402
from dorknet_amd.network.feed_forward_network import FeedForwardNetwork  # noqa: E402
from dorknet_amd.regularisers.l2 import l2  # noqa: E402

# (filter block, stride); relu names follow the reference (the fifth reuses "relu_4", :60)
CONVS = [((32, 1, 3, 3), 1), ((32, 32, 3, 3), 1), ((64, 32, 4, 4), 2), ((64, 64, 3, 3), 1), ((128, 64, 4, 4), 2)]


class MNISTNet(FeedForwardNetwork):
    def __init__(self, name, load_layers=True):
        super().__init__(name)
        if not load_layers:
            return
        for i, (shape, stride) in enumerate(CONVS, start=1):
            self.add_layer(ConvLayer("conv_%d" % i, filter_block_shape=shape, with_bias=False, stride=stride,
                                     weight_regulariser=l2(0.0001)))
            self.add_layer(BatchNormLayer("bn_%d" % i, incoming_chans=shape[0]))
            self.add_layer(ReLu("relu_%d" % min(i, 4)))
        self.add_layer(GlobalAveragePoolingLayer("global_pool"))
        self.add_layer(DenseLayer("dense_1", incoming_chans=128, output_dim=10, weight_regulariser=l2(0.0005)))
        self.set_loss_layer(SoftmaxWithCrossEntropy("softmax"))
