"""ResNet-18 with depthwise-separable blocks for the 120 ImageNet dog classes at 225x225
-- the model of BASELINE configs 3-4 (reference: examples/imagenet_dogs_225_resnet_18_depsep.py
:32-160), built on dorknet_amd.  Same layers, names, order, shapes, strides, paddings,
biases, regularisers and initialisation order as the reference class, so a fixed
``np.random.seed`` gives the reference's initial weights.

    python examples/resnet18_depsep.py --steps 5        # synthetic-data training loop
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dorknet_amd.layers.batch_norm import BatchNormLayer  # noqa: E402
from dorknet_amd.layers.activations import ReLu  # noqa: E402
from dorknet_amd.layers.convolution import ConvLayer  # noqa: E402
from dorknet_amd.layers.dense_layer import DenseLayer  # noqa: E402
from dorknet_amd.layers.depthwise_convolution import DepthwiseConvLayer  # noqa: E402
from dorknet_amd.layers.losses import SoftmaxWithCrossEntropy  # noqa: E402
from dorknet_amd.layers.pointwise_convolution import PointwiseConvLayer  # noqa: E402
from dorknet_amd.layers.pooling import GlobalAveragePoolingLayer  # noqa: E402
from dorknet_amd.layers.residual_block import ResidualBlock  # noqa: E402
from dorknet_amd.network.feed_forward_network import FeedForwardNetwork  # noqa: E402
from dorknet_amd.regularisers.l2 import l2  # noqa: E402

# (block name, (out, in, 3, 3), downsample) -- reference :124-150
BLOCKS = [("res1", (64, 64, 3, 3), False), ("res2", (64, 64, 3, 3), False),
          ("res3", (128, 64, 3, 3), True), ("res4", (128, 128, 3, 3), False),
          ("res5", (256, 128, 3, 3), True), ("res6", (256, 256, 3, 3), False),
          ("res7", (512, 256, 3, 3), True), ("res8", (512, 512, 3, 3), False)]


class ResNet18(FeedForwardNetwork):

    def depthwise_sep_layer(self, layer_name, incoming_chans, filter_block_shape, stride=1, padding=1,
                            with_bias=False, batch_norm_depthwise=True, relu_depthwise=False,
                            batch_norm_pointwise=True, depthwise_weight_regulariser=None,
                            pointwise_weight_regulariser=None, final_relu=True, add_layers=False):
        """dw(k x k, stride) -> [BN] -> [ReLU] -> pw(1x1) -> [BN] -> [ReLU]  (reference :34-70)"""
        out_chans, _, fr, fc = filter_block_shape
        seq = [DepthwiseConvLayer(layer_name + "_dw", filter_block_shape=(incoming_chans, fr, fc), stride=stride,
                                  padding=padding, with_bias=with_bias,
                                  weight_regulariser=depthwise_weight_regulariser)]
        if batch_norm_depthwise:
            seq.append(BatchNormLayer(layer_name + "_dw_bn", input_dimension=4, incoming_chans=incoming_chans))
        if relu_depthwise:
            seq.append(ReLu(layer_name + "dw_relu"))
        seq.append(PointwiseConvLayer(layer_name + "_pw", filter_block_shape=(out_chans, incoming_chans),
                                      with_bias=with_bias, weight_regulariser=pointwise_weight_regulariser))
        if batch_norm_pointwise:
            seq.append(BatchNormLayer(layer_name + "_pw_bn", input_dimension=4, incoming_chans=out_chans))
        if final_relu:
            seq.append(ReLu(layer_name + "pw_relu"))
        if not add_layers:
            return seq
        for layer in seq:
            self.add_layer(layer)

    def add_res_block(self, layer_name, first_filter_block_shape, downsample=False,
                      weight_regulariser_strength=0.0001, depthwise_sep=False):
        """Two (depthwise-separable or dense 3x3) units + skip + ReLU (reference :72-107)."""
        nf, inc, fr, fc = first_filter_block_shape
        s = weight_regulariser_strength
        stride = 2 if downsample else 1
        if depthwise_sep:
            chain = self.depthwise_sep_layer(layer_name + "_dw1", inc, first_filter_block_shape, stride=stride,
                                             padding=1, pointwise_weight_regulariser=l2(strength=s),
                                             final_relu=True)
            chain += self.depthwise_sep_layer(layer_name + "_dw2", nf, (nf, nf, fr, fc), stride=1, padding=1,
                                              pointwise_weight_regulariser=l2(strength=s), final_relu=False)
        else:
            chain = [ConvLayer(layer_name + "_conv1", filter_block_shape=first_filter_block_shape, stride=stride,
                               padding=1, with_bias=False, weight_regulariser=l2(strength=s)),
                     BatchNormLayer(layer_name + "_bn1", input_dimension=4, incoming_chans=nf),
                     ReLu(layer_name + "_relu1"),
                     ConvLayer(layer_name + "_conv2", filter_block_shape=(nf, nf, fr, fc), stride=1, padding=1,
                               with_bias=False, weight_regulariser=l2(strength=s)),
                     BatchNormLayer(layer_name + "_bn2", input_dimension=4, incoming_chans=nf)]
        skip = None
        if downsample:
            skip = PointwiseConvLayer(layer_name + "_pw_skip", filter_block_shape=(nf, inc), stride=2,
                                      with_bias=False, weight_regulariser=l2(strength=s))
        self.add_layer(ResidualBlock(layer_name, layer_list=chain, skip_projection=skip,
                                     post_skip_activation=ReLu(layer_name + "_relu2")))

    def __init__(self, name, load_layers=True, num_classes=120):
        super().__init__(name)
        if not load_layers:
            return
        # stem: 225 -> 112 (5x5/2 conv) -> 56 (1x1/2 pointwise)  (reference :112-122)
        self.add_layer(ConvLayer("conv0", filter_block_shape=(64, 3, 5, 5), with_bias=False, stride=2, padding=1,
                                 weight_regulariser=l2(0.0001)))
        self.add_layer(BatchNormLayer("conv0_bn", input_dimension=4, incoming_chans=64))
        self.add_layer(ReLu("conv0_relu"))
        self.add_layer(PointwiseConvLayer("pw0", filter_block_shape=(64, 64), with_bias=False, stride=2,
                                          weight_regulariser=l2(0.0001)))
        self.add_layer(BatchNormLayer("pw0_bn", input_dimension=4, incoming_chans=64))
        self.add_layer(ReLu("pw0_relu"))
        for name, shape, down in BLOCKS:
            self.add_res_block(name, shape, downsample=down, depthwise_sep=True)
        # head: 7x7 -> GAP -> dense -> softmax  (reference :152-160)
        self.add_layer(GlobalAveragePoolingLayer("global_pool1"))
        self.add_layer(DenseLayer("dense1", incoming_chans=512, output_dim=num_classes,
                                  weight_regulariser=l2(0.0001)))
        self.set_loss_layer(SoftmaxWithCrossEntropy("softmax1"))


def synthetic_batch(batch, num_classes=120, seed=0, size=225):
    """X ~ U[-128, 128) (the reference preprocessor's im - 128 range), one-hot labels."""
    import numpy as np
    rng = np.random.default_rng(seed)
    X = rng.uniform(-128, 128, size=(batch, 3, size, size)).astype(np.float32)
    y = rng.integers(0, num_classes, size=batch)
    onehot = np.zeros((batch, num_classes), dtype=np.float32)
    onehot[np.arange(batch), y] = 1.0
    return X, y, onehot


def main():
    import numpy as np
    import torch
    from dorknet_amd._tensor import as_device
    from dorknet_amd.optimisers.SGDMomentum import SGDMomentum
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=60)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    np.random.seed(0)
    net = ResNet18("DogsImageNet225ResNet18DepSep")
    net.to_gpu()
    sgd = SGDMomentum(net, 0.05 * (args.batch / 200.0), 0.9)
    X, y, onehot = synthetic_batch(args.batch)
    X, onehot = as_device(X), as_device(onehot)
    for i in range(args.steps):
        t0 = time.time()
        loss, scores = net.forward(X, onehot)
        net.backward()
        sgd.update_weights()
        torch.cuda.synchronize()
        print("step {} loss {:.5f} ({:.1f} ms)".format(i, float(loss), 1e3 * (time.time() - t0)))


if __name__ == "__main__":
    main()
