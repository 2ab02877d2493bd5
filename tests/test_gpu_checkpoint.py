"""h5 checkpoint round trip through the GPU: train one step on the
MI355X, save, load into a fresh host network, move it to the GPU; its test-mode outputs are
bit-identical to the trained network's, and loading into a network already on the GPU
overwrites its device tensors in place."""
import numpy as np
import pytest
import torch

from dorknet_amd.network import checkpoint

pytestmark = pytest.mark.gpu


def _have_h5():
    try:
        b = checkpoint._backend()
        if b.__name__.endswith("_h5lite"):
            b._load()
        return True
    except ImportError:
        return False


@pytest.mark.skipif(not _have_h5(), reason="neither h5py nor the HDF5 C library is available")
def test_train_save_load_infer(tmp_path):
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    from dorknet_amd._tensor import as_device
    from dorknet_amd.network.feed_forward_network import FeedForwardNetwork
    from dorknet_amd.optimisers.SGDMomentum import SGDMomentum
    np.random.seed(0)
    net = ResNet18("r")
    net.to_gpu()
    sgd = SGDMomentum(net, 0.01, 0.9)
    X, _, onehot = synthetic_batch(8, seed=5, size=97)
    X, onehot = as_device(X), as_device(onehot)
    net.forward(X, onehot)
    net.backward()
    sgd.update_weights()
    _, p_ref = net.forward(X, None, test_mode=True)
    p_ref = p_ref.clone()

    h5f, js = str(tmp_path / "w.h5"), str(tmp_path / "s.json")
    net.save_weights_to_h5(h5f)
    net.save_layer_structure_to_json(js)
    fresh = FeedForwardNetwork("x")
    fresh.load_network_from_json_and_h5(js, h5f)
    fresh.to_gpu()
    _, p = fresh.forward(X, None, test_mode=True)
    torch.cuda.synchronize()
    assert torch.equal(p, p_ref)

    # in-place load into a network already on the GPU (tensor objects are kept)
    np.random.seed(1)
    other = ResNet18("r")
    other.to_gpu()
    w0 = other.layers[0].learned_params["weights"]
    with checkpoint.open_h5(h5f, "r") as f:
        for layer in other.layers:
            layer.load_from_h5(f)
    assert other.layers[0].learned_params["weights"] is w0
    _, p2 = other.forward(X, None, test_mode=True)
    torch.cuda.synchronize()
    assert torch.equal(p2, p_ref)
