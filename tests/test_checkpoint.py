"""h5 checkpoints: the reference's file layout, written and read back.

The reference writes and reads these files with h5py (network/feed_forward_network.py:90-139
and the per-layer save_to_h5 / load_from_h5).  h5py is absent here; dorknet_amd goes through
the HDF5 C library (dorknet_amd/network/_h5lite.py).  These tests check the layout and the
attribute types h5py would produce for the reference's values, and a full ResNet-18-depsep
save -> load round trip.  The reference publishes no checkpoint files, so the format is pinned
by the reference's save/load code and by h5dump (when the image has it), not by a file the
reference wrote.
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from dorknet_amd.network import checkpoint

pytest.importorskip("numpy")

try:
    checkpoint._backend().File  # noqa: B018
    from dorknet_amd.network import _h5lite
    if checkpoint._backend() is _h5lite:
        _h5lite._load()
    HAVE_H5 = True
except ImportError:  # pragma: no cover - environment dependent
    HAVE_H5 = False

pytestmark = pytest.mark.skipif(not HAVE_H5, reason="neither h5py nor the HDF5 C library is available")


def _resnet():
    from examples.resnet18_depsep import ResNet18
    np.random.seed(3)
    net = ResNet18("DogsImageNet225ResNet18DepSep")
    rng = np.random.RandomState(4)
    for layer in _all_layers(net.layers):
        for d in (layer.learned_params, layer.grads):
            for k, v in (d or {}).items():
                d[k] = rng.standard_normal(np.shape(v)).astype(np.float32)
        if type(layer).__name__ == "BatchNormLayer":
            shp = layer._param_shape(layer.incoming_chans)
            layer.non_learned_params["running_mean"] = rng.standard_normal(shp).astype(np.float32)
            layer.non_learned_params["running_std"] = rng.rand(*shp).astype(np.float32) + 0.5
    return net


def _all_layers(layers):
    out = []
    for l in layers:
        out.append(l)
        if type(l).__name__ == "ResidualBlock":
            out += _all_layers(l.layer_list)
            if l.skip_projection is not None:
                out.append(l.skip_projection)
            out.append(l.post_skip_activation)
    return out


def _state(net):
    st = {}
    for l in _all_layers(net.layers):
        for dname in ("learned_params", "grads", "non_learned_params"):
            for k, v in (getattr(l, dname) or {}).items():
                st[(l.layer_name, dname, k)] = np.asarray(v)
    return st


def test_resnet_roundtrip(tmp_path):
    from dorknet_amd.network.feed_forward_network import FeedForwardNetwork
    from dorknet_amd.layers.losses import SoftmaxWithCrossEntropy
    net = _resnet()
    h5f, js = str(tmp_path / "w.h5"), str(tmp_path / "s.json")
    net.save_weights_to_h5(h5f)
    net.save_layer_structure_to_json(js)
    with open(js) as f:
        names = [k for k in json.load(f) if k != "name"]
    assert names == [l.layer_name for l in net.layers] + [net.loss_layer.layer_name]

    fresh = FeedForwardNetwork("x")
    fresh.load_network_from_json_and_h5(js, h5f)
    assert fresh.name == net.name
    assert isinstance(fresh.loss_layer, SoftmaxWithCrossEntropy)
    assert [type(l).__name__ for l in _all_layers(fresh.layers)] == [type(l).__name__ for l in _all_layers(net.layers)]
    a, b = _state(net), _state(fresh)
    assert a.keys() == b.keys()
    for k in a:
        assert a[k].shape == b[k].shape, k
        np.testing.assert_array_equal(a[k], b[k], err_msg=str(k))
    # constructor fields and regularisers come back
    for la, lb in zip(_all_layers(net.layers), _all_layers(fresh.layers)):
        for f in ("stride", "padding", "with_bias", "num_filters", "filter_chans", "f_rows", "f_cols", "num_channels",
                  "incoming_chans", "output_dim", "run_momentum", "eps", "input_dimension"):
            if hasattr(la, f) and getattr(la, f) is not None:
                assert getattr(la, f) == getattr(lb, f), (la.layer_name, f)
        ra, rb = getattr(la, "weight_regulariser", None), getattr(lb, "weight_regulariser", None)
        assert (ra is None) == (rb is None), la.layer_name
        if ra is not None:
            assert ra.type == rb.type and float(ra.strength) == float(rb.strength)
    assert repr(fresh.layers[0]) == repr(net.layers[0])


def test_layout_and_attribute_types(tmp_path):
    """The objects and attribute types the reference's save_to_h5 produces through h5py."""
    net = _resnet()
    h5f = str(tmp_path / "w.h5")
    net.save_weights_to_h5(h5f)
    with checkpoint.open_h5(h5f, "r") as f:
        info = f["conv0/layer_info"]
        assert info.shape is None  # create_dataset(name, dtype=np.float32): an empty dataset
        a = info.attrs
        assert a["type"] == "ConvLayer" and isinstance(a["type"], str)
        assert isinstance(a["with_bias"], np.bool_) and not a["with_bias"]
        for k in ("num_filters", "filter_chans", "f_rows", "f_cols", "stride", "padding"):
            assert isinstance(a[k], np.int64), k
        assert (a["num_filters"], a["filter_chans"], a["f_rows"], a["stride"], a["padding"]) == (64, 3, 5, 2, 1)
        w = f["conv0/weights"]
        assert w.dtype == np.float32 and w.shape == (64, 3, 5, 5)
        assert w.attrs["weight_regulariser_type"] == b"l2"  # np.string_ -> fixed-length bytes
        assert float(w.attrs["weight_regulariser_strength"]) == pytest.approx(1e-4)
        assert "conv0/grads/weights" in f and "conv0/bias" not in f
        bn = f["conv0_bn/layer_info"].attrs
        assert isinstance(bn["run_momentum"], np.float64) and bn["run_momentum"] == 0.95
        assert isinstance(bn["eps"], np.float64) and bn["input_dimension"] == 4
        assert f["conv0_bn/running_std"].shape == (1, 64, 1, 1)
        res = f["res3/layer_info"].attrs
        assert list(res["layer_type_list"])[:3] == ["DepthwiseConvLayer", "BatchNormLayer", "PointwiseConvLayer"]
        assert res["skip_projection_type"] == "PointwiseConvLayer"
        assert res["post_skip_activation_type"] == "ReLu"
        assert "res1/layer_info" in f and "skip_projection_type" not in f["res1/layer_info"].attrs
        assert f[net.loss_layer.layer_name + "/layer_info"].attrs["type"] == "SoftmaxWithCrossEntropy"
        assert sorted(f.keys()) == sorted(l.layer_name for l in _all_layers(net.layers) + [net.loss_layer])


@pytest.mark.skipif(shutil.which("h5dump") is None and not os.path.exists("/opt/conda/bin/h5dump"),
                    reason="h5dump not available")
def test_h5dump_reads_file(tmp_path):
    """HDF5's own dump tool parses the file and sees the h5py types."""
    net = _resnet()
    h5f = str(tmp_path / "w.h5")
    net.save_weights_to_h5(h5f)
    tool = shutil.which("h5dump") or "/opt/conda/bin/h5dump"
    out = subprocess.run([tool, "-A", "-g", "/conv0", h5f], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                         text=True, timeout=60).stdout
    assert 'DATASET "layer_info"' in out and "DATASPACE  NULL" in out
    assert '"FALSE"' in out and "H5T_STD_I64LE" in out and "STRSIZE H5T_VARIABLE" in out
    assert "STRSIZE 2;" in out  # b"l2", fixed length


def test_load_without_grads_and_missing_stats(tmp_path):
    from dorknet_amd.layers.batch_norm import BatchNormLayer
    from dorknet_amd.layers.pointwise_convolution import PointwiseConvLayer
    from dorknet_amd.regularisers.l2 import l2
    np.random.seed(0)
    pw = PointwiseConvLayer("pw", stride=2, filter_block_shape=(8, 4), with_bias=True, weight_regulariser=l2(0.5))
    h5f = str(tmp_path / "p.h5")
    with checkpoint.open_h5(h5f, "w") as f:
        pw.save_to_h5(f, save_grads=False)
    with checkpoint.open_h5(h5f, "r") as f:
        assert "pw/grads" not in f
        q = PointwiseConvLayer("pw")
        q.load_from_h5(f, load_grads=False)
    assert (q.stride, q.num_filters, q.num_channels, q.with_bias) == (2, 8, 4, True)
    np.testing.assert_array_equal(q.learned_params["weights"], pw.learned_params["weights"])
    np.testing.assert_array_equal(q.grads["bias"], np.zeros(8, np.float32))
    assert q.weight_regulariser.strength == 0.5
    bn = BatchNormLayer("bn", incoming_chans=4)
    with checkpoint.open_h5(str(tmp_path / "b.h5"), "w") as f:
        with pytest.raises(ValueError):
            bn.save_to_h5(f)
