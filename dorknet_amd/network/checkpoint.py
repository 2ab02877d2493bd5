"""h5 checkpoints in the reference's file layout (SURVEY.md section 8 f, row 3).

Reference: each layer's ``save_to_h5`` / ``load_from_h5`` (layers/convolution.py:226-281,
layers/depthwise_convolution.py:300-353, layers/pointwise_convolution.py:77-130,
layers/dense_layer.py:69-117, layers/batch_norm.py:176-232, layers/activations.py:49-55,
layers/pooling.py:38-44, layers/losses.py:36-42, layers/residual_block.py:99-151) and
``FeedForwardNetwork.save_weights_to_h5`` / ``load_network_from_json_and_h5``
(network/feed_forward_network.py:90-139).

Layout (one HDF5 file per network, every layer's objects under its ``layer_name``):

- ``<name>/layer_info``: an empty float32 dataset whose attributes describe the layer
  (``type`` = class name, plus the constructor's shape / stride / padding / bias fields);
- ``<name>/weights`` and ``<name>/bias`` (conv, depthwise, pointwise, dense), or
  ``<name>/gamma``, ``<name>/beta``, ``<name>/running_mean``, ``<name>/running_std`` (BN);
- ``<name>/grads/<param>`` when ``save_grads`` (the default);
- an l2 regulariser is recorded on the weights dataset as the fixed-length byte strings
  ``weight_regulariser_type = b"l2"`` and ``weight_regulariser_strength = b"<strength>"``
  (``np.string_`` in the reference) and restored only for type ``b"l2"``;
- a residual block stores ``layer_type_list`` / ``layer_name_list`` (string arrays) and the
  post-skip activation / skip projection type and name; its sub-layers are saved as
  top-level entries under their own names.

Files go through h5py when it is importable and otherwise through ``_h5lite`` (the same
subset over the HDF5 C library), which writes the objects h5py writes.  Parameters on the
GPU are copied to the host on save; a layer that is already on the GPU when loaded gets its
device tensors overwritten in place (the optimiser keeps references to them), a layer on the
host gets numpy arrays, as the reference's loader produces (call ``to_gpu()`` afterwards).
"""
from __future__ import annotations

import json

import numpy as np


def _backend():
    try:
        import h5py
        return h5py
    except ImportError:
        from . import _h5lite
        return _h5lite


def open_h5(fname, mode):
    return _backend().File(fname, mode)


# -- value helpers ------------------------------------------------------------------------

def _host(v):
    """numpy copy of a parameter (torch device tensor or numpy array)."""
    if v is None:
        return None
    if hasattr(v, "detach"):
        return v.detach().float().cpu().numpy()
    return np.asarray(v)


def _put(layer, store, key, value):
    """Set store[key] = value (numpy) -- in place on the device for a layer on the GPU."""
    value = np.asarray(value, dtype=np.float32)
    cur = store.get(key) if store is not None else None
    if getattr(layer, "is_on_gpu", False):
        import torch
        from .._tensor import to_param
        if isinstance(cur, torch.Tensor) and tuple(cur.shape) == value.shape:
            cur.copy_(torch.from_numpy(np.ascontiguousarray(value)))
        else:
            store[key] = to_param(value)
    else:
        store[key] = value


def _write(open_f, path, value):
    a = _host(value)
    d = open_f.create_dataset(path, a.shape, dtype=a.dtype)
    d[:] = a
    return d


def _info(open_f, layer):
    d = open_f.create_dataset(layer.layer_name + "/layer_info", dtype=np.float32)
    d.attrs["type"] = layer.__class__.__name__
    return d


def _attrs(open_f, layer):
    return open_f[layer.layer_name + "/layer_info"].attrs


def _as_str(v):
    return v.decode() if isinstance(v, (bytes, np.bytes_)) else str(v)


def _save_regulariser(dset, layer):
    reg = layer.weight_regulariser
    if reg is not None:
        dset.attrs["weight_regulariser_type"] = np.bytes_(str(reg.type).encode())
        dset.attrs["weight_regulariser_strength"] = np.bytes_(str(reg.strength).encode())


def _load_regulariser(open_f, layer):
    attrs = open_f[layer.layer_name + "/weights"].attrs
    t = attrs.get("weight_regulariser_type", None)
    if t is not None and _as_str(t) == "l2":
        from ..regularisers.l2 import l2
        layer.weight_regulariser = l2(strength=float(_as_str(attrs["weight_regulariser_strength"])))


def _save_params(open_f, layer, keys, save_grads, store="learned_params"):
    for k in keys:
        _write(open_f, layer.layer_name + "/" + k, getattr(layer, store)[k])
    if save_grads:
        for k in keys:
            _write(open_f, layer.layer_name + "/grads/" + k, layer.grads[k])


def _load_params(open_f, layer, keys, load_grads):
    if layer.learned_params is None:
        layer.learned_params = {}
    if layer.grads is None:
        layer.grads = {}
    for k in keys:
        _put(layer, layer.learned_params, k, open_f[layer.layer_name + "/" + k][:])
    for k in keys:
        path = layer.layer_name + "/grads/" + k
        if load_grads:
            _put(layer, layer.grads, k, open_f[path][:])
        elif k not in layer.grads or layer.grads[k] is None:
            _put(layer, layer.grads, k, np.zeros_like(open_f[layer.layer_name + "/" + k][:]))


# -- per layer type -----------------------------------------------------------------------

def _save_conv(layer, open_f, save_grads):
    d = _info(open_f, layer)
    d.attrs["with_bias"] = bool(layer.with_bias)
    for k in ("num_filters", "filter_chans", "f_rows", "f_cols", "stride", "padding"):
        d.attrs[k] = int(getattr(layer, k))
    w = _write(open_f, layer.layer_name + "/weights", layer.learned_params["weights"])
    _save_regulariser(w, layer)
    keys = ["weights"] + (["bias"] if layer.with_bias else [])
    if layer.with_bias:
        _write(open_f, layer.layer_name + "/bias", layer.learned_params["bias"])
    if save_grads:
        for k in keys:
            _write(open_f, layer.layer_name + "/grads/" + k, layer.grads[k])


def _load_conv(layer, open_f, load_grads):
    a = _attrs(open_f, layer)
    for k in ("num_filters", "filter_chans", "f_rows", "f_cols", "stride", "padding"):
        setattr(layer, k, int(a[k]))
    layer.with_bias = bool(a["with_bias"])
    _load_regulariser(open_f, layer)
    _load_params(open_f, layer, ["weights"] + (["bias"] if layer.with_bias else []), load_grads)


def _save_dw(layer, open_f, save_grads):
    d = _info(open_f, layer)
    d.attrs["stride"] = int(layer.stride)
    d.attrs["padding"] = int(layer.padding)
    d.attrs["with_bias"] = bool(layer.with_bias)
    for k in ("num_filters", "f_rows", "f_cols"):
        d.attrs[k] = int(getattr(layer, k))
    w = _write(open_f, layer.layer_name + "/weights", layer.learned_params["weights"])
    _save_regulariser(w, layer)
    if layer.with_bias:
        _write(open_f, layer.layer_name + "/bias", layer.learned_params["bias"])
    if save_grads:
        for k in ["weights"] + (["bias"] if layer.with_bias else []):
            _write(open_f, layer.layer_name + "/grads/" + k, layer.grads[k])


def _load_dw(layer, open_f, load_grads):
    a = _attrs(open_f, layer)
    for k in ("f_cols", "f_rows", "num_filters", "stride", "padding"):
        setattr(layer, k, int(a[k]))
    layer.with_bias = bool(a["with_bias"])
    _load_regulariser(open_f, layer)
    _load_params(open_f, layer, ["weights"] + (["bias"] if layer.with_bias else []), load_grads)


def _save_pw(layer, open_f, save_grads):
    d = _info(open_f, layer)
    d.attrs["with_bias"] = bool(layer.with_bias)
    d.attrs["num_filters"] = int(layer.num_filters)
    d.attrs["num_channels"] = int(layer.num_channels)
    d.attrs["stride"] = int(layer.stride)
    w = _write(open_f, layer.layer_name + "/weights", layer.learned_params["weights"])
    _save_regulariser(w, layer)
    if layer.with_bias:
        _write(open_f, layer.layer_name + "/bias", layer.learned_params["bias"])
    if save_grads:
        for k in ["weights"] + (["bias"] if layer.with_bias else []):
            _write(open_f, layer.layer_name + "/grads/" + k, layer.grads[k])


def _load_pw(layer, open_f, load_grads):
    a = _attrs(open_f, layer)
    layer.num_filters = int(a["num_filters"])
    layer.num_channels = int(a["num_channels"])
    stride = a.get("stride", None)  # older files have no stride (pointwise_convolution.py:111-115)
    layer.stride = int(stride) if stride else 1
    layer.with_bias = bool(a["with_bias"])
    _load_regulariser(open_f, layer)
    _load_params(open_f, layer, ["weights"] + (["bias"] if layer.with_bias else []), load_grads)


def _save_dense(layer, open_f, save_grads):
    d = _info(open_f, layer)
    d.attrs["incoming_chans"] = int(layer.incoming_chans)
    d.attrs["output_dim"] = int(layer.output_dim)
    d.attrs["with_bias"] = bool(layer.with_bias)
    w = _write(open_f, layer.layer_name + "/weights", layer.learned_params["weights"])
    _save_regulariser(w, layer)
    if layer.with_bias:
        _write(open_f, layer.layer_name + "/bias", layer.learned_params["bias"])
    if save_grads:
        for k in ["weights"] + (["bias"] if layer.with_bias else []):
            _write(open_f, layer.layer_name + "/grads/" + k, layer.grads[k])


def _load_dense(layer, open_f, load_grads):
    a = _attrs(open_f, layer)
    layer.incoming_chans = int(a["incoming_chans"])
    layer.output_dim = int(a["output_dim"])
    layer.with_bias = bool(a["with_bias"])
    _load_regulariser(open_f, layer)
    _load_params(open_f, layer, ["weights"] + (["bias"] if layer.with_bias else []), load_grads)


def _save_bn(layer, open_f, save_grads):
    d = _info(open_f, layer)
    d.attrs["input_dimension"] = int(layer.input_dimension)
    d.attrs["run_momentum"] = float(layer.run_momentum)
    d.attrs["incoming_chans"] = int(layer.incoming_chans)
    d.attrs["eps"] = float(layer.eps)
    for k in ("gamma", "beta"):
        _write(open_f, layer.layer_name + "/" + k, layer.learned_params[k])
    for k in ("running_mean", "running_std"):
        v = layer.non_learned_params.get(k)
        if v is None:
            raise ValueError("BatchNormLayer {}: running statistics are unset (no training-mode forward "
                             "yet); the reference cannot save this state either".format(layer.layer_name))
        _write(open_f, layer.layer_name + "/" + k, v)
    if save_grads:
        for k in ("gamma", "beta"):
            _write(open_f, layer.layer_name + "/grads/" + k, layer.grads[k])


def _load_bn(layer, open_f, load_grads):
    a = _attrs(open_f, layer)
    layer.eps = float(a["eps"])
    layer.incoming_chans = int(a["incoming_chans"])
    layer.input_dimension = int(a["input_dimension"])
    layer.run_momentum = float(a["run_momentum"])
    if layer.input_dimension not in {2, 4}:
        raise ValueError("BatchNorm input_dimension should have length 2 or 4...")
    layer.av_axis = (0, 2, 3) if layer.input_dimension == 4 else 0
    _load_params(open_f, layer, ["gamma", "beta"], load_grads)
    if layer.non_learned_params is None:
        layer.non_learned_params = {}
    for k in ("running_mean", "running_std"):
        _put(layer, layer.non_learned_params, k, open_f[layer.layer_name + "/" + k][:])
    if hasattr(layer, "_on_params_loaded"):
        layer._on_params_loaded()


def _save_plain(layer, open_f, save_grads):
    _info(open_f, layer)


def _load_plain(layer, open_f, load_grads):
    pass


def _new_layer(l_type, name):
    from ..layers.activations import ReLu
    from ..layers.batch_norm import BatchNormLayer
    from ..layers.convolution import ConvLayer
    from ..layers.dense_layer import DenseLayer
    from ..layers.depthwise_convolution import DepthwiseConvLayer
    from ..layers.losses import SoftmaxWithCrossEntropy
    from ..layers.pointwise_convolution import PointwiseConvLayer
    from ..layers.pooling import GlobalAveragePoolingLayer
    from ..layers.residual_block import ResidualBlock
    classes = {c.__name__: c for c in (ConvLayer, BatchNormLayer, ReLu, DepthwiseConvLayer, PointwiseConvLayer,
                                       GlobalAveragePoolingLayer, DenseLayer, ResidualBlock,
                                       SoftmaxWithCrossEntropy)}
    if l_type not in classes:
        raise ValueError("unknown layer type {!r} for layer {!r}".format(l_type, name))
    return classes[l_type](name)


def _save_residual(layer, open_f, save_grads):
    d = _info(open_f, layer)
    d.attrs["layer_type_list"] = [l.__class__.__name__ for l in layer.layer_list]
    d.attrs["layer_name_list"] = [l.layer_name for l in layer.layer_list]
    d.attrs["post_skip_activation_type"] = layer.post_skip_activation.__class__.__name__
    d.attrs["post_skip_activation_name"] = layer.post_skip_activation.layer_name
    if layer.skip_projection is not None:
        d.attrs["skip_projection_type"] = layer.skip_projection.__class__.__name__
        d.attrs["skip_projection_name"] = layer.skip_projection.layer_name
    for l in layer.layer_list:
        l.save_to_h5(open_f, save_grads=save_grads)
    if layer.skip_projection is not None:
        layer.skip_projection.save_to_h5(open_f, save_grads=save_grads)
    layer.post_skip_activation.save_to_h5(open_f, save_grads=save_grads)


def _load_residual(layer, open_f, load_grads):
    """residual_block.py:116-151.  Sub-layers are created from the stored types and names; a
    block that already holds a sub-layer of that name and type (e.g. one already on the GPU)
    loads into it in place instead."""
    a = _attrs(open_f, layer)

    def sub(t, n, current):
        have = {l.layer_name: l for l in current if l is not None}
        l = have.get(n)
        if l is None or type(l).__name__ != t:
            l = _new_layer(t, n)
            if getattr(layer, "is_on_gpu", False):
                l.load_from_h5(open_f, load_grads=load_grads)
                l.to_gpu()
                return l
        l.load_from_h5(open_f, load_grads=load_grads)
        return l

    types = [_as_str(t) for t in a["layer_type_list"]]
    names = [_as_str(n) for n in a["layer_name_list"]]
    layer.layer_list = [sub(t, n, layer.layer_list or []) for t, n in zip(types, names)]
    if a.get("skip_projection_type", None):
        t = _as_str(a["skip_projection_type"])
        if t != "PointwiseConvLayer":
            raise ValueError("ResidualBlock: unrecognised skip_projection type {}".format(t))
        layer.skip_projection = sub(t, _as_str(a["skip_projection_name"]), [layer.skip_projection])
    t = _as_str(a["post_skip_activation_type"])
    if t != "ReLu":
        raise ValueError("ResidualBlock: unrecognised post_skip_activation type {}".format(t))
    layer.post_skip_activation = sub(t, _as_str(a["post_skip_activation_name"]), [layer.post_skip_activation])


_HANDLERS = {
    "ConvLayer": (_save_conv, _load_conv),
    "DepthwiseConvLayer": (_save_dw, _load_dw),
    "PointwiseConvLayer": (_save_pw, _load_pw),
    "DenseLayer": (_save_dense, _load_dense),
    "BatchNormLayer": (_save_bn, _load_bn),
    "ReLu": (_save_plain, _load_plain),
    "GlobalAveragePoolingLayer": (_save_plain, _load_plain),
    "SoftmaxWithCrossEntropy": (_save_plain, _load_plain),
    "ResidualBlock": (_save_residual, _load_residual),
}


def _handler(layer, which):
    for cls in type(layer).__mro__:
        if cls.__name__ in _HANDLERS:
            return _HANDLERS[cls.__name__][which]
    raise NotImplementedError("no h5 checkpoint handler for {}".format(type(layer).__name__))


def save_layer(layer, open_f, save_grads=True):
    _handler(layer, 0)(layer, open_f, save_grads)


def load_layer(layer, open_f, load_grads=True):
    _handler(layer, 1)(layer, open_f, load_grads)


def load_network(network, json_fname, h5_fname):
    """network/feed_forward_network.py:106-139: the JSON names the layers in order (its values
    are their reprs), the h5 file holds each layer's type and parameters."""
    with open(json_fname, "r") as f:
        structure = json.load(f)
    with open_h5(h5_fname, "r") as f:
        network.name = structure["name"]
        del structure["name"]
        for layer_name in structure.keys():
            l_type = _as_str(f[layer_name + "/layer_info"].attrs["type"])
            layer = _new_layer(l_type, layer_name)
            layer.load_from_h5(f)
            if l_type == "SoftmaxWithCrossEntropy":
                network.loss_layer = layer
            else:
                network.layers.append(layer)
