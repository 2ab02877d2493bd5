"""h5 checkpoint layout (reference: per-layer save_to_h5 / load_from_h5, e.g.
layers/convolution.py:226-281, layers/batch_norm.py:176-232,
layers/residual_block.py:99-151; network/feed_forward_network.py:90-139).

h5py is not installed in this image, so the h5 entry points raise a clear error for
now; this row is ranked "next" (SURVEY.md section 8 f, row 3).
"""
from __future__ import annotations


def _h5py():
    try:
        import h5py  # noqa: F401
    except ImportError as e:  # pragma: no cover - environment dependent
        raise NotImplementedError("h5 checkpoints need h5py, which is not installed in this image") from e
    return h5py


def open_h5(fname, mode):
    return _h5py().File(fname, mode)


def save_layer(layer, open_f, save_grads=True):
    _h5py()
    raise NotImplementedError("h5 checkpoint save is not implemented yet (SURVEY.md 8f row 3)")


def load_layer(layer, open_f, load_grads=True):
    _h5py()
    raise NotImplementedError("h5 checkpoint load is not implemented yet (SURVEY.md 8f row 3)")


def load_network(network, json_fname, h5_fname):
    _h5py()
    raise NotImplementedError("h5 checkpoint load is not implemented yet (SURVEY.md 8f row 3)")
