"""Small helpers shared by the parameterised layers."""
from __future__ import annotations

import numpy as np
import torch

from .._hip import lib, stream_handle
from .._tensor import as_device


def l2_strength(reg):
    """Strength to fold into the weight-gradient kernel, or None when the regulariser
    is not an l2 (then its backward() is added separately)."""
    if reg is None:
        return 0.0
    if getattr(reg, "type", None) == "l2" and hasattr(reg, "strength"):
        return float(reg.strength)
    return None


def add_regulariser_grad(grad: torch.Tensor, weights: torch.Tensor, reg) -> None:
    """grads["weights"] += reg.backward(W) for a non-l2 regulariser (kept general like
    convolution.py:99-100)."""
    extra = as_device(reg.backward(weights)).contiguous()
    lib.dk_add_f32(grad.data_ptr(), extra.data_ptr(), grad.numel(), 0, grad.data_ptr(), 0, stream_handle())


def grad_buffer(layer, key: str, shape) -> torch.Tensor:
    """The layer's persistent gradient tensor for `key`, (re)allocated if missing or of
    the wrong shape.  Backward passes overwrite it in place: values follow the
    reference's "backward overwrites self.grads[k]" semantics while the tensor object
    stays stable for the optimiser table and data-parallel gradient buckets."""
    g = layer.grads.get(key)
    # fast path (every backward): the tensor this function handed out last time, same shape
    cache = layer.__dict__.setdefault("_grad_buffer_cache", {})
    hit = cache.get(key)
    if hit is not None and hit[0] is g and hit[1] == shape:
        return g
    shape_t = tuple(int(s) for s in shape)
    if not isinstance(g, torch.Tensor) or g.device.type != "cuda" or tuple(g.shape) != shape_t \
            or not g.is_contiguous():
        g = torch.empty(shape_t, dtype=torch.float32, device=torch.device("cuda", torch.cuda.current_device()))
        layer.grads[key] = g
    cache[key] = (g, shape)
    return g


def init_weights(shape, initialiser: str, fan_sum: float) -> np.ndarray:
    """Reference initialisers (convolution.py:24-28 and siblings), numpy's global RNG."""
    if initialiser == "glorot_uniform":
        limit = np.sqrt(6.0 / fan_sum)
        return np.random.uniform(low=-limit, high=limit, size=shape).astype(np.float32)
    elif initialiser == "normal":
        return 0.01 * np.random.randn(*shape).astype(np.float32)
    raise ValueError("unknown weight_initialiser {!r}".format(initialiser))


def patches_count(in_size: int, f: int, stride: int, padding: int):
    """The reference's output-size arithmetic: a float ((Hp - f)/stride) + 1
    (convolution.py:67-68), truncated by int() where used as a size."""
    full = ((in_size + 2 * padding - f) / stride) + 1
    return full, int(full)
