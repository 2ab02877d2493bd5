"""Device-tensor plumbing shared by the layers.

Activations keep the reference's logical NCHW shape (layers/convolution.py:86 already
returns an NCHW *view* of an NHWC buffer) and use channels_last strides, i.e. NHWC
bytes in HBM, which is what every kernel in libdorknet_hip.so reads and writes.
"""
from __future__ import annotations

import numpy as np
import torch

from ._hip import lib, stream_handle

F32 = torch.float32


_get_dev = getattr(torch._C, "_cuda_getDevice", None)


def device() -> torch.device:
    # (the raw C query: torch.cuda.current_device() re-checks initialisation on every call)
    if _get_dev is not None and torch.cuda.is_initialized():
        return torch.device("cuda", _get_dev())
    return torch.device("cuda", torch.cuda.current_device())


def as_device(x, dtype=F32) -> torch.Tensor:
    """numpy / torch (any device) -> torch tensor on the current HIP device (the
    cp.asarray of the reference's training loop, examples/...depsep.py:219-221)."""
    if hasattr(x, "materialize"):  # a BatchNorm output not yet written (layers/_bn_input.BNOut)
        x = x.materialize()
    if isinstance(x, torch.Tensor):
        if x.device.type != "cuda" or x.dtype != dtype:
            x = x.to(device=device(), dtype=dtype)
        return x
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=device())


BF16 = torch.bfloat16


def act_dtype(x) -> torch.dtype:
    """Storage type of an activation: bf16 if the tensor (or a BNOut's raw input) is bf16
    (BASELINE config 5: the layers then run their _bf16 entry points), else fp32."""
    t = getattr(x, "x", x) if hasattr(x, "materialize") else x
    return BF16 if isinstance(t, torch.Tensor) and t.dtype == BF16 else F32


_CUDA = torch.device("cuda")  # the current device (one process drives one GPU)


def empty_nhwc(n: int, c: int, h: int, w: int, dtype=F32) -> torch.Tensor:
    return torch.empty((n, c, h, w), dtype=dtype, device=_CUDA, memory_format=torch.channels_last)


def is_nhwc(x: torch.Tensor) -> bool:
    return x.is_contiguous(memory_format=torch.channels_last)


def to_nhwc(x, cpad: int = 1) -> torch.Tensor:
    """Return a channels_last device tensor (fp32, or bf16 for a bf16 input) whose channel
    count is padded (with zeros) up to a multiple of `cpad`.  No copy when `x` already
    qualifies."""
    x = as_device(x, act_dtype(x))
    if x.dim() != 4:
        raise ValueError(f"expected a 4-D (N, C, H, W) tensor, got shape {tuple(x.shape)}")
    n, c, h, w = x.shape
    cp = -(-c // cpad) * cpad
    if cp == c and is_nhwc(x):
        return x
    if x.dtype == BF16:
        # layout plumbing for a bf16 input given in NCHW: a copy into channels_last (+ zero
        # channels), no arithmetic
        out = torch.zeros((n, cp, h, w), dtype=BF16, device=x.device, memory_format=torch.channels_last)
        out[:, :c].copy_(x)
        return out
    if cp == c and x.is_contiguous():
        src = x
    else:
        src = x.contiguous()
    out = empty_nhwc(n, cp, h, w)
    lib.dk_nchw_to_nhwc_f32(src.data_ptr(), n, c, h, w, cp, out.data_ptr(), stream_handle())
    return out


def rows(x: torch.Tensor) -> torch.Tensor:
    """A row-major 2-D fp32 device tensor (dense-layer activations)."""
    x = as_device(x)
    return x if x.is_contiguous() else x.contiguous()


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def to_param(v) -> torch.Tensor:
    """Reference parameters start as numpy arrays (layers/layer.py:18-34 moves them with
    cp.asarray); here to_gpu() makes them fp32 device tensors."""
    if isinstance(v, torch.Tensor):
        return v.to(device=device(), dtype=F32).contiguous()
    return torch.as_tensor(np.ascontiguousarray(v, dtype=np.float32), device=device())


def scalar_zero() -> torch.Tensor:
    return torch.zeros((), dtype=F32, device=device())
