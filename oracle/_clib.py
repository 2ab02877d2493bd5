"""ctypes loader for oracle/lib/libdorknet_oracle.so (built by oracle/Makefile)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_DIR, "lib", "libdorknet_oracle.so")
_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_longlong
_SIGS = {
    "oracle_im2col": [_P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "oracle_row2im": [_P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "oracle_depthwise_conv": [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "oracle_depthwise_backward": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P],
    "oracle_bn_stats": [_P, _I, _I, _I, _I, _P, _P],
    "oracle_relu_forward_train": [_P, _L, _P, _P],
    "oracle_num_threads": [],
    "oracle_set_threads": [_I],
}


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _DIR])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        l = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            fn = getattr(l, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int if name in ("oracle_num_threads", "oracle_set_threads") else None
        _lib = l
    return _lib


def p(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data
