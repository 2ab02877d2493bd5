"""ctypes binding to libdorknet_hip.so (the C ABI declared in include/dorknet_hip.h).

The prototypes are parsed from the header itself, so the Python side and the C side
cannot drift apart.  There is no fallback: if the library (or a GPU) is missing, every
compute entry point raises.  This mirrors how the reference binds its kernels at
``to_gpu()`` time with ``cupy.RawKernel`` (layers/convolution.py:53-55,
layers/depthwise_convolution.py:53-55) -- except that here the kernels are compiled
ahead of time for gfx950 by ``__graft_entry__.build()``.
"""
from __future__ import annotations

import ctypes
import os
import re

import torch  # noqa: F401  -- loads torch's HIP runtime first; our .so binds to the same one

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG_DIR, "lib", "libdorknet_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_PKG_DIR), "include", "dorknet_hip.h")

DK_ERR_ARGS = 10001
DK_ERR_WORKSPACE = 10002

_SCALARS = {
    "int": ctypes.c_int,
    "long long": ctypes.c_longlong,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "size_t": ctypes.c_size_t,
}


class HipError(RuntimeError):
    """A dorknet_hip entry point returned a non-zero status."""


def parse_header(path: str = HEADER_PATH) -> dict[str, tuple[str, list[tuple[str, str]]]]:
    """Return {name: (return_type, [(c_type, arg_name), ...])} for every dk_* declaration."""
    with open(path) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(int|size_t)\s+(dk_\w+)\s*\(([^)]*)\)\s*;", text):
        ret, name, args = m.group(1), m.group(2), m.group(3).strip()
        params = []
        if args and args != "void":
            for a in args.split(","):
                a = " ".join(a.split())
                am = re.match(r"(.*?)(\w+)$", a)
                ctype, aname = am.group(1).strip(), am.group(2)
                params.append((ctype, aname))
        decls[name] = (ret, params)
    return decls


def _argtype(ctype: str):
    if "*" in ctype:
        return ctypes.c_void_p
    base = ctype.replace("const", "").strip()
    if base not in _SCALARS:
        raise TypeError(f"unsupported C type in header: {ctype!r}")
    return _SCALARS[base]


def _errcheck(result, func, args):
    if result != 0:
        what = {DK_ERR_ARGS: "bad arguments", DK_ERR_WORKSPACE: "workspace too small"}.get(result, "hipError")
        raise HipError(f"{func.__name__} failed with status {result} ({what})")
    return result


class _Lib:
    def __init__(self):
        self._lib = None
        self._decls = None

    def _load(self):
        if self._lib is not None:
            return
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"dorknet_amd HIP library not found at {LIB_PATH}; run `python -c "
                f"'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950). "
                f"There is no CPU fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        decls = parse_header()
        for name, (ret, params) in decls.items():
            fn = getattr(lib, name)
            fn.restype = ctypes.c_size_t if ret == "size_t" else ctypes.c_int
            fn.argtypes = [_argtype(t) for t, _ in params]
            if ret == "int" and not name.endswith(("_blocks", "_version", "_rows", "_count")) and not name.startswith("dk_debug"):
                fn.errcheck = _errcheck
        self._decls = decls
        self._lib = lib

    def __getattr__(self, name):
        if name.startswith("dk_"):
            self._load()
            fn = getattr(self._lib, name)
            setattr(self, name, fn)
            return fn
        raise AttributeError(name)

    @property
    def declarations(self):
        self._load()
        return self._decls


lib = _Lib()


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise RuntimeError("dorknet_amd runs its compute path on an MI355X GPU only (no CPU fallback); "
                           "no HIP device is visible")


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


class Workspace:
    """A grow-only device scratch buffer shared by kernels issued on one stream.

    Kernels on the same stream run in order, so consecutive launches may reuse the
    same bytes; torch's caching allocator keeps a replaced buffer alive until the
    work queued before the replacement has run (same-stream reuse semantics).
    """

    def __init__(self):
        self._buf = None

    def get(self, nbytes: int) -> int:
        nbytes = max(int(nbytes), 256)
        if self._buf is None or self._buf.numel() < nbytes:
            grow = nbytes if self._buf is None else max(nbytes, int(self._buf.numel() * 1.25))
            self._buf = torch.empty(grow, dtype=torch.uint8, device="cuda")
        return self._buf.data_ptr()

    def nbytes(self) -> int:
        return 0 if self._buf is None else self._buf.numel()


workspace = Workspace()


class Tickets:
    """Zeroed ticket words for the one-launch folds (dk_bn_*_from_partials_f32 `tickets`).
    Zeroed once when allocated; every call leaves them zero.  Calls on one stream only."""

    def __init__(self):
        self._buf = None

    def get(self, n: int) -> int:
        if self._buf is None or self._buf.numel() < n:
            self._buf = torch.zeros(max(int(n), 256), dtype=torch.int32, device="cuda")
        return self._buf.data_ptr()


tickets = Tickets()
