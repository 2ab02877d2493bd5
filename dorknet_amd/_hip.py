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

from ._env import enabled, getenv

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# DORKNET_HIP_LIB: another build of the same library (A/B runs of two builds on one box)
LIB_PATH = os.environ.get("DORKNET_HIP_LIB") or os.path.join(_PKG_DIR, "lib", "libdorknet_hip.so")
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


DK_FOLDED = 10100  # success, and the launch folded the armed BN partials (dk_bn_fold_arm_*)


def _errcheck(result, func, args):
    if result != 0 and result != DK_FOLDED:
        # a failed entry point may not have taken an in-launch fold armed for it: drop the
        # arming, or a later partials buffer at the same address would fold into stale outputs
        disarm_folds()
        what = {DK_ERR_ARGS: "bad arguments", DK_ERR_WORKSPACE: "workspace too small"}.get(result, "hipError")
        raise HipError(f"{func.__name__} failed with status {result} ({what})")
    return result


def disarm_folds() -> None:
    """Drop any in-launch BN fold arming (dk_bn_fold_disarm; thread-local C++ state)."""
    raw = lib._lib
    if raw is not None:
        raw.dk_bn_fold_disarm()


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
            counts = (name.endswith(("_blocks", "_version", "_rows", "_count", "_preferred", "_pending"))
                      or name.startswith("dk_debug"))
            if ret == "int" and not counts:
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


# The current device / stream as raw values straight from torch's C layer: every entry-point call
# asks for the stream, and torch.cuda.current_stream() (a Stream object, device-index resolution,
# availability checks) cost ~2.5 us of host time per call -- 300 calls per training step.
_get_dev = getattr(torch._C, "_cuda_getDevice", None)
_get_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_handle() -> int:
    if _get_raw_stream is not None:
        return _get_raw_stream(_get_dev())
    return torch.cuda.current_stream().cuda_stream


# The same for the stream objects the side / branch streams are joined with: torch.cuda.current_stream()
# and the torch.cuda.stream() context resolve the device index through Python on every call (~9 us
# and ~20 us); these go to the C layer directly.  One process drives one device (the current one).
_get_cur_stream = getattr(torch._C, "_cuda_getCurrentStream", None)
_set_cur_stream = getattr(torch._C, "_cuda_setStream", None)


def cur_stream():
    """torch.cuda.current_stream() for the current device."""
    if _get_cur_stream is None or _get_dev is None:
        return torch.cuda.current_stream()
    sid, di, dt = _get_cur_stream(_get_dev())
    return torch.cuda.Stream(stream_id=sid, device_index=di, device_type=dt)


class use_stream:
    """with use_stream(s): torch.cuda.stream(s) for a stream of the current device."""
    __slots__ = ("s", "prev", "ctx")

    def __init__(self, s):
        self.s = s
        self.prev = None
        self.ctx = None

    def __enter__(self):
        if _get_cur_stream is None or _set_cur_stream is None or _get_dev is None:
            self.ctx = torch.cuda.stream(self.s)
            self.ctx.__enter__()
            return self
        self.prev = _get_cur_stream(_get_dev())
        s = self.s
        _set_cur_stream(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)
        return self

    def __exit__(self, *exc):
        if self.ctx is not None:
            return self.ctx.__exit__(*exc)
        sid, di, dt = self.prev
        _set_cur_stream(stream_id=sid, device_index=di, device_type=dt)
        return False


class Workspace:
    """Grow-only device scratch buffers, one per stream.

    Kernels on the same stream run in order, so consecutive launches may reuse the
    same bytes; torch's caching allocator keeps a replaced buffer alive until the
    work queued before the replacement has run (same-stream reuse semantics).  Work on
    the weight-gradient side stream (see weight_grad_stream) gets its own buffer.
    """

    def __init__(self):
        self._bufs = {}

    def get(self, nbytes: int) -> int:
        nbytes = max(int(nbytes), 256)
        key = stream_handle()
        buf = self._bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            grow = nbytes if buf is None else max(nbytes, int(buf.numel() * 1.25))
            buf = torch.empty(grow, dtype=torch.uint8, device="cuda")
            self._bufs[key] = buf
        return buf.data_ptr()

    def nbytes(self) -> int:
        return sum(b.numel() for b in self._bufs.values())


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


class FoldResources:
    """Ticket words and group-row scratch for in-launch BN folds (dk_bn_fold_arm_*), one set
    per stream (the folding launches of a stream run in order; the tickets are left zero).
    DORKNET_INLAUNCH_FOLD=0 turns the in-launch folds off (the separate fold launches run)."""

    TICKETS = 16384
    SCRATCH = 8 << 20

    def __init__(self):
        self._res = {}

    def get(self):
        """(tickets ptr, ticket words, scratch ptr, scratch bytes) for the current stream."""
        key = stream_handle()
        r = self._res.get(key)
        if r is None:
            t = torch.zeros(self.TICKETS, dtype=torch.int32, device="cuda")
            sc = torch.empty(self.SCRATCH, dtype=torch.uint8, device="cuda")
            r = self._res[key] = (t, sc, (t.data_ptr(), self.TICKETS, sc.data_ptr(), self.SCRATCH))
        return r[2]


fold_resources = FoldResources()


def inlaunch_folds_enabled() -> bool:
    return enabled("DORKNET_INLAUNCH_FOLD")


# ---------------------------------------------------------------------------------------
# Weight gradients on a side stream.  A layer's weight gradient and its input gradient
# are independent (both read dy); the input gradient is on the critical path of the
# backward pass, the weight gradient only has to be done before the update (or its
# all-reduce bucket).  Running the weight gradients on a second stream lets them fill the
# GPU beside the small and tail-heavy kernels of the critical path.
# DORKNET_ASYNC_WGRAD=0 keeps everything on the caller's stream.
# ---------------------------------------------------------------------------------------
_SIDE = {}
_ASYNC_DEPTH = [0]


def async_wgrad_enabled() -> bool:
    """Side-stream weight gradients are used only inside async_weight_grads() (the network /
    data-parallel backward), which joins them before it returns: a layer's backward called
    on its own keeps the reference's contract that grads are final when it returns."""
    return _ASYNC_DEPTH[0] > 0 and enabled("DORKNET_ASYNC_WGRAD")


def side_stream():
    dev = _get_dev() if _get_dev is not None else torch.cuda.current_device()
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return s


class _SyncEvents:
    """Events for the cross-stream hand-overs (dk_sync_event_create: no system-scope fence, no timing),
    handed out round-robin; an event is free again once the wait on it has been enqueued, and a
    recorded branch completion is waited on within the same block, long before 64 more hand-overs."""
    N = 64

    def __init__(self):
        self._ev = []
        self._i = 0

    def next(self) -> int:
        if not self._ev:
            for _ in range(self.N):
                h = ctypes.c_void_p()
                lib.dk_sync_event_create(ctypes.addressof(h))
                self._ev.append(h.value)
        e = self._ev[self._i]
        self._i = (self._i + 1) % self.N
        return e


_sync_events = _SyncEvents()


def stream_wait(waiter, src) -> None:
    """waiter.wait_stream(src) through a fence-free event (dk_stream_wait_stream): the runtime's
    default event record carries a system-scope release, ~7 us of idle main stream per hand-over."""
    lib.dk_stream_wait_stream(waiter.cuda_stream, src.cuda_stream, _sync_events.next())


class weight_grad_stream:
    """with weight_grad_stream(dy, x, ...): launches inside go to the side stream, after
    everything already queued on the current stream.  The listed tensors are marked as in
    use by the side stream (so the caching allocator does not recycle them early)."""

    def __init__(self, *tensors):
        self.tensors = tensors
        self.ctx = None

    def __enter__(self):
        if not async_wgrad_enabled():
            return self
        main = cur_stream()
        side = side_stream()
        if main == side:
            return self
        stream_wait(side, main)
        self.ctx = use_stream(side)
        self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.ctx is None:
            return False
        self.ctx.__exit__(*exc)
        side = side_stream()
        for t in self.tensors:
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(side)
        return False


class async_weight_grads:
    """with async_weight_grads(): layers' weight gradients inside go to the side stream; the
    outermost exit makes the current stream wait for them."""

    def __enter__(self):
        _ASYNC_DEPTH[0] += 1
        return self

    def __exit__(self, *exc):
        if _ASYNC_DEPTH[0] == 1:
            flush_wgrad_reduces()  # (on the side stream, while it is still the weight-gradient stream)
        _ASYNC_DEPTH[0] -= 1
        if _ASYNC_DEPTH[0] == 0:
            join_weight_grads()
        return False


def side_stream_context():
    """torch.cuda.stream(side) while weight gradients run on the side stream (for work that
    must follow them, e.g. a gradient all-reduce), else a no-op context."""
    import contextlib
    if async_wgrad_enabled():
        return use_stream(side_stream())
    return contextlib.nullcontext()


class deferred_wgrad_reduce:
    """A fused backward entry point (dk_dwconv_bwd_bnbwd_*, dk_pwconv_bwd_bnbwd_f32) whose weight-
    gradient reduce goes to the side stream: its partial slab lives in a per-layer buffer instead of
    the stream workspace (the main stream's next launches would overwrite that before the side
    stream has read it), the entry point only records the reduce (dk_wgrad_reduce_defer) and
    flush() launches it on the side stream, ordered after the entry point.  Off (the reduce stays in
    the entry point) without side-stream weight gradients or with `defer` False.

        d = deferred_wgrad_reduce(layer, nbytes, defer)
        with d:
            entry(..., d.ws, nbytes, stream)
        d.flush()
    """
    __slots__ = ("on", "slab", "ws")

    def __init__(self, layer, nbytes, defer=True):
        self.on = (bool(defer) and async_wgrad_enabled() and not _INLINE_REDUCE[0]
                   and enabled("DORKNET_WGRAD_REDUCE_SIDE"))
        if self.on:
            slab = layer.__dict__.get("_dk_wgrad_slab")
            if slab is None or slab.numel() < nbytes:
                slab = layer._dk_wgrad_slab = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device="cuda")
            self.slab = slab
            self.ws = slab.data_ptr()
        else:
            self.slab = None
            self.ws = workspace.get(nbytes)

    def __enter__(self):
        if self.on:
            lib.dk_wgrad_reduce_defer(1)
        return self

    def __exit__(self, exc_type, *exc):
        if self.on:
            lib.dk_wgrad_reduce_defer(0 if exc_type is None else -1)
        return False

    def flush(self):
        """Launch the recorded reduces once FLUSH_EVERY (60, i.e. at the end of the backward) have
        collected: each flush makes the side stream wait for the main stream,
        and every such wait put a ~7 us gap between two main-stream kernels (an event marker); the
        slabs are per layer, so a recorded reduce can wait, and a flush runs all of them as one
        multi-task kernel.  flush_wgrad_reduces() launches the rest (the end of the backward, a
        data-parallel bucket's all-reduce).  Config 3 8.374 -> 8.339 ms, config 5 6.232 -> 6.147 ms
        (profiles/r05u_ab_flush_every_multi_*.txt)."""
        if self.on and lib.dk_wgrad_reduce_pending() >= FLUSH_EVERY:
            flush_wgrad_reduces()


# Recorded reduces per flush, at most 60 (the C queue holds 64): 60 = only before the network's last
# steps and at the end of the backward.  (A module constant; tests/test_gpu_streams.py sets it to
# check that batching leaves every gradient bit-identical.)
FLUSH_EVERY = 60


_INLINE_REDUCE = [False]


class inline_wgrad_reduces:
    """with inline_wgrad_reduces(): fused entry points keep their weight-gradient reduce on the
    main stream (deferred_wgrad_reduce off).  The network's last step: nothing follows it on the
    main stream to overlap, and a reduce sent to the side stream there costs two cross-stream hops
    (~12 us each) before the update can start."""

    def __enter__(self):
        self.prev = _INLINE_REDUCE[0]
        _INLINE_REDUCE[0] = True
        return self

    def __exit__(self, *exc):
        _INLINE_REDUCE[0] = self.prev
        return False


def early_flush_steps() -> int:
    """DORKNET_WGRAD_FLUSH_LAST (default 1): the network's backward flushes the recorded reduces
    before each of its last this-many steps (0: only at the end of the backward).  With the reduces
    batched until the end, the multi-task reduce ran after the last layer's kernels: ~90 us of tail
    before the update (profiles/r05x_tail_timelines.txt); flushed before the last step it overlaps that
    step's kernels (the stem's conv weight gradient, config 5's first depthwise backward)."""
    try:
        return max(0, int(getenv("DORKNET_WGRAD_FLUSH_LAST", "1")))
    except ValueError:
        return 1


def flush_wgrad_reduces() -> None:
    """Launch every recorded weight-gradient reduce (deferred_wgrad_reduce) on the side stream,
    ordered after the main stream."""
    if lib._lib is None or lib.dk_wgrad_reduce_pending() == 0:
        return
    with weight_grad_stream():
        lib.dk_wgrad_reduce_flush(stream_handle())


def join_weight_grads() -> None:
    """Make the current stream wait for every weight gradient queued on the side stream."""
    if not _SIDE:
        return
    s = _SIDE.get(_get_dev() if _get_dev is not None else torch.cuda.current_device())
    if s is not None:
        cur = cur_stream()
        if s != cur:
            stream_wait(cur, s)


# ---------------------------------------------------------------------------------------
# A residual block's skip projection on a branch stream.  The skip branch (a strided pointwise
# layer: its forward, and in backward its input gradient) depends only on the block's input (or
# the join's gradient), so it can run beside the main branch's chain instead of before it; the
# main stream waits for it only where the two branches meet (the join; the chain's first dgrad,
# which adds the skip gradient).  DORKNET_BRANCH_STREAM=0 keeps everything on one stream.
# ---------------------------------------------------------------------------------------
_BRANCH = {}
_CUDA_OK = []


def branch_stream_enabled() -> bool:
    if not enabled("DORKNET_BRANCH_STREAM"):
        return False
    if not _CUDA_OK:
        _CUDA_OK.append(torch.cuda.is_available())
    return _CUDA_OK[0]


def branch_stream():
    dev = _get_dev() if _get_dev is not None else torch.cuda.current_device()
    s = _BRANCH.get(dev)
    if s is None:
        s = _BRANCH[dev] = torch.cuda.Stream(device=dev)
    return s


def _tensors(obj):
    """The CUDA tensors an activation-like object holds (a tensor, or a BNOut / BNGrad record)."""
    if isinstance(obj, torch.Tensor):
        return [obj] if obj.is_cuda else []
    return [v for v in vars(obj).values() if isinstance(v, torch.Tensor) and v.is_cuda] if hasattr(obj, "__dict__") else []


def record_on(stream, *objs) -> None:
    """Mark the tensors of `objs` as in use by `stream` (the caching allocator keeps them until
    the work queued there so far is done)."""
    for o in objs:
        for t in _tensors(o):
            t.record_stream(stream)


class Branch:
    """A value computed on the branch stream: `resolve()` makes the current stream wait for it
    and returns it (marked as used by the current stream)."""

    def __init__(self, value, event):
        self.value = value
        self.event = event

    def resolve(self):
        # (the value is not marked as used by the current stream: freeing a block so marked records
        # an event on that stream -- a marker, ~6 us of idle main stream.  It needs none: the block
        # returns to the branch stream's pool, and every branch-stream use starts with on_branch's
        # wait for the main stream, which orders it after the kernels that consumed this value)
        lib.dk_stream_wait_event(cur_stream().cuda_stream, self.event)
        return self.value


def resolve(v):
    return v.resolve() if isinstance(v, Branch) else v


class on_branch:
    """with on_branch(*inputs) as b: launches inside go to the branch stream, after everything
    already queued on the current stream; the inputs are marked as used there.  b.done(value)
    records the branch's completion and returns a Branch for the consumer to resolve()."""

    def __init__(self, *inputs):
        self.inputs = inputs
        self.ctx = None

    def __enter__(self):
        main = cur_stream()
        br = branch_stream()
        stream_wait(br, main)
        record_on(br, *self.inputs)
        self.ctx = use_stream(br)
        self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        self.ctx.__exit__(*exc)
        return False

    def done(self, value):
        ev = _sync_events.next()
        lib.dk_sync_event_record(ev, branch_stream().cuda_stream)
        return Branch(value, ev)

