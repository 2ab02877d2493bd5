"""Sequential execution of a layer list with BatchNorm fusion.

Used by FeedForwardNetwork (network/feed_forward_network.py:47-70 in the reference) and
ResidualBlock (layers/residual_block.py:65-97).  Each layer keeps its own
forward/backward; the executor only decides how a BatchNormLayer (optionally followed by a
ReLu) runs, records the groups it ran, and replays them in reverse for backward:

  * "defer"  -- the next layer applies the normalisation (+ReLU) on load
                (``accepts_bn_input``; layers/_bn_input.py), so the BN output is never
                written: BatchNormLayer.forward_deferred hands over a BNOut;
  * "pair"   -- BN + ReLU in one apply pass (BatchNormLayer.forward_bn_relu);
  * "single" -- the layer on its own.

Backward is the same for all three: BatchNormLayer.backward[_bn_relu] recomputes what it
needs from the BN's raw input.  Set DORKNET_FUSE=0 to run every layer on its own (used by
the per-layer parity tests; results are bit-identical either way).
"""
from __future__ import annotations

from .._env import enabled
from .._hip import (DK_FOLDED, disarm_folds, early_flush_steps, flush_wgrad_reduces, inlaunch_folds_enabled,
                    inline_wgrad_reduces, lib, resolve)
from ._bn_input import accepts_bn_grad, accepts_bn_input, add_residual

# BatchNormLayer / ReLu (their modules import this one): bound on first use
_BN_RELU = []


def _bn_relu():
    if not _BN_RELU:
        from .activations import ReLu
        from .batch_norm import BatchNormLayer
        _BN_RELU.extend((BatchNormLayer, ReLu))
    return _BN_RELU


# Backward-progress listeners: f(layers) is called once the backward of `layers` (leaf layers of
# a chain step, or a residual block's skip projection) has been issued, i.e. their gradients are
# queued on the streams.  DataParallel launches a gradient bucket's all-reduce as soon as every
# layer it covers has been reported -- at sub-layer granularity inside residual blocks
# (residual_block.py:86-97), not once per top-level step.
_progress = []


class backward_progress:
    """with backward_progress(fn): fn(layers) after each step's backward (see _progress)."""

    def __init__(self, fn):
        self.fn = fn

    def __enter__(self):
        _progress.append(self.fn)
        return self

    def __exit__(self, *exc):
        _progress.remove(self.fn)
        return False


def notify_backward_done(layers):
    for f in list(_progress):
        f(layers)


def fusion_enabled() -> bool:
    return enabled("DORKNET_FUSE")


def fusable_pair(layer, nxt) -> bool:
    BatchNormLayer, ReLu = _bn_relu()
    return type(layer) is BatchNormLayer and type(nxt) is ReLu


def plan_group(layers, i, fuse, out_accepts=False, keep=()):
    """How to run layers[i:]: returns (group, mode).  `out_accepts`: whether whatever consumes
    the end of the list takes a BNOut; `keep`: layer names whose output must be materialised
    (e.g. a terminal layer)."""
    BatchNormLayer, ReLu = _bn_relu()
    layer = layers[i]
    if fuse and type(layer) is BatchNormLayer:
        relu = layers[i + 1] if i + 1 < len(layers) and type(layers[i + 1]) is ReLu else None
        group = (layer, relu) if relu is not None else (layer,)
        j = i + len(group)
        consumer_ok = accepts_bn_input(layers[j]) if j < len(layers) else out_accepts
        if consumer_ok and not any(l.layer_name in keep for l in group):
            return group, "defer"
        if relu is not None and layer.layer_name not in keep:
            return group, "pair"
    return (layer,), "single"


class StatsRequest:
    """Asks a producer layer (``produces_bn_stats``) to emit, with its forward output, the
    BatchNorm partial statistics of that output (the *_fwd_ex_f32 entry points); the
    BatchNormLayer that follows then skips its own statistics pass.

    With ``bn`` (the BatchNormLayer that will consume them) the producer also arms an in-launch
    fold (``arm`` before its launch, ``launched`` after it; dorknet_amd/csrc/fold_tail.h): the
    producer's last blocks then finalize the statistics themselves and the BatchNormLayer skips
    the fold launch too."""
    __slots__ = ("part", "rows", "bn", "armed", "folded")

    def __init__(self, bn=None):
        self.part = None   # fp64 device tensor [rows, 2, C], set by the producer
        self.rows = 0
        self.bn = bn
        self.armed = None   # (mean, std, invstd) the armed fold will write
        self.folded = None  # the same, once the producer's launch has folded

    def arm(self, part, P):
        """Before the producer's launch: `part` [rows, 2, C] will hold its partial sums over P
        pixels per channel."""
        if self.bn is not None and inlaunch_folds_enabled():
            self.armed = self.bn.arm_stats_fold(part, P)

    def launched(self, part, status):
        """After the producer's launch (`status`: the entry point's return value)."""
        self.part, self.rows = part, part.shape[0]
        if self.armed is not None:
            if status == DK_FOLDED:
                self.folded = self.armed
                self.bn._first_pending = False
            else:
                lib.dk_bn_fold_disarm()
            self.armed = None


def run_group(group, mode, X, test_mode=False, stats_req=None, bn_stats=None, join_out=False):
    if join_out:
        return group[0].forward(X, test_mode=test_mode, join_out=True)
    if mode == "defer":
        return group[0].forward_deferred(X, group[1] if len(group) == 2 else None, test_mode=test_mode,
                                         stats=bn_stats)
    if mode == "pair":
        return group[0].forward_bn_relu(X, group[1], test_mode=test_mode, stats=bn_stats)
    if bn_stats is not None and type(group[0]) is _bn_relu()[0]:
        return group[0].forward(X, test_mode=test_mode, stats=bn_stats)
    if stats_req is not None:
        return group[0].forward(X, test_mode=test_mode, bn_stats=stats_req)
    return group[0].forward(X, test_mode=test_mode)


def execute(layers, X, test_mode=False, out_accepts=False, keep=(), visit=None):
    """Run `layers` in order with the fusions above; also lets a producer hand the next
    BatchNormLayer its output statistics.  `visit(group, X)` is called after each group and
    may return True to stop early.  Returns (X, steps, stopped)."""
    BatchNormLayer = _bn_relu()[0]
    steps = []
    fuse = fusion_enabled()
    pending = None
    i = 0
    while i < len(layers):
        group, mode = plan_group(layers, i, fuse, out_accepts, keep)
        nxt = i + len(group)
        req = None
        if (fuse and not test_mode and mode == "single" and getattr(group[0], "produces_bn_stats", False)
                and nxt < len(layers) and type(layers[nxt]) is BatchNormLayer):
            req = StatsRequest(layers[nxt])
        # a residual block whose output the next block forms on load (JoinOut, layers/_bn_input.py)
        join_out = (fuse and mode == "single" and req is None and pending is None
                    and getattr(group[0], "produces_join", False) and nxt < len(layers)
                    and group[0].layer_name not in keep
                    and getattr(layers[nxt], "takes_join_input", None) is not None and layers[nxt].takes_join_input())
        try:
            X = run_group(group, mode, X, test_mode, stats_req=req, bn_stats=pending, join_out=join_out)
        except BaseException:
            disarm_folds()  # an arming the failed group left behind must not outlive it
            raise
        pending = req if req is not None and req.part is not None else None
        steps.append(group)
        i = nxt
        if visit is not None and visit(group, X):
            return X, steps, True
    return X, steps, False


def chain_forward(layers, X, test_mode=False, out_accepts=False):
    """Run `layers` in order; returns (output, steps).  The output is a BNOut when the list
    ends in a BatchNormLayer [+ ReLu] and `out_accepts`."""
    X, steps, _ = execute(layers, X, test_mode, out_accepts)
    return X, steps


def _join_of(step):
    """The post-skip ReLu of a residual block step whose join can be fused into the next
    block's first dgrad (its BatchNorm-on-load join: ReLu._join_bn), else None."""
    if len(step) != 1 or not enabled("DORKNET_FUSE_JOIN"):
        return None
    act = getattr(step[0], "post_skip_activation", None)
    if act is None or getattr(act, "_join_bn", None) is None:
        return None
    if getattr(act, "_mask", None) is None and getattr(act, "_join_y", None) is None:
        return None
    return act


def chain_backward(steps, dy, residual=None, after_step=None, need_input_grad=True, join=None):
    """Backward through `steps` in reverse.  `residual`: a gradient to add to the result (the
    residual join's other branch); the first layer adds it in its dgrad epilogue when it
    can (``accepts_residual``), otherwise it is added separately.  `after_step(i)` runs after
    step i's backward has been issued (DataParallel launches its gradient buckets there).
    need_input_grad=False: the caller discards the gradient w.r.t. the chain's input (the
    network's image gradient, which the reference's network.backward computes and drops,
    feed_forward_network.py:64-70), so a first layer with ``skips_input_grad`` computes only
    its parameter gradients and None is returned.  `join`: the residual join whose output is
    the chain's input (passed to a first layer that ``accepts_join``); a residual-block step
    likewise receives the previous block's join."""
    try:
        dy = _backward_steps(steps, dy, residual, after_step, need_input_grad, join)
    except BaseException:
        disarm_folds()  # an arming the failed step left behind must not outlive it
        raise
    return dy


def _backward_steps(steps, dy, residual, after_step, need_input_grad, join):
    BatchNormLayer = _bn_relu()[0]
    last = len(steps) - 1
    fuse = fusion_enabled()
    # the network's own chain (its image gradient is dropped): the weight-gradient reduces recorded
    # so far go to the side stream before the last steps, where they run beside those steps'
    # kernels instead of after the last one (_hip.early_flush_steps)
    early = early_flush_steps() if not need_input_grad else 0
    for i in range(last, -1, -1):
        if i < early:
            flush_wgrad_reduces()
        if i == 0 and early and enabled("DORKNET_WGRAD_INLINE_LAST"):
            with inline_wgrad_reduces():
                dy, residual = _backward_step(steps, i, dy, residual, need_input_grad, join, fuse, BatchNormLayer)
        else:
            dy, residual = _backward_step(steps, i, dy, residual, need_input_grad, join, fuse, BatchNormLayer)
        if _progress:
            notify_backward_done(steps[i])
        if after_step is not None:
            after_step(i)
    if residual is not None:
        dy = add_residual(dy, resolve(residual))
    return dy


def _backward_step(steps, i, dy, residual, need_input_grad, join, fuse, BatchNormLayer):
    """Step i of _backward_steps: (its input gradient, the residual still to add -- None once
    step 0 has added it in its dgrad epilogue)."""
    step = steps[i]
    # a BatchNorm whose producer can apply its backward while loading the gradient
    # (layers/_bn_input.py BNGrad) hands over a deferred gradient instead of writing it
    defer = (fuse and type(step[0]) is BatchNormLayer and i > 0 and len(steps[i - 1]) == 1
             and accepts_bn_grad(steps[i - 1][0], step[0]))
    if len(step) == 2:
        return step[0].backward_bn_relu(dy, step[1], defer=defer), residual
    if defer:
        return step[0].backward(dy, defer=True), residual
    if i == 0 and not need_input_grad and residual is None and getattr(step[0], "skips_input_grad", False):
        return step[0].backward(dy, need_dx=False), residual
    if i == 0 and residual is not None and getattr(step[0], "accepts_residual", False):
        residual = resolve(residual)  # a skip gradient from the branch stream: wait for it here
        if join is not None and getattr(step[0], "accepts_join", False):
            return step[0].backward(dy, residual=residual, join=join), None
        return step[0].backward(dy, residual=residual), None
    if (fuse and i >= 2 and len(step) == 1 and getattr(step[0], "lattice_ok", None) is not None
            and step[0].lattice_ok() and type(steps[i - 1][0]) is BatchNormLayer and len(steps[i - 2]) == 1
            and getattr(steps[i - 2][0], "accepts_lattice_grad", False)
            and accepts_bn_grad(steps[i - 2][0], steps[i - 1][0])
            and enabled("DORKNET_LATTICE")):
        # a stride-2 pointwise layer whose input gradient goes (through a deferred BatchNorm) to a
        # consumer that takes the lattice form: the widen's zeros are never written
        return step[0].backward(dy, lattice_out=True), residual
    if fuse and i > 0 and len(step) == 1 and getattr(step[0], "accepts_join", False) and \
            _join_of(steps[i - 1]) is not None:
        return step[0].backward(dy, join=_join_of(steps[i - 1])), residual
    return step[0].backward(dy), residual
