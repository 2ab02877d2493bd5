"""BatchNorm output that is applied by its consumer ("BN on load").

In the reference a BatchNormLayer writes its normalised output (layers/batch_norm.py:91-96),
an optional ReLu writes another copy (activations.py:37-42), and the next layer reads it.
Here, when the next layer can take it, the pair hands over a ``BNOut`` instead: the raw
input x (which BatchNormLayer keeps for its backward anyway) plus the per-channel mean,
1/std, gamma, beta and the ReLU flag.  Consumers apply ``bn_out`` as they load each tile
(the dk_*_bnx_f32 entry points), with the same arithmetic as dk_bn_apply_f32, so their
results are bit-identical to running the layers one by one -- the normalised activation
just never exists in HBM (forward and weight-gradient passes recompute it on load).

Anything that cannot consume it calls ``materialize()`` (one dk_bn_apply_f32 pass).

Aliasing: ``mean`` / ``invstd`` are the owning BatchNormLayer's per-layer buffers (and, in test
mode, its running statistics), which that layer's next forward rewrites in place.  A BNOut is
therefore valid until its owner's next forward: ``bn_args()`` and ``materialize()`` raise on a
stale one (a per-layer generation counter) instead of silently reading the newer statistics.
"""
from __future__ import annotations

import torch

from .._hip import DK_FOLDED, inlaunch_folds_enabled, lib, stream_handle
from .._tensor import empty_nhwc, is_nhwc, to_nhwc


class BNOut:
    __slots__ = ("x", "mean", "invstd", "gamma", "beta", "relu", "owner", "_y", "gen")

    def __init__(self, x, mean, invstd, gamma, beta, relu, owner=None):
        self.x = x            # raw input of the BatchNormLayer (NHWC storage, logical NCHW)
        self.mean = mean      # (C,) fp32 device tensors
        self.invstd = invstd
        self.gamma = gamma
        self.beta = beta
        self.relu = bool(relu)
        self.owner = owner    # the BatchNormLayer (its backward can take partial sums, see below)
        self._y = None
        self.gen = getattr(owner, "_dk_gen", 0)  # the owner's forward this record belongs to

    def _check_current(self):
        if self.owner is not None and getattr(self.owner, "_dk_gen", 0) != self.gen:
            raise RuntimeError("BNOut of {} used after that layer's next forward: its mean / invstd buffers "
                               "now hold the newer batch's statistics".format(self.owner.layer_name))

    @property
    def shape(self):
        return self.x.shape

    def dim(self):
        return self.x.dim()

    @property
    def device(self):
        return self.x.device

    @property
    def dtype(self):
        return self.x.dtype

    def bn_args(self):
        """(mean, invstd, gamma, beta, relu) for a dk_*_bnx_f32 call."""
        self._check_current()
        return (self.mean.data_ptr(), self.invstd.data_ptr(), self.gamma.data_ptr(), self.beta.data_ptr(),
                int(self.relu))

    def arm_partials(self, part):
        """Before a consumer's backward launch that writes stage 1 of this BatchNorm's backward
        into `part`: arm an in-launch fold (dorknet_amd/csrc/fold_tail.h), so that the launch
        also finalizes dgamma / dbeta / k12.  Returns a token for hand_backward_partials."""
        if self.owner is None or not inlaunch_folds_enabled():
            return None
        return self.owner.arm_bwd_fold(part)

    def hand_backward_partials(self, dx, part, status=0, token=None):
        """A consumer's backward computed stage 1 of this BatchNorm's backward (the
        *_dgrad_ex_f32 epilogue) while producing `dx`, the gradient w.r.t. this BNOut;
        `status` / `token`: the launch's return value and arm_partials' token."""
        folded = None
        if token is not None:
            if status == DK_FOLDED:
                folded = token
            else:
                lib.dk_bn_fold_disarm()
        if self.owner is not None:
            self.owner._pending_bwd = (dx, part, folded)

    def materialize(self):
        """The normalised tensor itself (computed once)."""
        if self._y is None:
            self._check_current()
            x = self.x
            y = empty_nhwc(*x.shape, dtype=x.dtype) if x.dim() == 4 else torch.empty_like(x)
            apply = lib.dk_bn_apply_bf16 if x.dtype == torch.bfloat16 else lib.dk_bn_apply_f32
            apply(x.data_ptr(), x.numel(), x.shape[1], self.mean.data_ptr(), self.invstd.data_ptr(),
                  self.gamma.data_ptr(), self.beta.data_ptr(), int(self.relu), y.data_ptr(), 0, stream_handle())
            self._y = y
        return self._y


class JoinOut:
    """A residual block's output y = ReLU(bnA(a) + bnB(b)) (residual_block.py:75) not yet written.

    The join pass (dk_bn_add_f32) writes y and the next block's first depthwise layer reads it back
    at once.  When that layer can take it (DepthwiseConvLayer.takes_join_input), the block hands over
    this record instead: the layer forms y as it loads its input window and stores it once
    (dk_dwconv_fwd_join_f32, bit-identical to the join pass), so y is written but not re-read.  `y`
    and `mask` are allocated here; ``materialize()`` runs the join pass for any other consumer.
    The closing ReLu's backward state is set when y is written (ReLu._join_written), the same state
    the join pass leaves."""
    __slots__ = ("A", "B", "relu_layer", "test_mode", "y", "mask", "written")

    def __init__(self, A, B, relu_layer, test_mode, need_mask=True):
        """need_mask: also store the join's ReLU mask (uint8).  A stride-1 consumer's fused backward
        takes the mask as y > 0 (DepthwiseConvLayer._join_ok, from_y) and does not need it."""
        self.A = A            # BNOut or NHWC tensor (the chain's output)
        self.B = B            # BNOut or NHWC tensor (the skip operand)
        self.relu_layer = relu_layer
        self.test_mode = test_mode
        x = A.x if isinstance(A, BNOut) else A
        self.y = empty_nhwc(*x.shape)
        self.mask = None if (test_mode or not need_mask) else torch.empty(
            x.shape, dtype=torch.uint8, device=x.device, memory_format=torch.channels_last)
        self.written = False

    def _like(self):
        return self.A.x if isinstance(self.A, BNOut) else self.A

    @property
    def shape(self):
        return self._like().shape

    def dim(self):
        return self._like().dim()

    @property
    def device(self):
        return self._like().device

    @property
    def dtype(self):
        return self._like().dtype

    @staticmethod
    def _operand(T):
        if isinstance(T, BNOut):
            return (T.x.data_ptr(), *T.bn_args())
        return (T.data_ptr(), 0, 0, 0, 0, 0)

    def join_args(self):
        """(a, a_mean, a_invstd, a_gamma, a_beta, a_relu, b, b_mean, ..., b_relu, y, mask) for
        dk_dwconv_fwd_join_f32 / dk_bn_add_f32."""
        return (*self._operand(self.A), *self._operand(self.B), self.y.data_ptr(),
                0 if self.mask is None else self.mask.data_ptr())

    def mark_written(self):
        self.written = True
        self.relu_layer._join_written(self)

    def mark_pooled(self):
        """The consumer pooled the join as it formed it (dk_gap_join_fwd_f32): y was never stored
        (only the mask), so it is dropped here and materialize() refuses."""
        self.y = None
        self.mark_written()

    def materialize(self):
        """y itself: the join pass (dk_bn_add_f32) unless a consumer already wrote it."""
        if self.written and self.y is None:
            raise RuntimeError("the residual join was pooled as it was formed (mark_pooled): y was never stored")
        if not self.written:
            a = self._operand(self.A)
            b = self._operand(self.B)
            y = self.y
            lib.dk_bn_add_f32(*a, *b, y.numel(), y.shape[1], 1, y.data_ptr(),
                              0 if self.mask is None else self.mask.data_ptr(), stream_handle())
            self.mark_written()
        return self.y


class BNGrad:
    """The gradient w.r.t. a BatchNormLayer's input with its last stage (the per-element
    apply, dk_bn_bwd_apply_f32) left to the producer of that input.

    BatchNormLayer._backward(defer=True) reduces its partial sums into k12 and returns this
    instead of writing dx; a producer with ``accepts_bn_grad`` forms dx = f(g, x) as its dgrad
    loads it (the *_dgrad_bnbwd_f32 entries) and stores it once for its weight gradient.
    ``materialize()`` is the unfused apply (bit-identical)."""
    __slots__ = ("_g", "x", "mean", "invstd", "gamma", "beta", "relu", "k12", "_dx", "lattice")

    def __init__(self, g, x, mean, invstd, gamma, beta, relu, k12, lattice=1):
        self._g = g           # gradient w.r.t. the BN (+ReLU) output, NHWC like x
        self.lattice = int(lattice)  # > 1: _g holds only the stride-`lattice` lattice, compact (see g_compact)
        self.x = x            # the BN's raw input
        self.mean = mean
        self.invstd = invstd
        self.gamma = gamma
        self.beta = beta
        self.relu = bool(relu)
        self.k12 = k12        # [k1[C], k2[C]] from dk_bn_bwd_from_partials_f32 / _finalize_f32
        self._dx = None

    @property
    def shape(self):
        return self.x.shape

    def dim(self):
        return self.x.dim()

    @property
    def dtype(self):
        return self.x.dtype

    @property
    def g(self):
        """The dense gradient (a lattice gradient is widened here: zeros off the lattice)."""
        if self.lattice > 1:
            self._g, self.lattice = widen_lattice(self._g, self.lattice, self.x.shape), 1
        return self._g

    @property
    def g_compact(self):
        """The gradient as held: with lattice > 1, [N][C][ceil(H/s)][ceil(W/s)] (NHWC)."""
        return self._g

    def bnbwd_args(self):
        """(mean, invstd, gamma, beta, relu, k12) for a *_dgrad_bnbwd_f32 call."""
        return (self.mean.data_ptr(), self.invstd.data_ptr(), self.gamma.data_ptr(), self.beta.data_ptr(),
                int(self.relu), self.k12.data_ptr())

    def materialize(self):
        if self._dx is None:
            x = self.x
            dx = empty_nhwc(*x.shape, dtype=x.dtype) if x.dim() == 4 else torch.empty_like(x)
            apply = lib.dk_bn_bwd_apply_bf16 if x.dtype == torch.bfloat16 else lib.dk_bn_bwd_apply_f32
            apply(x.data_ptr(), self.g.data_ptr(), x.numel(), x.shape[1], *self.bnbwd_args()[:5],
                  self.k12.data_ptr(), dx.data_ptr(), stream_handle())
            self._dx = dx
        return self._dx


def widen_lattice(g, s, shape):
    """Layout plumbing for a consumer that needs the dense gradient: the stride-s lattice gradient
    `g` placed on a zero grid of `shape` (what the reference's widen builds,
    pointwise_convolution.py:68-72)."""
    out = empty_nhwc(*shape, dtype=g.dtype)
    out.zero_()
    out[:, :, ::s, ::s] = g
    return out


def lattice_tag(t) -> int:
    """The stride s of a gradient handed over as its compact stride-s lattice (0: dense)."""
    return int(getattr(t, "_dk_lattice", 0) or 0) if isinstance(t, torch.Tensor) else 0


def dense_residual(residual, shape):
    """`residual` on the dense grid `shape` (N, C, H, W): a lattice-tagged gradient is widened."""
    s = lattice_tag(residual)
    return widen_lattice(residual, s, tuple(shape)) if s else residual


def lattice_operand(residual, like, s):
    """`residual` as the compact stride-s lattice operand for a dgrad shaped like `like` (the
    skip projection's un-widened input gradient: [N][ceil(H/s)][ceil(W/s)][C] NHWC), or None."""
    if lattice_tag(residual) != s or s < 2:
        return None
    N, C, H, W = like.shape
    r = residual
    if (r.is_cuda and r.dtype == like.dtype and r.dim() == 4 and is_nhwc(r)
            and tuple(r.shape) == (N, C, -(-H // s), -(-W // s))):
        return r
    return None


def accepts_bn_grad(layer, bn_layer) -> bool:
    f = getattr(layer, "accepts_bn_grad", None)
    return bool(f(bn_layer)) if f is not None else False


def materialize(X):
    return X.materialize() if isinstance(X, (BNOut, BNGrad, JoinOut)) else X


def accepts_bn_input(layer) -> bool:
    return bool(getattr(layer, "accepts_bn_input", False))


def residual_operand(residual, like):
    """`residual` as an NHWC device tensor shaped like `like` (for a fused residual addend),
    or None when there is none or it cannot be fused."""
    if residual is None:
        return None
    r = residual
    if isinstance(r, torch.Tensor) and r.is_cuda and r.dtype == like.dtype and tuple(r.shape) == tuple(
            like.shape) and r.dim() == 4 and is_nhwc(r):
        return r
    return None


def add_residual(dx, residual):
    """dx + residual (the unfused residual join, residual_block.py:94-97)."""
    a = to_nhwc(dx)
    b = to_nhwc(dense_residual(residual, a.shape))
    if a.shape != b.shape:
        raise ValueError("residual backward shape mismatch: {} vs {}".format(tuple(a.shape), tuple(b.shape)))
    out = empty_nhwc(*a.shape)
    lib.dk_add_f32(a.data_ptr(), b.data_ptr(), a.numel(), 0, out.data_ptr(), 0, stream_handle())
    return out
