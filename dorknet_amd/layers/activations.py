"""ReLU (reference: layers/activations.py).

``out = max(0, X)``; the backward mask is ``out > 0`` (gradient 0 at 0, :41).  The mask
is kept as uint8 (the reference stores an fp32 copy, :42); ``positive_locs`` still
returns the fp32 mask on request.  When the layer directly follows a BatchNormLayer in a
network or residual chain, the two run fused (BatchNormLayer.forward_bn_relu) and this
layer only records its output.
"""
from __future__ import annotations

import torch

from .._hip import lib, stream_handle
from .._tensor import act_dtype, as_device, empty_nhwc, is_nhwc as is_nhwc_t, rows, to_nhwc
from ._bn_input import BNOut, JoinOut
from .layer import Layer


def _same_layout(X):
    X = as_device(X, act_dtype(X))
    return to_nhwc(X) if X.dim() == 4 else rows(X)


class ReLu(Layer):

    def __init__(self, layer_name):
        super().__init__(layer_name)
        self._mask = None
        self._fused_out = None
        self._join_bn = None
        self._join_done = False
        self._join_y_ptr = None  # data_ptr of the fused join's output (_bn_add)
        self._join_y = None      # that output, when the join left no mask (JoinOut without one)

    def join_backward_done(self):
        """The consumer of this residual join's output applied this ReLU's backward (and stage 1
        of the join BatchNorm's) in its own dgrad epilogue (DepthwiseConvLayer, accepts_join):
        the gradient it returned is already dx, so backward() passes it through."""
        self._join_done = True

    def __repr__(self):
        return "ReLu({})".format(self.layer_name)

    def _empty_like(self, x):
        return empty_nhwc(*x.shape, dtype=x.dtype) if x.dim() == 4 else torch.empty_like(x)

    def forward(self, X, test_mode=False):
        self._require_on_gpu()
        st = stream_handle()
        x = _same_layout(X)
        y = self._empty_like(x)
        mask = None
        if not test_mode:
            mask = torch.empty(x.shape, dtype=torch.uint8, device=x.device,
                               memory_format=torch.channels_last if x.dim() == 4 else torch.contiguous_format)
        fwd = lib.dk_relu_fwd_bf16 if x.dtype == torch.bfloat16 else lib.dk_relu_fwd_f32
        fwd(x.data_ptr(), x.numel(), y.data_ptr(), 0 if mask is None else mask.data_ptr(), st)
        if not test_mode:
            self._mask, self._fused_out, self._join_bn = mask, None, None
            self._join_done = False
            self._join_y = None
        return y

    def forward_add(self, A, B, test_mode=False, defer=False, need_mask=True):
        """ReLU(A + B) in one pass -- the residual join (residual_block.py:75).  A and/or B may
        be a BatchNorm output not yet written (BNOut): the normalisation is applied on load.
        defer: the consumer of the result can form it on load (ResidualBlock.takes_join_input):
        return a JoinOut (layers/_bn_input.py) instead of running the join pass."""
        self._require_on_gpu()
        st = stream_handle()
        if isinstance(A, JoinOut):
            A = A.materialize()
        if isinstance(B, JoinOut):
            B = B.materialize()
        if defer and (isinstance(A, BNOut) or isinstance(B, BNOut)) and self._join_parts_ok(A, B):
            return JoinOut(A, B, self, test_mode, need_mask)
        if isinstance(A, BNOut) or isinstance(B, BNOut):
            y = self._bn_add(A, B, test_mode, st)
            if y is not None:
                return y
        a, b = _same_layout(A), _same_layout(B)
        if a.shape != b.shape:
            raise ValueError("residual join shape mismatch: {} vs {}".format(tuple(a.shape), tuple(b.shape)))
        y = self._empty_like(a)
        mask = None
        if not test_mode:
            mask = torch.empty(a.shape, dtype=torch.uint8, device=a.device,
                               memory_format=torch.channels_last if a.dim() == 4 else torch.contiguous_format)
        lib.dk_add_f32(a.data_ptr(), b.data_ptr(), a.numel(), 1, y.data_ptr(),
                       0 if mask is None else mask.data_ptr(), st)
        if not test_mode:
            self._mask, self._fused_out, self._join_bn = mask, None, None
            self._join_y = None
        return y

    @staticmethod
    def _join_parts_ok(A, B):
        if A.dim() != 4 or tuple(A.shape) != tuple(B.shape) or A.shape[1] % 4 or A.dtype != torch.float32:
            return False
        xs = [T.x if isinstance(T, BNOut) else T for T in (A, B)]
        return all(isinstance(x, torch.Tensor) and x.dtype == torch.float32 and is_nhwc_t(x) for x in xs)

    def _join_written(self, jo):
        """The join output of a JoinOut was written (by its consumer, or by its materialize):
        the backward state the join pass leaves (_bn_add)."""
        if not jo.test_mode:
            self._mask, self._fused_out = jo.mask, None
            self._join_bn = jo.A if isinstance(jo.A, BNOut) else None
            self._join_done = False
            self._join_y_ptr = None if jo.y is None else jo.y.data_ptr()  # (None: pooled, mark_pooled)
            self._join_y = jo.y if jo.mask is None else None

    def _bn_add(self, A, B, test_mode, st):
        def parts(T):
            if isinstance(T, BNOut):
                return T.x, T.bn_args()
            return to_nhwc(T), (0, 0, 0, 0, 0)
        if A.dim() != 4 or tuple(A.shape) != tuple(B.shape) or A.shape[1] % 4:
            return None
        (a, pa), (b, pb) = parts(A), parts(B)
        if not (is_nhwc_t(a) and is_nhwc_t(b)):
            return None
        y = empty_nhwc(*a.shape)
        mask = None
        if not test_mode:
            mask = torch.empty(a.shape, dtype=torch.uint8, device=a.device, memory_format=torch.channels_last)
        lib.dk_bn_add_f32(a.data_ptr(), *pa, b.data_ptr(), *pb, a.numel(), a.shape[1], 1, y.data_ptr(),
                          0 if mask is None else mask.data_ptr(), st)
        if not test_mode:
            self._mask, self._fused_out = mask, None
            self._join_bn = A if isinstance(A, BNOut) else None
            self._join_done = False
            self._join_y_ptr = y.data_ptr()  # a consumer holding y itself may take the mask as y > 0
            self._join_y = None
        return y

    def _attach_fused(self, y, test_mode):
        if not test_mode:
            self._mask, self._fused_out, self._join_bn = None, y, None
            self._join_y = None

    def _mask_from_join(self):
        """The join's ReLU mask from its stored output (y > 0), for a backward that needs the mask
        when the join left none (a JoinOut whose consumer takes it as y > 0)."""
        y = self._join_y
        mask = torch.empty(y.shape, dtype=torch.uint8, device=y.device, memory_format=torch.channels_last)
        lib.dk_relu_fwd_f32(y.data_ptr(), y.numel(), 0, mask.data_ptr(), stream_handle())  # mask-only pass
        self._mask, self._join_y = mask, None
        return mask

    @property
    def positive_locs(self):
        """fp32 mask (out > 0), as the reference's attribute (activations.py:42)."""
        if self._mask is None and self._join_y is not None:
            self._mask_from_join()
        if self._mask is not None:
            out = torch.empty(self._mask.shape, dtype=torch.float32, device=self._mask.device,
                              memory_format=torch.channels_last if self._mask.dim() == 4 else torch.contiguous_format)
            lib.dk_mask_to_f32(self._mask.data_ptr(), self._mask.numel(), out.data_ptr(), stream_handle())
            return out
        if self._fused_out is not None:
            y = as_device(self._fused_out)  # a BNOut is materialised here
            mask = torch.empty(y.shape, dtype=torch.uint8, device=y.device,
                               memory_format=torch.channels_last if y.dim() == 4 else torch.contiguous_format)
            lib.dk_relu_fwd_f32(y.data_ptr(), y.numel(), 0, mask.data_ptr(), stream_handle())  # mask-only pass
            out = self._empty_like(y)
            lib.dk_mask_to_f32(mask.data_ptr(), mask.numel(), out.data_ptr(), stream_handle())
            return out
        return None

    def backward(self, upstream_dx):
        self._require_on_gpu()
        if self._join_done:
            self._join_done = False
            return upstream_dx
        if self._mask is None and self._join_y is not None:
            self._mask_from_join()
        if self._mask is None:
            raise RuntimeError("ReLu {}: backward without a training-mode forward (or the layer ran fused with "
                               "the preceding BatchNormLayer; its backward is BatchNormLayer.backward_bn_relu)"
                               .format(self.layer_name))
        dy = _same_layout(upstream_dx)
        dx = self._empty_like(dy)
        bn = getattr(self, "_join_bn", None)
        if bn is not None and tuple(bn.x.shape) == tuple(dy.shape) and is_nhwc_t(dy):
            # the join's BN input: its backward stage 1 rides on this pass (residual_block.py:85-86)
            C = dy.shape[1]
            P = dy.numel() // C
            nb = lib.dk_bn_workspace_bytes(P, C)
            part = torch.empty((lib.dk_bn_partial_blocks(P, C), 2, C), dtype=torch.float64, device=dy.device)
            tok = bn.arm_partials(part)
            r = lib.dk_relu_bwd_bn_partial_f64(dy.data_ptr(), self._mask.data_ptr(), bn.x.data_ptr(), P, C,
                                               *bn.bn_args(), dx.data_ptr(), part.data_ptr(), nb, stream_handle())
            bn.hand_backward_partials(dx, part, r, tok)
            return dx
        bwd = lib.dk_relu_bwd_bf16 if dy.dtype == torch.bfloat16 else lib.dk_relu_bwd_f32
        bwd(dy.data_ptr(), self._mask.data_ptr(), dy.numel(), dx.data_ptr(), stream_handle())
        return dx

    def save_to_h5(self, open_f, save_grads=True):
        from ..network.checkpoint import save_layer
        save_layer(self, open_f, save_grads)

    def load_from_h5(self, open_f, load_grads=True):
        pass
