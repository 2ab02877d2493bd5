"""Depthwise (per-channel) convolution (reference: layers/depthwise_convolution.py).

The reference GPU path (forward_cp :85-102, backward_cp :198-221) pads the input into a
copy, runs one thread per output with nine global read-modify-writes, and in backward
funnels N*OH*OW atomicAdds into each weight.  Here: direct NHWC kernels with register
accumulation, bounds checks instead of a padded copy, and a two-stage deterministic
weight-gradient reduction (dk_dwconv_fwd_f32 / _dgrad_f32 / _wgrad_f32).

Public surface identical to the reference: constructor (:11-13), weights (C, R, S),
bias (C,), ``forward`` / ``backward`` / ``__repr__`` (:41-51).
"""
from __future__ import annotations


import torch

from .._env import getenv
from .._hip import HipError, deferred_wgrad_reduce, lib, stream_handle, weight_grad_stream, workspace
from .._tensor import BF16, empty_nhwc, ptr, to_nhwc
from ._bn_input import BNGrad, BNOut, JoinOut, add_residual, dense_residual, lattice_operand, residual_operand
from ._common import add_regulariser_grad, grad_buffer, init_weights, l2_strength
from .layer import Layer


class DepthwiseConvLayer(Layer):
    def __init__(self, layer_name, filter_block_shape=None,
                 stride=1, padding=1, with_bias=True,
                 weight_regulariser=None, weight_initialiser="normal"):
        """
        filter_block_shape = (num_incoming_channels, num_filter_rows, num_filter_cols)
        """
        super().__init__(layer_name)
        self.stride = stride
        self.padding = padding
        self.with_bias = with_bias
        self.weight_regulariser = weight_regulariser
        self.weight_initialiser = weight_initialiser
        if filter_block_shape is not None:
            self.num_filters, self.f_rows, self.f_cols = filter_block_shape
            weights = init_weights(tuple(filter_block_shape), weight_initialiser, 2 * self.num_filters)
            self.learned_params = {"weights": weights}
            self.grads = {"weights": weights * 0}
            if with_bias:
                bias = (weights[:, 0, 0] * 0).copy()
                self.learned_params["bias"] = bias
                self.grads["bias"] = bias * 0
        else:
            self.num_filters = None
            self.learned_params = {}
            self.grads = {}

    def __repr__(self):
        out = "DepthwiseConvLayer({}, ".format(self.layer_name)
        if self.num_filters is not None:
            out += "filter_block_shape=({}, {}, {}), ".format(self.num_filters, self.f_rows, self.f_cols)
        out += "stride={}, padding={}, with_bias={}, weight_regulariser={})".format(
            self.stride, self.padding, self.with_bias, repr(self.weight_regulariser))
        return out

    def _w_rsc(self, st):
        w = self.learned_params["weights"]
        C, R, S = w.shape
        w_rsc = torch.empty((R, S, C), dtype=torch.float32, device=w.device)
        lib.dk_dw_weight_rsc_f32(w.data_ptr(), C, R, S, w_rsc.data_ptr(), st)
        return w_rsc

    accepts_bn_input = True   # forward(BNOut): the preceding BatchNorm is applied on load
    produces_bn_stats = True  # forward(..., bn_stats=StatsRequest): emits the next BN's statistics

    def join_geometry_ok(self):
        """forward(JoinOut) can form the residual join on load (dk_dwconv_fwd_join_f32): 3 x 3, pad
        1, stride 1 or 2, no bias (the shapes and dtype are checked at the call)."""
        return (self.num_filters is not None and self.f_rows == 3 and self.f_cols == 3 and self.padding == 1
                and self.stride in (1, 2) and not self.with_bias)

    def _takes_join(self, X):
        return (self.join_geometry_ok() and X.dim() == 4 and X.dtype == torch.float32
                and X.shape[1] == self.num_filters and X.shape[1] % 4 == 0 and X.shape[1] <= 512)

    def forward(self, X, test_mode=False, bn_stats=None):
        self._require_on_gpu()
        st = stream_handle()
        if isinstance(X, JoinOut):
            if not X.written and self._takes_join(X):
                return self._forward_join(X, test_mode, bn_stats, st)
            X = X.materialize()
        bn = X if isinstance(X, BNOut) and X.dim() == 4 and X.shape[1] % 4 == 0 else None
        x = bn.x if bn is not None else to_nhwc(X)
        N, C, H, W = x.shape
        R, S = self.f_rows, self.f_cols
        # float-then-int output size (depthwise_convolution.py:89-90)
        self.num_row_patches = ((H + 2 * self.padding - R) / self.stride) + 1
        self.num_col_patches = ((W + 2 * self.padding - S) / self.stride) + 1
        OH, OW = int(self.num_row_patches), int(self.num_col_patches)
        bf = x.dtype == BF16  # bf16 storage (BASELINE config 5): the _bf16 entry points
        y = empty_nhwc(N, C, OH, OW, x.dtype)
        bias = self.learned_params["bias"] if self.with_bias else None
        stats = None
        if bn_stats is not None and not test_mode and self.stride in (1, 2):
            rows = (lib.dk_dwconv_fwd_bf16_stats_rows if bf else lib.dk_dwconv_fwd_stats_rows)(N, OH, OW, C, self.stride)
            if rows:
                stats = torch.empty((rows, 2, C), dtype=torch.float64, device=x.device)
        w = self.learned_params["weights"]  # W[C][R][S], read in place by the _ex entry
        fwd = lib.dk_dwconv_fwd_ex_bf16 if bf else lib.dk_dwconv_fwd_ex_f32
        if stats is not None:
            bn_stats.arm(stats, N * OH * OW)
        r = fwd(x.data_ptr(), N, H, W, C, w.data_ptr(), R, S, self.stride, self.padding, ptr(bias), y.data_ptr(), OH,
                OW, *(bn.bn_args() if bn is not None else (0, 0, 0, 0, 0)), ptr(stats), st)
        if stats is not None:
            bn_stats.launched(stats, r)
        if not test_mode:
            # the reference keeps the *padded* input (:87-88); padding is implicit here, and
            # a BNOut input is kept as the BatchNorm's raw input + parameters
            self.X = x
            self._bn_in = bn
        return y

    def _forward_join(self, J, test_mode, bn_stats, st):
        """forward on a residual block's output not yet written (JoinOut): the join is formed as the
        input window is loaded and stored once (dk_dwconv_fwd_join_f32); the layer then holds y as
        its input, exactly as after the join pass."""
        N, C, H, W = J.shape
        R, S = self.f_rows, self.f_cols
        self.num_row_patches = ((H + 2 * self.padding - R) / self.stride) + 1
        self.num_col_patches = ((W + 2 * self.padding - S) / self.stride) + 1
        OH, OW = int(self.num_row_patches), int(self.num_col_patches)
        y = empty_nhwc(N, C, OH, OW)
        stats = None
        if bn_stats is not None and not test_mode:
            rows = lib.dk_dwconv_fwd_stats_rows(N, OH, OW, C, self.stride)
            if rows:
                stats = torch.empty((rows, 2, C), dtype=torch.float64, device=J.device)
        if stats is not None:
            bn_stats.arm(stats, N * OH * OW)
        r = lib.dk_dwconv_fwd_join_f32(*J.join_args(), N, H, W, C, self.learned_params["weights"].data_ptr(),
                                       self.stride, 0, y.data_ptr(), OH, OW, ptr(stats), st)
        if stats is not None:
            bn_stats.launched(stats, r)
        J.mark_written()
        if not test_mode:
            self.X = J.y
            self._bn_in = None
        return y

    accepts_residual = True  # backward(dy, residual=R) returns dx + R (the residual join, fused)

    skips_input_grad = True  # backward(dy, need_dx=False): parameter gradients only (chain_backward)

    def accepts_bn_grad(self, bn_layer):
        """backward(BNGrad): the following BatchNorm's apply, this layer's dgrad and its weight
        gradient run as one pass -- 3x3, padding 1, no bias, C % 4 == 0: stride 1
        (dk_dwconv_bwd_bnbwd_f32 / _bf16) and stride 2 (dk_dwconv_bwd_s2_bnbwd_f32 / _bf16, C / 4
        dividing 256; DORKNET_DW_S2_FUSED=0 turns it off)."""
        bx = getattr(bn_layer, "X", None)
        return getattr(self, "X", None) is not None and bx is not None and self._takes_bn_grad(bx)

    def _takes_bn_grad(self, bx):
        x = self.X
        if x.dim() != 4 or bx.dim() != 4 or x.dtype not in (torch.float32, BF16) or bx.dtype != x.dtype:
            return False
        N, C, H, W = x.shape
        if not (self.f_rows == 3 and self.f_cols == 3 and self.padding == 1 and not self.with_bias and C % 4 == 0):
            return False
        if self.stride == 2:
            return (getenv("DORKNET_DW_S2_FUSED", "1") != "0" and 256 % (C // 4) == 0
                    and tuple(bx.shape) == (N, C, (H + 1) // 2, (W + 1) // 2))
        return self.stride == 1 and tuple(bx.shape) == tuple(x.shape)

    accepts_join = True  # backward(BNGrad, residual=R, join=relu): the input's residual join rides on dx

    def _join_ok(self, join, need_dx):
        """`join`: the ReLu that closed the residual block whose output is this layer's input
        (residual_block.py:75).  The fused backward takes over its backward and stage 1 of its
        BatchNorm's (dk_dwconv_bwd_bnbwd_join_f32) when this layer has no input BatchNorm."""
        x = self.X
        jb = getattr(join, "_join_bn", None)
        mask = getattr(join, "_mask", None)
        if not (need_dx and self._bn_in is None and jb is not None and tuple(jb.x.shape) == tuple(x.shape)
                and jb.x.dtype == torch.float32 and jb.x.is_contiguous(memory_format=torch.channels_last)):
            return False
        if mask is None:
            # a join that left no mask (JoinOut): the fused backwards take it as x > 0 (x is the
            # join's output); the plain join dgrad rebuilds it (ReLu._mask_from_join)
            return (getattr(join, "_join_y", None) is not None
                    and getattr(join, "_join_y_ptr", None) == x.data_ptr())
        return tuple(mask.shape) == tuple(x.shape) and mask.is_contiguous(memory_format=torch.channels_last)

    def takes_lattice_residual(self, join, s):
        """backward(dy, residual=R, join=relu) adds R given as the compact stride-s lattice (a
        strided pointwise skip projection's un-widened input gradient) in the fused join dgrad
        (dk_dwconv_dgrad_join_f32, residual_lattice = s): fp32, this layer's stride is s, and the
        join fuses.  Any other path widens such a residual first (dense_residual)."""
        x = getattr(self, "X", None)
        if (x is None or x.dim() != 4 or x.dtype != torch.float32 or self.stride != s or s < 2 or join is None
                or self.with_bias or not self._join_ok(join, True)):
            return False
        N, C, H, W = x.shape
        return lib.dk_dwconv_dgrad_join_rows(N, H, W, C, self.f_rows, self.f_cols, s, self.padding) > 0

    def _backward_bn_grad(self, G, residual, need_dx, join=None):
        """One-pass backward from the following BatchNorm's deferred gradient (see
        accepts_bn_grad): dx (+ the residual addend, + the input BatchNorm's backward partial
        sums, or the input's residual join: see _join_ok) and the weight gradient; dy itself is
        never written."""
        st = stream_handle()
        x = self.X
        N, C, H, W = x.shape
        R, S = self.f_rows, self.f_cols
        w = self.learned_params["weights"]
        gw = grad_buffer(self, "weights", (C, R, S))
        s = l2_strength(self.weight_regulariser)
        bn = self._bn_in
        dx = empty_nhwc(N, C, H, W, x.dtype) if need_dx else None
        if self.stride == 2:
            return self._backward_bn_grad_s2(G, residual, need_dx, dx, gw, s, w, join)
        if residual is not None:
            residual = dense_residual(residual, (N, C, H, W))
        res = residual_operand(residual, dx) if need_dx else None
        if need_dx and residual is not None and res is None:
            res = residual_operand(to_nhwc(residual), dx)
        if join is not None and self._join_ok(join, need_dx):
            jb = join._join_bn
            rows = lib.dk_dwconv_bwd_bnbwd_stats_rows(N, H, W, C)
            part = torch.empty((rows, 2, C), dtype=torch.float64, device=x.device)
            g = to_nhwc(G.g)
            nb = lib.dk_dwconv_bwd_bnbwd_workspace_bytes(N, H, W, C, R, S)
            # x IS the join's output: the kernel takes the mask as x > 0 instead of reading it
            # (DORKNET_JOIN_MASK=1 reads the stored mask)
            from_y = getattr(join, "_join_y_ptr", None) == x.data_ptr() and getenv("DORKNET_JOIN_MASK") != "1"
            if not from_y and join._mask is None:
                join._mask_from_join()
            tok = jb.arm_partials(part)
            # the weight-gradient reduce on the side stream (not with a non-l2 regulariser, whose
            # term is added to gw on this stream right after)
            red = deferred_wgrad_reduce(self, nb, s is not None)
            with red:
                r = lib.dk_dwconv_bwd_bnbwd_join_f32(g.data_ptr(), G.x.data_ptr(), N, H, W, C, *G.bnbwd_args(),
                                                     x.data_ptr(), w.data_ptr(), R, S, self.padding, s or 0.0,
                                                     gw.data_ptr(), dx.data_ptr(), ptr(res),
                                                     0 if from_y else join._mask.data_ptr(),
                                                     jb.x.data_ptr(), jb.mean.data_ptr(), jb.invstd.data_ptr(),
                                                     part.data_ptr(), red.ws, nb, st)
            red.flush()
            if s is None:
                add_regulariser_grad(gw, w, self.weight_regulariser)
            jb.hand_backward_partials(dx, part, r, tok)
            join.join_backward_done()
            if residual is not None and res is None:
                raise RuntimeError("{}: the fused join needs the residual in the dgrad epilogue".format(
                    self.layer_name))
            return dx
        part = None
        bf = x.dtype == BF16
        if need_dx and bn is not None:
            rows = (lib.dk_dwconv_bwd_bnbwd_bf16_stats_rows if bf else lib.dk_dwconv_bwd_bnbwd_stats_rows)(N, H, W, C)
            part = torch.empty((rows, 2, C), dtype=torch.float64, device=x.device)
        g = to_nhwc(G.g)
        nb = (lib.dk_dwconv_bwd_bnbwd_bf16_workspace_bytes if bf else lib.dk_dwconv_bwd_bnbwd_workspace_bytes)(
            N, H, W, C, R, S)
        tok = bn.arm_partials(part) if part is not None else None
        red = deferred_wgrad_reduce(self, nb, s is not None)
        with red:
            r = (lib.dk_dwconv_bwd_bnbwd_bf16 if bf else lib.dk_dwconv_bwd_bnbwd_f32)(
                g.data_ptr(), G.x.data_ptr(), N, H, W, C, *G.bnbwd_args(), x.data_ptr(), w.data_ptr(), R, S,
                self.padding, s or 0.0, gw.data_ptr(), ptr(dx), ptr(res),
                *(bn.bn_args() if bn is not None else (0, 0, 0, 0, 0)), ptr(part), red.ws, nb, st)
        red.flush()
        if s is None:
            add_regulariser_grad(gw, w, self.weight_regulariser)
        if not need_dx:
            return None
        if part is not None:
            bn.hand_backward_partials(dx, part, r, tok)
        if residual is not None and res is None:
            dx = add_residual(dx, residual)  # (a new tensor: the BN then recomputes its sums)
        return dx

    def _backward_bn_grad_s2(self, G, residual, need_dx, dx, gw, s, w, join=None):
        """The stride-2 form of _backward_bn_grad (dk_dwconv_bwd_s2_bnbwd_*): dx (+ the residual,
        + the input BatchNorm's backward partial sums) and the weight gradient, dy never written.
        With the input's residual join (fp32, _join_ok): dk_dwconv_bwd_s2_bnbwd_join_f32 -- dx
        masked by y > 0 (y = this layer's input, the join's output), stage 1 of the join's
        BatchNorm on the store, a strided skip's compact lattice residual added as such."""
        st = stream_handle()
        x = self.X
        N, C, H, W = x.shape
        OH, OW = (H + 1) // 2, (W + 1) // 2
        bn = self._bn_in
        bf = x.dtype == BF16
        if join is not None and need_dx and not bf and self._join_ok(join, True):
            return self._backward_bn_grad_s2_join(G, residual, dx, gw, s, w, join)
        if residual is not None:
            residual = dense_residual(residual, (N, C, H, W))
        res = residual_operand(residual, dx) if need_dx else None
        if need_dx and residual is not None and res is None:
            res = residual_operand(to_nhwc(residual), dx)
        if need_dx and residual is not None and res is None:
            raise NotImplementedError("{}: the fused stride-2 backward needs an NHWC residual".format(self.layer_name))
        part = None
        if need_dx and bn is not None:
            part = torch.empty((lib.dk_dwconv_bwd_s2_stats_rows(N, H, W, C), 2, C), dtype=torch.float64,
                               device=x.device)
        g = to_nhwc(G.g)
        nb = lib.dk_dwconv_bwd_s2_workspace_bytes(N, H, W, C)
        tok = bn.arm_partials(part) if part is not None else None
        red = deferred_wgrad_reduce(self, nb, s is not None)
        with red:
            r = (lib.dk_dwconv_bwd_s2_bnbwd_bf16 if bf else lib.dk_dwconv_bwd_s2_bnbwd_f32)(
                g.data_ptr(), G.x.data_ptr(), N, H, W, C, OH, OW, *G.bnbwd_args(), x.data_ptr(), w.data_ptr(),
                s or 0.0, gw.data_ptr(), ptr(dx), ptr(res),
                *(bn.bn_args() if bn is not None else (0, 0, 0, 0, 0)), ptr(part), red.ws, nb, st)
        red.flush()
        if s is None:
            add_regulariser_grad(gw, w, self.weight_regulariser)
        if not need_dx:
            return None
        if part is not None:
            bn.hand_backward_partials(dx, part, r, tok)
        return dx

    def _backward_bn_grad_s2_join(self, G, residual, dx, gw, s, w, join):
        st = stream_handle()
        x = self.X
        N, C, H, W = x.shape
        OH, OW = (H + 1) // 2, (W + 1) // 2
        jb = join._join_bn
        lat = lattice_operand(residual, dx, 2)
        if lat is None and residual is not None:
            residual = dense_residual(residual, (N, C, H, W))
        res = lat if lat is not None else residual_operand(residual, dx)
        if residual is not None and res is None:
            res = residual_operand(to_nhwc(residual), dx)
        part = torch.empty((lib.dk_dwconv_bwd_s2_stats_rows(N, H, W, C), 2, C), dtype=torch.float64, device=x.device)
        g = to_nhwc(G.g)
        nb = lib.dk_dwconv_bwd_s2_workspace_bytes(N, H, W, C)
        tok = jb.arm_partials(part)
        red = deferred_wgrad_reduce(self, nb, s is not None)
        with red:
            r = lib.dk_dwconv_bwd_s2_bnbwd_join_f32(
                g.data_ptr(), G.x.data_ptr(), N, H, W, C, OH, OW, *G.bnbwd_args(), x.data_ptr(), w.data_ptr(),
                s or 0.0, gw.data_ptr(), dx.data_ptr(), ptr(res), 2 if lat is not None else 0, jb.x.data_ptr(),
                jb.mean.data_ptr(), jb.invstd.data_ptr(), part.data_ptr(), red.ws, nb, st)
        red.flush()
        if s is None:
            add_regulariser_grad(gw, w, self.weight_regulariser)
        jb.hand_backward_partials(dx, part, r, tok)
        join.join_backward_done()
        return dx

    def backward(self, upstream_dx, residual=None, need_dx=True, join=None):
        self._require_on_gpu()
        if isinstance(upstream_dx, BNGrad):
            if self._takes_bn_grad(upstream_dx.x):
                return self._backward_bn_grad(upstream_dx, residual, need_dx, join)
            upstream_dx = upstream_dx.materialize()
        st = stream_handle()
        dy = to_nhwc(upstream_dx)
        x = self.X
        N, C, H, W = x.shape
        R, S = self.f_rows, self.f_cols
        OH, OW = int(self.num_row_patches), int(self.num_col_patches)
        P = N * OH * OW
        w = self.learned_params["weights"]
        bf = x.dtype == BF16
        if bf and (dy.dtype != BF16 or self.with_bias):
            raise NotImplementedError("{}: bf16 storage needs a bf16 gradient and no bias".format(self.layer_name))
        # the weight gradient runs on the side stream (_hip.weight_grad_stream)
        with weight_grad_stream(dy, x, *self._bn_tensors()):
            sst = stream_handle()
            if self.with_bias:
                gb = grad_buffer(self, "bias", (C,))
                nb = lib.dk_colsum_workspace_bytes(P, C)
                lib.dk_colsum_f32(dy.data_ptr(), P, C, gb.data_ptr(), workspace.get(nb), nb, sst)
            gw = grad_buffer(self, "weights", (C, R, S))
            s = l2_strength(self.weight_regulariser)
            nb = lib.dk_dwconv_wgrad_workspace_bytes(N, OH, OW, C, R, S)
            if bf:
                lib.dk_dwconv_wgrad_bnx_bf16(
                    dy.data_ptr(), x.data_ptr(), N, H, W, C, R, S, self.stride, self.padding, OH, OW,
                    w.data_ptr() if s else 0, s or 0.0, gw.data_ptr(), workspace.get(nb), nb,
                    *(self._bn_in.bn_args() if self._bn_in is not None else (0, 0, 0, 0, 0)), sst)
            elif self._bn_in is not None:
                lib.dk_dwconv_wgrad_bnx_f32(dy.data_ptr(), x.data_ptr(), N, H, W, C, R, S, self.stride,
                                            self.padding, OH, OW, w.data_ptr() if s else 0, s or 0.0, gw.data_ptr(),
                                            workspace.get(nb), nb, *self._bn_in.bn_args(), sst)
            else:
                lib.dk_dwconv_wgrad_f32(dy.data_ptr(), x.data_ptr(), N, H, W, C, R, S, self.stride, self.padding, OH,
                                        OW, w.data_ptr() if s else 0, s or 0.0, gw.data_ptr(), workspace.get(nb), nb,
                                        sst)
            if s is None:
                add_regulariser_grad(gw, w, self.weight_regulariser)
        if not need_dx:
            return None
        dx = empty_nhwc(N, C, H, W, x.dtype)
        nb = lib.dk_dwconv_dgrad_workspace_bytes(C, R, S)
        dgrad_ex = lib.dk_dwconv_dgrad_ex_bf16 if bf else lib.dk_dwconv_dgrad_ex_f32
        bn = self._bn_in
        jrows = (lib.dk_dwconv_dgrad_join_rows(N, H, W, C, R, S, self.stride, self.padding)
                 if join is not None and not bf and self._join_ok(join, True) else 0)
        # a residual handed over as its compact lattice is added as such by the join dgrad only
        lat = lattice_operand(residual, dx, self.stride) if jrows else None
        if lat is None and residual is not None:
            residual = dense_residual(residual, (N, C, H, W))
        res = lat if lat is not None else residual_operand(residual, dx)
        if residual is not None and res is None:
            jrows = 0
        # the input BatchNorm's stage-1 partials ride on the dgrad store: stride 1 in the dgrad's
        # epilogue, stride > 1 on the sub-pixel dgrad's store (same row count as its join form)
        rows = 0
        if bn is not None and R == S:
            if self.stride == 1:
                rows = lib.dk_dwconv_dgrad_stats_rows(N, H, W, C, 1)
            else:
                rows = lib.dk_dwconv_dgrad_join_rows(N, H, W, C, R, S, self.stride, self.padding)
        if rows and self.padding <= R - 1 and (residual is None or res is not None):
            # + stage 1 of the input BatchNorm's backward, in the dgrad epilogue (+ the residual)
            part = torch.empty((rows, 2, C), dtype=torch.float64, device=dx.device)
            tok = bn.arm_partials(part)
            r = dgrad_ex(dy.data_ptr(), N, OH, OW, C, w.data_ptr(), R, S, self.stride, self.padding, dx.data_ptr(), H,
                         W, workspace.get(nb), nb, ptr(res), bn.x.data_ptr(), *bn.bn_args(), part.data_ptr(), st)
            bn.hand_backward_partials(dx, part, r, tok)
            return dx
        if jrows:
            # the input's residual join: its ReLU backward and its BatchNorm's stage 1 on the store
            jb = join._join_bn
            if join._mask is None:
                join._mask_from_join()
            part = torch.empty((jrows, 2, C), dtype=torch.float64, device=dx.device)
            tok = jb.arm_partials(part)
            r = lib.dk_dwconv_dgrad_join_f32(dy.data_ptr(), N, OH, OW, C, w.data_ptr(), R, S, self.stride,
                                             self.padding, dx.data_ptr(), H, W, workspace.get(nb), nb, ptr(res),
                                             self.stride if lat is not None else 0, join._mask.data_ptr(), jb.x.data_ptr(), jb.mean.data_ptr(),
                                             jb.invstd.data_ptr(), part.data_ptr(), st)
            jb.hand_backward_partials(dx, part, r, tok)
            join.join_backward_done()
            return dx
        if bf:
            if residual is not None and res is None:
                raise NotImplementedError("{}: bf16 residual must be a bf16 NHWC tensor".format(self.layer_name))
            dgrad_ex(dy.data_ptr(), N, OH, OW, C, w.data_ptr(), R, S, self.stride, self.padding, dx.data_ptr(), H, W,
                     workspace.get(nb), nb, ptr(res), 0, 0, 0, 0, 0, 0, 0, st)
            return dx
        if res is not None:
            try:
                lib.dk_dwconv_dgrad_ex_f32(dy.data_ptr(), N, OH, OW, C, w.data_ptr(), R, S, self.stride,
                                           self.padding, dx.data_ptr(), H, W, workspace.get(nb), nb, res.data_ptr(),
                                           0, 0, 0, 0, 0, 0, 0, st)
                return dx
            except HipError:  # geometry without a fused residual (generic gather dgrad)
                pass
        lib.dk_dwconv_dgrad_f32(dy.data_ptr(), N, OH, OW, C, w.data_ptr(), R, S, self.stride, self.padding,
                                dx.data_ptr(), H, W, workspace.get(nb), nb, st)
        return add_residual(dx, residual) if residual is not None else dx

    def save_to_h5(self, open_f, save_grads=True):
        from ..network.checkpoint import save_layer
        save_layer(self, open_f, save_grads)

    def load_from_h5(self, open_f, load_grads=True):
        from ..network.checkpoint import load_layer
        load_layer(self, open_f, load_grads)
