"""1x1 (pointwise) convolution (reference: layers/pointwise_convolution.py).

The reference subsamples with a strided view (:48-49), copies the input into an NHWC
row matrix (:50), runs cuBLAS SGEMM (:51), and in backward widens the stride-s gradient
into a freshly zeroed buffer (:68-72).  Here the activations are already NHWC, so the
layer is the R = S = 1 case of the implicit-GEMM MFMA engine: subsampling is a strided
gather in the A-tile loader and the widen is fused into the dgrad epilogue.

Public surface identical to the reference: constructor (:7-8, note ``stride`` is the
second positional argument), weights (K, C), bias (K,), ``__repr__`` (:35-44), the
output spatial size ceil(H/s), and the backward output size (s*OH, s*OW).

Any channel count C is accepted, as by the reference's cp.dot over (K, C).  The kernels load
16 bytes per lane, so for C % 4 != 0 the input is zero-padded to Cp = 4*ceil(C/4) channels
(layout conversion), the weights to (K, Cp) (dk_conv_weight_krsc_f32 with R = S = 1), the
weight gradient is scattered back to (K, C) by the conv weight-gradient reduce, and the
input gradient is computed on Cp channels and returned as its first C.
"""
from __future__ import annotations


import torch

from .._env import getenv
from .._hip import deferred_wgrad_reduce, lib, stream_handle, weight_grad_stream, workspace
from .._tensor import BF16, empty_nhwc, ptr, to_nhwc
from ._bn_input import BNGrad, BNOut, add_residual, residual_operand
from ._common import add_regulariser_grad, grad_buffer, init_weights, l2_strength
from .layer import Layer


class PointwiseConvLayer(Layer):
    def __init__(self, layer_name, stride=1, filter_block_shape=None, with_bias=True,
                 weight_regulariser=None, weight_initialiser="normal"):
        """
        filter_block_shape = (num_filters, num_incoming_channels)
        """
        super().__init__(layer_name)
        self.stride = stride
        self.with_bias = with_bias
        self.weight_regulariser = weight_regulariser
        self.weight_initialiser = weight_initialiser
        if filter_block_shape is not None:
            self.num_filters, self.num_channels = filter_block_shape
            weights = init_weights(tuple(filter_block_shape), weight_initialiser,
                                   self.num_channels + self.num_filters)
            self.learned_params = {"weights": weights}
            self.grads = {"weights": weights * 0}
            if with_bias:
                bias = (weights[:, 0] * 0).copy()
                self.learned_params["bias"] = bias
                self.grads["bias"] = bias * 0
        else:
            self.num_filters = None
            self.learned_params = {}
            self.grads = {}

    def __repr__(self):
        out = "PointwiseConvLayer({}, ".format(self.layer_name)
        if self.num_filters is not None:
            out += "filter_block_shape=({}, {}), ".format(self.num_filters, self.num_channels)
        out += "stride={}, with_bias={}, weight_regulariser={}, is_on_gpu={})".format(
            self.stride, self.with_bias, repr(self.weight_regulariser), self.is_on_gpu)
        return out

    accepts_bn_input = True   # forward(BNOut): the preceding BatchNorm is applied on load
    produces_bn_stats = True  # forward(..., bn_stats=StatsRequest): emits the next BN's statistics

    def _padded_weights(self, w, Cp):
        """(K, C) weights zero-padded to (K, Cp) for a C % 4 != 0 input (a fresh copy per
        forward, so it always reflects the current weights)."""
        K, C = self.num_filters, self.num_channels
        wp = torch.empty((K, Cp), dtype=torch.float32, device=w.device)
        lib.dk_conv_weight_krsc_f32(w.data_ptr(), K, C, 1, 1, Cp, wp.data_ptr(), stream_handle())
        return wp

    def forward(self, X, test_mode=False, bn_stats=None):
        self._require_on_gpu()
        st = stream_handle()
        if X.shape[1] != self.num_channels:
            raise ValueError("PointwiseConvLayer {}: input has {} channels, weights expect {}".format(
                self.layer_name, X.shape[1], self.num_channels))
        bn = X if isinstance(X, BNOut) and X.dim() == 4 and X.shape[1] % 4 == 0 else None
        x = bn.x if bn is not None else to_nhwc(X, cpad=4)
        N, Cp, H, W = x.shape
        K = self.num_filters
        s = self.stride
        OH, OW = -(-H // s), -(-W // s)  # len(range(0, H, s)), as X[:, :, ::s, ::s]
        bf = x.dtype == BF16  # bf16 storage (BASELINE config 5): the _bf16 entry points
        y = empty_nhwc(N, K, OH, OW, x.dtype)
        w = self.learned_params["weights"]
        if Cp != self.num_channels:
            if bf:
                raise NotImplementedError("{}: bf16 storage needs C % 4 == 0".format(self.layer_name))
            w = self._padded_weights(w, Cp)
        self._wp = w
        bias = self.learned_params["bias"] if self.with_bias else None
        stats = None
        if bn_stats is not None and not test_mode:
            rows = (lib.dk_pwconv_fwd_bf16_stats_rows if bf else lib.dk_pwconv_fwd_stats_rows)(N, OH, OW, K, Cp)
            stats = torch.empty((rows, 2, K), dtype=torch.float64, device=x.device)
        if bn is not None or stats is not None or bf:
            fwd = lib.dk_pwconv_fwd_ex_bf16 if bf else lib.dk_pwconv_fwd_ex_f32
            if stats is not None:
                bn_stats.arm(stats, N * OH * OW)
            r = fwd(x.data_ptr(), N, H, W, Cp, w.data_ptr(), K, s, ptr(bias), y.data_ptr(), OH, OW,
                    *(bn.bn_args() if bn is not None else (0, 0, 0, 0, 0)), ptr(stats), st)
            if stats is not None:
                bn_stats.launched(stats, r)
        else:
            lib.dk_pwconv_fwd_f32(x.data_ptr(), N, H, W, Cp, w.data_ptr(), K, s, ptr(bias), y.data_ptr(), OH, OW, st)
        # the reference keeps the NHWC row copy as self.patches (:50); here the input itself
        # (or, for a BNOut, the BatchNorm's raw input + parameters)
        self.X = x
        self._bn_in = bn
        self.out_hw = (OH, OW)
        return y

    accepts_residual = True  # backward(dy, residual=R) returns dx + R (the residual join, fused)

    def accepts_bn_grad(self, bn_layer):
        """backward(BNGrad): the following BatchNorm's apply runs in this layer's dgrad loader
        (dk_pwconv_dgrad_bnbwd_f32, or _bf16 for bf16 storage) -- stride 1, 4-D, channel counts
        the 16-byte loads and the LDS coefficient table take."""
        x = getattr(self, "X", None)
        bx = getattr(bn_layer, "X", None)
        if x is not None and bx is not None and self._lattice_fused_ok(bx):
            return True  # (the strided stem layer: dk_pwconv_bwd_bnbwd_lattice_f32 when the lattice is asked for)
        return (x is not None and bx is not None and x.dtype in (torch.float32, BF16) and self.stride == 1
                and x.dim() == 4 and x.shape[1] == self.num_channels and self._takes_bn_grad(bx))

    def _lattice_fused_ok(self, bx, residual=None):
        """backward(BNGrad, lattice_out=True) as one pass (dk_pwconv_bwd_bnbwd_lattice_f32: the
        following BatchNorm's apply, the dgrad into the compact lattice, the weight gradient and the
        input BatchNorm's partials; dy never stored): fp32, lattice_ok(), K = C = 64, the input
        consumed as a BNOut, no residual (DORKNET_PW_LATTICE_FUSED=0: off)."""
        x = self.X
        if (residual is not None or self._bn_in is None or not self.lattice_ok() or bx.dtype != torch.float32
                or bx.dim() != 4 or getenv("DORKNET_PW_LATTICE_FUSED", "1") == "0"):
            return False
        N = x.shape[0]
        OH, OW = self.out_hw
        return (tuple(bx.shape) == (N, self.num_filters, OH, OW)
                and lib.dk_pwconv_bwd_fused_rows(N, OH, OW, self.num_filters, self.num_channels) > 0
                and self.num_filters == 64 and self.num_channels == 64)

    def _takes_bn_grad(self, bx):
        bf = self.X.dtype == BF16
        return (bx.dim() == 4 and bx.dtype == self.X.dtype and self.X.dtype in (torch.float32, BF16)
                and self.stride == 1 and self.X.shape[1] == self.num_channels
                and tuple(bx.shape) == (self.X.shape[0], self.num_filters, *self.out_hw)
                and self.num_filters % 4 == 0 and self.num_filters <= 2048 and not (bf and self.with_bias))

    skips_input_grad = True  # backward(dy, need_dx=False): parameter gradients only (chain_backward)

    def lattice_ok(self):
        """backward(dy, lattice_out=True) can hand over its widened input gradient as the compact
        stride-s lattice: stride > 1, fp32, no bias.  With the input consumed as a BNOut the
        partials of that BN ride on the dgrad (dk_pwconv_dgrad_lattice_f32); a plain input (a
        residual block's skip projection) gets the stride-1 GEMM into the compact grid."""
        x = getattr(self, "X", None)
        return (self.stride > 1 and x is not None and x.dim() == 4 and x.dtype == torch.float32
                and x.shape[1] == self.num_channels and not self.with_bias
                and tuple(x.shape[2:]) == (self.out_hw[0] * self.stride, self.out_hw[1] * self.stride))

    def backward(self, upstream_dx, residual=None, need_dx=True, lattice_out=False):
        """lattice_out: return the input gradient as the compact stride-s lattice (a tensor tagged
        `_dk_lattice = s`) when lattice_ok(); chain_backward asks for it only when the consumer of
        that gradient takes the lattice form."""
        self._require_on_gpu()
        st = stream_handle()
        x = self.X
        N, C, H, W = x.shape
        K, s = self.num_filters, self.stride
        OH, OW = self.out_hw
        P = N * OH * OW
        w = self.learned_params["weights"]
        if isinstance(upstream_dx, BNGrad):
            if need_dx and lattice_out and self._lattice_fused_ok(upstream_dx.x, residual):
                return self._bwd_fused_lattice(upstream_dx, st)
            if need_dx and self._fused_bwd_ok(upstream_dx, residual):
                # input gradient, weight gradient and the input BN's partials in one pass; dy
                # is formed from the BatchNorm's gradient as it is loaded and never stored
                return self._bwd_fused(upstream_dx, residual, st)
            if need_dx and self._takes_bn_grad(upstream_dx.x):
                # dgrad first: it forms (and stores) dy from the BatchNorm's gradient as it loads it
                bf = x.dtype == BF16
                dy = empty_nhwc(N, K, OH, OW, x.dtype)
                dx = (self._dgrad_bnbwd_bf16 if bf else self._dgrad_bnbwd)(upstream_dx, dy, residual, st)
                self._wgrad(dy, x, N, H, W, C, K, s, OH, OW, P, w, bf)
                return dx
            upstream_dx = upstream_dx.materialize()
        dy = to_nhwc(upstream_dx)
        bf = x.dtype == BF16
        if C != self.num_channels:
            return self._backward_padded(dy, residual, need_dx, st)
        if bf and (dy.dtype != BF16 or self.with_bias or s != 1):
            raise NotImplementedError("{}: bf16 storage needs a bf16 gradient, no bias, stride 1".format(
                self.layer_name))
        self._wgrad(dy, x, N, H, W, C, K, s, OH, OW, P, w, bf)
        if need_dx and lattice_out and residual is None and not bf and self.lattice_ok():
            return self._dgrad_lattice(dy, st)
        return self._dgrad(dy, residual, st) if need_dx else None

    def _dgrad_lattice(self, dy, st):
        """The widened input gradient kept as its lattice (+ the input BN's partials).  The values
        are the widened dgrad's at the lattice points bit for bit (the same GEMM tiles; only the
        epilogue's addressing differs)."""
        x = self.X
        N, C = x.shape[0], x.shape[1]
        K, s = self.num_filters, self.stride
        OH, OW = self.out_hw
        bn = self._bn_in
        dx = empty_nhwc(N, C, OH, OW)
        if bn is None:
            lib.dk_pwconv_dgrad_f32(dy.data_ptr(), N, OH, OW, K, self.learned_params["weights"].data_ptr(), C, 1,
                                    dx.data_ptr(), st)
            dx._dk_lattice = s
            return dx
        rows = lib.dk_pwconv_dgrad_stats_rows(N, OH, OW, K, C)
        part = torch.empty((rows, 2, C), dtype=torch.float64, device=dx.device)
        tok = bn.arm_partials(part)
        r = lib.dk_pwconv_dgrad_lattice_f32(dy.data_ptr(), N, OH, OW, K, self.learned_params["weights"].data_ptr(), C,
                                            s, dx.data_ptr(), bn.x.data_ptr(), *bn.bn_args(), part.data_ptr(), st)
        dx._dk_lattice = s
        bn.hand_backward_partials(dx, part, r, tok)
        return dx

    def _backward_padded(self, dy, residual, need_dx, st):
        """Backward for C % 4 != 0: the input was padded to Cp channels in forward."""
        x = self.X
        N, Cp, H, W = x.shape
        C, K, s = self.num_channels, self.num_filters, self.stride
        OH, OW = self.out_hw
        P = N * OH * OW
        w = self.learned_params["weights"]
        with weight_grad_stream(dy, x):
            sst = stream_handle()
            if self.with_bias:
                gb = grad_buffer(self, "bias", (K,))
                nb = lib.dk_colsum_workspace_bytes(P, K)
                lib.dk_colsum_f32(dy.data_ptr(), P, K, gb.data_ptr(), workspace.get(nb), nb, sst)
            gw = grad_buffer(self, "weights", (K, C))
            l2s = l2_strength(self.weight_regulariser)
            # the conv weight gradient with R = S = 1, pad 0: its reduce scatters (K, Cp) -> (K, C)
            nb = lib.dk_conv2d_wgrad_workspace_bytes(N, OH, OW, K, Cp, 1, 1)
            lib.dk_conv2d_wgrad_f32(dy.data_ptr(), x.data_ptr(), N, H, W, Cp, C, K, 1, 1, s, 0, OH, OW,
                                    w.data_ptr() if l2s else 0, l2s or 0.0, gw.data_ptr(), workspace.get(nb), nb,
                                    sst)
            if l2s is None:
                add_regulariser_grad(gw, w, self.weight_regulariser)
        if not need_dx:
            return None
        dxp = empty_nhwc(N, Cp, OH * s, OW * s)
        lib.dk_pwconv_dgrad_f32(dy.data_ptr(), N, OH, OW, K, self._wp.data_ptr(), Cp, s, dxp.data_ptr(), st)
        dx = dxp[:, :C]
        if residual is not None:
            dx = add_residual(dx, residual)
        return dx

    def _fused_bwd_ok(self, bg, residual):
        """dk_pwconv_bwd_bnbwd_f32 / _bf16 applies: stride 1, no bias, a residual (if any) that
        fuses, and a shape a fused kernel takes -- fp32: K = C = 64 (the streaming kernel of
        pw_stream.hip, which never stores dy) and K in {128, 256} (the weight-stationary kernel of
        pw_deep.hip), taken by default where the library prefers it; bf16 (config 5): K = C = 64
        (pw_stream_bf16.hip) and K in {128, 256} with C a multiple of 128 (pw_deep_bf16.hip).  DORKNET_PW_FUSED_BWD=1 / 0 forces the fp32 path on / off (its round-1
        tiled kernel for K or C = 128 measured 0.75 % slower than the unfused pair, DESIGN.md
        section 5)."""
        x = self.X
        if self.with_bias or not self._takes_bn_grad(bg.x):
            return False
        N, C, H, W = x.shape
        OH, OW = self.out_hw
        if x.dtype == BF16:
            if lib.dk_pwconv_bwd_fused_bf16_rows(N, OH, OW, self.num_filters, C) <= 0:
                return False
        elif x.dtype != torch.float32:
            return False
        else:
            if lib.dk_pwconv_bwd_fused_rows(N, OH, OW, self.num_filters, C) <= 0:
                return False
            env = getenv("DORKNET_PW_FUSED_BWD")
            if env is not None:
                if env != "1":
                    return False
            elif not lib.dk_pwconv_bwd_fused_preferred(N, OH, OW, self.num_filters, C):
                return False
        if residual is not None and residual_operand(residual, x) is None:
            return False
        return True

    def _bwd_fused(self, bg, residual, st):
        x = self.X
        N, C, H, W = x.shape
        K = self.num_filters
        OH, OW = self.out_hw
        w = self.learned_params["weights"]
        bf = x.dtype == BF16
        dx = empty_nhwc(N, C, OH, OW, x.dtype)
        bn = self._bn_in
        res = residual_operand(residual, dx)
        g = to_nhwc(bg.g)
        part = None
        rows_fn = lib.dk_pwconv_bwd_fused_bf16_rows if bf else lib.dk_pwconv_bwd_fused_rows
        if bn is not None:
            rows = rows_fn(N, OH, OW, K, C)
            part = torch.empty((rows, 2, C), dtype=torch.float64, device=dx.device)
        gw = grad_buffer(self, "weights", (K, C))
        l2s = l2_strength(self.weight_regulariser)
        nb = (lib.dk_pwconv_bwd_fused_bf16_workspace_bytes if bf else lib.dk_pwconv_bwd_fused_workspace_bytes)(
            N, OH, OW, K, C)
        tok = bn.arm_partials(part) if bn is not None else None
        # the weight-gradient reduce on the side stream (not with a non-l2 regulariser, whose term
        # is added to gw on this stream right after)
        red = deferred_wgrad_reduce(self, nb, l2s is not None)
        with red:
            r = (lib.dk_pwconv_bwd_bnbwd_bf16 if bf else lib.dk_pwconv_bwd_bnbwd_f32)(
                g.data_ptr(), bg.x.data_ptr(), N, OH, OW, K, *bg.bnbwd_args(), w.data_ptr(), C, l2s or 0.0,
                gw.data_ptr(), dx.data_ptr(), ptr(res), x.data_ptr(),
                *((*bn.bn_args(), part.data_ptr()) if bn is not None else (0,) * 6), red.ws, nb, st)
        red.flush()
        if l2s is None:
            add_regulariser_grad(gw, w, self.weight_regulariser)
        if not red.on:
            # the weight gradient was written on this stream: work queued on the side stream from
            # here on (a data-parallel bucket's all-reduce) must follow it
            with weight_grad_stream():
                pass
        if bn is not None:
            bn.hand_backward_partials(dx, part, r, tok)
        return dx

    def _bwd_fused_lattice(self, bg, st):
        x = self.X
        N, C, H, W = x.shape
        K, s = self.num_filters, self.stride
        OH, OW = self.out_hw
        w = self.learned_params["weights"]
        dx = empty_nhwc(N, C, OH, OW)
        bn = self._bn_in
        rows = lib.dk_pwconv_bwd_fused_rows(N, OH, OW, K, C)
        part = torch.empty((rows, 2, C), dtype=torch.float64, device=dx.device)
        gw = grad_buffer(self, "weights", (K, C))
        l2s = l2_strength(self.weight_regulariser)
        nb = lib.dk_pwconv_bwd_fused_workspace_bytes(N, OH, OW, K, C)
        tok = bn.arm_partials(part)
        red = deferred_wgrad_reduce(self, nb, l2s is not None)
        with red:
            r = lib.dk_pwconv_bwd_bnbwd_lattice_f32(
                to_nhwc(bg.g).data_ptr(), bg.x.data_ptr(), N, OH, OW, K, *bg.bnbwd_args(), w.data_ptr(), C,
                l2s or 0.0, gw.data_ptr(), dx.data_ptr(), x.data_ptr(), H, W, s, *bn.bn_args(), part.data_ptr(),
                red.ws, nb, st)
        red.flush()
        if l2s is None:
            add_regulariser_grad(gw, w, self.weight_regulariser)
        if not red.on:
            with weight_grad_stream():
                pass
        dx._dk_lattice = s
        bn.hand_backward_partials(dx, part, r, tok)
        return dx

    def _dgrad_bnbwd(self, bg, dy_out, residual, st):
        x = self.X
        N, C, H, W = x.shape
        K = self.num_filters
        OH, OW = self.out_hw
        w = self.learned_params["weights"]
        dx = empty_nhwc(N, C, OH, OW)
        bn = self._bn_in
        res = residual_operand(residual, dx)
        g = to_nhwc(bg.g)
        part = None
        if bn is not None:
            rows = lib.dk_pwconv_dgrad_bnbwd_stats_rows(N, OH, OW, K, C)
            part = torch.empty((rows, 2, C), dtype=torch.float64, device=dx.device)
        tok = bn.arm_partials(part) if bn is not None else None
        r = lib.dk_pwconv_dgrad_bnbwd_f32(g.data_ptr(), bg.x.data_ptr(), N, OH, OW, K, *bg.bnbwd_args(),
                                          dy_out.data_ptr(), w.data_ptr(), C, dx.data_ptr(), ptr(res),
                                          *((bn.x.data_ptr(), *bn.bn_args(), part.data_ptr()) if bn is not None
                                            else (0, 0, 0, 0, 0, 0, 0)), st)
        if bn is not None:
            bn.hand_backward_partials(dx, part, r, tok)
        if residual is not None and res is None:
            dx = add_residual(dx, residual)
        return dx

    def _dgrad_bnbwd_bf16(self, bg, dy_out, residual, st):
        """bf16 storage: dk_pwconv_dgrad_bnbwd_bf16 (dy formed on load, rounded to bf16 for the
        MFMA and for dy_out; the input BatchNorm's partials over the stored dx)."""
        x = self.X
        N, C, H, W = x.shape
        K = self.num_filters
        OH, OW = self.out_hw
        dx = empty_nhwc(N, C, OH, OW, x.dtype)
        bn = self._bn_in
        res = residual_operand(residual, dx)
        if residual is not None and res is None:
            raise NotImplementedError("{}: bf16 residual must be a bf16 NHWC tensor".format(self.layer_name))
        part = None
        if bn is not None:
            rows = lib.dk_pwconv_dgrad_bnbwd_bf16_stats_rows(N, OH, OW, K, C)
            part = torch.empty((rows, 2, C), dtype=torch.float64, device=dx.device)
        tok = bn.arm_partials(part) if bn is not None else None
        r = lib.dk_pwconv_dgrad_bnbwd_bf16(to_nhwc(bg.g).data_ptr(), bg.x.data_ptr(), N, OH, OW, K, *bg.bnbwd_args(),
                                           dy_out.data_ptr(), self.learned_params["weights"].data_ptr(), C,
                                           dx.data_ptr(), ptr(res),
                                           *((bn.x.data_ptr(), *bn.bn_args(), part.data_ptr()) if bn is not None
                                             else (0, 0, 0, 0, 0, 0, 0)), st)
        if bn is not None:
            bn.hand_backward_partials(dx, part, r, tok)
        return dx

    def _wgrad(self, dy, x, N, H, W, C, K, s, OH, OW, P, w, bf):
        # the weight gradient runs on the side stream (_hip.weight_grad_stream)
        with weight_grad_stream(dy, x, *self._bn_tensors()):
            sst = stream_handle()
            if self.with_bias:
                gb = grad_buffer(self, "bias", (K,))
                nb = lib.dk_colsum_workspace_bytes(P, K)
                lib.dk_colsum_f32(dy.data_ptr(), P, K, gb.data_ptr(), workspace.get(nb), nb, sst)
            gw = grad_buffer(self, "weights", (K, C))
            l2s = l2_strength(self.weight_regulariser)
            nb = lib.dk_pwconv_wgrad_workspace_bytes(N, OH, OW, K, C)
            if bf:
                lib.dk_pwconv_wgrad_bnx_bf16(
                    dy.data_ptr(), x.data_ptr(), N, H, W, C, K, s, OH, OW, w.data_ptr() if l2s else 0, l2s or 0.0,
                    gw.data_ptr(), workspace.get(nb), nb,
                    *(self._bn_in.bn_args() if self._bn_in is not None else (0, 0, 0, 0, 0)), sst)
            elif self._bn_in is not None:
                lib.dk_pwconv_wgrad_bnx_f32(dy.data_ptr(), x.data_ptr(), N, H, W, C, K, s, OH, OW,
                                            w.data_ptr() if l2s else 0, l2s or 0.0, gw.data_ptr(), workspace.get(nb),
                                            nb, *self._bn_in.bn_args(), sst)
            else:
                lib.dk_pwconv_wgrad_f32(dy.data_ptr(), x.data_ptr(), N, H, W, C, K, s, OH, OW,
                                        w.data_ptr() if l2s else 0, l2s or 0.0, gw.data_ptr(), workspace.get(nb), nb,
                                        sst)
            if l2s is None:
                add_regulariser_grad(gw, w, self.weight_regulariser)

    def _dgrad(self, dy, residual, st):
        x = self.X
        N, C, H, W = x.shape
        K, s = self.num_filters, self.stride
        OH, OW = self.out_hw
        w = self.learned_params["weights"]
        bf = x.dtype == BF16
        dx = empty_nhwc(N, C, OH * s, OW * s, x.dtype)  # widened shape, pointwise_convolution.py:68-72
        bn = self._bn_in
        res = residual_operand(residual, dx)
        if bf:
            if residual is not None and res is None:
                raise NotImplementedError("{}: bf16 residual must be a bf16 NHWC tensor".format(self.layer_name))
            if bn is not None and (OH, OW) == (H, W):
                rows = lib.dk_pwconv_dgrad_stats_rows(N, OH, OW, K, C)
                part = torch.empty((rows, 2, C), dtype=torch.float64, device=dx.device)
                tok = bn.arm_partials(part)
                r = lib.dk_pwconv_dgrad_ex_bf16(dy.data_ptr(), N, OH, OW, K, w.data_ptr(), C, s, dx.data_ptr(),
                                                ptr(res), bn.x.data_ptr(), *bn.bn_args(), part.data_ptr(), st)
                bn.hand_backward_partials(dx, part, r, tok)
            else:
                lib.dk_pwconv_dgrad_ex_bf16(dy.data_ptr(), N, OH, OW, K, w.data_ptr(), C, s, dx.data_ptr(), ptr(res),
                                            0, 0, 0, 0, 0, 0, 0, st)
            return dx
        if bn is not None and (OH * s, OW * s) == (H, W) and (res is None or s == 1):
            # + stage 1 of the input BatchNorm's backward, in the dgrad epilogue
            rows = lib.dk_pwconv_dgrad_stats_rows(N, OH, OW, K, C)
            part = torch.empty((rows, 2, C), dtype=torch.float64, device=dx.device)
            tok = bn.arm_partials(part)
            r = lib.dk_pwconv_dgrad_ex_f32(dy.data_ptr(), N, OH, OW, K, w.data_ptr(), C, s, dx.data_ptr(), ptr(res),
                                           bn.x.data_ptr(), *bn.bn_args(), part.data_ptr(), st)
            bn.hand_backward_partials(dx, part, r, tok)
        elif res is not None:
            lib.dk_pwconv_dgrad_ex_f32(dy.data_ptr(), N, OH, OW, K, w.data_ptr(), C, s, dx.data_ptr(), res.data_ptr(),
                                       0, 0, 0, 0, 0, 0, 0, st)
        else:
            lib.dk_pwconv_dgrad_f32(dy.data_ptr(), N, OH, OW, K, w.data_ptr(), C, s, dx.data_ptr(), st)
            if residual is not None:
                dx = add_residual(dx, residual)
        return dx

    def save_to_h5(self, open_f, save_grads=True):
        from ..network.checkpoint import save_layer
        save_layer(self, open_f, save_grads)

    def load_from_h5(self, open_f, load_grads=True):
        from ..network.checkpoint import load_layer
        load_layer(self, open_f, load_grads)
