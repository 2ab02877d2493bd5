"""Dense 2-D convolution (reference: layers/convolution.py).

The reference lowers the convolution to im2col + cuBLAS SGEMM: it zero-fills and
materialises a [N*OH*OW, C*R*S] patch matrix (convolution.py:69-74), multiplies it by
the flattened filters (:75), and in backward multiplies again and scatters the result
back with atomics (:101-111).  Here the same contraction runs as an implicit GEMM on the
fp32 MFMA units: patches are gathered straight from the NHWC activation into LDS tiles
and never exist in HBM (dk_conv2d_fwd_f32 / _dgrad_f32 / _wgrad_f32).  A narrow input (C <= 4:
the stem on the 3-channel image) takes the narrow-input kernels instead, which read the NCHW
image as given and reduce over k = (c, r, s) without channel padding (dk_conv2d_*_narrow_f32).

Public surface identical to the reference: constructor signature and defaults
(:13-14), ``learned_params`` / ``grads`` keys and shapes (weights (K, C, R, S), bias (K,)),
``forward(X, test_mode=False)`` -> (N, K, OH, OW), ``backward(upstream_dx)`` -> dx with
the input's shape, ``__repr__`` text (:40-51), and the float-then-int output-size
arithmetic (:67-68, :105-106).
"""
from __future__ import annotations


import torch

from .._env import getenv
from .._hip import lib, stream_handle, weight_grad_stream, workspace
from .._tensor import as_device, empty_nhwc, ptr, to_nhwc
from ._bn_input import BNGrad, BNOut
from ._common import add_regulariser_grad, grad_buffer, init_weights, l2_strength
from .layer import Layer


class ConvLayer(Layer):
    def __init__(self, layer_name, filter_block_shape=None, stride=1, padding=1,
                 with_bias=True, weight_regulariser=None, weight_initialiser="normal"):
        super().__init__(layer_name)
        self.stride = stride
        self.padding = padding
        self.patches = None
        self.weight_regulariser = weight_regulariser
        self.weight_initialiser = weight_initialiser
        self.with_bias = with_bias
        if filter_block_shape:
            self.num_filters, self.filter_chans, self.f_rows, self.f_cols = filter_block_shape
            weights = init_weights(tuple(filter_block_shape), weight_initialiser,
                                   self.filter_chans + self.num_filters)
            self.learned_params = {"weights": weights}
            self.grads = {"weights": weights * 0}
            if with_bias:
                bias = (weights[:, 0, 0, 0] * 0).copy()
                self.learned_params["bias"] = bias
                self.grads["bias"] = bias * 0
        else:
            self.num_filters = None
            self.learned_params = {}
            self.grads = {}

    def __repr__(self):
        out = "ConvLayer({}, ".format(self.layer_name)
        if self.num_filters is not None:
            out += "filter_block_shape=({},{},{},{}), ".format(self.num_filters, self.filter_chans,
                                                               self.f_rows, self.f_rows)
        out += "stride={}, padding={}, with_bias={}, weight_regulariser={})".format(
            self.stride, self.padding, self.with_bias, self.weight_regulariser)
        return out

    # -- helpers -------------------------------------------------------------------------

    def _out_size(self, H, W):
        # float arithmetic on the padded size, as convolution.py:67-68
        self.num_row_patches = ((H + 2 * self.padding - self.f_rows) / self.stride) + 1
        self.num_col_patches = ((W + 2 * self.padding - self.f_cols) / self.stride) + 1
        return int(self.num_row_patches), int(self.num_col_patches)

    # -- forward / backward --------------------------------------------------------------

    accepts_bn_input = True   # forward(BNOut): the preceding BatchNorm is applied on load
    produces_bn_stats = True  # forward(..., bn_stats=StatsRequest): emits the next BN's statistics

    def _narrow_ok(self, X):
        """The narrow-input kernels take this input (raw NCHW, C <= 4: the stem).
        DORKNET_NARROW=0 keeps every input on the implicit-GEMM path (A/B runs)."""
        if getenv("DORKNET_NARROW", "1") == "0":
            return False
        if isinstance(X, BNOut) or len(getattr(X, "shape", ())) != 4 or X.shape[1] != self.filter_chans:
            return False
        if isinstance(X, torch.Tensor) and X.dtype != torch.float32:
            return False
        N, C, H, W = (int(v) for v in X.shape)
        OH, OW = self._out_size(H, W)
        return bool(lib.dk_conv2d_narrow_preferred(N, C, H, W, self.num_filters, self.f_rows, self.f_cols,
                                                   self.stride, self.padding, OH, OW))

    def _forward_narrow(self, X, test_mode, bn_stats):
        st = stream_handle()
        x = as_device(X, torch.float32).contiguous()  # NCHW, as given
        N, C, H, W = x.shape
        K, R, S = self.num_filters, self.f_rows, self.f_cols
        OH, OW = self._out_size(H, W)
        y = empty_nhwc(N, K, OH, OW)
        bias = self.learned_params["bias"] if self.with_bias else None
        stats = None
        if bn_stats is not None and not test_mode:
            rows = lib.dk_conv2d_fwd_narrow_stats_rows(N, C, H, W, K, R, S, self.stride, self.padding, OH, OW)
            stats = torch.empty((rows, 2, K), dtype=torch.float64, device=x.device)
            bn_stats.arm(stats, N * OH * OW)
        r = lib.dk_conv2d_fwd_narrow_f32(x.data_ptr(), N, C, H, W, self.learned_params["weights"].data_ptr(), K, R,
                                         S, self.stride, self.padding, ptr(bias), y.data_ptr(), OH, OW, ptr(stats),
                                         st)
        if stats is not None:
            bn_stats.launched(stats, r)
        elif r:
            raise RuntimeError(f"dk_conv2d_fwd_narrow_f32 failed: {r}")
        self.X = x
        self._bn_in = None
        self._narrow = True
        return y

    def forward(self, X, test_mode=False, bn_stats=None):
        self._require_on_gpu()
        st = stream_handle()
        self.input_shape = tuple(X.shape)
        if self._narrow_ok(X):
            return self._forward_narrow(X, test_mode, bn_stats)
        self._narrow = False
        bn = X if isinstance(X, BNOut) and X.dim() == 4 and X.shape[1] % 4 == 0 else None
        x = bn.x if bn is not None else to_nhwc(X, cpad=4)
        N, Cp, H, W = x.shape
        K, C, R, S = self.num_filters, self.filter_chans, self.f_rows, self.f_cols
        OH, OW = self._out_size(H, W)
        w = self.learned_params["weights"]
        w_krsc = torch.empty((K, R, S, Cp), dtype=torch.float32, device=x.device)
        lib.dk_conv_weight_krsc_f32(w.data_ptr(), K, C, R, S, Cp, w_krsc.data_ptr(), st)
        y = empty_nhwc(N, K, OH, OW)
        bias = self.learned_params["bias"] if self.with_bias else None
        stats = None
        if bn_stats is not None and not test_mode:
            rows = lib.dk_conv2d_fwd_stats_rows(N, OH, OW, K, Cp, R, S)
            stats = torch.empty((rows, 2, K), dtype=torch.float64, device=x.device)
        if bn is not None or stats is not None:
            if stats is not None:
                bn_stats.arm(stats, N * OH * OW)
            r = lib.dk_conv2d_fwd_ex_f32(x.data_ptr(), N, H, W, Cp, w_krsc.data_ptr(), K, R, S, self.stride,
                                         self.padding, ptr(bias), y.data_ptr(), OH, OW,
                                         *(bn.bn_args() if bn is not None else (0, 0, 0, 0, 0)), ptr(stats), st)
            if stats is not None:
                bn_stats.launched(stats, r)
        else:
            lib.dk_conv2d_fwd_f32(x.data_ptr(), N, H, W, Cp, w_krsc.data_ptr(), K, R, S, self.stride, self.padding,
                                  ptr(bias), y.data_ptr(), OH, OW, st)
        # The reference caches the patch matrix (convolution.py:69-74); the implicit GEMM
        # only needs the (NHWC) input itself (for a BNOut: the BatchNorm's raw input).
        self.X = x
        self._bn_in = bn
        return y

    skips_input_grad = True  # backward(dy, need_dx=False): parameter gradients only (chain_backward)

    @property
    def accepts_lattice_grad(self):
        """The BN-deferred weight gradient takes a stride-2 lattice gradient (the narrow kernels)."""
        return bool(getattr(self, "_narrow", False))

    def accepts_bn_grad(self, bn_layer):
        """backward(BNGrad, need_dx=False): the following BatchNorm's apply runs in this layer's
        weight-gradient loader (dk_conv2d_wgrad_bnbwd_f32) -- the stem, whose input gradient
        the network drops.  With need_dx the gradient is materialised (the dgrad reads it)."""
        bx = getattr(bn_layer, "X", None)
        return getattr(self, "X", None) is not None and bx is not None and self._takes_bn_grad(bx)

    def _takes_bn_grad(self, bx):
        x = self.X
        OH, OW = int(self.num_row_patches), int(self.num_col_patches)
        return (bx.dim() == 4 and bx.dtype == torch.float32 and x.dtype == torch.float32 and not self.with_bias
                and self.num_filters % 4 == 0 and tuple(bx.shape) == (x.shape[0], self.num_filters, OH, OW))

    def _wgrad_bn_grad(self, G):
        """Weight gradient straight from the following BatchNorm's deferred gradient."""
        st = stream_handle()
        x = self.X
        N, Cp, H, W = x.shape
        K, C, R, S = self.num_filters, self.filter_chans, self.f_rows, self.f_cols
        OH, OW = int(self.num_row_patches), int(self.num_col_patches)
        w = self.learned_params["weights"]
        gw = grad_buffer(self, "weights", (K, C, R, S))
        s = l2_strength(self.weight_regulariser)
        if self._narrow:
            lat = G.lattice if G.lattice == 2 else 1
            g = G.g_compact if lat == 2 else to_nhwc(G.g)
            nb = lib.dk_conv2d_wgrad_narrow_workspace_bytes(N, Cp, H, W, K, R, S, self.stride, self.padding, OH, OW)
            r = lib.dk_conv2d_wgrad_bnbwd_narrow_f32(g.data_ptr(), G.x.data_ptr(), x.data_ptr(), N, Cp, H, W, K, R, S,
                                                     self.stride, self.padding, OH, OW, *G.bnbwd_args(), lat,
                                                     w.data_ptr() if s else 0, s or 0.0, gw.data_ptr(),
                                                     workspace.get(nb), nb, st)
            if r:
                raise RuntimeError(f"dk_conv2d_wgrad_bnbwd_narrow_f32 failed: {r}")
            if s is None:
                add_regulariser_grad(gw, w, self.weight_regulariser)
            return
        g = to_nhwc(G.g)
        nb = lib.dk_conv2d_wgrad_workspace_bytes(N, OH, OW, K, Cp, R, S)
        lib.dk_conv2d_wgrad_bnbwd_f32(g.data_ptr(), G.x.data_ptr(), x.data_ptr(), N, H, W, Cp, C, K, R, S,
                                      self.stride, self.padding, OH, OW, *G.bnbwd_args(), w.data_ptr() if s else 0,
                                      s or 0.0, gw.data_ptr(), workspace.get(nb), nb,
                                      *(self._bn_in.bn_args() if self._bn_in is not None else (0, 0, 0, 0, 0)), st)
        if s is None:
            add_regulariser_grad(gw, w, self.weight_regulariser)

    def backward(self, upstream_dx, need_dx=True):
        self._require_on_gpu()
        if isinstance(upstream_dx, BNGrad):
            if not need_dx and self._takes_bn_grad(upstream_dx.x):
                self._wgrad_bn_grad(upstream_dx)
                return None
            upstream_dx = upstream_dx.materialize()
        st = stream_handle()
        dy = to_nhwc(upstream_dx)
        x = self.X
        N, Cp, H, W = x.shape
        K, C, R, S = self.num_filters, self.filter_chans, self.f_rows, self.f_cols
        OH, OW = int(self.num_row_patches), int(self.num_col_patches)
        w = self.learned_params["weights"]
        P = N * OH * OW
        # the weight gradient runs on the side stream (_hip.weight_grad_stream)
        with weight_grad_stream(dy, x, *self._bn_tensors()):
            sst = stream_handle()
            if self.with_bias:
                gb = grad_buffer(self, "bias", (K,))
                nb = lib.dk_colsum_workspace_bytes(P, K)
                lib.dk_colsum_f32(dy.data_ptr(), P, K, gb.data_ptr(), workspace.get(nb), nb, sst)
            # weight gradient (+ l2 folded in, convolution.py:93-100)
            gw = grad_buffer(self, "weights", (K, C, R, S))
            s = l2_strength(self.weight_regulariser)
            if self._narrow:
                nb = lib.dk_conv2d_wgrad_narrow_workspace_bytes(N, Cp, H, W, K, R, S, self.stride, self.padding,
                                                                OH, OW)
                r = lib.dk_conv2d_wgrad_narrow_f32(dy.data_ptr(), x.data_ptr(), N, Cp, H, W, K, R, S, self.stride,
                                                   self.padding, OH, OW, w.data_ptr() if s else 0, s or 0.0,
                                                   gw.data_ptr(), workspace.get(nb), nb, sst)
                if r:
                    raise RuntimeError(f"dk_conv2d_wgrad_narrow_f32 failed: {r}")
            elif self._bn_in is not None:
                nb = lib.dk_conv2d_wgrad_workspace_bytes(N, OH, OW, K, Cp, R, S)
                lib.dk_conv2d_wgrad_bnx_f32(dy.data_ptr(), x.data_ptr(), N, H, W, Cp, C, K, R, S, self.stride,
                                            self.padding, OH, OW, w.data_ptr() if s else 0, s or 0.0, gw.data_ptr(),
                                            workspace.get(nb), nb, *self._bn_in.bn_args(), sst)
            else:
                nb = lib.dk_conv2d_wgrad_workspace_bytes(N, OH, OW, K, Cp, R, S)
                lib.dk_conv2d_wgrad_f32(dy.data_ptr(), x.data_ptr(), N, H, W, Cp, C, K, R, S, self.stride,
                                        self.padding, OH, OW, w.data_ptr() if s else 0, s or 0.0, gw.data_ptr(),
                                        workspace.get(nb), nb, sst)
            if s is None:
                add_regulariser_grad(gw, w, self.weight_regulariser)
        if not need_dx:
            return None
        # input gradient (convolution.py:101-117); shape = the forward input's shape
        Hin, Win = self.input_shape[2], self.input_shape[3]
        dx = empty_nhwc(N, C, Hin, Win)
        if self.stride == 1 and K % 4 == 0:
            w_crsk = torch.empty((C, R, S, K), dtype=torch.float32, device=x.device)
            lib.dk_conv_weight_crsk_f32(w.data_ptr(), K, C, R, S, w_crsk.data_ptr(), st)
            lib.dk_conv2d_dgrad_f32(dy.data_ptr(), N, OH, OW, K, w_crsk.data_ptr(), C, R, S, self.padding,
                                    dx.data_ptr(), Hin, Win, st)
        elif self.stride > 1 and lib.dk_conv2d_dgrad_subpixel_workspace_bytes(K, C, R, S, self.stride, self.padding):
            # strided, narrow input (the stem): sub-pixel gather, no column matrix
            nb = lib.dk_conv2d_dgrad_subpixel_workspace_bytes(K, C, R, S, self.stride, self.padding)
            lib.dk_conv2d_dgrad_subpixel_f32(dy.data_ptr(), N, OH, OW, K, w.data_ptr(), C, R, S, self.stride,
                                             self.padding, dx.data_ptr(), Hin, Win, workspace.get(nb), nb, st)
        else:
            # any stride (and stride 1 with K % 4 != 0): one implicit GEMM per sub-pixel phase of dx,
            # dy zero-padded to a multiple of 4 channels for the 16-byte loads
            Kp = -(-K // 4) * 4
            dyp = dy if Kp == K else to_nhwc(dy, cpad=4)
            nb = lib.dk_conv2d_dgrad_phase_workspace_bytes(K, C, R, S, self.stride)
            lib.dk_conv2d_dgrad_phase_f32(dyp.data_ptr(), N, OH, OW, Kp, K, w.data_ptr(), C, R, S, self.stride,
                                          self.padding, dx.data_ptr(), Hin, Win, workspace.get(nb), nb, st)
        return dx

    # -- checkpoint hooks (h5py is not available in this image; kept for API parity) ------

    def save_to_h5(self, open_f, save_grads=True):
        from ..network.checkpoint import save_layer
        save_layer(self, open_f, save_grads)

    def load_from_h5(self, open_f, load_grads=True):
        from ..network.checkpoint import load_layer
        load_layer(self, open_f, load_grads)
