"""Batch normalisation (reference: layers/batch_norm.py).

Training mode normalises with the batch statistics (population variance, eps = 1e-5),
keeps running **mean and std** (not var) with momentum ``run_momentum`` and first-batch
initialisation (batch_norm.py:76-89), and test mode uses the running statistics
(:101-115).  Backward follows the explicit formula of :125-174.

Implementation (dk_bn_* in libdorknet_hip.so): one fp64 statistics pass over X, a
finalize, an apply pass; backward = one reduce pass + one apply pass.  Only X and the
per-channel (mean, invstd) are kept for backward (the reference stores X_demean and
X_hat).  When a network/residual chain puts a plain ReLu right after this layer, the
pair runs fused (``forward_bn_relu`` / ``backward_bn_relu``): the ReLU is applied in the
same pass and its backward mask is recomputed from X.

With ``sync_group`` set (data-parallel SyncBN, see dorknet_amd.parallel), the per-channel
sums are all-reduced between the partial and finalize stages so every rank normalises
with full-batch statistics.
"""
from __future__ import annotations

import torch

from .._hip import fold_resources, lib, stream_handle, tickets, workspace
from .._tensor import BF16, act_dtype, as_device, empty_nhwc, rows, to_nhwc
from ._bn_input import BNGrad, BNOut, widen_lattice
from ._common import grad_buffer
from .layer import Layer


class BatchNormLayer(Layer):
    """
    https://arxiv.org/pdf/1502.03167.pdf
    """

    def __init__(self, layer_name, input_dimension=4,
                 incoming_chans=None, run_momentum=0.95, is_on_gpu=True):
        super().__init__(layer_name)
        import numpy as np
        self.eps = 1e-5
        self.input_dimension = input_dimension
        self.non_learned_params = {"running_mean": None, "running_std": None}
        self.run_momentum = run_momentum
        if self.input_dimension not in {2, 4}:
            raise ValueError("BatchNorm input_dimension should have length 2 or 4...")
        if self.input_dimension == 4:
            self.av_axis = (0, 2, 3)
        elif self.input_dimension == 2:
            self.av_axis = 0
        self.incoming_chans = incoming_chans
        self.sync_group = None
        if incoming_chans is not None:
            gamma = np.ones(incoming_chans, dtype=np.float32)
            beta = np.zeros(incoming_chans, dtype=np.float32)
            if self.input_dimension == 4:
                gamma = gamma[np.newaxis, :, np.newaxis, np.newaxis]
                beta = beta[np.newaxis, :, np.newaxis, np.newaxis]
            self.learned_params = {"gamma": gamma, "beta": beta}
            self.grads = {"gamma": np.zeros_like(gamma), "beta": np.zeros_like(beta)}
        else:
            self.learned_params = {}
            self.grads = {}

    def __repr__(self):
        return "BatchNormLayer({}, input_dimension={}, incoming_chans={}, run_momentum={})".format(
            self.layer_name, self.input_dimension, self.incoming_chans, self.run_momentum)

    # -- helpers -------------------------------------------------------------------------

    def _param_shape(self, C):
        return (1, C, 1, 1) if self.input_dimension == 4 else (C,)

    def _prep_input(self, X):
        if X.dim() == 4:
            x = to_nhwc(X)
            N, C, H, W = x.shape
            return x, N * H * W, C
        x = rows(X)
        return x, x.shape[0], x.shape[1]

    def _out_like(self, x):
        if x.dim() == 4:
            return empty_nhwc(*x.shape, dtype=x.dtype)
        return torch.empty_like(x)

    def _world(self):
        import torch.distributed as dist
        return dist.get_world_size(self.sync_group)

    def _persist(self, key, n, dev):
        """A per-layer fp32 device buffer reused every step: the batch statistics and the backward
        coefficients are rewritten by each forward / backward and read only within that step (every
        reader on another stream is joined into the main stream before the step ends), so a fresh
        allocation per call (~4 per layer and step) buys nothing but host time."""
        b = self.__dict__.get(key)
        if b is None or b.numel() != n or b.device != dev:
            b = torch.empty(n, dtype=torch.float32, device=dev)
            self.__dict__[key] = b
        return b

    def _stats_outputs(self, C, dev):
        """mean / std / invstd (this layer's per-step buffers) and the running statistics (allocated
        on the first batch)."""
        mean = self._persist("_dk_mean", C, dev)
        std = self._persist("_dk_std", C, dev)
        invstd = self._persist("_dk_invstd", C, dev)
        nlp = self.non_learned_params
        # _first_pending: an armed in-launch fold allocated the running statistics but did not run
        first = nlp["running_mean"] is None or getattr(self, "_first_pending", False)
        if nlp["running_mean"] is None:
            nlp["running_mean"] = torch.empty(self._param_shape(C), dtype=torch.float32, device=dev)
            nlp["running_std"] = torch.empty(self._param_shape(C), dtype=torch.float32, device=dev)
        rm, rs = as_device(nlp["running_mean"]), as_device(nlp["running_std"])
        nlp["running_mean"], nlp["running_std"] = rm, rs
        return mean, std, invstd, rm, rs, first

    def arm_stats_fold(self, part, P):
        """Arm the producer's launch that writes `part` ([rows, 2, C] partial sums over P pixels)
        to finalize this layer's batch statistics itself (dk_bn_fold_arm_stats, fold_tail.h).
        Returns the (mean, std, invstd) it will write, or None (SyncBN, or a mismatch)."""
        C = part.shape[-1]
        if self.sync_group is not None or part.dtype != torch.float64:
            return None
        mean, std, invstd, rm, rs, first = self._stats_outputs(C, part.device)
        self._first_pending = bool(first)
        # the producer's launch rewrites mean / std / invstd before this layer's forward runs: records
        # of the previous forward (BNOut, layers/_bn_input.py) are stale from here on
        self._dk_gen = getattr(self, "_dk_gen", 0) + 1
        t, nt, sc, nsc = fold_resources.get()
        lib.dk_bn_fold_arm_stats(part.data_ptr(), part.shape[0], C, float(P), float(self.eps),
                                 float(self.run_momentum), int(first), mean.data_ptr(), std.data_ptr(),
                                 invstd.data_ptr(), rm.data_ptr(), rs.data_ptr(), t, nt, sc, nsc)
        return mean, std, invstd

    def arm_bwd_fold(self, part):
        """Arm the consumer's backward launch that writes stage 1 of this layer's backward into
        `part` to finalize dgamma, dbeta and k12 itself (dk_bn_fold_arm_bwd).  Returns k12, or
        None (SyncBN: the partial sums are all-reduced first)."""
        x = getattr(self, "X", None)
        if self.sync_group is not None or x is None or part.dtype != torch.float64:
            return None
        C = x.shape[1]
        if part.shape[-1] != C:
            return None
        P = x.numel() // C
        gamma, beta = self.learned_params["gamma"], self.learned_params["beta"]
        dgamma = grad_buffer(self, "gamma", gamma.shape)
        dbeta = grad_buffer(self, "beta", beta.shape)
        k12 = self._persist("_dk_k12", 2 * C, x.device)
        t, nt, sc, nsc = fold_resources.get()
        lib.dk_bn_fold_arm_bwd(part.data_ptr(), part.shape[0], C, float(P), dgamma.data_ptr(), dbeta.data_ptr(),
                               k12.data_ptr(), t, nt, sc, nsc)
        return k12

    def _stats(self, x, P, C, st, partials=None):
        dev = x.device
        if partials is not None and getattr(partials, "folded", None) is not None:
            # the producer's launch folded them (fold_tail.h) -- running statistics included
            return partials.folded
        mean, std, invstd, rm, rs, first = self._stats_outputs(C, dev)
        self._first_pending = False
        if partials is not None and partials.part.shape[-1] != C:
            partials = None
        if partials is not None:
            nb = lib.dk_bn_partials_workspace_bytes(partials.rows, C)
            ws = workspace.get(nb)
        else:
            nb = lib.dk_bn_stats_workspace_bytes(P, C)
            ws = workspace.get(nb)
        if self.sync_group is None:
            if partials is not None:
                lib.dk_bn_stats_from_partials_f32(partials.part.data_ptr(), partials.rows, C, float(P),
                                                  float(self.eps), float(self.run_momentum), int(first),
                                                  mean.data_ptr(), std.data_ptr(), invstd.data_ptr(), rm.data_ptr(),
                                                  rs.data_ptr(), ws, nb, tickets.get(lib.dk_bn_fold_tickets_count(C)),
                                                  st)
            else:
                stats_fn = lib.dk_bn_stats_bf16 if x.dtype == BF16 else lib.dk_bn_stats_f32
                stats_fn(x.data_ptr(), P, C, float(self.eps), float(self.run_momentum), int(first),
                         mean.data_ptr(), std.data_ptr(), invstd.data_ptr(), rm.data_ptr(), rs.data_ptr(), ws, nb,
                         st)
        else:
            import torch.distributed as dist
            sums = torch.empty(2 * C, dtype=torch.float64, device=dev)
            if partials is not None:
                lib.dk_bn_reduce_partials_f64(partials.part.data_ptr(), partials.rows, C, sums.data_ptr(), ws, nb,
                                              st)
            else:
                lib.dk_bn_stats_partial_f64(x.data_ptr(), P, C, ws, nb, st)
                lib.dk_bn_collapse_f64(ws, lib.dk_bn_partial_blocks(P, C), C, sums.data_ptr(), st)
            dist.all_reduce(sums, group=self.sync_group)
            count = float(P) * self._world()
            lib.dk_bn_stats_finalize_f32(sums.data_ptr(), 1, C, count, float(self.eps), float(self.run_momentum),
                                         int(first), mean.data_ptr(), std.data_ptr(), invstd.data_ptr(),
                                         rm.data_ptr(), rs.data_ptr(), st)
        return mean, std, invstd

    # -- forward -------------------------------------------------------------------------

    def _normalisation(self, X, test_mode, stats=None):
        """(x, mean, invstd): batch statistics in training mode (kept for backward), the
        running statistics in test mode (batch_norm.py:76-115).  `stats`: partial sums of X
        already computed by the layer that produced it (layers/_chain.StatsRequest)."""
        self._require_on_gpu()
        st = stream_handle()
        x, P, C = self._prep_input(as_device(X, act_dtype(X)))
        if x.dtype == BF16 and (x.dim() != 4 or self.sync_group is not None):
            raise NotImplementedError("bf16 storage: 4-D inputs, local statistics only")
        self.input_shape = tuple(x.shape)
        self._pending_bwd = None
        if not test_mode:
            # mean / std / invstd are this layer's persistent buffers (_persist), and the running
            # statistics are updated in place, by every training forward: self.std, and the BNOut /
            # BNGrad records of an earlier forward, alias them.  The generation counter lets BNOut
            # detect a stale use (layers/_bn_input.py); a test-mode forward rewrites neither.
            self._dk_gen = getattr(self, "_dk_gen", 0) + 1
            mean, std, invstd = self._stats(x, P, C, st, stats)
            self.X = x
            self._mean, self._invstd = mean, invstd
            self.std = std.view(self._param_shape(C))
        else:
            rm = as_device(self.non_learned_params["running_mean"])
            rs = as_device(self.non_learned_params["running_std"]).contiguous()
            mean = rm.contiguous()
            invstd = torch.empty(C, dtype=torch.float32, device=x.device)
            lib.dk_bn_infer_params_f32(rs.data_ptr(), C, invstd.data_ptr(), st)
        return x, mean, invstd

    def _forward(self, X, test_mode, relu, stats=None):
        x, mean, invstd = self._normalisation(X, test_mode, stats)
        gamma, beta = self.learned_params["gamma"], self.learned_params["beta"]
        y = self._out_like(x)
        apply = lib.dk_bn_apply_bf16 if x.dtype == BF16 else lib.dk_bn_apply_f32
        apply(x.data_ptr(), x.numel(), x.shape[1], mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(),
              beta.data_ptr(), int(relu), y.data_ptr(), 0, stream_handle())
        return y

    def forward_deferred(self, X, relu_layer=None, test_mode=False, stats=None):
        """Statistics only; the normalisation (and the following ReLu, if given) is applied
        by the consumer as it loads its input (layers/_bn_input.py)."""
        x, mean, invstd = self._normalisation(X, test_mode, stats)
        out = BNOut(x, mean, invstd, self.learned_params["gamma"], self.learned_params["beta"],
                    relu_layer is not None, owner=self)
        if relu_layer is not None:
            relu_layer._attach_fused(out, test_mode)
        return out

    def forward(self, X, test_mode=False, use_express=False, stats=None):
        """X.shape = (batch_size, channel, height, width) or (batch_size, features)."""
        return self._forward(X, test_mode, relu=False, stats=stats)

    def forward_bn_relu(self, X, relu_layer, test_mode=False, stats=None):
        """BN followed by ReLU in one pass (activations.py:37-42 fused into the apply)."""
        y = self._forward(X, test_mode, relu=True, stats=stats)
        relu_layer._attach_fused(y, test_mode)
        return y

    # -- backward ------------------------------------------------------------------------

    def _backward(self, upstream_dx, relu, defer=False):
        """defer: when the coefficients come from a separate reduction (the partial sums of the
        consumer's dgrad epilogue, or the synchronised path), return a BNGrad and leave the
        apply to the producer of this layer's input (chain_backward)."""
        self._require_on_gpu()
        st = stream_handle()
        x = self.X
        lattice = getattr(upstream_dx, "_dk_lattice", 1)  # a compact stride-s lattice gradient (widen elided)
        dy = to_nhwc(upstream_dx) if x.dim() == 4 else rows(upstream_dx)
        bf = x.dtype == BF16
        if bf and dy.dtype != BF16:
            raise ValueError("{}: bf16 activations need a bf16 gradient".format(self.layer_name))
        C = x.shape[1]
        P = x.numel() // C
        gamma, beta = self.learned_params["gamma"], self.learned_params["beta"]
        dgamma = grad_buffer(self, "gamma", gamma.shape)
        dbeta = grad_buffer(self, "beta", beta.shape)
        dx = self._out_like(x)
        pending, self._pending_bwd = getattr(self, "_pending_bwd", None), None
        if lattice > 1 and not (defer and not bf and pending is not None and pending[0] is upstream_dx):
            # only a deferred hand-over keeps the lattice form: everything else takes the dense gradient
            dy, lattice, pending = widen_lattice(dy, lattice, x.shape), 1, None
        if pending is not None and pending[0].data_ptr() == dy.data_ptr() and pending[0].shape == dy.shape:
            # stage 1 was computed by the consumer's dgrad epilogue (layers/_bn_input.py)
            part = pending[1]
            nrows = part.shape[0]
            k12 = pending[2]
            nb = lib.dk_bn_partials_workspace_bytes(nrows, C)
            ws = workspace.get(nb)
            if k12 is not None:
                pass  # folded (and dgamma / dbeta written) inside the consumer's launch
            elif self.sync_group is None:
                k12 = self._persist("_dk_k12", 2 * C, x.device)
                lib.dk_bn_bwd_from_partials_f32(part.data_ptr(), nrows, C, float(P), dgamma.data_ptr(),
                                                dbeta.data_ptr(), k12.data_ptr(), ws, nb,
                                                tickets.get(lib.dk_bn_fold_tickets_count(C)), st)
            else:
                import torch.distributed as dist
                k12 = self._persist("_dk_k12", 2 * C, x.device)
                local = torch.empty(2 * C, dtype=torch.float64, device=x.device)
                lib.dk_bn_reduce_partials_f64(part.data_ptr(), nrows, C, local.data_ptr(), ws, nb, st)
                glob = local.clone()
                dist.all_reduce(glob, group=self.sync_group)
                lib.dk_bn_bwd_finalize_f32(local.data_ptr(), 1, glob.data_ptr(), 1, C, float(P) * self._world(),
                                           dgamma.data_ptr(), dbeta.data_ptr(), k12.data_ptr(), st)
            if defer:
                return BNGrad(dy, x, self._mean, self._invstd, gamma, beta, relu, k12, lattice=lattice)
            (lib.dk_bn_bwd_apply_bf16 if bf else lib.dk_bn_bwd_apply_f32)(
                x.data_ptr(), dy.data_ptr(), x.numel(), C, self._mean.data_ptr(), self._invstd.data_ptr(),
                gamma.data_ptr(), beta.data_ptr(), int(relu), k12.data_ptr(), dx.data_ptr(), st)
        elif self.sync_group is None:
            nb = lib.dk_bn_bwd_workspace_bytes(P, C)
            (lib.dk_bn_bwd_bf16 if bf else lib.dk_bn_bwd_f32)(
                x.data_ptr(), dy.data_ptr(), P, C, self._mean.data_ptr(), self._invstd.data_ptr(), gamma.data_ptr(),
                beta.data_ptr(), int(relu), dgamma.data_ptr(), dbeta.data_ptr(), dx.data_ptr(), workspace.get(nb), nb,
                st)
        else:
            import torch.distributed as dist
            nb = lib.dk_bn_workspace_bytes(P, C)
            ws = workspace.get(nb)
            lib.dk_bn_bwd_partial_f64(x.data_ptr(), dy.data_ptr(), P, C, self._mean.data_ptr(),
                                      self._invstd.data_ptr(), gamma.data_ptr(), beta.data_ptr(), int(relu), ws, nb,
                                      st)
            nblk = lib.dk_bn_partial_blocks(P, C)
            local = torch.empty(2 * C, dtype=torch.float64, device=x.device)
            glob = torch.empty(2 * C, dtype=torch.float64, device=x.device)
            lib.dk_bn_collapse_f64(ws, nblk, C, local.data_ptr(), st)
            lib.dk_bn_collapse_f64(ws, nblk, C, glob.data_ptr(), st)
            dist.all_reduce(glob, group=self.sync_group)
            k12 = self._persist("_dk_k12", 2 * C, x.device)
            lib.dk_bn_bwd_finalize_f32(local.data_ptr(), 1, glob.data_ptr(), 1, C, float(P) * self._world(),
                                       dgamma.data_ptr(), dbeta.data_ptr(), k12.data_ptr(), st)
            if defer and not bf:
                return BNGrad(dy, x, self._mean, self._invstd, gamma, beta, relu, k12)
            (lib.dk_bn_bwd_apply_bf16 if bf else lib.dk_bn_bwd_apply_f32)(
                x.data_ptr(), dy.data_ptr(), x.numel(), C, self._mean.data_ptr(), self._invstd.data_ptr(),
                gamma.data_ptr(), beta.data_ptr(), int(relu), k12.data_ptr(), dx.data_ptr(), st)
        return dx

    def backward(self, upstream_dx, defer=False):
        return self._backward(upstream_dx, relu=False, defer=defer)

    def backward_bn_relu(self, upstream_dx, relu_layer, defer=False):
        """Backward of the fused BN+ReLU pair; upstream_dx is the gradient w.r.t. the ReLU output."""
        return self._backward(upstream_dx, relu=True, defer=defer)

    def save_to_h5(self, open_f, save_grads=True):
        from ..network.checkpoint import save_layer
        save_layer(self, open_f, save_grads)

    def load_from_h5(self, open_f, load_grads=True):
        from ..network.checkpoint import load_layer
        load_layer(self, open_f, load_grads)
