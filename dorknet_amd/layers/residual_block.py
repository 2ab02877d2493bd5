"""Residual block (reference: layers/residual_block.py).

``forward``: post_skip_activation(layer_list(X) + skip_projection(X)) -- the join and a
ReLU post-activation run as one pass (ReLu.forward_add); BN+ReLU pairs inside the chain
run fused.  ``backward``: the activation's backward, the chain in reverse, plus the skip
branch (or identity), summed (:86-97).  ``regulariser_forward`` sums the chain's terms
only -- the skip projection's l2 is *not* in the loss (:78-84), while its gradient still
gets the l2 term in its own backward; and SGDMomentum never updates the skip projection
(optimisers/SGDMomentum.py:7-14).  Both quirks are kept.
"""
from __future__ import annotations


from .._env import enabled, getenv
from .._hip import branch_stream_enabled, lib, on_branch, resolve, stream_handle
from .._tensor import empty_nhwc, to_nhwc
from ._bn_input import JoinOut, accepts_bn_input, materialize
from ._chain import chain_backward, chain_forward, execute, fusion_enabled, notify_backward_done
from .activations import ReLu
from .batch_norm import BatchNormLayer
from .convolution import ConvLayer
from .depthwise_convolution import DepthwiseConvLayer
from .layer import Layer
from .pointwise_convolution import PointwiseConvLayer


def _add(a, b):
    a, b = to_nhwc(a), to_nhwc(b)
    if a.shape != b.shape:
        raise ValueError("residual backward shape mismatch: {} vs {}".format(tuple(a.shape), tuple(b.shape)))
    out = empty_nhwc(*a.shape)
    lib.dk_add_f32(a.data_ptr(), b.data_ptr(), a.numel(), 0, out.data_ptr(), 0, stream_handle())
    return out


class ResidualBlock(Layer):
    """
    A block with a skip connection around the provided layer_list.  The output of
    layer_list[-1] must have the same shape as skip_projection(X) because they are joined
    by addition - skip_projection=None means an identity projection.  The nonlinear
    activation (if not None) is applied after the join.
    """

    def __init__(self, layer_name, layer_list=None, skip_projection=None, post_skip_activation=None):
        super().__init__(layer_name)
        self.layer_list = layer_list
        self.skip_projection = skip_projection
        self.post_skip_activation = post_skip_activation
        if layer_list is None:
            self.layer_list = []
        self._steps = None

    def __repr__(self):
        return "ResidualBlock({}, layer_list={}, skip_projection={}, post_skip_activation={})".format(
            self.layer_name, self.layer_list, self.skip_projection, self.post_skip_activation)

    def to_gpu(self):
        if self.is_on_gpu:
            print("Layer already on GPU, ignoring request")
            return
        for layer in self.layer_list:
            layer.to_gpu()
        if self.skip_projection is not None:
            self.skip_projection.to_gpu()
        if self.post_skip_activation is not None:
            self.post_skip_activation.to_gpu()
        self.is_on_gpu = True

    # X may be a BNOut (the block input's BatchNorm applied on load by the chain's first layer,
    # the skip projection and the join); the chain's last BatchNorm is applied by the join.
    accepts_bn_input = True

    produces_join = True  # forward(..., join_out=True) may return its output as a JoinOut

    def takes_join_input(self):
        """forward(JoinOut): the previous block's join is formed by this block's first layer as it
        loads its input (DepthwiseConvLayer._forward_join) -- a depthwise first layer of the right
        geometry, fusion on.  The skip operand is then that written y: an identity skip reads it
        at the join, a skip projection (a downsampling block, whose first layer is the stride-2
        depthwise) reads it once the first layer has written it."""
        first = self.layer_list[0] if self.layer_list else None
        if not (isinstance(first, DepthwiseConvLayer) and first.join_geometry_ok() and fusion_enabled()
                and getenv("DORKNET_FUSE_JOIN_FWD") != "0"):
            return False
        return self.skip_projection is None or first.stride == 2

    def forward(self, X, test_mode=False, join_out=False):
        """join_out: the next layer takes its input as a JoinOut (takes_join_input): the join is
        handed over unwritten instead of running the join pass."""
        post = self.post_skip_activation
        join_fused = type(post) is ReLu
        skip = self.skip_projection
        if isinstance(X, JoinOut) and not self.takes_join_input():
            X = X.materialize()
        branch = skip is not None and branch_stream_enabled()
        skip_late = skip is not None and isinstance(X, JoinOut)
        if skip_late:
            # the chain's first layer writes the join as it loads it; the skip projection starts
            # once it has (on the branch stream, beside the rest of the chain)
            J, launched = X, []

            def after_first(group, out):
                if not launched:
                    launched.append(self._skip_forward(J.materialize(), test_mode, branch))
                return False
            X_tmp, self._steps, _ = execute(self.layer_list, X, test_mode=test_mode, out_accepts=join_fused,
                                            visit=after_first)
            skippee = launched[0]
        else:
            if branch:
                # the skip projection on the branch stream, beside the chain; joined at the join
                skippee = self._skip_forward(X, test_mode, True)
            X_tmp, self._steps = chain_forward(self.layer_list, X, test_mode=test_mode, out_accepts=join_fused)
            if skip is None:
                skippee = X
            elif not branch:
                skippee = self._skip_forward(X, test_mode, False)
        if branch:
            skippee = skippee.resolve()
        if join_fused:
            # a JoinOut consumer (takes_join_input: a depthwise layer) takes the join's mask in its
            # fused backward as y > 0; the mask is stored only when that fusion is off
            need_mask = not (enabled("DORKNET_FUSE_JOIN") and getenv("DORKNET_JOIN_MASK") != "1")
            return post.forward_add(X_tmp, skippee, test_mode=test_mode, defer=join_out, need_mask=need_mask)
        return post.forward(_add(materialize(X_tmp), materialize(skippee)), test_mode=test_mode)

    def _skip_forward(self, X, test_mode, branch):
        """skip_projection(X), on the branch stream when `branch` (a Branch to resolve())."""
        skip = self.skip_projection
        Xs = X if accepts_bn_input(skip) else materialize(X)
        if not branch:
            return skip.forward(Xs, test_mode=test_mode)
        with on_branch(Xs) as b:
            return b.done(skip.forward(Xs, test_mode=test_mode))

    def regulariser_forward(self):
        regularisation = 0
        for l in self.layer_list:
            if hasattr(l, "regulariser_forward"):
                regularisation += l.regulariser_forward()
        return regularisation

    accepts_join = True  # backward(dy, join=relu): the previous block's join may ride on the first dgrad

    def backward(self, upstream_dx, join=None):
        """`join` (optional): the previous block's post-skip ReLu -- this block's input is that
        join's output, so the chain's first layer may apply its backward in the dgrad epilogue
        (DepthwiseConvLayer.accepts_join; the ReLu then passes the gradient through)."""
        joined_dx = self.post_skip_activation.backward(upstream_dx)
        # the skip branch's gradient goes in first, so the chain's first layer can add it in
        # its dgrad epilogue instead of a separate join pass (residual_block.py:94-97)
        skip = self.skip_projection
        lattice = skip is not None and fusion_enabled() and self._lattice_skip(join)
        if skip is None:
            skip_dx = joined_dx
        elif branch_stream_enabled():
            # the skip gradient on the branch stream, beside the chain's backward; the chain's
            # first dgrad (or the separate add) waits for it
            with on_branch(joined_dx) as b:
                skip_dx = b.done(skip.backward(joined_dx, lattice_out=True) if lattice else skip.backward(joined_dx))
        elif lattice:
            # a strided skip's gradient stays its compact lattice: the first dgrad adds it there
            skip_dx = skip.backward(joined_dx, lattice_out=True)
        else:
            skip_dx = skip.backward(joined_dx)
        if skip is not None:
            notify_backward_done((skip,))
        if fusion_enabled():
            return chain_backward(self._steps, joined_dx, residual=skip_dx, join=join)
        return _add(chain_backward(self._steps, joined_dx), resolve(skip_dx))

    def _lattice_skip(self, join):
        """The skip projection may hand over its gradient as the stride-s lattice: it is a strided
        pointwise layer that can (lattice_ok), and the chain's first layer adds such a residual
        in its fused join dgrad (DepthwiseConvLayer.takes_lattice_residual).  DORKNET_LATTICE=0
        turns the hand-overs off."""
        skip = self.skip_projection
        if getenv("DORKNET_LATTICE") == "0" or not getattr(skip, "lattice_ok", None) or not skip.lattice_ok():
            return False
        first = self._steps[0][0] if self._steps else None
        f = getattr(first, "takes_lattice_residual", None)
        return bool(f is not None and f(join, skip.stride))

    def save_to_h5(self, open_f, save_grads=True):
        from ..network.checkpoint import save_layer
        save_layer(self, open_f, save_grads)

    def load_from_h5(self, open_f, load_grads=True):
        from ..network.checkpoint import load_layer
        load_layer(self, open_f, load_grads)


__all__ = ["ResidualBlock", "ConvLayer", "DepthwiseConvLayer", "PointwiseConvLayer", "ReLu", "BatchNormLayer"]
