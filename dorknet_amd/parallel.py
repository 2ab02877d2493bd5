"""Data parallelism over RCCL (one process per GPU, torch.distributed backend "nccl").

The reference is single-process.  Here each rank runs the same network
on its slice of the global batch; the only exchange is an all-reduce (average) of the
weight gradients, grouped into ~`bucket_bytes` buckets in reverse layer order and issued
asynchronously as soon as the backward pass has produced a bucket, so communication
overlaps the remaining backward work.  All gradient tensors are re-pointed into one flat
buffer so the kernels write straight into the buckets (no packing copies).

Batch norm: "local" (per-rank statistics, standard DDP semantics, the default for
throughput) or "sync" (SyncBN: per-channel sums all-reduced in forward and backward, so
the result equals single-process training on the concatenated batch).

Averaging: the reference's loss gradient is already divided by the local batch
(layers/losses.py:34), so the mean over ranks equals the full-batch gradient, and the
per-layer `+ strength * W` l2 term stays correct (a sum would scale it by world size).

Skip projections: the reference's SGDMomentum never updates them (optimisers/
SGDMomentum.py:7-14; `SGDMomentum(update_skip_projections=False)`, the default).  With the
same flag False here their gradients are left out of the buckets -- nothing reads them for
the update, so they stay rank-local (per-rank batch) instead of costing 172,032 floats of
all-reduce per step on ResNet-18-depsep.  Pass True together with the optimiser's True.

Stream ordering: weight gradients are written on two streams (the main stream -- BatchNorm
dgamma/dbeta, dense, the fused depthwise backward, the stem -- and the weight-gradient side
stream), and a downsampling block's skip projection runs its backward on the branch stream
(with side-stream weight gradients off, its weight gradient is written there).  A bucket's
all-reduce is issued from the side stream after making it wait for the main stream and the
branch stream, so RCCL reads the bucket only once every kernel issued so far on any of them
has written it.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ._hip import async_weight_grads, branch_stream, branch_stream_enabled, flush_wgrad_reduces, side_stream_context
from .layers._chain import backward_progress, chain_backward


def _all_layers(layers, skips=True):
    """Every layer (depth-first, forward order), including ResidualBlock children and
    (skips=True) skip projections."""
    out = []
    for l in layers:
        out.append(l)
        if hasattr(l, "layer_list"):
            out.extend(_all_layers(l.layer_list, skips))
            if skips and getattr(l, "skip_projection", None) is not None:
                out.append(l.skip_projection)
    return out


def grad_slots(network, skips=True):
    """[(top_level_index, layer, key, shape)] for every gradient, in forward order
    (skips=False: without the ResidualBlock skip projections' gradients)."""
    slots = []
    for ti, top in enumerate(network.layers):
        for l in _all_layers([top], skips):
            if not l.grads:
                continue
            for k, g in l.grads.items():
                slots.append((ti, l, k, tuple(g.shape)))
    return slots


def plan_buckets(slot_numels, slot_owner, bucket_bytes):
    """Group slots (given in forward order) into buckets in *reverse* order.
    Returns a list of buckets; each is (list_of_slot_indices, last_top_level_index) where
    the bucket is complete once backward has finished top-level layer `last...` (the
    smallest top-level index in it, since backward runs in reverse)."""
    buckets, cur, cur_bytes = [], [], 0
    for si in reversed(range(len(slot_numels))):
        cur.append(si)
        cur_bytes += 4 * slot_numels[si]
        if cur_bytes >= bucket_bytes:
            buckets.append(cur)
            cur, cur_bytes = [], 0
    if cur:
        buckets.append(cur)
    return [(b, min(slot_owner[s] for s in b)) for b in buckets]


class DataParallel:
    def __init__(self, network, group=None, batch_norm="local", bucket_bytes=2 << 20, device=None,
                 update_skip_projections=False):
        if batch_norm not in ("local", "sync"):
            raise ValueError("batch_norm must be 'local' or 'sync'")
        self.network = network
        self.group = group
        self.world = dist.get_world_size(group)
        self.batch_norm = batch_norm
        self.update_skip_projections = update_skip_projections
        # RCCL ("nccl") averages in the collective; gloo has no AVG: sum, then scale after wait
        self.native_avg = dist.get_backend(group) == "nccl"
        slots = grad_slots(network, skips=update_skip_projections)
        numels = [int(torch.Size(s[3]).numel()) for s in slots]
        self.total = sum(numels)
        dev = device if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                                 if torch.cuda.is_available() else torch.device("cpu"))
        self.flat = torch.zeros(self.total, dtype=torch.float32, device=dev)
        # offsets laid out in reverse order so each bucket is one contiguous range
        order = list(reversed(range(len(slots))))
        offs, off = {}, 0
        for si in order:
            offs[si] = off
            off += numels[si]
        for si, (_, layer, key, shape) in enumerate(slots):
            view = self.flat[offs[si]:offs[si] + numels[si]].view(shape)
            old = layer.grads[key]
            if isinstance(old, torch.Tensor):
                view.copy_(old.to(view.device))
            layer.grads[key] = view
        self.buckets = []
        for idxs, ready_after in plan_buckets(numels, [s[0] for s in slots], bucket_bytes):
            lo = min(offs[i] for i in idxs)
            hi = max(offs[i] + numels[i] for i in idxs)
            # the leaf layers whose gradients the bucket holds: it is complete once all of them
            # have been through backward (layers/_chain.py backward_progress)
            owners = frozenset(id(slots[i][1]) for i in idxs)
            self.buckets.append((lo, hi, ready_after, owners))
        self.launch_log = []  # (bucket index, layers reported so far) per launch, for tests
        # the optimiser must agree on which gradients are all-reduced (SGDMomentum checks too)
        network._dp_update_skip_projections = update_skip_projections
        opt_flag = getattr(network, "_opt_update_skip_projections", None)
        if opt_flag is not None and opt_flag != update_skip_projections:
            raise ValueError("DataParallel(update_skip_projections={}) disagrees with the optimiser's "
                             "update_skip_projections={}: skip-projection gradients would be updated "
                             "without being all-reduced (or all-reduced for nothing)".format(
                                 update_skip_projections, opt_flag))
        if batch_norm == "sync":
            from .layers.batch_norm import BatchNormLayer
            for l in _all_layers(network.layers):
                if isinstance(l, BatchNormLayer):
                    l.sync_group = group if group is not None else dist.group.WORLD
        self._works = []

    def _launch(self, lo, hi):
        flush_wgrad_reduces()  # reduces still recorded (batched) must land before the collective
        view = self.flat[lo:hi]
        op = dist.ReduceOp.AVG if self.native_avg else dist.ReduceOp.SUM
        if view.is_cuda:
            # issued from the weight-gradient side stream (when in use), after it has waited
            # for the main stream: the bucket's gradients are written on both (BatchNorm
            # dgamma/dbeta, dense, fused depthwise and stem weight gradients on main; the
            # GEMM weight gradients on the side stream), and the collective follows only the
            # stream it is issued from
            main = torch.cuda.current_stream()
            with side_stream_context():
                cur = torch.cuda.current_stream()
                if cur != main:
                    cur.wait_stream(main)
                if branch_stream_enabled():
                    # a skip projection's backward runs on the branch stream; without side-stream
                    # weight gradients its weight gradient is written there too
                    # (residual_block.py), so the collective also follows the branch stream
                    cur.wait_stream(branch_stream())
                work = dist.all_reduce(view, op=op, group=self.group, async_op=True)
        else:
            work = dist.all_reduce(view, op=op, group=self.group, async_op=True)
        self._works.append((work, view))

    def backward(self):
        """network.backward() with gradient all-reduce overlapped per bucket."""
        with async_weight_grads():
            self._backward()

    def _backward(self):
        net = self.network
        dy = net.loss_layer.backward()
        steps = net._steps
        pending = list(enumerate(self.buckets))
        done = set()
        self._works = []
        self.launch_log = []

        def progress(layers):
            # leaf layers (a chain step's, or a skip projection) whose gradients are now queued:
            # launch every bucket all of whose layers are done -- inside a residual block too, so
            # a block's buckets go out while the rest of its backward still runs
            done.update(id(l) for l in layers)
            still = []
            for bi, (lo, hi, _, owners) in pending:
                if owners <= done:
                    self._launch(lo, hi)
                    self.launch_log.append((bi, len(done)))
                else:
                    still.append((bi, (lo, hi, _, owners)))
            pending[:] = still

        with backward_progress(progress):
            chain_backward(steps, dy, need_input_grad=False)
        for bi, (lo, hi, _, _) in pending:
            self._launch(lo, hi)
            self.launch_log.append((bi, len(done)))
        self.finish()

    def allreduce_grads(self):
        """All-reduce every bucket now (for callers that ran network.backward() themselves)."""
        self._works = []
        for lo, hi, _, _ in self.buckets:
            self._launch(lo, hi)
        self.finish()

    def finish(self):
        for work, view in self._works:
            work.wait()
            if not self.native_avg:
                view.div_(self.world)
        self._works = []

    def broadcast_parameters(self, src=0):
        """Make every rank start from rank `src`'s parameters and running statistics."""
        for l in _all_layers(self.network.layers):
            for d in (l.learned_params, l.non_learned_params):
                if not d:
                    continue
                for v in d.values():
                    if isinstance(v, torch.Tensor):
                        dist.broadcast(v, src, group=self.group)
