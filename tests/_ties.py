"""ReLU decisions of the GPU path, replayed in the oracles (whole-network parity at any seed).

A ReLU whose input lies within fp32 rounding of zero may switch sides between two correct fp32
evaluations of the same network (activations.py:41: mask = out > 0), and a single switched
element moves the BatchNorm backward that follows by ~1/count (batch_norm.py:125-156) -- far past
a 1e-4 normwise bound at small batch.  So the whole-network tests take the GPU's own decision at
every ReLU (the mask it applies in forward and backward, read from the state the step leaves:
the stored mask, the join output y > 0, or the deferred BN+ReLU output recomputed with the same
arithmetic as its consumers) and replay it in the fp64 and fp32 oracles (oracle/net.py
OReLU.replay).  The replay is only honest if every place where the GPU and the fp64 oracle
disagree is a tie: ``tie_report`` lists the disagreements with the fp64 pre-activation there,
measured against the ReLU's own scale, and the tests bound it (TIE_REL).
"""
from __future__ import annotations

import numpy as np
import torch

# A disagreement counts as a tie when |z64| <= TIE_REL * rms_c(z64), z64 the fp64 oracle's
# pre-activation and rms_c its root mean square over the element's channel.  The GPU's
# pre-activations at res8 are ~1e-6 (relative) away from fp64 after 40 fp32 layers, so ties sit
# below ~1e-5 of the channel scale; a wrong value (a kernel bug) puts a disagreement at O(1).
TIE_REL = 1e-4


def _host(t):
    return t.detach().float().cpu().numpy()


def relu_pairs(layers, olayers):
    """(gpu ReLu, oracle OReLU) pairs in forward order, the residual blocks' joins included."""
    from dorknet_amd.layers.activations import ReLu
    out = []
    for l, ol in zip(layers, olayers):
        if isinstance(l, ReLu):
            out.append((l, ol))
        if hasattr(l, "layer_list"):
            out += relu_pairs(l.layer_list, ol.layer_list)
            out.append((l.post_skip_activation, ol.post_skip_activation))
    return out


def gpu_relu_state(relu):
    """(mask, pre) of a GPU ReLu after a training forward: the bool mask its backward applies and,
    where the step leaves the operands, the fp32 pre-activation it was decided on (else None)."""
    from dorknet_amd import _hip
    from dorknet_amd._tensor import empty_nhwc
    from dorknet_amd.layers._bn_input import BNOut
    fo = relu._fused_out
    if relu._mask is not None:
        return _host(relu._mask) != 0, None
    if relu._join_y is not None:
        return _host(relu._join_y) > 0, None
    if isinstance(fo, BNOut):
        # the deferred BN+ReLU output: its consumers (and the backward's mask recomputation) apply
        # bn_out to x on load, bit-identical to dk_bn_apply_f32 (layers/_bn_input.py)
        x = fo.x
        z = empty_nhwc(*x.shape)
        y = empty_nhwc(*x.shape)
        for relu_flag, out in ((0, z), (int(fo.relu), y)):
            _hip.lib.dk_bn_apply_f32(x.data_ptr(), x.numel(), x.shape[1], fo.mean.data_ptr(), fo.invstd.data_ptr(),
                                     fo.gamma.data_ptr(), fo.beta.data_ptr(), relu_flag, out.data_ptr(), 0,
                                     _hip.stream_handle())
        torch.cuda.synchronize()
        return _host(y) > 0, _host(z)
    if isinstance(fo, torch.Tensor):
        return _host(fo) > 0, None
    raise AssertionError("ReLu {}: no training-mode forward state".format(relu.layer_name))


def replay_gpu_decisions(net, onets):
    """Read every GPU ReLU's decision after net.forward and arm the oracles' ReLUs to replay it in
    their next forward.  Returns [(name, mask, pre_gpu)] in forward order."""
    states = []
    pairs = [relu_pairs(net.layers, o.layers) for o in onets]
    for i, (l, _) in enumerate(pairs[0]):
        mask, pre = gpu_relu_state(l)
        states.append((l.layer_name, mask, pre))
        for p in pairs:
            p[i][1].replay = mask
    return states


def tie_report(states, onet):
    """After the oracles' forward: the disagreements between the GPU's decision and the fp64
    oracle's own (z64 > 0).  Returns (count, worst) with worst = max |z64| / rms_c(z64) over the
    disagreements, and a list of (relu, index, z64, z_gpu, rel) for the message."""
    orelus = [ol for _, ol in relu_pairs_oracle(onet.layers)]  # (names may repeat: paired by position)
    assert len(orelus) == len(states)
    count, worst, rows = 0, 0.0, []
    for (name, mask, pre), ol in zip(states, orelus):
        z64 = np.asarray(ol.pre, np.float64)
        own = z64 > 0
        bad = np.argwhere(own != mask)
        if not len(bad):
            continue
        axis = (0, 2, 3) if z64.ndim == 4 else (0,)
        rms = np.sqrt((z64 ** 2).mean(axis=axis))
        for idx in bad:
            idx = tuple(idx)
            rel = abs(z64[idx]) / max(rms[idx[1]], 1e-300)
            count += 1
            worst = max(worst, rel)
            rows.append((name, idx, float(z64[idx]), None if pre is None else float(pre[idx]), rel))
    rows.sort(key=lambda r: -r[-1])
    return count, worst, rows


def relu_pairs_oracle(olayers):
    """(None, OReLU) pairs of an oracle network, in the order relu_pairs uses."""
    from oracle.net import OReLU
    out = []
    for ol in olayers:
        if isinstance(ol, OReLU):
            out.append((None, ol))
        if hasattr(ol, "layer_list"):
            out += relu_pairs_oracle(ol.layer_list)
            out.append((None, ol.post_skip_activation))
    return out
