"""BASELINE config 5 at its own batch (512): slices of the 16-unit bf16 depthwise-separable stack
(examples/mobilenet_stack.py; reference examples/imagenet_dogs_225_resnet_18_depsep.py:34-70)
run through the network's fused bf16 path -- bf16 activations, bf16 MFMA pointwise GEMMs with
fp32 accumulation -- against the torch fp64 twin (tests/_torch_twin.py) with the bf16 path's
roundings emulated.

Segments: the first unit (56 x 56 x 64, P = 1.6 M pixels per GEMM), a strided unit (res3_dw1:
stride-2 depthwise, 64 -> 128 pointwise at 28 x 28) and the last two units (512 channels at
7 x 7, the largest weight gradients).

The emulation rounds to bf16 where the GPU rounds: every tensor it stores in bf16 (layer outputs,
input gradients) and every bf16 MFMA operand (the pointwise weights, and a BatchNorm output
consumed on load by the pointwise layer).  A BatchNorm (+ReLU) applied on load by a depthwise
layer is computed in fp32 and not rounded, so the emulation does not round it either.

Tolerance: normwise relative 1e-2 against that emulation; where the
roundings themselves move a quantity by more (a sum with heavy cancellation, e.g. a BatchNorm's
shift gradient behind another BatchNorm), the bound is that movement -- the same
"excess over the arithmetic's own error" rule as the fp32 tests.  Each test also checks the
plain fp64 twin for the forward output.
"""
import numpy as np
import pytest
import torch

from tests._convert import rel_err
from tests._torch_twin import TorchTwin

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


class _Q(torch.autograd.Function):
    """Round to bf16 in forward (fwd=True) and round the incoming gradient in backward (bwd=True)."""

    @staticmethod
    def forward(ctx, x, fwd, bwd):
        ctx.bwd = bwd
        return x.to(BF16).to(x.dtype) if fwd else x.clone()

    @staticmethod
    def backward(ctx, g):
        return (g.to(BF16).to(g.dtype) if ctx.bwd else g), None, None


def _q(x, fwd=True, bwd=True):
    return _Q.apply(x, fwd, bwd)


class Bf16Twin(TorchTwin):
    """TorchTwin (fp64) with the bf16 path's roundings (module docstring)."""

    def __init__(self, layers, emulate=True):
        super().__init__(layers, np.float64)
        self.emulate = emulate

    def run(self, X, dY, input_grad=False):
        from dorknet_amd.layers.activations import ReLu
        from dorknet_amd.layers.batch_norm import BatchNormLayer
        from dorknet_amd.layers.depthwise_convolution import DepthwiseConvLayer
        from dorknet_amd.layers.pointwise_convolution import PointwiseConvLayer
        x = torch.tensor(np.asarray(X, np.float64), requires_grad=input_grad)
        h = x
        L = self.layers
        saved = {}
        for i, l in enumerate(L):
            if self.emulate and isinstance(l, PointwiseConvLayer):
                w = self._p(l, "weights")
                saved[l.layer_name] = w
                self.params[(l.layer_name, "weights")] = _q(w, True, False)  # bf16 MFMA operand
            h = self._layer(l, h)
            if self.emulate and isinstance(l, PointwiseConvLayer):
                self.params[(l.layer_name, "weights")] = saved[l.layer_name]
            if not self.emulate:
                continue
            nxt = L[i + 1] if i + 1 < len(L) else None
            if isinstance(l, (BatchNormLayer, ReLu)):
                # applied on load by the next layer: rounded as a pointwise MFMA operand, kept fp32
                # by a depthwise consumer; a ReLU after a BN is part of the same apply
                if isinstance(nxt, ReLu):
                    continue
                h = _q(h, fwd=not isinstance(nxt, DepthwiseConvLayer) or nxt is None, bwd=True)
            else:
                h = _q(h)  # a stored bf16 layer output; its gradient is stored bf16 too
        h.backward(torch.as_tensor(np.asarray(dY, np.float64)))
        grads = {}
        for (name, k), p in self.params.items():
            g = p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p)
            if k == "weights" and name in self.l2:
                g = g + self.l2[name] * p.detach()
            grads[(name, k)] = g.numpy()
        return h.detach().numpy(), (x.grad.numpy() if input_grad else None), grads


def _stack_layers(units, seed):
    from examples.mobilenet_stack import MobileNetStack
    np.random.seed(seed)
    net = MobileNetStack("mbs512")
    layers = net.layers[5 * units[0]:5 * units[1]]
    rng = np.random.default_rng(seed + 1)
    for l in layers:  # non-trivial BN affine parameters
        if "gamma" in (l.learned_params or {}):
            C = l.incoming_chans
            l.learned_params["gamma"] = (1 + 0.2 * rng.standard_normal((1, C, 1, 1))).astype(np.float32)
            l.learned_params["beta"] = (0.1 * rng.standard_normal((1, C, 1, 1))).astype(np.float32)
    return layers, rng


def _run_segment(units, in_shape, seed, monkeypatch, expect=()):
    from dorknet_amd.network.feed_forward_network import FeedForwardNetwork
    from tests.test_gpu_fullsize import Calls
    layers, rng = _stack_layers(units, seed)
    emu = Bf16Twin(layers)
    plain = Bf16Twin(layers, emulate=False)
    net = FeedForwardNetwork("seg")
    for l in layers:
        net.add_layer(l)
    net.to_gpu()
    calls = Calls(monkeypatch, ["dk_pwconv_fwd_ex_bf16", "dk_pwconv_dgrad_ex_bf16", "dk_pwconv_wgrad_bnx_bf16",
                                "dk_dwconv_fwd_ex_bf16", "dk_dwconv_dgrad_ex_bf16", "dk_dwconv_wgrad_bnx_bf16",
                                "dk_dwconv_bwd_s2_bnbwd_bf16"])
    X = torch.randn(in_shape, generator=torch.Generator().manual_seed(seed)).to(BF16)
    Xd = X.to("cuda").contiguous(memory_format=torch.channels_last)
    _, Y = net.forward(Xd, None)
    assert Y.dtype == BF16
    dY = torch.randn(tuple(Y.shape), generator=torch.Generator().manual_seed(seed + 2)).to(BF16)
    net.backward(dY.to("cuda").contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    assert {"dk_pwconv_fwd_ex_bf16"} | set(expect) <= calls.seen, calls.seen
    Yg = Y.float().cpu().numpy().astype(np.float64)
    grads = {(l.layer_name, k): l.grads[k].float().cpu().numpy().astype(np.float64)
             for l in layers for k in sorted(l.grads or {})}
    del Xd, Y
    torch.cuda.empty_cache()
    Xn, dYn = X.double().numpy(), dY.double().numpy()
    Ye, _, ge = emu.run(Xn, dYn)
    Yp, _, gp = plain.run(Xn, dYn)
    report = [("Y", rel_err(Yg, Ye), rel_err(Ye, Yp))]
    assert rel_err(Yg, Yp) <= 1e-2, ("Y vs plain fp64", rel_err(Yg, Yp))
    assert report[0][1] <= 1e-2, report[0]
    bad = []
    for key, want in ge.items():
        g = grads[key].reshape(want.shape)
        err, sens = rel_err(g, want), rel_err(want, gp[key])
        report.append((key, err, sens))
        if err > max(1e-2, sens):
            bad.append(report[-1])
    print("segment", units, "(name, GPU vs emulation, emulation vs plain fp64):")
    for r in report:
        print("  {:40s} {:.3e} {:.3e}".format(str(r[0]), r[1], r[2]))
    assert not bad, bad


def test_config5_first_unit_bs512(monkeypatch):
    _run_segment((0, 1), (512, 64, 56, 56), 51, monkeypatch)


def test_config5_strided_unit_bs512(monkeypatch):
    # the stride-2 depthwise backward runs fused (dk_dwconv_bwd_s2_bnbwd_bf16: dy never stored)
    _run_segment((4, 5), (512, 64, 56, 56), 53, monkeypatch, expect=["dk_dwconv_bwd_s2_bnbwd_bf16"])


def test_config5_last_two_units_bs512(monkeypatch):
    _run_segment((14, 16), (512, 512, 7, 7), 55, monkeypatch)
