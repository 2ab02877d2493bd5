"""The residual join formed by the next block's depthwise forward (dk_dwconv_fwd_join_f32).

residual_block.py:75 ends a block with y = ReLU(chain(X) + skip(X)); the next block's first layer (a
3 x 3 depthwise convolution, depthwise_convolution.py:85-102) reads y back at once.  The join entry
forms y as the depthwise window rows are loaded and stores it once.  Checked against the separate
join pass (dk_bn_add_f32) followed by dk_dwconv_fwd_ex_f32: y, its ReLU mask, the depthwise output and
its BatchNorm partial statistics bitwise, nothing written past y; and the network with the fusion on
vs off (DORKNET_FUSE_JOIN_FWD=0): loss and every gradient bitwise."""
import numpy as np
import pytest
import torch

from dorknet_amd._hip import lib, stream_handle

pytestmark = pytest.mark.gpu


def nhwc(a):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device="cuda").contiguous(
        memory_format=torch.channels_last)


def bn_params(C, rng):
    return [torch.as_tensor(v.astype(np.float32), device="cuda") for v in
            (rng.randn(C) * 0.3, rng.rand(C) + 0.5, 1 + 0.3 * rng.randn(C), 0.2 * rng.randn(C))]


@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("C,N,H,W", [(64, 2, 13, 11), (128, 3, 9, 16), (256, 2, 7, 7), (512, 2, 5, 6),
                                     (64, 4, 56, 56)])
@pytest.mark.parametrize("abn,brelu,bbn", [(True, 0, False), (True, 0, True), (True, 1, True), (False, 0, True)])
@pytest.mark.parametrize("stats", [True, False])
def test_join_fwd_matches_bn_add_then_dw(stride, C, N, H, W, abn, brelu, bbn, stats):
    rng = np.random.RandomState(C + N + H + 3 * stride + 5 * abn + 7 * bbn + brelu)
    a = nhwc(rng.randn(N, C, H, W) * 1.5)
    b = nhwc(rng.randn(N, C, H, W))
    pa, pb = bn_params(C, rng), bn_params(C, rng)
    w = torch.as_tensor((rng.randn(C, 3, 3) * 0.3).astype(np.float32), device="cuda")
    OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
    st = stream_handle()
    aa = (*(t.data_ptr() for t in pa), 0) if abn else (0, 0, 0, 0, 0)
    ba = (*(t.data_ptr() for t in pb), brelu) if bbn else (0, 0, 0, 0, 0)
    rows = lib.dk_dwconv_fwd_stats_rows(N, OH, OW, C, stride)
    # reference: the join pass, then the depthwise forward on its output
    y0 = nhwc(np.zeros((N, C, H, W)))
    m0 = torch.zeros((N, C, H, W), dtype=torch.uint8, device="cuda").contiguous(memory_format=torch.channels_last)
    lib.dk_bn_add_f32(a.data_ptr(), *aa, b.data_ptr(), *ba, a.numel(), C, 1, y0.data_ptr(), m0.data_ptr(), st)
    o0 = torch.full((N, C, OH, OW), float("nan"), device="cuda").contiguous(memory_format=torch.channels_last)
    p0 = torch.full((rows, 2, C), float("nan"), dtype=torch.float64, device="cuda") if stats else None
    lib.dk_dwconv_fwd_ex_f32(y0.data_ptr(), N, H, W, C, w.data_ptr(), 3, 3, stride, 1, 0, o0.data_ptr(), OH, OW,
                             0, 0, 0, 0, 0, p0.data_ptr() if stats else 0, st)
    # fused
    ybuf = torch.full((N * C * H * W + 4096,), 12345.0, device="cuda")
    y1 = ybuf[:N * C * H * W].view(N, H, W, C).permute(0, 3, 1, 2)
    m1 = torch.full((N, C, H, W), 7, dtype=torch.uint8, device="cuda").contiguous(memory_format=torch.channels_last)
    o1 = torch.full((N, C, OH, OW), float("nan"), device="cuda").contiguous(memory_format=torch.channels_last)
    p1 = torch.full((rows, 2, C), float("nan"), dtype=torch.float64, device="cuda") if stats else None
    rc = lib.dk_dwconv_fwd_join_f32(a.data_ptr(), *aa, b.data_ptr(), *ba, ybuf.data_ptr(), m1.data_ptr(), N, H, W, C,
                                    w.data_ptr(), stride, 0, o1.data_ptr(), OH, OW, p1.data_ptr() if stats else 0, st)
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert torch.equal(m0, m1)
    assert torch.equal(o0, o1)
    assert bool((ybuf[N * C * H * W:] == 12345.0).all())
    if stats:
        assert torch.equal(p0, p1)


@pytest.mark.parametrize("fwd_fuse", ["1", "0"])
@pytest.mark.parametrize("bwd_join", ["1", "0"])
def test_network_join_fwd_bitwise(monkeypatch, fwd_fuse, bwd_join):
    """ResNet-18-depsep training step (batch 4) with the blocks' joins formed by the next block's
    depthwise forward (stride 1, or stride 2 into a downsampling block) vs the join pass: loss, probabilities and every gradient bitwise --
    with the join's backward fused into the next depthwise backward (which takes the ReLU mask as
    y > 0, so the fused forward stores none) and without (DORKNET_FUSE_JOIN=0: the mask is stored)."""
    monkeypatch.setenv("DORKNET_FUSE_JOIN", bwd_join)
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    from dorknet_amd import _hip
    from tests._convert import all_layers
    X, _, onehot = synthetic_batch(4, seed=2)
    out = {}
    orig = _hip.lib.dk_dwconv_fwd_join_f32
    for fuse in (fwd_fuse, "0" if fwd_fuse == "1" else "1"):
        monkeypatch.setenv("DORKNET_FUSE_JOIN_FWD", fuse)
        seen = []
        monkeypatch.setattr(_hip.lib, "dk_dwconv_fwd_join_f32", lambda *a, seen=seen: seen.append(1) or orig(*a))
        np.random.seed(0)
        net = ResNet18("r18")
        net.to_gpu()
        loss, P = net.forward(torch.as_tensor(X, device="cuda"), torch.as_tensor(onehot, device="cuda"))
        net.backward()
        torch.cuda.synchronize()
        # every block's join but the last: res1 -> res2 ... res7 -> res8 (into res3 / res5 / res7 through their
        # stride-2 depthwise forward, the skip projection then reading the written y)
        assert len(seen) == (7 if fuse == "1" else 0), len(seen)
        out[fuse] = (float(loss), P.cpu().clone(),
                     {(l.layer_name, k): v.cpu().clone() for l in all_layers(net.layers) for k, v in (l.grads or {}).items()})
    a, b = out["1"], out["0"]
    assert a[0] == b[0]
    assert torch.equal(a[1], b[1])
    for key, g in a[2].items():
        assert torch.equal(g, b[2][key]), key


@pytest.mark.parametrize("C,N,H", [(512, 4, 7), (64, 3, 5), (6, 2, 9), (256, 2, 1)])
@pytest.mark.parametrize("abn,brelu,bbn", [(True, 0, False), (True, 1, True), (False, 0, True)])
@pytest.mark.parametrize("with_mask", [True, False])
def test_gap_join_matches_bn_add_then_gap(C, N, H, abn, brelu, bbn, with_mask):
    """The head's pooling of the last join (dk_gap_join_fwd_f32) against the join pass + the pooling
    (dk_bn_add_f32 -> dk_gap_fwd_f32): the pooled output and the ReLU mask bitwise (HW = 49 / 25 / 81 / 1:
    the eight-at-a-time loads with and without a remainder; C = 6: the C % 4 != 0 case the join pass
    does not take, checked against an elementwise torch join)."""
    rng = np.random.RandomState(C + N + H + 5 * abn + 7 * bbn + brelu)
    a = nhwc(rng.randn(N, C, H, H) * 1.5)
    b = nhwc(rng.randn(N, C, H, H))
    pa, pb = bn_params(C, rng), bn_params(C, rng)
    st = stream_handle()
    aa = (*(t.data_ptr() for t in pa), 0) if abn else (0, 0, 0, 0, 0)
    ba = (*(t.data_ptr() for t in pb), brelu) if bbn else (0, 0, 0, 0, 0)
    out1 = torch.full((N, C), float("nan"), device="cuda")
    m1 = torch.full((N, C, H, H), 7, dtype=torch.uint8, device="cuda").contiguous(memory_format=torch.channels_last)
    assert lib.dk_gap_join_fwd_f32(a.data_ptr(), *aa, b.data_ptr(), *ba, N, H * H, C,
                                   m1.data_ptr() if with_mask else 0, out1.data_ptr(), st) == 0
    if C % 4 == 0:
        y0 = nhwc(np.zeros((N, C, H, H)))
        m0 = torch.zeros((N, C, H, H), dtype=torch.uint8, device="cuda").contiguous(memory_format=torch.channels_last)
        lib.dk_bn_add_f32(a.data_ptr(), *aa, b.data_ptr(), *ba, a.numel(), C, 1, y0.data_ptr(), m0.data_ptr(), st)
    else:
        def bn(x, p, relu):
            m, i, g, be = (t.view(1, C, 1, 1) for t in p)
            r = g * ((x - m) * i) + be
            return torch.where(r > 0, r, torch.zeros_like(r)) if relu else r
        y0 = (bn(a, pa, 0) if abn else a) + (bn(b, pb, brelu) if bbn else b)
        m0 = (y0 > 0).to(torch.uint8)
        y0 = torch.where(y0 > 0, y0, torch.zeros_like(y0)).contiguous(memory_format=torch.channels_last)
    out0 = torch.empty((N, C), device="cuda")
    lib.dk_gap_fwd_f32(y0.data_ptr(), N, H * H, C, out0.data_ptr(), st)
    torch.cuda.synchronize()
    if C % 4 == 0:
        assert torch.equal(out0, out1)
    else:
        torch.testing.assert_close(out1, out0, rtol=1e-6, atol=1e-6)
    if with_mask:
        assert torch.equal(m0.contiguous(memory_format=torch.channels_last), m1)
