"""In-launch BatchNorm folds (dorknet_amd/csrc/fold_tail.h): every producer of BN partial rows,
armed with dk_bn_fold_arm_stats / dk_bn_fold_arm_bwd, finalizes the statistics (or the
backward coefficients) in its own last-arriving blocks and returns DK_FOLDED.  Each case checks
the in-launch results against the separate fold launch (dk_bn_stats_from_partials_f32 /
dk_bn_bwd_from_partials_f32) over the very partial rows the launch wrote -- the two reduce the
same fp64 rows in different fixed orders, so they agree to fp64 rounding, i.e. (almost always)
bitwise after the fp32 conversion -- that the tickets are left zero, and that an unarmed launch
returns 0.  Cases cover one group (few rows), two ticket levels (hundreds to 12,544 rows), several
channel slices (tiled GEMMs with N > the tile width, multi-slice depthwise backward) and the
layer-level path (network tests run with the folds on)."""
import numpy as np
import pytest
import torch

from dorknet_amd._hip import DK_FOLDED, lib, stream_handle

pytestmark = pytest.mark.gpu

EPS, MOM = 1e-5, 0.9


def nhwc(a):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device="cuda").contiguous(
        memory_format=torch.channels_last)


def vec(a):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device="cuda")


def bn_params(C, rng):
    return [vec(v) for v in (rng.randn(C) * 0.3, rng.rand(C) + 0.5, 1 + 0.3 * rng.randn(C), 0.2 * rng.randn(C))]


class Res:
    def __init__(self):
        self.t = torch.zeros(16384, dtype=torch.int32, device="cuda")
        self.sc = torch.empty(8 << 20, dtype=torch.uint8, device="cuda")

    def args(self):
        return self.t.data_ptr(), self.t.numel(), self.sc.data_ptr(), self.sc.numel()


def _close(a, b, what):
    a, b = a.double(), b.double()
    err = float((a - b).abs().max() / (b.abs().max() + 1e-30))
    assert err <= 1e-6, (what, err)


def check_stats(launch, rows, C, P, rng):
    """launch(part_ptr) -> status of a producer writing part[rows][2][C] (statistics of P pixels)."""
    res = Res()
    st = stream_handle()
    part = torch.full((rows, 2, C), float("nan"), dtype=torch.float64, device="cuda")
    rm0, rs0 = vec(rng.randn(C)), vec(rng.rand(C) + 0.5)
    got = [torch.empty(C, device="cuda") for _ in range(3)] + [rm0.clone(), rs0.clone()]
    assert lib.dk_bn_fold_arm_stats(part.data_ptr(), rows, C, float(P), EPS, MOM, 0, *(t.data_ptr() for t in got),
                                    *res.args()) == 0
    assert launch(part.data_ptr()) == DK_FOLDED
    want = [torch.empty(C, device="cuda") for _ in range(3)] + [rm0.clone(), rs0.clone()]
    nb = lib.dk_bn_partials_workspace_bytes(rows, C)
    ws = torch.empty(max(nb, 256), dtype=torch.uint8, device="cuda")
    tk = torch.zeros(256, dtype=torch.int32, device="cuda")
    assert lib.dk_bn_stats_from_partials_f32(part.data_ptr(), rows, C, float(P), EPS, MOM, 0,
                                             *(t.data_ptr() for t in want), ws.data_ptr(), nb, tk.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert torch.isfinite(part).all()
    for g, w, name in zip(got, want, ("mean", "std", "invstd", "running_mean", "running_std")):
        _close(g, w, name)
    assert int(res.t.abs().sum()) == 0, "tickets not left zero"
    # unarmed: the same launch returns 0
    assert launch(part.data_ptr()) == 0


def check_bwd(launch, rows, C, P):
    res = Res()
    st = stream_handle()
    part = torch.full((rows, 2, C), float("nan"), dtype=torch.float64, device="cuda")
    got = [torch.empty(C, device="cuda"), torch.empty(C, device="cuda"), torch.empty(2 * C, device="cuda")]
    assert lib.dk_bn_fold_arm_bwd(part.data_ptr(), rows, C, float(P), *(t.data_ptr() for t in got),
                                  *res.args()) == 0
    assert launch(part.data_ptr()) == DK_FOLDED
    want = [torch.empty(C, device="cuda"), torch.empty(C, device="cuda"), torch.empty(2 * C, device="cuda")]
    nb = lib.dk_bn_partials_workspace_bytes(rows, C)
    ws = torch.empty(max(nb, 256), dtype=torch.uint8, device="cuda")
    tk = torch.zeros(256, dtype=torch.int32, device="cuda")
    assert lib.dk_bn_bwd_from_partials_f32(part.data_ptr(), rows, C, float(P), *(t.data_ptr() for t in want),
                                           ws.data_ptr(), nb, tk.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert torch.isfinite(part).all()
    for g, w, name in zip(got, want, ("dgamma", "dbeta", "k12")):
        _close(g, w, name)
    assert int(res.t.abs().sum()) == 0, "tickets not left zero"
    assert launch(part.data_ptr()) == 0


@pytest.mark.parametrize("K,C,N,H,stream", [(64, 64, 32, 56, 1), (64, 64, 2, 5, 1), (64, 64, 256, 56, 0),
                                            (128, 128, 16, 28, 1), (256, 128, 8, 14, 1), (512, 512, 4, 7, 1)])
def test_pw_fwd_fold(K, C, N, H, stream):
    """stream 1: the streaming kernel for K = C = 64 (one row per persistent block); stream 0 at
    256 x 56 x 56: the tiled engine's 12,544 rows (112 groups of 112, two ticket levels)."""
    rng = np.random.RandomState(K + C + N)
    x = nhwc(rng.randn(N, C, H, H) + 0.2)
    w = vec(rng.randn(K, C) * 0.2)
    pi = bn_params(C, rng)
    st = stream_handle()
    y = torch.empty((N, K, H, H), device="cuda").contiguous(memory_format=torch.channels_last)
    lib.dk_debug_set_gemm_config(3, stream)
    try:
        rows = lib.dk_pwconv_fwd_stats_rows(N, H, H, K, C)
        check_stats(lambda p: lib.dk_pwconv_fwd_ex_f32(x.data_ptr(), N, H, H, C, w.data_ptr(), K, 1, 0, y.data_ptr(),
                                                       H, H, *(t.data_ptr() for t in pi), 1, p, st),
                    rows, K, N * H * H, rng)
    finally:
        lib.dk_debug_set_gemm_config(3, -1)


def test_stem_fwd_fold():
    rng = np.random.RandomState(3)
    N, H, Cp, K, R, s, pad = 8, 65, 4, 64, 5, 2, 2
    OH = (H + 2 * pad - R) // s + 1
    x = nhwc(np.concatenate([rng.randn(N, 3, H, H), np.zeros((N, 1, H, H))], 1))
    w = vec(rng.randn(K, R, R, Cp) * 0.1)
    y = torch.empty((N, K, OH, OH), device="cuda").contiguous(memory_format=torch.channels_last)
    rows = lib.dk_conv2d_fwd_stats_rows(N, OH, OH, K, Cp, R, R)
    st = stream_handle()
    check_stats(lambda p: lib.dk_conv2d_fwd_ex_f32(x.data_ptr(), N, H, H, Cp, w.data_ptr(), K, R, R, s, pad, 0,
                                                   y.data_ptr(), OH, OH, 0, 0, 0, 0, 0, p, st),
                rows, K, N * OH * OH, rng)


@pytest.mark.parametrize("N,H", [(8, 65), (64, 225)])
def test_stem_narrow_fwd_fold(N, H):
    """The narrow-input stem forward (NCHW image, one partial row per persistent block)."""
    rng = np.random.RandomState(N + H)
    C, K, R, s, pad = 3, 64, 5, 2, 1
    OH = (H + 2 * pad - R) // s + 1
    x = torch.from_numpy(rng.randn(N, C, H, H).astype(np.float32)).cuda()
    w = vec(rng.randn(K, C, R, R) * 0.1)
    y = torch.empty((N, K, OH, OH), device="cuda").contiguous(memory_format=torch.channels_last)
    rows = lib.dk_conv2d_fwd_narrow_stats_rows(N, C, H, H, K, R, R, s, pad, OH, OH)
    assert rows > 0
    st = stream_handle()
    check_stats(lambda p: lib.dk_conv2d_fwd_narrow_f32(x.data_ptr(), N, C, H, H, w.data_ptr(), K, R, R, s, pad, 0,
                                                       y.data_ptr(), OH, OH, p, st),
                rows, K, N * OH * OH, rng)


@pytest.mark.parametrize("C,N,H,stride", [(64, 64, 56, 1), (128, 16, 28, 2), (512, 8, 7, 1), (256, 2, 3, 1)])
def test_dw_fwd_fold(C, N, H, stride):
    rng = np.random.RandomState(C + N + stride)
    x = nhwc(rng.randn(N, C, H, H))
    w = vec(rng.randn(C, 3, 3) * 0.3)
    pi = bn_params(C, rng)
    OH = (H + 2 - 3) // stride + 1
    y = torch.empty((N, C, OH, OH), device="cuda").contiguous(memory_format=torch.channels_last)
    rows = lib.dk_dwconv_fwd_stats_rows(N, OH, OH, C, stride)
    st = stream_handle()
    check_stats(lambda p: lib.dk_dwconv_fwd_ex_f32(x.data_ptr(), N, H, H, C, w.data_ptr(), 3, 3, stride, 1, 0,
                                                   y.data_ptr(), OH, OH, *(t.data_ptr() for t in pi), 1, p, st),
                rows, C, N * OH * OH, rng)


@pytest.mark.parametrize("K,C,N,H,s", [(128, 128, 32, 28, 1), (256, 256, 16, 14, 1), (128, 64, 16, 28, 2)])
def test_pw_dgrad_ex_fold(K, C, N, H, s):
    """EpStoreBnBwd (stride 1, one slice per 64/128-wide N tile) and EpWidenBnBwd (stride 2)."""
    rng = np.random.RandomState(K + C + s)
    OH = H // s
    dy = nhwc(rng.randn(N, K, OH, OH))
    w = vec(rng.randn(K, C) * 0.2)
    xbn = nhwc(rng.randn(N, C, H, H))
    pi = bn_params(C, rng)
    dx = torch.empty((N, C, H, H), device="cuda").contiguous(memory_format=torch.channels_last)
    rows = lib.dk_pwconv_dgrad_stats_rows(N, OH, OH, K, C)
    st = stream_handle()
    check_bwd(lambda p: lib.dk_pwconv_dgrad_ex_f32(dy.data_ptr(), N, OH, OH, K, w.data_ptr(), C, s, dx.data_ptr(), 0,
                                                   xbn.data_ptr(), *(t.data_ptr() for t in pi), 1, p, st),
              rows, C, N * H * H)


@pytest.mark.parametrize("C,N,H", [(64, 16, 56), (128, 8, 28), (512, 4, 7)])
def test_relu_bwd_bn_partial_fold(C, N, H):
    rng = np.random.RandomState(C + N)
    P = N * H * H
    dy = nhwc(rng.randn(N, C, H, H))
    mask = torch.as_tensor((rng.rand(P * C) > 0.4).astype(np.uint8), device="cuda")
    x = nhwc(rng.randn(N, C, H, H))
    pi = bn_params(C, rng)
    dx = torch.empty_like(dy)
    rows = lib.dk_bn_partial_blocks(P, C)
    nb = lib.dk_bn_workspace_bytes(P, C)
    st = stream_handle()
    check_bwd(lambda p: lib.dk_relu_bwd_bn_partial_f64(dy.data_ptr(), mask.data_ptr(), x.data_ptr(), P, C,
                                                       *(t.data_ptr() for t in pi), 1, dx.data_ptr(), p, nb, st),
              rows, C, P)


@pytest.mark.parametrize("C,N,H", [(64, 16, 56), (128, 8, 28), (512, 4, 7)])
def test_dw_bwd_fused_fold(C, N, H):
    rng = np.random.RandomState(C + 7)
    g = nhwc(rng.randn(N, C, H, H))
    bx = nhwc(rng.randn(N, C, H, H))
    po = bn_params(C, rng)
    k12 = vec(rng.randn(2 * C) * 0.1)
    x = nhwc(rng.randn(N, C, H, H))
    w = vec(rng.randn(C, 3, 3) * 0.3)
    pi = bn_params(C, rng)
    dw = torch.empty((C, 3, 3), device="cuda")
    dx = torch.empty_like(x)
    rows = lib.dk_dwconv_bwd_bnbwd_stats_rows(N, H, H, C)
    nb = lib.dk_dwconv_bwd_bnbwd_workspace_bytes(N, H, H, C, 3, 3)
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    st = stream_handle()
    check_bwd(lambda p: lib.dk_dwconv_bwd_bnbwd_f32(g.data_ptr(), bx.data_ptr(), N, H, H, C,
                                                    *(t.data_ptr() for t in po), 1, k12.data_ptr(), x.data_ptr(),
                                                    w.data_ptr(), 3, 3, 1, 0.0, dw.data_ptr(), dx.data_ptr(), 0,
                                                    *(t.data_ptr() for t in pi), 1, p, ws.data_ptr(), nb, st),
              rows, C, N * H * H)


@pytest.mark.parametrize("N,H", [(64, 56), (2, 7)])
def test_pw_bwd_fused_fold(N, H):
    K = C = 64
    rng = np.random.RandomState(N)
    g = nhwc(rng.randn(N, K, H, H))
    bx = nhwc(rng.randn(N, K, H, H))
    po = bn_params(K, rng)
    k12 = vec(rng.randn(2 * K) * 0.1)
    w = vec(rng.randn(K, C) * 0.2)
    x = nhwc(rng.randn(N, C, H, H))
    pi = bn_params(C, rng)
    dw = torch.empty((K, C), device="cuda")
    dx = torch.empty_like(x)
    rows = lib.dk_pwconv_bwd_fused_rows(N, H, H, K, C)
    nb = lib.dk_pwconv_bwd_fused_workspace_bytes(N, H, H, K, C)
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    st = stream_handle()
    check_bwd(lambda p: lib.dk_pwconv_bwd_bnbwd_f32(g.data_ptr(), bx.data_ptr(), N, H, H, K,
                                                    *(t.data_ptr() for t in po), 1, k12.data_ptr(), w.data_ptr(), C,
                                                    0.0, dw.data_ptr(), dx.data_ptr(), 0, x.data_ptr(),
                                                    *(t.data_ptr() for t in pi), 1, p, ws.data_ptr(), nb, st),
              rows, C, N * H * H)


def test_layer_path_folds_match_separate_launches(monkeypatch):
    """The ResNet-18-depsep stem + res1 through the network API: DORKNET_INLAUNCH_FOLD=1 (the
    default) and =0 give the same outputs, gradients and running statistics (fp64 rounding)."""
    from examples.resnet18_depsep import ResNet18
    from dorknet_amd.network.feed_forward_network import FeedForwardNetwork
    from tests._convert import all_layers
    rng = np.random.RandomState(6)
    X = torch.as_tensor(rng.randn(4, 3, 65, 65).astype(np.float32) * 50, device="cuda")
    results = []
    for flag in ("1", "0"):
        monkeypatch.setenv("DORKNET_INLAUNCH_FOLD", flag)
        np.random.seed(5)
        layers = ResNet18("r18").layers[:8]
        net = FeedForwardNetwork("fold")
        for l in layers:
            net.add_layer(l)
        net.to_gpu()
        _, Y = net.forward(X, None)
        dY = torch.as_tensor(np.random.RandomState(7).randn(*Y.shape).astype(np.float32), device="cuda")
        net.backward(dY)
        torch.cuda.synchronize()
        out = {"Y": Y.float().clone()}
        for l in all_layers(layers):
            for k, v in (l.grads or {}).items():
                out[(l.layer_name, k)] = v.float().clone()
            nlp = getattr(l, "non_learned_params", None) or {}
            for k in ("running_mean", "running_std"):
                if nlp.get(k) is not None:
                    out[(l.layer_name, k)] = torch.as_tensor(nlp[k], device="cuda").float().clone()
        results.append(out)
    a, b = results
    assert a.keys() == b.keys() and len(a) > 20
    for k in a:
        _close(a[k], b[k], k)
