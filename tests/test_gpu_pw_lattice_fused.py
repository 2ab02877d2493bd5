"""The fused lattice backward of a strided pointwise layer (dk_pwconv_bwd_bnbwd_lattice_f32, the
stem's pw0: K = C = 64, stride 2, input consumed as a BNOut) against the stride-1 fused backward
(dk_pwconv_bwd_bnbwd_f32) over the gathered lattice of the same input: the two run the same
streaming kernel and differ only in where a tile's x rows are read from, so dx (the compact
lattice), the weight gradient and the input BatchNorm's partials are bit-identical.  The stride-1
entry's parity with the oracle is test_gpu_pw_stream.py's / test_gpu_fullsize.py's.
Reference: pointwise_convolution.py:56-77 (backward with stride), batch_norm.py:125-174."""
import numpy as np
import pytest
import torch

from dorknet_amd._hip import HipError, lib, stream_handle

pytestmark = pytest.mark.gpu


def _h(rng, N, C, H, W):
    a = torch.as_tensor(rng.randn(N, C, H, W).astype(np.float32), device="cuda")
    return a.contiguous(memory_format=torch.channels_last)


def _bn(C, rng):
    return [torch.as_tensor(v.astype(np.float32), device="cuda") for v in
            (rng.randn(C) * 0.3, rng.rand(C) + 0.5, 1 + 0.3 * rng.randn(C), 0.2 * rng.randn(C))]


def _call(fn, g, xo, N, OH, OW, po, k12, w, x, pi, with_part, extra):
    K, C = w.shape
    rows = lib.dk_pwconv_bwd_fused_rows(N, OH, OW, K, C)
    nb = lib.dk_pwconv_bwd_fused_workspace_bytes(N, OH, OW, K, C)
    ws = torch.empty(nb // 4 + 64, dtype=torch.float32, device="cuda")
    part = torch.full((rows, 2, C), float("nan"), dtype=torch.float64, device="cuda") if with_part else None
    dx = torch.full((N, C, OH, OW), float("nan"), device="cuda").contiguous(memory_format=torch.channels_last)
    dw = torch.full_like(w, float("nan"))
    head = (g.data_ptr(), xo.data_ptr(), N, OH, OW, K, *(t.data_ptr() for t in po), 1, k12.data_ptr(),
            w.data_ptr(), C, 0.0, dw.data_ptr(), dx.data_ptr())
    tail = (*(t.data_ptr() for t in pi), 1, part.data_ptr() if with_part else 0, ws.data_ptr(), nb, stream_handle())
    rc = fn(*head, *extra(x), *tail)
    torch.cuda.synchronize()
    assert rc in (0, 10100), rc
    return dx, dw, part


@pytest.mark.parametrize("N,H,W,OH,OW", [(2, 112, 112, 56, 56), (3, 20, 20, 10, 10), (1, 14, 22, 7, 11),
                                         (2, 15, 13, 8, 7), (5, 8, 8, 4, 4)])
@pytest.mark.parametrize("with_part", [True, False])
def test_lattice_matches_gathered_stride1(N, H, W, OH, OW, with_part):
    rng = np.random.RandomState(N * 31 + H + 3 * W)
    K = C = 64
    s = 2
    g, xo = _h(rng, N, K, OH, OW), _h(rng, N, K, OH, OW)
    x = _h(rng, N, C, H, W)
    po, pi = _bn(K, rng), _bn(C, rng)
    k12 = torch.as_tensor(rng.randn(2 * K).astype(np.float32) * 0.1, device="cuda")
    w = torch.as_tensor(rng.randn(K, C).astype(np.float32) * 0.2, device="cuda")
    xl = x[:, :, ::s, ::s].contiguous(memory_format=torch.channels_last)
    assert tuple(xl.shape) == (N, C, OH, OW)
    dx1, dw1, p1 = _call(lib.dk_pwconv_bwd_bnbwd_f32, g, xo, N, OH, OW, po, k12, w, xl, pi, with_part,
                         lambda t: (0, t.data_ptr()))
    dx2, dw2, p2 = _call(lib.dk_pwconv_bwd_bnbwd_lattice_f32, g, xo, N, OH, OW, po, k12, w, x, pi, with_part,
                         lambda t: (t.data_ptr(), H, W, s))
    assert bool(torch.isfinite(dx2).all()) and bool(torch.isfinite(dw2).all())
    assert torch.equal(dx1, dx2)
    assert torch.equal(dw1, dw2)
    if with_part:
        assert torch.equal(p1, p2)


def test_rejects_bad_geometry():
    """The lattice must fit in the input, stride >= 2, K = C = 64."""
    f = lib.dk_pwconv_bwd_bnbwd_lattice_f32
    args = lambda N, OH, OW, K, C, H, W, s: (16, 16, N, OH, OW, K, 16, 16, 16, 16, 1, 16, 16, C, 0.0, 16, 16, 16,
                                             H, W, s, 16, 16, 16, 16, 1, 0, 16, 1 << 30, 0)
    for bad in [(2, 8, 8, 64, 64, 14, 16, 2),  # (OH - 1) * 2 + 1 = 15 > 14
                (2, 8, 8, 64, 64, 16, 16, 1), (2, 8, 8, 128, 64, 16, 16, 2)]:
        with pytest.raises(HipError, match="bad arguments"):
            f(*args(*bad))
