"""Algorithmic work (flops, compulsory HBM bytes) per C-ABI call, for roofline reporting.

Formulas follow SURVEY.md 8(d): a conv/pw pass moves its input, output and weights once
(e = 4 bytes, fp32) and does 2*N*K*OH*OW*C*R*S flops; depthwise 2*N*C*OH*OW*R*S flops;
BN forward apply reads + writes each element, the BN reduce passes read it once; etc.
Only the *compulsory* bytes count (a stride-s pointwise layer reads N*OH*OW*C input
values, not N*H*W*C), so `achieved` is never inflated by bytes the algorithm does not need.

Each entry maps the positional arguments of the C function (include/dorknet_hip.h) to
(flops, bytes).  Unlisted entry points are treated as (0, 0).
"""
from __future__ import annotations

E = 4  # fp32

PEAK_F32_TFLOPS = 157.3   # MI355X fp32 MFMA / vector, dense (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0     # MI355X HBM3E spec
PEAK_BF16_TFLOPS = 2500.0  # MI355X bf16 MFMA, dense (no sparsity)


def _conv_fwd(x, N, H, W, C, w, K, R, S, stride, pad, bias, y, OH, OW, st):
    return 2 * N * OH * OW * K * C * R * S, E * (N * H * W * C + N * OH * OW * K + K * R * S * C)


def _conv_dgrad(dy, N, OH, OW, K, w, C, R, S, pad, dx, H, W, st):
    return 2 * N * OH * OW * K * C * R * S, E * (N * OH * OW * K + N * H * W * C + K * R * S * C)


def _conv_dgrad_strided(dy, N, OH, OW, K, w, C, R, S, stride, pad, dx, H, W, ws, nb, st):
    return 2 * N * OH * OW * K * C * R * S, E * (N * OH * OW * K + N * H * W * C + K * R * S * C)


def _conv_wgrad(dy, x, N, H, W, Cp, C, K, R, S, stride, pad, OH, OW, w, l2, dw, ws, nb, st):
    return 2 * N * OH * OW * K * C * R * S, E * (N * OH * OW * K + N * H * W * C + K * R * S * C)


def _pw_fwd(x, N, H, W, C, w, K, stride, bias, y, OH, OW, st):
    return 2 * N * OH * OW * K * C, E * (N * OH * OW * C + N * OH * OW * K + K * C)


def _pw_dgrad(dy, N, OH, OW, K, w, C, stride, dx, st):
    return 2 * N * OH * OW * K * C, E * (N * OH * OW * K + N * OH * OW * stride * stride * C + K * C)


def _pw_wgrad(dy, x, N, H, W, C, K, stride, OH, OW, w, l2, dw, ws, nb, st):
    return 2 * N * OH * OW * K * C, E * (N * OH * OW * K + N * OH * OW * C + K * C)


def _dw_fwd(x, N, H, W, C, w, R, S, stride, pad, bias, y, OH, OW, st):
    return 2 * N * C * OH * OW * R * S, E * (N * H * W * C + N * OH * OW * C + C * R * S)


def _dw_dgrad(dy, N, OH, OW, C, w, R, S, stride, pad, dx, H, W, ws, nb, st):
    return 2 * N * C * OH * OW * R * S, E * (N * OH * OW * C + N * H * W * C + C * R * S)


def _dw_wgrad(dy, x, N, H, W, C, R, S, stride, pad, OH, OW, w, l2, dw, ws, nb, st):
    return 2 * N * C * OH * OW * R * S, E * (N * OH * OW * C + N * H * W * C + C * R * S)


def _dense_fwd(x, B, IN, w, OUT, bias, y, st):
    return 2 * B * IN * OUT, E * (B * IN + B * OUT + IN * OUT)


def _dense_dgrad(dy, B, OUT, w, IN, dx, st):
    return 2 * B * IN * OUT, E * (B * IN + B * OUT + IN * OUT)


def _dense_wgrad(x, dy, B, IN, OUT, w, l2, dw, ws, nb, st):
    return 2 * B * IN * OUT, E * (B * IN + B * OUT + IN * OUT)


def _bn_stats(x, P, C, *rest):
    return 3 * P * C, E * P * C


def _bn_apply(x, numel, C, *rest):
    return 4 * numel, E * 2 * numel


def _bn_bwd(x, dy, P, C, *rest):
    return 12 * P * C, E * 5 * P * C   # reduce pass reads x, dy; apply pass reads x, dy, writes dx


def _relu_fwd(x, n, y, mask, st):
    return n, E * 2 * n + (n if mask else 0)


def _relu_bwd(dy, mask, n, dx, st):
    return n, E * 2 * n + n


def _add(a, b, n, relu, y, mask, st):
    return n, E * 3 * n + (n if mask else 0)


def _gap_fwd(x, N, HW, C, out, st):
    return N * HW * C, E * (N * HW * C + N * C)


def _gap_bwd(dy, N, HW, C, dx, st):
    return N * HW * C, E * (N * HW * C + N * C)


def _sgd(table, ntens, total_blocks, *rest):
    n = total_blocks * 256
    return 4 * n, 5 * E * n


def _l2_multi(table, ntens, total_blocks, *rest):
    n = total_blocks * 2048
    return 2 * n, E * n


def _colsum(x, M, N, *rest):
    return M * N, E * M * N


def _nchw_to_nhwc(x, N, C, H, W, Cp, y, st):
    return 0, E * (N * C * H * W + N * Cp * H * W)


def _bnx(f):
    """A *_bnx_* entry = the plain entry with 5 BatchNorm arguments before the stream; the
    compulsory bytes are the same (the BN output it replaces is never written or read)."""
    return lambda *a: f(*(a[:-6] + a[-1:]))


def _ex(f):
    """A *_fwd_ex_f32 entry: the plain arguments, 5 BatchNorm arguments, the statistics
    pointer, the stream.  The statistics are computed in the epilogue (no extra traffic
    beyond the partial sums, ignored here)."""
    return lambda *a: f(*(a[:-7] + a[-1:]))


def _bn_add(a, am, ai, ag, ab, ar, b, bm, bi, bg, bb, br, n, C, relu, y, mask, st):
    return n * (1 + 4 * (bool(am) + bool(bm))), E * 3 * n + (n if mask else 0)


MODEL = {
    "dk_conv2d_fwd_f32": _conv_fwd,
    "dk_conv2d_dgrad_f32": _conv_dgrad,
    "dk_conv2d_dgrad_phase_f32": lambda dy, N, OH, OW, Kp, K, w, C, R, S, stride, pad, dx, H, W, ws, nb, st:
        _conv_dgrad_strided(dy, N, OH, OW, K, w, C, R, S, stride, pad, dx, H, W, ws, nb, st),
    "dk_conv2d_dgrad_subpixel_f32": _conv_dgrad_strided,
    "dk_conv2d_wgrad_f32": _conv_wgrad,
    "dk_pwconv_fwd_f32": _pw_fwd,
    "dk_pwconv_dgrad_f32": _pw_dgrad,
    "dk_pwconv_wgrad_f32": _pw_wgrad,
    "dk_dwconv_fwd_f32": _dw_fwd,
    "dk_dwconv_dgrad_f32": _dw_dgrad,
    "dk_dwconv_wgrad_f32": _dw_wgrad,
    "dk_dense_fwd_f32": _dense_fwd,
    "dk_dense_dgrad_f32": _dense_dgrad,
    "dk_dense_wgrad_f32": _dense_wgrad,
    "dk_bn_stats_f32": _bn_stats,
    "dk_bn_apply_f32": _bn_apply,
    "dk_bn_bwd_f32": _bn_bwd,
    "dk_relu_fwd_f32": _relu_fwd,
    "dk_relu_bwd_f32": _relu_bwd,
    "dk_add_f32": _add,
    "dk_gap_fwd_f32": _gap_fwd,
    "dk_gap_bwd_f32": _gap_bwd,
    "dk_sgd_momentum_multi_f32": _sgd,
    "dk_colsum_f32": _colsum,
    "dk_l2_loss_multi_f32": _l2_multi,
    "dk_nchw_to_nhwc_f32": _nchw_to_nhwc,
    "dk_conv2d_fwd_bnx_f32": _bnx(_conv_fwd),
    "dk_conv2d_wgrad_bnx_f32": _bnx(_conv_wgrad),
    # wgrad with the following BN's backward apply on load: reads g and that BN's input
    # (N*OH*OW*K each) instead of dy
    "dk_conv2d_wgrad_bnbwd_f32": lambda g, ox, x, N, H, W, Cp, C, K, R, S, st_, pad, OH, OW, *rest: (
        2 * N * OH * OW * K * C * R * S + 6 * N * OH * OW * K,
        E * (2 * N * OH * OW * K + N * H * W * Cp + K * R * S * C)),
    # narrow-input stem kernels (conv_narrow.hip): the NCHW image read as given (C channels)
    "dk_conv2d_fwd_narrow_f32": lambda x, N, C, H, W, w, K, R, S, st_, pad, b, y, OH, OW, stats, st: (
        2 * N * OH * OW * K * C * R * S, E * (N * C * H * W + N * OH * OW * K + K * C * R * S)),
    "dk_conv2d_wgrad_narrow_f32": lambda dy, x, N, C, H, W, K, R, S, st_, pad, OH, OW, *rest: (
        2 * N * OH * OW * K * C * R * S, E * (N * OH * OW * K + N * C * H * W + K * C * R * S)),
    # (g read on its lattice only when g_lattice = 2: a quarter of the pixels)
    "dk_conv2d_wgrad_bnbwd_narrow_f32": lambda g, ox, x, N, C, H, W, K, R, S, st_, pad, OH, OW, m, i, ga, b, relu,
    k12, lat, *rest: (
        2 * N * OH * OW * K * C * R * S + 6 * N * OH * OW * K,
        E * (N * OH * OW * K + N * (-(-OH // lat)) * (-(-OW // lat)) * K + N * C * H * W + K * C * R * S)),
    # stride-s pointwise dgrad kept as its lattice (+ the input BN's partials at the lattice points)
    "dk_pwconv_dgrad_lattice_f32": lambda dy, N, OH, OW, K, w, C, s, dx, bx, *rest: (
        2 * N * OH * OW * K * C, E * (N * OH * OW * K + 2 * N * OH * OW * C + K * C)),
    "dk_pwconv_fwd_bnx_f32": _bnx(_pw_fwd),
    "dk_pwconv_wgrad_bnx_f32": _bnx(_pw_wgrad),
    "dk_dwconv_fwd_bnx_f32": _bnx(_dw_fwd),
    "dk_dwconv_wgrad_bnx_f32": _bnx(_dw_wgrad),
    "dk_bn_add_f32": _bn_add,
    "dk_conv2d_fwd_ex_f32": _ex(_conv_fwd),
    "dk_pwconv_fwd_ex_f32": _ex(_pw_fwd),
    "dk_dwconv_fwd_ex_f32": _ex(_dw_fwd),
    # dgrad + BN-backward partials: also reads the BN's raw input (same size as dx)
    # dgrad (+ the residual addend read) (+ the BN's raw input read for the BN-backward sums)
    "dk_pwconv_dgrad_ex_f32": lambda dy, N, OH, OW, K, w, C, s, dx, res, bx, m, i, g, b, r, part, st: (
        _pw_dgrad(dy, N, OH, OW, K, w, C, s, dx, st)[0],
        _pw_dgrad(dy, N, OH, OW, K, w, C, s, dx, st)[1] + E * N * OH * OW * C * ((bx != 0) + (res != 0) * s * s)),
    "dk_dwconv_dgrad_ex_f32": lambda dy, N, OH, OW, C, w, R, S, s, p, dx, H, W, ws, nb, res, bx, m, i, g, b, r, part,
    st: (_dw_dgrad(dy, N, OH, OW, C, w, R, S, s, p, dx, H, W, ws, nb, st)[0],
         _dw_dgrad(dy, N, OH, OW, C, w, R, S, s, p, dx, H, W, ws, nb, st)[1] + E * N * H * W * C * (
             (bx != 0) + (res != 0))),
    # dgrad with the following BN's backward apply on load: reads g and that BN's input
    # (P x K each), writes dy (P x K) once for the weight gradient, + the dgrad_ex terms
    "dk_pwconv_dgrad_bnbwd_f32": lambda g, ox, N, OH, OW, K, om, oi, og, ob, orl, k12, dyo, w, C, dx, res, bx, m, i,
    ga, b, r, part, st: (
        2 * N * OH * OW * K * C + 6 * N * OH * OW * K,
        E * (N * OH * OW * K * (2 + (dyo != 0)) + N * OH * OW * C * (1 + (bx != 0) + (res != 0)) + K * C)),
    # fused pointwise backward (dgrad + wgrad): reads g and the following BN's input (to form
    # dy), the layer's input x once (weight-gradient operand and the input BN's partials) and
    # the residual; writes dx; dW partials are per block (small)
    "dk_pwconv_bwd_bnbwd_f32": lambda g, ox, N, OH, OW, K, om, oi, og, ob, orl, k12, w, C, l2, dw, dx, res, x, m,
    i, ga, b, r, part, ws, nb, st: (
        2 * 2 * N * OH * OW * K * C + 6 * N * OH * OW * K,
        E * (2 * N * OH * OW * K + N * OH * OW * C * (2 + (res != 0)) + 2 * K * C)),
    # the same for a strided layer with dx kept as its lattice: x read at the lattice points only
    "dk_pwconv_bwd_bnbwd_lattice_f32": lambda g, ox, N, OH, OW, K, om, oi, og, ob, orl, k12, w, C, l2, dw, dx, x, H,
    W, s, m, i, ga, b, r, part, ws, nb, st: (
        2 * 2 * N * OH * OW * K * C + 6 * N * OH * OW * K,
        E * (2 * N * OH * OW * K + 2 * N * OH * OW * C + 2 * K * C)),
    # fused depthwise backward: reads g and the following BN's input (to form dy), the layer's
    # input (weight gradient; the input BN's partials), the residual addend; writes dx
    "dk_dwconv_bwd_bnbwd_f32": lambda g, ox, N, H, W, C, om, oi, og, ob, orl, k12, x, w, R, S, pad, l2, dw, dx, res,
    m, i, ga, b, r, part, ws, nb, st: (
        2 * 2 * N * H * W * C * R * S + 6 * N * H * W * C,
        E * (N * H * W * C * (3 + (dx != 0) + (res != 0)) + 2 * C * R * S)),
    # + the input's residual join: its ReLU mask (bytes) and its BatchNorm's raw input are read
    "dk_dwconv_bwd_bnbwd_join_f32": lambda g, ox, N, H, W, C, om, oi, og, ob, orl, k12, x, w, R, S, pad, l2, dw, dx,
    res, mask, jx, jm, ji, part, ws, nb, st: (
        2 * 2 * N * H * W * C * R * S + 10 * N * H * W * C,
        E * (N * H * W * C * (5 + (res != 0)) + 2 * C * R * S) + N * H * W * C * (mask != 0)),
    # strided dgrad + the join: dy, the residual (dense, or its compact lattice when
    # residual_lattice = s), the mask and bn_j's input read; dx written
    "dk_dwconv_dgrad_join_f32": lambda dy, N, OH, OW, C, w, R, S, s, p, dx, H, W, ws, nb, res, rl, mask, jx, jm, ji,
    part, st: (
        _dw_dgrad(dy, N, OH, OW, C, w, R, S, s, p, dx, H, W, ws, nb, st)[0] + 4 * N * H * W * C,
        E * (N * OH * OW * C + 2 * N * H * W * C + (res != 0) * (N * OH * OW * C if rl else N * H * W * C))
        + N * H * W * C),
    "dk_relu_bwd_bn_partial_f64": lambda dy, mask, x, P, C, *rest: (4 * P * C, E * 3 * P * C + P * C),
    "dk_bn_bwd_apply_f32": lambda x, dy, n, C, *rest: (6 * n, E * 3 * n),
}


def work(name: str, args) -> tuple[int, int]:
    f = MODEL.get(name)
    if f is None:
        return 0, 0
    return f(*args)


# Entry points whose flops run on bf16 MFMA (v_mfma_f32_32x32x16_bf16): their compute roof is the
# bf16 dense peak; every other entry computes in fp32 (f32 MFMA or VALU, the same 157.3 TF/s).
BF16_MFMA = {"dk_pwconv_fwd_ex_bf16", "dk_pwconv_dgrad_ex_bf16", "dk_pwconv_wgrad_bnx_bf16",
             "dk_pwconv_dgrad_bnbwd_bf16"}


def peak_tflops(name: str | None = None) -> float:
    return PEAK_BF16_TFLOPS if name in BF16_MFMA else PEAK_F32_TFLOPS


def bound_time_s(flops: float, nbytes: float, name: str | None = None) -> float:
    """Roofline lower bound on time for one call: max(flops / peak, bytes / BW)."""
    return max(flops / (peak_tflops(name) * 1e12), nbytes / (PEAK_HBM_GBS * 1e9))


def is_mfma_bound(flops: float, nbytes: float, name: str | None = None) -> bool:
    return flops / (peak_tflops(name) * 1e12) > nbytes / (PEAK_HBM_GBS * 1e9)


def _half(f):
    """A *_bf16 twin: the fp32 entry's arguments and flops; activations move as 2-byte bf16,
    so the compulsory bytes halve (weights and BN parameters, < 1 % of the bytes here, are
    counted at 2 bytes too -- a slight undercount, i.e. a conservative achieved rate)."""
    def g(*a):
        fl, by = f(*a)
        return fl, by // 2
    return g


for _n in ("dk_pwconv_fwd_ex", "dk_pwconv_dgrad_ex", "dk_pwconv_wgrad_bnx", "dk_dwconv_fwd_ex", "dk_dwconv_dgrad_ex",
           "dk_dwconv_wgrad_bnx", "dk_bn_stats", "dk_bn_apply", "dk_bn_bwd", "dk_bn_bwd_apply", "dk_relu_fwd",
           "dk_relu_bwd", "dk_pwconv_dgrad_bnbwd", "dk_dwconv_bwd_bnbwd"):
    if _n + "_f32" in MODEL:
        MODEL[_n + "_bf16"] = _half(MODEL[_n + "_f32"])
