// bf16 pointwise entry points (BASELINE config 5) on the implicit-GEMM engine's bf16 MFMA mode
// (gemm_engine.h).
#include "gemm_engine.h"

using namespace dk;

// ---------------------------------------------------------------------------------------
// bf16 storage twins of the pointwise entries (BASELINE config 5).  Activations bf16,
// weights / statistics / weight gradients fp32; the loaders widen bf16 to fp32 on load and
// the MFMAs are the exact-fp32 v_mfma_f32_32x32x2_f32 of the fp32 path, so the only
// numerical difference from fp32 storage is the rounding of each stored activation.
// ---------------------------------------------------------------------------------------
namespace dk {
static inline MatDescE<bf16_t> mat_h(const bf16_t* p, int rows, int ld, int ext) {
  return MatDescE<bf16_t>{p, (uint32_t)((size_t)rows * ld * sizeof(bf16_t)), ld, ext};
}
static inline ImgDescE<bf16_t> img_h(const bf16_t* x, int N, int H, int W, int C, int OH, int OW, int R, int S,
                                     int sa, int dr, int off, int M) {
  return set_magics(ImgDescE<bf16_t>{x, (uint32_t)((size_t)N * H * W * C * sizeof(bf16_t)), H, W, C, OH, OW, R, S,
                                     sa, dr, off, off, M});
}
static inline ImgDescE<bf16_t, true> img1_h(const bf16_t* x, int N, int H, int W, int C, int OH, int OW, int sa, int M) {
  return set_magics(ImgDescE<bf16_t, true>{x, (uint32_t)((size_t)N * H * W * C * sizeof(bf16_t)), H, W, C, OH, OW,
                                           1, 1, sa, 1, 0, 0, M});
}
static inline bool al8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; }
}  // namespace dk

// partial-statistics rows of dk_pwconv_fwd_ex_bf16: one per streaming block (K, C in {64, 128},
// pw_stream_bf16.hip), else one per M tile of the tiled engine
DK_API int dk_pwconv_fwd_bf16_stats_rows(int N, int OH, int OW, int K, int C) {
  const int M = N * OH * OW;
  if (pw_stream_bf16_fwd_ok(K, C, M)) return pw_stream_bf16_fwd_rows(M, K, C);
  return stats_rows(M, K, C, kRowFwdH, kMfBf16);
}

DK_API int dk_pwconv_fwd_ex_bf16(const bf16_t* x, int N, int H, int W, int C, const float* w_kc, int K, int stride,
                                 const float* bias, bf16_t* y, int OH, int OW, const float* bn_mean,
                                 const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu,
                                 double* stats, void* stream) {
  if (C % 4 || K % 4 || !al8(x) || !al8(y) || !aligned16(w_kc) || (bias && !aligned16(bias))) return DK_ERR_ARGS;
  if (!fits((size_t)N * H * W * C * 4) || !fits((size_t)N * OH * OW * K * 4)) return DK_ERR_ARGS;
  const hipStream_t st = as_stream(stream);
  if (stride == 1 && H == OH && W == OW && pw_stream_bf16_fwd_ok(K, C, N * OH * OW) && aligned16(x) &&
      (!bn_mean || bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta))) {
    // the streaming kernel (pw_stream_bf16.hip): bit-identical y, its own partial-row grouping
    const int M = N * OH * OW;
    FoldTail ft;
    if (stats) fold_take(stats, pw_stream_bf16_fwd_rows(M, K, C), K, pw_stream_bf16_fwd_slices(K, C), &ft);
    return fold_status(pw_stream_bf16_fwd(x, M, w_kc, K, C, bias, y, bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu,
                                          stats, st, stats ? &ft : nullptr),
                       stats ? ft : FoldTail{});
  }
  const ImgDescE<bf16_t, true> a = img1_h(x, N, H, W, C, OH, OW, stride, N * OH * OW);
  const MatDesc b = mat(w_kc, K, C, K);
  const int M = a.M;
  auto run = [&](const auto& da) -> int {
    using DA = std::decay_t<decltype(da)>;
    if (stats) {
      EpStoreStatsT<bf16_t> ep{};
      ep.out = y, ep.ldo = K, ep.bias = bias, ep.v4 = 1, ep.res = nullptr, ep.part = stats;
      return igemm_rows<LdImgKC, DA, LdMatKC, MatDesc, EpStoreStatsT<bf16_t>, kRowFwdH, kMfBf16>(da, b, ep, M, K, C, st);
    }
    EpStoreT<bf16_t> ep{y, K, bias, 1, nullptr};
    return igemm_rows<LdImgKC, DA, LdMatKC, MatDesc, EpStoreT<bf16_t>, kRowFwdH, kMfBf16>(da, b, ep, M, K, C, st);
  };
  if (bn_mean) {
    if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta) || C > 2048) return DK_ERR_ARGS;
    ImgBnDescE<bf16_t, true> ab;
    static_cast<ImgDescE<bf16_t, true>&>(ab) = a;
    ab.bn = BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
    return run(ab);
  }
  return run(a);
}

// Stride-1 pointwise dgrad (bf16): dx = dy . W (+ residual) and, with bn_x/part, the
// BN-backward partials of the BatchNorm whose output the layer consumed.
DK_API int dk_pwconv_dgrad_ex_bf16(const bf16_t* dy, int N, int OH, int OW, int K, const float* w_kc, int C,
                                   int stride, bf16_t* dx, const bf16_t* residual, const bf16_t* bn_x,
                                   const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                   const float* bn_beta, int bn_relu, double* part, void* stream) {
  const int M = N * OH * OW;
  if (stride != 1 || C % 4 || K % 4 || !al8(dy) || !al8(dx) || !aligned16(w_kc)) return DK_ERR_ARGS;
  if ((residual && !al8(residual)) || (bn_x && !al8(bn_x))) return DK_ERR_ARGS;
  if (!fits((size_t)M * K * 4) || !fits((size_t)M * C * 4) || (part != nullptr) != (bn_x != nullptr)) return DK_ERR_ARGS;
  const MatDescE<bf16_t> a = mat_h(dy, M, K, M);
  const MatDesc b = mat(w_kc, K, C, C);
  const hipStream_t st = as_stream(stream);
  if (!part) {
    EpStoreT<bf16_t> ep{dx, C, nullptr, 1, residual};
    return igemm_rows<LdMatKC, MatDescE<bf16_t>, LdMatIC, MatDesc, EpStoreT<bf16_t>, kRowPlain, kMfBf16>(a, b, ep, M, C,
                                                                                                           K, st);
  }
  if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
  EpStoreBnBwdT<bf16_t> ep{};
  ep.out = dx, ep.ldo = C, ep.bias = nullptr, ep.v4 = 1, ep.res = residual;
  ep.part = part;
  ep.xbn = bn_x;
  ep.bn = BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
  return igemm_rows<LdMatKC, MatDescE<bf16_t>, LdMatIC, MatDesc, EpStoreBnBwdT<bf16_t>, kRowPlain, kMfBf16>(
      a, b, ep, M, C, K, st);
}

// dw[k][c] = sum dy[m][k] * bn(x)[m][c] (+ l2 * w), bf16 activations, fp32 result.
DK_API int dk_pwconv_wgrad_bnx_bf16(const bf16_t* dy, const bf16_t* x, int N, int H, int W, int C, int K, int stride,
                                    int OH, int OW, const float* w_kc, float l2, float* dw_kc, void* ws,
                                    size_t ws_bytes, const float* bn_mean, const float* bn_invstd,
                                    const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream) {
  const int Kred = N * OH * OW;
  if (C % 4 || K % 4 || !al8(x) || !al8(dy) || !fits((size_t)N * H * W * C * 4) || !fits((size_t)Kred * K * 4))
    return DK_ERR_ARGS;
  if (ws_bytes < splitk_ws_bytes(K, C, Kred, kMfBf16)) return DK_ERR_WORKSPACE;
  const MatDescE<bf16_t> a = mat_h(dy, Kred, K, K);
  const ImgDescE<bf16_t> bi = img_h(x, N, H, W, C, OH, OW, 1, 1, stride, 1, 0, Kred);
  float* part = static_cast<float*>(ws);
  const hipStream_t st = as_stream(stream);
  int splits = 1, rc;
  if (bn_mean) {
    if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
    ImgBnDescE<bf16_t> b;
    static_cast<ImgDescE<bf16_t>&>(b) = bi;
    b.bn = BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
    rc = igemm_splitk<LdMatIC, MatDescE<bf16_t>, LdImgIC, ImgBnDescE<bf16_t>, kMfBf16>(a, b, part, K, C, Kred, st,
                                                                                       &splits);
  } else {
    rc = igemm_splitk<LdMatIC, MatDescE<bf16_t>, LdImgIC, ImgDescE<bf16_t>, kMfBf16>(a, bi, part, K, C, Kred, st,
                                                                                     &splits);
  }
  if (rc) return rc;
  return splitk_reduce(part, splits, K, C, dw_kc, w_kc, l2, 0, C, C, 1, 1, st);
}

DK_API int dk_pwconv_dgrad_bnbwd_bf16_stats_rows(int N, int OH, int OW, int K, int C) {
  const int M = N * OH * OW;
  if (pw_stream_bf16_dgrad_ok(K, C, M)) return pw_stream_bf16_dgrad_rows(M, K, C);
  return stats_rows(M, C, K, kRowBnBwd, kMfBf16);
}

// dk_pwconv_dgrad_bnbwd_f32 for bf16 storage: dy = the following BatchNorm's backward applied
// to (g, bn_x) as they are loaded (fp32), rounded to bf16 as the MFMA operand and as stored to
// dy_out (nullable) for the weight gradient; dx = dy . W (+ residual) stored bf16 with, given
// x / part, the input BatchNorm's backward partials over the stored dx.  Stride 1.
DK_API int dk_pwconv_dgrad_bnbwd_bf16(const bf16_t* g, const bf16_t* bn_x, int N, int OH, int OW, int K,
                                      const float* out_mean, const float* out_invstd, const float* out_gamma,
                                      const float* out_beta, int out_relu, const float* k12, bf16_t* dy_out,
                                      const float* w_kc, int C, bf16_t* dx, const bf16_t* residual, const bf16_t* x,
                                      const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                      const float* bn_beta, int bn_relu, double* part, void* stream) {
  const int M = N * OH * OW;
  if (C % 4 || K % 4 || !al8(g) || !al8(bn_x) || !al8(dx) || (dy_out && !al8(dy_out)) || !aligned16(w_kc))
    return DK_ERR_ARGS;
  if ((residual && !al8(residual)) || (x && !al8(x))) return DK_ERR_ARGS;
  if (!fits((size_t)M * K * 4) || !fits((size_t)M * C * 4) || (part != nullptr) != (x != nullptr)) return DK_ERR_ARGS;
  if (!out_mean || !out_invstd || !out_gamma || !out_beta || !k12 || (size_t)K * 32 > 64 * 1024) return DK_ERR_ARGS;
  if (pw_stream_bf16_dgrad_ok(K, C, M) && aligned16(g) && aligned16(bn_x) && (!dy_out || aligned16(dy_out)) &&
      (!part || bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta))) {
    // the streaming kernel (pw_stream_bf16.hip): bit-identical dy and dx, its own partial rows
    FoldTail ft;
    if (part) fold_take(part, pw_stream_bf16_dgrad_rows(M, K, C), C, pw_stream_bf16_dgrad_slices(K, C), &ft);
    return fold_status(pw_stream_bf16_dgrad_bnbwd(g, bn_x, M, K, C, out_mean, out_invstd, out_gamma, out_beta,
                                                  out_relu, k12, dy_out, w_kc, dx, residual, x, bn_mean, bn_invstd,
                                                  bn_gamma, bn_beta, bn_relu, part, as_stream(stream),
                                                  part ? &ft : nullptr),
                       part ? ft : FoldTail{});
  }
  MatBwdDescE<bf16_t> a;
  static_cast<MatDescE<bf16_t>&>(a) = mat_h(g, M, K, M);
  a.x = bn_x;
  a.bwd = BnBwdIn{out_mean, out_invstd, out_gamma, out_beta, k12, out_relu, K};
  a.dy_out = dy_out;
  const MatDesc b = mat(w_kc, K, C, C);
  const hipStream_t st = as_stream(stream);
  if (!part) {
    EpStoreT<bf16_t> ep{dx, C, nullptr, 1, residual};
    return igemm_rows<LdMatKC, MatBwdDescE<bf16_t>, LdMatIC, MatDesc, EpStoreT<bf16_t>, kRowBnBwd, kMfBf16>(
        a, b, ep, M, C, K, st);
  }
  if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
  EpStoreBnBwdT<bf16_t> ep{};
  ep.out = dx, ep.ldo = C, ep.bias = nullptr, ep.v4 = 1, ep.res = residual;
  ep.part = part;
  ep.xbn = x;
  ep.bn = BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
  return igemm_rows<LdMatKC, MatBwdDescE<bf16_t>, LdMatIC, MatDesc, EpStoreBnBwdT<bf16_t>, kRowBnBwd, kMfBf16>(
      a, b, ep, M, C, K, st);
}

// Fused pointwise backward for bf16 storage (dk_pwconv_bwd_bnbwd_f32's bf16 twin): the dgrad of
// dk_pwconv_dgrad_bnbwd_bf16 (dy formed on load from (g, bn_x), rounded to bf16 as the MFMA operand,
// dx bit-identical) and the weight gradient dW = dy^T bn_relu(x) (+ l2 w) in one pass, dy never
// stored.  K = C = 64, stride 1 (pw_stream_bf16.hip bwd_fused_kernel); rows = partial rows of part,
// the workspace holds rows fp32 [K][C] weight-gradient partial rows.
DK_API int dk_pwconv_bwd_fused_bf16_rows(int N, int OH, int OW, int K, int C) {
  if (N < 1 || OH < 1 || OW < 1 || (long long)N * OH * OW >= (1ll << 31)) return 0;
  const int M = N * OH * OW;
  if (pw_stream_bf16_bwd_ok(K, C, M)) return pw_stream_bf16_bwd_rows(M);
  if (pw_deep16_bwd_ok(K, C, M)) return pw_deep16_bwd_rows(M, K, C);
  return 0;
}

DK_API size_t dk_pwconv_bwd_fused_bf16_workspace_bytes(int N, int OH, int OW, int K, int C) {
  return (size_t)dk_pwconv_bwd_fused_bf16_rows(N, OH, OW, K, C) * K * C * sizeof(float);
}

DK_API int dk_pwconv_bwd_bnbwd_bf16(const bf16_t* g, const bf16_t* bn_x, int N, int OH, int OW, int K,
                                    const float* out_mean, const float* out_invstd, const float* out_gamma,
                                    const float* out_beta, int out_relu, const float* k12, const float* w_kc, int C,
                                    float l2, float* dw_kc, bf16_t* dx, const bf16_t* residual, const bf16_t* x,
                                    const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                    const float* bn_beta, int bn_relu, double* part, void* ws, size_t ws_bytes,
                                    void* stream) {
  const hipStream_t st = as_stream(stream);
  const int rows = dk_pwconv_bwd_fused_bf16_rows(N, OH, OW, K, C);
  if (rows <= 0) return DK_ERR_ARGS;
  if (!g || !bn_x || !x || !w_kc || !dw_kc || !dx || !out_mean || !out_invstd || !out_gamma || !out_beta || !k12)
    return DK_ERR_ARGS;
  if (part && !bn_mean) return DK_ERR_ARGS;
  if (bn_mean && !bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
  if (!aligned16(g) || !aligned16(bn_x) || !aligned16(w_kc) || !aligned16(ws) || !al8(x) || !al8(dx) ||
      (residual && !al8(residual)))
    return DK_ERR_ARGS;
  if (ws_bytes < (size_t)rows * K * C * sizeof(float)) return DK_ERR_WORKSPACE;
  const int M = N * OH * OW;
  float* wp = static_cast<float*>(ws);
  FoldTail ft;
  if (!pw_stream_bf16_bwd_ok(K, C, M)) {
    // K in {128, 256}: the weight-stationary kernel (pw_deep_bf16.hip); it needs the input BN's
    // partials whenever there is an input BN
    if ((bn_mean != nullptr) != (part != nullptr)) return DK_ERR_ARGS;
    if (part) fold_take(part, rows, C, pw_deep16_bwd_slices(M, K, C), &ft);
    int rc = pw_deep16_bwd_fused(g, bn_x, M, K, C, out_mean, out_invstd, out_gamma, out_beta, out_relu, k12, w_kc,
                                 dx, residual, x, bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu, part, wp, st,
                                 part ? &ft : nullptr);
    if (rc) return rc;
    return fold_status(wgrad_reduce(wp, rows, K, C, dw_kc, l2 != 0.f ? w_kc : nullptr, l2, st),
                       part ? ft : FoldTail{});
  }
  if (part) fold_take(part, rows, C, 1, &ft);
  int rc = pw_stream_bf16_bwd_fused(g, bn_x, M, out_mean, out_invstd, out_gamma, out_beta, out_relu, k12, w_kc, dx,
                                    residual, x, bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu, part, wp, st,
                                    part ? &ft : nullptr);
  if (rc) return rc;
  return fold_status(wgrad_reduce(wp, rows, K, C, dw_kc, l2 != 0.f ? w_kc : nullptr, l2, st), part ? ft : FoldTail{});
}
