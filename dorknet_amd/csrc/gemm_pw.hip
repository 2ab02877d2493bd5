// Pointwise (1x1) convolution entry points (layers/pointwise_convolution.py) on the implicit-GEMM
// engine (gemm_engine.h) and the streaming kernels (pw_stream.hip).
#include "gemm_engine.h"

using namespace dk;

// y[n,oh,ow,k] = sum_c x[n, oh*s, ow*s, c] * w[k][c] (+ bias)
DK_API int dk_pwconv_fwd_f32(const float* x, int N, int H, int W, int C, const float* w_kc, int K, int stride,
                             const float* bias, float* y, int OH, int OW, void* stream) {
  if (!fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  if (C % 4 == 0 && aligned16(x) && aligned16(w_kc) &&
      pw_deep_fwd_ok(K, C, N * OH * OW, (size_t)N * H * W * C * 4))
    // the deep streaming kernel (pw_deep.hip), bit-identical y (the strided skip projections)
    return pw_deep_fwd(x, N, H, W, stride, OH, OW, w_kc, K, C, bias, y, nullptr, nullptr, nullptr, nullptr, 0,
                       nullptr, as_stream(stream));
  MatDesc b = mat(w_kc, K, C, K);
  EpStore ep = ep_store(y, K, bias);
  if (C % 4 || !aligned16(x) || !aligned16(w_kc)) {
    // Unaligned channel count: scalar loads, stride 1 only (the rows are then a plain matrix).
    if (stride != 1) return DK_ERR_ARGS;
    MatDesc a = mat(x, N * H * W, C, N * H * W);
    return igemm_rows<LdMatKC1, MatDesc, LdMatKC1, MatDesc, EpStore>(a, b, ep, N * H * W, K, C, as_stream(stream));
  }
  return conv_fwd(img1(x, N, H, W, C, OH, OW, stride, N * OH * OW), w_kc, K, C, bias, y, stream);
}

// The same with x = the raw output of the previous layer and y = pw(bn(x)) (+ReLU inside).
DK_API int dk_pwconv_fwd_bnx_f32(const float* x, int N, int H, int W, int C, const float* w_kc, int K, int stride,
                                 const float* bias, float* y, int OH, int OW, const float* bn_mean,
                                 const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu,
                                 void* stream) {
  if (C % 4 || !aligned16(x) || !aligned16(w_kc) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
  return conv_fwd(with_bn(img1(x, N, H, W, C, OH, OW, stride, N * OH * OW), bn_mean, bn_invstd, bn_gamma,
                          bn_beta, bn_relu),
                  w_kc, K, C, bias, y, stream);
}

DK_API int dk_pwconv_fwd_stats_rows(int N, int OH, int OW, int K, int C) {
  const int M = N * OH * OW;
  // (the input extent does not change the choice for the shapes the network uses)
  if (pw_deep_fwd_ok(K, C, M, 0)) return pw_deep_fwd_rows(M, K, C);
  if (pw_stream_fwd_ok(K, C, M, 0)) return pw_stream_fwd_rows(M, K);
  return stats_rows(M, K, C);
}

DK_API int dk_pwconv_fwd_ex_f32(const float* x, int N, int H, int W, int C, const float* w_kc, int K, int stride,
                                const float* bias, float* y, int OH, int OW, const float* bn_mean,
                                const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu,
                                double* stats, void* stream) {
  if (C % 4 || !aligned16(x) || !aligned16(w_kc) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  if (pw_deep_fwd_ok(K, C, N * OH * OW, (size_t)N * H * W * C * 4)) {
    // the deep streaming kernel (pw_deep.hip): bit-identical y, its own partial rows and slices
    // (dk_pwconv_fwd_stats_rows sized the partials for it: no other path may take this call)
    if (bn_mean && !bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
    const int M = N * OH * OW;
    FoldTail ft;
    if (stats) fold_take(stats, pw_deep_fwd_rows(M, K, C), K, pw_deep_fwd_slices(M, K, C), &ft);
    return fold_status(pw_deep_fwd(x, N, H, W, stride, OH, OW, w_kc, K, C, bias, y, bn_mean, bn_invstd, bn_gamma,
                                   bn_beta, bn_relu, stats, as_stream(stream), stats ? &ft : nullptr),
                       stats ? ft : FoldTail{});
  }
  if (pw_stream_fwd_ok(K, C, N * OH * OW, (size_t)N * H * W * C * 4) && (!bn_mean || bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)))
    // K = C = 64 / 128: the persistent streaming kernel (pw_stream.hip), bit-identical outputs
  {
    FoldTail ft;
    if (stats) fold_take(stats, pw_stream_fwd_rows(N * OH * OW, K), K, 1, &ft);
    return fold_status(pw_stream_fwd(x, N, H, W, stride, OH, OW, w_kc, K, bias, y, bn_mean, bn_invstd, bn_gamma,
                                     bn_beta, bn_relu, stats, as_stream(stream), stats ? &ft : nullptr),
                       stats ? ft : FoldTail{});
  }
  return conv_fwd_ex(img1(x, N, H, W, C, OH, OW, stride, N * OH * OW), w_kc, K, C, bias, y, bn_mean,
                     bn_invstd, bn_gamma, bn_beta, bn_relu, stats, stream);
}

// Pointwise dgrad (pointwise_convolution.py:65-72): dx_rows = dy_rows . W; for stride > 1 the
// result is widened to (OH*s, OW*s) with zeros off the sampling lattice.
DK_API int dk_pwconv_dgrad_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kc, int C, int stride,
                               float* dx, void* stream) {
  const int M = N * OH * OW;
  if (!fits((size_t)M * K * 4)) return DK_ERR_ARGS;
  MatDesc a = mat(dy, M, K, M);
  MatDesc b = mat(w_kc, K, C, C);
  const hipStream_t st = as_stream(stream);
  const bool vec = vec_ok(a, K, 4) && vec_ok(b, 4, C);
  if (stride == 1 && vec && aligned16(dy) && aligned16(w_kc) && aligned16(dx) && pw_deep_dgrad_ok(K, C, M))
    // the deep dgrad kernel's plain form (pw_deep.hip): bit-identical dx (the skip projections)
    return pw_deep_dgrad_plain(dy, M, K, C, w_kc, dx, st);
  if (stride == 1) {
    EpStore ep = ep_store(dx, C, nullptr);
    if (vec) return igemm_rows<LdMatKC, MatDesc, LdMatIC, MatDesc, EpStore>(a, b, ep, M, C, K, st);
    return igemm_rows<LdMatKC1, MatDesc, LdMatIC1, MatDesc, EpStore>(a, b, ep, M, C, K, st);
  }
  EpWiden ep = ep_widen(dx, C, OH, OW, stride);
  if (vec) return igemm_rows<LdMatKC, MatDesc, LdMatIC, MatDesc, EpWiden>(a, b, ep, M, C, K, st);
  return igemm_rows<LdMatKC1, MatDesc, LdMatIC1, MatDesc, EpWiden>(a, b, ep, M, C, K, st);
}

DK_API int dk_pwconv_dgrad_stats_rows(int N, int OH, int OW, int K, int C) { return stats_rows(N * OH * OW, C, K); }
DK_API int dk_pwconv_dgrad_bnbwd_stats_rows(int N, int OH, int OW, int K, int C) {
  const int M = N * OH * OW;
  if (pw_deep_dgrad_ok(K, C, M)) return pw_deep_dgrad_rows(M, K, C);
  if (pw_stream_dgrad_ok(K, C, M)) return pw_stream_dgrad_rows(M);
  return stats_rows(M, C, K, kRowBnBwd);
}

// dgrad + the BN-backward partial sums of the BatchNorm whose output this layer consumed
// (bn_x = that BN's raw input, on the dx grid; part: dk_pwconv_dgrad_stats_rows() x 2 x C).
DK_API int dk_pwconv_dgrad_ex_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kc, int C, int stride,
                                  float* dx, const float* residual, const float* bn_x, const float* bn_mean,
                                  const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu,
                                  double* part, void* stream) {
  const int M = N * OH * OW;
  if (!fits((size_t)M * K * 4) || (part != nullptr) != (bn_x != nullptr)) return DK_ERR_ARGS;
  if (part && (!bn_mean || !bn_invstd || !bn_gamma || !bn_beta)) return DK_ERR_ARGS;
  if (part && residual && stride != 1) return DK_ERR_ARGS;  // off-lattice residual terms would need reducing
  MatDesc a = mat(dy, M, K, M);
  MatDesc b = mat(w_kc, K, C, C);
  const hipStream_t st = as_stream(stream);
  const bool vec = vec_ok(a, K, 4) && vec_ok(b, 4, C);
#define DK_ROWS(EPT, ep)                                                              \
  return vec ? igemm_rows<LdMatKC, MatDesc, LdMatIC, MatDesc, EPT>(a, b, ep, M, C, K, st) \
             : igemm_rows<LdMatKC1, MatDesc, LdMatIC1, MatDesc, EPT>(a, b, ep, M, C, K, st)
  if (!part) {
    if (stride == 1) {
      EpStore ep = ep_store(dx, C, nullptr, residual);
      DK_ROWS(EpStore, ep);
    }
    EpWiden ep = ep_widen(dx, C, OH, OW, stride, residual);
    DK_ROWS(EpWiden, ep);
  }
  const BnIn bn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
  const int xv4 = aligned16(bn_x) && bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta);
  if (stride == 1) {
    EpStoreBnBwd ep;
    static_cast<EpStore&>(ep) = ep_store(dx, C, nullptr, residual);
    ep.v4 = ep.v4 && xv4;
    ep.part = part;
    ep.xbn = bn_x;
    ep.bn = bn;
    DK_ROWS(EpStoreBnBwd, ep);
  }
  EpWidenBnBwd ep;
  static_cast<EpWiden&>(ep) = ep_widen(dx, C, OH, OW, stride);
  ep.v4 = ep.v4 && xv4;
  ep.part = part;
  ep.xbn = bn_x;
  ep.bn = bn;
  DK_ROWS(EpWidenBnBwd, ep);
#undef DK_ROWS
}

// dk_pwconv_dgrad_ex_f32 with the input BN's partials for stride > 1, the widened gradient kept
// compact (EpLatticeBnBwd): dx_lat[n][oh][ow][c] = the widened dx at (n, s*oh, s*ow, c), the
// rest of the widened grid being zero; part has dk_pwconv_dgrad_stats_rows() rows.
DK_API int dk_pwconv_dgrad_lattice_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kc, int C,
                                       int stride, float* dx_lat, const float* bn_x, const float* bn_mean,
                                       const float* bn_invstd, const float* bn_gamma, const float* bn_beta,
                                       int bn_relu, double* part, void* stream) {
  const int M = N * OH * OW;
  if (!fits((size_t)M * K * 4) || !fits((size_t)M * C * 4) || stride < 2 || !dx_lat || !bn_x || !part)
    return DK_ERR_ARGS;
  if (!bn_mean || !bn_invstd || !bn_gamma || !bn_beta) return DK_ERR_ARGS;
  MatDesc a = mat(dy, M, K, M);
  MatDesc b = mat(w_kc, K, C, C);
  const hipStream_t st = as_stream(stream);
  const bool vec = vec_ok(a, K, 4) && vec_ok(b, 4, C);
  EpLatticeBnBwd ep;
  static_cast<EpWiden&>(ep) = ep_widen(dx_lat, C, OH, OW, stride);
  ep.v4 = ep.v4 && aligned16(bn_x) && bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta);
  ep.part = part;
  ep.xbn = bn_x;
  ep.bn = BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
  return vec ? igemm_rows<LdMatKC, MatDesc, LdMatIC, MatDesc, EpLatticeBnBwd>(a, b, ep, M, C, K, st)
             : igemm_rows<LdMatKC1, MatDesc, LdMatIC1, MatDesc, EpLatticeBnBwd>(a, b, ep, M, C, K, st);
}

// dgrad of a stride-1 pointwise layer whose output fed a BatchNorm (+ReLU), with that BN's
// backward apply (dk_bn_bwd_apply_f32) done on load: g = the gradient w.r.t. the BN(+ReLU)
// output, bn_x = the BN's raw input (= this layer's output), k12 from
// dk_bn_bwd_from_partials_f32.  dy_out (nullable) receives dy = the gradient w.r.t. bn_x,
// bit-identical to dk_bn_bwd_apply_f32's, for this layer's weight gradient.  The epilogue
// options (residual, the partials of the BN before this layer) are those of
// dk_pwconv_dgrad_ex_f32 at stride 1; part has dk_pwconv_dgrad_bnbwd_stats_rows() rows.
DK_API int dk_pwconv_dgrad_bnbwd_f32(const float* g, const float* bn_x, int N, int OH, int OW, int K,
                                     const float* out_mean, const float* out_invstd, const float* out_gamma,
                                     const float* out_beta, int out_relu, const float* k12, float* dy_out,
                                     const float* w_kc, int C, float* dx, const float* residual, const float* x,
                                     const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                     const float* bn_beta, int bn_relu, double* part, void* stream) {
  const int M = N * OH * OW;
  if (!fits((size_t)M * K * 4) || (part != nullptr) != (x != nullptr)) return DK_ERR_ARGS;
  if (part && (!bn_mean || !bn_invstd || !bn_gamma || !bn_beta)) return DK_ERR_ARGS;
  if (!out_mean || !out_invstd || !out_gamma || !out_beta || !k12 || !bn_x) return DK_ERR_ARGS;
  MatBwdDesc a;
  static_cast<MatDesc&>(a) = mat(g, M, K, M);
  a.x = bn_x;
  a.bwd = BnBwdIn{out_mean, out_invstd, out_gamma, out_beta, k12, out_relu, K};
  a.dy_out = dy_out;
  MatDesc b = mat(w_kc, K, C, C);
  const hipStream_t st = as_stream(stream);
  // 16-byte loads of g, bn_x and dy_out; the LDS table holds 2 float4 per channel
  if (!vec_ok(b, 4, C) || K % 4 || !aligned16(g) || !aligned16(bn_x) || (dy_out && !aligned16(dy_out)) ||
      (size_t)K * 32 > 64 * 1024)
    return DK_ERR_ARGS;
  if (pw_deep_dgrad_ok(K, C, M)) {
    // the deep streaming kernel (pw_deep.hip): bit-identical dy and dx, its own partial rows
    // (sized by dk_pwconv_dgrad_bnbwd_stats_rows: no other path may take this call)
    if (part && !bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
    FoldTail ft;
    if (part) fold_take(part, pw_deep_dgrad_rows(M, K, C), C, pw_deep_dgrad_slices(M, K, C), &ft);
    return fold_status(pw_deep_dgrad_bnbwd(g, bn_x, M, K, C, out_mean, out_invstd, out_gamma, out_beta, out_relu, k12,
                                           dy_out, w_kc, dx, residual, part ? x : nullptr, bn_mean, bn_invstd,
                                           bn_gamma, bn_beta, bn_relu, part, st, part ? &ft : nullptr),
                       part ? ft : FoldTail{});
  }
  if (pw_stream_dgrad_ok(K, C, M)) {
    // K = C = 64: the persistent streaming kernel (pw_stream.hip), bit-identical results
    if (part && !bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
    FoldTail ft;
    if (part) fold_take(part, pw_stream_dgrad_rows(M), C, 1, &ft);
    return fold_status(pw_stream_dgrad_bnbwd(g, bn_x, M, out_mean, out_invstd, out_gamma, out_beta, out_relu, k12,
                                             dy_out, w_kc, dx, residual, part ? x : nullptr, bn_mean, bn_invstd,
                                             bn_gamma, bn_beta, bn_relu, part, st, part ? &ft : nullptr),
                       part ? ft : FoldTail{});
  }
  if (!part) {
    EpStore ep = ep_store(dx, C, nullptr, residual);
    return igemm_rows<LdMatKC, MatBwdDesc, LdMatIC, MatDesc, EpStore, kRowBnBwd>(a, b, ep, M, C, K, st);
  }
  EpStoreBnBwd ep;
  static_cast<EpStore&>(ep) = ep_store(dx, C, nullptr, residual);
  ep.v4 = ep.v4 && aligned16(x) && bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta);
  ep.part = part;
  ep.xbn = x;
  ep.bn = BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
  return igemm_rows<LdMatKC, MatBwdDesc, LdMatIC, MatDesc, EpStoreBnBwd, kRowBnBwd>(a, b, ep, M, C, K, st);
}

DK_API size_t dk_pwconv_wgrad_workspace_bytes(int N, int OH, int OW, int K, int C) {
  // (the bf16 twin's tiles can differ: the larger of the two)
  const int M = N * OH * OW;
  size_t a = splitk_ws_bytes(K, C, M), b = splitk_ws_bytes(K, C, M, kMfBf16);
  if (a < b) a = b;
  return a;
}

// dw[k][c] = sum_{n,oh,ow} dy[n,oh,ow,k] * x[n, oh*s, ow*s, c]  (+ l2 * w)   (pointwise_convolution.py:61-64)
DK_API int dk_pwconv_wgrad_f32(const float* dy, const float* x, int N, int H, int W, int C, int K, int stride,
                               int OH, int OW, const float* w_kc, float l2, float* dw_kc, void* ws, size_t ws_bytes,
                               void* stream) {
  if (C % 4 || !aligned16(x) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  const int M = N * OH * OW;
  return wgrad(dy, img(x, N, H, W, C, OH, OW, 1, 1, stride, 1, 0, M), K, C, w_kc, l2, dw_kc, 0, C, C, 1, 1,
               ws, ws_bytes, stream);
}

DK_API int dk_pwconv_wgrad_bnx_f32(const float* dy, const float* x, int N, int H, int W, int C, int K, int stride,
                                   int OH, int OW, const float* w_kc, float l2, float* dw_kc, void* ws,
                                   size_t ws_bytes, const float* bn_mean, const float* bn_invstd,
                                   const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream) {
  if (C % 4 || !aligned16(x) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
  const int M = N * OH * OW;
  return wgrad(dy,
               with_bn(img(x, N, H, W, C, OH, OW, 1, 1, stride, 1, 0, N * OH * OW), bn_mean, bn_invstd, bn_gamma,
                       bn_beta, bn_relu),
               K, C, w_kc, l2, dw_kc, 0, C, C, 1, 1, ws, ws_bytes, stream);
}

