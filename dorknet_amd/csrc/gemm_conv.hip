// Dense convolution entry points (layers/convolution.py) on the implicit-GEMM engine
// (gemm_engine.h), plus the engine's tuning knobs.
#include "gemm_engine.h"

using namespace dk;

namespace dk {

// Weight re-layouts (tiny; run once per call on the caller's stream).
__global__ void w_kcrs_to_krsc_kernel(const float* __restrict__ w, int K, int C, int R, int S, int Cp,
                                      float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // over K*R*S*Cp
  const int total = K * R * S * Cp;
  if (idx >= total) return;
  const int c = idx % Cp;
  int t = idx / Cp;
  const int s = t % S;
  t /= S;
  const int r = t % R;
  const int k = t / R;
  out[idx] = c < C ? w[(((size_t)k * C + c) * R + r) * S + s] : 0.f;
}

__global__ void w_kcrs_to_crsk_kernel(const float* __restrict__ w, int K, int C, int R, int S,
                                      float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // over C*R*S*K
  const int total = K * R * S * C;
  if (idx >= total) return;
  const int k = idx % K;
  int t = idx / K;
  const int s = t % S;
  t /= S;
  const int r = t % R;
  const int c = t / R;
  out[idx] = w[(((size_t)k * C + c) * R + r) * S + s];
}

// Sub-pixel phase sub-filters of a stride-st dgrad: for phase (a, b) the taps r = r0(a) + st*r',
// s = s0(b) + st*s' as a [C][R'][S'][Kp] matrix (Kp = K rounded up to 4, zero-filled).
__global__ void w_phase_kernel(const float* __restrict__ w, int K, int C, int R, int S, int st, int pad, int Kp,
                               float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // over C * R * S * Kp
  if (idx >= C * R * S * Kp) return;
  const int k = idx % Kp;
  int t = idx / Kp;
  const int s_ = t % S;
  t /= S;
  const int r = t % R;
  const int c = t / R;
  const int a = ((r - pad) % st + st) % st, b = ((s_ - pad) % st + st) % st;
  const int r0 = phase_r0(a, st, pad), s0 = phase_r0(b, st, pad);
  const int Rp = phase_taps(a, R, st, pad), Sp = phase_taps(b, S, st, pad);
  const int rp = (r - r0) / st, sp = (s_ - s0) / st;
  out[phase_block_offset(a, b, C, R, S, st, pad, Kp) + ((size_t)(c * Rp + rp) * Sp + sp) * Kp + k] =
      k < K ? w[(((size_t)k * C + c) * R + r) * S + s_] : 0.f;
}

}  // namespace dk

// Tuning knobs (knobs.hip): kind = the KnobId; cfg = -1 restores the default.
DK_API int dk_debug_set_gemm_config(int kind, int cfg) {
  // unused / retired numbers (knobs.hip) and the internal launch variant are refused
  if (kind < 0 || kind >= kNumKnobs || kind == 5 || kind == 6 || kind == 10 || kind == 12 || (kind >= 15 && kind <= 17) ||
      kind == 20 || kind == 22 || kind == kKnobEwVariant)
    return -1;
  knob_set(kind, cfg);
  return kind == kKnobRowCfg ? kNumRowCfg : kind == kKnobSplitCfg ? kNumSplitCfg : 0;
}

DK_API int dk_conv_weight_krsc_f32(const float* w_kcrs, int K, int C, int R, int S, int Cp, float* w_krsc,
                                   void* stream) {
  const int total = K * R * S * Cp;
  hipLaunchKernelGGL(w_kcrs_to_krsc_kernel, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), w_kcrs, K, C, R,
                     S, Cp, w_krsc);
  return launch_status();
}

DK_API int dk_conv_weight_crsk_f32(const float* w_kcrs, int K, int C, int R, int S, float* w_crsk, void* stream) {
  const int total = K * R * S * C;
  hipLaunchKernelGGL(w_kcrs_to_crsk_kernel, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), w_kcrs, K, C, R,
                     S, w_crsk);
  return launch_status();
}

DK_API int dk_conv2d_fwd_f32(const float* x, int N, int H, int W, int C, const float* w_krsc, int K, int R, int S,
                             int stride, int pad, const float* bias, float* y, int OH, int OW, void* stream) {
  if (C % 4 || !aligned16(x) || !aligned16(w_krsc) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  return conv_fwd(img(x, N, H, W, C, OH, OW, R, S, stride, 1, -pad, N * OH * OW), w_krsc, K, R * S * C, bias, y,
                  stream);
}

DK_API int dk_conv2d_fwd_bnx_f32(const float* x, int N, int H, int W, int C, const float* w_krsc, int K, int R, int S,
                                 int stride, int pad, const float* bias, float* y, int OH, int OW,
                                 const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                 const float* bn_beta, int bn_relu, void* stream) {
  if (C % 4 || !aligned16(x) || !aligned16(w_krsc) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
  return conv_fwd(with_bn(img(x, N, H, W, C, OH, OW, R, S, stride, 1, -pad, N * OH * OW), bn_mean, bn_invstd,
                          bn_gamma, bn_beta, bn_relu),
                  w_krsc, K, R * S * C, bias, y, stream);
}

DK_API int dk_conv2d_fwd_stats_rows(int N, int OH, int OW, int K, int C, int R, int S) {
  return stats_rows(N * OH * OW, K, R * S * C, kRowConv);
}

// Forward with optional BN on load (bn_mean != NULL) and optional output statistics
// (stats != NULL: dk_conv2d_fwd_stats_rows() x 2 x K doubles, for dk_bn_stats_from_partials_f32).
DK_API int dk_conv2d_fwd_ex_f32(const float* x, int N, int H, int W, int C, const float* w_krsc, int K, int R, int S,
                                int stride, int pad, const float* bias, float* y, int OH, int OW,
                                const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                const float* bn_beta, int bn_relu, double* stats, void* stream) {
  if (C % 4 || !aligned16(x) || !aligned16(w_krsc) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  return conv_fwd_ex(img(x, N, H, W, C, OH, OW, R, S, stride, 1, -pad, N * OH * OW), w_krsc, K, R * S * C, bias, y,
                     bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu, stats, stream);
}

// Stride-1 dgrad as an implicit GEMM: dx[n,h,w,c] = sum_{r,s,k} dy[n, h+pad-r, w+pad-s, k] * w[k][c][r][s]
DK_API int dk_conv2d_dgrad_f32(const float* dy, int N, int OH, int OW, int K, const float* w_crsk, int C, int R,
                               int S, int pad, float* dx, int H, int W, void* stream) {
  if (K % 4 || !aligned16(dy) || !aligned16(w_crsk) || !fits((size_t)N * OH * OW * K * 4)) return DK_ERR_ARGS;
  ImgDesc a = img(dy, N, OH, OW, K, H, W, R, S, 1, -1, pad, N * H * W);
  const int Ktot = R * S * K;
  MatDesc b = mat(w_crsk, C, Ktot, C);
  EpStore ep = ep_store(dx, C, nullptr);
  return igemm_rows<LdImgKC, ImgDesc, LdMatKC, MatDesc, EpStore>(a, b, ep, N * H * W, C, Ktot, as_stream(stream));
}

// Sub-pixel phase geometry of a stride-st, pad-p correlation's input gradient along one axis:
// phase a's taps are r0 + st*t (t < Rp), reading dy row i + nb0 - t for dx row st*i + a.
struct PhaseAxis {
  int r0, Rp, nb0, Op;
};
static inline PhaseAxis phase_axis(int a, int R, int st, int pad, int L) {
  PhaseAxis p;
  p.r0 = phase_r0(a, st, pad);
  p.Rp = phase_taps(a, R, st, pad);
  p.nb0 = (a + pad - p.r0) / st;
  p.Op = a < L ? (L - a + st - 1) / st : 0;
  return p;
}

DK_API size_t dk_conv2d_dgrad_phase_workspace_bytes(int K, int C, int R, int S, int stride) {
  if (K < 1 || C < 1 || R < 1 || S < 1 || stride < 1) return 0;
  const size_t kp = (size_t)((K + 3) / 4 * 4);
  return (size_t)C * R * S * kp * sizeof(float);
}

// Input gradient of any-stride convolution as one implicit GEMM per sub-pixel phase (replaces
// cp.dot(dy, W_flat) + row2im, convolution.py:101-117 / :205-222: no column matrix, no atomics):
// phase (a, b) is a stride-1 correlation of dy with its sub-filter, written to the dx pixels
// (st*i + a, st*j + b).  dy has Kp = K rounded up to 4 channels (zero-padded by the caller when
// K % 4 != 0); phases with no taps (R or S < stride) write zeros.
DK_API int dk_conv2d_dgrad_phase_f32(const float* dy, int N, int OH, int OW, int Kp, int K, const float* w_kcrs,
                                     int C, int R, int S, int stride, int pad, float* dx, int H, int W, void* ws,
                                     size_t ws_bytes, void* stream) {
  if (Kp % 4 || Kp < K || stride < 1 || stride > 8 || N < 1 || C < 1 || !aligned16(dy) || !aligned16(ws))
    return DK_ERR_ARGS;
  if (ws_bytes < dk_conv2d_dgrad_phase_workspace_bytes(K, C, R, S, stride) || Kp != (K + 3) / 4 * 4)
    return DK_ERR_WORKSPACE;
  if (!fits((size_t)N * OH * OW * Kp * 4) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  const hipStream_t st = as_stream(stream);
  float* wsub = static_cast<float*>(ws);
  const int total = C * R * S * Kp;
  hipLaunchKernelGGL(w_phase_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, w_kcrs, K, C, R, S, stride, pad, Kp,
                     wsub);
  int rc = launch_status();
  if (rc) return rc;
  for (int a = 0; a < stride; ++a)
    for (int b = 0; b < stride; ++b) {
      const PhaseAxis pa = phase_axis(a, R, stride, pad, H), pb = phase_axis(b, S, stride, pad, W);
      if (pa.Op == 0 || pb.Op == 0) continue;  // no dx pixels of this phase
      const int M = N * pa.Op * pb.Op;
      ImgDesc d = img(dy, N, OH, OW, Kp, pa.Op, pb.Op, pa.Rp, pb.Rp, 1, -1, pa.nb0, M);
      d.offw = pb.nb0;
      const int Ktot = pa.Rp * pb.Rp * Kp;
      const float* wp = wsub + phase_block_offset(a, b, C, R, S, stride, pad, Kp);
      MatDesc bm = mat(wp, C, Ktot > 0 ? Ktot : 4, C);
      EpPhase ep{dx, C, pa.Op, pb.Op, H, W, stride, a, b, al4(C) && aligned16(dx)};
      rc = igemm_rows<LdImgKC, ImgDesc, LdMatKC, MatDesc, EpPhase>(d, bm, ep, M, C, Ktot, st);
      if (rc) return rc;
    }
  return 0;
}

DK_API size_t dk_conv2d_wgrad_workspace_bytes(int N, int OH, int OW, int K, int Cp, int R, int S) {
  return splitk_ws_bytes(K, R * S * Cp, N * OH * OW);
}

DK_API int dk_conv2d_wgrad_f32(const float* dy, const float* x, int N, int H, int W, int Cp, int C, int K, int R,
                               int S, int stride, int pad, int OH, int OW, const float* w_kcrs, float l2,
                               float* dw_kcrs, void* ws, size_t ws_bytes, void* stream) {
  if (Cp % 4 || !aligned16(x) || !fits((size_t)N * H * W * Cp * 4)) return DK_ERR_ARGS;
  return wgrad(dy, img(x, N, H, W, Cp, OH, OW, R, S, stride, 1, -pad, N * OH * OW), K, R * S * Cp, w_kcrs, l2,
               dw_kcrs, 1, C, Cp, R, S, ws, ws_bytes, stream);
}

DK_API int dk_conv2d_wgrad_bnbwd_f32(const float* g, const float* bn_x, const float* x, int N, int H, int W, int Cp,
                                     int C, int K,
                                     int R, int S, int stride, int pad, int OH, int OW, const float* out_mean,
                                     const float* out_invstd, const float* out_gamma, const float* out_beta,
                                     int out_relu, const float* k12, const float* w_kcrs, float l2, float* dw_kcrs,
                                     void* ws, size_t ws_bytes, const float* bn_mean, const float* bn_invstd,
                                     const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream) {
  if (Cp % 4 || K % 4 || !aligned16(x) || !fits((size_t)N * H * W * Cp * 4)) return DK_ERR_ARGS;
  if (!out_mean || !out_invstd || !out_gamma || !out_beta || !k12) return DK_ERR_ARGS;
  const BnBwdIn bw{out_mean, out_invstd, out_gamma, out_beta, k12, out_relu, K};
  if (bn_mean) {
    if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
    return wgrad_bnbwd(g, bn_x,
                       with_bn(img(x, N, H, W, Cp, OH, OW, R, S, stride, 1, -pad, N * OH * OW), bn_mean,
                               bn_invstd, bn_gamma, bn_beta, bn_relu),
                       K, R * S * Cp, bw, w_kcrs, l2, dw_kcrs, C, Cp, R, S, ws, ws_bytes, stream);
  }
  return wgrad_bnbwd(g, bn_x, img(x, N, H, W, Cp, OH, OW, R, S, stride, 1, -pad, N * OH * OW), K,
                     R * S * Cp, bw, w_kcrs, l2, dw_kcrs, C, Cp, R, S, ws, ws_bytes, stream);
}

DK_API int dk_conv2d_wgrad_bnx_f32(const float* dy, const float* x, int N, int H, int W, int Cp, int C, int K, int R,
                                   int S, int stride, int pad, int OH, int OW, const float* w_kcrs, float l2,
                                   float* dw_kcrs, void* ws, size_t ws_bytes, const float* bn_mean,
                                   const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu,
                                   void* stream) {
  if (Cp % 4 || !aligned16(x) || !fits((size_t)N * H * W * Cp * 4)) return DK_ERR_ARGS;
  if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
  return wgrad(dy,
               with_bn(img(x, N, H, W, Cp, OH, OW, R, S, stride, 1, -pad, N * OH * OW), bn_mean, bn_invstd, bn_gamma,
                       bn_beta, bn_relu),
               K, R * S * Cp, w_kcrs, l2, dw_kcrs, 1, C, Cp, R, S, ws, ws_bytes, stream);
}

// Pointwise (1x1) forward with optional stride-s subsampling (pointwise_convolution.py:46-55):
