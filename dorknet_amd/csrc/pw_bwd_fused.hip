// Fused pointwise backward: input gradient AND weight gradient of a stride-1 pointwise layer in
// one pass over its pixels, with the following BatchNorm's backward applied as dy is formed.
//
// Reference: PointwiseConvLayer.backward (pointwise_convolution.py:57-75):
//   dW = dy_rows^T . patches (+ l2 * W),   dx_rows = dy_rows . W
// with dy the gradient the following BatchNorm returns (batch_norm.py:125-174, stage 3 =
// dk_bn_bwd_apply_f32) and patches this layer's input rows -- after the input BatchNorm
// (+ReLU) when the layer consumed a BNOut (layers/_bn_input.py).
//
// The separate kernels this replaces read dy (or g and the BN input) twice and write it once
// (dgrad forms and stores dy; the side-stream wgrad re-reads it together with x), and read the
// layer input x twice (wgrad operand; dgrad epilogue for the input BN's partials).  Here a
// block owns 64-pixel tiles; per tile it
//   1. loads g and x1 (the following BN's raw input), forms dy = bn_bwd_elem(x1, g) into LDS
//      (never stored), and loads the raw input x into LDS;
//   2. dx[64 x C]  = dy . W        (v_mfma_f32_32x32x2_f32; W's fragments live in registers
//                                   for the block's whole life)
//      dW[K x C] += dy^T . bn_in(x) (MFMA, accumulators in registers across the block's tiles)
//   3. adds the residual, stores dx (two 128-byte row segments per store instruction), and
//      accumulates the input BatchNorm's backward partials (sum g, sum g * x_hat, ReLU mask
//      recomputed from the raw x) per column in fp64.
// At the end each block writes one row of weight-gradient partials wpart[block][K][C] and one
// row of BN partials part[block][2][C]; dk_pwconv_bwd_bnbwd_f32 then reduces wpart in a fixed
// order (+ l2 * W).  Every element's arithmetic is the unfused path's (same fp32 operations);
// only the grouping of the fp32 / fp64 reductions differs.
//
// Channel counts: K (output channels) and C (input channels) in {64, 128} -- the 56x56 and
// 28x28 depthwise-separable units of ResNet-18-depsep, whose separate kernels are HBM-bound.
#include <stdlib.h>

#include <atomic>

#include "dk_common.h"
#include "fold_tail.h"

namespace dk {

struct PwOutBn {  // the BatchNorm after this layer
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  const float* k12;  // [k1[K], k2[K]]
  int relu;
};

template <int K, int C, bool BNIN, bool PF>
__global__ __launch_bounds__(256, 2) void pw_bwd_fused_kernel(const float* __restrict__ g, const float* __restrict__ x1,
                                                           PwOutBn ob, const float* __restrict__ x, BnIn ib,
                                                           const float* __restrict__ w,
                                                           const float* __restrict__ res, float* __restrict__ dx,
                                                           double* __restrict__ part, float* __restrict__ wpart,
                                                           int P, int tpb) {
  static_assert((K == 64 || K == 128) && (C == 64 || C == 128), "K, C in {64, 128}");
  constexpr int TP = 64;                  // pixels per tile
  constexpr int SK = K + 4, SC = C + 4;   // LDS row strides (floats)
  constexpr int NCB = C / 32, NKB = K / 32;
  constexpr int DXR = NCB == 4 ? 2 : 1;   // dx row halves per wave
  constexpr int WKB = NCB == 4 ? NKB : NKB / 2;  // weight-gradient k-blocks per wave
  constexpr int GV = TP * K / 4 / 256;    // float4 of g (and x1) per thread per tile
  constexpr int XV = TP * C / 4 / 256;    // float4 of x per thread per tile
  // LDS: dy twice -- [p][k] (dx A operand: 4 consecutive k per ds_read_b128) and [k][p] (dW A
  // operand: 4 consecutive pixels) -- bn_in(x) as [c][p] (dW B operand), and with an input BN
  // the raw x as [p][c] for the epilogue's partials.  Every MFMA operand is one b128 read per
  // 4 MFMAs; the BN transforms run once per element while staging.
  constexpr int SP = TP + 4;
  __shared__ __attribute__((aligned(16))) float dys[TP * SK];
  __shared__ __attribute__((aligned(16))) float dyT[K * SP];
  __shared__ __attribute__((aligned(16))) float xbT[C * SP];
  __shared__ __attribute__((aligned(16))) float xs[BNIN ? TP * SC : 4];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int cb = wave % NCB;                       // this wave's 32-column block of C
  const int rh0 = NCB == 4 ? 0 : wave / 2;         // first dx row half
  const int kb0 = NCB == 4 ? 0 : (wave / 2) * WKB; // first weight-gradient k-block
  const int col = cb * 32 + l32;                   // this lane's column (dx, dW, partials)

  // W fragments for the dx MFMAs: wr[4q + e] = W[8q + 4h + e][col]
  float wr[K / 2];
#pragma unroll
  for (int q = 0; q < K / 8; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) wr[4 * q + e] = w[(size_t)(8 * q + 4 * h + e) * C + col];

  // following-BN coefficients for this thread's 4 dy channels (fixed: 256 % (K/4) == 0)
  const int k4 = tid % (K / 4);
  const f32x4 om = ld4(ob.mean + 4 * k4), oi = ld4(ob.invstd + 4 * k4), oga = ld4(ob.gamma + 4 * k4),
              obe = ld4(ob.beta + 4 * k4), ok1 = ld4(ob.k12 + 4 * k4), ok2 = ld4(ob.k12 + K + 4 * k4);
  const f32x4 of = oga * oi;
  // input-BN parameters for this lane's column
  float im = 0.f, ii = 0.f, ig = 0.f, ibe = 0.f;
  if constexpr (BNIN) {
    im = ib.mean[col];
    ii = ib.invstd[col];
    ig = ib.gamma[col];
    ibe = ib.beta[col];
  }
  const int c4 = tid % (C / 4);

  const uint32_t gbytes = (uint32_t)((size_t)P * K * 4), xbytes = (uint32_t)((size_t)P * C * 4);
  const __amdgpu_buffer_rsrc_t rg = make_rsrc_v(g, gbytes), r1 = make_rsrc_v(x1, gbytes), rx = make_rsrc_v(x, xbytes);

  f32x16 dwacc[WKB];
#pragma unroll
  for (int t = 0; t < WKB; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) dwacc[t][r] = 0.f;
  double s1 = 0.0, s2 = 0.0;

  const int ntiles = (P + TP - 1) / TP;
  const int t0 = blockIdx.x * tpb, t1 = min(ntiles, t0 + tpb);
  // PF (software pipelining): the next tile's g / x1 / x loads are issued right after this
  // tile's operands reach LDS, so they are in flight during the MFMAs and the epilogue (at the
  // price of VGPRs: fewer resident waves).  Either way the residual is loaded before the MFMAs.
  f32x4 gv[GV], xv1[GV], xv[XV];
  auto load_tile = [&](int p0) {
#pragma unroll
    for (int j = 0; j < GV; ++j) {
      const int px = (tid + 256 * j) / (K / 4);
      const bool ok = p0 + px < P;
      const uint32_t e = (uint32_t)((p0 + px) * K + 4 * k4);
      gv[j] = bload4e<float>(rg, ok, e);
      xv1[j] = bload4e<float>(r1, ok, e);
    }
#pragma unroll
    for (int j = 0; j < XV; ++j) {
      const int px = (tid + 256 * j) / (C / 4);
      xv[j] = bload4e<float>(rx, p0 + px < P, (uint32_t)((p0 + px) * C + 4 * c4));
    }
  };
  if (t0 < t1) load_tile(t0 * TP);
  for (int tile = t0; tile < t1; ++tile) {
    const int p0 = tile * TP;
    if constexpr (!PF) {
      if (tile != t0) load_tile(p0);
    }
    // 1. operands -> LDS
#pragma unroll
    for (int j = 0; j < GV; ++j) {
      const int px = (tid + 256 * j) / (K / 4);
      f32x4 o = {0.f, 0.f, 0.f, 0.f};
      if (p0 + px < P) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float ge = gv[j][e];
          const float xe = xv1[j][e];
          if (ob.relu && !(bn_out(xe, om[e], oi[e], oga[e], obe[e]) > 0.f)) ge = 0.f;
          o[e] = bn_bwd_elem(xe, ge, om[e], oi[e], of[e], ok1[e], ok2[e]);
        }
      }
      st4(dys + px * SK + 4 * k4, o);
#pragma unroll
      for (int e = 0; e < 4; ++e) dyT[(4 * k4 + e) * SP + px] = o[e];
    }
#pragma unroll
    for (int j = 0; j < XV; ++j) {
      const int px = (tid + 256 * j) / (C / 4);
      f32x4 xb = xv[j];
      if constexpr (BNIN) {
        st4(xs + px * SC + 4 * c4, xv[j]);
        const f32x4 m4 = ld4(ib.mean + 4 * c4), i4 = ld4(ib.invstd + 4 * c4), g4 = ld4(ib.gamma + 4 * c4),
                    b4 = ld4(ib.beta + 4 * c4);
        xb = bn_in4(xv[j], m4, i4, g4, b4, ib.relu);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) xbT[(4 * c4 + e) * SP + px] = xb[e];
    }
    __syncthreads();
    if constexpr (PF) {
      if (tile + 1 < t1) load_tile(p0 + TP);
    }
    float rv[DXR][16];
#pragma unroll
    for (int rr = 0; rr < DXR; ++rr)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int p = p0 + (rh0 + rr) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        rv[rr][r] = (res && p < P) ? res[(size_t)p * C + col] : 0.f;
      }

    // 2a. dx = dy . W
    f32x16 dxacc[DXR];
#pragma unroll
    for (int rr = 0; rr < DXR; ++rr) {
#pragma unroll
      for (int r = 0; r < 16; ++r) dxacc[rr][r] = 0.f;
      const float* arow = dys + ((rh0 + rr) * 32 + l32) * SK + 4 * h;
#pragma unroll
      for (int q = 0; q < K / 8; ++q) {
        const f32x4 a = ld4(arow + 8 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          dxacc[rr] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[e], wr[4 * q + e], dxacc[rr], 0, 0, 0);
      }
    }
    // 2b. dW += dy^T . bn_in(x)   (rows beyond P: dy is zero there)
    {
      const float* brow = xbT + col * SP + 4 * h;
#pragma unroll 2
      for (int q = 0; q < TP / 8; ++q) {
        const f32x4 b = ld4(brow + 8 * q);
        f32x4 a[WKB];
#pragma unroll
        for (int t = 0; t < WKB; ++t) a[t] = ld4(dyT + ((kb0 + t) * 32 + l32) * SP + 4 * h + 8 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int t = 0; t < WKB; ++t)
            dwacc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t][e], b[e], dwacc[t], 0, 0, 0);
      }
    }

    // 3. dx (+ residual) -> HBM; input-BN backward partials
#pragma unroll
    for (int rr = 0; rr < DXR; ++rr) {
      const int rbase = (rh0 + rr) * 32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int p = p0 + row;
        if (p < P) {
          const float v = res ? dxacc[rr][r] + rv[rr][r] : dxacc[rr][r];
          dx[(size_t)p * C + col] = v;
          if constexpr (BNIN) {
            if (part) {
              const float xr = xs[row * SC + col];
              const float xh = (xr - im) * ii;
              const float gg = (ib.relu && !(bn_out(xr, im, ii, ig, ibe) > 0.f)) ? 0.f : v;
              s1 += (double)gg;
              s2 += (double)gg * (double)xh;
            }
          }
        }
      }
    }
    __syncthreads();  // the next tile overwrites dys / xs
  }

  // weight-gradient partials: wpart[block][k][c]
  float* wp = wpart + (size_t)blockIdx.x * K * C;
#pragma unroll
  for (int t = 0; t < WKB; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = (kb0 + t) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      wp[(size_t)k * C + col] = dwacc[t][r];
    }
  // BN partials: fixed-order sum over the lanes / waves sharing a column
  if constexpr (BNIN) {
    if (part) {
      double* red = reinterpret_cast<double*>(dys);  // [256][2]
      red[2 * tid] = s1;
      red[2 * tid + 1] = s2;
      __syncthreads();
      if (tid < C) {
        const int c = tid, cbk = c / 32, lc = c % 32;
        double a = 0.0, b = 0.0;
        for (int wv = 0; wv < 4; ++wv) {
          if (wv % NCB != cbk) continue;
          for (int hh = 0; hh < 2; ++hh) {
            const int t = wv * 64 + hh * 32 + lc;
            a += red[2 * t];
            b += red[2 * t + 1];
          }
        }
        part[((size_t)blockIdx.x * 2 + 0) * C + c] = a;
        part[((size_t)blockIdx.x * 2 + 1) * C + c] = b;
      }
    }
  }
}

// Prefetch variant per shape (measured, scripts/pwf_bench.py).
static bool pwf_prefetch(int K, int C) { return K * C <= 8192; }

template <int K, int C, bool BNIN>
static const void* pwf_kernel(bool pf) {
  return pf ? reinterpret_cast<const void*>(&pw_bwd_fused_kernel<K, C, BNIN, true>)
            : reinterpret_cast<const void*>(&pw_bwd_fused_kernel<K, C, BNIN, false>);
}

static bool pwf_supported(int K, int C) { return (K == 64 || K == 128) && (C == 64 || C == 128); }

// Blocks (= partial rows): one round of resident blocks, each taking a contiguous run of
// 64-pixel tiles.  Resident blocks per CU come from the occupancy of the K, C instantiation.
static int pwf_blocks(long long P, int K, int C, int* tpb_out) {
  // (atomic: concurrent first calls may both query, and store the same value)
  static std::atomic<int> occ[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
  const bool pf = pwf_prefetch(K, C);
  std::atomic<int>& oc = occ[4 * (K == 128) + 2 * (C == 128) + pf];
  int o = oc.load(std::memory_order_relaxed);
  if (o < 0) {
    const void* f = K == 64 ? (C == 64 ? pwf_kernel<64, 64, true>(pf) : pwf_kernel<64, 128, true>(pf))
                            : (C == 64 ? pwf_kernel<128, 64, true>(pf) : pwf_kernel<128, 128, true>(pf));
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, f, 256, 0) != hipSuccess || v < 1) v = 1;
    o = v;
    oc.store(v, std::memory_order_relaxed);
  }
  const long long ntiles = (P + 63) / 64;
  long long nblk = (long long)o * 256;
  if (nblk > ntiles) nblk = ntiles;
  if (nblk < 1) nblk = 1;
  const int tpb = (int)((ntiles + nblk - 1) / nblk);
  if (tpb_out) *tpb_out = tpb;
  return (int)((ntiles + tpb - 1) / tpb);
}

int splitk_reduce(const float* ws, int splits, int M, int N, float* out, const float* w, float l2, int mode, int C,
                  int Cp, int R, int S, hipStream_t st);

}  // namespace dk

using namespace dk;

DK_API int dk_pwconv_bwd_fused_rows(int N, int OH, int OW, int K, int C) {
  if (N < 1 || OH < 1 || OW < 1) return 0;
  const long long P = (long long)N * OH * OW;
  if (P >= (1ll << 31)) return 0;
  if (pw_stream_bwd_ok(K, C, (int)P)) return pw_stream_bwd_rows((int)P);
  if (pw_deep_bwd_ok(K, C, (int)P)) return pw_deep_bwd_rows((int)P, K, C);
  if (!pwf_supported(K, C)) return 0;
  return pwf_blocks(P, K, C, nullptr);
}

// 1 when the fused backward is the faster path for this shape (the streaming kernel of
// pw_stream.hip, K = C = 64; the weight-stationary deep kernel of pw_deep.hip, K in {128, 256});
// the layers use it by default there.
DK_API int dk_pwconv_bwd_fused_preferred(int N, int OH, int OW, int K, int C) {
  if (N < 1 || OH < 1 || OW < 1 || (long long)N * OH * OW >= (1ll << 31)) return 0;
  const int P = N * OH * OW;
  return (pw_stream_bwd_ok(K, C, P) || pw_deep_bwd_ok(K, C, P)) ? 1 : 0;
}

DK_API size_t dk_pwconv_bwd_fused_workspace_bytes(int N, int OH, int OW, int K, int C) {
  return (size_t)dk_pwconv_bwd_fused_rows(N, OH, OW, K, C) * K * C * sizeof(float);
}

// The stride-s form for a layer whose input gradient the consumer takes as the compact lattice
// (dk_pwconv_dgrad_lattice_f32's output; pointwise_convolution.py:57-75 with the widen's zeros never
// stored): dk_pwconv_bwd_bnbwd_f32's one pass over the OH x OW output pixels, x (N x H x W x C, the
// layer input, with its BatchNorm applied on load) read at the stride-s lattice, dx the compact
// N x OH x OW x C.  K = C = 64 (the streaming kernel: the ResNet stem's pw0).  Rows: as
// dk_pwconv_bwd_fused_rows(N, OH, OW, K, C).
DK_API int dk_pwconv_bwd_bnbwd_lattice_f32(const float* g, const float* bn_x, int N, int OH, int OW, int K,
                                           const float* out_mean, const float* out_invstd, const float* out_gamma,
                                           const float* out_beta, int out_relu, const float* k12, const float* w_kc,
                                           int C, float l2, float* dw_kc, float* dx, const float* x, int H, int W,
                                           int stride, const float* bn_mean, const float* bn_invstd,
                                           const float* bn_gamma, const float* bn_beta, int bn_relu, double* part,
                                           void* ws, size_t ws_bytes, void* stream) {
  const hipStream_t st = as_stream(stream);
  if (N < 1 || OH < 1 || OW < 1 || stride < 2 || H < (OH - 1) * stride + 1 || W < (OW - 1) * stride + 1)
    return DK_ERR_ARGS;
  const long long P = (long long)N * OH * OW;
  if (!pw_stream_bwd_ok(K, C, (int)P) || (long long)N * H * W * C * 4 >= (1ll << 31)) return DK_ERR_ARGS;
  if (!g || !bn_x || !x || !w_kc || !dw_kc || !dx || !out_mean || !out_invstd || !out_gamma || !out_beta || !k12 ||
      !bn_mean || !bn_invstd || !bn_gamma || !bn_beta)
    return DK_ERR_ARGS;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!al(g) || !al(bn_x) || !al(x) || !al(dx) || !al(ws)) return DK_ERR_ARGS;
  const int nb = pw_stream_bwd_rows((int)P);
  if (ws_bytes < (size_t)nb * K * C * sizeof(float)) return DK_ERR_WORKSPACE;
  float* wp = static_cast<float*>(ws);
  FoldTail ft;
  if (part) fold_take(part, nb, C, 1, &ft);
  const int lat[5] = {stride, H, W, OH, OW};
  int rc = pw_stream_bwd_fused(g, bn_x, (int)P, out_mean, out_invstd, out_gamma, out_beta, out_relu, k12, w_kc, dx,
                               nullptr, x, part ? bn_mean : nullptr, bn_invstd, bn_gamma, bn_beta, bn_relu, part,
                               bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu, wp, st, part ? &ft : nullptr, lat);
  if (rc) return rc;
  return fold_status(wgrad_reduce(wp, nb, K, C, dw_kc, l2 != 0.f ? w_kc : nullptr, l2, st), part ? ft : FoldTail{});
}

DK_API int dk_pwconv_bwd_bnbwd_f32(const float* g, const float* bn_x, int N, int OH, int OW, int K,
                                   const float* out_mean, const float* out_invstd, const float* out_gamma,
                                   const float* out_beta, int out_relu, const float* k12, const float* w_kc, int C,
                                   float l2, float* dw_kc, float* dx, const float* residual, const float* x,
                                   const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                   const float* bn_beta, int bn_relu, double* part, void* ws, size_t ws_bytes,
                                   void* stream) {
  const hipStream_t st = as_stream(stream);
  if (N < 1 || OH < 1 || OW < 1 || (long long)N * OH * OW >= (1ll << 31)) return DK_ERR_ARGS;
  // the deep kernel takes an input BN only with its partials (the rows / workspace queries assume the
  // deep kernel whenever its shape fits, so that combination is refused rather than re-routed)
  const bool deep = pw_deep_bwd_ok(K, C, N * OH * OW);
  if (deep && (bn_mean != nullptr) != (part != nullptr)) return DK_ERR_ARGS;
  if (!pwf_supported(K, C) && !deep) return DK_ERR_ARGS;
  if (!g || !bn_x || !x || !w_kc || !dw_kc || !dx || !out_mean || !out_invstd || !out_gamma || !out_beta || !k12)
    return DK_ERR_ARGS;
  if (part && !bn_mean) return DK_ERR_ARGS;  // the input BN's partials need the input BN
  if (bn_mean && (!bn_invstd || !bn_gamma || !bn_beta)) return DK_ERR_ARGS;
  const long long P = (long long)N * OH * OW;
  if (P * K * 4 >= (1ll << 31) || P * C * 4 >= (1ll << 31)) return DK_ERR_ARGS;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!al(g) || !al(bn_x) || !al(x) || !al(out_mean) || !al(out_invstd) || !al(out_gamma) || !al(out_beta) ||
      !al(k12) || !al(ws))
    return DK_ERR_ARGS;
  if (pw_stream_bwd_ok(K, C, (int)P)) {
    // K = C = 64: the persistent streaming kernel (pw_stream.hip)
    const int nb = pw_stream_bwd_rows((int)P);
    if (ws_bytes < (size_t)nb * K * C * sizeof(float)) return DK_ERR_WORKSPACE;
    float* wp = static_cast<float*>(ws);
    FoldTail ft;
    if (part) fold_take(part, nb, C, 1, &ft);
    int rc = pw_stream_bwd_fused(g, bn_x, (int)P, out_mean, out_invstd, out_gamma, out_beta, out_relu, k12, w_kc, dx,
                                 residual, x, bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu, part, bn_mean,
                                 bn_invstd, bn_gamma, bn_beta, bn_relu, wp, st, part ? &ft : nullptr);
    if (rc) return rc;
    return fold_status(wgrad_reduce(wp, nb, K, C, dw_kc, l2 != 0.f ? w_kc : nullptr, l2, st),
                       part ? ft : FoldTail{});
  }
  if (deep) {
    // K in {128, 256}: the weight-stationary fused kernel (pw_deep.hip)
    const int nb = pw_deep_bwd_rows((int)P, K, C);
    if (ws_bytes < (size_t)nb * K * C * sizeof(float)) return DK_ERR_WORKSPACE;
    float* wp = static_cast<float*>(ws);
    FoldTail ft;
    if (part) fold_take(part, nb, C, pw_deep_bwd_slices((int)P, K, C), &ft);
    int rc = pw_deep_bwd_bnbwd(g, bn_x, (int)P, K, C, out_mean, out_invstd, out_gamma, out_beta, out_relu, k12, w_kc,
                               dx, residual, x, bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu, part, wp, st,
                               part ? &ft : nullptr);
    if (rc) return rc;
    return fold_status(wgrad_reduce(wp, nb, K, C, dw_kc, l2 != 0.f ? w_kc : nullptr, l2, st),
                       part ? ft : FoldTail{});
  }
  int tpb = 1;
  const int nblk = pwf_blocks(P, K, C, &tpb);
  if (ws_bytes < (size_t)nblk * K * C * sizeof(float)) return DK_ERR_WORKSPACE;
  float* wpart = static_cast<float*>(ws);
  const PwOutBn ob{out_mean, out_invstd, out_gamma, out_beta, k12, out_relu};
  const BnIn ib{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
  const bool pf = pwf_prefetch(K, C);
#define PWF_LAUNCH1(K_, C_, BN_, PF_)                                                                              \
  hipLaunchKernelGGL((pw_bwd_fused_kernel<K_, C_, BN_, PF_>), dim3(nblk), dim3(256), 0, st, g, bn_x, ob, x, ib,    \
                     w_kc, residual, dx, part, wpart, (int)P, tpb);
#define PWF_LAUNCH(K_, C_)                                                                                         \
  if (K == K_ && C == C_) {                                                                                        \
    if (bn_mean) {                                                                                                 \
      if (pf) PWF_LAUNCH1(K_, C_, true, true) else PWF_LAUNCH1(K_, C_, true, false)                                \
    } else {                                                                                                       \
      if (pf) PWF_LAUNCH1(K_, C_, false, true) else PWF_LAUNCH1(K_, C_, false, false)                              \
    }                                                                                                              \
  }
  PWF_LAUNCH(64, 64)
  PWF_LAUNCH(64, 128)
  PWF_LAUNCH(128, 64)
  PWF_LAUNCH(128, 128)
#undef PWF_LAUNCH
#undef PWF_LAUNCH1
  int rc = launch_status();
  if (rc) return rc;
  return wgrad_reduce(wpart, nblk, K, C, dw_kc, l2 != 0.f ? w_kc : nullptr, l2, st);
}
