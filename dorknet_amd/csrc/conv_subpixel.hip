// Strided convolution input-gradient by sub-pixel decomposition (gfx950).
//
// Replaces the dgrad half of ConvLayer.backward for stride > 1 (layers/convolution.py:101-111:
// cp.dot(upstream, W_flat) into a [N*OH*OW, C*R*S] column matrix, then the atomicAdd
// row2im scatter :205-222).  The column matrix is M*C*R*S floats -- ~1 GB for the
// ResNet stem at batch 256 -- and writing it plus reading it back dominates that layer.
//
// Here no column matrix exists.  With h = ST*i + a (a = the sub-pixel phase), the taps
// that reach dx row h are exactly those r with (a + pad - r) % ST == 0, and they read dy row
// i + (a + pad - r)/ST.  So every tap r has a fixed phase a(r) and a fixed neighbour offset
// di(r): one "quad" (the ST x ST block of dx pixels sharing i, j) reads a small fixed dy
// neighbourhood, and each tap feeds exactly one phase of the quad.  Thread = quad; the dy
// neighbourhood of a 4 x 64 quad tile is staged through LDS 16 channels at a time, the
// weights are wave-uniform (scalar loads), and the k-sum is split over even/odd k so each
// multiply-add is one packed v_pk_fma_f32 (2 MACs) with both halves from register pairs.
//
// The output channel count C is small for the layers this serves (the stem: C = 3): each
// thread owns CO <= 4 channels of its quad; wider C runs as ceil(C / CO) channel groups.
#include "dk_common.h"

namespace dk {
namespace {

constexpr int kTI = 4;          // quad rows per block (one wave each)
constexpr int kTJ = 64;         // quad columns per block (one lane each)
constexpr int kKC = 16;         // dy channels staged per pass
constexpr int kKS = kKC + 4;    // LDS floats per staged pixel (80 B stride: conflict-free b128)

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int R, int S, int ST, int PAD, int CO>
__global__ __launch_bounds__(256) void conv_dgrad_subpixel_kernel(const float* __restrict__ dy, int OH, int OW,
                                                                 int K, const float* __restrict__ wt, int KP,
                                                                 int C, int ncg, float* __restrict__ dx, int H,
                                                                 int W, int QH, int QW) {
  using RP = SubPix<R, ST, PAD>;
  using SP = SubPix<S, ST, PAD>;
  constexpr int DR0 = RP::dmin(), DR1 = RP::dmax();
  constexpr int DS0 = SP::dmin(), DS1 = SP::dmax();
  constexpr int NR = DR1 - DR0 + 1, NS = DS1 - DS0 + 1;
  constexpr int LR = kTI + NR - 1, LC = kTJ + NS - 1;
  constexpr int KQ = kKC / 4;
  __shared__ __attribute__((aligned(16))) float tile[LR * LC * kKS];

  const int tid = threadIdx.x;
  const int li = tid >> 6, lj = tid & 63;
  // XCD-contiguous block order (vertically adjacent tiles share dy halo rows)
  const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int L = xcd_block(lin, gridDim.x * gridDim.y * gridDim.z);
  const int bx = L % gridDim.x, by = (L / gridDim.x) % gridDim.y, bz = L / (gridDim.x * gridDim.y);
  const int i0 = by * kTI, j0 = bx * kTJ;
  const int n = bz / ncg;
  const int cg = bz - n * ncg;
  const float* dyn = dy + (size_t)n * OH * OW * K;
  const bool vec = (K & 3) == 0 && (reinterpret_cast<uintptr_t>(dy) & 15) == 0;
  const float* wcg = wt + (size_t)cg * KP * (R * S * CO * 2);

  f32x2 acc[ST * ST][CO];
#pragma unroll
  for (int p = 0; p < ST * ST; ++p)
#pragma unroll
    for (int c = 0; c < CO; ++c) acc[p][c] = f32x2{0.f, 0.f};

  for (int k0 = 0; k0 < K; k0 += kKC) {
    for (int e = tid; e < LR * LC * KQ; e += 256) {
      const int q = e % KQ;
      const int p = e / KQ;
      const int row = p / LC, col = p - (p / LC) * LC;
      const int oh = i0 + DR0 + row, ow = j0 + DS0 + col;
      const int k = k0 + 4 * q;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if ((unsigned)oh < (unsigned)OH && (unsigned)ow < (unsigned)OW) {
        const float* src = dyn + ((size_t)oh * OW + ow) * K + k;
        if (vec) {
          if (k < K) v = ld4(src);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (k + t < K) v[t] = src[t];
        }
      }
      st4(&tile[p * kKS + 4 * q], v);
    }
    __syncthreads();

    const int kend = K - k0 < kKC ? K - k0 : kKC;
    for (int kk = 0; kk < kend; kk += 4) {
      f32x4 d[NR][NS];
#pragma unroll
      for (int a = 0; a < NR; ++a)
#pragma unroll
        for (int b = 0; b < NS; ++b) d[a][b] = ld4(&tile[((li + a) * LC + (lj + b)) * kKS + kk]);
      // weights: wt[cg][kp][r][s][c][2], kp = k pair; this 4-k step covers pairs kp, kp+1
      const float* w0 = wcg + (size_t)((k0 + kk) >> 1) * (R * S * CO * 2);
#pragma unroll
      for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const f32x4 dv = d[RP::nb(r) - DR0][SP::nb(s) - DS0];
          const f32x2 lo = f32x2{dv[0], dv[1]}, hi = f32x2{dv[2], dv[3]};
          const int ph = RP::phase(r) * ST + SP::phase(s);
          const float* wp = w0 + (r * S + s) * CO * 2;
#pragma unroll
          for (int c = 0; c < CO; ++c) {
            const f32x2 wa = *reinterpret_cast<const f32x2*>(wp + 2 * c);
            const f32x2 wb = *reinterpret_cast<const f32x2*>(wp + R * S * CO * 2 + 2 * c);
            acc[ph][c] = __builtin_elementwise_fma(lo, wa, acc[ph][c]);
            acc[ph][c] = __builtin_elementwise_fma(hi, wb, acc[ph][c]);
          }
        }
      }
    }
    __syncthreads();
  }

  const int qi = i0 + li, qj = j0 + lj;
  if (qi >= QH || qj >= QW) return;
#pragma unroll
  for (int a = 0; a < ST; ++a) {
    const int h = qi * ST + a;
    if (h >= H) continue;
#pragma unroll
    for (int b = 0; b < ST; ++b) {
      const int w = qj * ST + b;
      if (w >= W) continue;
      float* o = dx + (((size_t)n * H + h) * W + w) * C + cg * CO;
#pragma unroll
      for (int c = 0; c < CO; ++c)
        if (cg * CO + c < C) o[c] = acc[a * ST + b][c][0] + acc[a * ST + b][c][1];
    }
  }
}

// wt[cg][kp][r][s][c'][e] = W[k = 2kp + e][c = cg*CO + c'][r][s], zero outside K x C.
__global__ void w_subpixel_kernel(const float* __restrict__ w, int K, int C, int R, int S, int CO, int ncg, int KP,
                                  float* __restrict__ wt) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = ncg * KP * R * S * CO * 2;
  if (idx >= total) return;
  const int e = idx & 1;
  int t = idx >> 1;
  const int cc = t % CO;
  t /= CO;
  const int s = t % S;
  t /= S;
  const int r = t % R;
  t /= R;
  const int kp = t % KP;
  const int cg = t / KP;
  const int k = 2 * kp + e, c = cg * CO + cc;
  wt[idx] = (k < K && c < C) ? w[(((size_t)k * C + c) * R + r) * S + s] : 0.f;
}

constexpr int kMaxSubpixelC = 16;

struct Geometry {
  int co, ncg, kp;
  size_t wt_bytes;
};

Geometry geometry(int K, int C, int R, int S) {
  Geometry g;
  g.co = C < 4 ? C : 4;
  g.ncg = cdiv(C, g.co);
  g.kp = 2 * cdiv(K, 4);  // k pairs, padded so every 4-k step has two
  g.wt_bytes = (size_t)g.ncg * g.kp * R * S * g.co * 2 * sizeof(float);
  return g;
}

typedef void (*SubpixelKernel)(const float*, int, int, int, const float*, int, int, int, float*, int, int, int, int);

template <int R, int S, int ST, int PAD>
SubpixelKernel pick_co(int co) {
  switch (co) {
    case 1: return conv_dgrad_subpixel_kernel<R, S, ST, PAD, 1>;
    case 2: return conv_dgrad_subpixel_kernel<R, S, ST, PAD, 2>;
    case 3: return conv_dgrad_subpixel_kernel<R, S, ST, PAD, 3>;
    default: return conv_dgrad_subpixel_kernel<R, S, ST, PAD, 4>;
  }
}

// Instantiated geometries (R, S, stride, pad): the ResNet stem and the common strided convs.
SubpixelKernel pick(int R, int S, int st, int pad, int co) {
#define DK_GEOM(r, s, t, p) \
  if (R == r && S == s && st == t && pad == p) return pick_co<r, s, t, p>(co);
  DK_GEOM(5, 5, 2, 2)
  DK_GEOM(5, 5, 2, 1)
  DK_GEOM(3, 3, 2, 1)
  DK_GEOM(4, 4, 2, 1)
  DK_GEOM(7, 7, 2, 3)
  DK_GEOM(3, 3, 2, 0)
  DK_GEOM(2, 2, 2, 0)
#undef DK_GEOM
  return nullptr;
}

}  // namespace
}  // namespace dk

using namespace dk;

DK_API size_t dk_conv2d_dgrad_subpixel_workspace_bytes(int K, int C, int R, int S, int stride, int pad) {
  if (stride < 2 || C < 1 || C > kMaxSubpixelC || K < 1 || !pick(R, S, stride, pad, 4)) return 0;
  return geometry(K, C, R, S).wt_bytes;
}

DK_API int dk_conv2d_dgrad_subpixel_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kcrs, int C,
                                        int R, int S, int stride, int pad, float* dx, int H, int W, void* ws,
                                        size_t ws_bytes, void* stream) {
  const size_t need = dk_conv2d_dgrad_subpixel_workspace_bytes(K, C, R, S, stride, pad);
  if (need == 0) return DK_ERR_ARGS;
  if (ws_bytes < need) return DK_ERR_WORKSPACE;
  const Geometry g = geometry(K, C, R, S);
  if (N < 1 || H < 1 || W < 1 || (long long)N * g.ncg > 65535) return DK_ERR_ARGS;
  const hipStream_t st = as_stream(stream);
  float* wt = static_cast<float*>(ws);
  const int total = (int)(g.wt_bytes / sizeof(float));
  hipLaunchKernelGGL(w_subpixel_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, w_kcrs, K, C, R, S, g.co, g.ncg,
                     g.kp, wt);
  const int QH = cdiv(H, stride), QW = cdiv(W, stride);
  const dim3 grid(cdiv(QW, kTJ), cdiv(QH, kTI), N * g.ncg);
  hipLaunchKernelGGL(pick(R, S, stride, pad, g.co), grid, dim3(256), 0, st, dy, OH, OW, K, wt, g.kp, C, g.ncg, dx,
                     H, W, QH, QW);
  return launch_status();
}
