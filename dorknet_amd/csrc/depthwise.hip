// Depthwise (per-channel) convolution on NHWC fp32 for gfx950 -- direct, no MFMA.
//
// Replaces layers/depthwise_convolution.py:85-102 (+ CUDA forward_conv :105-121) and
// :198-221 (+ CUDA backward_conv :122-140).  Differences in *how* (same maths):
//   * channels are innermost, so a lane owns 4 adjacent channels (one float4) and a
//     wave covers 64*4 contiguous floats of a pixel row: fully coalesced;
//   * padding is handled by bounds checks instead of a padded copy (:57-64);
//   * forward accumulates in registers (the reference does 9 global read-modify-writes);
//   * wgrad reduces per-block partials in a fixed order (the reference issues N*OH*OW
//     atomicAdds on each of the C*R*S weight addresses): deterministic, no atomics;
//   * dgrad is a gather (each dx element sums its <= R*S contributions), no atomics.
#include "dk_common.h"

namespace dk {

// w[c][r][s] -> wt[r][s][c] so one float4 load fetches a tap for 4 channels.
__global__ void dw_weight_rsc_kernel(const float* __restrict__ w, int C, int RS, float* __restrict__ wt) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= C * RS) return;
  const int c = idx % C, t = idx / C;
  wt[idx] = w[(size_t)c * RS + t];
}

// y[n,oh,ow,c] = sum_{r,s} w[c][r][s] * x[n, oh*st + r - pad, ow*st + s - pad, c] (+ bias[c])
template <int R, int S>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                     const float* __restrict__ bias, float* __restrict__ y, int N,
                                                     int H, int W, int C, int OH, int OW, int st, int pad) {
  const int C4 = C >> 2;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)N * OH * OW * C4;
  if (idx >= total) return;
  const int cq = (int)(idx % C4);
  long long t = idx / C4;
  const int ow = (int)(t % OW);
  t /= OW;
  const int oh = (int)(t % OH);
  const int n = (int)(t / OH);
  const int c = cq * 4;
  f32x4 acc = bias ? ld4(bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  const int ih0 = oh * st - pad, iw0 = ow * st - pad;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int ih = ih0 + r;
    if ((unsigned)ih >= (unsigned)H) continue;
    const float* row = x + ((size_t)(n * H + ih) * W) * C + c;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int iw = iw0 + s;
      if ((unsigned)iw >= (unsigned)W) continue;
      const f32x4 xv = ld4(row + (size_t)iw * C);
      const f32x4 wv = ld4(wt + (r * S + s) * C + c);
      acc += xv * wv;
    }
  }
  st4(y + idx * 4, acc);
}

// dx[n,h,w,c] = sum_{r,s : h + pad - r = oh*st, w + pad - s = ow*st} w[c][r][s] * dy[n,oh,ow,c]
template <int R, int S>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const float* __restrict__ dy, const float* __restrict__ wt,
                                                       float* __restrict__ dx, int N, int H, int W, int C, int OH,
                                                       int OW, int st, int pad) {
  const int C4 = C >> 2;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)N * H * W * C4;
  if (idx >= total) return;
  const int cq = (int)(idx % C4);
  long long t = idx / C4;
  const int w = (int)(t % W);
  t /= W;
  const int h = (int)(t % H);
  const int n = (int)(t / H);
  const int c = cq * 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int hh = h + pad - r;
    if (hh < 0 || hh % st) continue;
    const int oh = hh / st;
    if (oh >= OH) continue;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int ww = w + pad - s;
      if (ww < 0 || ww % st) continue;
      const int ow = ww / st;
      if (ow >= OW) continue;
      const f32x4 g = ld4(dy + ((size_t)(n * OH + oh) * OW + ow) * C + c);
      const f32x4 wv = ld4(wt + (r * S + s) * C + c);
      acc += g * wv;
    }
  }
  st4(dx + idx * 4, acc);
}

// Partial wgrad: block b sums pixels [b*ppb, (b+1)*ppb) for every (c, r, s):
//   part[b][c][r*S+s] = sum dy[p][c] * x[shift(p, r, s)][c]
// Thread (cq, pl): channel group cq (4 channels), pixel lane pl.
template <int R, int S>
__global__ __launch_bounds__(256) void dw_wgrad_partial_kernel(const float* __restrict__ dy,
                                                               const float* __restrict__ x,
                                                               float* __restrict__ part, int N, int H, int W,
                                                               int C, int OH, int OW, int st, int pad, int ppb) {
  constexpr int RS = R * S;
  extern __shared__ float red[];  // [256][RS*4]
  const int C4 = C >> 2;
  const int cgt = C4 < 256 ? C4 : 256;
  const int PL = 256 / cgt;
  const int tid = threadIdx.x;
  const int cq = blockIdx.y * cgt + tid % cgt;
  const int pl = tid / cgt;
  const bool active = pl < PL && cq < C4;
  const int c = cq * 4;
  const int P = N * OH * OW;
  const int p0 = blockIdx.x * ppb;
  const int p1 = min(P, p0 + ppb);
  f32x4 acc[RS];
#pragma unroll
  for (int j = 0; j < RS; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (active) {
    for (int p = p0 + pl; p < p1; p += PL) {
      const int ow = p % OW;
      const int t = p / OW;
      const int oh = t % OH;
      const int n = t / OH;
      const f32x4 g = ld4(dy + (size_t)p * C + c);
      const int ih0 = oh * st - pad, iw0 = ow * st - pad;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int ih = ih0 + r;
        if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int iw = iw0 + s;
          if ((unsigned)iw >= (unsigned)W) continue;
          acc[r * S + s] += g * ld4(x + ((size_t)(n * H + ih) * W + iw) * C + c);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < RS; ++j) st4(red + (tid * RS + j) * 4, acc[j]);
  __syncthreads();
  // Fixed-order reduction over the PL pixel lanes of each (channel group, tap).
  const int items = cgt * RS * 4;
  for (int it = tid; it < items; it += 256) {
    const int e = it % 4;
    const int j = (it / 4) % RS;
    const int g = it / (4 * RS);
    if (blockIdx.y * cgt + g >= C4) continue;
    float s = 0.f;
    for (int q = 0; q < PL; ++q) s += red[((q * cgt + g) * RS + j) * 4 + e];
    const int cc = (blockIdx.y * cgt + g) * 4 + e;
    part[((size_t)blockIdx.x * C + cc) * RS + j] = s;
  }
}

__global__ void dw_wgrad_reduce_kernel(const float* __restrict__ part, int nblk, int C, int RS,
                                       const float* __restrict__ w, float l2, float* __restrict__ dw) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= C * RS) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += (double)part[(size_t)b * C * RS + idx];
  float v = (float)s;
  if (w) v = v + l2 * w[idx];
  dw[idx] = v;
}

static int dw_wgrad_blocks(int P) {
  int nblk = cdiv(P, 512);
  if (nblk > 1024) nblk = 1024;
  if (nblk < 1) nblk = 1;
  return nblk;
}

}  // namespace dk

using namespace dk;

#define DK_DW_DISPATCH(R_, S_, CALL) \
  if (R_ == 3 && S_ == 3) {          \
    CALL(3, 3);                      \
  } else if (R_ == 5 && S_ == 5) {   \
    CALL(5, 5);                      \
  } else if (R_ == 1 && S_ == 1) {   \
    CALL(1, 1);                      \
  } else {                           \
    return DK_ERR_ARGS;              \
  }

DK_API int dk_dw_weight_rsc_f32(const float* w_crs, int C, int R, int S, float* w_rsc, void* stream) {
  const int total = C * R * S;
  hipLaunchKernelGGL(dw_weight_rsc_kernel, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), w_crs, C, R * S,
                     w_rsc);
  return launch_status();
}

DK_API int dk_dwconv_fwd_f32(const float* x, int N, int H, int W, int C, const float* w_rsc, int R, int S, int stride,
                             int pad, const float* bias, float* y, int OH, int OW, void* stream) {
  if (C % 4) return DK_ERR_ARGS;
  const long long total = (long long)N * OH * OW * (C / 4);
  const dim3 grid((unsigned)cdivll(total, 256));
#define CALL(RR, SS)                                                                                                  \
  hipLaunchKernelGGL((dw_fwd_kernel<RR, SS>), grid, dim3(256), 0, as_stream(stream), x, w_rsc, bias, y, N, H, W, C, \
                     OH, OW, stride, pad)
  DK_DW_DISPATCH(R, S, CALL)
#undef CALL
  return launch_status();
}

DK_API int dk_dwconv_dgrad_f32(const float* dy, int N, int OH, int OW, int C, const float* w_rsc, int R, int S,
                               int stride, int pad, float* dx, int H, int W, void* stream) {
  if (C % 4) return DK_ERR_ARGS;
  const long long total = (long long)N * H * W * (C / 4);
  const dim3 grid((unsigned)cdivll(total, 256));
#define CALL(RR, SS)                                                                                                   \
  hipLaunchKernelGGL((dw_dgrad_kernel<RR, SS>), grid, dim3(256), 0, as_stream(stream), dy, w_rsc, dx, N, H, W, C, OH, \
                     OW, stride, pad)
  DK_DW_DISPATCH(R, S, CALL)
#undef CALL
  return launch_status();
}

DK_API size_t dk_dwconv_wgrad_workspace_bytes(int N, int OH, int OW, int C, int R, int S) {
  return (size_t)dw_wgrad_blocks(N * OH * OW) * C * R * S * sizeof(float);
}

// dw[c][r][s] = sum_{n,oh,ow} dy[n,oh,ow,c] * x[n, oh*st + r - pad, ow*st + s - pad, c] (+ l2 * w)
DK_API int dk_dwconv_wgrad_f32(const float* dy, const float* x, int N, int H, int W, int C, int R, int S, int stride,
                               int pad, int OH, int OW, const float* w_crs, float l2, float* dw_crs, void* ws,
                               size_t ws_bytes, void* stream) {
  if (C % 4) return DK_ERR_ARGS;
  const int P = N * OH * OW;
  const int nblk = dw_wgrad_blocks(P);
  if (ws_bytes < dk_dwconv_wgrad_workspace_bytes(N, OH, OW, C, R, S)) return DK_ERR_WORKSPACE;
  const int ppb = cdiv(P, nblk);
  const int C4 = C / 4;
  const int cgt = C4 < 256 ? C4 : 256;
  const dim3 grid(nblk, cdiv(C4, cgt));
  float* part = static_cast<float*>(ws);
  const size_t shm = (size_t)256 * R * S * 4 * sizeof(float);
#define CALL(RR, SS)                                                                                                 \
  if (shm > 65536)                                                                                                   \
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&dw_wgrad_partial_kernel<RR, SS>),                       \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);                                 \
  hipLaunchKernelGGL((dw_wgrad_partial_kernel<RR, SS>), grid, dim3(256), shm, as_stream(stream), dy, x, part, N, H, \
                     W, C, OH, OW, stride, pad, ppb)
  DK_DW_DISPATCH(R, S, CALL)
#undef CALL
  int rc = launch_status();
  if (rc) return rc;
  const int total = C * R * S;
  hipLaunchKernelGGL(dw_wgrad_reduce_kernel, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), part, nblk, C,
                     R * S, w_crs, l2, dw_crs);
  return launch_status();
}
