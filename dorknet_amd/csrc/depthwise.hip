// Depthwise (per-channel) convolution on NHWC fp32 for gfx950 -- direct, no MFMA.
//
// Replaces layers/depthwise_convolution.py:85-102 (+ CUDA forward_conv :105-121) and
// :198-221 (+ CUDA backward_conv :122-140).  Same maths, different data flow:
//   * channels are innermost, so a lane owns 4 adjacent channels (one float4) and a
//     wave covers 64*4 contiguous floats of a pixel row: fully coalesced;
//   * padding is handled by bounds checks instead of a padded copy (:57-64);
//   * a thread produces TW consecutive outputs along W, keeping an R x S window of
//     input float4s in registers and sliding it, so each output costs R*stride new
//     loads instead of R*S (the reference re-reads all R*S taps and does R*S global
//     read-modify-writes of the output);
//   * stride-1 dgrad is the forward kernel run on dy with the taps flipped;
//   * wgrad reduces per-block partials in a fixed order (reduce.hip) -- the reference
//     issues N*OH*OW atomicAdds on each of the C*R*S weight addresses.
#include "dk_common.h"

namespace dk {

constexpr int kTW = 8;  // outputs per thread along W

// w[c][r][s] -> wt[r][s][c] (flip != 0: wt[r][s][c] = w[c][R-1-r][S-1-s]) so one float4
// load fetches a tap for 4 channels.
__global__ void dw_weight_rsc_kernel(const float* __restrict__ w, int C, int R, int S, int flip,
                                     float* __restrict__ wt) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= C * R * S) return;
  const int c = idx % C, t = idx / C;
  int r = t / S, s = t - r * S;
  if (flip) {
    r = R - 1 - r;
    s = S - 1 - s;
  }
  wt[idx] = w[((size_t)c * R + r) * S + s];
}

// y[n,oh,ow,c] = sum_{r,s} w[r][s][c] * x[n, oh*ST + r - pad, ow*ST + s - pad, c] (+ bias[c])
// Thread = (n, oh, TW-wide chunk of ow, 4 channels).
template <int R, int S, int ST>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                     const float* __restrict__ bias, float* __restrict__ y, int N,
                                                     int H, int W, int C, int OH, int OW, int pad) {
  const int C4 = C >> 2;
  const int nwc = (OW + kTW - 1) / kTW;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)N * OH * nwc * C4;
  if (idx >= total) return;
  const int cq = (int)(idx % C4);
  long long t = idx / C4;
  const int wc = (int)(t % nwc);
  t /= nwc;
  const int oh = (int)(t % OH);
  const int n = (int)(t / OH);
  const int c = cq * 4;
  f32x4 wv[R][S];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int s = 0; s < S; ++s) wv[r][s] = ld4(wt + (r * S + s) * C + c);
  const f32x4 b0 = bias ? ld4(bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  const int ow0 = wc * kTW;
  const int ih0 = oh * ST - pad;
  const int iw0 = ow0 * ST - pad;
  bool rv[R];
  const float* rowp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int ih = ih0 + r;
    rv[r] = (unsigned)ih < (unsigned)H;
    rowp[r] = x + ((size_t)(n * H + (rv[r] ? ih : 0)) * W) * C + c;
  }
  auto load_col = [&](int r, int iw) -> f32x4 {
    return (rv[r] && (unsigned)iw < (unsigned)W) ? ld4(rowp[r] + (size_t)iw * C) : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  f32x4 win[R][S];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int s = 0; s < S; ++s) win[r][s] = load_col(r, iw0 + s);
  float* yrow = y + ((size_t)(n * OH + oh) * OW) * C + c;
#pragma unroll
  for (int j = 0; j < kTW; ++j) {
    if (j > 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          if (s + ST < S)
            win[r][s] = win[r][s + ST];
          else
            win[r][s] = load_col(r, iw0 + j * ST + s);
        }
      }
    }
    const int ow = ow0 + j;
    if (ow < OW) {
      f32x4 acc = b0;
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int s = 0; s < S; ++s) acc += win[r][s] * wv[r][s];
      st4(yrow + (size_t)ow * C, acc);
    }
  }
}

// General-stride dgrad gather (used for stride > 1):
// dx[n,h,w,c] = sum_{r,s : h + pad - r = oh*st, w + pad - s = ow*st} w[r][s][c] * dy[n,oh,ow,c]
template <int R, int S>
__global__ __launch_bounds__(256) void dw_dgrad_gather_kernel(const float* __restrict__ dy,
                                                              const float* __restrict__ wt, float* __restrict__ dx,
                                                              int N, int H, int W, int C, int OH, int OW, int st,
                                                              int pad) {
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
      acc += ld4(dy + ((size_t)(n * OH + oh) * OW + ow) * C + c) * ld4(wt + (r * S + s) * C + c);
    }
  }
  st4(dx + idx * 4, acc);
}

// wgrad partials: part[blk][c][r*S+s] = sum over the block's (n, oh, ow-chunk) items of
// dy[n,oh,ow,c] * x[n, oh*ST + r - pad, ow*ST + s - pad, c].  Thread (cq, pl): channel group
// cq, walks items pl, pl + PL, ... with the same sliding window as the forward kernel.
template <int R, int S, int ST>
__global__ __launch_bounds__(256) void dw_wgrad_partial_kernel(const float* __restrict__ dy,
                                                               const float* __restrict__ x,
                                                               float* __restrict__ part, int N, int H, int W,
                                                               int C, int OH, int OW, int pad, int ipb) {
  constexpr int RS = R * S;
  extern __shared__ float red[];  // [256][RS][4]
  const int C4 = C >> 2;
  const int cgt = C4 < 256 ? C4 : 256;
  const int PL = 256 / cgt;
  const int tid = threadIdx.x;
  const int cq = blockIdx.y * cgt + tid % cgt;
  const int pl = tid / cgt;
  const bool active = pl < PL && cq < C4;
  const int c = cq * 4;
  const int nwc = (OW + kTW - 1) / kTW;
  const int items = N * OH * nwc;
  const int i0 = blockIdx.x * ipb, i1 = min(items, i0 + ipb);
  f32x4 acc[R][S];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int s = 0; s < S; ++s) acc[r][s] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (active) {
    for (int it = i0 + pl; it < i1; it += PL) {
      const int wc = it % nwc;
      const int t = it / nwc;
      const int oh = t % OH;
      const int n = t / OH;
      const int ow0 = wc * kTW;
      const int ih0 = oh * ST - pad;
      const int iw0 = ow0 * ST - pad;
      bool rv[R];
      const float* rowp[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int ih = ih0 + r;
        rv[r] = (unsigned)ih < (unsigned)H;
        rowp[r] = x + ((size_t)(n * H + (rv[r] ? ih : 0)) * W) * C + c;
      }
      auto load_col = [&](int r, int iw) -> f32x4 {
        return (rv[r] && (unsigned)iw < (unsigned)W) ? ld4(rowp[r] + (size_t)iw * C)
                                                     : f32x4{0.f, 0.f, 0.f, 0.f};
      };
      f32x4 win[R][S];
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int s = 0; s < S; ++s) win[r][s] = load_col(r, iw0 + s);
      const float* grow = dy + ((size_t)(n * OH + oh) * OW) * C + c;
#pragma unroll
      for (int j = 0; j < kTW; ++j) {
        if (j > 0) {
#pragma unroll
          for (int r = 0; r < R; ++r)
#pragma unroll
            for (int s = 0; s < S; ++s) {
              if (s + ST < S)
                win[r][s] = win[r][s + ST];
              else
                win[r][s] = load_col(r, iw0 + j * ST + s);
            }
        }
        const int ow = ow0 + j;
        if (ow < OW) {
          const f32x4 g = ld4(grow + (size_t)ow * C);
#pragma unroll
          for (int r = 0; r < R; ++r)
#pragma unroll
            for (int s = 0; s < S; ++s) acc[r][s] += g * win[r][s];
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int s = 0; s < S; ++s) st4(red + (tid * RS + r * S + s) * 4, acc[r][s]);
  __syncthreads();
  // Fixed-order reduction over the PL pixel lanes of each (channel group, tap).
  const int nitems = cgt * RS * 4;
  for (int k = tid; k < nitems; k += 256) {
    const int e = k % 4;
    const int tap = (k / 4) % RS;
    const int g = k / (4 * RS);
    if (blockIdx.y * cgt + g >= C4) continue;
    float sum = 0.f;
    for (int q = 0; q < PL; ++q) sum += red[((q * cgt + g) * RS + tap) * 4 + e];
    const int cc = (blockIdx.y * cgt + g) * 4 + e;
    part[((size_t)blockIdx.x * C + cc) * RS + tap] = sum;
  }
}

static int dw_wgrad_blocks(int N, int OH, int OW, int C) {
  const int items = N * OH * ((OW + kTW - 1) / kTW);
  const int C4 = C / 4;
  const int cgt = C4 < 256 ? C4 : 256;
  const int PL = 256 / cgt;
  int nblk = cdiv(items, PL * 4);  // ~4 items (32 outputs) per thread
  if (nblk > 1024) nblk = 1024;
  if (nblk < 1) nblk = 1;
  return nblk;
}

}  // namespace dk

using namespace dk;

DK_API int dk_dw_weight_rsc_f32(const float* w_crs, int C, int R, int S, float* w_rsc, void* stream) {
  const int total = C * R * S;
  hipLaunchKernelGGL(dw_weight_rsc_kernel, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), w_crs, C, R, S, 0,
                     w_rsc);
  return launch_status();
}

template <int R, int S, int ST>
static void launch_dw_fwd(const float* x, const float* wt, const float* bias, float* y, int N, int H, int W, int C,
                          int OH, int OW, int pad, hipStream_t st) {
  const long long total = (long long)N * OH * ((OW + kTW - 1) / kTW) * (C / 4);
  hipLaunchKernelGGL((dw_fwd_kernel<R, S, ST>), dim3((unsigned)cdivll(total, 256)), dim3(256), 0, st, x, wt, bias, y,
                     N, H, W, C, OH, OW, pad);
}

static int dw_fwd_dispatch(const float* x, const float* wt, const float* bias, float* y, int N, int H, int W, int C,
                           int R, int S, int stride, int OH, int OW, int pad, hipStream_t st) {
#define DW_CASE(RR, SS, STR)                                                   \
  if (R == RR && S == SS && stride == STR) {                                   \
    launch_dw_fwd<RR, SS, STR>(x, wt, bias, y, N, H, W, C, OH, OW, pad, st);   \
    return launch_status();                                                    \
  }
  DW_CASE(3, 3, 1)
  DW_CASE(3, 3, 2)
  DW_CASE(5, 5, 1)
  DW_CASE(5, 5, 2)
  DW_CASE(1, 1, 1)
  DW_CASE(1, 1, 2)
#undef DW_CASE
  return DK_ERR_ARGS;
}

DK_API int dk_dwconv_fwd_f32(const float* x, int N, int H, int W, int C, const float* w_rsc, int R, int S, int stride,
                             int pad, const float* bias, float* y, int OH, int OW, void* stream) {
  if (C % 4) return DK_ERR_ARGS;
  return dw_fwd_dispatch(x, w_rsc, bias, y, N, H, W, C, R, S, stride, OH, OW, pad, as_stream(stream));
}

// w_rsc is the (unflipped) [R][S][C] copy; stride-1 dgrad flips it internally into ws.
DK_API size_t dk_dwconv_dgrad_workspace_bytes(int C, int R, int S) { return (size_t)C * R * S * sizeof(float); }

DK_API int dk_dwconv_dgrad_f32(const float* dy, int N, int OH, int OW, int C, const float* w_crs, int R, int S,
                               int stride, int pad, float* dx, int H, int W, void* ws, size_t ws_bytes,
                               void* stream) {
  if (C % 4) return DK_ERR_ARGS;
  if (ws_bytes < dk_dwconv_dgrad_workspace_bytes(C, R, S)) return DK_ERR_WORKSPACE;
  float* wt = static_cast<float*>(ws);
  const hipStream_t st = as_stream(stream);
  if (stride == 1 && pad <= R - 1 && pad <= S - 1 && R == S) {
    // dx = correlation of dy with the flipped filter, padding R-1-pad, stride 1
    hipLaunchKernelGGL(dw_weight_rsc_kernel, dim3(cdiv(C * R * S, 256)), dim3(256), 0, st, w_crs, C, R, S, 1, wt);
    int rc = launch_status();
    if (rc) return rc;
    return dw_fwd_dispatch(dy, wt, nullptr, dx, N, OH, OW, C, R, S, 1, H, W, R - 1 - pad, st);
  }
  hipLaunchKernelGGL(dw_weight_rsc_kernel, dim3(cdiv(C * R * S, 256)), dim3(256), 0, st, w_crs, C, R, S, 0, wt);
  int rc = launch_status();
  if (rc) return rc;
  const long long total = (long long)N * H * W * (C / 4);
  const dim3 grid((unsigned)cdivll(total, 256));
  if (R == 3 && S == 3)
    hipLaunchKernelGGL((dw_dgrad_gather_kernel<3, 3>), grid, dim3(256), 0, st, dy, wt, dx, N, H, W, C, OH, OW, stride,
                       pad);
  else if (R == 5 && S == 5)
    hipLaunchKernelGGL((dw_dgrad_gather_kernel<5, 5>), grid, dim3(256), 0, st, dy, wt, dx, N, H, W, C, OH, OW, stride,
                       pad);
  else if (R == 1 && S == 1)
    hipLaunchKernelGGL((dw_dgrad_gather_kernel<1, 1>), grid, dim3(256), 0, st, dy, wt, dx, N, H, W, C, OH, OW, stride,
                       pad);
  else
    return DK_ERR_ARGS;
  return launch_status();
}

DK_API size_t dk_dwconv_wgrad_workspace_bytes(int N, int OH, int OW, int C, int R, int S) {
  return (size_t)dw_wgrad_blocks(N, OH, OW, C) * C * R * S * sizeof(float);
}

// dw[c][r][s] = sum_{n,oh,ow} dy[n,oh,ow,c] * x[n, oh*st + r - pad, ow*st + s - pad, c] (+ l2 * w)
DK_API int dk_dwconv_wgrad_f32(const float* dy, const float* x, int N, int H, int W, int C, int R, int S, int stride,
                               int pad, int OH, int OW, const float* w_crs, float l2, float* dw_crs, void* ws,
                               size_t ws_bytes, void* stream) {
  if (C % 4) return DK_ERR_ARGS;
  if (ws_bytes < dk_dwconv_wgrad_workspace_bytes(N, OH, OW, C, R, S)) return DK_ERR_WORKSPACE;
  const int nblk = dw_wgrad_blocks(N, OH, OW, C);
  const int items = N * OH * ((OW + kTW - 1) / kTW);
  const int ipb = cdiv(items, nblk);
  const int C4 = C / 4;
  const int cgt = C4 < 256 ? C4 : 256;
  const dim3 grid(nblk, cdiv(C4, cgt));
  float* part = static_cast<float*>(ws);
  const size_t shm = (size_t)256 * R * S * 4 * sizeof(float);
  const hipStream_t st = as_stream(stream);
#define DW_WG(RR, SS, STR)                                                                                          \
  if (R == RR && S == SS && stride == STR) {                                                                        \
    if (shm > 65536)                                                                                                \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&dw_wgrad_partial_kernel<RR, SS, STR>),               \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);                              \
    hipLaunchKernelGGL((dw_wgrad_partial_kernel<RR, SS, STR>), grid, dim3(256), shm, st, dy, x, part, N, H, W, C, OH, \
                       OW, pad, ipb);                                                                               \
  } else
  DW_WG(3, 3, 1)
  DW_WG(3, 3, 2)
  DW_WG(5, 5, 1)
  DW_WG(5, 5, 2)
  DW_WG(1, 1, 1)
  DW_WG(1, 1, 2) { return DK_ERR_ARGS; }
#undef DW_WG
  int rc = launch_status();
  if (rc) return rc;
  return splitk_reduce(part, nblk, 1, C * R * S, dw_crs, w_crs, l2, 0, C, C, 1, 1, st);
}
