// Device-side input pipeline (SURVEY.md section 8 f, row 4): the per-image preprocessing of
// data_loading/image_preprocessor.py:16-39 and the mixup of data_loading/image_data_loader.py:
// 101-111, for a whole batch on the GPU.  Byte / elementwise work, HBM-bound: one thread per
// output element, coalesced along the output's innermost dimension.
//
//   resize   cv2.resize(im, (OW, OH)) with INTER_LINEAR (the reference's default): half-pixel
//            centres, edge replication, result rounded to nearest (ties to even) and saturated
//            to uint8.  Computed in fp32 with explicitly rounded operations (no contraction),
//            so oracle/pipeline.py's numpy restatement reproduces it bit for bit.  cv2 itself
//            interpolates uint8 in 11-bit fixed point; it is not in this image, so agreement
//            with cv2 is unpinned.
//   crop + cast + layout   im[r:r+OH, c:c+OW, :].astype(float32).transpose(2, 0, 1) - 128:
//            uint8 NHWC batch in, fp32 NCHW batch out (the layout the reference's X_batch has),
//            per-image crop offsets.  Exact.
//   mixup    X_mixed = p * X_m + (1 - p) * X and its mirror, for images and one-hot labels,
//            with p and 1 - p rounded to fp32 first as numpy does for a Python float times a
//            float32 array.  Exact.
#include "dk_common.h"

// Built with -ffp-contract=off (__graft_entry__.EXTRA_FLAGS): every fp32 / fp64 operation is
// rounded on its own, as in the numpy restatement.

namespace dk {

__global__ void resize_bilinear_u8_kernel(const uint8_t* __restrict__ src, int N, int H, int W, int C, int OH, int OW,
                                          double sy, double sx, uint8_t* __restrict__ dst) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // over N * OH * OW
  if (i >= (long long)N * OH * OW) return;
  const int ox = (int)(i % OW);
  const long long t = i / OW;
  const int oy = (int)(t % OH);
  const int n = (int)(t / OH);
  // source coordinate = (float)((o + 0.5) * scale - 0.5) in double as cv2's resize computes it,
  // clamped as cv2 does (below 0 -> 0; at or past the last pixel -> the last pixel, weight 0)
  auto coord = [](int o, double s, int L, int& i0, float& f) {
    const float v = (float)__dsub_rn(__dmul_rn(__dadd_rn((double)o, 0.5), s), 0.5);  // no fma contraction
    int k = (int)floorf(v);
    f = __fsub_rn(v, (float)k);
    if (k < 0) {
      k = 0;
      f = 0.f;
    }
    if (k >= L - 1) {
      k = L - 1;
      f = 0.f;
    }
    i0 = k;
  };
  int y0, x0;
  float fy, fx;
  coord(oy, sy, H, y0, fy);
  coord(ox, sx, W, x0, fx);
  const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
  const uint8_t* im = src + (size_t)n * H * W * C;
  const float gy = __fsub_rn(1.f, fy), gx = __fsub_rn(1.f, fx);
  uint8_t* out = dst + (size_t)i * C;
  for (int c = 0; c < C; ++c) {
    const float p00 = im[((size_t)y0 * W + x0) * C + c], p01 = im[((size_t)y0 * W + x1) * C + c];
    const float p10 = im[((size_t)y1 * W + x0) * C + c], p11 = im[((size_t)y1 * W + x1) * C + c];
    const float top = __fadd_rn(__fmul_rn(gx, p00), __fmul_rn(fx, p01));
    const float bot = __fadd_rn(__fmul_rn(gx, p10), __fmul_rn(fx, p11));
    const float v = __fadd_rn(__fmul_rn(gy, top), __fmul_rn(fy, bot));
    out[c] = (uint8_t)fminf(fmaxf(rintf(v), 0.f), 255.f);
  }
}

__global__ void u8_nhwc_to_nchw_kernel(const uint8_t* __restrict__ src, int N, int H, int W, int C,
                                       const int* __restrict__ crop, int OH, int OW, float shift,
                                       float* __restrict__ dst) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // over N * C * OH * OW (NCHW)
  if (i >= (long long)N * C * OH * OW) return;
  const int ox = (int)(i % OW);
  long long t = i / OW;
  const int oy = (int)(t % OH);
  t /= OH;
  const int c = (int)(t % C);
  const int n = (int)(t / C);
  // offsets clamped into the image (a bad offset cannot read out of bounds)
  const int r0 = crop ? min(max(crop[2 * n], 0), H - OH) : 0, c0 = crop ? min(max(crop[2 * n + 1], 0), W - OW) : 0;
  const uint8_t v = src[(((size_t)n * H + r0 + oy) * W + c0 + ox) * C + c];
  dst[i] = __fsub_rn((float)v, shift);
}

__global__ void mixup_kernel(const float* __restrict__ a, const float* __restrict__ b, long long n, float p, float q,
                             float* __restrict__ ab, float* __restrict__ ba) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = a[i], y = b[i];
  ab[i] = __fadd_rn(__fmul_rn(p, y), __fmul_rn(q, x));  // p * X_m + (1 - p) * X
  ba[i] = __fadd_rn(__fmul_rn(p, x), __fmul_rn(q, y));  // p * X + (1 - p) * X_m
}

}  // namespace dk

using namespace dk;

static inline unsigned blocks256(long long n) { return (unsigned)((n + 255) / 256); }

DK_API int dk_resize_bilinear_u8(const uint8_t* src, int N, int H, int W, int C, int OH, int OW, uint8_t* dst,
                                 void* stream) {
  if (!src || !dst || N < 1 || H < 1 || W < 1 || C < 1 || OH < 1 || OW < 1) return DK_ERR_ARGS;
  const double sy = (double)H / (double)OH, sx = (double)W / (double)OW;
  hipLaunchKernelGGL(resize_bilinear_u8_kernel, dim3(blocks256((long long)N * OH * OW)), dim3(256), 0,
                     as_stream(stream), src, N, H, W, C, OH, OW, sy, sx, dst);
  return launch_status();
}

DK_API int dk_u8_nhwc_to_nchw_f32(const uint8_t* src, int N, int H, int W, int C, const int* crop_rc, int OH, int OW,
                                  float shift, float* dst, void* stream) {
  if (!src || !dst || N < 1 || C < 1 || OH < 1 || OW < 1 || OH > H || OW > W) return DK_ERR_ARGS;
  hipLaunchKernelGGL(u8_nhwc_to_nchw_kernel, dim3(blocks256((long long)N * C * OH * OW)), dim3(256), 0,
                     as_stream(stream), src, N, H, W, C, crop_rc, OH, OW, shift, dst);
  return launch_status();
}

DK_API int dk_mixup_f32(const float* a, const float* b, long long n, float p, float one_minus_p, float* ab, float* ba,
                        void* stream) {
  if (!a || !b || !ab || !ba || n < 0) return DK_ERR_ARGS;
  if (n == 0) return 0;
  hipLaunchKernelGGL(mixup_kernel, dim3(blocks256(n)), dim3(256), 0, as_stream(stream), a, b, n, p, one_minus_p, ab,
                     ba);
  return launch_status();
}
