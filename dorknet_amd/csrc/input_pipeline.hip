// Device-side input pipeline (SURVEY.md section 8 f, row 4): the per-image preprocessing of
// data_loading/image_preprocessor.py:16-39 and the mixup of data_loading/image_data_loader.py:
// 101-111, for a whole batch on the GPU.  Byte / elementwise work, HBM-bound: one thread per
// output element, coalesced along the output's innermost dimension.
//
//   resize   cv2.resize(im, (OW, OH)) with INTER_LINEAR (the reference's default) for uint8:
//            OpenCV's 11-bit fixed-point algorithm (see resize_linear_u8_kernel), integer work,
//            bit-exact to oracle/pipeline.py's restatement.  cv2 is not in this image, so
//            agreement with cv2 itself is unpinned.
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

// cv2.resize INTER_LINEAR for CV_8U, OpenCV 4.3 (opencv-python 4.3.0.36, the reference's pin),
// imgproc/src/resize.cpp, restated from its published algorithm:
//   scale = 1 / (O / L) (cv::resize's inv_scale, then 1/inv_scale);
//   x: fx = (float)((ox + 0.5) * scale - 0.5), sx = floor(fx), fx -= sx; sx < 0 -> (sx, fx) = (0, 0);
//      sx >= L - 1 -> (sx, fx) = (L - 1, 0); weights (short) cvRound((1 - fx) * 2048), cvRound(fx * 2048)
//      (INTER_RESIZE_COEF_BITS = 11); outputs at or past the first sx + 1 >= L use src[sx] * 2048;
//   y: the same coordinate, rows sy and sy + 1 clipped to [0, H - 1], no weight clamping;
//   horizontal pass in int32: S = src[sx] * a0 + src[sx + C] * a1;
//   vertical pass FixedPtCast<int, uchar, 22>: (S0 * b0 + S1 * b1 + 2^21) >> 22, saturated to uint8;
//   an exact 2x downscale on both axes switches to INTER_AREA: (a + b + c + d + 2) >> 2 per 2x2 block;
//   the same size copies.
// Integer work, exact; the kernel and oracle/pipeline.py agree bit for bit.  OpenCV's x86 SIMD
// vertical pass (VResizeLinearVec_32s8u: >> 4, mulhi, (+2) >> 2) can round the bulk of a row
// differently in the last bit; cv2 is not installed here, so agreement with cv2 is unpinned.
struct CvAxis {
  int s0, s1;   // source indices of the two taps
  int a0, a1;   // weights (2048 = 1.0); (2048, 0) at and past the edge
};
__device__ __forceinline__ int cv_round(float v) { return (int)rintf(v); }

__device__ __forceinline__ CvAxis cv_axis_x(int o, double scale, int L) {
  float f = (float)((o + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  bool edge = false;
  if (s < 0) {
    s = 0;
    f = 0.f;
  }
  if (s + 1 >= L) {  // at or past xmax: src[sx] * ONE
    edge = true;
    if (s >= L - 1) {
      s = L - 1;
      f = 0.f;
    }
  }
  CvAxis a;
  a.s0 = s;
  a.s1 = min(s + 1, L - 1);
  if (edge) {
    a.a0 = 2048;
    a.a1 = 0;
  } else {
    a.a0 = cv_round((1.f - f) * 2048.f);
    a.a1 = cv_round(f * 2048.f);
  }
  return a;
}
__device__ __forceinline__ CvAxis cv_axis_y(int o, double scale, int L) {
  float f = (float)((o + 0.5) * scale - 0.5);
  const int s = (int)floorf(f);
  f -= (float)s;
  CvAxis a;
  a.s0 = min(max(s, 0), L - 1);
  a.s1 = min(max(s + 1, 0), L - 1);
  a.a0 = cv_round((1.f - f) * 2048.f);
  a.a1 = cv_round(f * 2048.f);
  return a;
}

// mode 0: linear, 1: exact 2x area, 2: copy
__global__ void resize_linear_u8_kernel(const uint8_t* __restrict__ src, int N, int H, int W, int C, int OH, int OW,
                                        double scy, double scx, int mode, uint8_t* __restrict__ dst) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // over N * OH * OW
  if (i >= (long long)N * OH * OW) return;
  const int ox = (int)(i % OW);
  const long long t = i / OW;
  const int oy = (int)(t % OH);
  const int n = (int)(t / OH);
  const uint8_t* im = src + (size_t)n * H * W * C;
  uint8_t* out = dst + (size_t)i * C;
  if (mode == 2) {
    for (int c = 0; c < C; ++c) out[c] = im[((size_t)oy * W + ox) * C + c];
    return;
  }
  if (mode == 1) {
    const size_t p = ((size_t)(2 * oy) * W + 2 * ox) * C, q = p + (size_t)W * C;
    for (int c = 0; c < C; ++c) out[c] = (uint8_t)((im[p + c] + im[p + C + c] + im[q + c] + im[q + C + c] + 2) >> 2);
    return;
  }
  const CvAxis ax = cv_axis_x(ox, scx, W), ay = cv_axis_y(oy, scy, H);
  const uint8_t* r0 = im + (size_t)ay.s0 * W * C;
  const uint8_t* r1 = im + (size_t)ay.s1 * W * C;
  for (int c = 0; c < C; ++c) {
    const int S0 = r0[ax.s0 * C + c] * ax.a0 + r0[ax.s1 * C + c] * ax.a1;
    const int S1 = r1[ax.s0 * C + c] * ax.a0 + r1[ax.s1 * C + c] * ax.a1;
    const int v = (S0 * ay.a0 + S1 * ay.a1 + (1 << 21)) >> 22;
    out[c] = (uint8_t)min(max(v, 0), 255);
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
  // cv::resize: inv_scale = dsize / ssize, scale = 1 / inv_scale
  const double scy = 1.0 / ((double)OH / (double)H), scx = 1.0 / ((double)OW / (double)W);
  const int iy = (int)rint(scy), ix = (int)rint(scx);
  const double eps = 2.220446049250313e-16;  // DBL_EPSILON
  const bool area2 = fabs(scx - ix) < eps && fabs(scy - iy) < eps && ix == 2 && iy == 2;
  const int mode = (OH == H && OW == W) ? 2 : area2 ? 1 : 0;
  hipLaunchKernelGGL(resize_linear_u8_kernel, dim3(blocks256((long long)N * OH * OW)), dim3(256), 0,
                     as_stream(stream), src, N, H, W, C, OH, OW, scy, scx, mode, dst);
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
