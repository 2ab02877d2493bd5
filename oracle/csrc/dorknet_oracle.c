/*
 * C/OpenMP restatement of the reference's Cython CPU kernels.  TEST INFRASTRUCTURE ONLY:
 * used as the CPU baseline (bench.py cpu_baseline, kind "port") and by the oracle's
 * "reference CPU path" network (oracle/cpu_path.py).  Compiled with the reference's
 * flags -O3 -ffast-math -fopenmp (setup.py:9-10).  Loop nests follow the .pyx files;
 * the outer prange over the batch (or channel) is the parallel loop; the reference's
 * inner pranges are nested parallel regions that libgomp serialises by default, so they
 * are plain loops here.
 *
 * PARITY UNPINNED (see oracle/ref.py): the reference's own build could not be run.
 */
#include <stddef.h>
#include <string.h>
#include <omp.h>

/* im2col_cy (layers/im2col.pyx:14-36): X (N, C, Hp, Wp) already padded ->
 * patches[N*OH*OW][C*R*S], row (i*OH + j)*OW + k, column (l*R + m)*S + n. */
void oracle_im2col(const float* X, int N, int C, int Hp, int Wp, int R, int S, int stride, int OH, int OW,
                   float* out) {
  const long long ncol = (long long)C * R * S;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < OH; ++j)
      for (int k = 0; k < OW; ++k) {
        float* row = out + ((long long)(i * OH + j) * OW + k) * ncol;
        for (int l = 0; l < C; ++l)
          for (int m = 0; m < R; ++m)
            for (int n = 0; n < S; ++n)
              row[(l * R + m) * S + n] = X[(((long long)i * C + l) * Hp + j * stride + m) * Wp + k * stride + n];
      }
}

/* row2im_cy (layers/im2col.pyx:207-234): scatter-add rows into padded (N, C, Hpd, Wpd). */
void oracle_row2im(const float* rows, int N, int C, int Hpd, int Wpd, int R, int S, int stride, int OH, int OW,
                   float* padded) {
  const long long ncol = (long long)C * R * S;
  memset(padded, 0, sizeof(float) * (size_t)N * C * Hpd * Wpd);
#pragma omp parallel for schedule(static)
  for (int b = 0; b < N; ++b)
    for (int j = 0; j < OH; ++j)
      for (int k = 0; k < OW; ++k) {
        const float* row = rows + ((long long)(b * OH + j) * OW + k) * ncol;
        for (int c = 0; c < C; ++c)
          for (int m = 0; m < R; ++m)
            for (int n = 0; n < S; ++n)
              padded[(((long long)b * C + c) * Hpd + stride * j + m) * Wpd + stride * k + n] += row[(c * R + m) * S + n];
      }
}

/* depthwise_conv_cy (layers/im2col.pyx:107-139): out (N, C, OH, OW) += X * f. */
void oracle_depthwise_conv(const float* X, const float* f, int N, int C, int Hp, int Wp, int R, int S, int stride,
                           int OH, int OW, float* out) {
  memset(out, 0, sizeof(float) * (size_t)N * C * OH * OW);
#pragma omp parallel for schedule(static)
  for (int b = 0; b < N; ++b)
    for (int c = 0; c < C; ++c) {
      const float* x = X + ((long long)b * C + c) * Hp * Wp;
      float* o = out + ((long long)b * C + c) * OH * OW;
      const float* w = f + (long long)c * R * S;
      for (int i = 0; i < OH; ++i)
        for (int j = 0; j < OW; ++j)
          for (int m = 0; m < R; ++m)
            for (int n = 0; n < S; ++n) o[i * OW + j] += x[(stride * i + m) * Wp + stride * j + n] * w[m * S + n];
    }
}

/* depthwise_backward_direct_cy (layers/im2col.pyx:141-178): padded_dx (N, C, Hpd, Wpd) and
 * per-batch dw (N, C, R, S) (summed over N by the caller, depthwise_convolution.py:193). */
void oracle_depthwise_backward(const float* dy, const float* X, const float* w, int N, int C, int Hp, int Wp, int R,
                               int S, int stride, int OH, int OW, int Hpd, int Wpd, float* padded_dx, float* dw) {
  memset(padded_dx, 0, sizeof(float) * (size_t)N * C * Hpd * Wpd);
  memset(dw, 0, sizeof(float) * (size_t)N * C * R * S);
#pragma omp parallel for schedule(static)
  for (int b = 0; b < N; ++b)
    for (int c = 0; c < C; ++c) {
      const float* g = dy + ((long long)b * C + c) * OH * OW;
      const float* x = X + ((long long)b * C + c) * Hp * Wp;
      float* d = padded_dx + ((long long)b * C + c) * Hpd * Wpd;
      float* dwb = dw + ((long long)b * C + c) * R * S;
      const float* wc = w + (long long)c * R * S;
      for (int i = 0; i < OH; ++i)
        for (int j = 0; j < OW; ++j)
          for (int m = 0; m < R; ++m)
            for (int n = 0; n < S; ++n) {
              dwb[m * S + n] += g[i * OW + j] * x[(stride * i + m) * Wp + stride * j + n];
              d[(stride * i + m) * Wpd + stride * j + n] += g[i * OW + j] * wc[m * S + n];
            }
    }
}

/* channelwise_mean_and_var_4d (layers/batch_norm_stats_cy.pyx:15-47): two passes, fp32
 * accumulators, population variance. */
void oracle_bn_stats(const float* A, int N, int C, int H, int W, float* mean, float* var) {
  const float count = (float)(N * H * W);
#pragma omp parallel for schedule(static)
  for (int c = 0; c < C; ++c) {
    float s = 0.f;
    for (int b = 0; b < N; ++b) {
      const float* p = A + ((long long)b * C + c) * H * W;
      for (int i = 0; i < H * W; ++i) s += p[i];
    }
    const float m = s / count;
    float v = 0.f;
    for (int b = 0; b < N; ++b) {
      const float* p = A + ((long long)b * C + c) * H * W;
      for (int i = 0; i < H * W; ++i) v += (p[i] - m) * (p[i] - m);
    }
    mean[c] = m;
    var[c] = v / count;
  }
}

/* relu_4d_forward_train / relu_2d_forward_train (layers/relu_cy.pyx:9-38, :65-88). */
void oracle_relu_forward_train(const float* X, long long n, float* out, float* mask) {
#pragma omp parallel for schedule(static)
  for (long long i = 0; i < n; ++i) {
    const int pos = X[i] > 0.0f;
    out[i] = pos ? X[i] : 0.0f;
    mask[i] = pos ? 1.0f : 0.0f;
  }
}

int oracle_num_threads(void) {
  int n = 1;
#pragma omp parallel
  {
#pragma omp single
    n = omp_get_num_threads();
  }
  return n;
}

/* The CPU-baseline thread configuration (bench.py cpu_baseline):
 * `threads` OpenMP threads and max-active-levels 1 (nested pranges serialised).  Set through
 * the API because libgomp reads OMP_* only once, when it is first loaded (possibly by torch
 * before this library).  Returns the thread count a parallel region then gets. */
int oracle_set_threads(int threads) {
  if (threads > 0) omp_set_num_threads(threads);
  omp_set_max_active_levels(1);
  return oracle_num_threads();
}
