// Deterministic fixed-order reductions of partial slabs, shared by the split-K GEMM
// (weight gradients), depthwise wgrad and batch norm.
//
// A partial slab is part[rows][W] (rows = split-K slices / blocks).  One block sums CPB
// adjacent columns with TPO threads per column: thread (j, q) sums rows q, q+TPO, ...
// (independent loads, so many are in flight), then the TPO lane sums are combined in a
// fixed order in LDS.  Same result on every run, no atomics.
#include "dk_common.h"

namespace dk {

template <int TPO>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int splits, int M, int N,
                                                            float* __restrict__ out, const float* __restrict__ w,
                                                            float l2, int mode, int C, int Cp, int R, int S) {
  constexpr int CPB = 256 / TPO;
  __shared__ double red[TPO][CPB];
  const int j = threadIdx.x % CPB;
  const int q = threadIdx.x / CPB;
  const long long total = (long long)M * N;
  const long long idx = (long long)blockIdx.x * CPB + j;
  double acc = 0.0;
  if (idx < total) {
    const float* p = ws + idx;
    int s = q;
    for (; s + 3 * TPO < splits; s += 4 * TPO) {
      const float a = p[(size_t)s * total], b = p[(size_t)(s + TPO) * total];
      const float c = p[(size_t)(s + 2 * TPO) * total], d = p[(size_t)(s + 3 * TPO) * total];
      acc += (double)a;
      acc += (double)b;
      acc += (double)c;
      acc += (double)d;
    }
    for (; s < splits; s += TPO) acc += (double)p[(size_t)s * total];
  }
  red[q][j] = acc;
  __syncthreads();
  if (q != 0 || idx >= total) return;
  double sum = 0.0;
#pragma unroll
  for (int k = 0; k < TPO; ++k) sum += red[k][j];
  const int m = (int)(idx / N), n = (int)(idx - (long long)m * N);
  size_t o;
  if (mode == 0) {
    o = (size_t)idx;
  } else {
    const int tap = n / Cp;
    const int c = n - tap * Cp;
    if (c >= C) return;
    const int r = tap / S, s2 = tap - r * S;
    o = (((size_t)m * C + c) * R + r) * S + s2;
  }
  float v = (float)sum;
  if (w) v = v + l2 * w[o];
  out[o] = v;
}

int splitk_reduce(const float* ws, int splits, int M, int N, float* out, const float* w, float l2, int mode, int C,
                  int Cp, int R, int S, hipStream_t st) {
  const long long total = (long long)M * N;
  if (splits >= 512) {
    // long slabs (one row per block of a fused backward): 64 lanes per column
    constexpr int TPO = 64, CPB = 256 / TPO;
    hipLaunchKernelGGL(splitk_reduce_kernel<TPO>, dim3((unsigned)cdivll(total, CPB)), dim3(256), 0, st, ws, splits,
                       M, N, out, w, l2, mode, C, Cp, R, S);
  } else if (splits >= 64) {
    constexpr int TPO = 16, CPB = 256 / TPO;
    hipLaunchKernelGGL(splitk_reduce_kernel<TPO>, dim3((unsigned)cdivll(total, CPB)), dim3(256), 0, st, ws, splits,
                       M, N, out, w, l2, mode, C, Cp, R, S);
  } else if (splits >= 8) {
    constexpr int TPO = 8, CPB = 256 / TPO;
    hipLaunchKernelGGL(splitk_reduce_kernel<TPO>, dim3((unsigned)cdivll(total, CPB)), dim3(256), 0, st, ws, splits,
                       M, N, out, w, l2, mode, C, Cp, R, S);
  } else {
    hipLaunchKernelGGL(splitk_reduce_kernel<1>, dim3((unsigned)cdivll(total, 256)), dim3(256), 0, st, ws, splits, M,
                       N, out, w, l2, mode, C, Cp, R, S);
  }
  return launch_status();
}

}  // namespace dk
