// Bandwidth ceiling probe (not on the training path): how fast can the GPU stream a given mix of
// read and write streams?  Each of nin inputs is read once, each of nout outputs written once,
// 16 bytes per lane per access, 4 accesses per lane in flight, a grid of every resident slot.
// scripts/stream_ceiling.py uses it to price the pointwise kernels' traffic mixes
// (dk_pwconv_dgrad_bnbwd_f32: 3 reads + 2 writes per element group).
#include "dk_common.h"

namespace dk {

template <int NIN, int NOUT, int NT>
__global__ __launch_bounds__(256) void stream_mix_kernel(const f32x4* __restrict__ a, const f32x4* __restrict__ b,
                                                         const f32x4* __restrict__ c, f32x4* __restrict__ o0,
                                                         f32x4* __restrict__ o1, long long n4) {
  constexpr int U = 4;
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 va[U], vb[U], vc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      va[u] = a[i + u * stride];
      if constexpr (NIN > 1) vb[u] = b[i + u * stride];
      if constexpr (NIN > 2) vc[u] = c[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f32x4 s = va[u];
      if constexpr (NIN > 1) s += vb[u];
      if constexpr (NIN > 2) s += vc[u];
      if constexpr (NT) {
        if constexpr (NOUT > 0) __builtin_nontemporal_store(s, o0 + i + u * stride);
        if constexpr (NOUT > 1) __builtin_nontemporal_store(s * 2.f, o1 + i + u * stride);
      } else {
        if constexpr (NOUT > 0) o0[i + u * stride] = s;
        if constexpr (NOUT > 1) o1[i + u * stride] = s * 2.f;
      }
      if constexpr (NOUT == 0) {
        if (s[0] == 12345.678f) o0[0] = s;  // keep the loads alive
      }
    }
  }
  for (; i < n4; i += stride) {
    f32x4 s = a[i];
    if constexpr (NIN > 1) s += b[i];
    if constexpr (NIN > 2) s += c[i];
    if constexpr (NOUT > 0) o0[i] = s;
    if constexpr (NOUT > 1) o1[i] = s * 2.f;
  }
}

}  // namespace dk

using namespace dk;

DK_API int dk_debug_stream_mix(const float* a, const float* b, const float* c, float* o0, float* o1, int nin,
                               int nout, long long numel, int blocks, void* stream) {
  const int nt = nout >= 10;  // nout + 10: nontemporal stores
  nout %= 10;
  const long long n4 = numel / 4;
  const dim3 grid(blocks > 0 ? blocks : 2048), blk(256);
  const hipStream_t st = as_stream(stream);
  const f32x4 *A = reinterpret_cast<const f32x4*>(a), *B = reinterpret_cast<const f32x4*>(b),
              *C = reinterpret_cast<const f32x4*>(c);
  f32x4 *O0 = reinterpret_cast<f32x4*>(o0), *O1 = reinterpret_cast<f32x4*>(o1);
#define DK_MIX(I, O)                                                                                       \
  if (nin == I && nout == O && !nt) hipLaunchKernelGGL((stream_mix_kernel<I, O, 0>), grid, blk, 0, st, A, B, C, O0, O1, n4); \
  else if (nin == I && nout == O) hipLaunchKernelGGL((stream_mix_kernel<I, O, 1>), grid, blk, 0, st, A, B, C, O0, O1, n4); else
  DK_MIX(1, 0) DK_MIX(1, 1) DK_MIX(2, 1) DK_MIX(2, 2) DK_MIX(3, 1) DK_MIX(3, 2) DK_MIX(1, 2) return DK_ERR_ARGS;
#undef DK_MIX
  return launch_status();
}
