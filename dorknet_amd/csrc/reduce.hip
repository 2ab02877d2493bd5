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

// Float4-column variant: thread (j, q) owns 4 adjacent columns (one 16-byte load per row) and
// sums rows q, q + TPO, ...; a wave reads 64 / CG rows of CG * 16 contiguous bytes, so the
// slab streams at full line width.  Four rows are loaded before they are added (same order).
template <int CG, int TPO>
__global__ __launch_bounds__(CG* TPO) void splitk_reduce4_kernel(const float* __restrict__ ws, int splits, int M,
                                                                  int N, float* __restrict__ out,
                                                                  const float* __restrict__ w, float l2, int mode,
                                                                  int C, int Cp, int R, int S) {
  __shared__ double red[TPO][CG][4];
  const int j = threadIdx.x % CG;
  const int q = threadIdx.x / CG;
  const long long total = (long long)M * N;
  const long long idx = ((long long)blockIdx.x * CG + j) * 4;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (idx < total) {
    const float* p = ws + idx;
    int s = q;
    for (; s + 3 * TPO < splits; s += 4 * TPO) {
      f32x4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = ld4(p + (size_t)(s + k * TPO) * total);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a0 += (double)v[k].x;
        a1 += (double)v[k].y;
        a2 += (double)v[k].z;
        a3 += (double)v[k].w;
      }
    }
    for (; s < splits; s += TPO) {
      const f32x4 v = ld4(p + (size_t)s * total);
      a0 += (double)v.x;
      a1 += (double)v.y;
      a2 += (double)v.z;
      a3 += (double)v.w;
    }
  }
  red[q][j][0] = a0;
  red[q][j][1] = a1;
  red[q][j][2] = a2;
  red[q][j][3] = a3;
  __syncthreads();
  // 4 * CG results per block, finalized in a fixed order over the TPO lane sums
  for (int t = threadIdx.x; t < 4 * CG; t += CG * TPO) {
    const int jj = t >> 2, e = t & 3;
    const long long o_idx = ((long long)blockIdx.x * CG + jj) * 4 + e;
    if (o_idx >= total) break;
    double sum = 0.0;
#pragma unroll 8
    for (int k = 0; k < TPO; ++k) sum += red[k][jj][e];
    const int m = (int)(o_idx / N), n = (int)(o_idx - (long long)m * N);
    size_t o;
    if (mode == 0) {
      o = (size_t)o_idx;
    } else {
      const int tap = n / Cp;
      const int c = n - tap * Cp;
      if (c >= C) continue;
      const int r = tap / S, s2 = tap - r * S;
      o = (((size_t)m * C + c) * R + r) * S + s2;
    }
    float v = (float)sum;
    if (w) v = v + l2 * w[o];
    out[o] = v;
  }
}

// Several float4-column reduces (mode 0) in one launch: the deferred weight-gradient reduces a flush
// batches (dk_wgrad_reduce_flush).  Task t owns blocks [block0, block0 + nblk) and sums its slab with
// splitk_reduce4_kernel's thread layout for its TPO (64 / 16 / 4 by the same split-count rule, so
// every column's sum is in the same order: bit-identical to the per-task launch); one launch instead
// of one per layer, each of which paid a launch and a serial tail of its own.
constexpr int kMultiMax = 32;
struct MultiTask {
  const float* ws;
  float* out;
  const float* w;
  float l2;
  int splits, total, tpo, block0;
};
struct MultiTasks {
  MultiTask t[kMultiMax];
  int n;
};
__device__ __forceinline__ void multi_reduce_task(const MultiTask& k, int blk, int tid, double* red) {
  const int TPO = k.tpo, CG = 256 / TPO;
  const int j = tid % CG, q = tid / CG;
  const long long total = k.total;
  const long long idx = ((long long)blk * CG + j) * 4;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (idx < total) {
    const float* p = k.ws + idx;
    int s = q;
    for (; s + 3 * TPO < k.splits; s += 4 * TPO) {
      f32x4 v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = ld4(p + (size_t)(s + e * TPO) * total);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a0 += (double)v[e].x;
        a1 += (double)v[e].y;
        a2 += (double)v[e].z;
        a3 += (double)v[e].w;
      }
    }
    for (; s < k.splits; s += TPO) {
      const f32x4 v = ld4(p + (size_t)s * total);
      a0 += (double)v.x;
      a1 += (double)v.y;
      a2 += (double)v.z;
      a3 += (double)v.w;
    }
  }
  // red[q][j][4] (TPO x CG x 4 doubles = 8 KB)
  double* r = red + ((size_t)q * CG + j) * 4;
  r[0] = a0;
  r[1] = a1;
  r[2] = a2;
  r[3] = a3;
  __syncthreads();
  for (int t = tid; t < 4 * CG; t += 256) {
    const int jj = t >> 2, e = t & 3;
    const long long o = ((long long)blk * CG + jj) * 4 + e;
    if (o >= total) break;
    double sum = 0.0;
    for (int l = 0; l < TPO; ++l) sum += red[((size_t)l * CG + jj) * 4 + e];
    float v = (float)sum;
    if (k.w) v = v + k.l2 * k.w[o];
    k.out[o] = v;
  }
}
__global__ __launch_bounds__(256) void splitk_multi_kernel(MultiTasks tasks) {
  __shared__ double red[256 * 4];
  int ti = 0;
  while (ti + 1 < tasks.n && (int)blockIdx.x >= tasks.t[ti + 1].block0) ++ti;  // uniform
  const MultiTask& k = tasks.t[ti];
  multi_reduce_task(k, (int)blockIdx.x - k.block0, threadIdx.x, red);
}
static int multi_tpo(int splits) { return splits >= 256 ? 64 : splits >= 32 ? 16 : 4; }

int splitk_reduce(const float* ws, int splits, int M, int N, float* out, const float* w, float l2, int mode, int C,
                  int Cp, int R, int S, hipStream_t st) {
  const long long total = (long long)M * N;
  if ((total & 3) == 0 && (reinterpret_cast<uintptr_t>(ws) & 15) == 0) {
    // Narrow outputs (a 64 x 64 weight gradient is 4096 floats) get 4-column-group blocks, so the
    // grid still spans the CUs (64 blocks of 16 groups left 3/4 of the chip idle).  Each
    // column's sum order is the same for every CG.
    const bool narrow = cdivll(total, 64) < 512;
    if (splits >= 256) {
      if (narrow)
        hipLaunchKernelGGL((splitk_reduce4_kernel<4, 64>), dim3((unsigned)cdivll(total, 16)), dim3(256), 0, st, ws,
                           splits, M, N, out, w, l2, mode, C, Cp, R, S);
      else
        hipLaunchKernelGGL((splitk_reduce4_kernel<16, 64>), dim3((unsigned)cdivll(total, 64)), dim3(1024), 0, st, ws,
                           splits, M, N, out, w, l2, mode, C, Cp, R, S);
    } else if (splits >= 32) {
      if (narrow)
        hipLaunchKernelGGL((splitk_reduce4_kernel<4, 16>), dim3((unsigned)cdivll(total, 16)), dim3(64), 0, st, ws,
                           splits, M, N, out, w, l2, mode, C, Cp, R, S);
      else
        hipLaunchKernelGGL((splitk_reduce4_kernel<16, 16>), dim3((unsigned)cdivll(total, 64)), dim3(256), 0, st, ws,
                           splits, M, N, out, w, l2, mode, C, Cp, R, S);
    } else {
      hipLaunchKernelGGL((splitk_reduce4_kernel<64, 4>), dim3((unsigned)cdivll(total, 256)), dim3(256), 0, st, ws,
                         splits, M, N, out, w, l2, mode, C, Cp, R, S);
    }
    return launch_status();
  }
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

namespace {
struct PendingReduce {
  const float* ws;
  int splits, M, N;
  float* out;
  const float* w;
  float l2;
};
// Recorded reduces, launched in order by the next flush (the caller batches several layers' reduces
// behind one cross-stream wait: each wait costs the main stream a ~7 us gap between kernels).
constexpr int kMaxPending = 64;
thread_local int t_defer = 0;
thread_local int t_npending = 0;
thread_local int t_mark = 0;  // queue depth when recording was last turned on (dk_wgrad_reduce_defer(1))
thread_local PendingReduce t_pending[kMaxPending];
}  // namespace

int wgrad_reduce(const float* ws, int splits, int M, int N, float* out, const float* w, float l2, hipStream_t st) {
  if (!t_defer) return splitk_reduce(ws, splits, M, N, out, w, l2, 0, N, N, 1, 1, st);
  if (t_npending == kMaxPending) return DK_ERR_ARGS;  // never flushed
  t_pending[t_npending++] = PendingReduce{ws, splits, M, N, out, w, l2};
  return 0;
}

}  // namespace dk

// Deferred weight-gradient reduce.  mode 1: the fused backward entry points called next on this
// host thread (dk_dwconv_bwd_bnbwd_f32 / _bf16 / _join_f32, dk_dwconv_bwd_s2_bnbwd_*,
// dk_pwconv_bwd_bnbwd_f32 / _bf16) leave their weight-gradient partial slab unreduced and record
// the reduce; mode 0: back to reducing in the entry point (recorded reduces stay for
// dk_wgrad_reduce_flush); mode -1: as 0 and drop the ones recorded since the last mode 1 (an entry
// point that failed inside it), keeping those of the layers before.
DK_API int dk_wgrad_reduce_defer(int mode) {
  if (mode < -1 || mode > 1) return dk::DK_ERR_ARGS;
  if (mode == 1 && !dk::t_defer) dk::t_mark = dk::t_npending;
  if (mode == -1 && dk::t_npending > dk::t_mark) dk::t_npending = dk::t_mark;
  dk::t_defer = mode == 1;
  return 0;
}

// Reduces recorded and not yet flushed on this host thread.
DK_API int dk_wgrad_reduce_pending(void) { return dk::t_npending; }

// Launch the recorded reduces on `stream`, in the order recorded (fixed order each, the same result
// as in the entry point).  The slabs must stay untouched until they have run; DK_ERR_ARGS if none is
// recorded.  If a launch fails, the reduces not launched stay recorded (in order) and the error is
// returned.
DK_API int dk_wgrad_reduce_flush(void* stream) {
  using namespace dk;
  if (t_npending == 0) return DK_ERR_ARGS;
  const int n = t_npending;
  const hipStream_t st = as_stream(stream);
  // float4-column slabs go into multi-task launches (same per-column order as splitk_reduce4_kernel),
  // the rest one launch each
  MultiTasks mt{};
  int blocks = 0;
  bool launched[kMaxPending] = {};
  int batch[kMultiMax];
  auto launch = [&]() -> int {
    if (mt.n == 0) return 0;
    hipLaunchKernelGGL(splitk_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, st, mt);
    const int rc = launch_status();
    if (rc == 0)
      for (int j = 0; j < mt.n; ++j) launched[batch[j]] = true;
    mt.n = 0;
    blocks = 0;
    return rc;
  };
  int rc = 0;
  for (int i = 0; i < n && rc == 0; ++i) {
    const PendingReduce& p = t_pending[i];
    const long long total = (long long)p.M * p.N;
    if ((total & 3) == 0 && (reinterpret_cast<uintptr_t>(p.ws) & 15) == 0 &&
        total < (1ll << 31)) {
      const int tpo = multi_tpo(p.splits), cg = 256 / tpo;
      const int nb = (int)cdivll(total, 4ll * cg);
      batch[mt.n] = i;
      mt.t[mt.n++] = MultiTask{p.ws, p.out, p.w, p.l2, p.splits, (int)total, tpo, blocks};
      blocks += nb;
      if (mt.n == kMultiMax) rc = launch();
    } else {
      rc = splitk_reduce(p.ws, p.splits, p.M, p.N, p.out, p.w, p.l2, 0, p.N, p.N, 1, 1, st);
      launched[i] = rc == 0;
    }
  }
  if (rc == 0) rc = launch();
  // keep what did not launch
  int k = 0;
  for (int i = 0; i < n; ++i)
    if (!launched[i]) t_pending[k++] = t_pending[i];
  t_npending = k;
  if (t_mark > k) t_mark = k;
  return rc;
}
