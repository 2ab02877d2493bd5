// Training-mode batch norm over an NHWC (or [rows][features]) fp32 tensor, gfx950.
//
// Replaces layers/batch_norm.py:54-174 (GPU branch: cp.mean / cp.var / elementwise /
// cp.sum, about ten CuPy kernels per layer and two saved full-size temporaries).
// Same maths, different data flow:
//   * statistics are one read of X: per-block fp64 partial sums of x and x^2, then a
//     fixed-order fp64 finalize (deterministic; population variance like cp.var);
//   * nothing but X and the per-channel (mean, std) is kept for backward: X_demean and
//     X_hat are recomputed on the fly (batch_norm.py:72-73 stores both);
//   * the optional ReLU that follows BN (activations.py:37-42) is fused into the
//     apply pass, and its backward mask is recomputed from X in the backward reduce;
//   * backward is one reduce pass (sum dy, sum dy*x_hat) and one apply pass.
//
// Per-channel parameter vectors (mean, std, invstd, gamma, beta, ...) are fp32 [C].
#include "dk_common.h"

namespace dk {

// The BN output for one element.  Forward apply and the backward ReLU-mask
// recompute call this same function so the mask is bit-identical to forward.
__device__ __forceinline__ float bn_out(float x, float mean, float invstd, float gamma, float beta) {
  const float xh = (x - mean) * invstd;
  return gamma * xh + beta;
}

// Stats partials.  Thread (cg, pl) owns channel group cg (V channels) and pixel lane pl.
// part[blk][0][c] = sum x, part[blk][1][c] = sum x^2 (fp64).
template <int V>
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(const float* __restrict__ x, int P, int C, int ppb,
                                                               double* __restrict__ part) {
  __shared__ double red[2][256][V];
  const int CG = C / V;
  const int cgt = CG < 256 ? CG : 256;
  const int PL = 256 / cgt;
  const int tid = threadIdx.x;
  const int cg = blockIdx.y * cgt + tid % cgt;
  const int pl = tid / cgt;
  const bool active = pl < PL && cg < CG;
  const int p0 = blockIdx.x * ppb, p1 = min(P, p0 + ppb);
  double s[V], q[V];
#pragma unroll
  for (int e = 0; e < V; ++e) s[e] = q[e] = 0.0;
  if (active) {
    for (int p = p0 + pl; p < p1; p += PL) {
      const float* src = x + (size_t)p * C + cg * V;
      float v[V];
      if constexpr (V == 4) {
        const f32x4 t = ld4(src);
        v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
      } else {
        v[0] = src[0];
      }
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const double d = (double)v[e];
        s[e] += d;
        q[e] += d * d;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    red[0][tid][e] = s[e];
    red[1][tid][e] = q[e];
  }
  __syncthreads();
  const int items = 2 * cgt * V;
  for (int it = tid; it < items; it += 256) {
    const int e = it % V;
    const int g = (it / V) % cgt;
    const int which = it / (V * cgt);
    const int cgg = blockIdx.y * cgt + g;
    if (cgg >= CG) continue;
    double acc = 0.0;
    for (int qq = 0; qq < PL; ++qq) acc += red[which][qq * cgt + g][e];
    part[((size_t)blockIdx.x * 2 + which) * C + cgg * V + e] = acc;
  }
}

// Finalize: mean, population var, std = sqrt(var + eps); running mean/std update
// (batch_norm.py:76-89: first call copies, later calls blend with `momentum`).
__global__ void bn_stats_finalize_kernel(const double* __restrict__ part, int nblk, int C, double count, float eps,
                                         float momentum, int first, float* __restrict__ mean_out,
                                         float* __restrict__ std_out, float* __restrict__ invstd_out,
                                         float* __restrict__ run_mean, float* __restrict__ run_std) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int b = 0; b < nblk; ++b) {
    s += part[((size_t)b * 2 + 0) * C + c];
    q += part[((size_t)b * 2 + 1) * C + c];
  }
  const double mean = s / count;
  double var = q / count - mean * mean;
  if (var < 0.0) var = 0.0;
  const float meanf = (float)mean;
  const float stdf = sqrtf((float)var + eps);
  mean_out[c] = meanf;
  std_out[c] = stdf;
  invstd_out[c] = 1.0f / stdf;
  if (run_mean) {
    if (first) {
      run_mean[c] = meanf;
      run_std[c] = stdf;
    } else {
      run_mean[c] = momentum * run_mean[c] + (1.0f - momentum) * meanf;
      run_std[c] = momentum * run_std[c] + (1.0f - momentum) * stdf;
    }
  }
}

// y = gamma * (x - mean) * invstd + beta, optionally ReLU'd (mask = y > 0 as uint8).
template <int V>
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ x, long long nvec, int C,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, int relu,
                                                       float* __restrict__ y, uint8_t* __restrict__ mask) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nvec) return;
  const int c0 = (int)((i * V) % C);
#pragma unroll
  for (int e = 0; e < V; ++e) {
    const int c = c0 + e;
    float o = bn_out(x[i * V + e], mean[c], invstd[c], gamma[c], beta[c]);
    if (relu) {
      const bool pos = o > 0.f;
      o = pos ? o : 0.f;
      if (mask) mask[i * V + e] = pos;
    }
    y[i * V + e] = o;
  }
}

// Backward reduce partials: sum dy_e and sum dy_e * x_hat, where dy_e = dy, or with
// relu: dy * (bn_out(x) > 0) -- the fused ReLU backward (activations.py:44-47).
template <int V>
__global__ __launch_bounds__(256) void bn_bwd_partial_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ dy, int P, int C, int ppb,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, int relu,
                                                             double* __restrict__ part) {
  __shared__ double red[2][256][V];
  const int CG = C / V;
  const int cgt = CG < 256 ? CG : 256;
  const int PL = 256 / cgt;
  const int tid = threadIdx.x;
  const int cg = blockIdx.y * cgt + tid % cgt;
  const int pl = tid / cgt;
  const bool active = pl < PL && cg < CG;
  const int p0 = blockIdx.x * ppb, p1 = min(P, p0 + ppb);
  double s[V], q[V];
  float mu[V], is[V], ga[V], be[V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    s[e] = q[e] = 0.0;
    const int c = active ? cg * V + e : 0;
    mu[e] = mean[c];
    is[e] = invstd[c];
    ga[e] = gamma[c];
    be[e] = beta[c];
  }
  if (active) {
    for (int p = p0 + pl; p < p1; p += PL) {
      const size_t off = (size_t)p * C + cg * V;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float xv = x[off + e];
        float g = dy[off + e];
        const float xh = (xv - mu[e]) * is[e];
        if (relu && !(bn_out(xv, mu[e], is[e], ga[e], be[e]) > 0.f)) g = 0.f;
        s[e] += (double)g;
        q[e] += (double)g * (double)xh;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    red[0][tid][e] = s[e];
    red[1][tid][e] = q[e];
  }
  __syncthreads();
  const int items = 2 * cgt * V;
  for (int it = tid; it < items; it += 256) {
    const int e = it % V;
    const int g = (it / V) % cgt;
    const int which = it / (V * cgt);
    const int cgg = blockIdx.y * cgt + g;
    if (cgg >= CG) continue;
    double acc = 0.0;
    for (int qq = 0; qq < PL; ++qq) acc += red[which][qq * cgt + g][e];
    part[((size_t)blockIdx.x * 2 + which) * C + cgg * V + e] = acc;
  }
}

// dgamma = sum dy_e * x_hat, dbeta = sum dy_e (batch_norm.py:159-174) from the *local*
// partials; k1 = mean(dy_e), k2 = sum(dy_e * x_hat) / count from the (possibly
// all-reduced, SyncBN) *global* partials.  Without SyncBN both are the same buffer.
__global__ void bn_bwd_finalize_kernel(const double* __restrict__ part_l, int nblk_l,
                                       const double* __restrict__ part_g, int nblk_g, int C, double count,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta,
                                       float* __restrict__ k12) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int b = 0; b < nblk_l; ++b) {
    s += part_l[((size_t)b * 2 + 0) * C + c];
    q += part_l[((size_t)b * 2 + 1) * C + c];
  }
  dgamma[c] = (float)q;
  dbeta[c] = (float)s;
  if (part_g != part_l || nblk_g != nblk_l) {
    s = q = 0.0;
    for (int b = 0; b < nblk_g; ++b) {
      s += part_g[((size_t)b * 2 + 0) * C + c];
      q += part_g[((size_t)b * 2 + 1) * C + c];
    }
  }
  k12[c] = (float)(s / count);
  k12[C + c] = (float)(q / count);
}

// out[w][c] = sum_b part[b][w][c]   (fixed order) -- the per-rank vector SyncBN all-reduces
__global__ void bn_collapse_kernel(const double* __restrict__ part, int nblk, int C, double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * C) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += part[(size_t)b * 2 * C + i];
  out[i] = s;
}

// dx = gamma * invstd * (dy_e - k1 - x_hat * k2)   (batch_norm.py:125-156, rearranged:
// (1/M) * X_demean / std^2 * sum(dy * X_demean) == x_hat * sum(dy * x_hat) / M)
template <int V>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                           long long nvec, int C, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, int relu,
                                                           const float* __restrict__ k12, float* __restrict__ dx) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nvec) return;
  const int c0 = (int)((i * V) % C);
#pragma unroll
  for (int e = 0; e < V; ++e) {
    const int c = c0 + e;
    const float xv = x[i * V + e];
    float g = dy[i * V + e];
    const float mu = mean[c], is = invstd[c], ga = gamma[c];
    if (relu && !(bn_out(xv, mu, is, ga, beta[c]) > 0.f)) g = 0.f;
    const float xh = (xv - mu) * is;
    dx[i * V + e] = (ga * is) * (g - k12[c] - xh * k12[C + c]);
  }
}

// Inference parameters from running stats: mean = running_mean, invstd = 1 / running_std
// (batch_norm.py:101-115 divides by running_std).
__global__ void bn_infer_params_kernel(const float* __restrict__ run_std, int C, float* __restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) invstd[c] = 1.0f / run_std[c];
}

static int bn_blocks(int P, int C) {
  // ~64 rows per pixel lane keeps fp64 accumulation short and gives >= 4 blocks per CU.
  int nblk = cdiv(P, 1024);
  if (nblk > 1024) nblk = 1024;
  if (nblk < 1) nblk = 1;
  (void)C;
  return nblk;
}

}  // namespace dk

using namespace dk;

DK_API int dk_bn_partial_blocks(int P, int C) { return bn_blocks(P, C); }

DK_API size_t dk_bn_workspace_bytes(int P, int C) { return (size_t)bn_blocks(P, C) * 2 * C * sizeof(double); }

static int bn_grid(const float* x, int C, int nblk, dim3* grid) {
  const bool vec = (C % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
  const int V = vec ? 4 : 1;
  const int CG = C / V;
  const int cgt = CG < 256 ? CG : 256;
  *grid = dim3(nblk, cdiv(CG, cgt));
  return vec;
}

// Stage 1 of forward statistics: part[nblk][2][C] (fp64 sum x, sum x^2) over x[P][C].
DK_API int dk_bn_stats_partial_f64(const float* x, int P, int C, void* ws, size_t ws_bytes, void* stream) {
  if (ws_bytes < dk_bn_workspace_bytes(P, C)) return DK_ERR_WORKSPACE;
  const int nblk = bn_blocks(P, C);
  const int ppb = cdiv(P, nblk);
  dim3 grid;
  if (bn_grid(x, C, nblk, &grid))
    hipLaunchKernelGGL(bn_stats_partial_kernel<4>, grid, dim3(256), 0, as_stream(stream), x, P, C, ppb,
                       static_cast<double*>(ws));
  else
    hipLaunchKernelGGL(bn_stats_partial_kernel<1>, grid, dim3(256), 0, as_stream(stream), x, P, C, ppb,
                       static_cast<double*>(ws));
  return launch_status();
}

// out[2][C] = fixed-order sum of part[nblk][2][C].
DK_API int dk_bn_collapse_f64(const void* part, int nblk, int C, void* out, void* stream) {
  hipLaunchKernelGGL(bn_collapse_kernel, dim3(cdiv(2 * C, 256)), dim3(256), 0, as_stream(stream),
                     static_cast<const double*>(part), nblk, C, static_cast<double*>(out));
  return launch_status();
}

// Stage 2: mean, population variance, std = sqrt(var + eps), invstd; running stats.
DK_API int dk_bn_stats_finalize_f32(const void* part, int nblk, int C, double count, float eps, float momentum,
                                    int first, float* mean, float* std_, float* invstd, float* run_mean,
                                    float* run_std, void* stream) {
  hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3(cdiv(C, 256)), dim3(256), 0, as_stream(stream),
                     static_cast<const double*>(part), nblk, C, count, eps, momentum, first, mean, std_, invstd,
                     run_mean, run_std);
  return launch_status();
}

// Forward statistics (both stages).  x is [P][C] (NHWC with P = N*H*W, or [rows][features]).
DK_API int dk_bn_stats_f32(const float* x, int P, int C, float eps, float momentum, int first, float* mean,
                           float* std_, float* invstd, float* run_mean, float* run_std, void* ws, size_t ws_bytes,
                           void* stream) {
  int rc = dk_bn_stats_partial_f64(x, P, C, ws, ws_bytes, stream);
  if (rc) return rc;
  return dk_bn_stats_finalize_f32(ws, bn_blocks(P, C), C, (double)P, eps, momentum, first, mean, std_, invstd,
                                  run_mean, run_std, stream);
}

DK_API int dk_bn_infer_params_f32(const float* run_std, int C, float* invstd, void* stream) {
  hipLaunchKernelGGL(bn_infer_params_kernel, dim3(cdiv(C, 256)), dim3(256), 0, as_stream(stream), run_std, C, invstd);
  return launch_status();
}

// y = gamma * (x - mean) * invstd + beta  [+ ReLU; mask (uint8) may be null]
DK_API int dk_bn_apply_f32(const float* x, long long numel, int C, const float* mean, const float* invstd,
                           const float* gamma, const float* beta, int relu, float* y, uint8_t* mask, void* stream) {
  const bool vec = (C % 4 == 0) && (numel % 4 == 0);
  if (vec) {
    const long long nvec = numel / 4;
    hipLaunchKernelGGL(bn_apply_kernel<4>, dim3((unsigned)cdivll(nvec, 256)), dim3(256), 0, as_stream(stream), x,
                       nvec, C, mean, invstd, gamma, beta, relu, y, mask);
  } else {
    hipLaunchKernelGGL(bn_apply_kernel<1>, dim3((unsigned)cdivll(numel, 256)), dim3(256), 0, as_stream(stream), x,
                       numel, C, mean, invstd, gamma, beta, relu, y, mask);
  }
  return launch_status();
}

// Backward stage 1: part[nblk][2][C] = (sum dy_e, sum dy_e * x_hat); relu != 0 fuses the
// following ReLU's backward (its mask is recomputed from x).
DK_API int dk_bn_bwd_partial_f64(const float* x, const float* dy, int P, int C, const float* mean,
                                 const float* invstd, const float* gamma, const float* beta, int relu, void* ws,
                                 size_t ws_bytes, void* stream) {
  if (ws_bytes < dk_bn_workspace_bytes(P, C)) return DK_ERR_WORKSPACE;
  const int nblk = bn_blocks(P, C);
  const int ppb = cdiv(P, nblk);
  dim3 grid;
  if (bn_grid(x, C, nblk, &grid))
    hipLaunchKernelGGL(bn_bwd_partial_kernel<4>, grid, dim3(256), 0, as_stream(stream), x, dy, P, C, ppb, mean,
                       invstd, gamma, beta, relu, static_cast<double*>(ws));
  else
    hipLaunchKernelGGL(bn_bwd_partial_kernel<1>, grid, dim3(256), 0, as_stream(stream), x, dy, P, C, ppb, mean,
                       invstd, gamma, beta, relu, static_cast<double*>(ws));
  return launch_status();
}

// Backward stage 2: dgamma/dbeta from the local partials, k12 = [k1[C], k2[C]] from the global ones.
DK_API int dk_bn_bwd_finalize_f32(const void* part_local, int nblk_local, const void* part_global, int nblk_global,
                                  int C, double count, float* dgamma, float* dbeta, float* k12, void* stream) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(cdiv(C, 256)), dim3(256), 0, as_stream(stream),
                     static_cast<const double*>(part_local), nblk_local, static_cast<const double*>(part_global),
                     nblk_global, C, count, dgamma, dbeta, k12);
  return launch_status();
}

// Backward stage 3: dx = gamma * invstd * (dy_e - k1 - x_hat * k2).
DK_API int dk_bn_bwd_apply_f32(const float* x, const float* dy, long long numel, int C, const float* mean,
                               const float* invstd, const float* gamma, const float* beta, int relu,
                               const float* k12, float* dx, void* stream) {
  const bool vec = (C % 4 == 0) && (numel % 4 == 0);
  if (vec) {
    const long long nvec = numel / 4;
    hipLaunchKernelGGL(bn_bwd_apply_kernel<4>, dim3((unsigned)cdivll(nvec, 256)), dim3(256), 0, as_stream(stream), x,
                       dy, nvec, C, mean, invstd, gamma, beta, relu, k12, dx);
  } else {
    hipLaunchKernelGGL(bn_bwd_apply_kernel<1>, dim3((unsigned)cdivll(numel, 256)), dim3(256), 0, as_stream(stream),
                       x, dy, numel, C, mean, invstd, gamma, beta, relu, k12, dx);
  }
  return launch_status();
}

DK_API size_t dk_bn_bwd_workspace_bytes(int P, int C) {
  return dk_bn_workspace_bytes(P, C) + 2 * (size_t)C * sizeof(float);
}

// Backward (all stages, local statistics).  Writes dgamma/dbeta [C] and dx [P][C].
DK_API int dk_bn_bwd_f32(const float* x, const float* dy, int P, int C, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, int relu, float* dgamma, float* dbeta, float* dx,
                         void* ws, size_t ws_bytes, void* stream) {
  if (ws_bytes < dk_bn_bwd_workspace_bytes(P, C)) return DK_ERR_WORKSPACE;
  const int nblk = bn_blocks(P, C);
  float* k12 = reinterpret_cast<float*>(static_cast<char*>(ws) + dk_bn_workspace_bytes(P, C));
  int rc = dk_bn_bwd_partial_f64(x, dy, P, C, mean, invstd, gamma, beta, relu, ws, ws_bytes, stream);
  if (rc) return rc;
  rc = dk_bn_bwd_finalize_f32(ws, nblk, ws, nblk, C, (double)P, dgamma, dbeta, k12, stream);
  if (rc) return rc;
  return dk_bn_bwd_apply_f32(x, dy, (long long)P * C, C, mean, invstd, gamma, beta, relu, k12, dx, stream);
}
