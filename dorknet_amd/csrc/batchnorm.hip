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
//     apply pass, and its backward mask is recomputed from X in the backward passes;
//   * backward is one reduce pass (sum dy, sum dy*x_hat) and one apply pass.
//
// Layout of the streaming kernels ("row loop"): a block owns a contiguous range of
// rows (pixels); thread (cg, pl) owns channel group cg (V = 4 channels, one float4) and
// walks rows pl, pl + PL, ... with four rows of loads in flight.  Per-channel
// parameters live in registers, so there is no per-element index arithmetic.
#include "dk_common.h"
#include "fold_tail.h"

namespace dk {


// V elements of storage type E (float, or bf16_t for BASELINE config 5) as fp32 values.
template <int V, class E = float>
struct VecT;
template <class E>
struct VecT<4, E> {
  using T = f32x4;
  __device__ static T load(const E* p) { return ld4(p); }
  __device__ static void store(E* p, T v) { st4(p, v); }
  __device__ static T stored(T v) { return rnd4<E>(v); }
};
template <class E>
struct VecT<1, E> {
  using T = float;
  __device__ static T load(const E* p) { return ld1(p); }
  __device__ static void store(E* p, T v) { st1(p, v); }
  __device__ static T stored(T v) { return rnd1<E>(v); }
};

__device__ __forceinline__ float el(const f32x4& v, int e) { return v[e]; }
__device__ __forceinline__ float el(const float& v, int) { return v; }
__device__ __forceinline__ void set_el(f32x4& v, int e, float x) { v[e] = x; }
__device__ __forceinline__ void set_el(float& v, int, float x) { v = x; }

// Geometry of the row loop, shared by host and device.
struct RowGeom {
  int CG;   // channel groups = C / V
  int cgt;  // channel groups per block (<= 256)
  int PL;   // pixel lanes = 256 / cgt
};

__host__ __device__ inline RowGeom row_geom(int C, int V, int cgt_cap = 256) {
  RowGeom g;
  g.CG = C / V;
  g.cgt = g.CG < cgt_cap ? g.CG : cgt_cap;
  g.PL = 256 / g.cgt;
  return g;
}

// ---------------------------------------------------------------------------------------
// forward statistics: part[blk][0][c] = sum x, part[blk][1][c] = sum x^2 (fp64)
// ---------------------------------------------------------------------------------------
template <int V, class E = float>
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(const E* __restrict__ x, int P, int C, int ppb,
                                                               double* __restrict__ part) {
  using VT = VecT<V, E>;
  __shared__ double red[2][256][V];
  const RowGeom g = row_geom(C, V);
  const int tid = threadIdx.x;
  const int cg = blockIdx.y * g.cgt + tid % g.cgt;
  const int pl = tid / g.cgt;
  const bool active = pl < g.PL && cg < g.CG;
  const int p0 = blockIdx.x * ppb, p1 = min(P, p0 + ppb);
  double s[V], q[V];
#pragma unroll
  for (int e = 0; e < V; ++e) s[e] = q[e] = 0.0;
  if (active) {
    const E* base = x + cg * V;
    const int PL = g.PL;
    int p = p0 + pl;
    for (; p + 3 * PL < p1; p += 4 * PL) {
      typename VT::T v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = VT::load(base + (size_t)(p + u * PL) * C);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const double d = (double)el(v[u], e);
          s[e] += d;
          q[e] += d * d;
        }
    }
    for (; p < p1; p += PL) {
      const typename VT::T v = VT::load(base + (size_t)p * C);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const double d = (double)el(v, e);
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
  const int items = 2 * g.cgt * V;
  for (int it = tid; it < items; it += 256) {
    const int e = it % V;
    const int gg = (it / V) % g.cgt;
    const int which = it / (V * g.cgt);
    const int cgg = blockIdx.y * g.cgt + gg;
    if (cgg >= g.CG) continue;
    double acc = 0.0;
    for (int qq = 0; qq < g.PL; ++qq) acc += red[which][qq * g.cgt + gg][e];
    part[((size_t)blockIdx.x * 2 + which) * C + cgg * V + e] = acc;
  }
}

// Fixed-order block sum of part[b][which][c] over b (one block per channel).
__device__ __forceinline__ void block_sum2(const double* __restrict__ part, int nblk, int C, int c, double* out_s,
                                           double* out_q) {
  __shared__ double rs[256], rq[256];
  double s = 0.0, q = 0.0;
  for (int b = threadIdx.x; b < nblk; b += 256) {
    s += part[((size_t)b * 2 + 0) * C + c];
    q += part[((size_t)b * 2 + 1) * C + c];
  }
  rs[threadIdx.x] = s;
  rq[threadIdx.x] = q;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      rs[threadIdx.x] += rs[threadIdx.x + o];
      rq[threadIdx.x] += rq[threadIdx.x + o];
    }
    __syncthreads();
  }
  *out_s = rs[0];
  *out_q = rq[0];
}

// Finalize (one block per channel): mean, population var, std = sqrt(var + eps);
// running mean/std update (batch_norm.py:76-89: first call copies, later calls blend).
__global__ __launch_bounds__(256) void bn_stats_finalize_kernel(const double* __restrict__ part, int nblk, int C,
                                                                double count, float eps, float momentum, int first,
                                                                float* __restrict__ mean_out,
                                                                float* __restrict__ std_out,
                                                                float* __restrict__ invstd_out,
                                                                float* __restrict__ run_mean,
                                                                float* __restrict__ run_std) {
  const int c = blockIdx.x;
  double s, q;
  block_sum2(part, nblk, C, c, &s, &q);
  if (threadIdx.x != 0) return;
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

// out[w][c] = sum_b part[b][w][c] (one block per channel) -- the per-rank vector SyncBN all-reduces.
__global__ __launch_bounds__(256) void bn_collapse_kernel(const double* __restrict__ part, int nblk, int C,
                                                          double* __restrict__ out) {
  const int c = blockIdx.x;
  double s, q;
  block_sum2(part, nblk, C, c, &s, &q);
  if (threadIdx.x == 0) {
    out[c] = s;
    out[C + c] = q;
  }
}

// Fixed-order reduction of partial rows part[nblk][2][C] (fp64) with the stage-2 maths fused
// in: block = 64 channels x 16 row lanes, each lane holding 16 rows (all loads in flight at
// once), up to kFoldRows rows per block.  With one block along x the block finishes the job
// (FINAL): mode 0 statistics (batch_norm.py:76-89), 1 backward coefficients (:125-174),
// 2 plain sums.  Otherwise it writes one folded row per block and runs again on those.
constexpr int kFoldLanes = 16, kFoldPerLane = 16, kFoldRows = kFoldLanes * kFoldPerLane;

// LEVEL 0: fold up to kFoldRows rows per block into out[blockIdx.x] (a later launch folds
// those).  1 (FINAL): one block along x folds every row and finalizes.  2 (TICKET): as 0,
// then the last block of each 64-column group to arrive (agent-scope ticket, zeroed by the
// caller once and put back to zero here) folds out[] and finalizes -- two levels, one launch.
template <int LEVEL>
__global__ __launch_bounds__(1024) void bn_fold_kernel(const double* __restrict__ part, int nblk, int C,
                                                       double* __restrict__ out, FoldOut o, unsigned* tickets) {
  __shared__ double red[kFoldLanes][64][2];
  __shared__ int last;
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  auto fold = [&](const double* src, int n, int b0, bool sc1) {
    double s = 0.0, q = 0.0;
    if (c < C) {
      double vs[kFoldPerLane], vq[kFoldPerLane];
#pragma unroll
      for (int k = 0; k < kFoldPerLane; ++k) {
        const int b = b0 + k * kFoldLanes;
        const int bb = b < n ? b : n - 1;  // clamp, load unconditionally, mask after
        vs[k] = sc1 ? pub_load(src + ((size_t)bb * 2 + 0) * C + c) : src[((size_t)bb * 2 + 0) * C + c];
        vq[k] = sc1 ? pub_load(src + ((size_t)bb * 2 + 1) * C + c) : src[((size_t)bb * 2 + 1) * C + c];
      }
#pragma unroll
      for (int k = 0; k < kFoldPerLane; ++k) {
        const bool in = b0 + k * kFoldLanes < n;
        s += in ? vs[k] : 0.0;
        q += in ? vq[k] : 0.0;
      }
    }
    red[rl][cl][0] = s;
    red[rl][cl][1] = q;
    __syncthreads();
  };
  auto total = [&](double& S, double& Q) {
    S = 0.0;
    Q = 0.0;
#pragma unroll
    for (int l = 0; l < kFoldLanes; ++l) {
      S += red[l][cl][0];
      Q += red[l][cl][1];
    }
  };
  fold(part, nblk, blockIdx.x * kFoldRows + rl, false);
  if constexpr (LEVEL == 1) {
    if (rl != 0 || c >= C) return;
    double S, Q;
    total(S, Q);
    bn_finalize_channel(c, C, S, Q, o);
  } else {
    if (rl == 0 && c < C) {
      double S, Q;
      total(S, Q);
      if constexpr (LEVEL == 0) {
        out[((size_t)blockIdx.x * 2 + 0) * C + c] = S;
        out[((size_t)blockIdx.x * 2 + 1) * C + c] = Q;
      } else {
        pub_store(out + ((size_t)blockIdx.x * 2 + 0) * C + c, S);
        pub_store(out + ((size_t)blockIdx.x * 2 + 1) * C + c, Q);
      }
    }
    if constexpr (LEVEL == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned* t = tickets + blockIdx.y;
        const unsigned old = __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = old + 1u == gridDim.x;
        if (last) {
          __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      __syncthreads();
      if (!last) return;
      fold(out, gridDim.x, rl, true);  // gridDim.x <= kFoldRows rows (checked on the host)
      if (rl != 0 || c >= C) return;
      double S, Q;
      total(S, Q);
      bn_finalize_channel(c, C, S, Q, o);
    }
  }
}

// ---------------------------------------------------------------------------------------
// forward apply: y = gamma * (x - mean) * invstd + beta  [+ ReLU, optional uint8 mask]
// ---------------------------------------------------------------------------------------
template <int V, class E = float>
__global__ __launch_bounds__(256) void bn_apply_kernel(const E* __restrict__ x, int P, int C, int ppb,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, int relu,
                                                       E* __restrict__ y, uint8_t* __restrict__ mask) {
  using VT = VecT<V, E>;
  const RowGeom g = row_geom(C, V);
  const int tid = threadIdx.x;
  const int cg = blockIdx.y * g.cgt + tid % g.cgt;
  const int pl = tid / g.cgt;
  if (pl >= g.PL || cg >= g.CG) return;
  const int c0 = cg * V;
  float mu[V], is[V], ga[V], be[V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    mu[e] = mean[c0 + e];
    is[e] = invstd[c0 + e];
    ga[e] = gamma[c0 + e];
    be[e] = beta[c0 + e];
  }
  const int p0 = blockIdx.x * ppb, p1 = min(P, p0 + ppb);
  const int PL = g.PL;
  auto one = [&](typename VT::T v, size_t off) {
    typename VT::T o;
    uint32_t mbits = 0;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      float r = bn_out(el(v, e), mu[e], is[e], ga[e], be[e]);
      if (relu) {
        const bool pos = r > 0.f;
        r = pos ? r : 0.f;
        mbits |= (uint32_t)pos << (8 * e);
      }
      set_el(o, e, r);
    }
    VT::store(y + off, o);
    if (mask) {
      if constexpr (V == 4)
        *reinterpret_cast<uint32_t*>(mask + off) = mbits;
      else
        mask[off] = (uint8_t)mbits;
    }
  };
  int p = p0 + pl;
  for (; p + 3 * PL < p1; p += 4 * PL) {
    typename VT::T v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = VT::load(x + (size_t)(p + u * PL) * C + c0);
#pragma unroll
    for (int u = 0; u < 4; ++u) one(v[u], (size_t)(p + u * PL) * C + c0);
  }
  for (; p < p1; p += PL) one(VT::load(x + (size_t)p * C + c0), (size_t)p * C + c0);
}

// ---------------------------------------------------------------------------------------
// backward reduce: sum dy_e and sum dy_e * x_hat, where dy_e = dy, or with relu:
// dy * (bn_out(x) > 0) -- the fused ReLU backward (activations.py:44-47).
// ---------------------------------------------------------------------------------------
// MASKED: dy is the upstream gradient of a ReLU that follows (the post-residual join's,
// residual_block.py:86): g = mask ? dy : 0 is written to gout and reduced -- the ReLU
// backward and this BN's backward reduction in one pass.
template <int V, bool MASKED = false, class E = float>
__global__ __launch_bounds__(256) void bn_bwd_partial_kernel(const E* __restrict__ x,
                                                             const E* __restrict__ dy, int P, int C, int ppb,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, int relu,
                                                             double* __restrict__ part,
                                                             const uint8_t* __restrict__ mask = nullptr,
                                                             E* __restrict__ gout = nullptr, FoldTail ft = FoldTail{},
                                                             int cgt_cap = 256) {
  using VT = VecT<V, E>;
  __shared__ double red[2][256][V];
  const RowGeom g = row_geom(C, V, cgt_cap);
  const int tid = threadIdx.x;
  const int cg = blockIdx.y * g.cgt + tid % g.cgt;
  const int pl = tid / g.cgt;
  const bool active = pl < g.PL && cg < g.CG;
  const int p0 = blockIdx.x * ppb, p1 = min(P, p0 + ppb);
  double s[V], q[V];
  float mu[V], is[V], ga[V], be[V];
  const int c0 = active ? cg * V : 0;
#pragma unroll
  for (int e = 0; e < V; ++e) {
    s[e] = q[e] = 0.0;
    mu[e] = mean[c0 + e];
    is[e] = invstd[c0 + e];
    ga[e] = gamma[c0 + e];
    be[e] = beta[c0 + e];
  }
  auto acc = [&](typename VT::T xv, typename VT::T gv) {
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const float xe = el(xv, e);
      float ge = el(gv, e);
      const float xh = (xe - mu[e]) * is[e];
      if (relu && !(bn_out(xe, mu[e], is[e], ga[e], be[e]) > 0.f)) ge = 0.f;
      s[e] += (double)ge;
      q[e] += (double)ge * (double)xh;
    }
  };
  if (active) {
    const int PL = g.PL;
    auto grad = [&](size_t off) -> typename VT::T {
      typename VT::T gv = VT::load(dy + off);
      if constexpr (MASKED) {
        if constexpr (V == 4) {
          // the 4 mask bytes of this float4 in one 32-bit load (off % 4 == 0 on the vector path)
          const uint32_t m4 = *reinterpret_cast<const uint32_t*>(mask + off);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (!((m4 >> (8 * e)) & 0xffu)) set_el(gv, e, 0.f);
        } else {
#pragma unroll
          for (int e = 0; e < V; ++e)
            if (!mask[off + e]) set_el(gv, e, 0.f);
        }
        VT::store(gout + off, gv);
      }
      return gv;
    };
    int p = p0 + pl;
    for (; p + 3 * PL < p1; p += 4 * PL) {
      typename VT::T xv[4], gv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t off = (size_t)(p + u * PL) * C + c0;
        xv[u] = VT::load(x + off);
        gv[u] = grad(off);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc(xv[u], gv[u]);
    }
    for (; p < p1; p += PL) {
      const size_t off = (size_t)p * C + c0;
      acc(VT::load(x + off), grad(off));
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    red[0][tid][e] = s[e];
    red[1][tid][e] = q[e];
  }
  __syncthreads();
  const int items = 2 * g.cgt * V;
  for (int it = tid; it < items; it += 256) {
    const int e = it % V;
    const int gg = (it / V) % g.cgt;
    const int which = it / (V * g.cgt);
    const int cgg = blockIdx.y * g.cgt + gg;
    if (cgg >= g.CG) continue;
    double a = 0.0;
    for (int qq = 0; qq < g.PL; ++qq) a += red[which][qq * g.cgt + gg][e];
    pub_store(part + ((size_t)blockIdx.x * 2 + which) * C + cgg * V + e, a);
  }
  if (ft.part) {
    const int c0 = blockIdx.y * g.cgt * V;
    fold_tail<256>(ft, blockIdx.x, c0, min(g.cgt * V, C - c0), blockIdx.y);
  }
}

// dgamma = sum dy_e * x_hat, dbeta = sum dy_e (batch_norm.py:159-174) from the *local*
// partials; k1 = mean(dy_e), k2 = sum(dy_e * x_hat) / count from the (possibly
// all-reduced, SyncBN) *global* partials.  Without SyncBN both are the same buffer.
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const double* __restrict__ part_l, int nblk_l,
                                                              const double* __restrict__ part_g, int nblk_g, int C,
                                                              double count, float* __restrict__ dgamma,
                                                              float* __restrict__ dbeta, float* __restrict__ k12) {
  const int c = blockIdx.x;
  double s, q;
  block_sum2(part_l, nblk_l, C, c, &s, &q);
  if (threadIdx.x == 0) {
    dgamma[c] = (float)q;
    dbeta[c] = (float)s;
  }
  if (part_g != part_l || nblk_g != nblk_l) {
    __syncthreads();
    block_sum2(part_g, nblk_g, C, c, &s, &q);
  }
  if (threadIdx.x == 0) {
    k12[c] = (float)(s / count);
    k12[C + c] = (float)(q / count);
  }
}

// dx = gamma * invstd * (dy_e - k1 - x_hat * k2)   (batch_norm.py:125-156, rearranged:
// (1/M) * X_demean / std^2 * sum(dy * X_demean) == x_hat * sum(dy * x_hat) / M)
template <int V, int U = 4, bool NT = false, class E = float>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const E* __restrict__ x, const E* __restrict__ dy,
                                                           int P, int C, int ppb, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, int relu,
                                                           const float* __restrict__ k12, E* __restrict__ dx) {
  using VT = VecT<V, E>;
  const RowGeom g = row_geom(C, V);
  const int tid = threadIdx.x;
  const int cg = blockIdx.y * g.cgt + tid % g.cgt;
  const int pl = tid / g.cgt;
  if (pl >= g.PL || cg >= g.CG) return;
  const int c0 = cg * V;
  float mu[V], is[V], ga[V], be[V], k1[V], k2[V], f[V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    mu[e] = mean[c0 + e];
    is[e] = invstd[c0 + e];
    ga[e] = gamma[c0 + e];
    be[e] = beta[c0 + e];
    k1[e] = k12[c0 + e];
    k2[e] = k12[C + c0 + e];
    f[e] = ga[e] * is[e];
  }
  auto one = [&](typename VT::T xv, typename VT::T gv, size_t off) {
    typename VT::T o;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const float xe = el(xv, e);
      float ge = el(gv, e);
      if (relu && !(bn_out(xe, mu[e], is[e], ga[e], be[e]) > 0.f)) ge = 0.f;
      set_el(o, e, bn_bwd_elem(xe, ge, mu[e], is[e], f[e], k1[e], k2[e]));
    }
    if constexpr (NT && V == 4 && sizeof(E) == 4)
      __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(dx + off));
    else
      VT::store(dx + off, o);
  };
  const int p0 = blockIdx.x * ppb, p1 = min(P, p0 + ppb);
  const int PL = g.PL;
  int p = p0 + pl;
  for (; p + (U - 1) * PL < p1; p += U * PL) {
    typename VT::T xv[U], gv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = (size_t)(p + u * PL) * C + c0;
      xv[u] = VT::load(x + off);
      gv[u] = VT::load(dy + off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(xv[u], gv[u], (size_t)(p + u * PL) * C + c0);
  }
  for (; p < p1; p += PL) {
    const size_t off = (size_t)p * C + c0;
    one(VT::load(x + off), VT::load(dy + off), off);
  }
}

// Inference parameters from running stats: mean = running_mean, invstd = 1 / running_std
// (batch_norm.py:101-115 divides by running_std).
__global__ void bn_infer_params_kernel(const float* __restrict__ run_std, int C, float* __restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) invstd[c] = 1.0f / run_std[c];
}

// Blocks for the reduce passes: ~32 row iterations per pixel lane, <= 1024 partials.
static int bn_blocks(int P, int C) {
  const int V = (C % 4 == 0) ? 4 : 1;
  const RowGeom g = row_geom(C, V);
  int nblk = cdiv(P, g.PL * 32);
  if (nblk > 1024) nblk = 1024;
  if (nblk < 1) nblk = 1;
  return nblk;
}

// Blocks for the streaming apply passes (no partials to keep small): up to 4096.
// Launch variant of dk_bn_bwd_apply_f32 (dk_debug_set_ew_variant).  Default 22 = rows in
// flight 4, nontemporal dx stores, 8 rows per pixel lane, up to 16384 blocks: measured
// best or within 1 % of best on every ResNet BatchNorm shape (scripts/ew_tune.py; -10 % on
// res1/res3 vs the row-loop defaults of the other BN passes).

static int bn_apply_blocks(int P, int C, int V) {
  const RowGeom g = row_geom(C, V);
  int nblk = cdiv(P, g.PL * 16);
  if (nblk > 4096) nblk = 4096;
  if (nblk < 1) nblk = 1;
  return nblk;
}

static inline bool vec_ok(const void* p, int C) { return (C % 4 == 0) && ((reinterpret_cast<uintptr_t>(p) & 15) == 0); }
// 4-element (float4 / 4 x bf16) access allowed for this storage type
template <class E>
static inline bool vec_ok_e(const E* p, int C) {
  return (C % 4 == 0) && ((reinterpret_cast<uintptr_t>(p) & (4 * sizeof(E) - 1)) == 0);
}

}  // namespace dk

using namespace dk;

DK_API int dk_bn_partial_blocks(int P, int C) { return bn_blocks(P, C); }

DK_API size_t dk_bn_workspace_bytes(int P, int C) { return (size_t)bn_blocks(P, C) * 2 * C * sizeof(double); }
static size_t bn_fold_offset(int P, int C) { return (size_t)bn_blocks(P, C) * 2 * C * sizeof(double); }

// Stage 1 of forward statistics: part[nblk][2][C] (fp64 sum x, sum x^2) over x[P][C].
template <class E>
static int bn_stats_partial_t(const E* x, int P, int C, void* ws, size_t ws_bytes, void* stream) {
  if (ws_bytes < dk_bn_workspace_bytes(P, C)) return DK_ERR_WORKSPACE;
  const int nblk = bn_blocks(P, C);
  const int ppb = cdiv(P, nblk);
  const bool vec = vec_ok_e(x, C);
  if (!vec && sizeof(E) != 4) return DK_ERR_ARGS;
  const RowGeom g = row_geom(C, vec ? 4 : 1);
  const dim3 grid(nblk, cdiv(g.CG, g.cgt));
  if (vec)
    hipLaunchKernelGGL((bn_stats_partial_kernel<4, E>), grid, dim3(256), 0, as_stream(stream), x, P, C, ppb,
                       static_cast<double*>(ws));
  else
    hipLaunchKernelGGL((bn_stats_partial_kernel<1, E>), grid, dim3(256), 0, as_stream(stream), x, P, C, ppb,
                       static_cast<double*>(ws));
  return launch_status();
}
DK_API int dk_bn_stats_partial_f64(const float* x, int P, int C, void* ws, size_t ws_bytes, void* stream) {
  return bn_stats_partial_t(x, P, C, ws, ws_bytes, stream);
}

// out[2][C] = fixed-order sum of part[nblk][2][C].
DK_API int dk_bn_collapse_f64(const void* part, int nblk, int C, void* out, void* stream) {
  hipLaunchKernelGGL(bn_collapse_kernel, dim3(C), dim3(256), 0, as_stream(stream), static_cast<const double*>(part),
                     nblk, C, static_cast<double*>(out));
  return launch_status();
}

// Stage 2: mean, population variance, std = sqrt(var + eps), invstd; running stats.
DK_API int dk_bn_stats_finalize_f32(const void* part, int nblk, int C, double count, float eps, float momentum,
                                    int first, float* mean, float* std_, float* invstd, float* run_mean,
                                    float* run_std, void* stream) {
  hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3(C), dim3(256), 0, as_stream(stream),
                     static_cast<const double*>(part), nblk, C, count, eps, momentum, first, mean, std_, invstd,
                     run_mean, run_std);
  return launch_status();
}

// Forward statistics (both stages).  x is [P][C] (NHWC with P = N*H*W, or [rows][features]).
template <class E>
static int bn_stats_t(const E* x, int P, int C, float eps, float momentum, int first, float* mean, float* std_,
                      float* invstd, float* run_mean, float* run_std, void* ws, size_t ws_bytes, void* stream) {
  const int nblk = bn_blocks(P, C);
  if (ws_bytes < bn_fold_offset(P, C) + dk_bn_partials_workspace_bytes(nblk, C)) return DK_ERR_WORKSPACE;
  int rc = bn_stats_partial_t(x, P, C, ws, ws_bytes, stream);
  if (rc) return rc;
  return dk_bn_stats_from_partials_f32(ws, nblk, C, (double)P, eps, momentum, first, mean, std_, invstd, run_mean,
                                       run_std, static_cast<char*>(ws) + bn_fold_offset(P, C),
                                       ws_bytes - bn_fold_offset(P, C), nullptr, stream);
}
DK_API int dk_bn_stats_f32(const float* x, int P, int C, float eps, float momentum, int first, float* mean,
                           float* std_, float* invstd, float* run_mean, float* run_std, void* ws, size_t ws_bytes,
                           void* stream) {
  return bn_stats_t(x, P, C, eps, momentum, first, mean, std_, invstd, run_mean, run_std, ws, ws_bytes, stream);
}
DK_API int dk_bn_stats_bf16(const bf16_t* x, int P, int C, float eps, float momentum, int first, float* mean,
                            float* std_, float* invstd, float* run_mean, float* run_std, void* ws, size_t ws_bytes,
                            void* stream) {
  return bn_stats_t(x, P, C, eps, momentum, first, mean, std_, invstd, run_mean, run_std, ws, ws_bytes, stream);
}

// Workspace of dk_bn_stats_f32: the partials plus their fold rows.
DK_API size_t dk_bn_stats_workspace_bytes(int P, int C) {
  return bn_fold_offset(P, C) + dk_bn_partials_workspace_bytes(bn_blocks(P, C), C);
}

// Statistics from partial sums written by a producer's epilogue (*_fwd_ex_f32): part[nblk][2][C].
DK_API size_t dk_bn_partials_workspace_bytes(int nblk, int C) {
  // fold levels: ceil(n / 256) rows each, until one block finishes
  size_t rows = 0;
  for (int n = nblk; n > kFoldRows; n = cdiv(n, kFoldRows)) rows += (size_t)cdiv(n, kFoldRows);
  return (rows > 0 ? rows : 1) * 2 * C * sizeof(double);
}

// Tuning knob (not thread-safe): launch variant of dk_bn_bwd_apply_f32 (-1 = built-in).
DK_API int dk_debug_set_ew_variant(int v) {
  knob_set(kKnobEwVariant, v);
  return 32;
}

DK_API int dk_bn_fold_tickets_count(int C) { return C < 1 ? 0 : cdiv(C, 64); }

// ---- in-launch folds (fold_tail.h): the arming of one partials buffer at a time per thread ----
namespace {
struct Armed {
  const void* part = nullptr;
  int nrows = 0, C = 0;
  FoldOut o{};
  unsigned* tickets = nullptr;
  int ntickets = 0;
  double* scratch = nullptr;
  size_t scratch_bytes = 0;
};
thread_local Armed g_armed;

int fold_group_rows(int nrows) {
  int g = 1;
  while ((long long)g * g < nrows) ++g;  // ceil(sqrt(nrows)): balances the two levels
  return g;
}
}  // namespace

bool dk::fold_take(const void* part, int nrows, int C, int nslices, FoldTail* ft) {
  ft->part = nullptr;
  Armed& a = g_armed;
  if (!part || a.part != part) return false;
  a.part = nullptr;  // one launch takes it
  if (a.nrows != nrows || a.C != C || C % 2 || nslices < 1 || nrows < 1) return false;
  const int G = fold_group_rows(nrows);
  const int ng = cdiv(nrows, G);
  if ((long long)ng * nslices + nslices > a.ntickets) return false;
  if ((size_t)ng * 2 * C * sizeof(double) > a.scratch_bytes) return false;
  ft->o = a.o;
  ft->part = static_cast<const double*>(part);
  ft->grp = a.scratch;
  ft->tickets = a.tickets;
  ft->nrows = nrows;
  ft->C = C;
  ft->G = G;
  ft->ngroups = ng;
  ft->nslices = nslices;
  return true;
}

int dk::fold_status(int rc, const FoldTail& ft) { return rc == 0 && ft.part ? DK_FOLDED : rc; }

static int fold_arm(const void* part, int nrows, int C, const FoldOut& o, unsigned* tickets, int ntickets,
                    void* scratch, size_t scratch_bytes) {
  if (!part || nrows < 1 || C < 1 || !tickets || ntickets < 2 || !scratch) return DK_ERR_ARGS;
  Armed& a = g_armed;
  a.part = part;
  a.nrows = nrows;
  a.C = C;
  a.o = o;
  a.tickets = tickets;
  a.ntickets = ntickets;
  a.scratch = static_cast<double*>(scratch);
  a.scratch_bytes = scratch_bytes;
  return 0;
}

DK_API int dk_bn_fold_arm_stats(const void* part, int nrows, int C, double count, float eps, float momentum,
                                int first, float* mean, float* std_, float* invstd, float* run_mean, float* run_std,
                                unsigned* tickets, int ntickets, void* scratch, size_t scratch_bytes) {
  FoldOut o{};
  o.mode = 0;
  o.count = count;
  o.eps = eps;
  o.momentum = momentum;
  o.first = first;
  o.mean = mean;
  o.std_ = std_;
  o.invstd = invstd;
  o.run_mean = run_mean;
  o.run_std = run_std;
  if (!mean || !std_ || !invstd) return DK_ERR_ARGS;
  return fold_arm(part, nrows, C, o, tickets, ntickets, scratch, scratch_bytes);
}

DK_API int dk_bn_fold_arm_bwd(const void* part, int nrows, int C, double count, float* dgamma, float* dbeta,
                              float* k12, unsigned* tickets, int ntickets, void* scratch, size_t scratch_bytes) {
  FoldOut o{};
  o.mode = 1;
  o.count = count;
  o.dgamma = dgamma;
  o.dbeta = dbeta;
  o.k12 = k12;
  if (!dgamma || !dbeta || !k12) return DK_ERR_ARGS;
  return fold_arm(part, nrows, C, o, tickets, ntickets, scratch, scratch_bytes);
}

DK_API int dk_bn_fold_disarm(void) {
  g_armed.part = nullptr;
  return 0;
}

// Scratch bytes / ticket words an in-launch fold of nrows x C in nslices slices needs.
DK_API size_t dk_bn_fold_scratch_bytes(int nrows, int C) {
  if (nrows < 1 || C < 1) return 0;
  return (size_t)cdiv(nrows, fold_group_rows(nrows)) * 2 * C * sizeof(double);
}
DK_API int dk_bn_fold_tickets_needed_count(int nrows, int nslices) {
  if (nrows < 1 || nslices < 1) return 0;
  return cdiv(nrows, fold_group_rows(nrows)) * nslices + nslices;
}

// Fold part[nblk][2][C] (fixed order) and apply the stage-2 maths: one launch for <= 256 rows,
// and with `tickets` (>= cdiv(C, 64) zeroed words) one launch for <= 256 * 256 rows.
static int fold_finalize(const double* part, int nblk, int C, double* ws, const FoldOut& o, hipStream_t st,
                         unsigned* tickets = nullptr) {
  const unsigned gy = (unsigned)cdiv(C, 64);
  if (tickets && nblk > kFoldRows && nblk <= kFoldRows * kFoldRows) {
    hipLaunchKernelGGL(bn_fold_kernel<2>, dim3(cdiv(nblk, kFoldRows), gy), dim3(1024), 0, st, part, nblk, C, ws, o,
                       tickets);
    return launch_status();
  }
  while (nblk > kFoldRows) {
    const int n2 = cdiv(nblk, kFoldRows);
    hipLaunchKernelGGL(bn_fold_kernel<0>, dim3(n2, gy), dim3(1024), 0, st, part, nblk, C, ws, o, nullptr);
    part = ws;
    ws += (size_t)n2 * 2 * C;
    nblk = n2;
  }
  hipLaunchKernelGGL(bn_fold_kernel<1>, dim3(1, gy), dim3(1024), 0, st, part, nblk, C, nullptr, o, nullptr);
  return launch_status();
}

DK_API int dk_bn_stats_from_partials_f32(const void* part, int nblk, int C, double count, float eps, float momentum,
                                         int first, float* mean, float* std_, float* invstd, float* run_mean,
                                         float* run_std, void* ws, size_t ws_bytes, unsigned* tickets,
                                         void* stream) {
  if (ws_bytes < dk_bn_partials_workspace_bytes(nblk, C) || nblk < 1) return DK_ERR_WORKSPACE;
  FoldOut o{};
  o.mode = 0;
  o.count = count;
  o.eps = eps;
  o.momentum = momentum;
  o.first = first;
  o.mean = mean;
  o.std_ = std_;
  o.invstd = invstd;
  o.run_mean = run_mean;
  o.run_std = run_std;
  return fold_finalize(static_cast<const double*>(part), nblk, C, static_cast<double*>(ws), o, as_stream(stream),
                       tickets);
}

// out[2][C] = the column sums of part[nblk][2][C] (SyncBN: the vector each rank all-reduces).
DK_API int dk_bn_reduce_partials_f64(const void* part, int nblk, int C, void* out, void* ws, size_t ws_bytes,
                                     void* stream) {
  if (ws_bytes < dk_bn_partials_workspace_bytes(nblk, C) || nblk < 1) return DK_ERR_WORKSPACE;
  FoldOut o{};
  o.mode = 2;
  o.sums = static_cast<double*>(out);
  return fold_finalize(static_cast<const double*>(part), nblk, C, static_cast<double*>(ws), o, as_stream(stream));
}

DK_API int dk_bn_infer_params_f32(const float* run_std, int C, float* invstd, void* stream) {
  hipLaunchKernelGGL(bn_infer_params_kernel, dim3(cdiv(C, 256)), dim3(256), 0, as_stream(stream), run_std, C, invstd);
  return launch_status();
}

// y = gamma * (x - mean) * invstd + beta  [+ ReLU; mask (uint8) may be null]
template <class E>
static int bn_apply_t(const E* x, long long numel, int C, const float* mean, const float* invstd, const float* gamma,
                      const float* beta, int relu, E* y, uint8_t* mask, void* stream) {
  const int P = (int)(numel / C);
  const bool vec = vec_ok_e(x, C) && vec_ok_e(y, C);
  if (!vec && sizeof(E) != 4) return DK_ERR_ARGS;
  const int V = vec ? 4 : 1;
  const RowGeom g = row_geom(C, V);
  const int nblk = bn_apply_blocks(P, C, V);
  const dim3 grid(nblk, cdiv(g.CG, g.cgt));
  const int ppb = cdiv(P, nblk);
  if (vec)
    hipLaunchKernelGGL((bn_apply_kernel<4, E>), grid, dim3(256), 0, as_stream(stream), x, P, C, ppb, mean, invstd,
                       gamma, beta, relu, y, mask);
  else
    hipLaunchKernelGGL((bn_apply_kernel<1, E>), grid, dim3(256), 0, as_stream(stream), x, P, C, ppb, mean, invstd,
                       gamma, beta, relu, y, mask);
  return launch_status();
}
DK_API int dk_bn_apply_f32(const float* x, long long numel, int C, const float* mean, const float* invstd,
                           const float* gamma, const float* beta, int relu, float* y, uint8_t* mask, void* stream) {
  return bn_apply_t(x, numel, C, mean, invstd, gamma, beta, relu, y, mask, stream);
}
DK_API int dk_bn_apply_bf16(const bf16_t* x, long long numel, int C, const float* mean, const float* invstd,
                            const float* gamma, const float* beta, int relu, bf16_t* y, uint8_t* mask, void* stream) {
  return bn_apply_t(x, numel, C, mean, invstd, gamma, beta, relu, y, mask, stream);
}

// Backward stage 1: part[nblk][2][C] = (sum dy_e, sum dy_e * x_hat); relu != 0 fuses the
// following ReLU's backward (its mask is recomputed from x).
template <class E>
static int bn_bwd_partial_t(const E* x, const E* dy, int P, int C, const float* mean, const float* invstd,
                            const float* gamma, const float* beta, int relu, void* ws, size_t ws_bytes, void* stream) {
  if (ws_bytes < dk_bn_workspace_bytes(P, C)) return DK_ERR_WORKSPACE;
  const int nblk = bn_blocks(P, C);
  const int ppb = cdiv(P, nblk);
  const bool vec = vec_ok_e(x, C) && vec_ok_e(dy, C);
  if (!vec && sizeof(E) != 4) return DK_ERR_ARGS;
  const RowGeom g = row_geom(C, vec ? 4 : 1);
  const dim3 grid(nblk, cdiv(g.CG, g.cgt));
  if (vec)
    hipLaunchKernelGGL((bn_bwd_partial_kernel<4, false, E>), grid, dim3(256), 0, as_stream(stream), x, dy, P, C, ppb,
                       mean, invstd, gamma, beta, relu, static_cast<double*>(ws), nullptr, nullptr);
  else
    hipLaunchKernelGGL((bn_bwd_partial_kernel<1, false, E>), grid, dim3(256), 0, as_stream(stream), x, dy, P, C, ppb,
                       mean, invstd, gamma, beta, relu, static_cast<double*>(ws), nullptr, nullptr);
  return launch_status();
}
DK_API int dk_bn_bwd_partial_f64(const float* x, const float* dy, int P, int C, const float* mean,
                                 const float* invstd, const float* gamma, const float* beta, int relu, void* ws,
                                 size_t ws_bytes, void* stream) {
  return bn_bwd_partial_t(x, dy, P, C, mean, invstd, gamma, beta, relu, ws, ws_bytes, stream);
}

// ReLU backward (mask from the forward join) fused with stage 1 of the backward of the BN
// that produced the join's input: dx = mask ? dy : 0 and part[nblk][2][C] over dx.
DK_API int dk_relu_bwd_bn_partial_f64(const float* dy, const uint8_t* mask, const float* x, int P, int C,
                                      const float* mean, const float* invstd, const float* gamma, const float* beta,
                                      int relu, float* dx, void* part, size_t part_bytes, void* stream) {
  if (part_bytes < dk_bn_workspace_bytes(P, C)) return DK_ERR_WORKSPACE;
  const int nblk = bn_blocks(P, C);
  const int ppb = cdiv(P, nblk);
  const bool vec = vec_ok(x, C) && vec_ok(dy, C) && vec_ok(dx, C) && (reinterpret_cast<uintptr_t>(mask) & 3) == 0;
  // the same partial rows (pixel ranges) as the other BN passes, but at most 32 channel groups per block:
  // the head's 7 x 7 x 512 join (P = 12,544) otherwise ran 196 blocks of 2 pixel lanes, one per CU
  // on 196 CUs, each lane walking 32 pixels
  const int cap = 32;
  const RowGeom g = row_geom(C, vec ? 4 : 1, cap);
  const dim3 grid(nblk, cdiv(g.CG, g.cgt));
  FoldTail ft;  // an armed in-launch fold of the partial rows (fold_tail.h)
  if (!fold_take(part, nblk, C, (int)grid.y, &ft) || ((g.cgt * (vec ? 4 : 1)) & 1)) ft.part = nullptr;
  if (vec)
    hipLaunchKernelGGL((bn_bwd_partial_kernel<4, true>), grid, dim3(256), 0, as_stream(stream), x, dy, P, C, ppb,
                       mean, invstd, gamma, beta, relu, static_cast<double*>(part), mask, dx, ft, cap);
  else
    hipLaunchKernelGGL((bn_bwd_partial_kernel<1, true>), grid, dim3(256), 0, as_stream(stream), x, dy, P, C, ppb,
                       mean, invstd, gamma, beta, relu, static_cast<double*>(part), mask, dx, ft, cap);
  return fold_status(launch_status(), ft);
}

// Backward stage 2 from partials of any origin (dk_bn_bwd_partial_f64, a consumer's
// dgrad_ex epilogue, dk_relu_bwd_bn_partial_f64): fixed-order fold, then the finalize.
DK_API int dk_bn_bwd_from_partials_f32(const void* part, int nblk, int C, double count, float* dgamma, float* dbeta,
                                       float* k12, void* ws, size_t ws_bytes, unsigned* tickets, void* stream) {
  if (ws_bytes < dk_bn_partials_workspace_bytes(nblk, C) || nblk < 1) return DK_ERR_WORKSPACE;
  FoldOut o{};
  o.mode = 1;
  o.count = count;
  o.dgamma = dgamma;
  o.dbeta = dbeta;
  o.k12 = k12;
  return fold_finalize(static_cast<const double*>(part), nblk, C, static_cast<double*>(ws), o, as_stream(stream),
                       tickets);
}

// Backward stage 2: dgamma/dbeta from the local partials, k12 = [k1[C], k2[C]] from the global ones.
DK_API int dk_bn_bwd_finalize_f32(const void* part_local, int nblk_local, const void* part_global, int nblk_global,
                                  int C, double count, float* dgamma, float* dbeta, float* k12, void* stream) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(256), 0, as_stream(stream),
                     static_cast<const double*>(part_local), nblk_local, static_cast<const double*>(part_global),
                     nblk_global, C, count, dgamma, dbeta, k12);
  return launch_status();
}

// Backward stage 3: dx = gamma * invstd * (dy_e - k1 - x_hat * k2).
template <class E>
static int bn_bwd_apply_t(const E* x, const E* dy, long long numel, int C, const float* mean, const float* invstd,
                          const float* gamma, const float* beta, int relu, const float* k12, E* dx, void* stream) {
  const int P = (int)(numel / C);
  const bool vec = vec_ok_e(x, C) && vec_ok_e(dy, C) && vec_ok_e(dx, C);
  if (!vec && sizeof(E) != 4) return DK_ERR_ARGS;
  const int V = vec ? 4 : 1;
  const RowGeom g = row_geom(C, V);
  const int var = knob(kKnobEwVariant);
  int nblk = bn_apply_blocks(P, C, V);
  if (var >= 0) {  // tuning knob: rows per pixel lane 16 / 8 / 32 / 64, cap 4096 / 16384
    const int rpl[4] = {16, 8, 32, 64};
    nblk = cdiv(P, g.PL * rpl[(var >> 2) & 3]);
    const int cap = (var & 16) ? 16384 : 4096;
    nblk = nblk < 1 ? 1 : (nblk > cap ? cap : nblk);
  }
  const dim3 grid(nblk, cdiv(g.CG, g.cgt));
  const int ppb = cdiv(P, nblk);
  if (vec && var >= 0) {
#define BBA(U_, NT_)                                                                                              \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<4, U_, NT_, E>), grid, dim3(256), 0, as_stream(stream), x, dy, P, C, ppb,   \
                     mean, \
                     invstd, gamma, beta, relu, k12, dx)
    switch (var & 3) {
      case 0: BBA(4, false); break;
      case 1: BBA(8, false); break;
      case 2: BBA(4, true); break;
      default: BBA(8, true); break;
    }
#undef BBA
  } else if (vec && nt_stores(kNtBnBwd))
    hipLaunchKernelGGL((bn_bwd_apply_kernel<4, 4, true, E>), grid, dim3(256), 0, as_stream(stream), x, dy, P, C, ppb,
                       mean, invstd, gamma, beta, relu, k12, dx);
  else if (vec)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<4, 4, false, E>), grid, dim3(256), 0, as_stream(stream), x, dy, P, C, ppb,
                       mean, invstd, gamma, beta, relu, k12, dx);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<1, 4, false, E>), grid, dim3(256), 0, as_stream(stream), x, dy, P, C, ppb,
                       mean, invstd, gamma, beta, relu, k12, dx);
  return launch_status();
}
DK_API int dk_bn_bwd_apply_f32(const float* x, const float* dy, long long numel, int C, const float* mean,
                               const float* invstd, const float* gamma, const float* beta, int relu,
                               const float* k12, float* dx, void* stream) {
  return bn_bwd_apply_t(x, dy, numel, C, mean, invstd, gamma, beta, relu, k12, dx, stream);
}
DK_API int dk_bn_bwd_apply_bf16(const bf16_t* x, const bf16_t* dy, long long numel, int C, const float* mean,
                                const float* invstd, const float* gamma, const float* beta, int relu,
                                const float* k12, bf16_t* dx, void* stream) {
  return bn_bwd_apply_t(x, dy, numel, C, mean, invstd, gamma, beta, relu, k12, dx, stream);
}

DK_API size_t dk_bn_bwd_workspace_bytes(int P, int C) {
  return bn_fold_offset(P, C) + 2 * (size_t)C * sizeof(float) + dk_bn_partials_workspace_bytes(bn_blocks(P, C), C);
}

// Backward (all stages, local statistics).  Writes dgamma/dbeta [C] and dx [P][C].
template <class E>
static int bn_bwd_t(const E* x, const E* dy, int P, int C, const float* mean, const float* invstd, const float* gamma,
                    const float* beta, int relu, float* dgamma, float* dbeta, E* dx, void* ws, size_t ws_bytes,
                    void* stream) {
  if (ws_bytes < dk_bn_bwd_workspace_bytes(P, C)) return DK_ERR_WORKSPACE;
  const int nblk = bn_blocks(P, C);
  char* base = static_cast<char*>(ws);
  float* k12 = reinterpret_cast<float*>(base + bn_fold_offset(P, C));
  const size_t fold_off = bn_fold_offset(P, C) + 2 * (size_t)C * sizeof(float);
  int rc = bn_bwd_partial_t(x, dy, P, C, mean, invstd, gamma, beta, relu, ws, ws_bytes, stream);
  if (rc) return rc;
  rc = dk_bn_bwd_from_partials_f32(ws, nblk, C, (double)P, dgamma, dbeta, k12, base + fold_off, ws_bytes - fold_off,
                                   nullptr, stream);
  if (rc) return rc;
  return bn_bwd_apply_t(x, dy, (long long)P * C, C, mean, invstd, gamma, beta, relu, k12, dx, stream);
}
DK_API int dk_bn_bwd_f32(const float* x, const float* dy, int P, int C, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, int relu, float* dgamma, float* dbeta, float* dx,
                         void* ws, size_t ws_bytes, void* stream) {
  return bn_bwd_t(x, dy, P, C, mean, invstd, gamma, beta, relu, dgamma, dbeta, dx, ws, ws_bytes, stream);
}
DK_API int dk_bn_bwd_bf16(const bf16_t* x, const bf16_t* dy, int P, int C, const float* mean, const float* invstd,
                          const float* gamma, const float* beta, int relu, float* dgamma, float* dbeta, bf16_t* dx,
                          void* ws, size_t ws_bytes, void* stream) {
  return bn_bwd_t(x, dy, P, C, mean, invstd, gamma, beta, relu, dgamma, dbeta, dx, ws, ws_bytes, stream);
}
