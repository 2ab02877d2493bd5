// Elementwise / small-reduction kernels around the convolution hot path, gfx950.
//   ReLU fwd/bwd ............ layers/activations.py:14-47 (mask kept as uint8, not fp32)
//   residual add (+ReLU) ..... layers/residual_block.py:65-97
//   global average pool ...... layers/pooling.py:23-36
//   softmax + cross-entropy .. layers/losses.py:13-34 (no max shift, as the reference)
//   SGD momentum (multi-tensor, one launch) ... optimisers/SGDMomentum.py:31-39
//   l2 loss term ............. regularisers/l2.py:12-14
//   bias gradients (column sums), NCHW -> NHWC(+channel pad) layout conversion
#include "dk_common.h"

namespace dk {

// Vectorised elementwise kernels: each thread handles float4 chunks (grid-stride), the
// uint8 masks as one 32-bit word per chunk; a scalar tail handles n % 4.
template <class E = float>  // E: activation storage (float or bf16_t)
__global__ __launch_bounds__(256) void relu_fwd_kernel(const E* __restrict__ x, long long n, E* __restrict__ y,
                                                       uint8_t* __restrict__ mask, int vec) {
  const long long nv = vec ? (n >> 2) : 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    f32x4 v = ld4(x + 4 * i);
    uint32_t m = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool pos = v[e] > 0.f;
      v[e] = pos ? v[e] : 0.f;
      m |= (uint32_t)pos << (8 * e);
    }
    if (y) st4(y + 4 * i, v);  // (y == NULL: the mask only)
    if (mask) reinterpret_cast<uint32_t*>(mask)[i] = m;
  }
  for (long long i = 4 * nv + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = ld1(x + i);
    const bool pos = v > 0.f;
    if (y) st1(y + i, pos ? v : 0.f);
    if (mask) mask[i] = pos;
  }
}

template <class E = float>
__global__ __launch_bounds__(256) void relu_bwd_kernel(const E* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                       long long n, E* __restrict__ dx, int vec) {
  const long long nv = vec ? (n >> 2) : 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    f32x4 g = ld4(dy + 4 * i);
    const uint32_t m = reinterpret_cast<const uint32_t*>(mask)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) g[e] = ((m >> (8 * e)) & 0xff) ? g[e] : 0.f;
    st4(dx + 4 * i, g);
  }
  for (long long i = 4 * nv + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    st1(dx + i, mask[i] ? ld1(dy + i) : 0.f);
}

__global__ void mask_to_f32_kernel(const uint8_t* __restrict__ mask, long long n, float* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = mask[i] ? 1.f : 0.f;
}

// y = a + b, optionally ReLU'd with mask.
__global__ __launch_bounds__(256) void add_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                  long long n, int relu, float* __restrict__ y,
                                                  uint8_t* __restrict__ mask, int vec) {
  const long long nv = vec ? (n >> 2) : 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    f32x4 v = ld4(a + 4 * i) + ld4(b + 4 * i);
    if (relu) {
      uint32_t m = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool pos = v[e] > 0.f;
        v[e] = pos ? v[e] : 0.f;
        m |= (uint32_t)pos << (8 * e);
      }
      if (mask) reinterpret_cast<uint32_t*>(mask)[i] = m;
    }
    st4(y + 4 * i, v);
  }
  for (long long i = 4 * nv + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float v = a[i] + b[i];
    if (relu) {
      const bool pos = v > 0.f;
      v = pos ? v : 0.f;
      if (mask) mask[i] = pos;
    }
    y[i] = v;
  }
}

// Residual join with the BatchNorm(s) of its inputs applied on load:
// y = [ReLU](bnA(a) + bnB(b)), bnX = identity when its mean is null.  Element i has channel
// i % C (NHWC rows).  Bit-identical to dk_bn_apply_f32 on each input followed by dk_add_f32.
__device__ __forceinline__ f32x4 bn_in4_at(f32x4 v, const BnIn& bn, int c) {
  if (!bn.mean) return v;
  return bn_in4(v, ld4(bn.mean + c), ld4(bn.invstd + c), ld4(bn.gamma + c), ld4(bn.beta + c), bn.relu);
}

__global__ __launch_bounds__(256) void bn_add_kernel(const float* __restrict__ a, BnIn ba, const float* __restrict__ b,
                                                     BnIn bb, long long n, int C, int relu, float* __restrict__ y,
                                                     uint8_t* __restrict__ mask, int nt) {
  const long long nv = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    const int c = (int)((uint32_t)(4 * i) % (uint32_t)C);
    f32x4 v = bn_in4_at(ld4(a + 4 * i), ba, c) + bn_in4_at(ld4(b + 4 * i), bb, c);
    if (relu) {
      uint32_t m = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool pos = v[e] > 0.f;
        v[e] = pos ? v[e] : 0.f;
        m |= (uint32_t)pos << (8 * e);
      }
      if (mask) reinterpret_cast<uint32_t*>(mask)[i] = m;
    }
    if (nt)
      st4nt(y + 4 * i, v);
    else
      st4(y + 4 * i, v);
  }
}

// out[n][c] = mean_{hw} x[n][hw][c]
// (the HW loads of a channel are issued eight at a time and added in order: the sum, and so the
// result, is the one-at-a-time loop's; issued one by one they left the kernel latency-bound)
__global__ void gap_fwd_kernel(const float* __restrict__ x, int N, int HW, int C, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i - n * C;
  const float* p = x + (size_t)n * HW * C + c;
  float s = 0.f;
  int k = 0;
  for (; k + 8 <= HW; k += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(size_t)(k + u) * C];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; k < HW; ++k) s += p[(size_t)k * C];
  out[i] = s / (float)HW;
}

// The pooling of the network's last residual join (the head: y = ReLU(bnA(a) + bnB(b)),
// residual_block.py:75, is read only by the global average pooling, pooling.py:23-30):
// out[n][c] = mean_hw y, every y formed as bn_add_kernel forms it (bn_relu_out of each operand, one
// add, the (v > 0) ? v : 0 ReLU) and summed in gap_fwd_kernel's order (loads eight at a time, added
// one by one) -- bit-identical to the join pass followed by dk_gap_fwd_f32 -- with y never stored:
// only its ReLU mask (the join's backward, activations.py:44-47), when given.
__global__ __launch_bounds__(256) void gap_join_kernel(const float* __restrict__ a, BnIn ba, const float* __restrict__ b,
                                                       BnIn bb, int N, int HW, int C, uint8_t* __restrict__ mask,
                                                       float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i - n * C;
  const float am = ba.mean ? ba.mean[c] : 0.f, ai = ba.mean ? ba.invstd[c] : 0.f;
  const float ag = ba.mean ? ba.gamma[c] : 0.f, abt = ba.mean ? ba.beta[c] : 0.f;
  const float bm = bb.mean ? bb.mean[c] : 0.f, bi = bb.mean ? bb.invstd[c] : 0.f;
  const float bg = bb.mean ? bb.gamma[c] : 0.f, bbt = bb.mean ? bb.beta[c] : 0.f;
  const size_t base = (size_t)n * HW * C + c;
  auto join = [&](float av, float bv, int k) {
    const float va = ba.mean ? bn_relu_out(av, am, ai, ag, abt, ba.relu) : av;
    const float vb = bb.mean ? bn_relu_out(bv, bm, bi, bg, bbt, bb.relu) : bv;
    float v = va + vb;
    const bool pos = v > 0.f;
    v = pos ? v : 0.f;
    if (mask) mask[base + (size_t)k * C] = (uint8_t)pos;
    return v;
  };
  float s = 0.f;
  int k = 0;
  for (; k + 8 <= HW; k += 8) {
    float va[8], vb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      va[u] = a[base + (size_t)(k + u) * C];
      vb[u] = b[base + (size_t)(k + u) * C];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += join(va[u], vb[u], k + u);
  }
  for (; k < HW; ++k) s += join(a[base + (size_t)k * C], b[base + (size_t)k * C], k);
  out[i] = s / (float)HW;
}

// dx[n][hw][c] = (1/HW) * dy[n][c]; gap_bwd4_kernel: four channels per thread (C % 4 == 0, 16-byte aligned)
__global__ void gap_bwd_kernel(const float* __restrict__ dy, int N, int HW, int C, float* __restrict__ dx) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)N * HW * C;
  if (i >= total) return;
  const int c = (int)(i % C);
  const int n = (int)(i / ((long long)HW * C));
  dx[i] = (1.0f / (float)HW) * dy[(size_t)n * C + c];
}
__global__ void gap_bwd4_kernel(const float* __restrict__ dy, int N, int HW, int C, float* __restrict__ dx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // float4 index; N * HW * C < 2^31 (checked)
  const int C4 = C >> 2;
  if (i >= N * HW * C4) return;
  const int c4 = i % C4;
  const int n = i / (HW * C4);
  const f32x4 g = ld4(dy + (size_t)n * C + 4 * c4);
  const float f = 1.0f / (float)HW;
  st4(dx + (size_t)i * 4, f32x4{f * g[0], f * g[1], f * g[2], f * g[3]});
}

// p = e^x / sum e^x per row (no max subtraction, losses.py:15-16);
// loss = mean_b -log(sum_j p[b][j] * y[b][j])  (losses.py:23-26).  One block.
template <bool V4>
__global__ __launch_bounds__(1024) void softmax_xent_fwd_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ y, int B, int K,
                                                                float* __restrict__ p, float* __restrict__ loss) {
  // K <= 128 (every model here): four lanes per row, 256 rows per pass; a lane holds the row's columns
  // part, part + 4, ... (all its loads issued at once), the four lane sums combined by two quad
  // exchanges (the same value in every lane of the quad).  The row losses go through LDS and wave 0
  // adds them in a fixed order (rows past B are 0).
  // K > 128: one wave per row (rows w, w + 16, ...), per-wave fp64 sums combined in a fixed order.
  __shared__ double red[16];
  __shared__ double rl[256];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double acc = 0.0;
  if (K <= 128) {
    // lane `part` of a row's quad holds the row's float4 columns part, part + 4, ... (K % 4 == 0 and
    // 16-byte rows: V4, one load per 4 columns -- the block's memory requests, all through one CU,
    // were this kernel's time), else its scalar columns part, part + 4, ...
    constexpr int KPT = 32;
    const int part = threadIdx.x & 3, r = threadIdx.x >> 2;
    auto col = [&](int j) { return V4 ? 4 * (part + 4 * (j >> 2)) + (j & 3) : part + 4 * j; };
    for (int b0 = 0; b0 < B; b0 += 256) {
      const int b = b0 + r;
      const bool live = b < B;
      float e[KPT], yv[KPT];
      if constexpr (V4) {
#pragma unroll
        for (int i = 0; i < KPT / 4; ++i) {
          const int k = 4 * (part + 4 * i);
          const bool in = live && k < K;
          const f32x4 xv = in ? ld4(x + (size_t)b * K + k) : f32x4{0.f, 0.f, 0.f, 0.f};
          const f32x4 yq = in && y ? ld4(y + (size_t)b * K + k) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            e[4 * i + u] = xv[u];
            yv[4 * i + u] = yq[u];
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
          const int k = col(j);
          const bool in = live && k < K;
          e[j] = in ? x[(size_t)b * K + k] : 0.f;
          yv[j] = in && y ? y[(size_t)b * K + k] : 0.f;
        }
      }
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < KPT; ++j) {
        e[j] = col(j) < K ? expf(e[j]) : 0.f;
        s += e[j];
      }
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      const float inv = 1.0f / s;
      float dot = 0.f;
#pragma unroll
      for (int j = 0; j < KPT; ++j) {
        const float v = inv * e[j];
        e[j] = v;
        dot += v * yv[j];
      }
      if constexpr (V4) {
#pragma unroll
        for (int i = 0; i < KPT / 4; ++i) {
          const int k = 4 * (part + 4 * i);
          if (live && k < K) st4(p + (size_t)b * K + k, f32x4{e[4 * i], e[4 * i + 1], e[4 * i + 2], e[4 * i + 3]});
        }
      } else {
#pragma unroll
        for (int j = 0; j < KPT; ++j)
          if (live && col(j) < K) p[(size_t)b * K + col(j)] = e[j];
      }
      dot += __shfl_xor(dot, 1, 64);
      dot += __shfl_xor(dot, 2, 64);
      if (part == 0) rl[r] = live && y ? (double)(-logf(dot)) : 0.0;
      __syncthreads();
      if (wv == 0) {
        // fixed order: lane l adds rows 4l .. 4l + 3, then a 64-lane tree (thread 0 alone, one LDS
        // read and one dependent fp64 add per row, took ~10 us)
        double t = ((rl[4 * lane] + rl[4 * lane + 1]) + rl[4 * lane + 2]) + rl[4 * lane + 3];
        t = wave_sum(t);
        if (lane == 0) acc += t;
      }
      __syncthreads();
    }
  } else {
    for (int b = wv; b < B; b += 16) {
      const float* xr = x + (size_t)b * K;
      float* pr = p + (size_t)b * K;
      float s = 0.f;
      for (int j = lane; j < K; j += 64) s += expf(xr[j]);
      s = wave_sum(s);
      const float inv = 1.0f / s;
      float dot = 0.f;
      for (int j = lane; j < K; j += 64) {
        const float v = inv * expf(xr[j]);
        pr[j] = v;
        if (y) dot += v * y[(size_t)b * K + j];
      }
      if (y) {
        dot = wave_sum(dot);
        acc += (double)(-logf(dot));
      }
    }
  }
  if (lane == 0) red[wv] = acc;
  __syncthreads();
  if (threadIdx.x == 0 && loss) {
    double t = 0.0;
    for (int w = 0; w < 16; ++w) t += red[w];
    *loss = (float)((1.0 / (double)B) * t);
  }
}

// dx = (1/B) * (p - y)   (losses.py:29-34)
__global__ void softmax_xent_bwd_kernel(const float* __restrict__ p, const float* __restrict__ y, int B, int K,
                                        float* __restrict__ dx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * K) return;
  dx[i] = (1.0f / (float)B) * (p[i] - y[i]);
}

// Multi-tensor SGD momentum: for every listed tensor t and element i
//   d = (-lr) * g + mom * v;  w += d;  v = d      (SGDMomentum.py:33-39, same op order)
struct SgdEntry {
  float* w;
  const float* g;
  float* v;
  long long n;
  long long block0;  // first block index owned by this tensor
};

constexpr int kSgdLdsTable = 1024;
__global__ __launch_bounds__(256) void sgd_momentum_multi_kernel(const SgdEntry* __restrict__ tab, int ntens,
                                                                 float lr, float mom, float gscale) {
  // find the tensor owning this block: the block0 column is loaded into LDS in parallel (one
  // load latency) and searched there; the old linear scan of the global table was ~100
  // dependent loads for the last blocks.
  __shared__ long long b0s[kSgdLdsTable];
  __shared__ int owner;
  const long long b = blockIdx.x;
  int t = 0;
  if (ntens <= kSgdLdsTable) {
    for (int i = threadIdx.x; i < ntens; i += blockDim.x) b0s[i] = tab[i].block0;
    __syncthreads();
    if (threadIdx.x == 0) {
      int lo = 0, hi = ntens - 1;  // last entry with block0 <= b
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (b0s[mid] <= b) lo = mid; else hi = mid - 1;
      }
      owner = lo;
    }
    __syncthreads();
    t = owner;
  } else {
    while (t + 1 < ntens && tab[t + 1].block0 <= b) ++t;
  }
  const SgdEntry e = tab[t];
  const long long i = (b - e.block0) * 256 + threadIdx.x;
  if (i >= e.n) return;
  const float g = gscale == 1.0f ? e.g[i] : __fmul_rn(gscale, e.g[i]);
  const float d = __fadd_rn(__fmul_rn(-lr, g), __fmul_rn(mom, e.v[i]));
  e.w[i] = __fadd_rn(e.w[i], d);
  e.v[i] = d;
}

// out[0] = 0.5 * strength * sum w^2 (one block, fp64 accumulate).  With accumulate != 0,
// adds into out[0] instead of overwriting.
__global__ __launch_bounds__(256) void l2_loss_kernel(const float* __restrict__ w, long long n, float strength,
                                                      int accumulate, float* __restrict__ out) {
  __shared__ double red[256];
  double s = 0.0;
  for (long long i = threadIdx.x; i < n; i += 256) {
    const double v = w[i];
    s += v * v;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float v = (float)(0.5 * (double)strength * red[0]);
    out[0] = accumulate ? out[0] + v : v;
  }
}

// Multi-tensor l2 loss term, stage 1: block b (owning a 2048-element chunk of tensor t)
// writes part[b] = 0.5 * strength_t * sum(w^2) over its chunk (fp64).
struct L2Entry {
  const float* w;
  long long n;
  long long block0;
  float strength;
  float pad_;
};

constexpr int kL2Chunk = 2048;

__global__ __launch_bounds__(256) void l2_multi_partial_kernel(const L2Entry* __restrict__ tab, int ntens,
                                                               double* __restrict__ part) {
  __shared__ double red[256];
  int t = 0;
  const long long b = blockIdx.x;
  while (t + 1 < ntens && tab[t + 1].block0 <= b) ++t;
  const L2Entry e = tab[t];
  const long long i0 = (b - e.block0) * kL2Chunk;
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < kL2Chunk / 256; ++k) {
    const long long i = i0 + k * 256 + threadIdx.x;
    if (i < e.n) {
      const double v = e.w[i];
      s += v * v;
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[b] = 0.5 * (double)e.strength * red[0];
}

// Stage 2 (one block): out[0] = (add_to ? add_to[0] : 0) + sum_b part[b], fixed order.
__global__ __launch_bounds__(256) void l2_multi_final_kernel(const double* __restrict__ part, long long nparts,
                                                             const float* __restrict__ add_to,
                                                             float* __restrict__ out) {
  __shared__ double red[256];
  double s = 0.0;
  for (long long i = threadIdx.x; i < nparts; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)((add_to ? (double)add_to[0] : 0.0) + red[0]);
}

// Column sums of an [M][N] matrix, stage 1: ws[chunk][n] = sum of rows in the chunk.
__global__ void colsum_partial_kernel(const float* __restrict__ in, int M, int N, int rpc, double* __restrict__ ws) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int r0 = blockIdx.y * rpc, r1 = min(M, r0 + rpc);
  double s = 0.0;
  int r = r0;
  for (; r + 8 <= r1; r += 8) {  // 8 loads in flight, added in row order
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = in[(size_t)(r + k) * N + n];
#pragma unroll
    for (int k = 0; k < 8; ++k) s += (double)v[k];
  }
  for (; r < r1; ++r) s += (double)in[(size_t)r * N + n];
  ws[(size_t)blockIdx.y * N + n] = s;
}

__global__ void colsum_final_kernel(const double* __restrict__ ws, int chunks, int N, float* __restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  double s = 0.0;
  for (int k = 0; k < chunks; ++k) s += ws[(size_t)k * N + n];
  out[n] = (float)s;
}

// NCHW -> NHWC with channel padding to 4 (C <= 4, the stem): thread = one pixel, C coalesced
// plane reads (consecutive threads, consecutive w) and one 16-byte store.
__global__ void nchw_to_nhwc4_kernel(const float* __restrict__ x, int N, int C, long long HW,
                                     float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)N * HW) return;
  const long long n = i / HW, p = i - n * HW;
  const float* xs = x + (size_t)n * C * HW + p;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < C; ++c) v[c] = __builtin_nontemporal_load(xs + (size_t)c * HW);
  st4(y + (size_t)i * 4, v);
}

// NCHW -> NHWC with channel padding to Cp (zeros).
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int N, int C, int H, int W, int Cp,
                                    float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)N * H * W * Cp;
  if (i >= total) return;
  const int c = (int)(i % Cp);
  long long t = i / Cp;
  const int w = (int)(t % W);
  t /= W;
  const int h = (int)(t % H);
  const int n = (int)(t / H);
  y[i] = c < C ? x[(((size_t)n * C + c) * H + h) * W + w] : 0.f;
}

// NHWC with padded channels (Cp) -> NHWC with C channels (drop the pad).
__global__ void nhwc_unpad_kernel(const float* __restrict__ x, long long P, int Cp, int C, float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * C) return;
  const long long p = i / C;
  const int c = (int)(i - p * C);
  y[i] = x[p * Cp + c];
}

__global__ __launch_bounds__(256) void scale_kernel(const float* __restrict__ x, long long n, float s,
                                                    float* __restrict__ y, int vec) {
  const long long nv = vec ? (n >> 2) : 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride)
    st4(y + 4 * i, s * ld4(x + 4 * i));
  for (long long i = 4 * nv + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = s * x[i];
}

static int colsum_chunks(int M) {
  int chunks = cdiv(M, 64);
  if (chunks > 512) chunks = 512;
  if (chunks < 1) chunks = 1;
  return chunks;
}

static inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
static inline bool al4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3) == 0; }

static inline dim3 grid1(long long n) { return dim3((unsigned)cdivll(n, 256)); }

// Grid for the float4 grid-stride kernels: one float4 per thread, capped at 16k blocks.
static inline dim3 grid4(long long n) {
  long long b = cdivll((n + 3) / 4, 256);
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return dim3((unsigned)b);
}

}  // namespace dk

using namespace dk;

DK_API int dk_relu_fwd_f32(const float* x, long long n, float* y, uint8_t* mask, void* stream) {
  hipLaunchKernelGGL(relu_fwd_kernel<float>, grid4(n), dim3(256), 0, as_stream(stream), x, n, y, mask,
                     (int)(al16(x) && al16(y) && al4(mask)));
  return launch_status();
}

DK_API int dk_relu_bwd_f32(const float* dy, const uint8_t* mask, long long n, float* dx, void* stream) {
  hipLaunchKernelGGL(relu_bwd_kernel<float>, grid4(n), dim3(256), 0, as_stream(stream), dy, mask, n, dx,
                     (int)(al16(dy) && al16(dx) && al4(mask)));
  return launch_status();
}

static inline bool al8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; }

DK_API int dk_relu_fwd_bf16(const bf16_t* x, long long n, bf16_t* y, uint8_t* mask, void* stream) {
  hipLaunchKernelGGL(relu_fwd_kernel<bf16_t>, grid4(n), dim3(256), 0, as_stream(stream), x, n, y, mask,
                     (int)(al8(x) && al8(y) && al4(mask)));
  return launch_status();
}

DK_API int dk_relu_bwd_bf16(const bf16_t* dy, const uint8_t* mask, long long n, bf16_t* dx, void* stream) {
  hipLaunchKernelGGL(relu_bwd_kernel<bf16_t>, grid4(n), dim3(256), 0, as_stream(stream), dy, mask, n, dx,
                     (int)(al8(dy) && al8(dx) && al4(mask)));
  return launch_status();
}

DK_API int dk_mask_to_f32(const uint8_t* mask, long long n, float* out, void* stream) {
  hipLaunchKernelGGL(mask_to_f32_kernel, grid1(n), dim3(256), 0, as_stream(stream), mask, n, out);
  return launch_status();
}

DK_API int dk_add_f32(const float* a, const float* b, long long n, int relu, float* y, uint8_t* mask, void* stream) {
  hipLaunchKernelGGL(add_kernel, grid4(n), dim3(256), 0, as_stream(stream), a, b, n, relu, y, mask,
                     (int)(al16(a) && al16(b) && al16(y) && al4(mask)));
  return launch_status();
}

DK_API int dk_bn_add_f32(const float* a, const float* a_mean, const float* a_invstd, const float* a_gamma,
                         const float* a_beta, int a_relu, const float* b, const float* b_mean, const float* b_invstd,
                         const float* b_gamma, const float* b_beta, int b_relu, long long n, int C, int relu, float* y,
                         uint8_t* mask, void* stream) {
  const BnIn ba{a_mean, a_invstd, a_gamma, a_beta, a_relu}, bb{b_mean, b_invstd, b_gamma, b_beta, b_relu};
  auto params_ok = [](const BnIn& p) {
    return !p.mean || (p.invstd && p.gamma && p.beta && al16(p.mean) && al16(p.invstd) && al16(p.gamma) &&
                       al16(p.beta));
  };
  if (C < 4 || C % 4 || n % C || n >= (1ll << 31) || !al16(a) || !al16(b) || !al16(y) || !al4(mask) || !params_ok(ba) || !params_ok(bb))
    return DK_ERR_ARGS;
  hipLaunchKernelGGL(bn_add_kernel, grid4(n), dim3(256), 0, as_stream(stream), a, ba, b, bb, n, C, relu, y, mask,
                     nt_stores(kNtBnAdd));
  return launch_status();
}

DK_API int dk_gap_fwd_f32(const float* x, int N, int HW, int C, float* out, void* stream) {
  hipLaunchKernelGGL(gap_fwd_kernel, grid1((long long)N * C), dim3(256), 0, as_stream(stream), x, N, HW, C, out);
  return launch_status();
}

DK_API int dk_gap_join_fwd_f32(const float* a, const float* a_mean, const float* a_invstd, const float* a_gamma,
                               const float* a_beta, int a_relu, const float* b, const float* b_mean,
                               const float* b_invstd, const float* b_gamma, const float* b_beta, int b_relu, int N,
                               int HW, int C, uint8_t* mask, float* out, void* stream) {
  const BnIn ba{a_mean, a_invstd, a_gamma, a_beta, a_relu}, bb{b_mean, b_invstd, b_gamma, b_beta, b_relu};
  auto params_ok = [](const BnIn& p) { return !p.mean || (p.invstd && p.gamma && p.beta); };
  if (!a || !b || !out || N < 1 || HW < 1 || C < 1 || (long long)N * HW * C >= (1ll << 31) || !params_ok(ba) ||
      !params_ok(bb))
    return DK_ERR_ARGS;
  hipLaunchKernelGGL(gap_join_kernel, grid1((long long)N * C), dim3(256), 0, as_stream(stream), a, ba, b, bb, N, HW, C,
                     mask, out);
  return launch_status();
}

DK_API int dk_gap_bwd_f32(const float* dy, int N, int HW, int C, float* dx, void* stream) {
  if (C % 4 == 0 && (long long)N * HW * C < (1ll << 31) && (reinterpret_cast<uintptr_t>(dy) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(dx) & 15) == 0)
    hipLaunchKernelGGL(gap_bwd4_kernel, grid1((long long)N * HW * C / 4), dim3(256), 0, as_stream(stream), dy, N, HW,
                       C, dx);
  else
    hipLaunchKernelGGL(gap_bwd_kernel, grid1((long long)N * HW * C), dim3(256), 0, as_stream(stream), dy, N, HW, C,
                       dx);
  return launch_status();
}

DK_API int dk_softmax_xent_fwd_f32(const float* x, const float* y_onehot, int B, int K, float* p, float* loss,
                                   void* stream) {
  const bool v4 = K % 4 == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(p) |
                                   reinterpret_cast<uintptr_t>(y_onehot)) & 15) == 0;
  if (v4)
    hipLaunchKernelGGL(softmax_xent_fwd_kernel<true>, dim3(1), dim3(1024), 0, as_stream(stream), x, y_onehot, B, K, p,
                       loss);
  else
    hipLaunchKernelGGL(softmax_xent_fwd_kernel<false>, dim3(1), dim3(1024), 0, as_stream(stream), x, y_onehot, B, K,
                       p, loss);
  return launch_status();
}

DK_API int dk_softmax_xent_bwd_f32(const float* p, const float* y_onehot, int B, int K, float* dx, void* stream) {
  hipLaunchKernelGGL(softmax_xent_bwd_kernel, grid1((long long)B * K), dim3(256), 0, as_stream(stream), p, y_onehot, B,
                     K, dx);
  return launch_status();
}

// table: device array of ntens SgdEntry records (40 bytes each, see include/dorknet_hip.h),
// total_blocks = sum over tensors of ceil(n / 256) (== block0 of a virtual entry ntens).
DK_API int dk_sgd_momentum_multi_f32(const void* table, int ntens, long long total_blocks, float lr, float momentum,
                                     float grad_scale, void* stream) {
  if (ntens <= 0) return 0;
  hipLaunchKernelGGL(sgd_momentum_multi_kernel, dim3((unsigned)total_blocks), dim3(256), 0, as_stream(stream),
                     static_cast<const SgdEntry*>(table), ntens, lr, momentum, grad_scale);
  return launch_status();
}

DK_API int dk_l2_loss_f32(const float* w, long long n, float strength, int accumulate, float* out, void* stream) {
  hipLaunchKernelGGL(l2_loss_kernel, dim3(1), dim3(256), 0, as_stream(stream), w, n, strength, accumulate, out);
  return launch_status();
}

// All l2 loss terms of a network in two launches.  table: ntens L2Entry records (32 bytes:
// { const float* w; int64 n; int64 first_block; float strength; float pad }), first_block =
// sum of ceil(n / 2048) over the preceding entries, total_blocks = that sum over all.
// out[0] = add_to[0] (may be null) + sum_t 0.5 * strength_t * sum(w_t^2).
DK_API size_t dk_l2_multi_workspace_bytes(long long total_blocks) { return (size_t)total_blocks * sizeof(double); }

DK_API int dk_l2_loss_multi_f32(const void* table, int ntens, long long total_blocks, const float* add_to,
                                float* out, void* ws, size_t ws_bytes, void* stream) {
  if (ntens <= 0 || total_blocks <= 0) return DK_ERR_ARGS;
  if (ws_bytes < dk_l2_multi_workspace_bytes(total_blocks)) return DK_ERR_WORKSPACE;
  hipLaunchKernelGGL(l2_multi_partial_kernel, dim3((unsigned)total_blocks), dim3(256), 0, as_stream(stream),
                     static_cast<const L2Entry*>(table), ntens, static_cast<double*>(ws));
  int rc = launch_status();
  if (rc) return rc;
  hipLaunchKernelGGL(l2_multi_final_kernel, dim3(1), dim3(256), 0, as_stream(stream), static_cast<const double*>(ws),
                     total_blocks, add_to, out);
  return launch_status();
}

DK_API size_t dk_colsum_workspace_bytes(int M, int N) { return (size_t)colsum_chunks(M) * N * sizeof(double); }

DK_API int dk_colsum_f32(const float* in, int M, int N, float* out, void* ws, size_t ws_bytes, void* stream) {
  if (ws_bytes < dk_colsum_workspace_bytes(M, N)) return DK_ERR_WORKSPACE;
  const int chunks = colsum_chunks(M);
  const int rpc = cdiv(M, chunks);
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(cdiv(N, 256), chunks), dim3(256), 0, as_stream(stream), in, M, N, rpc,
                     static_cast<double*>(ws));
  int rc = launch_status();
  if (rc) return rc;
  hipLaunchKernelGGL(colsum_final_kernel, dim3(cdiv(N, 256)), dim3(256), 0, as_stream(stream),
                     static_cast<const double*>(ws), chunks, N, out);
  return launch_status();
}

DK_API int dk_nchw_to_nhwc_f32(const float* x, int N, int C, int H, int W, int Cp, float* y, void* stream) {
  if (Cp == 4 && C <= 4 && al16(y)) {
    hipLaunchKernelGGL(nchw_to_nhwc4_kernel, grid1((long long)N * H * W), dim3(256), 0, as_stream(stream), x, N, C,
                       (long long)H * W, y);
    return launch_status();
  }
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, grid1((long long)N * H * W * Cp), dim3(256), 0, as_stream(stream), x, N, C, H,
                     W, Cp, y);
  return launch_status();
}

DK_API int dk_nhwc_unpad_f32(const float* x, long long P, int Cp, int C, float* y, void* stream) {
  hipLaunchKernelGGL(nhwc_unpad_kernel, grid1(P * C), dim3(256), 0, as_stream(stream), x, P, Cp, C, y);
  return launch_status();
}

// y = s * x (l2 backward, regularisers/l2.py:16-17; gradient averaging in data parallel)
DK_API int dk_scale_f32(const float* x, long long n, float s, float* y, void* stream) {
  hipLaunchKernelGGL(scale_kernel, grid4(n), dim3(256), 0, as_stream(stream), x, n, s, y, (int)(al16(x) && al16(y)));
  return launch_status();
}

DK_API int dk_abi_version(void) { return 1; }

// ---------------------------------------------------------------------------------------
// fp32 <-> bf16 storage casts (BASELINE config 5 inputs / checks): round to nearest even.
// ---------------------------------------------------------------------------------------
namespace dk {
__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, long long n, bf16_t* __restrict__ y) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n && ((n & 3) == 0)) {
    st4(y + i, ld4(x + i));
  } else {
    for (long long k = i; k < n && k < i + 4; ++k) st1(y + k, x[k]);
  }
}
__global__ void cast_bf16_f32_kernel(const bf16_t* __restrict__ x, long long n, float* __restrict__ y) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n && ((n & 3) == 0)) {
    st4(y + i, ld4(x + i));
  } else {
    for (long long k = i; k < n && k < i + 4; ++k) y[k] = ld1(x + k);
  }
}
}  // namespace dk

DK_API int dk_cast_f32_to_bf16(const float* x, long long n, uint16_t* y, void* stream) {
  if (n <= 0) return 0;
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(y) & 7)) return DK_ERR_ARGS;
  hipLaunchKernelGGL(dk::cast_f32_bf16_kernel, dim3((unsigned)dk::cdivll(n, 1024)), dim3(256), 0,
                     dk::as_stream(stream), x, n, y);
  return dk::launch_status();
}

DK_API int dk_cast_bf16_to_f32(const uint16_t* x, long long n, float* y, void* stream) {
  if (n <= 0) return 0;
  if ((reinterpret_cast<uintptr_t>(x) & 7) || (reinterpret_cast<uintptr_t>(y) & 15)) return DK_ERR_ARGS;
  hipLaunchKernelGGL(dk::cast_bf16_f32_kernel, dim3((unsigned)dk::cdivll(n, 1024)), dim3(256), 0,
                     dk::as_stream(stream), x, n, y);
  return dk::launch_status();
}
