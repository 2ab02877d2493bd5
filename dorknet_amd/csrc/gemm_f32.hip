// Implicit-GEMM engine on fp32 MFMA (v_mfma_f32_32x32x2_f32) for gfx950.
//
// Every dense contraction on the hot path is one instance of
//     C[m][n] (+)= sum_k  A(m, k) * B(n, k)
// where A and B are *views* of NHWC activations / weights, never materialised:
//   * conv forward  (replaces im2col + cp.dot, layers/convolution.py:58-87, :187-203)
//       m = output pixel (n,oh,ow), n = output channel, k = (r,s,c) with c innermost
//   * conv dgrad    (replaces cp.dot + row2im, convolution.py:101-117, :205-222)
//       stride 1: m = input pixel, k = (r,s,k_out), A gathers dy at (h+p-r, w+p-s)
//       stride >1: one such GEMM per sub-pixel phase (a, b) of dx, with the phase's sub-filter
//       (dk_conv2d_dgrad_phase_f32): no column matrix, no scatter
//   * conv wgrad    (replaces cp.dot(upstream.T, patches), convolution.py:93-100)
//       m = output channel, n = (r,s,c), k = output pixel; split-K over pixels with a
//       fixed-order second stage (no atomics, deterministic)
//   * pointwise fwd/dgrad/wgrad (layers/pointwise_convolution.py:46-75) as the
//       R=S=1 case; stride-2 subsampling is a strided gather, the backward "widen"
//       is fused into the epilogue
//   * dense fwd/dgrad/wgrad (layers/dense_layer.py:46-67)
//
// Data movement: operand tiles go global -> registers (one K-tile of prefetch) -> LDS
// (two buffers, one barrier per K-tile).  Global reads are buffer loads whose
// out-of-range offsets return 0 in hardware, so padding, ragged tiles and the K tail need
// no branches.  An operand whose source is K-contiguous (activation rows, weight rows)
// is kept K-contiguous in LDS ([rows][BK+4]) and read with one conflict-free
// ds_read_b128 per lane that feeds four MFMAs; an operand whose source is
// row-contiguous (wgrad operands) is kept [BK][rows] and read with ds_read_b32.  Because
// the MFMA sums over k in any order, the four MFMAs of a q-block use k = 8q + 4h + t
// (h = lane half, t = 0..3) on both operands.
#include <stdlib.h>

#include "dk_common.h"
#include "fold_tail.h"

namespace dk {

// ----------------------------------------------------------------------------
// Buffer loads (OOB -> 0)
// ----------------------------------------------------------------------------

constexpr uint32_t kOOB = 0x80000000u;  // an offset past any buffer we build (tensors < 2 GiB)

__device__ __forceinline__ float bload1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}

// ----------------------------------------------------------------------------
// Operand descriptors
// ----------------------------------------------------------------------------

// Implicit-im2col view of an NHWC tensor x[n][ih][iw][c] (C % 4 == 0, < 2 GiB).
// Row/pixel index m -> (n, oh, ow) over an OH x OW grid; tap (r,s) reads
// (ih, iw) = (oh*sa + dr*r + off, ow*sa + dr*s + off), zero outside [0,H)x[0,W).
// E: element type of the tensor (float, or bf16_t for BASELINE config 5's bf16 storage); the
// loaders widen to fp32 as they load.
// K1: a 1x1 filter (pointwise): k is the channel, no tap arithmetic per K-tile.
template <class E, bool K1 = false>
struct ImgDescE {
  static constexpr bool kBnIn = false;
  static constexpr bool kBnBwd = false;
  static constexpr bool k1x1 = K1;
  using Elem = E;
  const E* x;
  uint32_t bytes;
  int H, W, C;
  int OH, OW;
  int R, S;
  int sa, dr, off;
  int offw;  // column offset (= off except for the sub-pixel phase views of the strided dgrad)
  int M;  // N * OH * OW
  // division-free index arithmetic in the per-K-tile loader paths: q = umulhi(n, m) for
  // the divisors C, S, OW, OH (set_magics; 0 = divide).  Exact while n * d < 2^32.
  uint32_t mC, mS, mOW, mOH;
};
using ImgDesc = ImgDescE<float>;

__device__ __forceinline__ int fdiv(int n, int d, uint32_t m) {
  return m ? (int)__umulhi((uint32_t)n, m) : n / d;
}

// The same view of bn(x) (+ReLU): the loaders apply the BatchNorm of the layer that
// produced x to every in-image element (padding stays exactly 0, as in the reference,
// which pads the BN output).
template <class E, bool K1 = false>
struct ImgBnDescE : ImgDescE<E, K1> {
  static constexpr bool kBnIn = true;
  BnIn bn;
};
using ImgBnDesc = ImgBnDescE<float>;

// Row-major matrix p[row][ld]; `ext` bounds the non-reduction index.
template <class E>
struct MatDescE {
  static constexpr bool kBnIn = false;
  static constexpr bool kBnBwd = false;
  using Elem = E;
  const E* p;
  uint32_t bytes;
  int ld;
  int ext;
};
using MatDesc = MatDescE<float>;

// The backward of the BatchNorm that followed this layer, applied as its gradient is loaded
// (stage 3 of batch_norm.py:125-174, = dk_bn_bwd_apply_f32, bit for bit): p holds
// g, the gradient w.r.t. the BN (+ReLU) output; x is the BN's raw input (same layout); the
// loader forms dy = gamma*invstd * (g' - k1 - x_hat*k2) (g' = g masked by the fused ReLU,
// recomputed from x) and the blocks of the first column tile also store dy to dy_out (for
// the weight gradient, which reads it afterwards).
struct BnBwdIn {
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  const float* k12;  // [k1[C], k2[C]] (dk_bn_bwd_from_partials_f32)
  int relu;
  int C;
};
struct MatBwdDesc : MatDescE<float> {
  static constexpr bool kBnBwd = true;
  const float* x;
  BnBwdIn bwd;
  float* dy_out;
};

// ----------------------------------------------------------------------------
// Loaders.  K-contiguous ("KC") loaders fill T[ROWS][BK+4]; row-contiguous ("IC")
// loaders fill T[BK][ROWS].  frag(T, row, q, h) returns the four k values
// 8q + 4h + {0,1,2,3} of `row` for the MFMA loop.
// ----------------------------------------------------------------------------

template <int ROWS, int BK>
struct KCLayout {
  static constexpr int SK = BK + 4;  // row stride in floats: (BK+4)/4 odd -> conflict-free b128 reads
  static constexpr int BUF = ROWS * SK;
  __device__ static __forceinline__ f32x4 frag(const float* T, int row, int q, int h) {
    return ld4(T + row * SK + 8 * q + 4 * h);
  }
};

template <int ROWS, int BK>
struct ICLayout {
  static constexpr int S = ROWS;
  static constexpr int BUF = BK * ROWS;
  __device__ static __forceinline__ f32x4 frag(const float* T, int row, int q, int h) {
    const float* p = T + (8 * q + 4 * h) * S + row;
    return f32x4{p[0], p[S], p[2 * S], p[3 * S]};
  }
};

// Implicit-im2col rows of an NHWC image (K-contiguous).
template <int ROWS, int BK, int NT>
struct LdImgKC : KCLayout<ROWS, BK> {
  static constexpr bool kTable = true;  // reads the BN table from LDS (see igemm_f32)
  using L = KCLayout<ROWS, BK>;
  static constexpr int KQ = BK / 4;
  static constexpr int RSTEP = NT / KQ;
  static constexpr int NR = ROWS >= RSTEP ? ROWS / RSTEP : 1;
  int kq, rb;
  bool active;
  int base[NR], ih0[NR], iw0[NR];
  f32x4 v[NR];
  // input BatchNorm (ImgBnDesc): per-channel {mean, invstd, gamma, beta} table in LDS
  // (filled by the kernel prologue), this k-tile's channel, in-image rows
  const f32x4* tab;
  int tc;  // table stride (channels)
  int cch;
  uint32_t okm;
  int relu;

  template <class D>
  __device__ __forceinline__ void init(const D& d, int row0, int tid) {
    kq = tid % KQ;
    rb = tid / KQ;
    active = rb < ROWS;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int m = row0 + rb + j * RSTEP;
      if (active && m < d.M) {
        const int ow = m % d.OW;
        const int t = m / d.OW;
        const int oh = t % d.OH;
        const int n = t / d.OH;
        ih0[j] = oh * d.sa + d.off;
        iw0[j] = ow * d.sa + d.offw;
        base[j] = (n * d.H + ih0[j]) * d.W + iw0[j];
      } else {
        ih0[j] = -(1 << 28);
        iw0[j] = -(1 << 28);
        base[j] = 0;
      }
    }
    if constexpr (D::kBnIn) relu = d.bn.relu;
  }

  template <class D>
  __device__ __forceinline__ void load(const D& d, int k0, int Ktot) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc_v(d.x, d.bytes);
    const int k = k0 + 4 * kq;
    const bool kv = k < Ktot;
    int c = k, dri = 0, dsi = 0, doff = 0;
    if constexpr (!D::k1x1) {
      const int tap = fdiv(k, d.C, d.mC);
      c = k - tap * d.C;
      const int r = fdiv(tap, d.S, d.mS);
      const int s = tap - r * d.S;
      dri = d.dr * r;
      dsi = d.dr * s;
      doff = dri * d.W + dsi;
    }
    uint32_t om = 0;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int ih = ih0[j] + dri, iw = iw0[j] + dsi;
      const bool ok = kv && (unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W;
      v[j] = bload4e<typename D::Elem>(rs, ok, (uint32_t)((base[j] + doff) * d.C + c));
      om |= (uint32_t)ok << j;
    }
    if constexpr (D::kBnIn) {
      cch = kv ? c : 0;
      okm = om;
    }
  }

  template <class D>
  __device__ __forceinline__ void store(float* T) const {
    if (!active) return;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      f32x4 o = v[j];
      if constexpr (D::kBnIn) {
        const float* tb = reinterpret_cast<const float*>(tab) + cch;
        const f32x4 t = bn_in4(o, ld4(tb), ld4(tb + tc), ld4(tb + 2 * tc), ld4(tb + 3 * tc), relu);
        if ((okm >> j) & 1u) o = t;
      }
      st4(T + (rb + j * RSTEP) * L::SK + 4 * kq, o);
    }
  }
};

// Row-major matrix p[i][ld], k along the row (K-contiguous).  VEC: float4 loads
// (ld % 4 == 0, Ktot % 4 == 0); otherwise four scalar loads.
template <int ROWS, int BK, int NT, bool VEC>
struct LdMatKCT : KCLayout<ROWS, BK> {
  static constexpr bool kTable = false;  // reads the BN table from LDS (see igemm_f32)
  using L = KCLayout<ROWS, BK>;
  static constexpr int KQ = BK / 4;
  static constexpr int RSTEP = NT / KQ;
  static constexpr int NR = ROWS >= RSTEP ? ROWS / RSTEP : 1;
  int kq, rb, row0;
  bool active;
  f32x4 v[NR];
  // BN backward on load (MatBwdDesc): the BN's raw input, the parameter table in LDS
  // ({mean, invstd, gamma, beta}, {k1, k2, gamma*invstd, 0} per channel), dy write-through
  f32x4 xv[NR];
  const f32x4* tab;
  int tc;  // table stride (channels)
  float* dyo;
  bool writer;
  int kcur;
  uint32_t eoff[NR];
  uint32_t okm;

  template <class D>
  __device__ __forceinline__ void init(const D&, int row0_, int tid) {
    kq = tid % KQ;
    rb = tid / KQ;
    row0 = row0_;
    active = rb < ROWS;
  }

  template <class D>
  __device__ __forceinline__ void load(const D& d, int k0, int Ktot) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc_v(d.p, d.bytes);
    const int k = k0 + 4 * kq;
    static_assert(VEC || sizeof(typename D::Elem) == 4, "scalar loads: fp32 storage only");
    static_assert(VEC || !D::kBnBwd, "BN backward on load: 16-byte loads only");
    uint32_t om = 0;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int i = row0 + rb + j * RSTEP;
      const bool iv = active && i < d.ext;
      const uint32_t base = (uint32_t)(i * d.ld + k) * 4u;
      if constexpr (VEC) {
        v[j] = bload4e<typename D::Elem>(rs, iv && k < Ktot, (uint32_t)(i * d.ld + k));
        if constexpr (D::kBnBwd) {
          const __amdgpu_buffer_rsrc_t rx = make_rsrc_v(d.x, d.bytes);
          xv[j] = bload4e<float>(rx, iv && k < Ktot, (uint32_t)(i * d.ld + k));
          eoff[j] = (uint32_t)(i * d.ld + k);
          om |= (uint32_t)(iv && k < Ktot) << j;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][e] = bload1(rs, (iv && k + e < Ktot) ? base + 4u * e : kOOB);
      }
    }
    if constexpr (D::kBnBwd) {
      kcur = k;
      okm = om;
    }
  }

  template <class D>
  __device__ __forceinline__ void store(float* T) {
    if (!active) return;
    if constexpr (D::kBnBwd) {
      if (okm) {
        // dy for channels kcur..kcur+3 (all four < Ktot when any row is valid: Ktot % 4 == 0)
        const float* tb = reinterpret_cast<const float*>(tab) + kcur;
        const f32x4 mu = ld4(tb), is = ld4(tb + tc), ga = ld4(tb + 2 * tc), be = ld4(tb + 3 * tc);
        const f32x4 k1 = ld4(tb + 4 * tc), k2 = ld4(tb + 5 * tc), ff = ld4(tb + 6 * tc);
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          if (!((okm >> j) & 1u)) continue;
          f32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float xe = xv[j][e];
            float ge = v[j][e];
            if (relu_flag && !(bn_out(xe, mu[e], is[e], ga[e], be[e]) > 0.f)) ge = 0.f;
            o[e] = bn_bwd_elem(xe, ge, mu[e], is[e], ff[e], k1[e], k2[e]);
          }
          v[j] = o;
          if (writer) st4(dyo + eoff[j], o);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NR; ++j) st4(T + (rb + j * RSTEP) * L::SK + 4 * kq, v[j]);
  }
  int relu_flag = 0;
};
template <int ROWS, int BK, int NT>
using LdMatKC = LdMatKCT<ROWS, BK, NT, true>;
template <int ROWS, int BK, int NT>
using LdMatKC1 = LdMatKCT<ROWS, BK, NT, false>;

// Row-major matrix p[k][ld], i along the row (row-contiguous).
template <int ROWS, int BK, int NT, bool VEC>
struct LdMatICT : ICLayout<ROWS, BK> {
  static constexpr bool kTable = false;  // reads the BN table from LDS (see igemm_f32)
  using L = ICLayout<ROWS, BK>;
  static constexpr int IQ = ROWS / 4;
  static constexpr int KSTEP = NT / IQ;
  static constexpr int NK = BK >= KSTEP ? BK / KSTEP : 1;
  int iq, kb, i0;
  bool active;
  f32x4 v[NK];
  // BN backward on load (MatBwdDesc; wgrad's dy operand, i = channel): the BN's raw input and
  // the coefficient table in LDS, as LdMatKCT
  f32x4 xv[NK];
  uint32_t okm;
  const f32x4* tab;
  int tc;  // table stride (channels)
  float* dyo;
  bool writer;
  int relu_flag = 0;

  template <class D>
  __device__ __forceinline__ void init(const D&, int row0, int tid) {
    iq = tid % IQ;
    kb = tid / IQ;
    i0 = row0 + 4 * iq;
    active = kb < BK;
  }

  template <class D>
  __device__ __forceinline__ void load(const D& d, int k0, int Ktot) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc_v(d.p, d.bytes);
    static_assert(VEC || sizeof(typename D::Elem) == 4, "scalar loads: fp32 storage only");
    static_assert(VEC || !D::kBnBwd, "BN backward on load: 16-byte loads only");
    uint32_t om = 0;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int k = k0 + kb + j * KSTEP;
      const bool kv = active && k < Ktot;
      const uint32_t base = (uint32_t)(k * d.ld + i0) * 4u;
      if constexpr (VEC) {
        v[j] = bload4e<typename D::Elem>(rs, kv && i0 < d.ext, (uint32_t)(k * d.ld + i0));
        if constexpr (D::kBnBwd) {
          const __amdgpu_buffer_rsrc_t rx = make_rsrc_v(d.x, d.bytes);
          xv[j] = bload4e<float>(rx, kv && i0 < d.ext, (uint32_t)(k * d.ld + i0));
          om |= (uint32_t)(kv && i0 < d.ext) << j;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][e] = bload1(rs, (kv && i0 + e < d.ext) ? base + 4u * e : kOOB);
      }
    }
    if constexpr (D::kBnBwd) okm = om;
  }

  template <class D>
  __device__ __forceinline__ void store(float* T) {
    if (!active) return;
    if constexpr (D::kBnBwd) {
      if (okm) {
        // dy for channels i0..i0+3 (all < ext when any pixel is valid: ext % 4 == 0)
        const float* tb = reinterpret_cast<const float*>(tab) + i0;
        const f32x4 mu = ld4(tb), is = ld4(tb + tc), ga = ld4(tb + 2 * tc), be = ld4(tb + 3 * tc);
        const f32x4 k1 = ld4(tb + 4 * tc), k2 = ld4(tb + 5 * tc), ff = ld4(tb + 6 * tc);
#pragma unroll
        for (int j = 0; j < NK; ++j) {
          f32x4 o = {0.f, 0.f, 0.f, 0.f};
          if ((okm >> j) & 1u) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float xe = xv[j][e];
              float ge = v[j][e];
              if (relu_flag && !(bn_out(xe, mu[e], is[e], ga[e], be[e]) > 0.f)) ge = 0.f;
              o[e] = bn_bwd_elem(xe, ge, mu[e], is[e], ff[e], k1[e], k2[e]);
            }
          }
          v[j] = o;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NK; ++j) st4(T + (kb + j * KSTEP) * L::S + 4 * iq, v[j]);
  }
};
template <int ROWS, int BK, int NT>
using LdMatIC = LdMatICT<ROWS, BK, NT, true>;
template <int ROWS, int BK, int NT>
using LdMatIC1 = LdMatICT<ROWS, BK, NT, false>;

// Implicit-im2col image with i = (r,s,c) (c innermost) and k = pixel (row-contiguous).
// Used by wgrad: B(i=(r,s,c), k=m) = x[pixel(m) shifted by tap (r,s)][c].
template <int ROWS, int BK, int NT>
struct LdImgIC : ICLayout<ROWS, BK> {
  static constexpr bool kTable = false;  // reads the BN table from LDS (see igemm_f32)
  using L = ICLayout<ROWS, BK>;
  static constexpr int IQ = ROWS / 4;
  static constexpr int KSTEP = NT / IQ;
  static constexpr int NK = BK >= KSTEP ? BK / KSTEP : 1;
  int iq, kb;
  bool active, colv;
  int c, dri, dsi;
  f32x4 v[NK];
  f32x4 bm, bi, bg, bb;  // input BatchNorm of this thread's (fixed) 4 channels
  uint32_t okm;
  int relu;

  template <class D>
  __device__ __forceinline__ void init(const D& d, int row0, int tid) {
    iq = tid % IQ;
    kb = tid / IQ;
    active = kb < BK;
    const int j = row0 + 4 * iq;
    colv = active && j < d.R * d.S * d.C;
    const int tap = j / d.C;
    c = j - tap * d.C;
    const int r = tap / d.S;
    const int s = tap - r * d.S;
    dri = d.dr * r;
    dsi = d.dr * s;
    if constexpr (D::kBnIn) {
      const int cc = colv ? c : 0;
      bm = ld4(d.bn.mean + cc);
      bi = ld4(d.bn.invstd + cc);
      bg = ld4(d.bn.gamma + cc);
      bb = ld4(d.bn.beta + cc);
      relu = d.bn.relu;
    }
  }

  template <class D>
  __device__ __forceinline__ void load(const D& d, int k0, int Ktot) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc_v(d.x, d.bytes);
    uint32_t om = 0;
#pragma unroll
    for (int jj = 0; jj < NK; ++jj) {
      const int m = k0 + kb + jj * KSTEP;
      const int t = fdiv(m, d.OW, d.mOW);
      const int ow = m - t * d.OW;
      const int n = fdiv(t, d.OH, d.mOH);
      const int oh = t - n * d.OH;
      const int ih = oh * d.sa + dri + d.off;
      const int iw = ow * d.sa + dsi + d.off;
      const bool ok = colv && m < d.M && (unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W;
      v[jj] = bload4e<typename D::Elem>(rs, ok, (uint32_t)(((n * d.H + ih) * d.W + iw) * d.C + c));
      om |= (uint32_t)ok << jj;
    }
    if constexpr (D::kBnIn) okm = om;
  }

  template <class D>
  __device__ __forceinline__ void store(float* T) const {
    if (!active) return;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      f32x4 o = v[j];
      if constexpr (D::kBnIn) {
        if ((okm >> j) & 1u) o = bn_in4(o, bm, bi, bg, bb, relu);
      }
      st4(T + (kb + j * KSTEP) * L::S + 4 * iq, o);
    }
  }
};

// ----------------------------------------------------------------------------
// Epilogues
// ----------------------------------------------------------------------------

// The kernel stages its accumulator tile through LDS and hands every thread 16-byte row
// chunks: put4(m, n, v) covers columns n..n+3 (all < N; only when the epilogue's v4 flag
// says the destination allows 16-byte stores), put1 a single column otherwise.  Epilogues
// with kColStats also fold a per-column reduction of what they store into a[e] / b[e].

// out[m][n] = acc (+ bias[n]) (+ res[m][n]: a residual addend laid out like out).
template <class O>
struct EpStoreT {  // O: output element type (float, or bf16_t: rounded on store)
  static constexpr bool kColStats = false;
  O* out;
  int ldo;
  const float* bias;
  int v4;  // out, ldo, bias and res allow 16-byte (4-element) access
  const O* res;
  // per-row operands the 16-byte path needs, loaded for all of a thread's rows before any
  // store (loads cannot be hoisted over stores to a possibly aliasing output)
  struct Pre {
    f32x4 r, x;
  };
  __device__ __forceinline__ Pre pre4(int m, int n) const {
    Pre p;
    p.r = res ? ld4(res + (size_t)m * ldo + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    return p;
  }
  __device__ __forceinline__ f32x4 value4(int n, f32x4 v, const Pre& p) const {
    if (bias) v += ld4(bias + n);
    if (res) v += p.r;
    return rnd4<O>(v);  // the value the store keeps
  }
  __device__ __forceinline__ float value1(int m, int n, float v) const {
    if (bias) v += bias[n];
    if (res) v += ld1(res + (size_t)m * ldo + n);
    return rnd1<O>(v);
  }
  __device__ __forceinline__ void put4(int m, int n, f32x4 v, const Pre& p, int, double*, double*) const {
    st4(out + (size_t)m * ldo + n, value4(n, v, p));
  }
  __device__ __forceinline__ void put1(int m, int n, float v, int, double&, double&) const {
    st1(out + (size_t)m * ldo + n, value1(m, n, v));
  }
};
using EpStore = EpStoreT<float>;

// EpStore + the BatchNorm statistics of the stored output (layers/batch_norm.py:76-80's
// mean/var, as fp64 sum / sum of squares per column): part[m_tile][2][N], one row per
// BM-row tile, reduced in a fixed order by dk_bn_stats_from_partials_f32.  Saves the
// separate statistics pass over y.
template <class O>
struct EpStoreStatsT : EpStoreT<O> {
  static constexpr bool kColStats = true;
  using Pre = typename EpStoreT<O>::Pre;
  double* part;
  FoldTail ft{};  // armed in-launch fold of part (fold_tail.h; set by launch_igemm)
  __device__ __forceinline__ void put4(int m, int n, f32x4 v, const Pre& p, int, double* a, double* b) const {
    const f32x4 o = this->value4(n, v, p);
    st4(this->out + (size_t)m * this->ldo + n, o);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const double d = (double)o[e];
      a[e] += d;
      b[e] += d * d;
    }
  }
  __device__ __forceinline__ void put1(int m, int n, float v, int, double& a, double& b) const {
    const float o = this->value1(m, n, v);
    st1(this->out + (size_t)m * this->ldo + n, o);
    a += (double)o;
    b += (double)o * (double)o;
  }
};
using EpStoreStats = EpStoreStatsT<float>;

// The BatchNorm-backward reduction of the layer whose input gradient this GEMM produces
// (batch_norm.py:125-174's sum(dy) and sum(dy * x_hat), with the fused ReLU's mask
// recomputed from the BN's raw input x as in dk_bn_bwd_partial_f64): part[m_tile][2][N].
__device__ __forceinline__ void bn_bwd_contrib(float g, float x, float mu, float is, float ga, float be, int relu,
                                               double& a, double& b) {
  const float xh = (x - mu) * is;
  if (relu && !(bn_out(x, mu, is, ga, be) > 0.f)) g = 0.f;
  a += (double)g;
  b += (double)g * (double)xh;
}
__device__ __forceinline__ void bn_bwd_contrib4(f32x4 g, f32x4 x, const BnIn& bn, int n, double* a, double* b) {
  const f32x4 mu = ld4(bn.mean + n), is = ld4(bn.invstd + n), ga = ld4(bn.gamma + n), be = ld4(bn.beta + n);
#pragma unroll
  for (int e = 0; e < 4; ++e) bn_bwd_contrib(g[e], x[e], mu[e], is[e], ga[e], be[e], bn.relu, a[e], b[e]);
}

template <class O>
struct EpStoreBnBwdT : EpStoreT<O> {
  static constexpr bool kColStats = true;
  using Pre = typename EpStoreT<O>::Pre;
  double* part;
  FoldTail ft{};  // armed in-launch fold of part (fold_tail.h; set by launch_igemm)
  const O* xbn;  // [M][ldo], the BN's raw input
  BnIn bn;
  __device__ __forceinline__ Pre pre4(int m, int n) const {
    Pre p = EpStoreT<O>::pre4(m, n);
    p.x = ld4(xbn + (size_t)m * this->ldo + n);
    return p;
  }
  __device__ __forceinline__ void put4(int m, int n, f32x4 v, const Pre& p, int, double* a, double* b) const {
    v = this->value4(n, v, p);
    st4(this->out + (size_t)m * this->ldo + n, v);
    bn_bwd_contrib4(v, p.x, bn, n, a, b);
  }
  __device__ __forceinline__ void put1(int m, int n, float v, int, double& a, double& b) const {
    v = this->value1(m, n, v);
    const size_t o = (size_t)m * this->ldo + n;
    st1(this->out + o, v);
    bn_bwd_contrib(v, ld1(xbn + o), bn.mean[n], bn.invstd[n], bn.gamma[n], bn.beta[n], bn.relu, a, b);
  }
};
using EpStoreBnBwd = EpStoreBnBwdT<float>;

// Pointwise stride-st backward "widen" (pointwise_convolution.py:68-72) fused: the GEMM
// row m = (b, oh, ow) of an OH x OW grid lands at (b, oh*st, ow*st) of an
// (OH*st) x (OW*st) grid and the other st*st-1 positions of that cell are zero.
struct EpWiden {
  static constexpr bool kColStats = false;
  float* out;
  int ldo;
  int OH, OW, st;
  int v4;
  const float* res;  // optional residual addend on the widened grid (off-lattice: out = res)
  __device__ __forceinline__ size_t cell(int m) const {
    const int ow = m % OW;
    const int t = m / OW;
    const int oh = t % OH;
    const int b = t / OH;
    return (size_t)(b * OH * st + oh * st) * (OW * st) + (size_t)ow * st;
  }
  struct Pre {
    f32x4 x;
  };
  __device__ __forceinline__ Pre pre4(int, int) const { return Pre{}; }
  __device__ __forceinline__ void put4(int m, int n, f32x4 v, const Pre&, int, double*, double*) const {
    const size_t c0 = cell(m);
    const size_t W2 = (size_t)OW * st;
    for (int dy = 0; dy < st; ++dy)
      for (int dx = 0; dx < st; ++dx) {
        const size_t o = (c0 + dy * W2 + dx) * ldo + n;
        f32x4 t = (dy | dx) ? f32x4{0.f, 0.f, 0.f, 0.f} : v;
        if (res) t += ld4(res + o);
        st4(out + o, t);
      }
  }
  __device__ __forceinline__ void put1(int m, int n, float v, int, double&, double&) const {
    const size_t c0 = cell(m);
    const size_t W2 = (size_t)OW * st;
    for (int dy = 0; dy < st; ++dy)
      for (int dx = 0; dx < st; ++dx) {
        const size_t o = (c0 + dy * W2 + dx) * ldo + n;
        out[o] = ((dy | dx) ? 0.f : v) + (res ? res[o] : 0.f);
      }
  }
};

// EpWiden + the BN-backward reduction over the written (lattice) points; the zeros off the
// lattice contribute nothing.
struct EpWidenBnBwd : EpWiden {
  static constexpr bool kColStats = true;
  double* part;
  FoldTail ft{};
  const float* xbn;  // the BN's raw input on the widened grid
  BnIn bn;
  __device__ __forceinline__ Pre pre4(int m, int n) const { return Pre{ld4(xbn + cell(m) * ldo + n)}; }
  __device__ __forceinline__ void put4(int m, int n, f32x4 v, const Pre& p, int sp, double* a, double* b) const {
    EpWiden::put4(m, n, v, p, sp, a, b);
    bn_bwd_contrib4(v, p.x, bn, n, a, b);
  }
  __device__ __forceinline__ void put1(int m, int n, float v, int sp, double& a, double& b) const {
    EpWiden::put1(m, n, v, sp, a, b);
    bn_bwd_contrib(v, xbn[cell(m) * ldo + n], bn.mean[n], bn.invstd[n], bn.gamma[n], bn.beta[n], bn.relu, a, b);
  }
};

// EpWidenBnBwd with the widened gradient kept compact: only the lattice points are stored, as
// the OH x OW grid out[m][n]; the BN-backward sums read the BN's input at the lattice points of
// the widened grid.  The consumer takes the off-lattice zeros as implied (dk_conv2d_wgrad_bnbwd_
// narrow_f32 with g_lattice = 2), so they are neither written nor read.
struct EpLatticeBnBwd : EpWiden {
  static constexpr bool kColStats = true;
  double* part;
  FoldTail ft{};
  const float* xbn;  // the BN's raw input on the widened grid
  BnIn bn;
  __device__ __forceinline__ Pre pre4(int m, int n) const { return Pre{ld4(xbn + cell(m) * ldo + n)}; }
  __device__ __forceinline__ void put4(int m, int n, f32x4 v, const Pre& p, int, double* a, double* b) const {
    st4(out + (size_t)m * ldo + n, v);
    bn_bwd_contrib4(v, p.x, bn, n, a, b);
  }
  __device__ __forceinline__ void put1(int m, int n, float v, int, double& a, double& b) const {
    out[(size_t)m * ldo + n] = v;
    bn_bwd_contrib(v, xbn[cell(m) * ldo + n], bn.mean[n], bn.invstd[n], bn.gamma[n], bn.beta[n], bn.relu, a, b);
  }
};

// Split-K partial tile: ws[split][M][N].
struct EpPartial {
  static constexpr bool kColStats = false;
  float* ws;
  int M, N;
  int v4;
  struct Pre {};
  __device__ __forceinline__ Pre pre4(int, int) const { return Pre{}; }
  __device__ __forceinline__ void put4(int m, int n, f32x4 v, const Pre&, int split, double*, double*) const {
    st4(ws + ((size_t)split * M + m) * N + n, v);
  }
  __device__ __forceinline__ void put1(int m, int n, float v, int split, double&, double&) const {
    ws[((size_t)split * M + m) * N + n] = v;
  }
};

// The output rows of one sub-pixel phase (a, b) of a stride-st input gradient: GEMM row
// m = (n, i, j) of an OHp x OWp grid is dx pixel (n, st*i + a, st*j + b) of an H x W image.
struct EpPhase {
  static constexpr bool kColStats = false;
  float* out;
  int ldo;
  int OHp, OWp, H, W, st, a, b;
  int v4;
  struct Pre {};
  __device__ __forceinline__ size_t pix(int m) const {
    const int j = m % OWp;
    const int t = m / OWp;
    const int i = t % OHp;
    const int n = t / OHp;
    return ((size_t)n * H + st * i + a) * W + (size_t)st * j + b;
  }
  __device__ __forceinline__ Pre pre4(int, int) const { return Pre{}; }
  __device__ __forceinline__ void put4(int m, int n, f32x4 v, const Pre&, int, double*, double*) const {
    st4(out + pix(m) * ldo + n, v);
  }
  __device__ __forceinline__ void put1(int m, int n, float v, int, double&, double&) const {
    out[pix(m) * ldo + n] = v;
  }
};

// ----------------------------------------------------------------------------
// The kernel
// ----------------------------------------------------------------------------

template <int BM, int BN, int BK, int WM, int WN, class LA, class DA, class LB, class DB, class EP>
__global__ __launch_bounds__(64 * WM * WN) void igemm_f32(DA da, DB db, EP ep, int M, int N, int Ktot,
                                                           int kt_per_split) {
  constexpr int TM = BM / (32 * WM);
  constexpr int TN = BN / (32 * WN);
  static_assert(TM >= 1 && TN >= 1 && BM == 32 * WM * TM && BN == 32 * WN * TN, "tile");
  static_assert(BK % 8 == 0, "BK");
  constexpr int ABUF = LA::BUF, BBUF = LB::BUF;
  // operand double buffers; the epilogue reuses the same LDS for the staged C tile
  // ([BM][BN+8]) and, with kColStats, the fp64 column-sum scratch
  constexpr int SMEM_OPS = 2 * (ABUF + BBUF);
  constexpr int SMEM_EPI = BM * (BN + 8);
  constexpr int SMEM_RED = EP::kColStats ? (64 * WM * WN / (BN / 4)) * BN * 4 : 0;
  constexpr int SMEM = SMEM_OPS > SMEM_EPI ? (SMEM_OPS > SMEM_RED ? SMEM_OPS : SMEM_RED)
                                           : (SMEM_EPI > SMEM_RED ? SMEM_EPI : SMEM_RED);
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  float* const As = smem;
  float* const Bs = smem + 2 * ABUF;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int l32 = lane & 31, h = lane >> 5;

  const int tiles_n = (N + BN - 1) / BN;
  const int bid = xcd_block(blockIdx.x, gridDim.x);  // neighbouring M-tiles share an XCD's L2
  const int m0 = (bid / tiles_n) * BM;
  const int n0 = (bid % tiles_n) * BN;
  const int KT = (Ktot + BK - 1) / BK;
  const int kt0 = blockIdx.y * kt_per_split;
  const int kt1 = min(KT, kt0 + kt_per_split);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][u][r] = 0.f;

  if (kt0 < kt1) {
    LA la;
    LB lb;
    la.init(da, m0, tid);
    lb.init(db, n0, tid);
    la.load(da, kt0 * BK, Ktot);  // first tile in flight before anything else
    lb.load(db, kt0 * BK, Ktot);
    if constexpr (DA::kBnIn && LA::kTable) {
      // BN-on-load parameter table for the A operand: {mean, invstd, gamma, beta} per channel
      // ([4][C]: consecutive channel quads of a lane group in consecutive 16-byte slots)
      extern __shared__ f32x4 bn_tab[];
      float* const bt = reinterpret_cast<float*>(bn_tab);
      for (int c = tid; c < da.C; c += 64 * WM * WN) {
        bt[c] = da.bn.mean[c];
        bt[da.C + c] = da.bn.invstd[c];
        bt[2 * da.C + c] = da.bn.gamma[c];
        bt[3 * da.C + c] = da.bn.beta[c];
      }
      la.tab = bn_tab;
      la.tc = da.C;
      __syncthreads();
    }
    if constexpr (DA::kBnBwd) {
      // BN-backward-on-load table for the A operand (channel = k), one array per coefficient
      // ([7][C]: mean, invstd, gamma, beta, k1, k2, gamma*invstd) so that the lanes of a
      // 16-lane group, which hold consecutive channel quads, read consecutive 16-byte slots
      // (the per-channel {.,.,.,.}{.,.,.,.} pairs put those quads 128 bytes apart: 4-way bank
      // conflicts on every ds_read_b128)
      extern __shared__ f32x4 bwd_tab[];
      float* const bt = reinterpret_cast<float*>(bwd_tab);
      const BnBwdIn& b = da.bwd;
      for (int c = tid; c < b.C; c += 64 * WM * WN) {
        const float ga = b.gamma[c], is = b.invstd[c];
        bt[c] = b.mean[c];
        bt[b.C + c] = is;
        bt[2 * b.C + c] = ga;
        bt[3 * b.C + c] = b.beta[c];
        bt[4 * b.C + c] = b.k12[c];
        bt[5 * b.C + c] = b.k12[b.C + c];
        bt[6 * b.C + c] = ga * is;
      }
      la.tab = bwd_tab;
      la.tc = b.C;
      la.dyo = da.dy_out;
      la.writer = da.dy_out != nullptr && n0 == 0;
      la.relu_flag = b.relu;
      __syncthreads();
    }
    la.template store<DA>(As);
    lb.template store<DB>(Bs);
    __syncthreads();
    int cur = 0;
    const int arow = wm * 32 * TM + l32;
    const int brow = wn * 32 * TN + l32;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) {
        la.load(da, (kt + 1) * BK, Ktot);
        lb.load(db, (kt + 1) * BK, Ktot);
      }
      const float* A_t = As + cur * ABUF;
      const float* B_t = Bs + cur * BBUF;
#pragma unroll
      for (int q = 0; q < BK / 8; ++q) {
        f32x4 af[TM], bf[TN];
#pragma unroll
        for (int t = 0; t < TM; ++t) af[t] = LA::frag(A_t, arow + 32 * t, q, h);
#pragma unroll
        for (int u = 0; u < TN; ++u) bf[u] = LB::frag(B_t, brow + 32 * u, q, h);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int t = 0; t < TM; ++t)
#pragma unroll
            for (int u = 0; u < TN; ++u)
              acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[t][e], bf[u][e], acc[t][u], 0, 0, 0);
      }
      if (more) {
        la.template store<DA>(As + (cur ^ 1) * ABUF);
        lb.template store<DB>(Bs + (cur ^ 1) * BBUF);
      }
      __syncthreads();
      cur ^= 1;
    }
  }

  // Epilogue: the accumulator tile goes through LDS ([BM][BN+8]; the +8 puts the two lane
  // halves' rows 4 apart on opposite bank halves) so that each thread stores 16-byte row
  // chunks -- 4x fewer store instructions than storing the MFMA C layout directly.
  constexpr int NT = 64 * WM * WN;
  constexpr int LDT = BN + 8;
  constexpr int NC4 = BN / 4;
  constexpr int RSTEP = NT / NC4;
  static_assert(NT % NC4 == 0, "epilogue thread map");
  __syncthreads();  // the MFMA loop's last LDS reads are done
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        smem[(wm * 32 * TM + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * LDT + wn * 32 * TN + u * 32 + l32] =
            acc[t][u][r];
  __syncthreads();
  const int c4 = tid % NC4, rl0 = tid / NC4;
  const int col = n0 + 4 * c4;
  const bool full = ep.v4 && col + 3 < N;
  double sa[4] = {0.0, 0.0, 0.0, 0.0}, sb[4] = {0.0, 0.0, 0.0, 0.0};
  constexpr int RPT = BM / RSTEP;  // rows per thread
  static_assert(BM % RSTEP == 0, "epilogue rows");
  if (full) {
    typename EP::Pre pre[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int row = m0 + rl0 + i * RSTEP;
      if (row < M) pre[i] = ep.pre4(row, col);
    }
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int rl = rl0 + i * RSTEP;
      if (m0 + rl < M) ep.put4(m0 + rl, col, ld4(smem + rl * LDT + 4 * c4), pre[i], blockIdx.y, sa, sb);
    }
  } else {
    for (int rl = rl0; rl < BM; rl += RSTEP) {
      const int row = m0 + rl;
      if (row >= M) break;
      const f32x4 v = ld4(smem + rl * LDT + 4 * c4);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (col + e < N) ep.put1(row, col + e, v[e], blockIdx.y, sa[e], sb[e]);
    }
  }

  if constexpr (EP::kColStats) {
    // per-column fp64 sums of this tile, fixed order: the thread's rows, then the RSTEP
    // threads sharing its column chunk -> part[m_tile][.][col]
    __syncthreads();  // done reading the staged tile
    double* red = reinterpret_cast<double*>(smem);  // [RSTEP][BN][2]
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[(rl0 * BN + 4 * c4 + e) * 2 + 0] = sa[e];
      red[(rl0 * BN + 4 * c4 + e) * 2 + 1] = sb[e];
    }
    __syncthreads();
    const int mt = bid / tiles_n;
    for (int i = tid; i < BN; i += NT) {
      const int cc = n0 + i;
      if (cc >= N) continue;
      double s1 = 0.0, s2 = 0.0;
      for (int k = 0; k < RSTEP; ++k) {
        s1 += red[(k * BN + i) * 2 + 0];
        s2 += red[(k * BN + i) * 2 + 1];
      }
      pub_store(ep.part + ((size_t)mt * 2 + 0) * N + cc, s1);
      pub_store(ep.part + ((size_t)mt * 2 + 1) * N + cc, s2);
    }
    if (ep.ft.part) {
      __syncthreads();  // done with red[]: the fold reuses the tile's LDS
      fold_tail<64 * WM * WN>(ep.ft, mt, n0, min(BN, N - n0), bid % tiles_n, reinterpret_cast<double2*>(smem));
    }
  }
}

static inline int aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Buffer resources address < 2 GiB (32-bit offsets with kOOB as the out-of-range marker).
static inline bool fits(size_t bytes) { return bytes < ((size_t)1 << 31); }

static inline int al4(int v) { return (v & 3) == 0; }
static inline EpStore ep_store(float* out, int ldo, const float* bias, const float* res = nullptr) {
  return EpStore{out, ldo, bias, al4(ldo) && aligned16(out) && (!bias || aligned16(bias)) && (!res || aligned16(res)),
                 res};
}
static inline EpWiden ep_widen(float* out, int ldo, int OH, int OW, int st, const float* res = nullptr) {
  return EpWiden{out, ldo, OH, OW, st, al4(ldo) && aligned16(out) && (!res || aligned16(res)), res};
}


// ----------------------------------------------------------------------------
// Host-side launch helpers and tile selection
// ----------------------------------------------------------------------------

// Tile configurations.  Row problems (forward / dgrad: output-stationary, one pass over
// K) and split-K problems (wgrad: K = pixels, split over blocks) have separate tables.
// The heuristics below pick one per shape; dk_debug_set_gemm_config() overrides the
// choice for tuning runs (scripts/gemm_tune.py).
//                 id  BM   BN  BK  WM WN
#define DK_ROW_CONFIGS(X) \
  X(0, 256, 64, 16, 4, 1)  \
  X(1, 128, 64, 16, 2, 1)  \
  X(2, 128, 64, 32, 2, 1)  \
  X(3, 256, 64, 32, 4, 1)  \
  X(4, 128, 128, 16, 2, 2) \
  X(5, 128, 128, 32, 2, 2) \
  X(6, 64, 64, 16, 2, 2)   \
  X(7, 128, 32, 16, 4, 1)  \
  X(8, 64, 64, 32, 2, 2)   \
  X(9, 256, 128, 16, 4, 2) \
  X(10, 64, 64, 64, 2, 2)  \
  X(11, 128, 64, 64, 2, 1) \
  X(12, 64, 128, 16, 2, 2) \
  X(13, 64, 128, 32, 2, 2) \
  X(14, 128, 64, 16, 2, 2) \
  X(15, 128, 64, 32, 2, 2) \
  X(16, 128, 128, 32, 2, 4) \
  X(17, 128, 128, 16, 2, 4)
#define DK_SPLITK_CONFIGS(X) \
  X(0, 64, 64, 16, 2, 2)     \
  X(1, 64, 64, 32, 2, 2)     \
  X(2, 64, 64, 64, 2, 2)     \
  X(3, 128, 128, 16, 2, 2)   \
  X(4, 128, 128, 32, 2, 2)   \
  X(5, 128, 64, 32, 2, 2)    \
  X(6, 64, 128, 32, 2, 2)

struct TileCfg {
  int BM, BN, BK;
};
#define DK_CFG_ENTRY(id, bm, bn, bk, wm, wn) {bm, bn, bk},
static const TileCfg kRowCfg[] = {DK_ROW_CONFIGS(DK_CFG_ENTRY)};
static const TileCfg kSplitCfg[] = {DK_SPLITK_CONFIGS(DK_CFG_ENTRY)};
#undef DK_CFG_ENTRY
static const int kNumRowCfg = sizeof(kRowCfg) / sizeof(kRowCfg[0]);
static const int kNumSplitCfg = sizeof(kSplitCfg) / sizeof(kSplitCfg[0]);

static int g_cfg_override[2] = {-1, -1};  // tuning knob only (see header)
// Split-K grids fill the resident block slots once (g_fill_splits; tuning knob
// dk_debug_set_gemm_config(2, 0/1)).  A persistent tile loop for the row problems was measured
// and dropped (scripts/ab_step.py: 11.77 ms/step with one block per tile, 11.89 / 11.98 with
// 1 / 2 resident waves of persistent blocks, and the loop slowed the one-tile case too).
static int g_fill_splits = 1;
constexpr int kNumCUs = 256;  // MI355X

template <int BM, int BN, int BK, int WM, int WN, template <int, int, int> class LA, class DA,
          template <int, int, int> class LB, class DB, class EP>
static int launch_igemm(const DA& da, const DB& db, const EP& ep, int M, int N, int Ktot, int splits,
                        hipStream_t st,
                        int* splits_used = nullptr) {
  constexpr int NT = 64 * WM * WN;
  using A = LA<BM, BK, NT>;
  using B = LB<BN, BK, NT>;
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  const int KT = cdiv(Ktot, BK);
  if (splits < 1) splits = 1;
  if (splits > KT) splits = KT > 0 ? KT : 1;
  size_t dyn = 0;
  if constexpr (DA::kBnIn && A::kTable) {
    dyn = (size_t)da.C * sizeof(f32x4);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&igemm_f32<BM, BN, BK, WM, WN, A, DA, B, DB, EP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
  }
  if constexpr (DA::kBnBwd) {
    dyn = (size_t)da.bwd.C * 2 * sizeof(f32x4);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&igemm_f32<BM, BN, BK, WM, WN, A, DA, B, DB, EP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
  }
  // resident blocks per CU of this instantiation (queried once; immutable afterwards)
  static int occ = -1;
  if (occ < 0) {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &o, reinterpret_cast<const void*>(&igemm_f32<BM, BN, BK, WM, WN, A, DA, B, DB, EP>), NT, dyn) !=
            hipSuccess || o < 1)
      o = 1;
    occ = o;
  }
  const int slots = occ * kNumCUs;
  if (g_fill_splits && splits_used && splits > 1 && tiles * splits > slots && tiles <= slots) {
    // split-K: no second, partly filled round of blocks (the stem's 64x128 weight-gradient
    // tiles fit 3 per CU: 1024 splits ran as 768 + 256 blocks)
    splits = slots / tiles;
  }
  const int kps = KT > 0 ? cdiv(KT, splits) : 1;
  splits = KT > 0 ? cdiv(KT, kps) : 1;
  if (splits_used) *splits_used = splits;
  if constexpr (EP::kColStats) {
    // an armed in-launch fold of the column statistics (fold_tail.h): rows = M tiles, one
    // channel slice per N tile
    EP e = ep;
    if (!e.part || splits != 1 || !fold_take(e.part, cdiv(M, BM), N, cdiv(N, BN), &e.ft)) e.ft.part = nullptr;
    hipLaunchKernelGGL((igemm_f32<BM, BN, BK, WM, WN, A, DA, B, DB, EP>), dim3(tiles, splits), dim3(NT), dyn, st, da,
                       db, e, M, N, Ktot, kps);
    return fold_status(launch_status(), e.ft);
  }
  hipLaunchKernelGGL((igemm_f32<BM, BN, BK, WM, WN, A, DA, B, DB, EP>), dim3(tiles, splits), dim3(NT), dyn, st, da,
                     db, ep, M, N, Ktot, kps);
  return launch_status();
}

// Row-problem kinds with their own tile choice: plain loaders, and the BN-backward-on-load A
// operand (dk_pwconv_dgrad_bnbwd_f32), whose per-element transform is repeated for every column
// tile -- wide column tiles amortise it.
enum : int { kRowPlain = 0, kRowBnBwd = 1, kRowConv = 2 };  // kRowConv: R x S > 1 image forward

static int row_config(int M, int N, int K, int kind = kRowPlain) {
  if (g_cfg_override[0] >= 0) return g_cfg_override[0];
  (void)M;
  if (kind == kRowBnBwd) {
    // Measured on MI355X (scripts/gemm_tune.py --fused-only, profiles/r01h_gemm_tune_fused.txt)
    if (N <= 64) return 8;                // 64x64x32
    if (N <= 128) return 16;              // 128x128x32, 2x4 waves
    if (N <= 256) return K >= 512 ? 13 : 6;
    return 9;                             // 256x128x16
  }
  // The stem (K = 5*5*4 = 100, 64 filters): 128x64x16 with 2x2 waves, 555 vs 687 us
  // (scripts/gemm_tune.py --only conv0, profiles/r01j_gemm_tune_conv.txt)
  if (kind == kRowConv && K <= 128 && N <= 64) return 14;
  // Measured on MI355X (scripts/gemm_tune.py, profiles/r01c_gemm_tune.md): 64x64 tiles win on
  // every ResNet shape; a deeper k-tile pays once the reduction is longer than ~100.
  return K <= 128 ? 6 : 8;
}

// Output-stationary problems (fwd / dgrad).
template <template <int, int, int> class LA, class DA, template <int, int, int> class LB, class DB, class EP,
          int KIND = kRowPlain>
static int igemm_rows(const DA& da, const DB& db, const EP& ep, int M, int N, int Ktot, hipStream_t st) {
  switch (row_config(M, N, Ktot, KIND)) {
#define DK_CASE(id, bm, bn, bk, wm, wn) \
  case id:                              \
    return launch_igemm<bm, bn, bk, wm, wn, LA, DA, LB, DB, EP>(da, db, ep, M, N, Ktot, 1, st);
    DK_ROW_CONFIGS(DK_CASE)
#undef DK_CASE
    default:
      return DK_ERR_ARGS;
  }
}

// Reduction-heavy problems (wgrad): split K over enough blocks to fill the chip.
static int splitk_config(int M, int N, int Kred) {
  if (g_cfg_override[1] >= 0) return g_cfg_override[1];
  (void)Kred;
  // Wide column tiles when M <= 64 < N: the A operand (for the stem the BN-backward-on-load dy,
  // formed from 2 x 822 MB) is streamed half as often -- the stem (N = R*S*Cp = 100) in one
  // column tile; BASELINE config 2's 3x3 conv (N = 576): 594 vs 628 us (profiles/r01j_gemm_tune_all.txt).
  if (M <= 64 && N > 64) return 6;  // 64x128x32
  return 1;  // 64x64x32: best or within 3% of best on every other measured wgrad shape
}

// Blocks a split-K weight gradient aims for (tuning knob DORKNET_WGRAD_BLOCKS, read once).
static int wgrad_target_blocks() {
  static int v = -1;
  if (v < 0) {
    const char* s = getenv("DORKNET_WGRAD_BLOCKS");
    v = (s && atoi(s) > 0) ? atoi(s) : 1024;
  }
  return v;
}

static int wgrad_splits(int M, int N, int Kred, const TileCfg& c) {
  const int tiles = cdiv(M, c.BM) * cdiv(N, c.BN);
  const int KT = cdiv(Kred, c.BK);
  int splits = cdiv(wgrad_target_blocks(), tiles);
  if (splits > KT) splits = KT;
  if (splits < 1) splits = 1;
  const int kps = cdiv(KT, splits);
  return cdiv(KT, kps);
}

template <template <int, int, int> class LA, class DA, template <int, int, int> class LB, class DB>
static int igemm_splitk(const DA& da, const DB& db, float* ws, int M, int N, int Kred, hipStream_t st,
                        int* splits_out) {
  const int id = splitk_config(M, N, Kred);
  if (id < 0 || id >= kNumSplitCfg) return DK_ERR_ARGS;
  const int splits = wgrad_splits(M, N, Kred, kSplitCfg[id]);  // the workspace's upper bound
  *splits_out = splits;
  EpPartial ep{ws, M, N, al4(N) && aligned16(ws)};
  switch (id) {
#define DK_CASE(cid, bm, bn, bk, wm, wn) \
  case cid:                              \
    return launch_igemm<bm, bn, bk, wm, wn, LA, DA, LB, DB, EpPartial>(da, db, ep, M, N, Kred, splits, st, splits_out);
    DK_SPLITK_CONFIGS(DK_CASE)
#undef DK_CASE
    default:
      return DK_ERR_ARGS;
  }
}

static size_t splitk_ws_bytes(int M, int N, int Kred) {
  int id = splitk_config(M, N, Kred);
  if (id < 0 || id >= kNumSplitCfg) id = 0;
  return (size_t)wgrad_splits(M, N, Kred, kSplitCfg[id]) * (size_t)M * (size_t)N * sizeof(float);
}

// Weight re-layouts (tiny; run once per call on the caller's stream).
__global__ void w_kcrs_to_krsc_kernel(const float* __restrict__ w, int K, int C, int R, int S, int Cp,
                                      float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // over K*R*S*Cp
  const int total = K * R * S * Cp;
  if (idx >= total) return;
  const int c = idx % Cp;
  int t = idx / Cp;
  const int s = t % S;
  t /= S;
  const int r = t % R;
  const int k = t / R;
  out[idx] = c < C ? w[(((size_t)k * C + c) * R + r) * S + s] : 0.f;
}

__global__ void w_kcrs_to_crsk_kernel(const float* __restrict__ w, int K, int C, int R, int S,
                                      float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // over C*R*S*K
  const int total = K * R * S * C;
  if (idx >= total) return;
  const int k = idx % K;
  int t = idx / K;
  const int s = t % S;
  t /= S;
  const int r = t % R;
  const int c = t / R;
  out[idx] = w[(((size_t)k * C + c) * R + r) * S + s];
}

// Taps of sub-pixel phase a along an axis of length-R filters (stride st, padding pad): r0 + st*t.
__host__ __device__ __forceinline__ int phase_r0(int a, int st, int pad) { return (a + pad) % st; }
__host__ __device__ __forceinline__ int phase_taps(int a, int R, int st, int pad) {
  const int r0 = phase_r0(a, st, pad);
  return r0 < R ? (R - r0 + st - 1) / st : 0;
}
// Offset (floats) of phase (a, b)'s sub-filter block: the blocks are laid out in (a, b) order.
__host__ __device__ __forceinline__ size_t phase_block_offset(int a, int b, int C, int R, int S, int st, int pad,
                                                              int Kp) {
  size_t off = 0;
  for (int i = 0; i < a * st + b; ++i)
    off += (size_t)C * phase_taps(i / st, R, st, pad) * phase_taps(i % st, S, st, pad) * Kp;
  return off;
}

// Sub-pixel phase sub-filters of a stride-st dgrad: for phase (a, b) the taps r = r0(a) + st*r',
// s = s0(b) + st*s' as a [C][R'][S'][Kp] matrix (Kp = K rounded up to 4, zero-filled).
__global__ void w_phase_kernel(const float* __restrict__ w, int K, int C, int R, int S, int st, int pad, int Kp,
                               float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // over C * R * S * Kp
  if (idx >= C * R * S * Kp) return;
  const int k = idx % Kp;
  int t = idx / Kp;
  const int s_ = t % S;
  t /= S;
  const int r = t % R;
  const int c = t / R;
  const int a = ((r - pad) % st + st) % st, b = ((s_ - pad) % st + st) % st;
  const int r0 = phase_r0(a, st, pad), s0 = phase_r0(b, st, pad);
  const int Rp = phase_taps(a, R, st, pad), Sp = phase_taps(b, S, st, pad);
  const int rp = (r - r0) / st, sp = (s_ - s0) / st;
  out[phase_block_offset(a, b, C, R, S, st, pad, Kp) + ((size_t)(c * Rp + rp) * Sp + sp) * Kp + k] =
      k < K ? w[(((size_t)k * C + c) * R + r) * S + s_] : 0.f;
}

// rows x ld matrix; ext = extent of the non-reduction index (rows for a K-contiguous
// operand, valid columns for a row-contiguous one).
static inline MatDesc mat(const float* p, int rows, int ld, int ext) {
  return MatDesc{p, (uint32_t)((size_t)rows * ld * sizeof(float)), ld, ext};
}
static inline bool vec_ok(const MatDesc& d, int kext, int iext) {
  return d.ld % 4 == 0 && kext % 4 == 0 && iext % 4 == 0 && aligned16(d.p);
}

// Magic multiplier for q = umulhi(n, m) == n / d (exact for n * d < 2^32); 0 = not usable.
static inline uint32_t magic(long long d, long long nmax) {
  if (d <= 1 || nmax * d >= (1ll << 32)) return 0;
  return (uint32_t)((1ull << 32) / (unsigned long long)d + 1);
}
template <class Dsc>
static inline Dsc set_magics(Dsc d) {
  const long long ktot = (long long)d.R * d.S * d.C;
  d.mC = magic(d.C, ktot);
  d.mS = magic(d.S, ktot);
  d.mOW = magic(d.OW, d.M);
  d.mOH = magic(d.OH, d.M);
  return d;
}
static inline ImgDesc img(const float* x, int N, int H, int W, int C, int OH, int OW, int R, int S, int sa, int dr,
                          int off, int M) {
  return set_magics(
      ImgDesc{x, (uint32_t)((size_t)N * H * W * C * sizeof(float)), H, W, C, OH, OW, R, S, sa, dr, off, off, M});
}
// A pointwise (1x1, stride sa) view: k = channel.
static inline ImgDescE<float, true> img1(const float* x, int N, int H, int W, int C, int OH, int OW, int sa, int M) {
  return set_magics(ImgDescE<float, true>{x, (uint32_t)((size_t)N * H * W * C * sizeof(float)), H, W, C, OH, OW, 1,
                                          1, sa, 1, 0, 0, M});
}

}  // namespace dk

using namespace dk;

// ============================================================================
// C ABI
// ============================================================================

// Tuning knob: kind 0 = row problems (fwd/dgrad), 1 = split-K (wgrad); cfg -1 = heuristic.
// Returns the number of configurations of that kind.  Not thread-safe; for tuning runs.
DK_API int dk_debug_set_gemm_config(int kind, int cfg) {
  if (kind == 2) {
    g_fill_splits = cfg < 0 ? 1 : cfg;
    return 0;
  }
  if (kind == 3) {  // streaming pointwise kernels (pw_stream.hip) on / off
    pw_stream_set(cfg < 0 ? 1 : cfg);
    return 0;
  }
  if (kind < 0 || kind > 1) return -1;
  g_cfg_override[kind] = cfg;
  return kind == 0 ? kNumRowCfg : kNumSplitCfg;
}

DK_API int dk_conv_weight_krsc_f32(const float* w_kcrs, int K, int C, int R, int S, int Cp, float* w_krsc,
                                   void* stream) {
  const int total = K * R * S * Cp;
  hipLaunchKernelGGL(w_kcrs_to_krsc_kernel, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), w_kcrs, K, C, R,
                     S, Cp, w_krsc);
  return launch_status();
}

DK_API int dk_conv_weight_crsk_f32(const float* w_kcrs, int K, int C, int R, int S, float* w_crsk, void* stream) {
  const int total = K * R * S * C;
  hipLaunchKernelGGL(w_kcrs_to_crsk_kernel, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), w_kcrs, K, C, R,
                     S, w_crsk);
  return launch_status();
}

// y[n,oh,ow,k] = sum_{r,s,c} x[n, oh*stride + r - pad, ow*stride + s - pad, c] * w[k][r][s][c] (+ bias[k])
template <class E, bool K1>
static inline ImgBnDescE<E, K1> with_bn(const ImgDescE<E, K1>& d, const float* mean, const float* invstd,
                                        const float* gamma, const float* beta, int relu) {
  ImgBnDescE<E, K1> o;
  static_cast<ImgDescE<E, K1>&>(o) = d;
  o.bn = BnIn{mean, invstd, gamma, beta, relu};
  return o;
}
static inline bool bn_ok(const float* mean, const float* invstd, const float* gamma, const float* beta) {
  return mean && invstd && gamma && beta && aligned16(mean) && aligned16(invstd) && aligned16(gamma) &&
         aligned16(beta);
}

template <class D>
static int conv_fwd(const D& a, const float* w_krsc, int K, int Ktot, const float* bias, float* y, void* stream,
                    double* stats = nullptr) {
  if constexpr (D::kBnIn) {
    if (a.C > 2048) return DK_ERR_ARGS;  // the LDS parameter table holds <= 2048 channels (32 KB)
  }
  MatDesc b = mat(w_krsc, K, Ktot, K);
  constexpr int kind = D::k1x1 ? kRowPlain : kRowConv;
  if (stats) {
    EpStoreStats ep;
    static_cast<EpStore&>(ep) = ep_store(y, K, bias);
    ep.part = stats;
    return igemm_rows<LdImgKC, D, LdMatKC, MatDesc, EpStoreStats, kind>(a, b, ep, a.M, K, Ktot, as_stream(stream));
  }
  EpStore ep = ep_store(y, K, bias);
  return igemm_rows<LdImgKC, D, LdMatKC, MatDesc, EpStore, kind>(a, b, ep, a.M, K, Ktot, as_stream(stream));
}

// Rows of BatchNorm partial statistics a *_fwd_ex_f32 call writes (one per output tile row).
static int stats_rows(int M, int N, int Ktot, int kind = kRowPlain) {
  return cdiv(M, kRowCfg[row_config(M, N, Ktot, kind)].BM);
}

// Forward with an optional input BatchNorm (bn_mean != NULL, see *_bnx_*) and optional output
// statistics (stats != NULL: stats_rows x 2 x K doubles).
template <class D0>
static int conv_fwd_ex(const D0& base, const float* w, int K, int Ktot, const float* bias, float* y,
                       const float* bn_mean, const float* bn_invstd, const float* bn_gamma, const float* bn_beta,
                       int bn_relu, double* stats, void* stream) {
  if (bn_mean) {
    if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
    return conv_fwd(with_bn(base, bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu), w, K, Ktot, bias, y, stream, stats);
  }
  return conv_fwd(base, w, K, Ktot, bias, y, stream, stats);
}

DK_API int dk_conv2d_fwd_f32(const float* x, int N, int H, int W, int C, const float* w_krsc, int K, int R, int S,
                             int stride, int pad, const float* bias, float* y, int OH, int OW, void* stream) {
  if (C % 4 || !aligned16(x) || !aligned16(w_krsc) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  return conv_fwd(img(x, N, H, W, C, OH, OW, R, S, stride, 1, -pad, N * OH * OW), w_krsc, K, R * S * C, bias, y,
                  stream);
}

DK_API int dk_conv2d_fwd_bnx_f32(const float* x, int N, int H, int W, int C, const float* w_krsc, int K, int R, int S,
                                 int stride, int pad, const float* bias, float* y, int OH, int OW,
                                 const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                 const float* bn_beta, int bn_relu, void* stream) {
  if (C % 4 || !aligned16(x) || !aligned16(w_krsc) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
  return conv_fwd(with_bn(img(x, N, H, W, C, OH, OW, R, S, stride, 1, -pad, N * OH * OW), bn_mean, bn_invstd,
                          bn_gamma, bn_beta, bn_relu),
                  w_krsc, K, R * S * C, bias, y, stream);
}

DK_API int dk_conv2d_fwd_stats_rows(int N, int OH, int OW, int K, int C, int R, int S) {
  return stats_rows(N * OH * OW, K, R * S * C, kRowConv);
}

// Forward with optional BN on load (bn_mean != NULL) and optional output statistics
// (stats != NULL: dk_conv2d_fwd_stats_rows() x 2 x K doubles, for dk_bn_stats_from_partials_f32).
DK_API int dk_conv2d_fwd_ex_f32(const float* x, int N, int H, int W, int C, const float* w_krsc, int K, int R, int S,
                                int stride, int pad, const float* bias, float* y, int OH, int OW,
                                const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                const float* bn_beta, int bn_relu, double* stats, void* stream) {
  if (C % 4 || !aligned16(x) || !aligned16(w_krsc) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  return conv_fwd_ex(img(x, N, H, W, C, OH, OW, R, S, stride, 1, -pad, N * OH * OW), w_krsc, K, R * S * C, bias, y,
                     bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu, stats, stream);
}

// Stride-1 dgrad as an implicit GEMM: dx[n,h,w,c] = sum_{r,s,k} dy[n, h+pad-r, w+pad-s, k] * w[k][c][r][s]
DK_API int dk_conv2d_dgrad_f32(const float* dy, int N, int OH, int OW, int K, const float* w_crsk, int C, int R,
                               int S, int pad, float* dx, int H, int W, void* stream) {
  if (K % 4 || !aligned16(dy) || !aligned16(w_crsk) || !fits((size_t)N * OH * OW * K * 4)) return DK_ERR_ARGS;
  ImgDesc a = img(dy, N, OH, OW, K, H, W, R, S, 1, -1, pad, N * H * W);
  const int Ktot = R * S * K;
  MatDesc b = mat(w_crsk, C, Ktot, C);
  EpStore ep = ep_store(dx, C, nullptr);
  return igemm_rows<LdImgKC, ImgDesc, LdMatKC, MatDesc, EpStore>(a, b, ep, N * H * W, C, Ktot, as_stream(stream));
}

// Sub-pixel phase geometry of a stride-st, pad-p correlation's input gradient along one axis:
// phase a's taps are r0 + st*t (t < Rp), reading dy row i + nb0 - t for dx row st*i + a.
struct PhaseAxis {
  int r0, Rp, nb0, Op;
};
static inline PhaseAxis phase_axis(int a, int R, int st, int pad, int L) {
  PhaseAxis p;
  p.r0 = phase_r0(a, st, pad);
  p.Rp = phase_taps(a, R, st, pad);
  p.nb0 = (a + pad - p.r0) / st;
  p.Op = a < L ? (L - a + st - 1) / st : 0;
  return p;
}

DK_API size_t dk_conv2d_dgrad_phase_workspace_bytes(int K, int C, int R, int S, int stride) {
  if (K < 1 || C < 1 || R < 1 || S < 1 || stride < 1) return 0;
  const size_t kp = (size_t)((K + 3) / 4 * 4);
  return (size_t)C * R * S * kp * sizeof(float);
}

// Input gradient of any-stride convolution as one implicit GEMM per sub-pixel phase (replaces
// cp.dot(dy, W_flat) + row2im, convolution.py:101-117 / :205-222: no column matrix, no atomics):
// phase (a, b) is a stride-1 correlation of dy with its sub-filter, written to the dx pixels
// (st*i + a, st*j + b).  dy has Kp = K rounded up to 4 channels (zero-padded by the caller when
// K % 4 != 0); phases with no taps (R or S < stride) write zeros.
DK_API int dk_conv2d_dgrad_phase_f32(const float* dy, int N, int OH, int OW, int Kp, int K, const float* w_kcrs,
                                     int C, int R, int S, int stride, int pad, float* dx, int H, int W, void* ws,
                                     size_t ws_bytes, void* stream) {
  if (Kp % 4 || Kp < K || stride < 1 || stride > 8 || N < 1 || C < 1 || !aligned16(dy) || !aligned16(ws))
    return DK_ERR_ARGS;
  if (ws_bytes < dk_conv2d_dgrad_phase_workspace_bytes(K, C, R, S, stride) || Kp != (K + 3) / 4 * 4)
    return DK_ERR_WORKSPACE;
  if (!fits((size_t)N * OH * OW * Kp * 4) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  const hipStream_t st = as_stream(stream);
  float* wsub = static_cast<float*>(ws);
  const int total = C * R * S * Kp;
  hipLaunchKernelGGL(w_phase_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, w_kcrs, K, C, R, S, stride, pad, Kp,
                     wsub);
  int rc = launch_status();
  if (rc) return rc;
  for (int a = 0; a < stride; ++a)
    for (int b = 0; b < stride; ++b) {
      const PhaseAxis pa = phase_axis(a, R, stride, pad, H), pb = phase_axis(b, S, stride, pad, W);
      if (pa.Op == 0 || pb.Op == 0) continue;  // no dx pixels of this phase
      const int M = N * pa.Op * pb.Op;
      ImgDesc d = img(dy, N, OH, OW, Kp, pa.Op, pb.Op, pa.Rp, pb.Rp, 1, -1, pa.nb0, M);
      d.offw = pb.nb0;
      const int Ktot = pa.Rp * pb.Rp * Kp;
      const float* wp = wsub + phase_block_offset(a, b, C, R, S, stride, pad, Kp);
      MatDesc bm = mat(wp, C, Ktot > 0 ? Ktot : 4, C);
      EpPhase ep{dx, C, pa.Op, pb.Op, H, W, stride, a, b, al4(C) && aligned16(dx)};
      rc = igemm_rows<LdImgKC, ImgDesc, LdMatKC, MatDesc, EpPhase>(d, bm, ep, M, C, Ktot, st);
      if (rc) return rc;
    }
  return 0;
}

DK_API size_t dk_conv2d_wgrad_workspace_bytes(int N, int OH, int OW, int K, int Cp, int R, int S) {
  return splitk_ws_bytes(K, R * S * Cp, N * OH * OW);
}

// dw[k][c][r][s] = sum_{n,oh,ow} dy[n,oh,ow,k] * x[n, oh*stride + r - pad, ow*stride + s - pad, c]  (+ l2 * w)
// Weight gradient through the split-K engine: part = dy^T . im2col(x) then the fixed-order
// reduce (+ l2 * w) into the KCRS (mode 1) or [K][C] (mode 0) layout.
template <class D>
static int wgrad(const float* dy, const D& b, int K, int Ncol, const float* w, float l2, float* dw, int mode, int C,
                 int Cp, int R, int S, void* ws, size_t ws_bytes, void* stream) {
  const int Kred = b.M;
  if (!fits((size_t)Kred * K * 4)) return DK_ERR_ARGS;
  if (ws_bytes < splitk_ws_bytes(K, Ncol, Kred)) return DK_ERR_WORKSPACE;
  MatDesc a = mat(dy, Kred, K, K);
  int splits = 1;
  float* part = static_cast<float*>(ws);
  const hipStream_t st = as_stream(stream);
  int rc = vec_ok(a, 4, K) ? igemm_splitk<LdMatIC, MatDesc, LdImgIC, D>(a, b, part, K, Ncol, Kred, st, &splits)
                           : igemm_splitk<LdMatIC1, MatDesc, LdImgIC, D>(a, b, part, K, Ncol, Kred, st, &splits);
  if (rc) return rc;
  return splitk_reduce(part, splits, K, Ncol, dw, w, l2, mode, C, Cp, R, S, st);
}

DK_API int dk_conv2d_wgrad_f32(const float* dy, const float* x, int N, int H, int W, int Cp, int C, int K, int R,
                               int S, int stride, int pad, int OH, int OW, const float* w_kcrs, float l2,
                               float* dw_kcrs, void* ws, size_t ws_bytes, void* stream) {
  if (Cp % 4 || !aligned16(x) || !fits((size_t)N * H * W * Cp * 4)) return DK_ERR_ARGS;
  return wgrad(dy, img(x, N, H, W, Cp, OH, OW, R, S, stride, 1, -pad, N * OH * OW), K, R * S * Cp, w_kcrs, l2,
               dw_kcrs, 1, C, Cp, R, S, ws, ws_bytes, stream);
}

// Weight gradient with the following BatchNorm's backward applied as dy is loaded: g is the
// gradient w.r.t. that BN's (+ReLU) output, bn_x its raw input (= this layer's output), out_* /
// k12 its parameters and folded coefficients -- dy = dk_bn_bwd_apply_f32(bn_x, g) bit for bit,
// never stored (the stem, whose input gradient is not needed: the apply pass over its
// 64 x 112 x 112 output per image and the re-read of dy become one read of g and bn_x).
// bn_* (optional): this layer's input BatchNorm applied on load, as dk_conv2d_wgrad_bnx_f32.
template <class D>
static int wgrad_bnbwd(const float* g, const float* bn_x, const D& b, int K, int Ncol, const BnBwdIn& bw,
                       const float* w, float l2, float* dw, int C, int Cp, int R, int S, void* ws, size_t ws_bytes,
                       void* stream) {
  const int Kred = b.M;
  if (!fits((size_t)Kred * K * 4)) return DK_ERR_ARGS;
  if (ws_bytes < splitk_ws_bytes(K, Ncol, Kred)) return DK_ERR_WORKSPACE;
  MatDesc a0 = mat(g, Kred, K, K);
  if (!vec_ok(a0, 4, K) || !aligned16(bn_x)) return DK_ERR_ARGS;
  MatBwdDesc a;
  static_cast<MatDesc&>(a) = a0;
  a.x = bn_x;
  a.bwd = bw;
  a.dy_out = nullptr;
  int splits = 1;
  float* part = static_cast<float*>(ws);
  const hipStream_t st = as_stream(stream);
  int rc = igemm_splitk<LdMatIC, MatBwdDesc, LdImgIC, D>(a, b, part, K, Ncol, Kred, st, &splits);
  if (rc) return rc;
  return splitk_reduce(part, splits, K, Ncol, dw, w, l2, 1, C, Cp, R, S, st);
}

DK_API int dk_conv2d_wgrad_bnbwd_f32(const float* g, const float* bn_x, const float* x, int N, int H, int W, int Cp,
                                     int C, int K,
                                     int R, int S, int stride, int pad, int OH, int OW, const float* out_mean,
                                     const float* out_invstd, const float* out_gamma, const float* out_beta,
                                     int out_relu, const float* k12, const float* w_kcrs, float l2, float* dw_kcrs,
                                     void* ws, size_t ws_bytes, const float* bn_mean, const float* bn_invstd,
                                     const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream) {
  if (Cp % 4 || K % 4 || !aligned16(x) || !fits((size_t)N * H * W * Cp * 4)) return DK_ERR_ARGS;
  if (!out_mean || !out_invstd || !out_gamma || !out_beta || !k12) return DK_ERR_ARGS;
  const BnBwdIn bw{out_mean, out_invstd, out_gamma, out_beta, k12, out_relu, K};
  if (bn_mean) {
    if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
    return wgrad_bnbwd(g, bn_x,
                       with_bn(img(x, N, H, W, Cp, OH, OW, R, S, stride, 1, -pad, N * OH * OW), bn_mean,
                               bn_invstd, bn_gamma, bn_beta, bn_relu),
                       K, R * S * Cp, bw, w_kcrs, l2, dw_kcrs, C, Cp, R, S, ws, ws_bytes, stream);
  }
  return wgrad_bnbwd(g, bn_x, img(x, N, H, W, Cp, OH, OW, R, S, stride, 1, -pad, N * OH * OW), K,
                     R * S * Cp, bw, w_kcrs, l2, dw_kcrs, C, Cp, R, S, ws, ws_bytes, stream);
}

DK_API int dk_conv2d_wgrad_bnx_f32(const float* dy, const float* x, int N, int H, int W, int Cp, int C, int K, int R,
                                   int S, int stride, int pad, int OH, int OW, const float* w_kcrs, float l2,
                                   float* dw_kcrs, void* ws, size_t ws_bytes, const float* bn_mean,
                                   const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu,
                                   void* stream) {
  if (Cp % 4 || !aligned16(x) || !fits((size_t)N * H * W * Cp * 4)) return DK_ERR_ARGS;
  if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
  return wgrad(dy,
               with_bn(img(x, N, H, W, Cp, OH, OW, R, S, stride, 1, -pad, N * OH * OW), bn_mean, bn_invstd, bn_gamma,
                       bn_beta, bn_relu),
               K, R * S * Cp, w_kcrs, l2, dw_kcrs, 1, C, Cp, R, S, ws, ws_bytes, stream);
}

// Pointwise (1x1) forward with optional stride-s subsampling (pointwise_convolution.py:46-55):
// y[n,oh,ow,k] = sum_c x[n, oh*s, ow*s, c] * w[k][c] (+ bias)
DK_API int dk_pwconv_fwd_f32(const float* x, int N, int H, int W, int C, const float* w_kc, int K, int stride,
                             const float* bias, float* y, int OH, int OW, void* stream) {
  if (!fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  MatDesc b = mat(w_kc, K, C, K);
  EpStore ep = ep_store(y, K, bias);
  if (C % 4 || !aligned16(x) || !aligned16(w_kc)) {
    // Unaligned channel count: scalar loads, stride 1 only (the rows are then a plain matrix).
    if (stride != 1) return DK_ERR_ARGS;
    MatDesc a = mat(x, N * H * W, C, N * H * W);
    return igemm_rows<LdMatKC1, MatDesc, LdMatKC1, MatDesc, EpStore>(a, b, ep, N * H * W, K, C, as_stream(stream));
  }
  return conv_fwd(img1(x, N, H, W, C, OH, OW, stride, N * OH * OW), w_kc, K, C, bias, y, stream);
}

// The same with x = the raw output of the previous layer and y = pw(bn(x)) (+ReLU inside).
DK_API int dk_pwconv_fwd_bnx_f32(const float* x, int N, int H, int W, int C, const float* w_kc, int K, int stride,
                                 const float* bias, float* y, int OH, int OW, const float* bn_mean,
                                 const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu,
                                 void* stream) {
  if (C % 4 || !aligned16(x) || !aligned16(w_kc) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
  return conv_fwd(with_bn(img1(x, N, H, W, C, OH, OW, stride, N * OH * OW), bn_mean, bn_invstd, bn_gamma,
                          bn_beta, bn_relu),
                  w_kc, K, C, bias, y, stream);
}

DK_API int dk_pwconv_fwd_stats_rows(int N, int OH, int OW, int K, int C) {
  const int M = N * OH * OW;
  // (the input extent does not change the choice for the shapes the network uses)
  if (pw_stream_fwd_ok(K, C, M, 0)) return pw_stream_fwd_rows(M, K);
  return stats_rows(M, K, C);
}

DK_API int dk_pwconv_fwd_ex_f32(const float* x, int N, int H, int W, int C, const float* w_kc, int K, int stride,
                                const float* bias, float* y, int OH, int OW, const float* bn_mean,
                                const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu,
                                double* stats, void* stream) {
  if (C % 4 || !aligned16(x) || !aligned16(w_kc) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  if (pw_stream_fwd_ok(K, C, N * OH * OW, (size_t)N * H * W * C * 4) && (!bn_mean || bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)))
    // K = C = 64 / 128: the persistent streaming kernel (pw_stream.hip), bit-identical outputs
  {
    FoldTail ft;
    if (stats) fold_take(stats, pw_stream_fwd_rows(N * OH * OW, K), K, 1, &ft);
    return fold_status(pw_stream_fwd(x, N, H, W, stride, OH, OW, w_kc, K, bias, y, bn_mean, bn_invstd, bn_gamma,
                                     bn_beta, bn_relu, stats, as_stream(stream), stats ? &ft : nullptr),
                       stats ? ft : FoldTail{});
  }
  return conv_fwd_ex(img1(x, N, H, W, C, OH, OW, stride, N * OH * OW), w_kc, K, C, bias, y, bn_mean,
                     bn_invstd, bn_gamma, bn_beta, bn_relu, stats, stream);
}

// Pointwise dgrad (pointwise_convolution.py:65-72): dx_rows = dy_rows . W; for stride > 1 the
// result is widened to (OH*s, OW*s) with zeros off the sampling lattice.
DK_API int dk_pwconv_dgrad_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kc, int C, int stride,
                               float* dx, void* stream) {
  const int M = N * OH * OW;
  if (!fits((size_t)M * K * 4)) return DK_ERR_ARGS;
  MatDesc a = mat(dy, M, K, M);
  MatDesc b = mat(w_kc, K, C, C);
  const hipStream_t st = as_stream(stream);
  const bool vec = vec_ok(a, K, 4) && vec_ok(b, 4, C);
  if (stride == 1) {
    EpStore ep = ep_store(dx, C, nullptr);
    if (vec) return igemm_rows<LdMatKC, MatDesc, LdMatIC, MatDesc, EpStore>(a, b, ep, M, C, K, st);
    return igemm_rows<LdMatKC1, MatDesc, LdMatIC1, MatDesc, EpStore>(a, b, ep, M, C, K, st);
  }
  EpWiden ep = ep_widen(dx, C, OH, OW, stride);
  if (vec) return igemm_rows<LdMatKC, MatDesc, LdMatIC, MatDesc, EpWiden>(a, b, ep, M, C, K, st);
  return igemm_rows<LdMatKC1, MatDesc, LdMatIC1, MatDesc, EpWiden>(a, b, ep, M, C, K, st);
}

DK_API int dk_pwconv_dgrad_stats_rows(int N, int OH, int OW, int K, int C) { return stats_rows(N * OH * OW, C, K); }
DK_API int dk_pwconv_dgrad_bnbwd_stats_rows(int N, int OH, int OW, int K, int C) {
  const int M = N * OH * OW;
  if (pw_stream_dgrad_ok(K, C, M)) return pw_stream_dgrad_rows(M);
  return stats_rows(M, C, K, kRowBnBwd);
}

// dgrad + the BN-backward partial sums of the BatchNorm whose output this layer consumed
// (bn_x = that BN's raw input, on the dx grid; part: dk_pwconv_dgrad_stats_rows() x 2 x C).
DK_API int dk_pwconv_dgrad_ex_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kc, int C, int stride,
                                  float* dx, const float* residual, const float* bn_x, const float* bn_mean,
                                  const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu,
                                  double* part, void* stream) {
  const int M = N * OH * OW;
  if (!fits((size_t)M * K * 4) || (part != nullptr) != (bn_x != nullptr)) return DK_ERR_ARGS;
  if (part && (!bn_mean || !bn_invstd || !bn_gamma || !bn_beta)) return DK_ERR_ARGS;
  if (part && residual && stride != 1) return DK_ERR_ARGS;  // off-lattice residual terms would need reducing
  MatDesc a = mat(dy, M, K, M);
  MatDesc b = mat(w_kc, K, C, C);
  const hipStream_t st = as_stream(stream);
  const bool vec = vec_ok(a, K, 4) && vec_ok(b, 4, C);
#define DK_ROWS(EPT, ep)                                                              \
  return vec ? igemm_rows<LdMatKC, MatDesc, LdMatIC, MatDesc, EPT>(a, b, ep, M, C, K, st) \
             : igemm_rows<LdMatKC1, MatDesc, LdMatIC1, MatDesc, EPT>(a, b, ep, M, C, K, st)
  if (!part) {
    if (stride == 1) {
      EpStore ep = ep_store(dx, C, nullptr, residual);
      DK_ROWS(EpStore, ep);
    }
    EpWiden ep = ep_widen(dx, C, OH, OW, stride, residual);
    DK_ROWS(EpWiden, ep);
  }
  const BnIn bn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
  const int xv4 = aligned16(bn_x) && bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta);
  if (stride == 1) {
    EpStoreBnBwd ep;
    static_cast<EpStore&>(ep) = ep_store(dx, C, nullptr, residual);
    ep.v4 = ep.v4 && xv4;
    ep.part = part;
    ep.xbn = bn_x;
    ep.bn = bn;
    DK_ROWS(EpStoreBnBwd, ep);
  }
  EpWidenBnBwd ep;
  static_cast<EpWiden&>(ep) = ep_widen(dx, C, OH, OW, stride);
  ep.v4 = ep.v4 && xv4;
  ep.part = part;
  ep.xbn = bn_x;
  ep.bn = bn;
  DK_ROWS(EpWidenBnBwd, ep);
#undef DK_ROWS
}

// dk_pwconv_dgrad_ex_f32 with the input BN's partials for stride > 1, the widened gradient kept
// compact (EpLatticeBnBwd): dx_lat[n][oh][ow][c] = the widened dx at (n, s*oh, s*ow, c), the
// rest of the widened grid being zero; part has dk_pwconv_dgrad_stats_rows() rows.
DK_API int dk_pwconv_dgrad_lattice_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kc, int C,
                                       int stride, float* dx_lat, const float* bn_x, const float* bn_mean,
                                       const float* bn_invstd, const float* bn_gamma, const float* bn_beta,
                                       int bn_relu, double* part, void* stream) {
  const int M = N * OH * OW;
  if (!fits((size_t)M * K * 4) || !fits((size_t)M * C * 4) || stride < 2 || !dx_lat || !bn_x || !part)
    return DK_ERR_ARGS;
  if (!bn_mean || !bn_invstd || !bn_gamma || !bn_beta) return DK_ERR_ARGS;
  MatDesc a = mat(dy, M, K, M);
  MatDesc b = mat(w_kc, K, C, C);
  const hipStream_t st = as_stream(stream);
  const bool vec = vec_ok(a, K, 4) && vec_ok(b, 4, C);
  EpLatticeBnBwd ep;
  static_cast<EpWiden&>(ep) = ep_widen(dx_lat, C, OH, OW, stride);
  ep.v4 = ep.v4 && aligned16(bn_x) && bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta);
  ep.part = part;
  ep.xbn = bn_x;
  ep.bn = BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
  return vec ? igemm_rows<LdMatKC, MatDesc, LdMatIC, MatDesc, EpLatticeBnBwd>(a, b, ep, M, C, K, st)
             : igemm_rows<LdMatKC1, MatDesc, LdMatIC1, MatDesc, EpLatticeBnBwd>(a, b, ep, M, C, K, st);
}

// dgrad of a stride-1 pointwise layer whose output fed a BatchNorm (+ReLU), with that BN's
// backward apply (dk_bn_bwd_apply_f32) done on load: g = the gradient w.r.t. the BN(+ReLU)
// output, bn_x = the BN's raw input (= this layer's output), k12 from
// dk_bn_bwd_from_partials_f32.  dy_out (nullable) receives dy = the gradient w.r.t. bn_x,
// bit-identical to dk_bn_bwd_apply_f32's, for this layer's weight gradient.  The epilogue
// options (residual, the partials of the BN before this layer) are those of
// dk_pwconv_dgrad_ex_f32 at stride 1; part has dk_pwconv_dgrad_bnbwd_stats_rows() rows.
DK_API int dk_pwconv_dgrad_bnbwd_f32(const float* g, const float* bn_x, int N, int OH, int OW, int K,
                                     const float* out_mean, const float* out_invstd, const float* out_gamma,
                                     const float* out_beta, int out_relu, const float* k12, float* dy_out,
                                     const float* w_kc, int C, float* dx, const float* residual, const float* x,
                                     const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                     const float* bn_beta, int bn_relu, double* part, void* stream) {
  const int M = N * OH * OW;
  if (!fits((size_t)M * K * 4) || (part != nullptr) != (x != nullptr)) return DK_ERR_ARGS;
  if (part && (!bn_mean || !bn_invstd || !bn_gamma || !bn_beta)) return DK_ERR_ARGS;
  if (!out_mean || !out_invstd || !out_gamma || !out_beta || !k12 || !bn_x) return DK_ERR_ARGS;
  MatBwdDesc a;
  static_cast<MatDesc&>(a) = mat(g, M, K, M);
  a.x = bn_x;
  a.bwd = BnBwdIn{out_mean, out_invstd, out_gamma, out_beta, k12, out_relu, K};
  a.dy_out = dy_out;
  MatDesc b = mat(w_kc, K, C, C);
  const hipStream_t st = as_stream(stream);
  // 16-byte loads of g, bn_x and dy_out; the LDS table holds 2 float4 per channel
  if (!vec_ok(b, 4, C) || K % 4 || !aligned16(g) || !aligned16(bn_x) || (dy_out && !aligned16(dy_out)) ||
      (size_t)K * 32 > 64 * 1024)
    return DK_ERR_ARGS;
  if (pw_stream_dgrad_ok(K, C, M)) {
    // K = C = 64: the persistent streaming kernel (pw_stream.hip), bit-identical results
    if (part && !bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
    FoldTail ft;
    if (part) fold_take(part, pw_stream_dgrad_rows(M), C, 1, &ft);
    return fold_status(pw_stream_dgrad_bnbwd(g, bn_x, M, out_mean, out_invstd, out_gamma, out_beta, out_relu, k12,
                                             dy_out, w_kc, dx, residual, part ? x : nullptr, bn_mean, bn_invstd,
                                             bn_gamma, bn_beta, bn_relu, part, st, part ? &ft : nullptr),
                       part ? ft : FoldTail{});
  }
  if (!part) {
    EpStore ep = ep_store(dx, C, nullptr, residual);
    return igemm_rows<LdMatKC, MatBwdDesc, LdMatIC, MatDesc, EpStore, kRowBnBwd>(a, b, ep, M, C, K, st);
  }
  EpStoreBnBwd ep;
  static_cast<EpStore&>(ep) = ep_store(dx, C, nullptr, residual);
  ep.v4 = ep.v4 && aligned16(x) && bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta);
  ep.part = part;
  ep.xbn = x;
  ep.bn = BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
  return igemm_rows<LdMatKC, MatBwdDesc, LdMatIC, MatDesc, EpStoreBnBwd, kRowBnBwd>(a, b, ep, M, C, K, st);
}

DK_API size_t dk_pwconv_wgrad_workspace_bytes(int N, int OH, int OW, int K, int C) {
  return splitk_ws_bytes(K, C, N * OH * OW);
}

// dw[k][c] = sum_{n,oh,ow} dy[n,oh,ow,k] * x[n, oh*s, ow*s, c]  (+ l2 * w)   (pointwise_convolution.py:61-64)
DK_API int dk_pwconv_wgrad_f32(const float* dy, const float* x, int N, int H, int W, int C, int K, int stride,
                               int OH, int OW, const float* w_kc, float l2, float* dw_kc, void* ws, size_t ws_bytes,
                               void* stream) {
  if (C % 4 || !aligned16(x) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  return wgrad(dy, img(x, N, H, W, C, OH, OW, 1, 1, stride, 1, 0, N * OH * OW), K, C, w_kc, l2, dw_kc, 0, C, C, 1, 1,
               ws, ws_bytes, stream);
}

DK_API int dk_pwconv_wgrad_bnx_f32(const float* dy, const float* x, int N, int H, int W, int C, int K, int stride,
                                   int OH, int OW, const float* w_kc, float l2, float* dw_kc, void* ws,
                                   size_t ws_bytes, const float* bn_mean, const float* bn_invstd,
                                   const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream) {
  if (C % 4 || !aligned16(x) || !fits((size_t)N * H * W * C * 4)) return DK_ERR_ARGS;
  if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
  return wgrad(dy,
               with_bn(img(x, N, H, W, C, OH, OW, 1, 1, stride, 1, 0, N * OH * OW), bn_mean, bn_invstd, bn_gamma,
                       bn_beta, bn_relu),
               K, C, w_kc, l2, dw_kc, 0, C, C, 1, 1, ws, ws_bytes, stream);
}

// Dense (dense_layer.py:46-55): y[b][o] = sum_i x[b][i] * w[i][o] (+ bias[o]);  w stored (in, out).
DK_API int dk_dense_fwd_f32(const float* x, int B, int IN, const float* w_io, int OUT, const float* bias, float* y,
                            void* stream) {
  MatDesc a = mat(x, B, IN, B);
  MatDesc b = mat(w_io, IN, OUT, OUT);
  EpStore ep = ep_store(y, OUT, bias);
  const hipStream_t st = as_stream(stream);
  const bool va = vec_ok(a, IN, 4), vb = vec_ok(b, 4, OUT);
  if (va && vb) return igemm_rows<LdMatKC, MatDesc, LdMatIC, MatDesc, EpStore>(a, b, ep, B, OUT, IN, st);
  return igemm_rows<LdMatKC1, MatDesc, LdMatIC1, MatDesc, EpStore>(a, b, ep, B, OUT, IN, st);
}

// dx[b][i] = sum_o dy[b][o] * w[i][o]   (dense_layer.py:67)
DK_API int dk_dense_dgrad_f32(const float* dy, int B, int OUT, const float* w_io, int IN, float* dx, void* stream) {
  MatDesc a = mat(dy, B, OUT, B);
  MatDesc b = mat(w_io, IN, OUT, IN);
  EpStore ep = ep_store(dx, IN, nullptr);
  const hipStream_t st = as_stream(stream);
  if (vec_ok(a, OUT, 4) && vec_ok(b, OUT, 4))
    return igemm_rows<LdMatKC, MatDesc, LdMatKC, MatDesc, EpStore>(a, b, ep, B, IN, OUT, st);
  return igemm_rows<LdMatKC1, MatDesc, LdMatKC1, MatDesc, EpStore>(a, b, ep, B, IN, OUT, st);
}

DK_API size_t dk_dense_wgrad_workspace_bytes(int B, int IN, int OUT) { return splitk_ws_bytes(IN, OUT, B); }

// dw[i][o] = sum_b x[b][i] * dy[b][o] (+ l2 * w)   (dense_layer.py:61-66)
DK_API int dk_dense_wgrad_f32(const float* x, const float* dy, int B, int IN, int OUT, const float* w_io, float l2,
                              float* dw_io, void* ws, size_t ws_bytes, void* stream) {
  if (ws_bytes < splitk_ws_bytes(IN, OUT, B)) return DK_ERR_WORKSPACE;
  MatDesc a = mat(x, B, IN, IN);
  MatDesc b = mat(dy, B, OUT, OUT);
  int splits = 1;
  const hipStream_t st = as_stream(stream);
  int rc;
  if (vec_ok(a, 4, IN) && vec_ok(b, 4, OUT))
    rc = igemm_splitk<LdMatIC, MatDesc, LdMatIC, MatDesc>(a, b, static_cast<float*>(ws), IN, OUT, B, st, &splits);
  else
    rc = igemm_splitk<LdMatIC1, MatDesc, LdMatIC1, MatDesc>(a, b, static_cast<float*>(ws), IN, OUT, B, st, &splits);
  if (rc) return rc;
  return splitk_reduce(static_cast<float*>(ws), splits, IN, OUT, dw_io, w_io, l2, 0, OUT, OUT, 1, 1, st);
}

// ---------------------------------------------------------------------------------------
// bf16 storage twins of the pointwise entries (BASELINE config 5).  Activations bf16,
// weights / statistics / weight gradients fp32; the loaders widen bf16 to fp32 on load and
// the MFMAs are the exact-fp32 v_mfma_f32_32x32x2_f32 of the fp32 path, so the only
// numerical difference from fp32 storage is the rounding of each stored activation.
// ---------------------------------------------------------------------------------------
namespace dk {
static inline MatDescE<bf16_t> mat_h(const bf16_t* p, int rows, int ld, int ext) {
  return MatDescE<bf16_t>{p, (uint32_t)((size_t)rows * ld * sizeof(bf16_t)), ld, ext};
}
static inline ImgDescE<bf16_t> img_h(const bf16_t* x, int N, int H, int W, int C, int OH, int OW, int R, int S,
                                     int sa, int dr, int off, int M) {
  return set_magics(ImgDescE<bf16_t>{x, (uint32_t)((size_t)N * H * W * C * sizeof(bf16_t)), H, W, C, OH, OW, R, S,
                                     sa, dr, off, off, M});
}
static inline ImgDescE<bf16_t, true> img1_h(const bf16_t* x, int N, int H, int W, int C, int OH, int OW, int sa, int M) {
  return set_magics(ImgDescE<bf16_t, true>{x, (uint32_t)((size_t)N * H * W * C * sizeof(bf16_t)), H, W, C, OH, OW,
                                           1, 1, sa, 1, 0, 0, M});
}
static inline bool al8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; }
}  // namespace dk

// partial-statistics rows of dk_pwconv_fwd_ex_bf16 (always the tiled engine: one row per M tile)
DK_API int dk_pwconv_fwd_bf16_stats_rows(int N, int OH, int OW, int K, int C) { return stats_rows(N * OH * OW, K, C); }

DK_API int dk_pwconv_fwd_ex_bf16(const bf16_t* x, int N, int H, int W, int C, const float* w_kc, int K, int stride,
                                 const float* bias, bf16_t* y, int OH, int OW, const float* bn_mean,
                                 const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu,
                                 double* stats, void* stream) {
  if (C % 4 || K % 4 || !al8(x) || !al8(y) || !aligned16(w_kc) || (bias && !aligned16(bias))) return DK_ERR_ARGS;
  if (!fits((size_t)N * H * W * C * 4) || !fits((size_t)N * OH * OW * K * 4)) return DK_ERR_ARGS;
  const ImgDescE<bf16_t, true> a = img1_h(x, N, H, W, C, OH, OW, stride, N * OH * OW);
  const MatDesc b = mat(w_kc, K, C, K);
  const hipStream_t st = as_stream(stream);
  const int M = a.M;
  auto run = [&](const auto& da) -> int {
    using DA = std::decay_t<decltype(da)>;
    if (stats) {
      EpStoreStatsT<bf16_t> ep{};
      ep.out = y, ep.ldo = K, ep.bias = bias, ep.v4 = 1, ep.res = nullptr, ep.part = stats;
      return igemm_rows<LdImgKC, DA, LdMatKC, MatDesc, EpStoreStatsT<bf16_t>>(da, b, ep, M, K, C, st);
    }
    EpStoreT<bf16_t> ep{y, K, bias, 1, nullptr};
    return igemm_rows<LdImgKC, DA, LdMatKC, MatDesc, EpStoreT<bf16_t>>(da, b, ep, M, K, C, st);
  };
  if (bn_mean) {
    if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta) || C > 2048) return DK_ERR_ARGS;
    ImgBnDescE<bf16_t, true> ab;
    static_cast<ImgDescE<bf16_t, true>&>(ab) = a;
    ab.bn = BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
    return run(ab);
  }
  return run(a);
}

// Stride-1 pointwise dgrad (bf16): dx = dy . W (+ residual) and, with bn_x/part, the
// BN-backward partials of the BatchNorm whose output the layer consumed.
DK_API int dk_pwconv_dgrad_ex_bf16(const bf16_t* dy, int N, int OH, int OW, int K, const float* w_kc, int C,
                                   int stride, bf16_t* dx, const bf16_t* residual, const bf16_t* bn_x,
                                   const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                   const float* bn_beta, int bn_relu, double* part, void* stream) {
  const int M = N * OH * OW;
  if (stride != 1 || C % 4 || K % 4 || !al8(dy) || !al8(dx) || !aligned16(w_kc)) return DK_ERR_ARGS;
  if ((residual && !al8(residual)) || (bn_x && !al8(bn_x))) return DK_ERR_ARGS;
  if (!fits((size_t)M * K * 4) || !fits((size_t)M * C * 4) || (part != nullptr) != (bn_x != nullptr)) return DK_ERR_ARGS;
  const MatDescE<bf16_t> a = mat_h(dy, M, K, M);
  const MatDesc b = mat(w_kc, K, C, C);
  const hipStream_t st = as_stream(stream);
  if (!part) {
    EpStoreT<bf16_t> ep{dx, C, nullptr, 1, residual};
    return igemm_rows<LdMatKC, MatDescE<bf16_t>, LdMatIC, MatDesc, EpStoreT<bf16_t>>(a, b, ep, M, C, K, st);
  }
  if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
  EpStoreBnBwdT<bf16_t> ep{};
  ep.out = dx, ep.ldo = C, ep.bias = nullptr, ep.v4 = 1, ep.res = residual;
  ep.part = part;
  ep.xbn = bn_x;
  ep.bn = BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
  return igemm_rows<LdMatKC, MatDescE<bf16_t>, LdMatIC, MatDesc, EpStoreBnBwdT<bf16_t>>(a, b, ep, M, C, K, st);
}

// dw[k][c] = sum dy[m][k] * bn(x)[m][c] (+ l2 * w), bf16 activations, fp32 result.
DK_API int dk_pwconv_wgrad_bnx_bf16(const bf16_t* dy, const bf16_t* x, int N, int H, int W, int C, int K, int stride,
                                    int OH, int OW, const float* w_kc, float l2, float* dw_kc, void* ws,
                                    size_t ws_bytes, const float* bn_mean, const float* bn_invstd,
                                    const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream) {
  const int Kred = N * OH * OW;
  if (C % 4 || K % 4 || !al8(x) || !al8(dy) || !fits((size_t)N * H * W * C * 4) || !fits((size_t)Kred * K * 4))
    return DK_ERR_ARGS;
  if (ws_bytes < splitk_ws_bytes(K, C, Kred)) return DK_ERR_WORKSPACE;
  const MatDescE<bf16_t> a = mat_h(dy, Kred, K, K);
  const ImgDescE<bf16_t> bi = img_h(x, N, H, W, C, OH, OW, 1, 1, stride, 1, 0, Kred);
  float* part = static_cast<float*>(ws);
  const hipStream_t st = as_stream(stream);
  int splits = 1, rc;
  if (bn_mean) {
    if (!bn_ok(bn_mean, bn_invstd, bn_gamma, bn_beta)) return DK_ERR_ARGS;
    ImgBnDescE<bf16_t> b;
    static_cast<ImgDescE<bf16_t>&>(b) = bi;
    b.bn = BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
    rc = igemm_splitk<LdMatIC, MatDescE<bf16_t>, LdImgIC, ImgBnDescE<bf16_t>>(a, b, part, K, C, Kred, st, &splits);
  } else {
    rc = igemm_splitk<LdMatIC, MatDescE<bf16_t>, LdImgIC, ImgDescE<bf16_t>>(a, bi, part, K, C, Kred, st, &splits);
  }
  if (rc) return rc;
  return splitk_reduce(part, splits, K, C, dw_kc, w_kc, l2, 0, C, C, 1, 1, st);
}
