// Implicit-GEMM engine for gfx950: fp32 MFMA (v_mfma_f32_32x32x2_f32), and a bf16 MFMA mode
// (v_mfma_f32_32x32x16_bf16, operands rounded to bf16 as they are staged; BASELINE config 5).
// The entry points live in gemm_conv.hip, gemm_pw.hip, gemm_dense.hip and gemm_bf16.hip.
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
#pragma once
#include <stdlib.h>

#include <mutex>
#include <type_traits>

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
template <class E>
struct MatBwdDescE : MatDescE<E> {
  static constexpr bool kBnBwd = true;
  const E* x;       // the BN's raw input, laid out like p (same element type)
  BnBwdIn bwd;
  E* dy_out;        // dy write-through (rounded to E when E is bf16)
};
using MatBwdDesc = MatBwdDescE<float>;

// ----------------------------------------------------------------------------
// Loaders.  K-contiguous ("KC") loaders fill T[ROWS][BK+4]; row-contiguous ("IC")
// loaders fill T[BK][ROWS].  frag(T, row, q, h) returns the four k values
// 8q + 4h + {0,1,2,3} of `row` for the MFMA loop.
// ----------------------------------------------------------------------------

// LDS element type TT: float (the f32 MFMA engine) or bf16_t (the bf16 MFMA engine, BASELINE
// config 5: operands rounded to bf16 as they are staged).  Row strides per element type:
//   KC fp32: BK+4 floats, (BK+4)/4 odd -> conflict-free ds_read_b128;
//   KC bf16: BK+8 elements = an odd multiple of 16 bytes -> the 16 rows of a ds_read_b128 lane group
//            start on 16 distinct 4-bank groups;
//   IC bf16: a row stride of an odd multiple of 64 bytes -> the 4 k-rows of each 32-lane half of
//            a ds_read_b64_tr_b16 fall on 4 distinct 16-bank groups (MI355X_MICROARCH.md LDS).
template <int ROWS, int BK>
struct KCLayout {
  static constexpr bool kIC = false;
  static constexpr int SK = BK + 4;  // row stride in floats: (BK+4)/4 odd -> conflict-free b128 reads
  static constexpr int BUF = ROWS * SK;
  static constexpr int SKH = BK + 8;  // bf16 row stride (elements)
  static constexpr int BUFH = ROWS * SKH;
  template <class TT>
  __device__ static constexpr int stride() { return sizeof(TT) == 4 ? SK : SKH; }
  __device__ static __forceinline__ f32x4 frag(const float* T, int row, int q, int h) {
    return ld4(T + row * SK + 8 * q + 4 * h);
  }
  // bf16 operand of v_mfma_f32_32x32x16_bf16, k-step s: k = 16s + 8h + j, j = 0..7 of `row`
  __device__ static __forceinline__ bf16x8 fragh(const bf16_t* T, int row, int s, int h) {
    return *reinterpret_cast<const bf16x8*>(T + row * SKH + 16 * s + 8 * h);
  }
};

template <int ROWS, int BK>
struct ICLayout {
  static constexpr bool kIC = true;
  static constexpr int S = ROWS;
  static constexpr int BUF = BK * ROWS;
  static constexpr int SH = 2 * ((ROWS / 2 + 15) / 32 * 32 + 16);  // bf16 row stride: 2*(16 mod 32) elements
  static constexpr int BUFH = BK * SH;
  template <class TT>
  __device__ static constexpr int stride() { return sizeof(TT) == 4 ? S : SH; }
  __device__ static __forceinline__ f32x4 frag(const float* T, int row, int q, int h) {
    const float* p = T + (8 * q + 4 * h) * S + row;
    return f32x4{p[0], p[S], p[2 * S], p[3 * S]};
  }
  // bf16 operand, k-step s: the 8 k-rows 16s + 8h .. +7 of column `row`, gathered by two
  // ds_read_b64_tr_b16 (each delivers 4 k-rows of 16 consecutive columns to a 16-lane group:
  // lane 4q+p supplies the address of k-row q, columns 4p..4p+3 of its group's block).
  // row0: the 32-column tile's first column (row = row0 + lane & 31).
  __device__ static __forceinline__ bf16x8 fragh(const bf16_t* T, int row0, int s, int h, int lane) {
    const int i = lane & 15, g = (lane >> 4) & 1;
    const bf16_t* p = T + (16 * s + 8 * h + (i >> 2)) * SH + row0 + 16 * g + 4 * (i & 3);
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * SH));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
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

  template <class D, class TT>
  __device__ __forceinline__ void store(TT* T) const {
    if (!active) return;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      f32x4 o = v[j];
      if constexpr (D::kBnIn) {
        const float* tb = reinterpret_cast<const float*>(tab) + cch;
        const f32x4 t = bn_in4(o, ld4(tb), ld4(tb + tc), ld4(tb + 2 * tc), ld4(tb + 3 * tc), relu);
        if ((okm >> j) & 1u) o = t;
      }
      st4(T + (rb + j * RSTEP) * L::template stride<TT>() + 4 * kq, o);
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
  void* dyo;  // D::Elem* (MatBwdDescE)
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
          xv[j] = bload4e<typename D::Elem>(rx, iv && k < Ktot, (uint32_t)(i * d.ld + k));
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

  template <class D, class TT>
  __device__ __forceinline__ void store(TT* T) {
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
          if (writer) st4(static_cast<typename D::Elem*>(dyo) + eoff[j], o);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NR; ++j) st4(T + (rb + j * RSTEP) * L::template stride<TT>() + 4 * kq, v[j]);
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
  void* dyo;
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
          xv[j] = bload4e<typename D::Elem>(rx, kv && i0 < d.ext, (uint32_t)(k * d.ld + i0));
          om |= (uint32_t)(kv && i0 < d.ext) << j;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][e] = bload1(rs, (kv && i0 + e < d.ext) ? base + 4u * e : kOOB);
      }
    }
    if constexpr (D::kBnBwd) okm = om;
  }

  template <class D, class TT>
  __device__ __forceinline__ void store(TT* T) {
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
    for (int j = 0; j < NK; ++j) st4(T + (kb + j * KSTEP) * L::template stride<TT>() + 4 * iq, v[j]);
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

  template <class D, class TT>
  __device__ __forceinline__ void store(TT* T) const {
    if (!active) return;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      f32x4 o = v[j];
      if constexpr (D::kBnIn) {
        if ((okm >> j) & 1u) o = bn_in4(o, bm, bi, bg, bb, relu);
      }
      st4(T + (kb + j * KSTEP) * L::template stride<TT>() + 4 * iq, o);
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
  int nt = 0;  // nontemporal 16-byte stores (tuning knob nt_stores(), set by launch_igemm)
  __device__ __forceinline__ void store4(O* p, f32x4 v) const {
    if (nt)
      st4nt(p, v);
    else
      st4(p, v);
  }
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
    store4(out + (size_t)m * ldo + n, value4(n, v, p));
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
    this->store4(this->out + (size_t)m * this->ldo + n, o);
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
    this->store4(this->out + (size_t)m * this->ldo + n, v);
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

// The bf16 operand fragment of a loader's layout (KC: one ds_read_b128; IC: two transposing
// ds_read_b64_tr_b16 of the 32-column tile starting at row - lane & 31).
template <class L>
__device__ __forceinline__ bf16x8 frag_h(const bf16_t* T, int row, int s, int h, int lane) {
  if constexpr (L::kIC)
    return L::fragh(T, row - (lane & 31), s, h, lane);
  else
    return L::fragh(T, row, s, h);
}

// MF: the MFMA the operands feed -- kMfF32 (v_mfma_f32_32x32x2_f32 on fp32 LDS tiles, exact fp32)
// or kMfBf16 (v_mfma_f32_32x32x16_bf16 on bf16 LDS tiles: each operand element rounded to bf16
// (RNE) as it is staged, products exact, fp32 accumulation; BASELINE config 5's bf16 path).
enum : int { kMfF32 = 0, kMfBf16 = 1 };

template <int BM, int BN, int BK, int WM, int WN, class LA, class DA, class LB, class DB, class EP, int MF = kMfF32>
__global__ __launch_bounds__(64 * WM * WN) void igemm_f32(DA da, DB db, EP ep, int M, int N, int Ktot,
                                                           int kt_per_split) {
  constexpr int TM = BM / (32 * WM);
  constexpr int TN = BN / (32 * WN);
  constexpr bool H = MF == kMfBf16;
  static_assert(TM >= 1 && TN >= 1 && BM == 32 * WM * TM && BN == 32 * WN * TN, "tile");
  static_assert(BK % (H ? 16 : 8) == 0, "BK");
  using TT = typename std::conditional<H, bf16_t, float>::type;  // LDS operand element
  constexpr int ABUF = H ? LA::BUFH : LA::BUF, BBUF = H ? LB::BUFH : LB::BUF;  // elements
  // operand double buffers; the epilogue reuses the same LDS for the staged C tile
  // ([BM][BN+8]) and, with kColStats, the fp64 column-sum scratch (sizes in floats)
  constexpr int SMEM_OPS = (2 * (ABUF + BBUF) * (int)sizeof(TT) + 3) / 4;
  constexpr int SMEM_EPI = BM * (BN + 8);
  constexpr int SMEM_RED = EP::kColStats ? (64 * WM * WN / (BN / 4)) * BN * 4 : 0;
  constexpr int SMEM = SMEM_OPS > SMEM_EPI ? (SMEM_OPS > SMEM_RED ? SMEM_OPS : SMEM_RED)
                                           : (SMEM_EPI > SMEM_RED ? SMEM_EPI : SMEM_RED);
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  TT* const As = reinterpret_cast<TT*>(smem);
  TT* const Bs = As + 2 * ABUF;

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
      const TT* A_t = As + cur * ABUF;
      const TT* B_t = Bs + cur * BBUF;
      if constexpr (H) {
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {
          bf16x8 af[TM], bf[TN];
#pragma unroll
          for (int t = 0; t < TM; ++t) af[t] = frag_h<LA>(A_t, arow + 32 * t, s, h, lane);
#pragma unroll
          for (int u = 0; u < TN; ++u) bf[u] = frag_h<LB>(B_t, brow + 32 * u, s, h, lane);
#pragma unroll
          for (int t = 0; t < TM; ++t)
#pragma unroll
            for (int u = 0; u < TN; ++u)
              acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[t], bf[u], acc[t][u], 0, 0, 0);
        }
      } else {
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

// Split-K grids fill the resident block slots once (g_fill_splits; tuning knob
// dk_debug_set_gemm_config(2, 0/1)).  A persistent tile loop for the row problems was measured
// and dropped (scripts/ab_step.py: 11.77 ms/step with one block per tile, 11.89 / 11.98 with
// 1 / 2 resident waves of persistent blocks, and the loop slowed the one-tile case too).
constexpr int kNumCUs = 256;  // MI355X

// Epilogues with an `nt` member take the nontemporal-store knob (nt_stores()).
template <class E>
static inline auto set_nt(E& e, int) -> decltype(e.nt = 0, void()) {
  e.nt = nt_stores(kNtGemm);
}
template <class E>
static inline void set_nt(E&, long) {}

// Launch facts of one kernel instantiation, by dynamic LDS size: its static LDS (queried once),
// the largest dynamic size set on it so far (hipFuncSetAttribute only when a launch needs more),
// and resident blocks per CU for each distinct dynamic size it has been launched with (the
// BN-on-load tables make the dynamic LDS a function of the layer's channel count, and with it the
// occupancy that sizes split-K grids).  Thread-safe: one mutex per instantiation; the table is
// small (one entry per distinct channel count) and a full table falls back to querying.
struct LaunchFacts {
  std::mutex mu;
  bool init = false;
  size_t lds_static = 0, dyn_set = 0;
  static constexpr int kMax = 16;
  int n = 0;
  size_t dyn[kMax];
  int occ[kMax];
};

// Resident blocks per CU of `fn` at `dyn` bytes of dynamic LDS, or -1 when static + dynamic LDS
// exceeds the CU's 160 KB (the runtime would abort the queue on such a launch).
static int launch_occupancy(LaunchFacts& f, const void* fn, int nt, size_t dyn) {
  std::lock_guard<std::mutex> lock(f.mu);
  if (!f.init) {
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, fn) == hipSuccess) f.lds_static = fa.sharedSizeBytes;
    f.init = true;
  }
  if (f.lds_static + dyn > (size_t)160 * 1024) return -1;
  if (dyn > f.dyn_set) {
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
    f.dyn_set = dyn;
  }
  for (int i = 0; i < f.n; ++i)
    if (f.dyn[i] == dyn) return f.occ[i];
  int o = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, fn, nt, dyn) != hipSuccess || o < 1) o = 1;
  if (f.n < LaunchFacts::kMax) {
    f.dyn[f.n] = dyn;
    f.occ[f.n] = o;
    ++f.n;
  }
  return o;
}

template <int BM, int BN, int BK, int WM, int WN, template <int, int, int> class LA, class DA,
          template <int, int, int> class LB, class DB, class EP, int MF = kMfF32>
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
  if constexpr (DA::kBnIn && A::kTable) dyn = (size_t)da.C * sizeof(f32x4);
  if constexpr (DA::kBnBwd) dyn = (size_t)da.bwd.C * 2 * sizeof(f32x4);
  static LaunchFacts facts;
  const int occ = launch_occupancy(facts, reinterpret_cast<const void*>(&igemm_f32<BM, BN, BK, WM, WN, A, DA, B, DB, EP, MF>),
                                   NT, dyn);
  if (occ < 0) return DK_ERR_ARGS;
  const int slots = occ * kNumCUs;
  if (knob(kKnobFillSplits) && splits_used && splits > 1 && tiles * splits > slots && tiles <= slots) {
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
    set_nt(e, 0);
    if (!e.part || splits != 1 || !fold_take(e.part, cdiv(M, BM), N, cdiv(N, BN), &e.ft)) e.ft.part = nullptr;
    hipLaunchKernelGGL((igemm_f32<BM, BN, BK, WM, WN, A, DA, B, DB, EP, MF>), dim3(tiles, splits), dim3(NT), dyn, st, da,
                       db, e, M, N, Ktot, kps);
    return fold_status(launch_status(), e.ft);
  }
  EP e = ep;
  set_nt(e, 0);
  hipLaunchKernelGGL((igemm_f32<BM, BN, BK, WM, WN, A, DA, B, DB, EP, MF>), dim3(tiles, splits), dim3(NT), dyn, st, da,
                     db, e, M, N, Ktot, kps);
  return launch_status();
}

// Row-problem kinds with their own tile choice: plain loaders, and the BN-backward-on-load A
// operand (dk_pwconv_dgrad_bnbwd_f32), whose per-element transform is repeated for every column
// tile -- wide column tiles amortise it.
// kRowConv: R x S > 1 image forward; kRowFwdH: the bf16 pointwise forward (its own tuning)
enum : int { kRowPlain = 0, kRowBnBwd = 1, kRowConv = 2, kRowFwdH = 3 };

static inline int row_config(int M, int N, int K, int kind = kRowPlain, int mf = kMfF32) {
  if (knob(kKnobRowCfg) >= 0) return knob(kKnobRowCfg);
  (void)M;
  if (mf == kMfBf16) {
    // bf16 MFMA (config 5's 14 x 14 and 7 x 7 units at batch 512; scripts/gemm_tune_deep.py --bf16,
    // profiles/r03k_bf16_gemm_tune.txt): the tiles with 8 waves or 128 columns, whose blocks run
    // more MFMAs per dependent load round trip
    if (kind == kRowBnBwd) return N <= 128 ? 16 : (N <= 256 ? (K >= 512 ? 13 : 16) : 13);
    if (kind == kRowFwdH && N >= 256) return (K >= 512 && N >= 512) ? 16 : 13;
  }
  if (kind == kRowFwdH) kind = kRowPlain;
  if (kind == kRowBnBwd) {
    // Measured on MI355X (scripts/gemm_tune.py --fused-only, profiles/r01h_gemm_tune_fused.txt)
    if (N <= 64) return 8;                // 64x64x32
    if (N <= 128) return 16;              // 128x128x32, 2x4 waves
    // C = K = 256 at 14 x 14, batch 256: 98 vs 107 us (scripts/gemm_tune_deep.py, profiles/r03q_f32_tune.txt)
    if (N <= 256) return K >= 512 ? 13 : 16;
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
          int KIND = kRowPlain, int MF = kMfF32>
static int igemm_rows(const DA& da, const DB& db, const EP& ep, int M, int N, int Ktot, hipStream_t st) {
  switch (row_config(M, N, Ktot, KIND, MF)) {
#define DK_CASE(id, bm, bn, bk, wm, wn) \
  case id:                              \
    return launch_igemm<bm, bn, bk, wm, wn, LA, DA, LB, DB, EP, MF>(da, db, ep, M, N, Ktot, 1, st);
    DK_ROW_CONFIGS(DK_CASE)
#undef DK_CASE
    default:
      return DK_ERR_ARGS;
  }
}

// Reduction-heavy problems (wgrad): split K over enough blocks to fill the chip.
static inline int splitk_config(int M, int N, int Kred, int mf = kMfF32) {
  if (knob(kKnobSplitCfg) >= 0) return knob(kKnobSplitCfg);
  (void)Kred;
  // bf16 MFMA: 128 x 128 tiles for the 14 x 14 / 7 x 7 weight gradients (profiles/r03k_bf16_gemm_tune.txt)
  if (mf == kMfBf16 && M >= 128 && N >= 128) return 4;
  // Wide column tiles when M <= 64 < N: the A operand (for the stem the BN-backward-on-load dy,
  // formed from 2 x 822 MB) is streamed half as often -- the stem (N = R*S*Cp = 100) in one
  // column tile; BASELINE config 2's 3x3 conv (N = 576): 594 vs 628 us (profiles/r01j_gemm_tune_all.txt).
  if (M <= 64 && N > 64) return 6;  // 64x128x32
  return 1;  // 64x64x32: best or within 3% of best on every other measured wgrad shape
}

// Blocks a split-K weight gradient aims for (knob kKnobWgradBlocks, kind 18; default 1024).
static inline int wgrad_target_blocks() {
  const int v = knob(kKnobWgradBlocks);
  return v > 0 ? v : 1024;
}

static inline int wgrad_splits(int M, int N, int Kred, const TileCfg& c) {
  const int tiles = cdiv(M, c.BM) * cdiv(N, c.BN);
  const int KT = cdiv(Kred, c.BK);
  int splits = cdiv(wgrad_target_blocks(), tiles);
  if (splits > KT) splits = KT;
  if (splits < 1) splits = 1;
  const int kps = cdiv(KT, splits);
  return cdiv(KT, kps);
}

template <template <int, int, int> class LA, class DA, template <int, int, int> class LB, class DB, int MF = kMfF32>
static int igemm_splitk(const DA& da, const DB& db, float* ws, int M, int N, int Kred, hipStream_t st,
                        int* splits_out) {
  const int id = splitk_config(M, N, Kred, MF);
  if (id < 0 || id >= kNumSplitCfg) return DK_ERR_ARGS;
  const int splits = wgrad_splits(M, N, Kred, kSplitCfg[id]);  // the workspace's upper bound
  *splits_out = splits;
  EpPartial ep{ws, M, N, al4(N) && aligned16(ws)};
  switch (id) {
#define DK_CASE(cid, bm, bn, bk, wm, wn) \
  case cid:                              \
    return launch_igemm<bm, bn, bk, wm, wn, LA, DA, LB, DB, EpPartial, MF>(da, db, ep, M, N, Kred, splits, st, \
                                                                           splits_out);
    DK_SPLITK_CONFIGS(DK_CASE)
#undef DK_CASE
    default:
      return DK_ERR_ARGS;
  }
}

static inline size_t splitk_ws_bytes(int M, int N, int Kred, int mf = kMfF32) {
  int id = splitk_config(M, N, Kred, mf);
  if (id < 0 || id >= kNumSplitCfg) id = 0;
  return (size_t)wgrad_splits(M, N, Kred, kSplitCfg[id]) * (size_t)M * (size_t)N * sizeof(float);
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
static inline int stats_rows(int M, int N, int Ktot, int kind = kRowPlain, int mf = kMfF32) {
  return cdiv(M, kRowCfg[row_config(M, N, Ktot, kind, mf)].BM);
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

}  // namespace dk
