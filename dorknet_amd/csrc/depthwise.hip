// Depthwise (per-channel) convolution on NHWC fp32 for gfx950 -- direct, no MFMA.
//
// Replaces layers/depthwise_convolution.py:85-102 (+ CUDA forward_conv :105-121) and
// :198-221 (+ CUDA backward_conv :122-140).  Same maths, different data flow:
//   * channels are innermost, so a lane owns 4 adjacent channels (one float4) and a
//     wave covers 64*4 contiguous floats of a pixel row: fully coalesced;
//   * padding is handled by bounds checks instead of a padded copy (:57-64);
//   * a thread produces TW consecutive outputs along W, keeping an R x S window of
//     input float4s in registers and sliding it, so each output costs R*stride new
//     loads instead of R*S (the reference re-reads all R*S taps and does R*S global
//     read-modify-writes of the output);
//   * stride-1 dgrad is the forward kernel run on dy with the taps flipped;
//   * wgrad reduces per-block partials in a fixed order (reduce.hip) -- the reference
//     issues N*OH*OW atomicAdds on each of the C*R*S weight addresses.
#include <numeric>
#include <type_traits>

#include "dk_common.h"
#include "fold_tail.h"

namespace dk {


// w[c][r][s] -> wt[r][s][c] (flip != 0: wt[r][s][c] = w[c][R-1-r][S-1-s]) so one float4
// load fetches a tap for 4 channels.
__global__ void dw_weight_rsc_kernel(const float* __restrict__ w, int C, int R, int S, int flip,
                                     float* __restrict__ wt) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= C * R * S) return;
  const int c = idx % C, t = idx / C;
  int r = t / S, s = t - r * S;
  if (flip) {
    r = R - 1 - r;
    s = S - 1 - s;
  }
  wt[idx] = w[((size_t)c * R + r) * S + s];
}

// Activation reads are buffer loads (bload4e, dk_common.h): out-of-range offsets return 0 in
// hardware, so the padding needs no branches and every load of a thread can be in flight.

// Per-thread filter taps for channels c..c+3: wl 0 = the [R][S][C] copy (dk_dw_weight_rsc_f32),
// 1 = the reference layout W[C][R][S] read directly (4*R*S contiguous floats), 2 = W[C][R][S]
// with the taps flipped (stride-1 dgrad).  No re-layout launch for layouts 1 and 2.
template <int R, int S, int WL>
__device__ __forceinline__ void load_dw_weights(f32x4 (&wv)[R][S], const float* __restrict__ w, int c, int C) {
  if constexpr (WL == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int s = 0; s < S; ++s) wv[r][s] = ld4(w + (r * S + s) * C + c);
  } else {
    constexpr int RS = R * S;
    f32x4 f[RS];  // floats c*RS .. (c+4)*RS-1
#pragma unroll
    for (int i = 0; i < RS; ++i) f[i] = ld4(w + (size_t)c * RS + 4 * i);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int tap = WL == 2 ? (R - 1 - r) * S + (S - 1 - s) : r * S + s;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = e * RS + tap;
          wv[r][s][e] = f[k >> 2][k & 3];
        }
      }
  }
}

// bn_relu_out on 4 channels in packed fp32 (v_pk_add / v_pk_mul / v_pk_fma: the same IEEE
// operations two lanes per instruction, bit-identical to bn_out), the ReLU as a compile-time
// v_max_f32 (max(r, 0) is the reference's (r > 0) ? r : 0; a NaN gives 0 both ways) instead of a
// compare and select on the run-time flag.
template <bool RELU>
__device__ __forceinline__ f32x4 bn_in4p(f32x4 v, f32x4 m, f32x4 is, f32x4 g, f32x4 b) {
  // x + (-mean) is x - mean exactly; written as an add it packs (v_pk_add_f32)
  const f32x2 h0 = (f32x2{v[0], v[1]} + f32x2{-m[0], -m[1]}) * f32x2{is[0], is[1]};
  const f32x2 h1 = (f32x2{v[2], v[3]} + f32x2{-m[2], -m[3]}) * f32x2{is[2], is[3]};
  const f32x2 o0 = __builtin_elementwise_fma(f32x2{g[0], g[1]}, h0, f32x2{b[0], b[1]});
  const f32x2 o1 = __builtin_elementwise_fma(f32x2{g[2], g[3]}, h1, f32x2{b[2], b[3]});
  f32x4 o = {o0[0], o0[1], o1[0], o1[1]};
  if constexpr (RELU) {
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = __builtin_fmaxf(o[e], 0.f);
  }
  return o;
}

// One input row of a strip: NC float4s at (ih, iw0 ..), BN-on-load applied, padding 0.
template <int NC, bool BN, bool RELU, class T = float>
__device__ __forceinline__ void load_row(f32x4 (&row)[NC], __amdgpu_buffer_rsrc_t rs, int n, int ih, int iw0, int H,
                                         int W, int C, int c, f32x4 bm, f32x4 bi, f32x4 bg, f32x4 bb) {
  const bool rv = (unsigned)ih < (unsigned)H;
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int iw = iw0 + q;
    const bool ok = rv && (unsigned)iw < (unsigned)W;
    row[q] = bload4e<T>(rs, ok, (uint32_t)(((n * H + ih) * W + iw) * C + c));
    if constexpr (BN) {
      const f32x4 t = bn_in4p<RELU>(row[q], bm, bi, bg, bb);
      row[q] = ok ? t : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}
// The same with the ReLU flag read at run time (the weight-gradient kernel).
template <int NC, bool BN, class T = float>
__device__ __forceinline__ void load_row(f32x4 (&row)[NC], __amdgpu_buffer_rsrc_t rs, int n, int ih, int iw0, int H,
                                         int W, int C, int c, const BnIn& bn, f32x4 bm, f32x4 bi, f32x4 bg,
                                         f32x4 bb) {
  const bool rv = (unsigned)ih < (unsigned)H;
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int iw = iw0 + q;
    const bool ok = rv && (unsigned)iw < (unsigned)W;
    row[q] = bload4e<T>(rs, ok, (uint32_t)(((n * H + ih) * W + iw) * C + c));
    if constexpr (BN) {
      const f32x4 t = bn_in4(row[q], bm, bi, bg, bb, bn.relu);
      row[q] = ok ? t : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

// Outputs per thread along W: the input strip R x ((TW-1)*ST + S) float4s is loaded at once.
// Stride 2 takes two: its window (R x 5 float4s, two rows of it new each output row) then leaves
// the join-forming variant two waves per SIMD (with four outputs, R x 9, it ran at one).
// Nontemporal-store family of a strided depthwise dgrad: bf16 has its own (12, on: config 5 5.747 ->
// 5.718 ms, profiles/r06ay_ab_nt_stem.txt), fp32 keeps family 10 (off: neutral or slower).
template <class T>
constexpr int dgrad_nt_fam() {
  return sizeof(T) == 2 ? kNtDwDgrad16 : kNtDwDgrad;
}

template <int ST>
struct DwTile {
  static constexpr int TW = ST == 2 ? 2 : 4;    // outputs per thread along W
};

// Output rows per thread (the input window slides down a segment of them).  Round 3 measured 8
// best or within noise of best on every training shape of configs 3 and 5 (scripts/dw_fwd_seg.py,
// profiles/r03q_dw_seg_{f32,bf16}.txt: fewer rows per thread re-load the window more often and the
// extra blocks do not pay for it).
// Balanced segments (OH = 28 -> 4 x 7 rather than 8 + 8 + 8 + 4: short last segments left threads
// idle; profiles/r04dw2_dwseg.txt).  At most 14 rows since round 5: with the row prefetch really in
// flight (the unconditional load below) a row costs less and the window's prologue more, and
// 14 rows per thread measured config 5 5.93 -> 5.84 ms, config 3 8.146 -> 8.132 ms
// (profiles/r05ai_ab_dw_fwd_rows_per_thread.txt; whole columns were faster still for bf16, slower
// for fp32).
// bf16 (whole): a thread slides down its whole output column -- config 5 5.776 -> 5.731 ms, while
// fp32 measured slower that way (config 3 7.764 -> 7.786 ms; profiles/r06av_ab_dw_fwd_rows_bf16.txt).
static inline int dw_fwd_seg(int OH, bool whole) {
  const int seg = knob(kKnobDwSeg);  // tuning knob (kind 8): rows per thread; -1 = this rule
  if (seg > 0) return seg;
  if (whole) return OH;
  const int nseg = (OH + 13) / 14;
  return (OH + nseg - 1) / nseg;
}

// y[n,oh,ow,c] = sum_{r,s} w[r][s][c] * x[n, oh*ST + r - pad, ow*ST + s - pad, c] (+ bias[c])
// Thread = (n, oh, TW-wide chunk of ow, 4 channels); consecutive threads take consecutive
// channel groups, so a wave reads whole pixel rows.
// res (optional, laid out like y): added to every output -- the residual join's other
// gradient term when this kernel computes a dgrad (residual_block.py:94-97).
// STATS: also a per-channel reduction of this block's outputs -> part[block][2][C]; needs
// 256 % (C/4) == 0 so that a block covers every channel (thread tid always has channel group
// tid % (C/4)).  STATS == 1: BatchNorm statistics of y (fp64 sum, sum of squares);
// STATS == 2 (this kernel computing a stride-1 dgrad): the BN-backward sums of the BatchNorm
// whose output the layer consumed -- sum(g), sum(g * x_hat) with g = y masked by that BN's
// fused ReLU (batch_norm.py:125-174, dk_bn_bwd_partial_f64); xo is that BN's raw input.
// T: activation storage (float, or bf16_t for BASELINE config 5); compute is fp32, and the
// statistics see the stored (rounded) outputs.
// JOIN: the layer's input is a residual block's output y = ReLU(bnA(a) + bnB(b)) (residual_block.py:75,
// the join dk_bn_add_f32 computes), formed here as the window rows are loaded -- x is a (the chain's
// last BatchNorm's raw input), jf.b the skip operand -- and stored once (jf.y, and the ReLU mask
// jf.mask): each thread stores the rows and columns of its window that no other thread's window
// owns (its output columns' input columns, its segment's input rows), so the separate join pass and
// this layer's re-read of y disappear.  Bit-identical to dk_bn_add_f32 (the same per-element
// operations: bn_relu_out of each operand, one add, the (v > 0) ? v : 0 ReLU).  3 x 3, pad 1, fp32.
struct JoinFwd {
  const float* b;  // the skip operand (raw; a BatchNorm input when bb.mean)
  BnIn ba, bb;     // the BatchNorms applied to a and b (mean == nullptr: none)
  float* y;        // the join output, NHWC like a
  uint8_t* mask;   // its ReLU mask (nullable)
};

template <int R, int S, int ST, bool BN, bool RELU, int STATS, int WL, class T = float, bool JOIN = false>
__global__ __launch_bounds__(256, JOIN ? 2 : 1) void dw_fwd_kernel(const T* __restrict__ x, uint32_t xbytes,
                                                     const float* __restrict__ wt, const float* __restrict__ bias,
                                                     T* __restrict__ y, int N, int H, int W, int C, int OH, int OW,
                                                     int pad, BnIn bn, double* __restrict__ part,
                                                     const T* __restrict__ xo, BnIn obn,
                                                     const T* __restrict__ res, FoldTail ft, int nt, int SEG,
                                                     JoinFwd jf) {
  static_assert(!JOIN || (R == 3 && S == 3 && !BN && sizeof(T) == 4), "the join is formed for 3 x 3 fp32 layers");
  constexpr int TW = DwTile<ST>::TW;
  constexpr int NC = (TW - 1) * ST + S;
  const int C4 = C >> 2;
  const int nwc = (OW + TW - 1) / TW;
  const int nseg = (OH + SEG - 1) / SEG;
  // XCD-contiguous block order: the row segments sharing input rows share an L2
  const long long idx = (long long)xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const long long total = (long long)N * nseg * nwc * C4;
  const bool live = idx < total;
  // the join's BatchNorm terms per channel group, in LDS (in registers they cost the kernel its second
  // wave per SIMD)
  __shared__ f32x4 jtab[JOIN ? 8 : 1][JOIN ? 128 : 1];
  if constexpr (JOIN) {
    for (int i = threadIdx.x; i < 8 * (C >> 2); i += 256) {
      const int t = i / (C >> 2), q = i - t * (C >> 2);
      const BnIn& b = t < 4 ? jf.ba : jf.bb;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (b.mean) v = ld4((t & 3) == 0 ? b.mean + 4 * q : (t & 3) == 1 ? b.invstd + 4 * q : (t & 3) == 2 ? b.gamma + 4 * q
                                                                                                         : b.beta + 4 * q);
      jtab[t][q] = v;
    }
    __syncthreads();
  }
  if (STATS == 0 && !live) return;
  const int cq = (int)(idx % C4);
  const int c = cq * 4;
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  if (live) {
    long long t = idx / C4;
    const int wc = (int)(t % nwc);
    t /= nwc;
    const int sg = (int)(t % nseg);
    const int n = (int)(t / nseg);
    const int ow0 = wc * TW;
    const int iw0 = ow0 * ST - pad;
    const int oh0 = sg * SEG, oh1 = min(OH, oh0 + SEG);
    const __amdgpu_buffer_rsrc_t rs = make_rsrc_v(x, xbytes);
    f32x4 bm, bi, bg, bb;
    if constexpr (BN) {
      bm = ld4(bn.mean + c);
      bi = ld4(bn.invstd + c);
      bg = ld4(bn.gamma + c);
      bb = ld4(bn.beta + c);
    }
    f32x4 wv[R][S];
    load_dw_weights<R, S, WL>(wv, wt, c, C);
    const f32x4 b0 = bias ? ld4(bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 om, oi, og, ob;
    if constexpr (STATS == 2) {
      om = ld4(obn.mean + c);
      oi = ld4(obn.invstd + c);
      og = ld4(obn.gamma + c);
      ob = ld4(obn.beta + c);
    }
    // The input window as a ring: logical row r of output row oh0 + P (P mod PER) is held in slot
    // (P ST + r) % R, so sliding the window down one output row moves no registers -- the row loop
    // is unrolled PER times, one copy per ring phase (the register moves of a shifted window were a
    // seventh of this VALU-bound kernel's instructions)
    // (stride 2 keeps the shifted window: two of its three rows are new each output row, and the
    // unrolled ring took it past 256 registers)
    constexpr bool RING = ST == 1;
    constexpr int PER = RING ? R / std::gcd(R, ST) : 1;
    f32x4 win[R][NC];
    // the join (JOIN): operand b's resource, both operands' BatchNorm terms, and the rows / columns
    // of the window this thread stores y for (input rows oh0 ST .. oh1 ST - 1, columns q = 1 .. 4 ST)
    const __amdgpu_buffer_rsrc_t rjb = make_rsrc_v(JOIN ? jf.b : nullptr, JOIN ? xbytes : 0u);
    const int own_r0 = oh0 * ST, own_r1 = oh1 * ST;
    // y = ReLU(bnA(a) + bnB(b)) for one window row from its raw operands; stored where this thread owns it
    auto join_row = [&](f32x4 (&dst)[NC], const f32x4* ra, const f32x4* rb, int ih) __attribute__((always_inline)) {
      const bool rv = (unsigned)ih < (unsigned)H;
      const bool own = rv && ih >= own_r0 && ih < own_r1;
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const int iw = iw0 + q;
        const bool ok = rv && (unsigned)iw < (unsigned)W;
        f32x4 va = ra[q], vb = rb[q];
        if (jf.ba.mean) va = bn_in4(va, jtab[0][cq], jtab[1][cq], jtab[2][cq], jtab[3][cq], jf.ba.relu);
        if (jf.bb.mean) vb = bn_in4(vb, jtab[4][cq], jtab[5][cq], jtab[6][cq], jtab[7][cq], jf.bb.relu);
        f32x4 v = va + vb;
        uint32_t m = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool pos = v[e] > 0.f;
          v[e] = pos ? v[e] : 0.f;
          m |= (uint32_t)pos << (8 * e);
        }
        dst[q] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
        if (q >= 1 && q <= TW * ST && own && ok) {
          const size_t e0 = ((size_t)(n * H + ih) * W + iw) * C + c;
          st4(jf.y + e0, v);
          if (jf.mask) *reinterpret_cast<uint32_t*>(jf.mask + e0) = m;
        }
      }
    };
    auto join_load = [&](f32x4 (&dst)[NC], int ih) __attribute__((always_inline)) {
      f32x4 ra[NC], rb[NC];
      const bool rv = (unsigned)ih < (unsigned)H;
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const bool ok = rv && (unsigned)(iw0 + q) < (unsigned)W;
        const uint32_t e = (uint32_t)(((n * H + ih) * W + iw0 + q) * C + c);
        ra[q] = bload4e<float>(rs, ok, e);
        rb[q] = bload4e<float>(rjb, ok, e);
      }
      join_row(dst, ra, rb, ih);
    };
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if constexpr (JOIN)
        join_load(win[r], oh0 * ST - pad + r);
      else
        load_row<NC, BN, RELU, T>(win[r], rs, n, oh0 * ST - pad + r, iw0, H, W, C, c, bm, bi, bg, bb);
    }
    // stride 1: the next output row's new input row is loaded one row ahead (bf16 kept packed, 2
    // registers per 4 channels) and widened / normalised when it enters the window; stride 2 loads
    // it in the row that uses it (its window leaves no registers for a prefetch)
    constexpr bool PFR = ST == 1 && R == 3;
    using PT = typename std::conditional<sizeof(T) == 2, uint2, f32x4>::type;
    PT pre[PFR ? NC : 1];
    f32x4 preb[(PFR && JOIN) ? NC : 1];
    // (unconditional: a row past the segment reads nothing.  Issued under a branch, the loads went
    // to temporaries copied into pre at the branch's end, which waited for them right there -- the
    // prefetch was never in flight under the row's FMAs)
    auto load_pre = [&](int ih, bool live_row) {
      if constexpr (PFR) {
        const bool rv = live_row && (unsigned)ih < (unsigned)H;
#pragma unroll
        for (int q = 0; q < NC; ++q) {
          const bool ok = rv && (unsigned)(iw0 + q) < (unsigned)W;
          const uint32_t e = (uint32_t)(((n * H + ih) * W + iw0 + q) * C + c);
          if constexpr (JOIN) preb[q] = bload4e<float>(rjb, ok, e);
          if constexpr (sizeof(T) == 2)
            pre[q] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(ok ? e * 2u : kOOBBytes),
                                                                                    0, 0));
          else
            pre[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(ok ? e * 4u : kOOBBytes),
                                                                                     0, 0));
        }
      }
    };
    load_pre((oh0 + 1) * ST - pad + R - 1, oh0 + 1 < oh1);
    // one output row at ring phase P; false once the segment is done
    auto row = [&](int oh, auto PC) __attribute__((always_inline)) -> bool {
      constexpr int P = decltype(PC)::value;
      if (oh >= oh1) return false;
      // this row's residual / BN-input operands (dgrad only), issued ahead of the window
      // loads and FMAs
      const size_t pix0 = (size_t)(n * OH + oh) * OW + ow0;
      f32x4 rv[TW], xv[TW];
      if constexpr (WL == 2) {
#pragma unroll
        for (int j = 0; j < TW; ++j) {
          const bool in = ow0 + j < OW;
          rv[j] = (res && in) ? ld4(res + (pix0 + j) * C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
          if constexpr (STATS == 2) xv[j] = in ? ld4(xo + (pix0 + j) * C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      if (oh > oh0) {
        if constexpr (!RING) {
#pragma unroll
          for (int r = 0; r + ST < R; ++r)
#pragma unroll
            for (int q = 0; q < NC; ++q) win[r][q] = win[r + ST][q];
        }
        // the ST rows that enter the window: logical rows R - ST .. R - 1
#pragma unroll
        for (int r = R - ST; r < R; ++r) {
          if (r < 0) continue;
          const int slot = RING ? (P * ST + r) % R : r;
          if constexpr (PFR && JOIN) {
            join_row(win[slot], pre, preb, oh * ST - pad + r);
            load_pre((oh + 1) * ST - pad + R - 1, oh + 1 < oh1);
          } else if constexpr (PFR) {
            // the prefetched row: widened, BN applied on the in-image elements (as load_row)
            const int ih = oh * ST - pad + r;
            const bool rv = (unsigned)ih < (unsigned)H;
#pragma unroll
            for (int q = 0; q < NC; ++q) {
              f32x4 v;
              if constexpr (sizeof(T) == 2)
                v = bf16x4_to_f32(pre[q]);
              else
                v = pre[q];
              if constexpr (BN) {
                const bool ok = rv && (unsigned)(iw0 + q) < (unsigned)W;
                const f32x4 t = bn_in4p<RELU>(v, bm, bi, bg, bb);
                v = ok ? t : f32x4{0.f, 0.f, 0.f, 0.f};
              }
              win[slot][q] = v;
            }
            load_pre((oh + 1) * ST - pad + R - 1, oh + 1 < oh1);
          } else if constexpr (JOIN) {
            // (stride 2: both entering rows' operands are loaded before either is joined, below)
            if (r == R - ST) {
              f32x4 ra[ST][NC], rb[ST][NC];
#pragma unroll
              for (int k = 0; k < ST; ++k) {
                const int ih = oh * ST - pad + r + k;
                const bool rv = (unsigned)ih < (unsigned)H;
#pragma unroll
                for (int q = 0; q < NC; ++q) {
                  const bool ok = rv && (unsigned)(iw0 + q) < (unsigned)W;
                  const uint32_t e = (uint32_t)(((n * H + ih) * W + iw0 + q) * C + c);
                  ra[k][q] = bload4e<float>(rs, ok, e);
                  rb[k][q] = bload4e<float>(rjb, ok, e);
                }
              }
#pragma unroll
              for (int k = 0; k < ST; ++k) join_row(win[r + k], ra[k], rb[k], oh * ST - pad + r + k);
            }
          } else {
            load_row<NC, BN, RELU, T>(win[slot], rs, n, oh * ST - pad + r, iw0, H, W, C, c, bm, bi, bg, bb);
          }
        }
      }
      T* yrow = y + ((size_t)(n * OH + oh) * OW) * C + c;
      // bf16 statistics: the row's (at most TW) stored values summed in fp32 first -- their 8-bit
      // significands (16-bit squares) add exactly unless they span more than ~8 binades -- and
      // added to the fp64 sums once per row: a third of the fp64 work of this VALU-bound kernel
      constexpr bool RS = STATS == 1 && sizeof(T) == 2;
      f32x4 r1 = {0.f, 0.f, 0.f, 0.f}, r2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < TW; ++j) {
        // (the first tap's fma takes the bias as its addend: no copy of b0 per output)
        f32x4 acc = win[RING ? (P * ST) % R : 0][j * ST] * wv[0][0] + b0;
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int s = 0; s < S; ++s)
            if (r + s > 0) acc += win[RING ? (P * ST + r) % R : r][j * ST + s] * wv[r][s];
        if (ow0 + j < OW) {
          if constexpr (WL == 2) {
            if (res) acc += rv[j];  // residual addend
          }
          acc = st4_kept(yrow + (size_t)(ow0 + j) * C, acc, nt);  // acc = what the store keeps
          if constexpr (RS) {
            r1 += acc;
#pragma unroll
            for (int e = 0; e < 4; ++e) r2[e] = __builtin_fmaf(acc[e], acc[e], r2[e]);
          } else if constexpr (STATS == 1) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const double v = (double)acc[e];
              s1[e] += v;
              s2[e] += v * v;
            }
          } else if constexpr (STATS == 2) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float g = acc[e];
              const float xh = (xv[j][e] - om[e]) * oi[e];
              if (obn.relu && !(bn_out(xv[j][e], om[e], oi[e], og[e], ob[e]) > 0.f)) g = 0.f;
              s1[e] += (double)g;
              s2[e] += (double)g * (double)xh;
            }
          }
        }
      }
      if constexpr (RS) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s1[e] += (double)r1[e];
          s2[e] += (double)r2[e];
        }
      }
      return true;
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    static_assert(PER >= 1 && PER <= 5, "ring period");
    for (int oh = oh0;; oh += PER) {
      if (!row(oh, I0{})) break;
      if constexpr (PER > 1)
        if (!row(oh + 1, I1{})) break;
      if constexpr (PER > 2)
        if (!row(oh + 2, I2{})) break;
      if constexpr (PER > 3)
        if (!row(oh + 3, I3{})) break;
      if constexpr (PER > 4)
        if (!row(oh + 4, I4{})) break;
    }
  }
  if constexpr (STATS != 0) {
    // fixed-order block reduction over the 256 / C4 threads of each channel group
    // (not padded like the other kernels' tables: the padding did not change this kernel's time)
    __shared__ double red[256][8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[threadIdx.x][e] = s1[e];
      red[threadIdx.x][4 + e] = s2[e];
    }
    __syncthreads();
    const int per = 256 / C4;
    for (int i = threadIdx.x; i < C4 * 8; i += 256) {
      const int g = i >> 3, e = i & 7;
      double a = 0.0;
      for (int k = 0; k < per; ++k) a += red[k * C4 + g][e];
      pub_store(part + ((size_t)blockIdx.x * 2 + (e >> 2)) * C + g * 4 + (e & 3), a);
    }
    if (ft.part) fold_tail<256>(ft, blockIdx.x, 0, C, 0);
  }
}

// Stride > 1 dgrad by sub-pixel decomposition (see SubPix): thread = 4 channels of TWQ
// consecutive ST x ST quads of dx; the dy neighbourhood columns are shared by adjacent quads.
// JOIN: this layer's input is a residual block's output y = ReLU(bn_j(xj) + skip) (the join,
// residual_block.py:75) and the join's ReLU backward and stage 1 of bn_j's backward ride on the
// dx store: dx = (dgrad + res) * mask (the join's stored ReLU mask), partials (sum dx,
// sum dx * xhat_j) -- what dk_relu_bwd_bn_partial_f64 computes from the stored dx, bit for bit
// for dx (activations.py:44-47, batch_norm.py:125-147).
// bnmode (sub-pixel dgrad only): the layer's input is instead a BatchNorm (+ReLU) output applied on
// load (a BNOut); dx is stored as computed (the gradient w.r.t. that BN's output) and the partials
// are stage 1 of that BN's backward, its ReLU mask recomputed from its raw input x
// (dk_bn_bwd_partial_f64, batch_norm.py:125-147) -- x is then of the kernel's storage type.
struct JoinBwd {
  const uint8_t* mask;
  const void* x;  // bn_j's raw input (fp32; bnmode: the BN's raw input, storage type)
  const float* mean;
  const float* invstd;
  int res_lat;  // sub-pixel dgrad: the residual given on the stride-ST lattice only (phase (0, 0)), compact
  const float* gamma;  // bnmode: the BN's affine parameters and ReLU flag
  const float* beta;
  int relu;
  int bnmode;
};

template <int R, int S, int ST, int PAD, class T = float, bool JOIN = false>
__global__ __launch_bounds__(256) void dw_dgrad_subpixel_kernel(const T* __restrict__ dy, uint32_t dybytes,
                                                                const float* __restrict__ wt, T* __restrict__ dx,
                                                                int N, int H, int W, int C, int OH, int OW,
                                                                const T* __restrict__ res, JoinBwd jn,
                                                                double* __restrict__ part, FoldTail ft, int nt) {
  using RP = SubPix<R, ST, PAD>;
  using SP = SubPix<S, ST, PAD>;
  constexpr int DR0 = RP::dmin(), NR = RP::dmax() - RP::dmin() + 1;
  constexpr int DS0 = SP::dmin(), NS = SP::dmax() - SP::dmin() + 1;
  constexpr int TWQ = 4;
  constexpr int NCOL = TWQ + NS - 1;
  const int C4 = C >> 2;
  const int QH = (H + ST - 1) / ST, QW = (W + ST - 1) / ST;
  const int nqc = (QW + TWQ - 1) / TWQ;
  const int blk = xcd_block(blockIdx.x, gridDim.x);
  const long long idx = (long long)blk * blockDim.x + threadIdx.x;
  const bool live = idx < (long long)N * QH * nqc * C4;
  if (!JOIN && !live) return;
  const int cq = (int)(idx % C4);
  long long t = idx / C4;
  const int qc = (int)(t % nqc);
  t /= nqc;
  const int qi = (int)(t % QH);
  const int n = (int)(t / QH);
  const int c = cq * 4;
  const int j0 = qc * TWQ;
  // JOIN (see JoinBwd): the join's mask and bn_j statistics ride on the store; per-thread fp64
  // sums, then a fixed-order block reduction into part[blk][2][C] (a block spans whole pixels:
  // C/4 divides 256)
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  f32x4 jm{}, ji{}, jg{}, jb{};
  if constexpr (JOIN) {
    if (live) {
      jm = ld4(jn.mean + c);
      ji = ld4(jn.invstd + c);
      if (jn.bnmode) {
        jg = ld4(jn.gamma + c);
        jb = ld4(jn.beta + c);
      }
    }
  }
  if (live) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc_v(dy, dybytes);
    f32x4 d[NR][NCOL];
#pragma unroll
    for (int a = 0; a < NR; ++a) {
      const int oh = qi + DR0 + a;
#pragma unroll
      for (int b = 0; b < NCOL; ++b) {
        const int ow = j0 + DS0 + b;
        const bool ok = (unsigned)oh < (unsigned)OH && (unsigned)ow < (unsigned)OW;
        d[a][b] = bload4e<T>(rs, ok, (uint32_t)(((n * OH + oh) * OW + ow) * C + c));
      }
    }
    f32x4 wv[R][S];
    load_dw_weights<R, S, 1>(wv, wt, c, C);  // wt = W[C][R][S]
    // a quad's store operands (residual addend; JOIN: the join mask / BN raw input), as buffer
    // loads one quad ahead: no branch around a load (which made the waitcnt pass drain every
    // memory operation per quad) and the next quad's loads in flight under this quad's FMAs
    const size_t pixels = (size_t)N * H * W;
    const __amdgpu_buffer_rsrc_t rres = make_rsrc_v(
        res, res ? (uint32_t)((JOIN && jn.res_lat ? (size_t)N * QH * QW : pixels) * C * sizeof(T)) : 0u);
    const __amdgpu_buffer_rsrc_t rjx = make_rsrc_v(JOIN ? jn.x : nullptr, JOIN ? (uint32_t)(pixels * C * sizeof(T)) : 0u);
    const __amdgpu_buffer_rsrc_t rjm = make_rsrc_v(JOIN ? jn.mask : nullptr, (JOIN && jn.mask) ? (uint32_t)(pixels * C) : 0u);
    struct QOps {
      f32x4 rv[ST][ST], jx[ST][ST];
      uint32_t jmk[ST][ST];
    };
    auto load_q = [&](int q, QOps& o) {
      const int j = j0 + q;
#pragma unroll
      for (int a = 0; a < ST; ++a)
#pragma unroll
        for (int b = 0; b < ST; ++b) {
          const int h = qi * ST + a, w = j * ST + b;
          const bool ok = j < QW && h < H && w < W;
          const uint32_t off = (uint32_t)((((size_t)n * H + h) * W + w) * C + c);
          if (JOIN && jn.res_lat)  // compact lattice residual: phase (0, 0) only, at quad (qi, j)
            o.rv[a][b] = bload4e<T>(rres, ok && a == 0 && b == 0, (uint32_t)((((size_t)n * QH + qi) * QW + j) * C + c));
          else
            o.rv[a][b] = bload4e<T>(rres, ok, off);
          if constexpr (JOIN) {
            o.jmk[a][b] = __builtin_amdgcn_raw_buffer_load_b32(rjm, (int)(ok ? off : kOOBBytes), 0, 0);
            o.jx[a][b] = bload4e<T>(rjx, ok, off);
          }
        }
    };
    const __amdgpu_buffer_rsrc_t rdx = make_rsrc_v(dx, (uint32_t)(pixels * C * sizeof(T)));
    QOps qo[2];
    load_q(0, qo[0]);
#pragma unroll
    for (int q = 0; q < TWQ; ++q) {
      const int j = j0 + q;
      if (q + 1 < TWQ) load_q(q + 1, qo[(q + 1) & 1]);
      f32x4 acc[ST][ST];
      const QOps& cur = qo[q & 1];
#pragma unroll
      for (int a = 0; a < ST; ++a)
#pragma unroll
        for (int b = 0; b < ST; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int s = 0; s < S; ++s)
          acc[RP::phase(r)][SP::phase(s)] += d[RP::nb(r) - DR0][q + SP::nb(s) - DS0] * wv[r][s];
#pragma unroll
      for (int a = 0; a < ST; ++a) {
        const int h = qi * ST + a;
#pragma unroll
        for (int b = 0; b < ST; ++b) {
          const int w = j * ST + b;
          // unconditional: a pixel outside dx is dropped by the buffer store and adds 0 to the sums
          const bool ok = j < QW && h < H && w < W;
          const uint32_t off = (uint32_t)((((size_t)n * H + h) * W + w) * C + c);
          f32x4 o = res ? acc[a][b] + cur.rv[a][b] : acc[a][b];
          if constexpr (JOIN) {
            if (jn.bnmode) {
              o = rnd4<T>(o);  // the partials see dx as stored
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float xv = cur.jx[a][b][e];
                const float xn = (xv - jm[e]) * ji[e];
                const bool kill = !ok || (jn.relu && !(bn_out(xv, jm[e], ji[e], jg[e], jb[e]) > 0.f));
                const float g = kill ? 0.f : o[e];
                s1[e] += (double)g;
                s2[e] += (double)g * (double)xn;
              }
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                if (!((cur.jmk[a][b] >> (8 * e)) & 0xffu)) o[e] = 0.f;  // dy * mask (activations.py:46)
                const float xn = (cur.jx[a][b][e] - jm[e]) * ji[e];
                const float g = ok ? o[e] : 0.f;
                s1[e] += (double)g;
                s2[e] += (double)g * (double)xn;
              }
            }
          }
          bstore4e_nt<T>(rdx, ok, off, o, nt);
        }
      }
    }
  }
  if constexpr (JOIN) {
    __shared__ double red[256][9];  // (padded: [256][8] put 16 lanes' writes on one bank pair)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[threadIdx.x][e] = s1[e];
      red[threadIdx.x][4 + e] = s2[e];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < C * 2; i += 256) {  // i = (which, channel)
      const int which = i / C, ch = i - which * C;
      const int q4 = ch >> 2, e = ch & 3;
      double a = 0.0;
      for (int k = q4; k < 256; k += C4) a += red[k][4 * which + e];
      pub_store(part + ((size_t)blk * 2 + which) * C + ch, a);
    }
    if (ft.part) fold_tail<256>(ft, blk, 0, C, 0);
  }
}

// General-stride dgrad gather (used for stride > 1 geometries without a sub-pixel kernel):
// dx[n,h,w,c] = sum_{r,s : h + pad - r = oh*st, w + pad - s = ow*st} w[r][s][c] * dy[n,oh,ow,c]
template <int R, int S>
__global__ __launch_bounds__(256) void dw_dgrad_gather_kernel(const float* __restrict__ dy,
                                                              const float* __restrict__ wt, float* __restrict__ dx,
                                                              int N, int H, int W, int C, int OH, int OW, int st,
                                                              int pad) {
  const int C4 = C >> 2;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)N * H * W * C4;
  if (idx >= total) return;
  const int cq = (int)(idx % C4);
  long long t = idx / C4;
  const int w = (int)(t % W);
  t /= W;
  const int h = (int)(t % H);
  const int n = (int)(t / H);
  const int c = cq * 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int hh = h + pad - r;
    if (hh < 0 || hh % st) continue;
    const int oh = hh / st;
    if (oh >= OH) continue;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int ww = w + pad - s;
      if (ww < 0 || ww % st) continue;
      const int ow = ww / st;
      if (ow >= OW) continue;
      acc += ld4(dy + ((size_t)(n * OH + oh) * OW + ow) * C + c) * ld4(wt + (r * S + s) * C + c);
    }
  }
  st4(dx + idx * 4, acc);
}

// wgrad partials: part[blk][c][r*S+s] = sum over the block's (n, oh, ow-chunk) items of
// dy[n,oh,ow,c] * x[n, oh*ST + r - pad, ow*ST + s - pad, c].  Thread (cq, pl): channel group
// cq, walks items pl, pl + PL, ...; per item it loads the input strip and TW dy values at once.
template <int ST>
struct DwWgTile {
  static constexpr int TW = ST == 1 ? 4 : 2;
};

// Items of the weight-gradient walk: (n, column chunk of TW outputs, segment of kWgSeg output
// rows).  Down a segment the R-row input window slides by ST rows per output row, so each
// output row loads ST new input rows instead of R.
constexpr int kWgSeg = 8;

template <int R, int S, int ST, bool BN, class T = float>
__global__ __launch_bounds__(256) void dw_wgrad_partial_kernel(const T* __restrict__ dy, uint32_t dybytes,
                                                               const T* __restrict__ x, uint32_t xbytes,
                                                               float* __restrict__ part, int N, int H, int W,
                                                               int C, int OH, int OW, int pad, int ipb, BnIn bn) {
  constexpr int RS = R * S;
  constexpr int TW = DwWgTile<ST>::TW;
  constexpr int NC = (TW - 1) * ST + S;
  extern __shared__ float red[];  // [256][RS][4]
  const int C4 = C >> 2;
  const int cgt = C4 < 256 ? C4 : 256;
  const int PL = 256 / cgt;
  const int tid = threadIdx.x;
  const int cq = blockIdx.y * cgt + tid % cgt;
  const int pl = tid / cgt;
  const bool active = pl < PL && cq < C4;
  const int c = cq * 4;
  const int nwc = (OW + TW - 1) / TW;
  const int nseg = (OH + kWgSeg - 1) / kWgSeg;
  const int items = N * nseg * nwc;
  const int i0 = blockIdx.x * ipb, i1 = min(items, i0 + ipb);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc_v(x, xbytes), rg = make_rsrc_v(dy, dybytes);
  f32x4 bm, bi, bg, bb;
  if constexpr (BN) {
    const int cc = active ? c : 0;
    bm = ld4(bn.mean + cc);
    bi = ld4(bn.invstd + cc);
    bg = ld4(bn.gamma + cc);
    bb = ld4(bn.beta + cc);
  }
  f32x4 acc[R][S];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int s = 0; s < S; ++s) acc[r][s] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (active) {
    for (int it = i0 + pl; it < i1; it += PL) {
      const int wc = it % nwc;
      const int t = it / nwc;
      const int sg = t % nseg;
      const int n = t / nseg;
      const int ow0 = wc * TW;
      const int iw0 = ow0 * ST - pad;
      const int oh0 = sg * kWgSeg, oh1 = min(OH, oh0 + kWgSeg);
      f32x4 win[R][NC];
#pragma unroll
      for (int r = 0; r < R; ++r)
        load_row<NC, BN, T>(win[r], rx, n, oh0 * ST - pad + r, iw0, H, W, C, c, bn, bm, bi, bg, bb);
      for (int oh = oh0; oh < oh1; ++oh) {
        if (oh > oh0) {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            if (r + ST < R) {
#pragma unroll
              for (int q = 0; q < NC; ++q) win[r][q] = win[r + ST][q];
            } else {
              load_row<NC, BN, T>(win[r], rx, n, oh * ST - pad + r, iw0, H, W, C, c, bn, bm, bi, bg, bb);
            }
          }
        }
        f32x4 g[TW];
#pragma unroll
        for (int j = 0; j < TW; ++j)
          g[j] = bload4e<T>(rg, ow0 + j < OW, (uint32_t)(((n * OH + oh) * OW + ow0 + j) * C + c));
#pragma unroll
        for (int j = 0; j < TW; ++j)
#pragma unroll
          for (int r = 0; r < R; ++r)
#pragma unroll
            for (int s = 0; s < S; ++s) acc[r][s] += g[j] * win[r][j * ST + s];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int s = 0; s < S; ++s) st4(red + (tid * RS + r * S + s) * 4, acc[r][s]);
  __syncthreads();
  // Fixed-order reduction over the PL pixel lanes of each (channel group, tap).
  const int nitems = cgt * RS * 4;
  for (int k = tid; k < nitems; k += 256) {
    const int e = k % 4;
    const int tap = (k / 4) % RS;
    const int gq = k / (4 * RS);
    if (blockIdx.y * cgt + gq >= C4) continue;
    float sum = 0.f;
    for (int q = 0; q < PL; ++q) sum += red[((q * cgt + gq) * RS + tap) * 4 + e];
    const int cc = (blockIdx.y * cgt + gq) * 4 + e;
    part[((size_t)blockIdx.x * C + cc) * RS + tap] = sum;
  }
}

// The whole stride-1 depthwise backward in one pass, when the layer's output fed a BatchNorm
// (the depthwise_sep_layer's dw -> BN -> pw, example :34-70): the layer's gradient
// dy = BN backward(g, x1) (stage 3 of batch_norm.py:125-174, = dk_bn_bwd_apply_f32 bit for bit)
// is formed once per element in LDS and never stored; the same 3x3 window of it feeds
//   dx[h][w]   = sum_{r,s} W[2-r][2-s] * dy[h-1+r][w-1+s]                      (pad 1)
//   dW[a][b]  += xb[h][w] * dy[h+1-a][w+1-b]                                  (per-block partials)
// where xb is the layer's input (bn_in(X) when it consumed a BNOut).  Reindexing the weight
// gradient (depthwise_convolution.py:198-221) by input pixel makes its dy taps exactly the
// dgrad's window.
// Block = a run of images (nranges runs over the batch; one image each when the grid fits the
// chip anyway), a CL-column strip, CG channel groups of 4 (CG * CL = 256); it walks the rows of
// its images top to bottom as one tall image -- the zero dy row H of an image is row -1 of the
// next, so the 3x3 window and the one-row prefetch run on across image boundaries and a small
// image's blocks do not each pay the prologue and the reductions.  Per row: the block forms dy row h+1 for its CL + 2 columns into one of two
// LDS slots (g and x1 for the row after were loaded one iteration earlier), one barrier, then
// each thread slides its 3x3 register window down by that row and produces dx[h][w] for its 4
// channels.  dx is bit-identical to dk_bn_bwd_apply_f32 -> dk_dwconv_dgrad_ex_f32 (same tap
// order); the input BatchNorm's backward partials (spart) and the weight-gradient partials
// (wpart) are per-block fixed-order sums, one row per (image, strip), each block writing its
// channel range.
struct BnBwdOut {  // the BatchNorm after this layer: dy = bn_bwd_elem(x1, g)
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  const float* k12;
  int relu;
};

// T: activation storage (float, or bf16_t for BASELINE config 5): g, x1, x, dx and res are T,
// dy stays fp32 (LDS ring), and the input BN's partials see dx as stored (rounded).
// CPT: adjacent output columns per thread (CL / CPT threads per channel group).  With 2 a thread's
// 3 x 4 window and its per-channel terms (LDS ptab, one read per row) serve two pixels: per element
// half the LDS reads, the bound of the one-column form on bf16 (twice the elements per byte).
// RES: a residual addend may be given (false: none -- its loads and widening are compiled out).
// JM (JOIN): the join's ReLU mask bytes may be given (false: the mask is y > 0, no mask loads).
template <bool BNX, bool STATS, bool RELU1, bool JOIN = false, class T = float, int CPT = 1, int NT = 256,
          bool RES = true, bool JM = true>
__global__ __launch_bounds__(NT, NT == 64 ? 2 : 1) void dw_bwd_fused_kernel(const T* __restrict__ g, const T* __restrict__ x1,
                                                           uint32_t bytes, BnBwdOut ob, const T* __restrict__ x,
                                                           BnIn bn, const float* __restrict__ w_crs,
                                                           T* __restrict__ dx, const T* __restrict__ res,
                                                           double* __restrict__ spart, float* __restrict__ wpart,
                                                           int N, int H, int W, int C, int CL, FoldTail ft,
                                                           JoinBwd jn = JoinBwd{}, int nt = 0, int nranges = 0) {
  static_assert(!(JOIN && sizeof(T) != 4), "the join fusion is fp32 only");
  static_assert(CPT == 1 || CPT == 2, "columns per thread");
  static_assert(!STATS || BNX, "input-BN partials need the input BN");
  static_assert(!(JOIN && (STATS || BNX)), "the join's partials replace the input BN's");
  constexpr bool PART = STATS || JOIN;
  const int CP = CL / CPT;               // threads per channel group
  const int CG = NT / CP;                // channel groups per block
  const int NI = (CL + 2) * CG;         // dy float4s per LDS row (with the 1-column halos)
  constexpr int R = 3, S = 3, RS = 9, WC = CPT + 2;  // window columns
  extern __shared__ f32x4 ring[];       // [2][NI]; reused by the final reductions
  const int tid = threadIdx.x;
  const int cg = tid % CG, cl = tid / CG;
  const int nct = (W + CL - 1) / CL, ncht = (C >> 2) / CG;
  const int bid = xcd_block(blockIdx.x, gridDim.x);
  const int cht = bid % ncht;
  const int strip = bid / ncht;  // (image run, column strip): the partial-sum row
  const int ct = strip % nct, nr = strip / nct;
  const int n0 = nranges ? (int)((long long)nr * N / nranges) : nr;
  const int n1 = nranges ? (int)((long long)(nr + 1) * N / nranges) : nr + 1;
  const int c = (cht * CG + cg) * 4;
  const int w = ct * CL + CPT * cl;  // this thread's first output column
  bool win_ok[CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) win_ok[j] = w + j < W;
  const int wl = ct * CL - 1;  // LDS column 0
  // this thread's dy items: columns wl + CPT cl + j (LDS columns CPT cl + j) and, for tid < 2 CG
  // (wave 0), the halo column wl + CL + cl, channel c
  const bool two = tid < 2 * CG;
  const int col0 = wl + CPT * cl, col1 = wl + CL + cl;
  bool cok0[CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) cok0[j] = (unsigned)(col0 + j) < (unsigned)W;
  const bool cok1 = two && (unsigned)col1 < (unsigned)W;
  const __amdgpu_buffer_rsrc_t rg = make_rsrc_v(g, bytes), r1 = make_rsrc_v(x1, bytes), rx = make_rsrc_v(x, bytes);
  // the optional operands as buffers too (an absent one covers 0 bytes: its loads return 0), so
  // every load of the row loop is an unconditional buffer load and the waitcnt pass keeps the
  // dx store of a row in flight across the loop's back edge (a branch around a global load made
  // it wait for everything, stores included, at the end of every row)
  const __amdgpu_buffer_rsrc_t rres = make_rsrc_v(res, res ? bytes : 0u);
  const __amdgpu_buffer_rsrc_t rjx = make_rsrc_v(JOIN ? jn.x : nullptr, JOIN ? bytes : 0u);
  const __amdgpu_buffer_rsrc_t rjm = make_rsrc_v(JOIN ? jn.mask : nullptr, (JOIN && jn.mask) ? bytes / 4u : 0u);
  // the per-channel BatchNorm terms and the (flipped) filters live in LDS, read where used:
  // held in registers they kept the kernel at 2 waves per SIMD, too few to hide a row's loads
  __shared__ f32x4 ptab[13 + RS][NT == 64 ? 16 : 32];  // [term][channel group]; CG <= 32 (16: dwb_geom)
  for (int i = tid; i < 13 * CG; i += NT) {
    const int t = i / CG, q = i - t * CG;
    const int cc = (cht * CG + q) * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    switch (t) {
      case 0: v = ld4(ob.mean + cc); break;
      case 1: v = ld4(ob.invstd + cc); break;
      case 2: v = ld4(ob.k12 + cc); break;
      case 3: v = ld4(ob.k12 + C + cc); break;
      case 4: v = ld4(ob.gamma + cc) * ld4(ob.invstd + cc); break;
      case 5: if (RELU1) v = ld4(ob.gamma + cc); break;
      case 6: if (RELU1) v = ld4(ob.beta + cc); break;
      case 7: if (BNX) v = ld4(bn.mean + cc); break;
      case 8: if (BNX) v = ld4(bn.invstd + cc); break;
      case 9: if (BNX) v = ld4(bn.gamma + cc); break;
      case 10: if (BNX) v = ld4(bn.beta + cc); break;
      case 11: if (JOIN) v = ld4(jn.mean + cc); break;
      default: if (JOIN) v = ld4(jn.invstd + cc); break;
    }
    ptab[t][q] = v;
  }
  if (tid < CG) {
    f32x4 wv0[R][S];
    load_dw_weights<R, S, 2>(wv0, w_crs, c, C);  // flipped taps
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int s = 0; s < S; ++s) ptab[13 + r * S + s][cg] = wv0[r][s];
  }
  __syncthreads();
#define om ptab[0][cg]
#define oi ptab[1][cg]
#define ok1 ptab[2][cg]
#define ok2 ptab[3][cg]
#define of ptab[4][cg]
#define og ptab[5][cg]
#define obt ptab[6][cg]
#define bm ptab[7][cg]
#define bi ptab[8][cg]
#define bg ptab[9][cg]
#define bb ptab[10][cg]
#define jm ptab[11][cg]
#define ji ptab[12][cg]
#define WV(r, s) ptab[13 + (r) * S + (s)][cg]
  auto xform = [&](f32x4 gv, f32x4 xv, bool ok) {
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float ge = gv[e];
      if constexpr (RELU1) {
        if (!(bn_out(xv[e], om[e], oi[e], og[e], obt[e]) > 0.f)) ge = 0.f;
      }
      o[e] = bn_bwd_elem(xv[e], ge, om[e], oi[e], of[e], ok1[e], ok2[e]);
    }
    return ok ? o : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto pix = [&](int nn, int hh, int ww) { return (uint32_t)(((nn * H + hh) * W + ww) * C + c); };
  // Prefetched operands, PF rows ahead: raw g / x1 of the dy rows to publish, and this thread's
  // input / residual (/ join mask and bn_j input) of the dx rows to finish.  bf16 keeps them packed
  // (2 registers per 4 channels, widened where used) two rows ahead -- the same registers one fp32
  // row takes -- so twice the bytes are in flight per row step; fp32 stays one row ahead.
  using Raw = typename std::conditional<sizeof(T) == 2, uint2, f32x4>::type;
  constexpr int PF = sizeof(T) == 2 ? 2 : 1;
  struct DyQ {
    Raw g0[CPT], x0[CPT], g1, x1;
  };
  struct XQ {
    Raw xr[CPT], rv[CPT];
    f32x4 jxin[CPT];    // (the kernel's #defines take jm / ji)
    uint32_t jmask[CPT];
  };
  DyQ dq[PF];
  XQ xq[PF];
  auto raw_load = [&](__amdgpu_buffer_rsrc_t r, bool ok, uint32_t e) -> Raw {
    if constexpr (sizeof(T) == 2)
      return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)(ok ? e * 2u : kOOBBytes), 0, 0));
    else
      return bload4e<float>(r, ok, e);
  };
  auto widen = [](Raw v) -> f32x4 {
    if constexpr (sizeof(T) == 2)
      return bf16x4_to_f32(v);
    else
      return v;
  };
  // unconditional loads (rows past the run or the zero row H read nothing): no branch around a
  // load, so the waitcnt pass counts them instead of draining every memory operation
  auto load_dy_row = [&](DyQ& q, int nn, int hh) {
    const bool rok = (unsigned)hh < (unsigned)H && nn < n1;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      q.g0[j] = raw_load(rg, rok && cok0[j], pix(nn, hh, col0 + j));
      q.x0[j] = raw_load(r1, rok && cok0[j], pix(nn, hh, col0 + j));
    }
    q.g1 = raw_load(rg, rok && cok1, pix(nn, hh, col1));
    q.x1 = raw_load(r1, rok && cok1, pix(nn, hh, col1));
  };
  auto load_x_row = [&](XQ& q, int nn, int hh) {
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const bool okj = win_ok[j] && hh < H && nn < n1;
      q.xr[j] = raw_load(rx, okj, pix(nn, hh, w + j));
      if constexpr (RES)
        q.rv[j] = raw_load(rres, okj, pix(nn, hh, w + j));
      else
        q.rv[j] = Raw{};
      if constexpr (JOIN) {
        if constexpr (JM)
          q.jmask[j] = __builtin_amdgcn_raw_buffer_load_b32(rjm, (int)(okj ? pix(nn, hh, w + j) : kOOBBytes), 0, 0);  // 4 mask bytes
        else
          q.jmask[j] = 0u;
        q.jxin[j] = bload4e<float>(rjx, okj, pix(nn, hh, w + j));
      }
    }
  };
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  f32x4 wacc[R][S];
  f32x4 d[R][WC];
#pragma unroll
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int s = 0; s < S; ++s) wacc[r][s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < WC; ++s) d[r][s] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // load cursors: the (image, row) of the dy row PF steps ahead (row H = the zero row) and of the
  // next x row (rows 0 .. H-1 of each image of the run)
  constexpr bool ROT = sizeof(T) == 2 && CPT == 2;
  int pn = n0, prr = 0, xn = n0, xhh = 0;
  // the x queue: the next x row (rows 0 .. H-1 of each image of the run); ROT: one entry per
  // iteration instead, the first of each image empty (the iteration that publishes an image's row
  // 0 finishes no dx row), so that its slots rotate with the iterations (xhh = entry, row xhh - 1)
  auto next_x = [&](XQ& q) {
    if constexpr (ROT) {
      load_x_row(q, xhh > 0 ? xn : n1, xhh - 1);
      if (++xhh > H) xhh = 0, ++xn;
    } else {
      load_x_row(q, xn, xhh);
      if (++xhh == H) xhh = 0, ++xn;
    }
  };
#pragma unroll
  for (int k = 0; k < PF; ++k) {
    load_dy_row(dq[k], pn, prr);
    if (++prr > H) prr = 0, ++pn;
    next_x(xq[k]);
  }
  // ROT (bf16, two columns per thread): the row loop is unrolled by 6 (a multiple of the 3 window
  // rows, of PF and of the 2 LDS slots) and the window and both load queues rotate by name -- phase
  // P publishes into d[P % 3] and consumes / refills slot P % PF -- instead of by register copies:
  // the copy of a queue slot at the loop latch waited for the loads still in flight (s_waitcnt
  // vmcnt near 0 on the back edge), so no load stayed in flight across iterations.
  // 512 x 56 x 56 x 64: 282 -> 251-270 us; config 5 6.16 -> 6.06 ms
  // (profiles/r05ac_dwb_bf16_rotated_queue.txt).  fp32 and one column per thread keep the original
  // loop: rotated, they took more registers (the one-column kernels lost their third wave per SIMD;
  // profiles/r05aa_dwb_rotation_experiments.txt).
  if constexpr (ROT) {
    int n = n0, rr = 0, it = 0;
    auto step = [&](auto ph) __attribute__((always_inline)) {
      constexpr int P = decltype(ph)::value;
      constexpr int QP = ROT ? P % PF : 0, WP = ROT ? P % 3 : 0;
      const int rowok = rr < H;
      f32x4 d0[CPT];
  #pragma unroll
      for (int j = 0; j < CPT; ++j) d0[j] = xform(widen(dq[QP].g0[j]), widen(dq[QP].x0[j]), rowok && cok0[j]);
      // the halo columns: wave 0 only (2 CG <= 64) -- a wave-uniform branch with two columns per thread
      f32x4 d1 = {0.f, 0.f, 0.f, 0.f};
      if (CPT == 1 || tid < 64) d1 = xform(widen(dq[QP].g1), widen(dq[QP].x1), rowok && cok1);
      if constexpr (ROT) {
        load_dy_row(dq[QP], pn, prr);
      } else {
  #pragma unroll
        for (int k = 0; k + 1 < PF; ++k) dq[k] = dq[k + 1];
        load_dy_row(dq[PF - 1], pn, prr);
      }
      if (++prr > H) prr = 0, ++pn;
      f32x4* slot = ring + (ROT ? (P & 1) : (it & 1)) * NI;
      ++it;
  #pragma unroll
      for (int j = 0; j < CPT; ++j) slot[(CPT * cl + j) * CG + cg] = d0[j];  // = slot[tid] for CPT 1
      if (two) slot[CL * CG + tid] = d1;
      __syncthreads();
  #pragma unroll
      for (int s = 0; s < WC; ++s) {
        if constexpr (ROT) {
          d[WP][s] = slot[(CPT * cl + s) * CG + cg];  // window row r now in d[(WP + 1 + r) % 3]
        } else {
          d[0][s] = d[1][s];
          d[1][s] = d[2][s];
          d[2][s] = slot[(CPT * cl + s) * CG + cg];
        }
      }
      const int nn = n;
      if (++rr > H) {
        rr = 0;
        ++n;
      }
      if (rr == 1) {  // just published row 0 of an image: no dx row to finish yet
        if constexpr (ROT) next_x(xq[QP]);  // (its empty entry)
        return;
      }
      const int h = (rr == 0 ? H + 1 : rr) - 2;  // the dx row of image nn finished now
      f32x4 xh[CPT], rh[CPT];
  #pragma unroll
      for (int q = 0; q < CPT; ++q) {
        xh[q] = widen(xq[QP].xr[q]);
        rh[q] = RES ? widen(xq[QP].rv[q]) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      f32x4 jh[CPT];
      uint32_t jmh[CPT];
  #pragma unroll
      for (int q = 0; q < CPT; ++q) {
        jh[q] = xq[QP].jxin[q];
        jmh[q] = xq[QP].jmask[q];
      }
      if constexpr (ROT) {
        next_x(xq[QP]);
      } else {
  #pragma unroll
        for (int k = 0; k + 1 < PF; ++k) xq[k] = xq[k + 1];
        next_x(xq[PF - 1]);
      }
      T* dxcol = dx ? dx + (size_t)pix(nn, 0, w) : nullptr;
      // the input BN's output (+ReLU) for the weight gradient (bn_relu_out), and its ReLU mask (BN
      // output > 0) kept as 4 bits for the backward partials (recomputing bn_out there re-read the
      // BN terms from LDS once per element)
      f32x4 xb[CPT];
      uint32_t rmask[CPT];
  #pragma unroll
      for (int q = 0; q < CPT; ++q) {
        xb[q] = xh[q];
        rmask[q] = 0xfu;
      }
      if constexpr (BNX) {
        const f32x4 vbm = bm, vbi = bi, vbg = bg, vbb = bb;
  #pragma unroll
        for (int q = 0; q < CPT; ++q) {
          f32x4 xr;
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            xr[e] = bn_out(xh[q][e], vbm[e], vbi[e], vbg[e], vbb[e]);
            if (!(xr[e] > 0.f)) {
              rmask[q] &= ~(1u << e);
              if (bn.relu) xr[e] = 0.f;
            }
          }
          if (!bn.relu) rmask[q] = 0xfu;
          xb[q] = win_ok[q] ? xr : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      f32x4 acc[CPT];
  #pragma unroll
      for (int q = 0; q < CPT; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  #pragma unroll
      for (int r = 0; r < R; ++r)
  #pragma unroll
        for (int s = 0; s < S; ++s) {
          const f32x4 wv = WV(r, s);
  #pragma unroll
          for (int q = 0; q < CPT; ++q) {
            acc[q] += d[ROT ? (WP + 1 + r) % 3 : r][q + s] * wv;
            wacc[r][s] += d[ROT ? (WP + 1 + r) % 3 : r][q + s] * xb[q];
          }
        }
  #pragma unroll
      for (int q = 0; q < CPT; ++q) {
        if (!win_ok[q]) continue;
        if (RES && res) acc[q] += rh[q];
        T* dxp = dxcol ? dxcol + (size_t)h * W * C + (size_t)q * C : nullptr;
        if constexpr (JOIN) {
          acc[q] = rnd4<T>(acc[q]);
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            // dy * mask (activations.py:46); no mask given: this layer's input is the join's output
            // y = max(v, 0), and y > 0 is exactly the stored mask (v > 0)
            const bool keep = (JM && jn.mask) ? ((jmh[q] >> (8 * e)) & 0xffu) != 0u : xh[q][e] > 0.f;
            if (!keep) acc[q][e] = 0.f;
            const float xn = (jh[q][e] - jm[e]) * ji[e];
            s1[e] += (double)acc[q][e];
            s2[e] += (double)acc[q][e] * (double)xn;
          }
          if (dxp) {
            if (nt)
              st4nt(dxp, acc[q]);
            else
              st4(dxp, acc[q]);
          }
        } else if (dxp) {
          acc[q] = st4_kept(dxp, acc[q], nt);  // acc = what the store keeps
        } else {
          acc[q] = rnd4<T>(acc[q]);
        }
        if constexpr (STATS) {
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            float ge = acc[q][e];
            const float xn = (xh[q][e] - bm[e]) * bi[e];
            if (!((rmask[q] >> e) & 1u)) ge = 0.f;
            s1[e] += (double)ge;
            s2[e] += (double)ge * (double)xn;
          }
        }
      }
    };
    // flattened (image, row) loop: publish dy row rr of image n, then finish dx row rr - 1
    using std::integral_constant;
    const int iters = (n1 - n0) * (H + 1);
    while (it + 6 <= iters) {
      step(integral_constant<int, 0>{});
      step(integral_constant<int, 1>{});
      step(integral_constant<int, 2>{});
      step(integral_constant<int, 3>{});
      step(integral_constant<int, 4>{});
      step(integral_constant<int, 5>{});
    }
    // the last iters % 6 iterations, phases continuing from 0
    const int left = iters - it;
    if (left > 0) step(integral_constant<int, 0>{});
    if (left > 1) step(integral_constant<int, 1>{});
    if (left > 2) step(integral_constant<int, 2>{});
    if (left > 3) step(integral_constant<int, 3>{});
    if (left > 4) step(integral_constant<int, 4>{});
  } else {
    // flattened (image, row) loop: publish dy row rr of image n, then finish dx row rr - 1
    const int iters = (n1 - n0) * (H + 1);
    int n = n0, rr = 0;
    for (int it = 0; it < iters; ++it) {
      const int rowok = rr < H;
      f32x4 d0[CPT];
  #pragma unroll
      for (int j = 0; j < CPT; ++j) d0[j] = xform(widen(dq[0].g0[j]), widen(dq[0].x0[j]), rowok && cok0[j]);
      // the halo columns: wave 0 only (2 CG <= 64) -- a wave-uniform branch with two columns per thread
      f32x4 d1 = {0.f, 0.f, 0.f, 0.f};
      if (CPT == 1 || tid < 64) d1 = xform(widen(dq[0].g1), widen(dq[0].x1), rowok && cok1);
  #pragma unroll
      for (int k = 0; k + 1 < PF; ++k) dq[k] = dq[k + 1];
      load_dy_row(dq[PF - 1], pn, prr);
      if (++prr > H) prr = 0, ++pn;
      f32x4* slot = ring + (it & 1) * NI;
  #pragma unroll
      for (int j = 0; j < CPT; ++j) slot[(CPT * cl + j) * CG + cg] = d0[j];  // = slot[tid] for CPT 1
      if (two) slot[CL * CG + tid] = d1;
      __syncthreads();
  #pragma unroll
      for (int s = 0; s < WC; ++s) {
        d[0][s] = d[1][s];
        d[1][s] = d[2][s];
        d[2][s] = slot[(CPT * cl + s) * CG + cg];
      }
      const int nn = n;
      if (++rr > H) {
        rr = 0;
        ++n;
      }
      if (rr == 1) continue;  // just published row 0 of an image: no dx row to finish yet
      const int h = (rr == 0 ? H + 1 : rr) - 2;  // the dx row of image nn finished now
      f32x4 xh[CPT], rh[CPT];
  #pragma unroll
      for (int q = 0; q < CPT; ++q) {
        xh[q] = widen(xq[0].xr[q]);
        rh[q] = RES ? widen(xq[0].rv[q]) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      f32x4 jh[CPT];
      uint32_t jmh[CPT];
  #pragma unroll
      for (int q = 0; q < CPT; ++q) {
        jh[q] = xq[0].jxin[q];
        jmh[q] = xq[0].jmask[q];
      }
  #pragma unroll
      for (int k = 0; k + 1 < PF; ++k) xq[k] = xq[k + 1];
      load_x_row(xq[PF - 1], xn, xhh);
      if (++xhh == H) xhh = 0, ++xn;
      T* dxcol = dx ? dx + (size_t)pix(nn, 0, w) : nullptr;
      // the input BN's output (+ReLU) for the weight gradient (bn_relu_out), and its ReLU mask (BN
      // output > 0) kept as 4 bits for the backward partials (recomputing bn_out there re-read the
      // BN terms from LDS once per element)
      f32x4 xb[CPT];
      uint32_t rmask[CPT];
  #pragma unroll
      for (int q = 0; q < CPT; ++q) {
        xb[q] = xh[q];
        rmask[q] = 0xfu;
      }
      if constexpr (BNX) {
        const f32x4 vbm = bm, vbi = bi, vbg = bg, vbb = bb;
  #pragma unroll
        for (int q = 0; q < CPT; ++q) {
          f32x4 xr;
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            xr[e] = bn_out(xh[q][e], vbm[e], vbi[e], vbg[e], vbb[e]);
            if (!(xr[e] > 0.f)) {
              rmask[q] &= ~(1u << e);
              if (bn.relu) xr[e] = 0.f;
            }
          }
          if (!bn.relu) rmask[q] = 0xfu;
          xb[q] = win_ok[q] ? xr : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      f32x4 acc[CPT];
  #pragma unroll
      for (int q = 0; q < CPT; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  #pragma unroll
      for (int r = 0; r < R; ++r)
  #pragma unroll
        for (int s = 0; s < S; ++s) {
          const f32x4 wv = WV(r, s);
  #pragma unroll
          for (int q = 0; q < CPT; ++q) {
            acc[q] += d[r][q + s] * wv;
            wacc[r][s] += d[r][q + s] * xb[q];
          }
        }
  #pragma unroll
      for (int q = 0; q < CPT; ++q) {
        if (!win_ok[q]) continue;
        if (RES && res) acc[q] += rh[q];
        T* dxp = dxcol ? dxcol + (size_t)h * W * C + (size_t)q * C : nullptr;
        if constexpr (JOIN) {
          acc[q] = rnd4<T>(acc[q]);
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            // dy * mask (activations.py:46); no mask given: this layer's input is the join's output
            // y = max(v, 0), and y > 0 is exactly the stored mask (v > 0)
            const bool keep = (JM && jn.mask) ? ((jmh[q] >> (8 * e)) & 0xffu) != 0u : xh[q][e] > 0.f;
            if (!keep) acc[q][e] = 0.f;
            const float xn = (jh[q][e] - jm[e]) * ji[e];
            s1[e] += (double)acc[q][e];
            s2[e] += (double)acc[q][e] * (double)xn;
          }
          if (dxp) {
            if (nt)
              st4nt(dxp, acc[q]);
            else
              st4(dxp, acc[q]);
          }
        } else if (dxp) {
          acc[q] = st4_kept(dxp, acc[q], nt);  // acc = what the store keeps
        } else {
          acc[q] = rnd4<T>(acc[q]);
        }
        if constexpr (STATS) {
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            float ge = acc[q][e];
            const float xn = (xh[q][e] - bm[e]) * bi[e];
            if (!((rmask[q] >> e) & 1u)) ge = 0.f;
            s1[e] += (double)ge;
            s2[e] += (double)ge * (double)xn;
          }
        }
      }
    }
  }
  // fixed-order block reductions over the CP column lanes of each channel group
  __syncthreads();
  if constexpr (PART) {
    double(*red)[8] = reinterpret_cast<double(*)[8]>(ring);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[tid][e] = s1[e];
      red[tid][4 + e] = s2[e];
    }
    __syncthreads();
    for (int i = tid; i < CG * 8; i += NT) {
      const int gq = i >> 3, e = i & 7;
      double a = 0.0;
      for (int k = 0; k < CP; ++k) a += red[k * CG + gq][e];
      pub_store(spart + ((size_t)strip * 2 + (e >> 2)) * C + (cht * CG + gq) * 4 + (e & 3), a);
    }
    __syncthreads();
  }
  float* wred = reinterpret_cast<float*>(ring);  // [NT][RS][4]
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int s = 0; s < S; ++s) st4(wred + (tid * RS + r * S + s) * 4, wacc[r][s]);
  __syncthreads();
  // wpart[strip][c][a][b], (a, b) = (2-r, 2-s)
  for (int i = tid; i < CG * 4 * RS; i += NT) {
    const int cc = i / RS, tap = i - cc * RS;
    const int a = tap / S, b = tap - a * S;
    const int gq = cc >> 2, e = cc & 3;
    const int fl = (R - 1 - a) * S + (S - 1 - b);
    float sum = 0.f;
    for (int k = 0; k < CP; ++k) sum += wred[((k * CG + gq) * RS + fl) * 4 + e];
    wpart[((size_t)strip * C + cht * CG * 4) * RS + i] = sum;
  }
  if constexpr (PART) {
    if (ft.part) fold_tail<NT>(ft, strip, cht * CG * 4, CG * 4, cht);
  }
#undef om
#undef oi
#undef ok1
#undef ok2
#undef of
#undef og
#undef obt
#undef bm
#undef bi
#undef bg
#undef bb
#undef jm
#undef ji
#undef WV
}

// The whole stride-2 depthwise backward in one pass (3x3, pad 1; the strided twin of
// dw_bwd_fused_kernel): the layer's gradient dy = BN backward(g, x1) (the following BatchNorm,
// batch_norm.py:125-174 stage 3) is formed as its window is loaded and never stored, and per
// sub-pixel quad (the ST x ST dx pixels of dw_dgrad_subpixel_kernel) the same dy taps give
//   dx[2i + a][2j + b] = sum over the taps of phase (a, b) of W[r][s] dy[i + nb(r)][j + nb(s)]
//   dW[r][s]         += xb[2i + phase(r)][2j + phase(s)] dy[i + nb(r)][j + nb(s)]
// (depthwise_convolution.py:198-221 reindexed by input pixel), xb = the layer's input as the
// forward saw it (BNX: the input BatchNorm (+ReLU) applied on load).  dx is bit-identical to
// dk_bn_bwd_apply -> dk_dwconv_dgrad_ex (same dy values in fp32, same tap order); the input BN's
// backward partials (STATS: stage 1 over the stored dx, its ReLU mask recomputed from x) and the
// weight gradient are per-block fixed-order sums.  A thread keeps one channel quad and walks items
// (image, quad row, TWQ-quad column segment) with the grid's stride, so the partial rows are one per
// block, not one per item.
// JOIN (fp32; config 3's downsampling blocks): the layer's input x is a residual block's output
// y = ReLU(bn_j(x_j) + skip) (residual_block.py:75): dx = (dgrad + residual) * (y > 0) -- the join's
// ReLU backward, its mask read off y, which the weight gradient loads anyway -- and the partials are
// stage 1 of bn_j's backward over that dx (jn.x = x_j, jn.mean / invstd); jn.res_lat: the residual
// is the stride-2 lattice only (a strided skip projection's input gradient, compact).
// RES: a residual addend may be given (false: its loads and adds are compiled out).
template <bool BNX, bool STATS, bool RELU1, class T, bool JOIN = false, bool RES = true>
__global__ __launch_bounds__(256, 2) void dw_bwd_s2_kernel(const T* __restrict__ g, const T* __restrict__ x1,
                                                          uint32_t ybytes, BnBwdOut ob, const T* __restrict__ x,
                                                          uint32_t xbytes, BnIn bn, const float* __restrict__ w_crs,
                                                          T* __restrict__ dx, const T* __restrict__ res,
                                                          double* __restrict__ spart, float* __restrict__ wpart,
                                                          int N, int H, int W, int C, int OH, int OW, FoldTail ft,
                                                          int nt, JoinBwd jn = JoinBwd{}) {
  static_assert(!STATS || BNX, "input-BN partials need the input BN");
  static_assert(!JOIN || (!BNX && sizeof(T) == 4), "the join form: fp32, no input BN");
  constexpr bool PART = STATS || JOIN;
  constexpr int R = 3, S = 3, ST = 2, PAD = 1, RS = 9, TWQ = JOIN ? 1 : 2;  // (the join form's operands need the registers)
  using SP = SubPix<R, ST, PAD>;
  constexpr int D0 = SP::dmin(), ND = SP::dmax() - SP::dmin() + 1, NCOL = TWQ + ND - 1;
  extern __shared__ f32x4 scratch[];  // the final reductions
  const int tid = threadIdx.x;
  const int C4 = C >> 2, IPB = 256 / C4;  // items a block works on at once (C4 divides 256)
  const int cq = tid % C4, il = tid / C4, c = 4 * cq;
  const int QH = (H + 1) / 2, QW = (W + 1) / 2, nqc = (QW + TWQ - 1) / TWQ;
  const int items = N * QH * nqc;
  const __amdgpu_buffer_rsrc_t rg = make_rsrc_v(g, ybytes), r1 = make_rsrc_v(x1, ybytes), rx = make_rsrc_v(x, xbytes);
  const int QHW = (JOIN && jn.res_lat) ? QH * QW : H * W;  // residual pixels per image
  const __amdgpu_buffer_rsrc_t rres = make_rsrc_v(res, res ? (uint32_t)((size_t)N * QHW * C * sizeof(T)) : 0u);
  const __amdgpu_buffer_rsrc_t rdx = make_rsrc_v(dx, dx ? xbytes : 0u);
  const __amdgpu_buffer_rsrc_t rjx = make_rsrc_v(JOIN ? jn.x : nullptr, JOIN ? xbytes : 0u);
  f32x4 jm = {0.f, 0.f, 0.f, 0.f}, ji = jm;
  if constexpr (JOIN) {
    jm = ld4(jn.mean + c);
    ji = ld4(jn.invstd + c);
  }
  // this thread's channel terms: the following BN (dy), the filters W[c][r][s], the input BN
  const f32x4 om = ld4(ob.mean + c), oi = ld4(ob.invstd + c), ok1 = ld4(ob.k12 + c), ok2 = ld4(ob.k12 + C + c);
  const f32x4 of = ld4(ob.gamma + c) * oi;
  f32x4 og = {0.f, 0.f, 0.f, 0.f}, obt = og;
  if constexpr (RELU1) {
    og = ld4(ob.gamma + c);
    obt = ld4(ob.beta + c);
  }
  f32x4 bm = {0.f, 0.f, 0.f, 0.f}, bi = bm, bg = bm, bb = bm;
  if constexpr (BNX) {
    bm = ld4(bn.mean + c);
    bi = ld4(bn.invstd + c);
    bg = ld4(bn.gamma + c);
    bb = ld4(bn.beta + c);
  }
  f32x4 wv[R][S];
  load_dw_weights<R, S, 1>(wv, w_crs, c, C);
  f32x4 wacc[R][S];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int s = 0; s < S; ++s) wacc[r][s] = f32x4{0.f, 0.f, 0.f, 0.f};
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  for (int item = blockIdx.x * IPB + il; item < items; item += gridDim.x * IPB) {
    const int qc = item % nqc;
    const int t = item / nqc;
    const int qi = t % QH, n = t / QH;
    const int j0 = qc * TWQ;
    // the dy window: rows qi + D0 .., columns j0 + D0 .., formed from (g, x1) on load
    f32x4 d[ND][NCOL];
#pragma unroll
    for (int a = 0; a < ND; ++a) {
      const int oh = qi + D0 + a;
#pragma unroll
      for (int b = 0; b < NCOL; ++b) {
        const int ow = j0 + D0 + b;
        const bool ok = (unsigned)oh < (unsigned)OH && (unsigned)ow < (unsigned)OW;
        const uint32_t e = (uint32_t)(((n * OH + oh) * OW + ow) * C + c);
        const f32x4 gv = bload4e<T>(rg, ok, e), xv = bload4e<T>(r1, ok, e);
        f32x4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float ge = gv[k];
          if constexpr (RELU1) {
            if (!(bn_out(xv[k], om[k], oi[k], og[k], obt[k]) > 0.f)) ge = 0.f;
          }
          o[k] = bn_bwd_elem(xv[k], ge, om[k], oi[k], of[k], ok1[k], ok2[k]);
        }
        d[a][b] = ok ? o : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int q = 0; q < TWQ; ++q) {
      const int j = j0 + q;
      f32x4 xb[ST][ST], xr[ST][ST], acc[ST][ST], jxv[ST][ST];
      bool okp[ST][ST];
#pragma unroll
      for (int a = 0; a < ST; ++a)
#pragma unroll
        for (int b = 0; b < ST; ++b) {
          const int h = qi * ST + a, w = j * ST + b;
          okp[a][b] = j < QW && h < H && w < W;
          const uint32_t e = (uint32_t)(((n * H + h) * W + w) * C + c);
          xr[a][b] = bload4e<T>(rx, okp[a][b], e);
          if (JOIN && jn.res_lat)  // compact lattice residual: phase (0, 0) only, at quad (qi, j)
            acc[a][b] = bload4e<T>(rres, okp[a][b] && a == 0 && b == 0, (uint32_t)(((n * QH + qi) * QW + j) * C + c));
          else
            acc[a][b] = (RES && res) ? bload4e<T>(rres, okp[a][b], e) : f32x4{0.f, 0.f, 0.f, 0.f};
          if constexpr (JOIN) jxv[a][b] = bload4e<float>(rjx, okp[a][b], e);
          f32x4 v = xr[a][b];
          if constexpr (BNX) v = bn_in4(v, bm, bi, bg, bb, bn.relu);
          xb[a][b] = okp[a][b] ? v : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      // dgrad in dw_dgrad_subpixel_kernel's tap order (the residual added after, as there)
      f32x4 dg[ST][ST];
#pragma unroll
      for (int a = 0; a < ST; ++a)
#pragma unroll
        for (int b = 0; b < ST; ++b) dg[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const f32x4 dv = d[SP::nb(r) - D0][q + SP::nb(s) - D0];
          dg[SP::phase(r)][SP::phase(s)] += dv * wv[r][s];
          wacc[r][s] += dv * xb[SP::phase(r)][SP::phase(s)];
        }
#pragma unroll
      for (int a = 0; a < ST; ++a)
#pragma unroll
        for (int b = 0; b < ST; ++b) {
          const int h = qi * ST + a, w = j * ST + b;
          const uint32_t e = (uint32_t)(((n * H + h) * W + w) * C + c);
          f32x4 o = (RES && res) ? dg[a][b] + acc[a][b] : dg[a][b];
          o = rnd4<T>(o);  // the partials see dx as stored
          if constexpr (JOIN) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              if (!(xr[a][b][k] > 0.f)) o[k] = 0.f;  // dy * mask (activations.py:46), mask = y > 0
              const float xn = (jxv[a][b][k] - jm[k]) * ji[k];
              const float gk = okp[a][b] ? o[k] : 0.f;
              s1[k] += (double)gk;
              s2[k] += (double)gk * (double)xn;
            }
          }
          bstore4e_nt<T>(rdx, okp[a][b], e, o, nt);
          if constexpr (STATS) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float xv = xr[a][b][k];
              const float xn = (xv - bm[k]) * bi[k];
              const bool kill = !okp[a][b] || (bn.relu && !(bn_out(xv, bm[k], bi[k], bg[k], bb[k]) > 0.f));
              const float gk = kill ? 0.f : o[k];
              s1[k] += (double)gk;
              s2[k] += (double)gk * (double)xn;
            }
          }
        }
    }
  }
  // fixed-order block reductions over the IPB item lanes of each channel quad
  if constexpr (PART) {
    double(*red)[8] = reinterpret_cast<double(*)[8]>(scratch);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      red[tid][k] = s1[k];
      red[tid][4 + k] = s2[k];
    }
    __syncthreads();
    for (int i = tid; i < C * 2; i += 256) {  // i = (which, channel)
      const int which = i / C, ch = i - which * C;
      const int q4 = ch >> 2, k = ch & 3;
      double a = 0.0;
      for (int l = q4; l < 256; l += C4) a += red[l][4 * which + k];
      pub_store(spart + ((size_t)blockIdx.x * 2 + which) * C + ch, a);
    }
    __syncthreads();
  }
  float* wred = reinterpret_cast<float*>(scratch);  // [256][RS][4]
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int s = 0; s < S; ++s) st4(wred + (tid * RS + r * S + s) * 4, wacc[r][s]);
  __syncthreads();
  // wpart[block][c][r][s]
  for (int i = tid; i < C * RS; i += 256) {
    const int ch = i / RS, tap = i - ch * RS;
    const int q4 = ch >> 2, k = ch & 3;
    float a = 0.f;
    for (int l = q4; l < 256; l += C4) a += wred[(l * RS + tap) * 4 + k];
    wpart[(size_t)blockIdx.x * C * RS + i] = a;
  }
  if constexpr (PART) {
    if (ft.part) fold_tail<256>(ft, blockIdx.x, 0, C, 0);
  }
}

// Block geometry of the fused stride-1 backward: CG channel groups of 4 x CL / CPT column lanes
// (CG * CL / CPT = 256 threads), a CL-column strip.  One column per thread: 16 columns x 64
// channels, or 8 x 128 for narrow images; fewer channel groups (wider strips) when C / 4 has no
// such factor.  Two columns per thread (knob kind 21; W >= 12): CG in {16, 32}
// with the strip width (32 or 16 columns) that pads the row least, ties to the wider.  fp32 and bf16
// alike: 512 x 56 x 56 x 64 bf16 328 -> 284 us, 256 x 56 x 56 x 64 fp32 205 -> 182 us (dwb_bench.py).
struct DwbGeom {
  int cpt, cl, cg, nt;
};
static inline DwbGeom dwb_geom(int W, int C, int cpt, int nt = 256) {
  const int C4 = C / 4;
  if (cpt == 2 && W >= 12 && C4 % 16 == 0) {
    const int pad32 = (W + 31) / 32 * 32 - W, pad16 = (W + 15) / 16 * 16 - W;
    if (C4 % 32 == 0 && pad16 < pad32) return DwbGeom{2, 16, 32, 256};
    return DwbGeom{2, 32, 16, 256};
  }
  int cg = W > 8 ? 16 : 32;
  while (cg > 1 && C4 % cg) cg >>= 1;
  return DwbGeom{1, 256 / cg, cg, 256};
}
static inline int dwb_cpt(size_t) { return knob(kKnobDwbCols) == 2 ? 2 : 1; }
static inline int dwb_nt(size_t) { return 256; }
// Image runs of the fused stride-1 backward: one image per block while N * column strips * channel
// tiles blocks fit knob kind 7 (default 768 = three resident blocks per CU: its LDS and
// registers allow three); above that the batch is dealt into runs so the grid is one round (a
// second, partial round of blocks cost small images up to twice the time: 7 x 7 x 512 ran 1024
// one-image blocks).  0 = one image per block always.
static inline int dwb_target_blocks() { return knob(kKnobDwbBlocks); }  // kind 7
static inline int dwb_nranges(int N, int W, int C, const DwbGeom& g) {
  const int per_image = ((W + g.cl - 1) / g.cl) * ((C / 4) / g.cg);
  // the two-column form holds two blocks per CU (its registers; eight one-wave blocks), the
  // one-column form three
  const int t = g.cpt == 2 ? dwb_target_blocks() * 2 / 3 * (256 / g.nt) : dwb_target_blocks();
  if (t <= 0 || (long long)N * per_image <= t) return N;
  const int r = t / per_image;
  return r < 1 ? 1 : (r > N ? N : r);
}
static inline int dwb_strips(int N, int W, int C, const DwbGeom& g) {
  return dwb_nranges(N, W, C, g) * ((W + g.cl - 1) / g.cl);
}

static int dw_wgrad_blocks(int N, int OH, int OW, int C) {
  const int C4 = C / 4;
  const int cgt = C4 < 256 ? C4 : 256;
  const int PL = 256 / cgt;
  int nblk = (int)cdivll((long long)N * OH * OW, (long long)PL * 16);  // ~16 outputs per thread
  if (nblk > 1024) nblk = 1024;
  if (nblk < 1) nblk = 1;
  return nblk;
}

static inline bool fits(size_t bytes) { return bytes < ((size_t)1 << 31); }
static inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
static inline bool bn_ok(const BnIn& bn) {
  return !bn.mean || (bn.invstd && bn.gamma && bn.beta && aligned16(bn.mean) && aligned16(bn.invstd) &&
                      aligned16(bn.gamma) && aligned16(bn.beta));
}

template <int ST>
static long long dw_fwd_threads(int N, int OH, int OW, int C, bool whole) {
  constexpr int TW = DwTile<ST>::TW;
  const int SEG = dw_fwd_seg(OH, whole);
  return (long long)N * ((OH + SEG - 1) / SEG) * ((OW + TW - 1) / TW) * (C / 4);
}

// part: per-block sums (mode 1: output statistics; mode 2 with xo/obn: BN-backward sums).
// wl: weight layout (load_dw_weights).  Only the combinations the entry points use exist.
template <int R, int S, int ST, class T>
static int launch_dw_fwd(const T* x, const float* wt, const float* bias, T* y, int N, int H, int W, int C, int OH,
                         int OW, int pad, const BnIn& bn, double* part, const T* xo, const BnIn& obn, int wl,
                         const T* res, hipStream_t st, const JoinFwd* jn = nullptr) {
  const uint32_t xb = (uint32_t)((size_t)N * H * W * C * sizeof(T));
  constexpr bool whole = sizeof(T) == 2;
  const dim3 grid((unsigned)cdivll(dw_fwd_threads<ST>(N, OH, OW, C, whole), 256));
  FoldTail ft;  // an armed in-launch fold of the partial rows (fold_tail.h)
  if (!part || !fold_take(part, (int)grid.x, C, 1, &ft)) ft.part = nullptr;
  const JoinFwd jf = jn ? *jn : JoinFwd{};
  if constexpr (R == 3 && S == 3 && sizeof(T) == 4) {
    if (jn) {
      // the residual join formed on load (JOIN): reference-layout filters, no input BN
      if (wl != 1 || bn.mean || xo || pad != 1) return DK_ERR_ARGS;
      if (part)
        hipLaunchKernelGGL((dw_fwd_kernel<R, S, ST, false, false, 1, 1, T, true>), grid, dim3(256), 0, st, x, xb, wt,
                           bias, y, N, H, W, C, OH, OW, pad, bn, part, xo, obn, res, ft, nt_stores(kNtDwFwd),
                           dw_fwd_seg(OH, whole), jf);
      else
        hipLaunchKernelGGL((dw_fwd_kernel<R, S, ST, false, false, 0, 1, T, true>), grid, dim3(256), 0, st, x, xb, wt,
                           bias, y, N, H, W, C, OH, OW, pad, bn, part, xo, obn, res, ft, nt_stores(kNtDwFwd),
                           dw_fwd_seg(OH, whole), jf);
      return fold_status(launch_status(), ft);
    }
  }
  if (jn) return DK_ERR_ARGS;
#define DW_LAUNCH1(B, RL, ST_, WL_)                                                                                  \
  hipLaunchKernelGGL((dw_fwd_kernel<R, S, ST, B, RL, ST_, WL_, T>), grid, dim3(256), 0, st, x, xb, wt, bias, y, N, H, \
                     W, C, OH, OW, pad, bn, part, xo, obn, res, ft, nt_stores(kNtDwFwd), dw_fwd_seg(OH, whole), jf)
#define DW_LAUNCH(B, ST_, WL_)            \
  do {                                    \
    if (B && bn.relu)                     \
      DW_LAUNCH1(B, B, ST_, WL_);         \
    else                                  \
      DW_LAUNCH1(B, false, ST_, WL_);     \
  } while (0)
  const int mode = part ? (xo ? 2 : 1) : 0;
  if (wl == 0 && !bn.mean && mode == 0)
    DW_LAUNCH(false, 0, 0);
  else if (wl == 0 && bn.mean && mode == 0)
    DW_LAUNCH(true, 0, 0);
  else if (wl == 1 && bn.mean && mode == 1)
    DW_LAUNCH(true, 1, 1);
  else if (wl == 1 && bn.mean && mode == 0)
    DW_LAUNCH(true, 0, 1);
  else if (wl == 1 && !bn.mean && mode == 1)
    DW_LAUNCH(false, 1, 1);
  else if (wl == 1 && !bn.mean && mode == 0)
    DW_LAUNCH(false, 0, 1);
  else if (wl == 2 && !bn.mean && mode == 0)
    DW_LAUNCH(false, 0, 2);
  else if (wl == 2 && !bn.mean && mode == 2)
    DW_LAUNCH(false, 2, 2);
  else
    return DK_ERR_ARGS;
#undef DW_LAUNCH
#undef DW_LAUNCH1
  return fold_status(launch_status(), ft);
}

template <class T>
static int dw_fwd_dispatch(const T* x, const float* wt, const float* bias, T* y, int N, int H, int W, int C, int R,
                           int S, int stride, int OH, int OW, int pad, const BnIn& bn, hipStream_t st,
                           double* part = nullptr, const T* xo = nullptr, const BnIn& obn = BnIn{}, int wl = 0,
                           const T* res = nullptr, const JoinFwd* jn = nullptr) {
  if (res && (!aligned16(res) || wl != 2)) return DK_ERR_ARGS;  // residual addend: dgrad only
  if (C % 4 || !aligned16(x) || !aligned16(wt) || !fits((size_t)N * H * W * C * 4) || !bn_ok(bn)) return DK_ERR_ARGS;
  if (part && (C / 4 > 256 || 256 % (C / 4))) return DK_ERR_ARGS;
  if (xo && (bn.mean || !obn.mean || !aligned16(xo) || !bn_ok(obn))) return DK_ERR_ARGS;
#define DW_CASE(RR, SS, STR)                                                                     \
  if (R == RR && S == SS && stride == STR)                                                           \
    return launch_dw_fwd<RR, SS, STR, T>(x, wt, bias, y, N, H, W, C, OH, OW, pad, bn, part, xo, obn, wl, res, st, jn);
  DW_CASE(3, 3, 1)
  DW_CASE(3, 3, 2)
  DW_CASE(5, 5, 1)
  DW_CASE(5, 5, 2)
  DW_CASE(1, 1, 1)
  DW_CASE(1, 1, 2)
#undef DW_CASE
  return DK_ERR_ARGS;
}

template <class T>
static int dw_wgrad(const T* dy, const T* x, int N, int H, int W, int C, int R, int S, int stride, int pad, int OH,
                    int OW, const float* w_crs, float l2, float* dw_crs, void* ws, size_t ws_bytes, const BnIn& bn,
                    hipStream_t st);

}  // namespace dk

using namespace dk;

DK_API int dk_dw_weight_rsc_f32(const float* w_crs, int C, int R, int S, float* w_rsc, void* stream) {
  const int total = C * R * S;
  hipLaunchKernelGGL(dw_weight_rsc_kernel, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), w_crs, C, R, S, 0,
                     w_rsc);
  return launch_status();
}

DK_API int dk_dwconv_fwd_f32(const float* x, int N, int H, int W, int C, const float* w_rsc, int R, int S, int stride,
                             int pad, const float* bias, float* y, int OH, int OW, void* stream) {
  return dw_fwd_dispatch(x, w_rsc, bias, y, N, H, W, C, R, S, stride, OH, OW, pad, BnIn{}, as_stream(stream));
}

DK_API int dk_dwconv_fwd_bnx_f32(const float* x, int N, int H, int W, int C, const float* w_rsc, int R, int S,
                                 int stride, int pad, const float* bias, float* y, int OH, int OW,
                                 const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                 const float* bn_beta, int bn_relu, void* stream) {
  if (!bn_mean) return DK_ERR_ARGS;
  return dw_fwd_dispatch(x, w_rsc, bias, y, N, H, W, C, R, S, stride, OH, OW, pad,
                         BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu}, as_stream(stream));
}

// Rows of BatchNorm partial statistics dk_dwconv_fwd_ex_f32 writes; 0 = statistics not
// supported for this channel count (C/4 must divide 256).
static int dw_fwd_stats_rows(int N, int OH, int OW, int C, int stride, bool whole) {
  if (C % 4 || C / 4 > 256 || 256 % (C / 4)) return 0;
  const long long thr =
      stride == 1 ? dw_fwd_threads<1>(N, OH, OW, C, whole) : dw_fwd_threads<2>(N, OH, OW, C, whole);
  return (int)cdivll(thr, 256);
}
DK_API int dk_dwconv_fwd_stats_rows(int N, int OH, int OW, int C, int stride) {
  return dw_fwd_stats_rows(N, OH, OW, C, stride, false);
}
// The bf16 forward's rows (dk_dwconv_fwd_ex_bf16: whole output columns per thread, fewer blocks).
DK_API int dk_dwconv_fwd_bf16_stats_rows(int N, int OH, int OW, int C, int stride) {
  return dw_fwd_stats_rows(N, OH, OW, C, stride, true);
}

// Reads the filters in the reference layout W[C][R][S] (no re-layout copy).
DK_API int dk_dwconv_fwd_ex_f32(const float* x, int N, int H, int W, int C, const float* w_crs, int R, int S,
                                int stride, int pad, const float* bias, float* y, int OH, int OW,
                                const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                const float* bn_beta, int bn_relu, double* stats, void* stream) {
  if (stride != 1 && stride != 2) return DK_ERR_ARGS;
  return dw_fwd_dispatch<float>(x, w_crs, bias, y, N, H, W, C, R, S, stride, OH, OW, pad,
                         BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu}, as_stream(stream), stats, nullptr,
                         BnIn{}, 1);
}

// The layer's input is the residual join y = ReLU(bnA(a) + bnB(b)) (dk_bn_add_f32's operands), formed
// as the window is loaded and stored once into y_join (+ its ReLU mask, nullable); the rest as
// dk_dwconv_fwd_ex_f32 without an input BatchNorm.  3 x 3 filters, pad 1, stride 1 or 2.
DK_API int dk_dwconv_fwd_join_f32(const float* a, const float* a_mean, const float* a_invstd, const float* a_gamma,
                                  const float* a_beta, int a_relu, const float* b, const float* b_mean,
                                  const float* b_invstd, const float* b_gamma, const float* b_beta, int b_relu,
                                  float* y_join, uint8_t* mask, int N, int H, int W, int C, const float* w_crs,
                                  int stride, const float* bias, float* y, int OH, int OW, double* stats,
                                  void* stream) {
  if (stride != 1 && stride != 2) return DK_ERR_ARGS;
  const JoinFwd jf{b, BnIn{a_mean, a_invstd, a_gamma, a_beta, a_relu}, BnIn{b_mean, b_invstd, b_gamma, b_beta, b_relu},
                   y_join, mask};
  if (!b || !y_join || !aligned16(b) || !aligned16(y_join) || !bn_ok(jf.ba) || !bn_ok(jf.bb) || C > 512) return DK_ERR_ARGS;
  if (mask && (reinterpret_cast<uintptr_t>(mask) & 3)) return DK_ERR_ARGS;
  return dw_fwd_dispatch<float>(a, w_crs, bias, y, N, H, W, C, 3, 3, stride, OH, OW, 1, BnIn{}, as_stream(stream),
                                stats, nullptr, BnIn{}, 1, nullptr, &jf);
}

// w_rsc is the (unflipped) [R][S][C] copy; stride-1 dgrad flips it internally into ws.
DK_API size_t dk_dwconv_dgrad_workspace_bytes(int C, int R, int S) { return (size_t)C * R * S * sizeof(float); }

// Input gradient.  res (optional): added to dx (the residual join's other gradient term);
// bn_x/obn/part (optional, stride 1 only): + stage 1 of the backward of the BatchNorm whose
// output the layer consumed.
template <class T>
static int dw_dgrad(const T* dy, int N, int OH, int OW, int C, const float* w_crs, int R, int S, int stride, int pad,
                    T* dx, int H, int W, void* ws, size_t ws_bytes, const T* res, const T* bn_x, const BnIn& obn,
                    double* part, hipStream_t st, const JoinBwd* jn = nullptr) {
  if (C % 4) return DK_ERR_ARGS;
  if (ws_bytes < dk_dwconv_dgrad_workspace_bytes(C, R, S)) return DK_ERR_WORKSPACE;
  float* wt = static_cast<float*>(ws);
  if (stride == 1 && pad <= R - 1 && pad <= S - 1 && R == S) {
    // dx = correlation of dy with the flipped filter (read flipped from W[C][R][S]), padding R-1-pad
    if (part && dk_dwconv_fwd_stats_rows(N, H, W, C, 1) == 0) return DK_ERR_ARGS;
    return dw_fwd_dispatch(dy, w_crs, nullptr, dx, N, OH, OW, C, R, S, 1, H, W, R - 1 - pad, BnIn{}, st,
                           part ? part : nullptr, part ? bn_x : nullptr, part ? obn : BnIn{}, 2, res);
  }
  JoinBwd bnj{};
  if (part && !jn) {
    // the input BatchNorm's stage-1 partials on the sub-pixel store (JoinBwd::bnmode)
    if (!bn_x || !obn.mean || !obn.invstd || !obn.gamma || !obn.beta || (C / 4) > 256 || 256 % (C / 4))
      return DK_ERR_ARGS;
    bnj = JoinBwd{nullptr, bn_x, obn.mean, obn.invstd, 0, obn.gamma, obn.beta, obn.relu, 1};
    jn = &bnj;
  }
  if (!fits((size_t)N * OH * OW * C * 4) || !aligned16(dy) || !aligned16(dx) || !aligned16(w_crs) ||
      (res && !aligned16(res)))
    return DK_ERR_ARGS;
  const uint32_t gb = (uint32_t)((size_t)N * OH * OW * C * sizeof(T));
#define DW_SUBPIX(RR, SS, STR, PD)                                                                                   \
  if (R == RR && S == SS && stride == STR && pad == PD) {                                                            \
    const long long items = (long long)N * cdiv(H, STR) * cdiv(cdiv(W, STR), 4) * (C / 4);                         \
    const dim3 grid((unsigned)cdivll(items, 256));                                                                   \
    if (jn) {                                                                                                        \
      if (sizeof(T) != sizeof(float) && !jn->bnmode) return DK_ERR_ARGS; /* the join fusion: fp32 only */            \
      FoldTail ft;                                                                                                   \
      if (!fold_take(part, (int)grid.x, C, 1, &ft)) ft.part = nullptr;                                              \
      hipLaunchKernelGGL((dw_dgrad_subpixel_kernel<RR, SS, STR, PD, T, true>), grid, dim3(256), 0, st, dy, gb,      \
                         w_crs, dx, N, H, W, C, OH, OW, res, *jn, part, ft, nt_stores(dgrad_nt_fam<T>()));                  \
      return fold_status(launch_status(), ft);                                                                       \
    }                                                                                                                \
    hipLaunchKernelGGL((dw_dgrad_subpixel_kernel<RR, SS, STR, PD, T>), grid, dim3(256), 0, st, dy, gb, w_crs, dx, N, \
                       H, W, C, OH, OW, res, JoinBwd{}, nullptr, FoldTail{}, nt_stores(dgrad_nt_fam<T>()));                 \
    return launch_status();                                                                                          \
  }
  DW_SUBPIX(3, 3, 2, 1)
  DW_SUBPIX(5, 5, 2, 2)
  DW_SUBPIX(1, 1, 2, 0)
#undef DW_SUBPIX
  if (res || jn) return DK_ERR_ARGS;  // generic gather path: no residual / join fusion
  if constexpr (sizeof(T) != sizeof(float)) {
    return DK_ERR_ARGS;  // generic gather path: fp32 storage only
  } else {
  hipLaunchKernelGGL(dw_weight_rsc_kernel, dim3(cdiv(C * R * S, 256)), dim3(256), 0, st, w_crs, C, R, S, 0, wt);
  int rc = launch_status();
  if (rc) return rc;
  const long long total = (long long)N * H * W * (C / 4);
  const dim3 grid((unsigned)cdivll(total, 256));
  if (R == 3 && S == 3)
    hipLaunchKernelGGL((dw_dgrad_gather_kernel<3, 3>), grid, dim3(256), 0, st, dy, wt, dx, N, H, W, C, OH, OW, stride,
                       pad);
  else if (R == 5 && S == 5)
    hipLaunchKernelGGL((dw_dgrad_gather_kernel<5, 5>), grid, dim3(256), 0, st, dy, wt, dx, N, H, W, C, OH, OW, stride,
                       pad);
  else if (R == 1 && S == 1)
    hipLaunchKernelGGL((dw_dgrad_gather_kernel<1, 1>), grid, dim3(256), 0, st, dy, wt, dx, N, H, W, C, OH, OW, stride,
                       pad);
  else
    return DK_ERR_ARGS;
  return launch_status();
  }
}

DK_API int dk_dwconv_dgrad_f32(const float* dy, int N, int OH, int OW, int C, const float* w_crs, int R, int S,
                               int stride, int pad, float* dx, int H, int W, void* ws, size_t ws_bytes,
                               void* stream) {
  return dw_dgrad<float>(dy, N, OH, OW, C, w_crs, R, S, stride, pad, dx, H, W, ws, ws_bytes, nullptr, nullptr, BnIn{},
                  nullptr, as_stream(stream));
}

DK_API int dk_dwconv_dgrad_stats_rows(int N, int H, int W, int C, int stride) {
  if (stride != 1) return 0;
  return dk_dwconv_fwd_stats_rows(N, H, W, C, 1);
}

DK_API int dk_dwconv_dgrad_ex_f32(const float* dy, int N, int OH, int OW, int C, const float* w_crs, int R, int S,
                                  int stride, int pad, float* dx, int H, int W, void* ws, size_t ws_bytes,
                                  const float* residual, const float* bn_x, const float* bn_mean,
                                  const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu,
                                  double* part, void* stream) {
  if ((part != nullptr) != (bn_x != nullptr)) return DK_ERR_ARGS;
  return dw_dgrad(dy, N, OH, OW, C, w_crs, R, S, stride, pad, dx, H, W, ws, ws_bytes, residual, bn_x,
                  BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu}, part, as_stream(stream));
}

DK_API size_t dk_dwconv_wgrad_workspace_bytes(int N, int OH, int OW, int C, int R, int S) {
  return (size_t)dw_wgrad_blocks(N, OH, OW, C) * C * R * S * sizeof(float);
}

namespace dk {
template <class T>
static int dw_wgrad(const T* dy, const T* x, int N, int H, int W, int C, int R, int S, int stride, int pad, int OH,
                    int OW, const float* w_crs, float l2, float* dw_crs, void* ws, size_t ws_bytes,
                    const BnIn& bn, hipStream_t st) {
  if (C % 4 || !aligned16(x) || !aligned16(dy) || !bn_ok(bn)) return DK_ERR_ARGS;
  if (!fits((size_t)N * H * W * C * 4) || !fits((size_t)N * OH * OW * C * 4)) return DK_ERR_ARGS;
  if (ws_bytes < dk_dwconv_wgrad_workspace_bytes(N, OH, OW, C, R, S)) return DK_ERR_WORKSPACE;
  const int nblk = dw_wgrad_blocks(N, OH, OW, C);
  const int C4 = C / 4;
  const int cgt = C4 < 256 ? C4 : 256;
  const dim3 grid(nblk, cdiv(C4, cgt));
  float* part = static_cast<float*>(ws);
  const size_t shm = (size_t)256 * R * S * 4 * sizeof(float);
  const uint32_t xb = (uint32_t)((size_t)N * H * W * C * sizeof(T)), gb = (uint32_t)((size_t)N * OH * OW * C * sizeof(T));
#define DW_WG_LAUNCH(RR, SS, STR, B)                                                                                 \
  {                                                                                                                  \
    const int items = N * cdiv(OH, kWgSeg) * ((OW + DwWgTile<STR>::TW - 1) / DwWgTile<STR>::TW);                     \
    const int ipb = cdiv(items, nblk);                                                                               \
    if (shm > 65536)                                                                                                 \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&dw_wgrad_partial_kernel<RR, SS, STR, B, T>),          \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);                               \
    hipLaunchKernelGGL((dw_wgrad_partial_kernel<RR, SS, STR, B, T>), grid, dim3(256), shm, st, dy, gb, x, xb, part, N, \
                       H, W, C, OH, OW, pad, ipb, bn);                                                               \
  }
#define DW_WG(RR, SS, STR)                 \
  if (R == RR && S == SS && stride == STR) { \
    if (bn.mean)                           \
      DW_WG_LAUNCH(RR, SS, STR, true)      \
    else                                   \
      DW_WG_LAUNCH(RR, SS, STR, false)     \
  } else
  DW_WG(3, 3, 1)
  DW_WG(3, 3, 2)
  DW_WG(5, 5, 1)
  DW_WG(5, 5, 2)
  DW_WG(1, 1, 1)
  DW_WG(1, 1, 2) { return DK_ERR_ARGS; }
#undef DW_WG
#undef DW_WG_LAUNCH
  int rc = launch_status();
  if (rc) return rc;
  return splitk_reduce(part, nblk, 1, C * R * S, dw_crs, w_crs, l2, 0, C, C, 1, 1, st);
}
}  // namespace dk

// dw[c][r][s] = sum_{n,oh,ow} dy[n,oh,ow,c] * x[n, oh*st + r - pad, ow*st + s - pad, c] (+ l2 * w)
DK_API int dk_dwconv_wgrad_f32(const float* dy, const float* x, int N, int H, int W, int C, int R, int S, int stride,
                               int pad, int OH, int OW, const float* w_crs, float l2, float* dw_crs, void* ws,
                               size_t ws_bytes, void* stream) {
  return dw_wgrad(dy, x, N, H, W, C, R, S, stride, pad, OH, OW, w_crs, l2, dw_crs, ws, ws_bytes, BnIn{},
                  as_stream(stream));
}

// Fused stride-1 backward (dw_bwd_fused_kernel).  Workspace: the weight-gradient partials.
DK_API int dk_dwconv_bwd_bnbwd_stats_rows(int N, int H, int W, int C) {
  (void)H;
  return (C < 4 || C % 4) ? 0 : dwb_strips(N, W, C, dwb_geom(W, C, dwb_cpt(4)));
}
// (the join entry dk_dwconv_bwd_bnbwd_join_f32 has the fp32 geometry: these rows)

DK_API size_t dk_dwconv_bwd_bnbwd_workspace_bytes(int N, int H, int W, int C, int R, int S) {
  return (size_t)dk_dwconv_bwd_bnbwd_stats_rows(N, H, W, C) * C * R * S * sizeof(float);
}

// bf16 storage: its block geometry may differ (two columns per thread, dwb_geom)
DK_API int dk_dwconv_bwd_bnbwd_bf16_stats_rows(int N, int H, int W, int C) {
  (void)H;
  return (C < 4 || C % 4) ? 0 : dwb_strips(N, W, C, dwb_geom(W, C, dwb_cpt(2), dwb_nt(2)));
}

DK_API size_t dk_dwconv_bwd_bnbwd_bf16_workspace_bytes(int N, int H, int W, int C, int R, int S) {
  return (size_t)dk_dwconv_bwd_bnbwd_bf16_stats_rows(N, H, W, C) * C * R * S * sizeof(float);
}

namespace dk {
template <class T>
static int dw_bwd_fused(const T* g, const T* bn_x, int N, int H, int W, int C, const float* out_mean,
                        const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu,
                        const float* k12, const T* x, const float* w_crs, int R, int S, int pad, float l2,
                        float* dw_crs, T* dx, const T* residual, const float* bn_mean, const float* bn_invstd,
                        const float* bn_gamma, const float* bn_beta, int bn_relu, double* part, void* ws,
                        size_t ws_bytes, void* stream) {
  const hipStream_t st = as_stream(stream);
  if (R != 3 || S != 3 || pad != 1 || C % 4 || N < 1 || H < 1 || W < 1) return DK_ERR_ARGS;
  const DwbGeom geo = dwb_geom(W, C, dwb_cpt(sizeof(T)), dwb_nt(sizeof(T)));
  const int cl = geo.cl;
  if (!g || !bn_x || !x || !w_crs || !dw_crs || !out_mean || !out_invstd || !out_gamma || !out_beta || !k12)
    return DK_ERR_ARGS;
  const BnIn bn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
  if (part && !bn_mean) return DK_ERR_ARGS;  // the input BN's partials need the input BN
  if (!aligned16(g) || !aligned16(bn_x) || !aligned16(x) || (dx && !aligned16(dx)) ||
      (residual && !aligned16(residual)) || !bn_ok(bn) || !aligned16(out_mean) || !aligned16(out_invstd) ||
      !aligned16(out_gamma) || !aligned16(out_beta) || !aligned16(k12) || !aligned16(w_crs))
    return DK_ERR_ARGS;
  const size_t bytes = (size_t)N * H * W * C * sizeof(T);
  if (!fits(bytes)) return DK_ERR_ARGS;
  const size_t need = sizeof(T) == 2 ? dk_dwconv_bwd_bnbwd_bf16_workspace_bytes(N, H, W, C, R, S)
                                      : dk_dwconv_bwd_bnbwd_workspace_bytes(N, H, W, C, R, S);
  if (ws_bytes < need) return DK_ERR_WORKSPACE;
  const int strips = dwb_strips(N, W, C, geo);
  const int nranges = dwb_nranges(N, W, C, geo);
  const int ncht = (C / 4) / geo.cg;
  float* wpart = static_cast<float*>(ws);
  const BnBwdOut ob{out_mean, out_invstd, out_gamma, out_beta, k12, out_relu};
  const dim3 grid((unsigned)(strips * ncht));
  FoldTail ft;  // an armed in-launch fold of the input BN's partial rows (fold_tail.h)
  if (!part || !fold_take(part, strips, C, ncht, &ft)) ft.part = nullptr;
  size_t shm = (size_t)geo.nt * 9 * 4 * sizeof(float);  // the weight-gradient reduction
  const size_t ring = (size_t)2 * (cl + 2) * geo.cg * sizeof(f32x4);
  if (ring > shm) shm = ring;
  // two columns per thread (knob 21)
  constexpr int CPT2 = 2;
#define DWB_LAUNCH(BNX_, STATS_, RELU1_)                                                                             \
  {                                                                                                                  \
    auto k = geo.cpt == 2 ? (residual ? dw_bwd_fused_kernel<BNX_, STATS_, RELU1_, false, T, CPT2>                 \
                                      : dw_bwd_fused_kernel<BNX_, STATS_, RELU1_, false, T, CPT2, 256, false>)    \
                          : (residual ? dw_bwd_fused_kernel<BNX_, STATS_, RELU1_, false, T>                       \
                                      : dw_bwd_fused_kernel<BNX_, STATS_, RELU1_, false, T, 1, 256, false>);      \
    if (shm > 65536)                                                                                                 \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,       \
                                (int)shm);                                                                           \
    hipLaunchKernelGGL(k, grid, dim3(geo.nt), shm, st, g, bn_x, (uint32_t)bytes, ob, x, bn, w_crs, dx, residual, part,  \
                       wpart, N, H, W, C, cl, ft, JoinBwd{}, nt_stores(kNtDwBwd), nranges);                                                        \
  }
  if (out_relu) {
    if (part) DWB_LAUNCH(true, true, true) else if (bn_mean) DWB_LAUNCH(true, false, true)
    else DWB_LAUNCH(false, false, true)
  } else {
    if (part) DWB_LAUNCH(true, true, false) else if (bn_mean) DWB_LAUNCH(true, false, false)
    else DWB_LAUNCH(false, false, false)
  }
#undef DWB_LAUNCH
  int rc = launch_status();
  if (rc) return rc;
  return fold_status(wgrad_reduce(wpart, strips, 1, C * R * S, dw_crs, l2 != 0.f ? w_crs : nullptr, l2, st), ft);
}
}  // namespace dk

DK_API int dk_dwconv_bwd_bnbwd_f32(const float* g, const float* bn_x, int N, int H, int W, int C,
                                   const float* out_mean, const float* out_invstd, const float* out_gamma,
                                   const float* out_beta, int out_relu, const float* k12, const float* x,
                                   const float* w_crs, int R, int S, int pad, float l2, float* dw_crs, float* dx,
                                   const float* residual, const float* bn_mean, const float* bn_invstd,
                                   const float* bn_gamma, const float* bn_beta, int bn_relu, double* part,
                                   void* ws, size_t ws_bytes, void* stream) {
  return dw_bwd_fused(g, bn_x, N, H, W, C, out_mean, out_invstd, out_gamma, out_beta, out_relu, k12, x, w_crs, R, S,
                      pad, l2, dw_crs, dx, residual, bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu, part, ws,
                      ws_bytes, stream);
}

// bf16 storage twin (BASELINE config 5): g, bn_x, x, dx, residual bf16; dy formed in fp32.
DK_API int dk_dwconv_bwd_bnbwd_bf16(const bf16_t* g, const bf16_t* bn_x, int N, int H, int W, int C,
                                    const float* out_mean, const float* out_invstd, const float* out_gamma,
                                    const float* out_beta, int out_relu, const float* k12, const bf16_t* x,
                                    const float* w_crs, int R, int S, int pad, float l2, float* dw_crs, bf16_t* dx,
                                    const bf16_t* residual, const float* bn_mean, const float* bn_invstd,
                                    const float* bn_gamma, const float* bn_beta, int bn_relu, double* part,
                                    void* ws, size_t ws_bytes, void* stream) {
  return dw_bwd_fused(g, bn_x, N, H, W, C, out_mean, out_invstd, out_gamma, out_beta, out_relu, k12, x, w_crs, R, S,
                      pad, l2, dw_crs, dx, residual, bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu, part, ws,
                      ws_bytes, stream);
}

// Rows of join partials dk_dwconv_dgrad_join_f32 writes (0: the geometry has no join variant).
DK_API int dk_dwconv_dgrad_join_rows(int N, int H, int W, int C, int R, int S, int stride, int pad) {
  if (C % 4 || C / 4 > 256 || 256 % (C / 4)) return 0;
  const bool ok = (R == 3 && S == 3 && stride == 2 && pad == 1) || (R == 5 && S == 5 && stride == 2 && pad == 2) ||
                  (R == 1 && S == 1 && stride == 2 && pad == 0);
  if (!ok) return 0;
  const long long items = (long long)N * cdiv(H, stride) * cdiv(cdiv(W, stride), 4) * (C / 4);
  return (int)cdivll(items, 256);
}

// Strided (sub-pixel) input gradient whose input is a residual join's output: dx = (dgrad +
// residual) * join_mask and part (dk_dwconv_dgrad_join_rows x 2 x C) = stage 1 of the join
// BatchNorm's backward over that dx (see dk_dwconv_bwd_bnbwd_join_f32).  Takes an in-launch fold
// arming (dk_bn_fold_arm_bwd).
DK_API int dk_dwconv_dgrad_join_f32(const float* dy, int N, int OH, int OW, int C, const float* w_crs, int R, int S,
                                    int stride, int pad, float* dx, int H, int W, void* ws, size_t ws_bytes,
                                    const float* residual, int residual_lattice, const uint8_t* join_mask,
                                    const float* join_x, const float* join_mean, const float* join_invstd,
                                    double* part, void* stream) {
  if (residual_lattice != 0 && residual_lattice != stride) return DK_ERR_ARGS;
  if (!join_mask || !join_x || !join_mean || !join_invstd || !part ||
      dk_dwconv_dgrad_join_rows(N, H, W, C, R, S, stride, pad) == 0)
    return DK_ERR_ARGS;
  if (!aligned16(join_x) || !aligned16(join_mean) || !aligned16(join_invstd) ||
      (reinterpret_cast<uintptr_t>(join_mask) & 3))
    return DK_ERR_ARGS;
  const JoinBwd jn{join_mask, join_x, join_mean, join_invstd, residual_lattice ? 1 : 0};
  return dw_dgrad<float>(dy, N, OH, OW, C, w_crs, R, S, stride, pad, dx, H, W, ws, ws_bytes, residual, nullptr,
                         BnIn{}, part, as_stream(stream), &jn);
}

// ---- fused stride-2 depthwise backward (dw_bwd_s2_kernel) ----
namespace dk {
static int dws2_blocks(int N, int H, int W, int C) {
  const int C4 = C / 4, IPB = 256 / C4;
  const long long items = (long long)N * ((H + 1) / 2) * ((((W + 1) / 2) + 1) / 2);
  long long b = (items + IPB - 1) / IPB;
  const int target = knob(kKnobDwbBlocks) * 2 / 3;  // two resident blocks per CU
  if (target > 0 && b > target) b = target;
  return b < 1 ? 1 : (int)b;
}
static bool dws2_ok(int N, int H, int W, int C, int OH, int OW) {
  return N >= 1 && H >= 1 && W >= 1 && C >= 4 && C % 4 == 0 && 256 % (C / 4) == 0 && OH == (H + 1) / 2 &&
         OW == (W + 1) / 2;
}
}  // namespace dk

DK_API int dk_dwconv_bwd_s2_stats_rows(int N, int H, int W, int C) {
  return dk::dws2_ok(N, H, W, C, (H + 1) / 2, (W + 1) / 2) ? dk::dws2_blocks(N, H, W, C) : 0;
}

DK_API size_t dk_dwconv_bwd_s2_workspace_bytes(int N, int H, int W, int C) {
  return (size_t)dk_dwconv_bwd_s2_stats_rows(N, H, W, C) * C * 9 * sizeof(float);
}

namespace dk {
template <class T>
static int dw_bwd_s2(const T* g, const T* bn_x, int N, int H, int W, int C, int OH, int OW, const float* out_mean,
                     const float* out_invstd, const float* out_gamma, const float* out_beta, int out_relu,
                     const float* k12, const T* x, const float* w_crs, float l2, float* dw_crs, T* dx,
                     const T* residual, const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                     const float* bn_beta, int bn_relu, double* part, void* ws, size_t ws_bytes, void* stream) {
  const hipStream_t st = as_stream(stream);
  if (!dws2_ok(N, H, W, C, OH, OW)) return DK_ERR_ARGS;
  if (!g || !bn_x || !x || !w_crs || !dw_crs || !out_mean || !out_invstd || !out_gamma || !out_beta || !k12)
    return DK_ERR_ARGS;
  const BnIn bn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu};
  if (part && !bn_mean) return DK_ERR_ARGS;
  if (!aligned16(out_mean) || !aligned16(out_invstd) || !aligned16(out_gamma) || !aligned16(out_beta) ||
      !aligned16(k12) || !bn_ok(bn) ||
      ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(bn_x) | reinterpret_cast<uintptr_t>(x) |
        reinterpret_cast<uintptr_t>(dx) | reinterpret_cast<uintptr_t>(residual)) & (4 * sizeof(T) - 1)))
    return DK_ERR_ARGS;  // (dx and the residual take 4-channel vector stores / loads too; null passes)
  const size_t xb = (size_t)N * H * W * C * sizeof(T), yb = (size_t)N * OH * OW * C * sizeof(T);
  if (!fits(xb)) return DK_ERR_ARGS;
  if (ws_bytes < dk_dwconv_bwd_s2_workspace_bytes(N, H, W, C)) return DK_ERR_WORKSPACE;
  const int blocks = dws2_blocks(N, H, W, C);
  float* wpart = static_cast<float*>(ws);
  const BnBwdOut ob{out_mean, out_invstd, out_gamma, out_beta, k12, out_relu};
  FoldTail ft;
  if (!part || !fold_take(part, blocks, C, 1, &ft)) ft.part = nullptr;
  const size_t shm = (size_t)256 * 9 * 4 * sizeof(float);
#define DWS2_LAUNCH(BNX_, STATS_, RELU1_)                                                                           \
  do {                                                                                                              \
    if (residual)                                                                                                   \
      hipLaunchKernelGGL((dw_bwd_s2_kernel<BNX_, STATS_, RELU1_, T>), dim3(blocks), dim3(256), shm, st, g, bn_x,   \
                         (uint32_t)yb, ob, x, (uint32_t)xb, bn, w_crs, dx, residual, part, wpart, N, H, W, C, OH, OW, \
                         ft, nt_stores(dgrad_nt_fam<T>()));                                                                \
    else                                                                                                            \
      hipLaunchKernelGGL((dw_bwd_s2_kernel<BNX_, STATS_, RELU1_, T, false, false>), dim3(blocks), dim3(256), shm,  \
                         st, g, bn_x, (uint32_t)yb, ob, x, (uint32_t)xb, bn, w_crs, dx, residual, part, wpart, N, H, \
                         W, C, OH, OW, ft, nt_stores(dgrad_nt_fam<T>()));                                                  \
  } while (0)
  if (out_relu) {
    if (part) DWS2_LAUNCH(true, true, true); else if (bn_mean) DWS2_LAUNCH(true, false, true);
    else DWS2_LAUNCH(false, false, true);
  } else {
    if (part) DWS2_LAUNCH(true, true, false); else if (bn_mean) DWS2_LAUNCH(true, false, false);
    else DWS2_LAUNCH(false, false, false);
  }
#undef DWS2_LAUNCH
  int rc = launch_status();
  if (rc) return rc;
  return fold_status(wgrad_reduce(wpart, blocks, 1, C * 9, dw_crs, l2 != 0.f ? w_crs : nullptr, l2, st), ft);
}
}  // namespace dk

// Fused stride-2 depthwise backward (3x3, pad 1): as dk_dwconv_bwd_bnbwd_f32 for a stride-2 layer.
// g / bn_x: the following BatchNorm's output gradient and raw input (N x OH x OW x C); x: this
// layer's input (N x H x W x C) with the input BN bn_* applied on load (bn_mean NULL: none); dx
// (NULL: weight gradient only) gets dgrad (+ residual); part: the input BN's stage-1 partials,
// dk_dwconv_bwd_s2_stats_rows rows.  OH = ceil(H / 2), OW = ceil(W / 2); C / 4 divides 256.
DK_API int dk_dwconv_bwd_s2_bnbwd_f32(const float* g, const float* bn_x, int N, int H, int W, int C, int OH, int OW,
                                      const float* out_mean, const float* out_invstd, const float* out_gamma,
                                      const float* out_beta, int out_relu, const float* k12, const float* x,
                                      const float* w_crs, float l2, float* dw_crs, float* dx, const float* residual,
                                      const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                      const float* bn_beta, int bn_relu, double* part, void* ws, size_t ws_bytes,
                                      void* stream) {
  return dk::dw_bwd_s2(g, bn_x, N, H, W, C, OH, OW, out_mean, out_invstd, out_gamma, out_beta, out_relu, k12, x,
                       w_crs, l2, dw_crs, dx, residual, bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu, part, ws,
                       ws_bytes, stream);
}

// The join form (fp32): x is a residual block's output y = ReLU(bn_j(join_x) + skip), no input BN;
// dx = (dgrad + residual) * (y > 0) and part (dk_dwconv_bwd_s2_stats_rows x 2 x C, required) gets
// stage 1 of bn_j's backward (dk_dwconv_dgrad_join_f32's work on the stride-2 path).
// residual_lattice = 2: the residual is the compact stride-2 lattice [N][OH][OW][C] (0: dense).
DK_API int dk_dwconv_bwd_s2_bnbwd_join_f32(const float* g, const float* bn_x, int N, int H, int W, int C, int OH,
                                           int OW, const float* out_mean, const float* out_invstd,
                                           const float* out_gamma, const float* out_beta, int out_relu,
                                           const float* k12, const float* x, const float* w_crs, float l2,
                                           float* dw_crs, float* dx, const float* residual, int residual_lattice,
                                           const float* join_x, const float* join_mean, const float* join_invstd,
                                           double* part, void* ws, size_t ws_bytes, void* stream) {
  using namespace dk;
  const hipStream_t st = as_stream(stream);
  if (!dws2_ok(N, H, W, C, OH, OW) || (residual_lattice != 0 && residual_lattice != 2)) return DK_ERR_ARGS;
  if (!g || !bn_x || !x || !w_crs || !dw_crs || !dx || !out_mean || !out_invstd || !out_gamma || !out_beta || !k12 ||
      !join_x || !join_mean || !join_invstd || !part)
    return DK_ERR_ARGS;
  if (!aligned16(out_mean) || !aligned16(out_invstd) || !aligned16(out_gamma) || !aligned16(out_beta) ||
      !aligned16(k12) || !aligned16(g) || !aligned16(bn_x) || !aligned16(x) || !aligned16(dx) ||
      !aligned16(join_x) || !aligned16(join_mean) || !aligned16(join_invstd) || (residual && !aligned16(residual)))
    return DK_ERR_ARGS;
  const size_t xb = (size_t)N * H * W * C * sizeof(float), yb = (size_t)N * OH * OW * C * sizeof(float);
  if (!fits(xb)) return DK_ERR_ARGS;
  if (ws_bytes < dk_dwconv_bwd_s2_workspace_bytes(N, H, W, C)) return DK_ERR_WORKSPACE;
  const int blocks = dws2_blocks(N, H, W, C);
  float* wpart = static_cast<float*>(ws);
  const BnBwdOut ob{out_mean, out_invstd, out_gamma, out_beta, k12, out_relu};
  JoinBwd jn{};
  jn.x = join_x;
  jn.mean = join_mean;
  jn.invstd = join_invstd;
  jn.res_lat = residual && residual_lattice == 2;
  FoldTail ft;
  if (!fold_take(part, blocks, C, 1, &ft)) ft.part = nullptr;
  const size_t shm = (size_t)256 * 9 * 4 * sizeof(float);
  if (out_relu)
    hipLaunchKernelGGL((dw_bwd_s2_kernel<false, false, true, float, true>), dim3(blocks), dim3(256), shm, st, g, bn_x,
                       (uint32_t)yb, ob, x, (uint32_t)xb, BnIn{}, w_crs, dx, residual, part, wpart, N, H, W, C, OH, OW,
                       ft, nt_stores(kNtDwDgrad), jn);
  else
    hipLaunchKernelGGL((dw_bwd_s2_kernel<false, false, false, float, true>), dim3(blocks), dim3(256), shm, st, g,
                       bn_x, (uint32_t)yb, ob, x, (uint32_t)xb, BnIn{}, w_crs, dx, residual, part, wpart, N, H, W, C,
                       OH, OW, ft, nt_stores(kNtDwDgrad), jn);
  int rc = launch_status();
  if (rc) return rc;
  return fold_status(wgrad_reduce(wpart, blocks, 1, C * 9, dw_crs, l2 != 0.f ? w_crs : nullptr, l2, st), ft);
}

DK_API int dk_dwconv_bwd_s2_bnbwd_bf16(const bf16_t* g, const bf16_t* bn_x, int N, int H, int W, int C, int OH,
                                       int OW, const float* out_mean, const float* out_invstd, const float* out_gamma,
                                       const float* out_beta, int out_relu, const float* k12, const bf16_t* x,
                                       const float* w_crs, float l2, float* dw_crs, bf16_t* dx,
                                       const bf16_t* residual, const float* bn_mean, const float* bn_invstd,
                                       const float* bn_gamma, const float* bn_beta, int bn_relu, double* part,
                                       void* ws, size_t ws_bytes, void* stream) {
  return dk::dw_bwd_s2(g, bn_x, N, H, W, C, OH, OW, out_mean, out_invstd, out_gamma, out_beta, out_relu, k12, x,
                       w_crs, l2, dw_crs, dx, residual, bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu, part, ws,
                       ws_bytes, stream);
}

// dk_dwconv_bwd_bnbwd_f32 for a layer whose input is a residual join's output (no input BN): dx
// is the gradient w.r.t. the join's pre-ReLU sum, dx = (dgrad + residual) * join_mask, and part
// (stats_rows x 2 x C) gets stage 1 of the backward of the join's BatchNorm (join_x: its raw
// input; join_mean / join_invstd) -- dk_relu_bwd_bn_partial_f64's work, without re-reading dx.
// join_mask == nullptr: x is the join's output itself and the mask is x > 0 (not read).
DK_API int dk_dwconv_bwd_bnbwd_join_f32(const float* g, const float* bn_x, int N, int H, int W, int C,
                                        const float* out_mean, const float* out_invstd, const float* out_gamma,
                                        const float* out_beta, int out_relu, const float* k12, const float* x,
                                        const float* w_crs, int R, int S, int pad, float l2, float* dw_crs, float* dx,
                                        const float* residual, const uint8_t* join_mask, const float* join_x,
                                        const float* join_mean, const float* join_invstd, double* part, void* ws,
                                        size_t ws_bytes, void* stream) {
  const hipStream_t st = as_stream(stream);
  if (R != 3 || S != 3 || pad != 1 || C % 4 || N < 1 || H < 1 || W < 1) return DK_ERR_ARGS;
  const DwbGeom geo = dwb_geom(W, C, dwb_cpt(4));
  const int cl = geo.cl;
  if (!g || !bn_x || !x || !w_crs || !dw_crs || !dx || !out_mean || !out_invstd || !out_gamma || !out_beta ||
      !k12 || !join_x || !join_mean || !join_invstd || !part)
    return DK_ERR_ARGS;
  if (!aligned16(g) || !aligned16(bn_x) || !aligned16(x) || !aligned16(dx) || (residual && !aligned16(residual)) ||
      !aligned16(out_mean) || !aligned16(out_invstd) || !aligned16(out_gamma) || !aligned16(out_beta) ||
      !aligned16(k12) || !aligned16(w_crs) || !aligned16(join_x) || !aligned16(join_mean) ||
      !aligned16(join_invstd) || (reinterpret_cast<uintptr_t>(join_mask) & 3))
    return DK_ERR_ARGS;
  const size_t bytes = (size_t)N * H * W * C * sizeof(float);
  if (!fits(bytes)) return DK_ERR_ARGS;
  if (ws_bytes < dk_dwconv_bwd_bnbwd_workspace_bytes(N, H, W, C, R, S)) return DK_ERR_WORKSPACE;
  const int strips = dwb_strips(N, W, C, geo);
  const int nranges = dwb_nranges(N, W, C, geo);
  const int ncht = (C / 4) / geo.cg;
  float* wpart = static_cast<float*>(ws);
  const BnBwdOut ob{out_mean, out_invstd, out_gamma, out_beta, k12, out_relu};
  const JoinBwd jn{join_mask, join_x, join_mean, join_invstd};
  const dim3 grid((unsigned)(strips * ncht));
  FoldTail ft;  // an armed in-launch fold of the join BN's partial rows (fold_tail.h)
  if (!fold_take(part, strips, C, ncht, &ft)) ft.part = nullptr;
  size_t shm = (size_t)256 * 9 * 4 * sizeof(float);
  const size_t ring = (size_t)2 * (cl + 2) * geo.cg * sizeof(f32x4);
  if (ring > shm) shm = ring;
#define DWJ_LAUNCH(RELU1_)                                                                                           \
  {                                                                                                                  \
    auto k = geo.cpt == 2                                                                                          \
                 ? (join_mask ? (residual ? dw_bwd_fused_kernel<false, false, RELU1_, true, float, 2>                \
                                          : dw_bwd_fused_kernel<false, false, RELU1_, true, float, 2, 256, false>)   \
                              : (residual ? dw_bwd_fused_kernel<false, false, RELU1_, true, float, 2, 256, true, false> \
                                          : dw_bwd_fused_kernel<false, false, RELU1_, true, float, 2, 256, false, false>)) \
                 : (residual ? dw_bwd_fused_kernel<false, false, RELU1_, true>                                        \
                             : dw_bwd_fused_kernel<false, false, RELU1_, true, float, 1, 256, false>);               \
    if (shm > 65536)                                                                                                 \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,       \
                                (int)shm);                                                                           \
    hipLaunchKernelGGL(k, grid, dim3(256), shm, st, g, bn_x, (uint32_t)bytes, ob, x, BnIn{}, w_crs, dx, residual,    \
                       part, wpart, N, H, W, C, cl, ft, jn, nt_stores(kNtDwBwd), nranges);                                                         \
  }
  if (out_relu)
    DWJ_LAUNCH(true)
  else
    DWJ_LAUNCH(false)
#undef DWJ_LAUNCH
  int rc = launch_status();
  if (rc) return rc;
  return fold_status(wgrad_reduce(wpart, strips, 1, C * R * S, dw_crs, l2 != 0.f ? w_crs : nullptr, l2, st), ft);
}

DK_API int dk_dwconv_wgrad_bnx_f32(const float* dy, const float* x, int N, int H, int W, int C, int R, int S,
                                   int stride, int pad, int OH, int OW, const float* w_crs, float l2, float* dw_crs,
                                   void* ws, size_t ws_bytes, const float* bn_mean, const float* bn_invstd,
                                   const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream) {
  if (!bn_mean) return DK_ERR_ARGS;
  return dw_wgrad(dy, x, N, H, W, C, R, S, stride, pad, OH, OW, w_crs, l2, dw_crs, ws, ws_bytes,
                  BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu}, as_stream(stream));
}

// ---------------------------------------------------------------------------------------
// bf16 storage (BASELINE config 5): activations / gradients bf16, weights and their
// gradients fp32, all arithmetic fp32 (same kernels, T = bf16_t).
// ---------------------------------------------------------------------------------------
DK_API int dk_dwconv_fwd_ex_bf16(const bf16_t* x, int N, int H, int W, int C, const float* w_crs, int R, int S,
                                 int stride, int pad, const float* bias, bf16_t* y, int OH, int OW,
                                 const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                                 const float* bn_beta, int bn_relu, double* stats, void* stream) {
  if (stride != 1 && stride != 2) return DK_ERR_ARGS;
  return dw_fwd_dispatch<bf16_t>(x, w_crs, bias, y, N, H, W, C, R, S, stride, OH, OW, pad,
                                 BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu}, as_stream(stream), stats,
                                 nullptr, BnIn{}, 1);
}

DK_API int dk_dwconv_dgrad_ex_bf16(const bf16_t* dy, int N, int OH, int OW, int C, const float* w_crs, int R, int S,
                                   int stride, int pad, bf16_t* dx, int H, int W, void* ws, size_t ws_bytes,
                                   const bf16_t* residual, const bf16_t* bn_x, const float* bn_mean,
                                   const float* bn_invstd, const float* bn_gamma, const float* bn_beta, int bn_relu,
                                   double* part, void* stream) {
  if ((part != nullptr) != (bn_x != nullptr)) return DK_ERR_ARGS;
  return dw_dgrad<bf16_t>(dy, N, OH, OW, C, w_crs, R, S, stride, pad, dx, H, W, ws, ws_bytes, residual, bn_x,
                          BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu}, part, as_stream(stream));
}

DK_API int dk_dwconv_wgrad_bnx_bf16(const bf16_t* dy, const bf16_t* x, int N, int H, int W, int C, int R, int S,
                                    int stride, int pad, int OH, int OW, const float* w_crs, float l2, float* dw_crs,
                                    void* ws, size_t ws_bytes, const float* bn_mean, const float* bn_invstd,
                                    const float* bn_gamma, const float* bn_beta, int bn_relu, void* stream) {
  return dw_wgrad<bf16_t>(dy, x, N, H, W, C, R, S, stride, pad, OH, OW, w_crs, l2, dw_crs, ws, ws_bytes,
                          BnIn{bn_mean, bn_invstd, bn_gamma, bn_beta, bn_relu}, as_stream(stream));
}
