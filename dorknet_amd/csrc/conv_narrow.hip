// Narrow-input convolution: the stem (conv0, 64 x 3 x 5 x 5 stride 2 on the 3-channel image;
// reference layers/convolution.py:58-100 with examples/imagenet_dogs_225_resnet_18_depsep.py:112-116),
// forward and weight gradient straight from the NCHW image.
//
// The generic implicit GEMM pads C = 3 to 4 and tiles k = (r, s, c) by 16: 112 MFMA k-steps'
// worth of work for a 75-long reduction, on an NHWC copy of the input.  Here one block owns a
// run of whole output rows (n, oh); per row it stages the R x C input rows it reads (NCHW, each a
// contiguous image row, zero-padded into an LDS row of odd stride) and runs
// v_mfma_f32_16x16x4_f32 with k = (c, r, s) -- the reference's KCRS weight order, so the
// weights are read in place -- padded only to a multiple of 4 (76 for the stem).
//
//  forward:  y[n, oh, ow, k] = sum_{c,r,s} x[n, c, st*oh + r - pad, st*ow + s - pad] * w[k][c][r][s]
//            tile = one output row (OW <= 128 pixels, 16-pixel MFMA row tiles) x all K <= 64
//            filters (wave w: filters 16w..16w+15); A = the staged rows read at
//            off(k) + st*ow, B = the weights in registers; + bias; optional BatchNorm
//            statistics of y per block (fp64) with the in-launch fold (fold_tail.h).
//  wgrad:    dw[k][c][r][s] = sum_{n,oh,ow} dy[n, oh, ow, k] * x[...]: the block's output rows
//            are the reduction, dy (formed on load from the following BatchNorm's gradient and
//            input, bn_bwd_elem, when that BN's backward is deferred) staged per row in LDS;
//            one [K][C*R*S] partial per block, then the fixed-order split-K reduce (+ l2 * w).
#include "dk_common.h"
#include "fold_tail.h"

namespace dk {
namespace nar {

constexpr int NT = 256;  // 4 waves: wave w owns filters [16w, 16w + 16)

struct Geo {
  int N, C, H, W, K, R, S, st, pad, OH, OW;
  int Kred;  // C * R * S
  int KK;    // ceil(Kred / 4) MFMA k-steps (forward)
  int Wp;    // staged columns per input row: st * (16 * T - 1) + S
  int CS;    // LDS row stride (odd: consecutive k land on opposite bank parities)
  int rows;  // N * OH output rows
  int rpb;   // output rows per block
  int nt;    // forward: nontemporal output stores (nt_stores(kNtStem))
};

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ih mod R for input rows ih >= -R (the padding rows above the image)
template <int R>
__device__ __forceinline__ int ring_slot(int ih) {
  return (ih + R * 4) % R;
}

// The R x C input rows an output row (n, oh) reads: thread = staged column (Wp <= 256), one
// register per (c, r) -- loaded for the next row while the current row's MFMAs run, stored
// to LDS row (c * R + r) after the row's barrier.  Zero outside the image.
template <int C, int R, int ST>
struct RowStage {
  float v[C][R];
  __device__ __forceinline__ void load(const float* __restrict__ x, const Geo& g, int n, int oh) {
    const __amdgpu_buffer_rsrc_t rsx = make_rsrc_v(x, (uint32_t)((size_t)g.N * C * g.H * g.W * 4));
    const int iw = (int)threadIdx.x - g.pad;
    const bool wok = (int)threadIdx.x < g.Wp && (unsigned)iw < (unsigned)g.W;
    const int voff = wok ? iw * 4 : (int)kOOBBytes;  // lane part of the offset (bytes)
    const int ih0 = ST * oh - g.pad;
    // rows outside the image read nothing (lane offset past the buffer, scalar offset 0): every
    // load is unconditional, so the waitcnt pass counts them exactly instead of draining all
    // memory operations -- the previous row's output stores included -- before the LDS staging
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool rok = (unsigned)(ih0 + r) < (unsigned)g.H;  // uniform
      const int vo = rok ? voff : (int)kOOBBytes;
#pragma unroll
      for (int c = 0; c < C; ++c)
        v[c][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                rsx, vo, rok ? (((n * C + c) * g.H + ih0 + r) * g.W) * 4 : 0, 0));
    }
  }
  __device__ __forceinline__ void store(float* xin, const Geo& g) const {
    if ((int)threadIdx.x >= g.Wp) return;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int r = 0; r < R; ++r) xin[(c * R + r) * g.CS + threadIdx.x] = v[c][r];
  }
  // Ring variant (the weight gradient): channel c's input row ih sits in LDS row c * R + (ih mod R),
  // so an output row of the same image stages only its ST new rows (window rows R - ST .. R - 1)
  // instead of all R; a block's first row, or the first row of a new image, stages all R.  Rows
  // left out read nothing (offset past the buffer) and are not stored.  The window wraps in the
  // ring: the per-k offsets are rebuilt per output row.
  __device__ __forceinline__ void load_ring(const float* __restrict__ x, const Geo& g, int n, int oh, bool full) {
    const __amdgpu_buffer_rsrc_t rsx = make_rsrc_v(x, (uint32_t)((size_t)g.N * C * g.H * g.W * 4));
    const int iw = (int)threadIdx.x - g.pad;
    const bool wok = (int)threadIdx.x < g.Wp && (unsigned)iw < (unsigned)g.W;
    const int voff = wok ? iw * 4 : (int)kOOBBytes;
    const int ih0 = ST * oh - g.pad;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool rok = (full || r >= R - ST) && (unsigned)(ih0 + r) < (unsigned)g.H;  // uniform
      const int vo = rok ? voff : (int)kOOBBytes;
#pragma unroll
      for (int c = 0; c < C; ++c)
        v[c][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                rsx, vo, rok ? (((n * C + c) * g.H + ih0 + r) * g.W) * 4 : 0, 0));
    }
  }
  __device__ __forceinline__ void store_ring(float* xin, const Geo& g, int oh, bool full) const {
    if ((int)threadIdx.x >= g.Wp) return;
    const int sb = ring_slot<R>(ST * oh - g.pad);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!full && r < R - ST) continue;  // (uniform)
      const int slot = sb + r >= R ? sb + r - R : sb + r;
#pragma unroll
      for (int c = 0; c < C; ++c) xin[(c * R + slot) * g.CS + threadIdx.x] = v[c][r];
    }
  }
};

// Offset of reduction index k = (c*R + r)*S + s in the staged rows (padded k: the zero row).
template <int C, int R, int S>
__device__ __forceinline__ int koff(int k, int CS) {
  if (k >= C * R * S) return C * R * CS;
  const int row = k / S;
  return row * CS + (k - row * S);
}

template <int T, int C, int R, int S, int ST>
__global__ __launch_bounds__(NT, 2) void fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                    const float* __restrict__ bias, float* __restrict__ y, Geo g,
                                                    double* __restrict__ part, FoldTail ft) {
  constexpr int KRED = C * R * S, KK = (KRED + 3) / 4;
  extern __shared__ float xin[];  // (C*R + 1) rows x CS
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int col = 16 * wave + li;  // this lane's filter (B column, C/D column)
  const bool cok = col < g.K;
  float b[KK];  // B = W[col][k = 4kk + lg] (KCRS: k = (c, r, s))
  int off[KK];  // A: staged-row offset of k
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    const int k = 4 * kk + lg;
    b[kk] = (cok && k < KRED) ? w[(size_t)col * KRED + k] : 0.f;
    off[kk] = koff<C, R, S>(k, g.CS);
  }
  for (int e = tid; e < g.CS; e += NT) xin[C * R * g.CS + e] = 0.f;
  const float bv = (bias && cok) ? bias[col] : 0.f;
  double sa = 0.0, sb = 0.0;
  const int blk = xcd_block(blockIdx.x, gridDim.x);  // consecutive row runs share an XCD's L2
  const int r0 = blk * g.rpb, r1 = min(g.rows, r0 + g.rpb);
  RowStage<C, R, ST> rs;
  // (all R rows restaged per output row: a ring of the rows, as the weight gradient's, measured
  // 3-6 % slower here -- profiles/r04p_stem_ab.txt -- the per-row offset shift costs more than the
  // loads it saves)
  if (r0 < r1) rs.load(x, g, r0 / g.OH, r0 % g.OH);
  const float* const xl = xin + ST * li;
  const uint32_t kb = (uint32_t)g.K * 4u;                                    // bytes per output pixel
  const uint32_t vbase = cok ? (uint32_t)(4 * lg * g.K + col) * 4u : kOOBBytes;  // lane part of the store offset
  for (int row = r0; row < r1; ++row) {
    __syncthreads();  // the previous row's LDS reads are done
    rs.store(xin, g);
    __syncthreads();
    if (row + 1 < r1) rs.load(x, g, (row + 1) / g.OH, (row + 1) % g.OH);  // in flight under the MFMAs
    f32x4 acc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // A values one k-step ahead: k-step kk + 1's LDS reads are issued before k-step kk's T MFMAs
    // (the scheduler otherwise waited out an LDS round trip every two MFMAs); the groups pin the
    // order, the k order of every accumulator is unchanged.
    float a[2][T];
#pragma unroll
    for (int t = 0; t < T; ++t) a[0][t] = xl[off[0] + 16 * ST * t];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      if (kk + 1 < KK) {
#pragma unroll
        for (int t = 0; t < T; ++t) a[(kk + 1) & 1][t] = xl[off[kk + 1] + 16 * ST * t];
      }
#pragma unroll
      for (int t = 0; t < T; ++t) acc[t] = mfma16(a[kk & 1][t], b[kk], acc[t]);
      if (kk + 1 < KK) __builtin_amdgcn_sched_group_barrier(0x100, T, 0);  // the next k-step's reads
      __builtin_amdgcn_sched_group_barrier(0x008, T, 0);                  // this k-step's MFMAs
    }
    // C/D: row (output pixel) 16t + 4lg + v, column = filter col.  Branch-free: buffer stores on the
    // row's bytes (a filter past K reads kOOBBytes, a pixel past OW lands past the row's range: both
    // dropped by the range check) and the statistics take 0 for them, in the same order.
    const __amdgpu_buffer_rsrc_t ry = make_rsrc_v(y + (size_t)row * g.OW * g.K, (uint32_t)g.OW * g.K * 4u);
    auto epilogue = [&](auto pol) {
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int ow = 16 * t + 4 * lg + v;
          const float o = acc[t][v] + bv;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, o), ry, (int)(vbase + (16 * t + v) * kb),
                                                0, decltype(pol)::value);
          const double od = cok && ow < g.OW ? (double)o : 0.0;
          sa += od;
          sb += od * od;
        }
    };
    if (g.nt)
      epilogue(std::integral_constant<int, 2>{});
    else
      epilogue(std::integral_constant<int, 0>{});
  }
  if (!part) return;
  // per-filter totals of the block: lane groups lg = 0..3 added in a fixed order
  double s1 = sa + __shfl_xor(sa, 16, 64), s2 = sb + __shfl_xor(sb, 16, 64);
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 32, 64);
  if (lg == 0 && cok) {
    pub_store(part + ((size_t)blk * 2 + 0) * g.K + col, s1);
    pub_store(part + ((size_t)blk * 2 + 1) * g.K + col, s2);
  }
  if (ft.part) fold_tail<NT>(ft, blk, 0, g.K, 0);
}

// The following BatchNorm's backward applied as dy is loaded (BNDEF) -- bit-identical to
// dk_bn_bwd_apply_f32 -- or dy as given.
struct DyIn {
  const float* g;    // dy, or the gradient w.r.t. the BN (+ReLU) output
  const float* bnx;  // BNDEF: the BN's raw input (= this layer's output)
  const float *mean, *invstd, *gamma, *beta, *k12;
  int relu;
  int lat;  // BNDEF: g given on the stride-lat lattice only (1 or 2; compact, zero elsewhere)
};

// Weight gradient.  MFMA C[filter][n] += A[filter][pixel] * B[pixel][n] over the pixels of the
// block's rows, 4 per v_mfma_f32_16x16x4_f32: lane (li, lg) of wave w holds A = dy[pixel 4q + lg]
// [filter 16w + li] -- loaded straight from HBM in that layout (dwords: 4 lane groups x 64
// contiguous bytes, the 4 waves together 4 whole 256-byte pixel rows), the BN backward applied
// in registers with the lane's own filter's coefficients, then parked in the wave's LDS A table
// -- and B = the staged input row value for column n = (c, r, s) = 16nt + li at pixel 4q + lg.
// Row stride CS = 8 (mod 32): the <= 4 input rows a 16-column window touches sit 8 banks apart
// and a row's 5 taps x 2 pixels (stride 2) cover 7 banks, so the B reads are conflict-free
// (same-address lanes broadcast).  The next row's dy and input rows are loaded while this
// row's MFMAs run.

template <bool BNDEF, int QC>
struct DyRow {
  float gq[QC], xq[QC];
  // voff: the lane's byte offset (lg * K + filt) * 4 within a pixel quad, kOOBBytes for a filter
  // past K.  Pixels past OW (a ragged or padded quad) read the next row (or 0 past the tensor:
  // the whole offset is in the range-checked vector offset) and are zeroed by the caller.
  // voffg: the lane's offset in a lattice g (d.lat == 2: even pixels only, compact -- the
  // pointwise stride-2 layer after the stem hands over its gradient without the zeros of the
  // widen, pointwise_convolution.py:68-72).
  __device__ __forceinline__ void load(const DyIn& d, const Geo& g, int row, int voff, int voffg) {
    const uint32_t bytes = (uint32_t)((size_t)g.rows * g.OW * g.K * 4);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc_v(d.bnx, bytes);
    // the row base goes into the range-checked vector offset (a scalar offset is not checked:
    // the padded quads of the last row would read past the tensor)
    const uint32_t rbase = (uint32_t)row * g.OW * g.K * 4;
    const int qstep = 16 * g.K;  // bytes per pixel quad
    if (d.lat == 1) {
      const __amdgpu_buffer_rsrc_t rg = make_rsrc_v(d.g, bytes);
#pragma unroll
      for (int q = 0; q < QC; ++q)
        gq[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, (int)((uint32_t)voff + rbase + q * qstep), 0, 0));
    } else {
      const int n = row / g.OH, oh = row - n * g.OH;
      const int OHc = (g.OH + 1) / 2, OWc = (g.OW + 1) / 2;
      if (oh & 1) {  // an off-lattice row: g is zero
#pragma unroll
        for (int q = 0; q < QC; ++q) gq[q] = 0.f;
      } else {
        const __amdgpu_buffer_rsrc_t rg = make_rsrc_v(d.g, (uint32_t)((size_t)g.N * OHc * OWc * g.K * 4));
        const uint32_t rb = (uint32_t)((n * OHc + (oh >> 1)) * OWc) * g.K * 4;
#pragma unroll
        for (int q = 0; q < QC; ++q)
          gq[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, (int)((uint32_t)voffg + rb + q * (qstep >> 1)), 0, 0));
      }
    }
    if constexpr (BNDEF) {
#pragma unroll
      for (int q = 0; q < QC; ++q)
        xq[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, (int)((uint32_t)voff + rbase + q * qstep), 0, 0));
    }
  }
};

// QC: pixel quads per row, compile-time (>= ceil(OW / 4); the quads past OW are zero).
template <int C, int R, int S, int ST, bool BNDEF, int QC>
__global__ __launch_bounds__(NT, 3) void wgrad_kernel(DyIn d, const float* __restrict__ x, Geo g,
                                                      float* __restrict__ ws) {
  constexpr int KRED = C * R * S, NTN = (KRED + 15) / 16;
  extern __shared__ float smem[];
  float* const xin = smem;  // (C + 1) * R rows x CS: the ring, then R zero rows
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // A table: [wave][q / 2][lane][q & 1] -- the pair (q, q + 1) of a lane is one 8-byte store and load
  static_assert(QC % 2 == 0, "pixel quads come in pairs");
  float* const at = smem + (C + 1) * R * g.CS + wave * QC * 64 + 2 * lane;
  const int li = lane & 15, lg = lane >> 4;
  const int filt = 16 * wave + li;  // this lane's filter (A row)
  const int voff = filt < g.K ? (lg * g.K + filt) * 4 : (int)kOOBBytes;
  // lattice g: lanes of odd pixels (lg odd) read nothing; even ones the compact pixel lg / 2
  const int voffg = d.lat == 1 ? voff : ((filt < g.K && !(lg & 1)) ? ((lg >> 1) * g.K + filt) * 4 : (int)kOOBBytes);
  // B column n = 16 nt + li is k = (c, r, s): staged row c * R + ((ih0 + r) mod R) (single ring,
  // RowStage::store_ring<false>): offset = lo + sb * CS, less R rows once sb >= R - r; padded k
  // read the R zero rows after the ring (no wrap)
  int offlo[NTN], thr[NTN];
#pragma unroll
  for (int nt = 0; nt < NTN; ++nt) {
    const int k = 16 * nt + li;
    const int rw = k / S, c = rw / R, r = rw - c * R;
    offlo[nt] = k < KRED ? rw * g.CS + (k - rw * S) + ST * lg : C * R * g.CS + ST * lg;
    thr[nt] = k < KRED ? R - r : R;
  }
  for (int e = tid; e < R * g.CS; e += NT) xin[C * R * g.CS + e] = 0.f;
  float mu = 0.f, is = 0.f, ga = 0.f, be = 0.f, k1 = 0.f, k2 = 0.f, f = 0.f;
  if (BNDEF && filt < g.K) {
    mu = d.mean[filt];
    is = d.invstd[filt];
    ga = d.gamma[filt];
    be = d.beta[filt];
    k1 = d.k12[filt];
    k2 = d.k12[g.K + filt];
    f = ga * is;
  }
  f32x4 acc[NTN];
#pragma unroll
  for (int nt = 0; nt < NTN; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int blk = xcd_block(blockIdx.x, gridDim.x);
  const int r0 = blk * g.rpb, r1 = min(g.rows, r0 + g.rpb);
  RowStage<C, R, ST> rs;
  DyRow<BNDEF, QC> dr;
  if (r0 < r1) {
    rs.load_ring(x, g, r0 / g.OH, r0 % g.OH, true);
    dr.load(d, g, r0, voff, voffg);
  }
  for (int row = r0; row < r1; ++row) {
    const int oh = row % g.OH;
    const bool full = row == r0 || oh == 0;
    __syncthreads();  // the previous row's LDS reads are done
    rs.store_ring(xin, g, oh, full);
    int offn[NTN];
    {
      const int sb = ring_slot<R>(ST * oh - g.pad);
#pragma unroll
      for (int nt = 0; nt < NTN; ++nt) offn[nt] = offlo[nt] + (sb >= thr[nt] ? (sb - R) * g.CS : sb * g.CS);
    }
    // dy -> this lane's slots of the wave's A table, two pixel quads at a time in packed fp32 (v_pk_*:
    // the same IEEE operations as bn_bwd_elem / bn_out per element, bit-identical; the per-element form
    // made this the kernel's main VALU work, 4.2 VALU instructions per MFMA, profiles/r06g_sq_ratios_c3.md)
    const bool edge = 4 * QC > g.OW || 16 * (wave + 1) > g.K;  // (uniform) ragged / padded quads or filters
#pragma unroll
    for (int q = 0; q < QC; q += 2) {
      f32x2 ge = {dr.gq[q], dr.gq[q + 1]};
      if constexpr (BNDEF) {
        const f32x2 xe = {dr.xq[q], dr.xq[q + 1]};
        const f32x2 xh = (xe - f32x2{mu, mu}) * f32x2{is, is};
        if (d.relu) {
          const f32x2 bo = __builtin_elementwise_fma(f32x2{ga, ga}, xh, f32x2{be, be});  // bn_out
          ge[0] = bo[0] > 0.f ? ge[0] : 0.f;
          ge[1] = bo[1] > 0.f ? ge[1] : 0.f;
        }
        ge = f32x2{f, f} * __builtin_elementwise_fma(-xh, f32x2{k2, k2}, ge - f32x2{k1, k1});  // bn_bwd_elem
      }
      if (edge) {
#pragma unroll
        for (int e = 0; e < 2; ++e)
          if (4 * (q + e) + lg >= g.OW || filt >= g.K) ge[e] = 0.f;  // ragged / padded quad, filter past K
      }
      *reinterpret_cast<f32x2*>(at + q * 64) = ge;
    }
    __syncthreads();
    if (row + 1 < r1) {  // in flight under this row's MFMAs
      rs.load_ring(x, g, (row + 1) / g.OH, (row + 1) % g.OH, (row + 1) % g.OH == 0);
      dr.load(d, g, row + 1, voff, voffg);
    }
#pragma unroll
    for (int q = 0; q < QC; q += 2) {
      const f32x2 a2 = *reinterpret_cast<const f32x2*>(at + q * 64);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float* bq = xin + 4 * ST * (q + e);
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt) acc[nt] = mfma16(a2[e], bq[offn[nt]], acc[nt]);
      }
    }
  }
  // partial dw of this block: ws[blk][k][n] (C/D row = filter 16w + 4lg + v, column n)
#pragma unroll
  for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int k = 16 * wave + 4 * lg + v, nn = 16 * nt + li;
      if (k < g.K && nn < KRED) ws[((size_t)blk * g.K + k) * KRED + nn] = acc[nt][v];
    }
}

// ---------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------

// The (C, R, S, stride) shapes instantiated: 3-channel 5x5 / 7x7 / 3x3 stems, 1-channel (MNIST) 3x3 / 5x5.
#define DK_NARROW_SHAPES(X) \
  X(3, 5, 5, 2)             \
  X(3, 7, 7, 2)             \
  X(3, 3, 3, 1)             \
  X(3, 3, 3, 2)             \
  X(1, 3, 3, 1)             \
  X(1, 5, 5, 1)

static bool shape_ok(int C, int R, int S, int st) {
#define DK_SHAPE_OK(c, r, s, t) \
  if (C == c && R == r && S == s && st == t) return true;
  DK_NARROW_SHAPES(DK_SHAPE_OK)
#undef DK_SHAPE_OK
  return false;
}

static int quads(int OW) {  // the compiled pixel-quad counts (wgrad_kernel QC)
  const int q = cdiv(OW, 4);
  return q <= 4 ? 4 : q <= 8 ? 8 : q <= 16 ? 16 : q <= 28 ? 28 : 32;
}

static bool supported(int N, int C, int H, int W, int K, int R, int S, int st, int pad, int OH, int OW) {
  // staged columns: one per thread -- the forward's st * (16 * ceil(OW / 16) - 1) + S and the weight
  // gradient's st * (4 * quads(OW) - 1) + S (its padded pixel quads read staged zeros)
  if (!shape_ok(C, R, S, st) || OW < 1 || OW > 128 || st * (16 * cdiv(OW, 16) - 1) + S > NT ||
      st * (4 * quads(OW) - 1) + S > NT)
    return false;
  return N > 0 && K >= 4 && K <= 64 && K % 4 == 0 && pad >= 0 && OH >= 1 && OW <= 128 && H >= 1 && W >= 1 &&
         (size_t)N * OH * OW * K * 4 < ((size_t)1 << 31) && (size_t)N * C * H * W * 4 < ((size_t)1 << 31);
}

static Geo geo(int N, int C, int H, int W, int K, int R, int S, int st, int pad, int OH, int OW, bool wgrad = false) {
  Geo g{};
  g.N = N, g.C = C, g.H = H, g.W = W, g.K = K, g.R = R, g.S = S, g.st = st, g.pad = pad, g.OH = OH, g.OW = OW;
  g.Kred = C * R * S;
  g.KK = cdiv(g.Kred, 4);
  const int T = cdiv(OW, 16);
  // staged columns: every pixel the kernel's tiles touch (the weight gradient's padded quads
  // included: their B reads must see zeros -- a * 0 is not 0 for uninitialised LDS)
  g.Wp = wgrad ? st * (4 * quads(OW) - 1) + S : st * (16 * T - 1) + S;
  g.CS = wgrad ? (g.Wp + 23) / 32 * 32 + 8 : (g.Wp | 1);  // wgrad: 8 (mod 32); forward: odd
  g.rows = N * OH;
  return g;
}

// staged rows: forward C * R + 1 zero row; weight gradient the C * R ring + R zero rows
static size_t rows_lds(const Geo& g) { return (size_t)(g.C + 1) * g.R * g.CS * sizeof(float); }
static size_t fwd_lds(const Geo& g) { return (size_t)(g.C * g.R + 1) * g.CS * sizeof(float); }
static size_t wgrad_lds(const Geo& g) { return rows_lds(g) + (size_t)4 * quads(g.OW) * 64 * sizeof(float); }

using FwdFn = void (*)(const float*, const float*, const float*, float*, Geo, double*, FoldTail);
using WgrFn = void (*)(DyIn, const float*, Geo, float*);

template <int C, int R, int S, int ST>
static FwdFn fwd_fn_t(int T) {
  switch (T) {
    case 1: return fwd_kernel<1, C, R, S, ST>;
    case 2: return fwd_kernel<2, C, R, S, ST>;
    case 3: return fwd_kernel<3, C, R, S, ST>;
    case 4: return fwd_kernel<4, C, R, S, ST>;
    case 5: return fwd_kernel<5, C, R, S, ST>;
    case 6: return fwd_kernel<6, C, R, S, ST>;
    case 7: return fwd_kernel<7, C, R, S, ST>;
    default: return fwd_kernel<8, C, R, S, ST>;
  }
}
static FwdFn fwd_fn(const Geo& g) {
  const int T = cdiv(g.OW, 16);
#define DK_FWD_FN(c, r, s, t) \
  if (g.C == c && g.R == r && g.S == s && g.st == t) return fwd_fn_t<c, r, s, t>(T);
  DK_NARROW_SHAPES(DK_FWD_FN)
#undef DK_FWD_FN
  return nullptr;
}
template <bool BNDEF>
static WgrFn wgrad_fn(const Geo& g) {
#define DK_WGR_FN(c, r, s, t)                                     \
  if (g.C == c && g.R == r && g.S == s && g.st == t) switch (quads(g.OW)) { \
      case 4: return wgrad_kernel<c, r, s, t, BNDEF, 4>;                    \
      case 8: return wgrad_kernel<c, r, s, t, BNDEF, 8>;                    \
      case 16: return wgrad_kernel<c, r, s, t, BNDEF, 16>;                  \
      case 28: return wgrad_kernel<c, r, s, t, BNDEF, 28>;                  \
      default: return wgrad_kernel<c, r, s, t, BNDEF, 32>;                  \
    }
  DK_NARROW_SHAPES(DK_WGR_FN)
#undef DK_WGR_FN
  return nullptr;
}

// Blocks of a launch: every block resident at once (one round), each a run of whole rows.
static int grid_for(const void* fn, size_t lds, Geo& g) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, NT, lds) != hipSuccess || occ < 1) occ = 1;
  const int slots = occ * 256;  // MI355X CUs
  const int grid0 = g.rows < slots ? g.rows : slots;
  g.rpb = cdiv(g.rows, grid0);
  return cdiv(g.rows, g.rpb);
}

}  // namespace nar
}  // namespace dk

using namespace dk;
using namespace dk::nar;

DK_API int dk_conv2d_narrow_preferred(int N, int C, int H, int W, int K, int R, int S, int stride, int pad, int OH,
                                      int OW) {
  return supported(N, C, H, W, K, R, S, stride, pad, OH, OW) ? 1 : 0;
}

DK_API int dk_conv2d_fwd_narrow_stats_rows(int N, int C, int H, int W, int K, int R, int S, int stride, int pad,
                                           int OH, int OW) {
  if (!supported(N, C, H, W, K, R, S, stride, pad, OH, OW)) return 0;
  Geo g = geo(N, C, H, W, K, R, S, stride, pad, OH, OW);
  return grid_for(reinterpret_cast<const void*>(fwd_fn(g)), fwd_lds(g), g);
}

DK_API int dk_conv2d_fwd_narrow_f32(const float* x_nchw, int N, int C, int H, int W, const float* w_kcrs, int K, int R,
                                    int S, int stride, int pad, const float* bias, float* y, int OH, int OW,
                                    double* stats, void* stream) {
  if (!supported(N, C, H, W, K, R, S, stride, pad, OH, OW) || !x_nchw || !w_kcrs || !y) return DK_ERR_ARGS;
  Geo g = geo(N, C, H, W, K, R, S, stride, pad, OH, OW);
  g.nt = nt_stores(kNtStem);
  const FwdFn fn = fwd_fn(g);
  const size_t lds = fwd_lds(g);
  const int grid = grid_for(reinterpret_cast<const void*>(fn), lds, g);
  if (lds > 65536) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  FoldTail ft{};
  if (!stats || !fold_take(stats, grid, K, 1, &ft)) ft.part = nullptr;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(NT), lds, as_stream(stream), x_nchw, w_kcrs, bias, y, g, stats, ft);
  return fold_status(launch_status(), ft);
}

DK_API size_t dk_conv2d_wgrad_narrow_workspace_bytes(int N, int C, int H, int W, int K, int R, int S, int stride,
                                                     int pad, int OH, int OW) {
  if (!supported(N, C, H, W, K, R, S, stride, pad, OH, OW)) return 0;
  Geo g = geo(N, C, H, W, K, R, S, stride, pad, OH, OW, true);
  const int grid = grid_for(reinterpret_cast<const void*>(wgrad_fn<true>(g)), wgrad_lds(g), g);
  Geo g2 = g;
  const int grid2 = grid_for(reinterpret_cast<const void*>(wgrad_fn<false>(g)), wgrad_lds(g), g2);
  return (size_t)(grid > grid2 ? grid : grid2) * K * g.Kred * sizeof(float);
}

static int wgrad_narrow(const DyIn& d, bool bndef, const float* x, int N, int C, int H, int W, int K, int R, int S,
                        int stride, int pad, int OH, int OW, const float* w_kcrs, float l2, float* dw, void* ws,
                        size_t ws_bytes, void* stream) {
  if (!supported(N, C, H, W, K, R, S, stride, pad, OH, OW) || !x || !dw || !ws || !d.g) return DK_ERR_ARGS;
  if ((reinterpret_cast<uintptr_t>(d.g) | reinterpret_cast<uintptr_t>(d.bnx) | reinterpret_cast<uintptr_t>(ws)) & 15)
    return DK_ERR_ARGS;
  if (ws_bytes < dk_conv2d_wgrad_narrow_workspace_bytes(N, C, H, W, K, R, S, stride, pad, OH, OW))
    return DK_ERR_WORKSPACE;
  Geo g = geo(N, C, H, W, K, R, S, stride, pad, OH, OW, true);
  const WgrFn fn = bndef ? wgrad_fn<true>(g) : wgrad_fn<false>(g);
  const size_t lds = wgrad_lds(g);
  const int grid = grid_for(reinterpret_cast<const void*>(fn), lds, g);
  if (lds > 65536) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const hipStream_t st = as_stream(stream);
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(fn, dim3(grid), dim3(NT), lds, st, d, x, g, part);
  const int rc = launch_status();
  if (rc) return rc;
  return splitk_reduce(part, grid, K, g.Kred, dw, w_kcrs, l2, 0, C, C, R, S, st);
}

DK_API int dk_conv2d_wgrad_narrow_f32(const float* dy, const float* x_nchw, int N, int C, int H, int W, int K, int R,
                                      int S, int stride, int pad, int OH, int OW, const float* w_kcrs, float l2,
                                      float* dw_kcrs, void* ws, size_t ws_bytes, void* stream) {
  DyIn d{};
  d.g = dy;
  d.lat = 1;
  return wgrad_narrow(d, false, x_nchw, N, C, H, W, K, R, S, stride, pad, OH, OW, w_kcrs, l2, dw_kcrs, ws, ws_bytes,
                      stream);
}

DK_API int dk_conv2d_wgrad_bnbwd_narrow_f32(const float* g, const float* bn_x, const float* x_nchw, int N, int C,
                                            int H, int W, int K, int R, int S, int stride, int pad, int OH, int OW,
                                            const float* out_mean, const float* out_invstd, const float* out_gamma,
                                            const float* out_beta, int out_relu, const float* k12, int g_lattice,
                                            const float* w_kcrs, float l2, float* dw_kcrs, void* ws,
                                            size_t ws_bytes, void* stream) {
  if (!bn_x || !out_mean || !out_invstd || !out_gamma || !out_beta || !k12) return DK_ERR_ARGS;
  if (g_lattice != 1 && g_lattice != 2) return DK_ERR_ARGS;
  if ((reinterpret_cast<uintptr_t>(out_mean) | reinterpret_cast<uintptr_t>(out_invstd) |
       reinterpret_cast<uintptr_t>(out_gamma) | reinterpret_cast<uintptr_t>(out_beta) |
       reinterpret_cast<uintptr_t>(k12)) & 15)
    return DK_ERR_ARGS;
  DyIn d{g, bn_x, out_mean, out_invstd, out_gamma, out_beta, k12, out_relu, g_lattice};
  return wgrad_narrow(d, true, x_nchw, N, C, H, W, K, R, S, stride, pad, OH, OW, w_kcrs, l2, dw_kcrs, ws, ws_bytes,
                      stream);
}
