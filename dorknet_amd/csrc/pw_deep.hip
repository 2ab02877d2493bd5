// fp32 kernels for the deep pointwise layers (layers/pointwise_convolution.py:46-75 at the 28 x 28 /
// 14 x 14 / 7 x 7 units of ResNet-18-depsep: 128 / 256 / 512 channels on a side).  These GEMMs are
// MFMA-bound (arithmetic intensity 32-256 flop/B against the fp32 ridge of ~20); the tiled engine
// and pw_stream.hip's K = C = 128 forward reach 0.35-0.48 of the fp32 MFMA peak on them.
//
// What bounds them on gfx950 (profiles/r04_mfma_valu_overlap.txt, scripts/mfma_valu.hip): f32 VALU
// work does not overlap v_mfma_f32_32x32x2_f32 on a SIMD -- 4 MFMAs alone run at 0.87-0.91 of the
// peak, with one v_fma_f32 per MFMA 0.82-0.86, two 0.81-0.83, eight 0.67 -- while f64 VALU work
// mostly does (one v_fma_f64 per MFMA: 0.88-0.90).  So the design goal is few f32 VALU instructions
// per MFMA: the tiled engine's BN-on-load loaders and the first streaming kernels issued 5-8.
//
// Structure: weight-stationary waves over a block-shared pixel tile.
//   * a block owns NB = 128 output columns (blockIdx.y) and walks 32-pixel row tiles (blockIdx.x,
//     + gridDim.x, ...); its 4 waves own 32 columns each, with their B fragments -- the whole
//     reduction of their columns, KR / 2 VGPRs per lane in the v_mfma_f32_32x32x2_f32 layout -- loaded
//     into registers once;
//   * the block stages each pixel tile (32 x KR) once: coalesced 16-byte row loads, the BatchNorm
//     (+ReLU) applied on load (forward) or the following BatchNorm's backward formed on load (dgrad)
//     once per element by the block -- not once per column slice -- into an LDS tile (double
//     buffered; row stride KR + 4 floats, odd in float4s: conflict-free ds_read_b128);
//   * per 4 MFMAs a wave reads one ds_read_b128 of A and no other operand; the next tile's global
//     loads are in flight during the MFMAs; one barrier per tile;
//   * the epilogue works in the MFMA C layout (lane = output column): BatchNorm partial sums stay in
//     registers across the block's tiles, one partial row per block and column group.
// MFMA k order 8q + 4h + e (h = lane half), as the tiled engine: outputs are bit-identical to it.
#include <stdlib.h>

#include <algorithm>

#include "dk_common.h"
#include "fold_tail.h"

// Timing experiments only (scripts/pwd_exp.sh builds variant libraries; 0 in the product build):
// bit 0 drops the epilogue stores, bit 1 the on-load transforms, bit 3 the weight loads.
#ifndef DK_PWD_EXP
#define DK_PWD_EXP 0
#endif

namespace dk {
namespace pwd {

constexpr int TR = 32;       // pixels per tile
constexpr int NW = 4;        // waves per block (one 32-column MFMA block each)
constexpr int NB = 32 * NW;  // output columns per block
constexpr int NT = 64 * NW;  // threads per block
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Waves per SIMD the registers are sized for: the B fragments take KR / 2 VGPRs per lane.
template <int KR>
constexpr int fwd_wps() {
  return KR <= 64 ? 4 : KR <= 128 ? 3 : KR <= 256 ? 2 : 1;
}
template <int KR>
constexpr int dgrad_wps() {
  return KR <= 128 ? 2 : 1;
}

__device__ __forceinline__ uint32_t off4(int m, int ld, int c) { return ((uint32_t)m * ld + c) * 4u; }

// A buffer resource over rows [tile * TR, nrows) of a [nrows][ld] tensor: the tile's row offset goes
// into the (uniform) base address, so a lane's offset within the tile is the same for every tile (no
// per-tile VALU address arithmetic), and the range check still drops rows past nrows.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const float* p, int ld, int tile, int nrows) {
  const int rows = nrows - tile * TR;
  return make_rsrc_v(p + (size_t)tile * TR * ld, rows > 0 ? (uint32_t)rows * ld * 4u : 0u);
}

// acc = the 32 x 32 tile product of the LDS pixel tile (lane: row l32, k = 8q + 4h + e at ap + 8q) and the
// lane's B fragments, k-pairs in ascending order (the tiled engine's).  The A reads run kAD float4s
// ahead of their MFMAs (scheduling barriers keep each read D groups ahead): left to itself the
// scheduler issued each read just before its MFMAs, exposing the LDS latency every 8 MFMAs -- a
// quarter of the MFMA time at one wave per SIMD.
constexpr int kAD = 4;

// The first row tile of walker blockIdx.x in column group blockIdx.y.  With ntiles = q G + r, the r
// walkers that take an extra tile are rotated by a multiple of 8 per column group so that a CU's
// blocks of different groups (ids x and x + G y) do not all take one, and walker x of every group
// still stays on one XCD (ids congruent mod 8 when G is a multiple of 8).
__device__ __forceinline__ int first_tile(int ntiles) {
  const int G = gridDim.x, r = ntiles % G, s = (r + 7) & ~7;
  return (int)((blockIdx.x + (unsigned)blockIdx.y * (unsigned)s) % (unsigned)G);
}
template <int KQ>
__device__ __forceinline__ void mfma_tile(const float* ap, const f32x4* bw, f32x16& acc) {
  constexpr int D = KQ < kAD ? KQ : kAD;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  f32x4 ab[D];
#pragma unroll
  for (int i = 0; i < D; ++i) ab[i] = ld4(ap + 8 * i);
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const f32x4 av = ab[q % D];
    if (q + D < KQ) ab[q % D] = ld4(ap + 8 * (q + D));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], bw[q][e], acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// bn_out in packed fp32 (v_pk_mul / v_pk_fma: two lanes of the same IEEE operations per
// instruction, bit-identical to the scalar form): the forward's staging transform is its main VALU
// work, and f32 VALU does not overlap the MFMAs (the dgrad's per-element form packs as well left to
// the compiler; written this way it took more registers).
__device__ __forceinline__ f32x2 lo2(f32x4 v) { return f32x2{v[0], v[1]}; }
__device__ __forceinline__ f32x2 hi2(f32x4 v) { return f32x2{v[2], v[3]}; }
__device__ __forceinline__ f32x4 cat4(f32x2 a, f32x2 b) { return f32x4{a[0], a[1], b[0], b[1]}; }
// (x - mean) * invstd
__device__ __forceinline__ f32x4 xhat4(f32x4 x, f32x4 m, f32x4 i) {
  return cat4((lo2(x) - lo2(m)) * lo2(i), (hi2(x) - hi2(m)) * hi2(i));
}
// gamma * xh + beta (fma)
__device__ __forceinline__ f32x4 affine4(f32x4 xh, f32x4 g, f32x4 b) {
  return cat4(__builtin_elementwise_fma(lo2(g), lo2(xh), lo2(b)), __builtin_elementwise_fma(hi2(g), hi2(xh), hi2(b)));
}

struct FwdArgs {
  const float* x;     // [input pixels][KR] (the preceding BN's raw input when BN)
  const float* w;     // [N][KR]
  const float* bias;  // [N] nullable
  float* y;           // [M][N]
  const float *im, *iis, *ig, *ib;  // input BN (BN on load)
  int irelu;
  double* part;       // [gridDim.x][2][N]: (sum y, sum y^2) per block
  int M, N, H, W, OH, OW, sa;
  uint32_t xbytes;
  FoldTail ft;
  int nt;             // nontemporal y stores (nt_stores(kNtPwd))
};

// The block's partial row of column sums (fwd: sum y, sum y^2; dgrad: the BN-backward sums) from
// each lane's per-column fp64 accumulators, then the in-launch fold when armed.
__device__ __forceinline__ void partial_row(double ps, double pq, double* part, int N, int n0, const FoldTail& ft,
                                            float* scratch) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  double(*const red)[NB] = reinterpret_cast<double(*)[NB]>(scratch);  // [2][NB]
  ps += __shfl_xor(ps, 32, 64);
  pq += __shfl_xor(pq, 32, 64);
  __syncthreads();  // the pixel tiles become scratch
  if (h == 0) {
    red[0][32 * wave + l32] = ps;
    red[1][32 * wave + l32] = pq;
  }
  __syncthreads();
  for (int i = tid; i < 2 * NB; i += NT) {
    const int which = i / NB, c = i - which * NB;
    pub_store(part + ((size_t)blockIdx.x * 2 + which) * N + n0 + c, red[which][c]);
  }
  if (ft.part) {
    __syncthreads();  // red is read before the fold overwrites it
    fold_tail<NT>(ft, blockIdx.x, n0, NB, blockIdx.y, reinterpret_cast<double2*>(scratch));
  }
}

template <int KR, bool BN, bool STATS, bool STRIDED, bool HB>
__global__ __launch_bounds__(NT, fwd_wps<KR>()) void fwd_kernel(FwdArgs a) {
  constexpr int SK = KR + 4, KV = KR / 4, LV = TR * KV / NT, KQ = KR / 8;
  static_assert(KR % 32 == 0 && (SK / 4) % 2 == 1 && NT % KV == 0, "pwd::fwd_kernel shape");
  __shared__ __attribute__((aligned(16))) float As[2][TR * SK];
  static_assert(sizeof(double) * 2 * NT <= sizeof(float) * 2 * TR * SK, "fold scratch fits in the tiles");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * NB, N = a.N;
  const int col = n0 + 32 * wave + l32;
  const float bias = HB ? a.bias[col] : 0.f;
  const bool irelu = a.irelu != 0;
  // staging: lane loads float4 kv = tid % KV of rows tid / KV + j * (NT / KV): fixed channels
  const int kv = tid % KV, r0 = tid / KV;
  f32x4 mu, is, ga, be;
  if constexpr (BN) {
    mu = ld4(a.im + 4 * kv);
    is = ld4(a.iis + 4 * kv);
    ga = ld4(a.ig + 4 * kv);
    be = ld4(a.ib + 4 * kv);
  }
  const __amdgpu_buffer_rsrc_t rx = make_rsrc_v(a.x, a.xbytes);
  const int ntiles = (a.M + TR - 1) / TR, G = gridDim.x;
  // lane offsets within a tile (the tile's row offset is in the resource base: tile_rsrc)
  uint32_t lofs[LV], eofs[16];
#pragma unroll
  for (int j = 0; j < LV; ++j) lofs[j] = off4(r0 + j * (NT / KV), KR, 4 * kv);
#pragma unroll
  for (int r = 0; r < 16; ++r) eofs[r] = off4(4 * h + (r & 3) + 8 * (r >> 2), N, col);

  auto load_tile = [&](int tile, f32x4* st) {
    const __amdgpu_buffer_rsrc_t rt = tile_rsrc(a.x, KR, tile, a.M);
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      if constexpr (STRIDED) {
        // output pixel (n, oh, ow) reads input pixel (n, sa oh, sa ow); pixels past M map past the
        // input (zeros)
        const int m = tile * TR + r0 + j * (NT / KV);
        const int ow = m % a.OW, q = m / a.OW, oh = q % a.OH, n = q / a.OH;
        const int row = (n * a.H + oh * a.sa) * a.W + ow * a.sa;
        st[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)off4(row, KR, 4 * kv), 0, 0));
      } else {
        st[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rt, (int)lofs[j], 0, 0));
      }
    }
  };
  // the BatchNorm (+ReLU) on load; max(r, 0) is the reference's (r > 0) ? r : 0 (a NaN gives 0 both ways)
  auto stage = [&](float* dst, const f32x4* st) {
    if (BN && irelu) {
#pragma unroll
      for (int j = 0; j < LV; ++j) {
        f32x4 v = st[j];
        if (!(DK_PWD_EXP & 2)) {
          v = affine4(xhat4(v, mu, is), ga, be);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = __builtin_fmaxf(v[e], 0.f);
        }
        st4(dst + (r0 + j * (NT / KV)) * SK + 4 * kv, v);
      }
    } else {
#pragma unroll
      for (int j = 0; j < LV; ++j) {
        f32x4 v = st[j];
        if constexpr (BN) v = affine4(xhat4(v, mu, is), ga, be);
        st4(dst + (r0 + j * (NT / KV)) * SK + 4 * kv, v);
      }
    }
  };

  int t = first_tile(ntiles);
  f32x4 bw[KQ];
  {
    f32x4 st[LV];
    load_tile(t, st);
    // this lane's B fragments, W[col][8q + 4h + e] for every q, e, loaded once after the first tile's
    // pixels: staging waits only for those, and the first tile's MFMAs for each fragment in turn, so
    // the weight loads (L2-resident; 32-128 KB per block) overlap the first tile's work
#pragma unroll
    for (int q = 0; q < KQ; ++q)
      bw[q] = (DK_PWD_EXP & 8) ? f32x4{0.01f * q, 0.02f, 0.03f, (float)col} : ld4(a.w + (size_t)col * KR + 8 * q + 4 * h);
    stage(&As[0][0], st);
  }
  __syncthreads();
  double ps = 0.0, pq = 0.0;
  int buf = 0;
  for (; t < ntiles; t += G) {
    f32x4 nst[LV];
    load_tile(t + G, nst);  // in flight during the MFMAs
    const float* ap = &As[buf][0] + l32 * SK + 4 * h;
    f32x16 acc;
    mfma_tile<KQ>(ap, bw, acc);
    // epilogue: rows (r & 3) + 8 (r >> 2) + 4h of the tile, column col
    const int mb = t * TR + 4 * h;
    const __amdgpu_buffer_rsrc_t ry = tile_rsrc(a.y, N, t, a.M);
    if constexpr (HB) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += bias;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = acc[r];  // (not bit_cast(acc[r]): hipcc 7.2 stored element 0 for every r)
      if (!(DK_PWD_EXP & 1))
        bstore_nt(__builtin_bit_cast(uint32_t, v), ry, (int)eofs[r], 0, a.nt);
    }
    if constexpr (STATS) {
      if (t * TR + TR <= a.M) {  // a whole tile (uniform): no row masks
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const double d = (double)acc[r];
          ps += d;
          pq += d * d;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int dm = (r & 3) + 8 * (r >> 2);
          const double d = (mb + dm < a.M) ? (double)acc[r] : 0.0;
          ps += d;
          pq += d * d;
        }
      }
    }
    stage(&As[buf ^ 1][0], nst);
    __syncthreads();
    buf ^= 1;
  }
  if constexpr (STATS) partial_row(ps, pq, a.part, N, n0, a.ft, &As[0][0]);
}

// ---------------------------------------------------------------------------------------
// BN-backward-on-load dgrad (layers/pointwise_convolution.py:57-75 + layers/batch_norm.py:125-174):
// dx[M][N] = dy . W (+ residual), dy = the following BatchNorm's backward of (g, x_out) formed on
// load (bn_bwd_elem, bit-identical to dk_bn_bwd_apply_f32) and written through by column group 0
// for the weight gradient, and the input BatchNorm's backward partials of the stored dx.  KR = the
// layer's output channels K (the reduction), N = its input channels C.
// ---------------------------------------------------------------------------------------
struct DgradArgs {
  const float* g;     // [M][KR]
  const float* xo;    // [M][KR] the following BN's raw input
  float* dy_out;      // [M][KR] nullable
  const float* w;     // [KR][N]
  float* dx;          // [M][N]
  const float* res;   // [M][N] nullable
  const float* xi;    // [M][N] the input BN's raw input (partials), nullable
  const float *om, *ois, *og, *ob, *k12;  // following BN
  int orelu;
  const float *im, *iis, *ig, *ib;  // input BN (partials)
  int irelu;
  double* part;       // [gridDim.x][2][N]
  int M, N;
  FoldTail ft;
  int nt;             // nontemporal dy / dx stores (nt_stores(kNtPwd))
};

template <int KR, bool RES, bool PART>
__global__ __launch_bounds__(NT, dgrad_wps<KR>()) void dgrad_kernel(DgradArgs a) {
  constexpr int SK = KR + 4, KV = KR / 4, LV = TR * KV / NT, KQ = KR / 8;
  static_assert(KR % 32 == 0 && (SK / 4) % 2 == 1 && NT % KV == 0, "pwd::dgrad_kernel shape");
  __shared__ __attribute__((aligned(16))) float As[2][TR * SK];
  static_assert(sizeof(double) * 2 * NT <= sizeof(float) * 2 * TR * SK, "fold scratch fits in the tiles");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * NB, N = a.N;
  const int col = n0 + 32 * wave + l32;
  const int kv = tid % KV, r0 = tid / KV;
  const f32x4 mu = ld4(a.om + 4 * kv), is = ld4(a.ois + 4 * kv), ga = ld4(a.og + 4 * kv), be = ld4(a.ob + 4 * kv);
  const f32x4 k1 = ld4(a.k12 + 4 * kv), k2 = ld4(a.k12 + KR + 4 * kv);
  f32x4 f;
#pragma unroll
  for (int e = 0; e < 4; ++e) f[e] = ga[e] * is[e];
  const float pm = PART ? a.im[col] : 0.f, pis = PART ? a.iis[col] : 0.f, pga = PART ? a.ig[col] : 0.f,
              pbe = PART ? a.ib[col] : 0.f;
  const bool orelu = a.orelu != 0, irelu = a.irelu != 0;

  // dy written through by column group 0 only (the others' stores go to a zero-size resource)
  const bool writer = a.dy_out != nullptr && blockIdx.y == 0;
  const int ntiles = (a.M + TR - 1) / TR, G = gridDim.x;
  // lane offsets within a tile (the tile's row offset is in the resource base: tile_rsrc)
  uint32_t lofs[LV], eofs[16];
#pragma unroll
  for (int j = 0; j < LV; ++j) lofs[j] = off4(r0 + j * (NT / KV), KR, 4 * kv);
#pragma unroll
  for (int r = 0; r < 16; ++r) eofs[r] = off4(4 * h + (r & 3) + 8 * (r >> 2), N, col);

  auto load_tile = [&](int tile, f32x4* sg, f32x4* sx) {
    const __amdgpu_buffer_rsrc_t rg = tile_rsrc(a.g, KR, tile, a.M), rx = tile_rsrc(a.xo, KR, tile, a.M);
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      sg[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)lofs[j], 0, 0));
      sx[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)lofs[j], 0, 0));
    }
  };
  auto stage = [&](int tile, float* dst, const f32x4* sg, const f32x4* sx) {
    const __amdgpu_buffer_rsrc_t rdy = tile_rsrc(writer ? a.dy_out : a.g, KR, tile, writer ? a.M : 0);
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      const int r = r0 + j * (NT / KV);
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xe = sx[j][e];
        float ge = sg[j][e];
        const bool kill = (!(bn_out(xe, mu[e], is[e], ga[e], be[e]) > 0.f)) & orelu;
        ge = kill ? 0.f : ge;
        v[e] = (DK_PWD_EXP & 2) ? ge + xe : bn_bwd_elem(xe, ge, mu[e], is[e], f[e], k1[e], k2[e]);
      }
      st4(dst + r * SK + 4 * kv, v);
      bstore_nt(__builtin_bit_cast(u32x4, v), rdy, (int)lofs[j], 0, a.nt);
    }
  };

  int t = first_tile(ntiles);
  f32x4 bw[KQ];
  {
    f32x4 sg[LV], sx[LV];
    load_tile(t, sg, sx);
    // B fragments W[8q + 4h + e][col], after the first tile's loads (as the forward)
#pragma unroll
    for (int q = 0; q < KQ; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) bw[q][e] = (DK_PWD_EXP & 8) ? 0.01f * q + e : a.w[(size_t)(8 * q + 4 * h + e) * N + col];
    stage(t, &As[0][0], sg, sx);
  }
  __syncthreads();
  double ps = 0.0, pq = 0.0;
  int buf = 0;
  for (; t < ntiles; t += G) {
    f32x4 ng[LV], nx[LV];
    load_tile(t + G, ng, nx);
    // the epilogue's C-layout operands of this tile, in flight during the MFMAs
    const int mb = t * TR + 4 * h;
    const __amdgpu_buffer_rsrc_t rxi = tile_rsrc(PART ? a.xi : a.g, N, t, PART ? a.M : 0);
    const __amdgpu_buffer_rsrc_t rr = tile_rsrc(RES ? a.res : a.g, N, t, RES ? a.M : 0);
    const __amdgpu_buffer_rsrc_t rdx = tile_rsrc(a.dx, N, t, a.M);
    float exi[16], ers[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if constexpr (PART)
        exi[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rxi, (int)eofs[r], 0, 0));
      if constexpr (RES)
        ers[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, (int)eofs[r], 0, 0));
    }
    const float* ap = &As[buf][0] + l32 * SK + 4 * h;
    f32x16 acc;
    mfma_tile<KQ>(ap, bw, acc);
    if constexpr (RES) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += ers[r];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = acc[r];  // (not bit_cast(acc[r]): hipcc 7.2 stored element 0 for every r)
      if (!(DK_PWD_EXP & 1))
        bstore_nt(__builtin_bit_cast(uint32_t, v), rdx, (int)eofs[r], 0, a.nt);
    }
    if constexpr (PART) {
      const bool full = t * TR + TR <= a.M;  // a whole tile (uniform): no row masks
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dm = (r & 3) + 8 * (r >> 2);
        const float x = exi[r];
        const float xh = (x - pm) * pis;
        const bool kill = ((!(pga * xh + pbe > 0.f)) & irelu) | (!full && mb + dm >= a.M);
        const float gv = kill ? 0.f : acc[r];
        ps += (double)gv;
        pq += (double)gv * (double)xh;
      }
    }
    stage(t + G, &As[buf ^ 1][0], ng, nx);
    __syncthreads();
    buf ^= 1;
  }
  if constexpr (PART) partial_row(ps, pq, a.part, N, n0, a.ft, &As[0][0]);
}

// ---------------------------------------------------------------------------------------
// Weight gradient (layers/pointwise_convolution.py:61-64): dW[k][c] = sum_m dy[m][k] xh[m][c] with
// xh = the input BatchNorm (+ReLU) applied on load (bn_out, as the forward).  Output-stationary
// waves: a wave owns a TK x TC block of dW -- (TK / 32) x (TC / 32) accumulator tiles, up to 256
// AGPRs at one wave per SIMD -- and streams its own contiguous run of pixel pairs, each pair one
// v_mfma_f32_32x32x2_f32 k-step.  The tiles are interleaved so that both operands come straight
// from global memory in one 16-byte (or 8-byte) load per lane: lane (i, h) loads dy[2p + h][k0 +
// TKQ i .. + TKQ) and x[2p + h][c0 + TCQ i .. + TCQ), and element a (b) of those is row i of k-tile
// a (column i of c-tile b): k = k0 + TKQ i + a, c = c0 + TCQ j + b.  Every operand element is
// loaded and transformed by exactly one lane (no LDS staging, no barriers in the loop), loads run
// kWD pairs ahead in a register ring; the BN on load is packed fp32 arithmetic (v_pk_*), bitwise
// bn_out.  The block's 4 waves split one dW block's pixel run four ways and add their tiles in
// LDS (fixed order) into one partial row; the partial rows go through splitk_reduce (fp64, + l2 w).
// ---------------------------------------------------------------------------------------
constexpr int kWD = 8;  // pixel pairs in flight per wave (16: 4-14 % slower, profiles/r04q_pwd_bench_kwd16.txt)

struct WgradArgs {
  const float* dy;  // [M][K]
  const float* x;   // [M][C] (the input BN's raw input when BN)
  const float *im, *iis, *ig, *ib;
  int irelu;
  float* part;      // [chunks][K][C]
  int M, K, C, chunks;
};

template <int Q>
struct VecOf;
template <>
struct VecOf<2> {
  typedef f32x2 T;
  static __device__ __forceinline__ T load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
  }
};
template <>
struct VecOf<4> {
  typedef f32x4 T;
  static __device__ __forceinline__ T load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
  }
};

template <int TKQ, int TCQ>
constexpr int wgrad_lds_floats() {
  return 2 * (32 * TKQ) * (32 * TCQ + 4);
}

template <int TKQ, int TCQ, bool BN, bool RELU>
__global__ __launch_bounds__(NT, 1) void wgrad_kernel(WgradArgs a) {
  constexpr int TK = 32 * TKQ, TC = 32 * TCQ, SR = TC + 4;  // LDS row stride (floats)
  typedef typename VecOf<TKQ>::T AV;
  typedef typename VecOf<TCQ>::T BV;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2][TK][SR]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int K = a.K, C = a.C, tiles_c = C / TC, ntiles = (K / TK) * tiles_c;
  // block -> (dW block, pixel chunk): chunk % 8 follows blockIdx % 8, so every dW block of one
  // pixel chunk runs on one XCD and shares its L2 copy of the chunk's dy and x
  const int id = blockIdx.x, rest = id >> 3;
  const int tile = rest % ntiles, chunk = (id & 7) + 8 * (rest / ntiles);
  const int k0 = (tile / tiles_c) * TK, c0 = (tile % tiles_c) * TC;
  // this wave's pixel pairs [pb, pe)
  const int npairs = (a.M + 1) >> 1, nsub = a.chunks * 4, sub = chunk * 4 + wave;
  const int pb = (int)((long long)npairs * sub / nsub), pe = (int)((long long)npairs * (sub + 1) / nsub);
  const uint32_t aoff = (uint32_t)(h * K + k0 + TKQ * l32) * 4u, boff = (uint32_t)(h * C + c0 + TCQ * l32) * 4u;
  BV mu, is, ga, be;
  if constexpr (BN) {
#pragma unroll
    for (int e = 0; e < TCQ; ++e) {
      const int c = c0 + TCQ * l32 + e;
      mu[e] = a.im[c];
      is[e] = a.iis[c];
      ga[e] = a.ig[c];
      be[e] = a.ib[c];
    }
  }
  // pair p's operands: one resource per tensor (range-checked: a ragged last pixel reads zeros),
  // the pair's row offset added to the lane offset; pairs past pe read zeros (offset past any
  // tensor), so they add nothing
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc_v(a.dy, (uint32_t)a.M * K * 4u);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc_v(a.x, (uint32_t)a.M * C * 4u);
  auto load_pair = [&](int p, AV& av, BV& bv) __attribute__((always_inline)) {
    const bool ok = p < pe;
    const uint32_t oa = ok ? (uint32_t)p * (uint32_t)(2 * K * 4) : kOOBBytes;
    const uint32_t ob = ok ? (uint32_t)p * (uint32_t)(2 * C * 4) : kOOBBytes;
    av = VecOf<TKQ>::load(rdy, aoff + oa);
    bv = VecOf<TCQ>::load(rx, boff + ob);
  };
  f32x16 acc[TKQ][TCQ];
#pragma unroll
  for (int i = 0; i < TKQ; ++i)
#pragma unroll
    for (int j = 0; j < TCQ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  AV ra[kWD];
  BV rb[kWD];
  // (issued in ring order: the waitcnt pass merges this order with the loop's at the loop head,
  // and a reordered prologue made it wait for every load there, every iteration)
#pragma unroll
  for (int s = 0; s < kWD; ++s) {
    load_pair(pb + s, ra[s], rb[s]);
    __builtin_amdgcn_sched_barrier(0);
  }
  for (int p = pb; p < pe; p += kWD) {
#pragma unroll
    for (int s = 0; s < kWD; ++s) {
      const AV av = ra[s];
      BV bv = rb[s];
      if constexpr (BN) {
        // bn_out elementwise in packed pairs: ((x - mean) * invstd) then fma(gamma, xh, beta)
#pragma unroll
        for (int e = 0; e < TCQ; e += 2) {
          const f32x2 xv = {bv[e], bv[e + 1]}, m2 = {mu[e], mu[e + 1]}, i2 = {is[e], is[e + 1]};
          const f32x2 g2 = {ga[e], ga[e + 1]}, b2 = {be[e], be[e + 1]};
          const f32x2 xh = (xv - m2) * i2;
          const f32x2 o = __builtin_elementwise_fma(g2, xh, b2);
          bv[e] = o[0];
          bv[e + 1] = o[1];
        }
        if constexpr (RELU) {
#pragma unroll
          for (int e = 0; e < TCQ; ++e) bv[e] = __builtin_fmaxf(bv[e], 0.f);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TKQ; ++i)
#pragma unroll
        for (int j = 0; j < TCQ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      // refill the ring slot once its operands are consumed (in place: loading it before the
      // MFMAs made the compiler rotate the ring through copies that waited for every load)
      load_pair(p + s + kWD, ra[s], rb[s]);
    }
  }
  // the block's 4 partial tiles added in LDS: (w0 + w2) + (w1 + w3); element (i, j, r) of a lane
  // is dW[k0 + TKQ (8 (r >> 2) + 4h + (r & 3)) + i][c0 + TCQ l32 + j].  The lane's base offsets are
  // pinned here (asm barrier) so the per-element addresses stay base + constant: hoisted above the
  // loop they took ~100 VGPRs and the 4 x 4 variant spilled.
  int lb = TKQ * 4 * h * SR + TCQ * l32;
  uint32_t gofs = (uint32_t)((k0 + TKQ * 4 * h) * C + c0 + TCQ * l32) * 4u;
  asm volatile("" : "+v"(lb), "+v"(gofs));
  auto tile_io = [&](float* base, bool add, bool store) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TKQ; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float* q = base + lb + (TKQ * (8 * (r >> 2) + (r & 3)) + i) * SR;
        if (store) {
          BV v;
#pragma unroll
          for (int j = 0; j < TCQ; ++j) v[j] = acc[i][j][r];
          *reinterpret_cast<BV*>(q) = v;
        } else {
          const BV v = *reinterpret_cast<const BV*>(q);
#pragma unroll
          for (int j = 0; j < TCQ; ++j) acc[i][j][r] = add ? acc[i][j][r] + v[j] : v[j];
        }
        __builtin_amdgcn_sched_barrier(0);  // one row at a time
      }
  };
  if (wave >= 2) tile_io(red + (wave - 2) * TK * SR, false, true);
  __syncthreads();
  if (wave < 2) tile_io(red + wave * TK * SR, true, false);
  __syncthreads();
  if (wave == 1) tile_io(red, false, true);
  __syncthreads();
  if (wave == 0) {
    tile_io(red, true, false);
    const __amdgpu_buffer_rsrc_t rp = make_rsrc_v(a.part + (size_t)chunk * K * C, (uint32_t)K * C * 4u);
#pragma unroll
    for (int i = 0; i < TKQ; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dk = TKQ * (8 * (r >> 2) + (r & 3)) + i;
        BV v;
#pragma unroll
        for (int j = 0; j < TCQ; ++j) v[j] = acc[i][j][r];
        if constexpr (TCQ == 4)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rp, (int)gofs, dk * C * 4, 0);
        else
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rp, (int)gofs, dk * C * 4, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
  }
}

// ---------------------------------------------------------------------------------------
// Host side: the instantiated reductions and the grid.
// ---------------------------------------------------------------------------------------
#define DK_PWD_KR(X) X(64) X(128) X(256) X(512)

static int occupancy(const void* fn) {
  int v = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, fn, NT, 0) != hipSuccess || v < 1) v = 1;
  return v;
}

template <int KR>
static int fwd_occ() {
  static const int occ = [] {
#define DK_F(B_, S_, T_) reinterpret_cast<const void*>(&fwd_kernel<KR, B_, S_, T_, false>), \
                         reinterpret_cast<const void*>(&fwd_kernel<KR, B_, S_, T_, true>)
    const void* fs[] = {DK_F(true, true, false), DK_F(true, false, false), DK_F(false, true, false),
                        DK_F(false, false, false), DK_F(true, true, true), DK_F(true, false, true),
                        DK_F(false, true, true), DK_F(false, false, true)};
#undef DK_F
    int o = 1 << 20;
    for (const void* f : fs) o = std::min(o, occupancy(f));
    return o;
  }();
  return occ;
}
template <int KR>
static int dgrad_occ() {
  static const int occ = [] {
    const void* fs[] = {reinterpret_cast<const void*>(&dgrad_kernel<KR, true, true>),
                        reinterpret_cast<const void*>(&dgrad_kernel<KR, true, false>),
                        reinterpret_cast<const void*>(&dgrad_kernel<KR, false, true>),
                        reinterpret_cast<const void*>(&dgrad_kernel<KR, false, false>)};
    int o = 1 << 20;
    for (const void* f : fs) o = std::min(o, occupancy(f));
    return o;
  }();
  return occ;
}

// Row-tile walkers per column group: every resident slot once (all blocks of a CU run at the same
// time, so each CU gets the same number of blocks and each block within one tile of the same share),
// at most one walker per tile; a multiple of the 8 XCDs when that costs no extra tile per walker, so
// that walker x of every column group runs on one XCD (block id x + gx * y) and the groups of a row
// tile share that XCD's L2 copy of its pixels.  A function of (M, N, occupancy) only: callers
// allocate exactly the partial rows the launch writes.
static int grid_x(int M, int N, int occ) {
  const int ntiles = (M + TR - 1) / TR;
  const int groups = N / NB;
  int slots = occ * 256 / groups;
  if (slots < 1) slots = 1;
  int gx = std::min(ntiles, slots);
  const int g8 = gx / 8 * 8;
  if (g8 >= 8 && (ntiles + g8 - 1) / g8 == (ntiles + gx - 1) / gx) gx = g8;
  return gx;
}

}  // namespace pwd

// DORKNET_PW_DEEP=0 (or the streaming switch DORKNET_PW_STREAM=0) keeps the earlier paths; knob 11.
static int g_pwd = -1;
static bool pwd_enabled() {
  if (g_pwd < 0) {
    const char* e = getenv("DORKNET_PW_DEEP");
    g_pwd = (e && e[0] == '0') ? 0 : 1;
  }
  return g_pwd == 1 && pw_stream_enabled();
}
void pw_deep_set(int v) { g_pwd = v < 0 ? -1 : v; }

static bool pwd_kr(int KR) { return KR == 64 || KR == 128 || KR == 256 || KR == 512; }

// The shapes the deep kernels take: reduction KR in {64, 128, 256, 512} with at least 128 channels
// on one side (K = C = 64 stays on pw_stream.hip), outputs a multiple of the block's 128 columns.
bool pw_deep_fwd_ok(int K, int C, int M, size_t xbytes) {
  if (!pwd_enabled() || M <= 0 || (K < 128 && C < 128) || !pwd_kr(C) || K % pwd::NB) return false;
  return xbytes < ((size_t)1 << 31) && (size_t)M * K * 4 < ((size_t)1 << 31);
}
bool pw_deep_dgrad_ok(int K, int C, int M) {
  if (!pwd_enabled() || M <= 0 || (K < 128 && C < 128) || !pwd_kr(K) || C % pwd::NB) return false;
  return (size_t)M * (K > C ? K : C) * 4 < ((size_t)1 << 31);
}

int pw_deep_fwd_rows(int M, int K, int C) {
#define DK_ROWS(kr) \
  if (C == kr) return pwd::grid_x(M, K, pwd::fwd_occ<kr>());
  DK_PWD_KR(DK_ROWS)
#undef DK_ROWS
  return 0;
}
int pw_deep_fwd_slices(int M, int K, int C) { return K / pwd::NB; }
int pw_deep_dgrad_rows(int M, int K, int C) {
#define DK_ROWS(kr) \
  if (K == kr) return pwd::grid_x(M, C, pwd::dgrad_occ<kr>());
  DK_PWD_KR(DK_ROWS)
#undef DK_ROWS
  return 0;
}
int pw_deep_dgrad_slices(int M, int K, int C) { return C / pwd::NB; }

// Weight gradient: K, C multiples of the dW block (TK = 128 when K >= 128, else 64; TC likewise),
// stride 1, at least 128 channels on one side; chunks = pixel chunks per dW block (a multiple of
// 8, about one wave per SIMD in all).
static int wg_q(int n) { return n >= 128 ? 4 : 2; }
// Off by default (DORKNET_PW_DEEP_WGRAD=1 or knob 12 = 1 turn it on): faster alone (square layers,
// profiles/r04n_pwd_bench.txt) but a slower step (profiles/r04s_ab_deep.txt: 8.664 vs 8.593 ms per
// step) -- a block takes a whole CU (one wave per SIMD, 512 registers, 135 KB of LDS), so on the
// side stream it shuts the main stream's kernels out of the CUs it holds instead of sharing them.
static int g_pwd_wg = -1;
void pw_deep_wgrad_set(int v) { g_pwd_wg = v < 0 ? -1 : v; }
static bool pwd_wgrad_enabled() {
  if (g_pwd_wg < 0) {
    const char* e = getenv("DORKNET_PW_DEEP_WGRAD");
    g_pwd_wg = (e && e[0] == '1') ? 1 : 0;
  }
  return g_pwd_wg == 1;
}
bool pw_deep_wgrad_ok(int K, int C, int M) {
  if (!pwd_wgrad_enabled()) return false;
  // square layers only: at K = 2C (the widening layers) the tiled engine measured as fast or faster
  // (profiles/r04n_pwd_bench.txt: 28x28 64->128 52.6 vs 52.9 us, 14x14 128->256 50.6 vs 50.5,
  // 7x7 256->512 48.8 vs 46.2)
  if (K != C) return false;
  if (!pwd_enabled() || M <= 1 || (K < 128 && C < 128) || K % 64 || C % 64 || K > 1024 || C > 1024) return false;
  if (K % (32 * wg_q(K)) || C % (32 * wg_q(C))) return false;
  return (size_t)M * (K > C ? K : C) * 4 < ((size_t)1 << 31);
}
int pw_deep_wgrad_chunks(int M, int K, int C) {
  const int ntiles = (K / (32 * wg_q(K))) * (C / (32 * wg_q(C)));
  int ch = 256 / ntiles;
  ch = ch < 8 ? 8 : ch / 8 * 8;
  // at least a few pixel pairs per wave
  while (ch > 8 && (long long)ch * 4 * 16 > (M + 1) / 2) ch -= 8;
  return ch;
}
size_t pw_deep_wgrad_ws_bytes(int M, int K, int C) {
  return (size_t)pw_deep_wgrad_chunks(M, K, C) * K * C * sizeof(float);
}

int pw_deep_wgrad(const float* dy, const float* x, int M, int K, int C, const float* im, const float* iis,
                  const float* ig, const float* ib, int irelu, float* part, hipStream_t st) {
  const int chunks = pw_deep_wgrad_chunks(M, K, C);
  pwd::WgradArgs a{dy, x, im, iis, ig, ib, irelu, part, M, K, C, chunks};
  const int tkq = wg_q(K), tcq = wg_q(C);
  const int ntiles = (K / (32 * tkq)) * (C / (32 * tcq));
  const dim3 grid((unsigned)(ntiles * chunks));
#define DK_WG(TKQ_, TCQ_)                                                                                         \
  if (tkq == TKQ_ && tcq == TCQ_) {                                                                               \
    const size_t lds = sizeof(float) * pwd::wgrad_lds_floats<TKQ_, TCQ_>();                                        \
    const void* fs[3] = {reinterpret_cast<const void*>(&pwd::wgrad_kernel<TKQ_, TCQ_, false, false>),              \
                         reinterpret_cast<const void*>(&pwd::wgrad_kernel<TKQ_, TCQ_, true, false>),               \
                         reinterpret_cast<const void*>(&pwd::wgrad_kernel<TKQ_, TCQ_, true, true>)};               \
    static const bool attr = [&] {                                                                                \
      for (const void* f : fs) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
      return true;                                                                                                \
    }();                                                                                                          \
    (void)attr;                                                                                                   \
    if (im && irelu)                                                                                              \
      hipLaunchKernelGGL((pwd::wgrad_kernel<TKQ_, TCQ_, true, true>), grid, dim3(pwd::NT), lds, st, a);           \
    else if (im)                                                                                                  \
      hipLaunchKernelGGL((pwd::wgrad_kernel<TKQ_, TCQ_, true, false>), grid, dim3(pwd::NT), lds, st, a);          \
    else                                                                                                          \
      hipLaunchKernelGGL((pwd::wgrad_kernel<TKQ_, TCQ_, false, false>), grid, dim3(pwd::NT), lds, st, a);         \
    return launch_status();                                                                                       \
  }
  DK_WG(4, 4)
  DK_WG(4, 2)
  DK_WG(2, 4)
#undef DK_WG
  return DK_ERR_ARGS;
}

int pw_deep_fwd(const float* x, int N, int H, int W, int stride, int OH, int OW, const float* w, int K, int C,
                const float* bias, float* y, const float* im, const float* iis, const float* ig, const float* ib,
                int irelu, double* part, hipStream_t st, const FoldTail* ft) {
  const int M = N * OH * OW;
  const bool strided = stride != 1 || H != OH || W != OW;
  pwd::FwdArgs a{x, w, bias, y, im, iis, ig, ib, irelu, part, M, K, H, W, OH, OW, stride,
                 (uint32_t)((size_t)N * H * W * C * 4)};
  if (ft && part) a.ft = *ft;
  a.nt = nt_stores(kNtPwd);
  const dim3 grid(pw_deep_fwd_rows(M, K, C), K / pwd::NB);
  if (grid.x == 0) return DK_ERR_ARGS;
#define DK_L(kr, B_, S_, T_)                                                                          \
  do {                                                                                                \
    if (bias)                                                                                         \
      hipLaunchKernelGGL((pwd::fwd_kernel<kr, B_, S_, T_, true>), grid, dim3(pwd::NT), 0, st, a);     \
    else                                                                                              \
      hipLaunchKernelGGL((pwd::fwd_kernel<kr, B_, S_, T_, false>), grid, dim3(pwd::NT), 0, st, a);    \
  } while (0)
#define DK_FWD(kr)                    \
  if (C == kr) {                      \
    if (strided) {                    \
      if (im && part)                 \
        DK_L(kr, true, true, true);   \
      else if (im)                    \
        DK_L(kr, true, false, true);  \
      else if (part)                  \
        DK_L(kr, false, true, true);  \
      else                            \
        DK_L(kr, false, false, true); \
    } else if (im && part)            \
      DK_L(kr, true, true, false);    \
    else if (im)                      \
      DK_L(kr, true, false, false);   \
    else if (part)                    \
      DK_L(kr, false, true, false);   \
    else                              \
      DK_L(kr, false, false, false);  \
    return launch_status();           \
  }
  DK_PWD_KR(DK_FWD)
#undef DK_FWD
#undef DK_L
  return DK_ERR_ARGS;
}

int pw_deep_dgrad_bnbwd(const float* g, const float* bn_x, int M, int K, int C, const float* om, const float* ois,
                        const float* og, const float* ob, int orelu, const float* k12, float* dy_out, const float* w,
                        float* dx, const float* res, const float* x, const float* im, const float* iis,
                        const float* ig, const float* ib, int irelu, double* part, hipStream_t st,
                        const FoldTail* ft) {
  pwd::DgradArgs a{g, bn_x, dy_out, w, dx, res, x, om, ois, og, ob, k12, orelu, im, iis, ig, ib, irelu, part, M, C};
  if (ft && part) a.ft = *ft;
  a.nt = nt_stores(kNtPwd);
  const dim3 grid(pw_deep_dgrad_rows(M, K, C), C / pwd::NB);
  if (grid.x == 0) return DK_ERR_ARGS;
#define DK_L(kr, R_, P_) hipLaunchKernelGGL((pwd::dgrad_kernel<kr, R_, P_>), grid, dim3(pwd::NT), 0, st, a)
#define DK_DG(kr)             \
  if (K == kr) {              \
    if (res && x)             \
      DK_L(kr, true, true);   \
    else if (res)             \
      DK_L(kr, true, false);  \
    else if (x)               \
      DK_L(kr, false, true);  \
    else                      \
      DK_L(kr, false, false); \
    return launch_status();   \
  }
  DK_PWD_KR(DK_DG)
#undef DK_DG
#undef DK_L
  return DK_ERR_ARGS;
}

}  // namespace dk
