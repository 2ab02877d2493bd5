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
#include <atomic>

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
  const int nc = N - n0 < NB ? N - n0 : NB;  // (NB except the C = 64 fused backward's one column group)
  for (int i = tid; i < 2 * NB; i += NT) {
    const int which = i / NB, c = i - which * NB;
    if (c < nc) pub_store(part + ((size_t)blockIdx.x * 2 + which) * N + n0 + c, red[which][c]);
  }
  if (ft.part) {
    __syncthreads();  // red is read before the fold overwrites it
    fold_tail<NT>(ft, blockIdx.x, n0, nc, blockIdx.y, reinterpret_cast<double2*>(scratch));
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

// PLAIN: the gradient is given as is (g = dy; no following BatchNorm: the skip projections' dgrad,
// dk_pwconv_dgrad_f32 at stride 1 into the compact lattice) -- no xo loads, no transform, no write-through.
template <int KR, bool RES, bool PART, bool PLAIN = false>
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
  f32x4 mu = {}, is = {}, ga = {}, be = {}, k1 = {}, k2 = {}, f = {};
  if constexpr (!PLAIN) {
    mu = ld4(a.om + 4 * kv), is = ld4(a.ois + 4 * kv), ga = ld4(a.og + 4 * kv), be = ld4(a.ob + 4 * kv);
    k1 = ld4(a.k12 + 4 * kv), k2 = ld4(a.k12 + KR + 4 * kv);
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = ga[e] * is[e];
  }
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
      if constexpr (!PLAIN)
        sx[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)lofs[j], 0, 0));
    }
  };
  auto stage = [&](int tile, float* dst, const f32x4* sg, const f32x4* sx) {
    const __amdgpu_buffer_rsrc_t rdy = tile_rsrc(writer ? a.dy_out : a.g, KR, tile, writer ? a.M : 0);
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      const int r = r0 + j * (NT / KV);
      f32x4 v = sg[j];
      if constexpr (!PLAIN)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xe = sx[j][e];
        float ge = sg[j][e];
        const bool kill = (!(bn_out(xe, mu[e], is[e], ga[e], be[e]) > 0.f)) & orelu;
        ge = kill ? 0.f : ge;
        v[e] = (DK_PWD_EXP & 2) ? ge + xe : bn_bwd_elem(xe, ge, mu[e], is[e], f[e], k1[e], k2[e]);
      }
      st4(dst + r * SK + 4 * kv, v);
      if constexpr (!PLAIN) bstore_nt(__builtin_bit_cast(u32x4, v), rdy, (int)lofs[j], 0, a.nt);
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
// The K = 512 dgrad at two waves per SIMD (round 6).  dgrad_kernel<512> holds each wave's B fragments
// for 32 columns x 512 k in 256 VGPRs, so it runs one wave per SIMD and one block per CU, with no
// second wave to cover its staging and barriers (0.28 of the fp32 MFMA peak in the step).  Here a
// block of 8 waves owns the same 128 columns, 16 per wave, on v_mfma_f32_16x16x4_f32: a wave's B
// fragments are 16 columns x 512 k = 128 VGPRs, so two waves share each SIMD.
//   * the same exact-fp32 k order as the 32 x 32 x 2 kernels (MFMA i consumes k(i, 0..3), below), so
//     dx and dy are bit-identical to dgrad_kernel and the tiled engine;
//   * 16-pixel tiles (one 16 x 16 MFMA block per wave and tile; the LDS tile is 34 KB, double
//     buffered), staged once per block with the BatchNorm backward formed on load, the next tile's
//     global loads in flight during the MFMAs, one barrier per tile;
//   * the LDS row is stored k-permuted, in four regions (one per MFMA k group kg = lane >> 4) holding
//     the values in the order the MFMAs consume them, so one ds_read_b128 feeds four MFMAs;
//   * the following BN's per-channel terms live in an LDS table (no registers through the MFMAs).
// k order: the 32 x 32 x 2 chain consumes k = 8q + e then 8q + 4 + e for e = 0..3, q = 0..K/8-1
// (exact fp32, an fmaf chain in k order: MI355X_MICROARCH.md).  MFMA i of the 16 x 16 x 4 chain takes
// four consecutive of those, k(i, kg) = 8 (i >> 1) + 2 (i & 1) + (kg >> 1) + 4 (kg & 1).
// ---------------------------------------------------------------------------------------
constexpr int TR16 = 16;          // pixels per tile
constexpr int NW16 = 8;           // waves per block, 16 columns each (the block's NB = 128 columns)
constexpr int NT16 = 64 * NW16;   // threads per block

template <int KR>
struct K16 {
  static constexpr int RS = KR / 4 + 4;  // region stride (floats): KR / 4 values per k group, + 4
  static constexpr int SK = 4 * RS + 4;  // row stride: odd in float4s (conflict-free row-strided b128 reads)
  static constexpr int KV = KR / 4;      // float4s per pixel row
  static constexpr int LV = TR16 * KV / NT16;
  static constexpr int NQ = KR / 16;     // ds_read_b128 per row block (4 MFMAs each)
};

// acc = the 16 x 16 tile product: A from the lane's k-group region (row l & 15), four values per read
template <int NQ>
__device__ __forceinline__ void mfma16_tile(const float* ap, const f32x4* bw, f32x4& acc) {
  constexpr int D = 4;
  acc = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 ab[D];
#pragma unroll
  for (int i = 0; i < D; ++i) ab[i] = ld4(ap + 4 * i);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const f32x4 av = ab[q % D];
    if (q + D < NQ) ab[q % D] = ld4(ap + 4 * (q + D));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bw[q][u], acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int KR, bool RES, bool PART, bool PLAIN = false>
__global__ __launch_bounds__(NT16, 2) void dgrad16_kernel(DgradArgs a) {
  using L = K16<KR>;
  constexpr int SK = L::SK, RS = L::RS, KV = L::KV, LV = L::LV, NQ = L::NQ;
  static_assert(KR % 256 == 0 && (SK / 4) % 2 == 1 && NT16 % KV == 0 && LV >= 1, "pwd::dgrad16_kernel shape");
  __shared__ __attribute__((aligned(16))) float As[2][TR16 * SK];
  __shared__ __attribute__((aligned(16))) f32x4 bnt[7][KV];
  static_assert(sizeof(double) * 2 * NT16 <= sizeof(float) * 2 * TR16 * SK, "fold scratch fits in the tiles");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, kg = lane >> 4;
  const int n0 = blockIdx.y * NB, N = a.N;
  const int col = n0 + 16 * wave + c16;
  // staging lanes: lanes 0-31 of a wave take the even float4s of its 64-float4 stretch of a pixel row,
  // lanes 32-63 the odd ones, so the 16 lanes of one LDS store all write one k-group region's 32
  // contiguous floats (in stretch order, even and odd neighbours hit the regions 4 banks apart: 3.6
  // conflict cycles per LDS instruction, profiles/r06g_sq_ratios_c3.md); the wave's global loads still
  // cover the stretch's 1 KB
  const int kvl = tid % KV, r0 = tid / KV;
  const int kv = (kvl & ~63) | ((kvl & 31) << 1) | ((kvl >> 5) & 1);
  if (!PLAIN && tid < KV) {
    const f32x4 ga = ld4(a.og + 4 * tid), is = ld4(a.ois + 4 * tid);
    bnt[0][tid] = ld4(a.om + 4 * tid);
    bnt[1][tid] = is;
    bnt[2][tid] = ga;
    bnt[3][tid] = ld4(a.ob + 4 * tid);
    bnt[4][tid] = ld4(a.k12 + 4 * tid);
    bnt[5][tid] = ld4(a.k12 + KR + 4 * tid);
    f32x4 f;
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = ga[e] * is[e];
    bnt[6][tid] = f;
  }
  const float pm = PART ? a.im[col] : 0.f, pis = PART ? a.iis[col] : 0.f, pga = PART ? a.ig[col] : 0.f,
              pbe = PART ? a.ib[col] : 0.f;
  const bool orelu = a.orelu != 0, irelu = a.irelu != 0;
  const bool writer = a.dy_out != nullptr && blockIdx.y == 0;
  const int ntiles = (a.M + TR16 - 1) / TR16, G = gridDim.x;
  uint32_t lofs[LV];
#pragma unroll
  for (int j = 0; j < LV; ++j) lofs[j] = off4(r0 + j * (NT16 / KV), KR, 4 * kv);
  // C layout of a 16 x 16 block: lane (c16, kg) holds rows 4 kg + r, column col
  const uint32_t cbase = off4(4 * kg, N, col);
  // staging destinations: float4 kv of a row (k = 4 kv .. + 3) goes to regions (kv & 1) and (kv & 1) + 2
  // at position kv & ~1, as two float2 (see the k order above)
  const int sreg = (kv & 1) * RS + (kv & ~1);

  auto tile_rsrc16 = [&](const float* p, int ld, int tile, int nrows) {
    const int rows = nrows - tile * TR16;
    return make_rsrc_v(p + (size_t)tile * TR16 * ld, rows > 0 ? (uint32_t)rows * ld * 4u : 0u);
  };
  auto load_tile = [&](int tile, f32x4* sg, f32x4* sx) {
    const __amdgpu_buffer_rsrc_t rg = tile_rsrc16(a.g, KR, tile, a.M), rx = tile_rsrc16(a.xo, KR, tile, a.M);
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      sg[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)lofs[j], 0, 0));
      if constexpr (!PLAIN)
        sx[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)lofs[j], 0, 0));
    }
  };
  auto stage = [&](int tile, float* dst, const f32x4* sg, const f32x4* sx) {
    const __amdgpu_buffer_rsrc_t rdy = tile_rsrc16(writer ? a.dy_out : a.g, KR, tile, writer ? a.M : 0);
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      const int r = r0 + j * (NT16 / KV);
      f32x4 v = sg[j];
      if constexpr (!PLAIN) {
        const f32x4 mu = bnt[0][kv], is = bnt[1][kv], ga = bnt[2][kv], be = bnt[3][kv], k1 = bnt[4][kv],
                    k2 = bnt[5][kv], f = bnt[6][kv];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xe = sx[j][e];
          float ge = sg[j][e];
          const bool kill = (!(bn_out(xe, mu[e], is[e], ga[e], be[e]) > 0.f)) & orelu;
          ge = kill ? 0.f : ge;
          v[e] = bn_bwd_elem(xe, ge, mu[e], is[e], f[e], k1[e], k2[e]);
        }
      }
      float* d = dst + r * SK + sreg;
      *reinterpret_cast<f32x2*>(d) = f32x2{v[0], v[2]};
      *reinterpret_cast<f32x2*>(d + 2 * RS) = f32x2{v[1], v[3]};
      if constexpr (!PLAIN) bstore_nt(__builtin_bit_cast(u32x4, v), rdy, (int)lofs[j], 0, a.nt);
    }
  };

  __syncthreads();  // the BN table
  int t = first_tile(ntiles);
  f32x4 bw[NQ];
  {
    f32x4 sg[LV], sx[LV];
    load_tile(t, sg, sx);
    // B fragments W[k(i, kg)][col], i = 4q + u, after the first tile's loads
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = 4 * q + u;
        const int k = 8 * (i >> 1) + 2 * (i & 1) + (kg >> 1) + 4 * (kg & 1);
        bw[q][u] = a.w[(size_t)k * N + col];
      }
    stage(t, &As[0][0], sg, sx);
  }
  __syncthreads();
  double ps = 0.0, pq = 0.0;
  int buf = 0;
  for (; t < ntiles; t += G) {
    f32x4 ng[LV], nx[LV];
    load_tile(t + G, ng, nx);
    const int mb = t * TR16 + 4 * kg;
    const __amdgpu_buffer_rsrc_t rxi = tile_rsrc16(PART ? a.xi : a.g, N, t, PART ? a.M : 0);
    const __amdgpu_buffer_rsrc_t rr = tile_rsrc16(RES ? a.res : a.g, N, t, RES ? a.M : 0);
    const __amdgpu_buffer_rsrc_t rdx = tile_rsrc16(a.dx, N, t, a.M);
    float exi[4], ers[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if constexpr (PART)
        exi[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rxi, (int)cbase, r * N * 4, 0));
      if constexpr (RES)
        ers[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, (int)cbase, r * N * 4, 0));
    }
    f32x4 acc;
    mfma16_tile<NQ>(&As[buf][0] + c16 * SK + kg * RS, bw, acc);
    if constexpr (RES) {
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] += ers[r];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = acc[r];
      bstore_nt(__builtin_bit_cast(uint32_t, v), rdx, (int)cbase, r * N * 4, a.nt);
    }
    if constexpr (PART) {
      const bool full = t * TR16 + TR16 <= a.M;  // a whole tile (uniform): no row masks
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = exi[r];
        const float xh = (x - pm) * pis;
        const bool kill = ((!(pga * xh + pbe > 0.f)) & irelu) | (!full && mb + r >= a.M);
        const float gv = kill ? 0.f : acc[r];
        ps += (double)gv;
        pq += (double)gv * (double)xh;
      }
    }
    stage(t + G, &As[buf ^ 1][0], ng, nx);
    __syncthreads();
    buf ^= 1;
  }
  if constexpr (PART) {
    // the block's partial row: the four k-group lanes of a column, then the waves' columns
    double(*const red)[NB] = reinterpret_cast<double(*)[NB]>(&As[0][0]);  // [2][NB]
    ps += __shfl_xor(ps, 16, 64);
    pq += __shfl_xor(pq, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    pq += __shfl_xor(pq, 32, 64);
    __syncthreads();  // the pixel tiles become scratch
    if (kg == 0) {
      red[0][16 * wave + c16] = ps;
      red[1][16 * wave + c16] = pq;
    }
    __syncthreads();
    for (int i = tid; i < 2 * NB; i += NT16) {
      const int which = i / NB, c = i - which * NB;
      pub_store(a.part + ((size_t)blockIdx.x * 2 + which) * N + n0 + c, red[which][c]);
    }
    if (a.ft.part) {
      __syncthreads();  // red is read before the fold overwrites it
      fold_tail<NT16>(a.ft, blockIdx.x, n0, NB, blockIdx.y, reinterpret_cast<double2*>(&As[0][0]));
    }
  }
}

// ---------------------------------------------------------------------------------------
// Fused backward (layers/pointwise_convolution.py:57-75 with the following BatchNorm's backward,
// batch_norm.py:125-174, formed on load): the dgrad above plus the weight gradient
//   dW[k][c] = sum_m dy[m][k] * bn_relu(x)[m][c]
// in the same pass, so dy is never stored and the layer input is read once (the dgrad's epilogue
// loads it for the input BatchNorm's partials anyway).  Per 32-pixel tile a wave
//   1. runs the dgrad MFMAs of its 32 columns (B fragments W resident, A = the LDS dy tile);
//   2. stores dx and reduces the input BN's partials from its C-layout x loads;
//   3. applies the input BN (+ReLU) to those same x values in registers -- lane (l32, h) holds
//      x[4h + (s & 3) + 8 (s >> 2)][col] for s = 0..15, which is exactly the A operand of k-step s
//      of v_mfma_f32_32x32x2_f32 with rows = its column and the k pair = pixels (s, h) -- and runs
//      dW^T[col][k] += bn_relu(x)^T . dy with B = the LDS dy tile read as one ds_read_b128 per 4
//      MFMAs (k-tile kt covers channels 4 l32 + (kt & 3) + 128 (kt >> 2)).
// The wave's dW block (its 32 columns x all KR channels, KR / 2 accumulator registers) lives in
// registers for the block's life; at the end it goes through LDS into a coalesced partial row
// wpart[blockIdx.x][KR][N], which splitk_reduce sums in a fixed order (+ l2 W).  dx and the BN
// partials are bit-identical to dgrad_kernel's; dW regroups the fp32 sum over pixels.
// ---------------------------------------------------------------------------------------
struct BwdArgs {
  const float* g;     // [M][KR]
  const float* xo;    // [M][KR] the following BN's raw input
  const float* w;     // [KR][N]
  float* dx;          // [M][N]
  const float* res;   // [M][N] nullable
  const float* xi;    // [M][N] the layer input (the input BN's raw input when BNIN)
  const float *om, *ois, *og, *ob, *k12;  // following BN
  int orelu;
  const float *im, *iis, *ig, *ib;  // input BN
  int irelu;
  double* part;       // [gridDim.x][2][N] (BNIN)
  float* wpart;       // [gridDim.x][KR][N]
  int M, N;
  FoldTail ft;
  int nt;             // nontemporal dx stores (nt_stores(kNtPwd))
};

template <int KR>
constexpr int bwd_wps() {
  return KR <= 128 ? 2 : 1;
}

template <int KR, bool RES, bool BNIN>
__global__ __launch_bounds__(NT, bwd_wps<KR>()) void bwd_kernel(BwdArgs a) {
  constexpr int SK = KR + 4, KV = KR / 4, LV = TR * KV / NT, KQ = KR / 8, NKT = KR / 32, NU = KR / 128;
  static_assert(KR % 128 == 0 && (SK / 4) % 2 == 1 && NT % KV == 0, "pwd::bwd_kernel shape");
  __shared__ __attribute__((aligned(16))) float As[2][TR * SK];
  // the following BN's per-channel terms (mean, invstd, gamma, beta, k1, k2, gamma * invstd): read
  // from LDS by the staging transform, so they hold no registers through the MFMA phases
  __shared__ __attribute__((aligned(16))) f32x4 bnt[7][KV];
  static_assert(sizeof(double) * 2 * NT <= sizeof(float) * 2 * TR * SK, "fold scratch fits in the tiles");
  static_assert(32 * (NB + 4) <= 2 * TR * SK, "dW transpose tile fits in the tiles");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * NB, N = a.N;
  const int col = n0 + 32 * wave + l32;
  // C = 64 (the stride-2 block's first pointwise layer): one column group of 64, so waves 2 and 3 only
  // stage the dy tiles (wave-uniform; N is a multiple of 32)
  const bool wact = n0 + 32 * wave < N;
  const int kv = tid % KV, r0 = tid / KV;
  if (tid < KV) {
    const f32x4 ga = ld4(a.og + 4 * tid), is = ld4(a.ois + 4 * tid);
    bnt[0][tid] = ld4(a.om + 4 * tid);
    bnt[1][tid] = is;
    bnt[2][tid] = ga;
    bnt[3][tid] = ld4(a.ob + 4 * tid);
    bnt[4][tid] = ld4(a.k12 + 4 * tid);
    bnt[5][tid] = ld4(a.k12 + KR + 4 * tid);
    f32x4 f;
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = ga[e] * is[e];
    bnt[6][tid] = f;
  }
  __syncthreads();
  const float pm = BNIN && wact ? a.im[col] : 0.f, pis = BNIN && wact ? a.iis[col] : 0.f,
              pga = BNIN && wact ? a.ig[col] : 0.f, pbe = BNIN && wact ? a.ib[col] : 0.f;
  const bool orelu = a.orelu != 0, irelu = a.irelu != 0;

  const int ntiles = (a.M + TR - 1) / TR, G = gridDim.x;
  uint32_t lofs[LV];
#pragma unroll
  for (int j = 0; j < LV; ++j) lofs[j] = off4(r0 + j * (NT / KV), KR, 4 * kv);
  // C-layout element offsets within a tile: a lane base + a uniform row offset
  const uint32_t cbase = off4(4 * h, N, col);

  auto load_tile = [&](int tile, f32x4* sg, f32x4* sx) {
    const __amdgpu_buffer_rsrc_t rg = tile_rsrc(a.g, KR, tile, a.M), rx = tile_rsrc(a.xo, KR, tile, a.M);
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      sg[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)lofs[j], 0, 0));
      sx[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)lofs[j], 0, 0));
    }
  };
  auto stage = [&](float* dst, const f32x4* sg, const f32x4* sx) {
    const f32x4 mu = bnt[0][kv], is = bnt[1][kv], ga = bnt[2][kv], be = bnt[3][kv], k1 = bnt[4][kv], k2 = bnt[5][kv],
                f = bnt[6][kv];
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
        v[e] = bn_bwd_elem(xe, ge, mu[e], is[e], f[e], k1[e], k2[e]);
      }
      st4(dst + r * SK + 4 * kv, v);
    }
  };

  int t = first_tile(ntiles);
  f32x4 bw[KQ];
  {
    f32x4 sg[LV], sx[LV];
    load_tile(t, sg, sx);
#pragma unroll
    for (int q = 0; q < KQ; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) bw[q][e] = wact ? a.w[(size_t)(8 * q + 4 * h + e) * N + col] : 0.f;
    stage(&As[0][0], sg, sx);
  }
  __syncthreads();
  f32x16 dw[NKT];
#pragma unroll
  for (int i = 0; i < NKT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) dw[i][r] = 0.f;
  double ps = 0.0, pq = 0.0;
  int buf = 0;
  for (; t < ntiles; t += G) {
    f32x4 ng[LV], nx[LV];
    load_tile(t + G, ng, nx);
    const float* tile = &As[buf][0];
    if (wact) {
    // the tile's C-layout operands (layer input, residual), in flight during the dgrad MFMAs
    const int mb = t * TR + 4 * h;
    const __amdgpu_buffer_rsrc_t rxi = tile_rsrc(a.xi, N, t, a.M);
    const __amdgpu_buffer_rsrc_t rr = tile_rsrc(RES ? a.res : a.xi, N, t, RES ? a.M : 0);
    const __amdgpu_buffer_rsrc_t rdx = tile_rsrc(a.dx, N, t, a.M);
    float ex[16], ers[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ro = ((r & 3) + 8 * (r >> 2)) * N * 4;
      ex[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rxi, (int)cbase, ro, 0));
      if constexpr (RES) ers[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, (int)cbase, ro, 0));
    }
    f32x16 acc;
    mfma_tile<KQ>(tile + l32 * SK + 4 * h, bw, acc);
    if constexpr (RES) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += ers[r];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = acc[r];
      bstore_nt(__builtin_bit_cast(uint32_t, v), rdx, (int)cbase, ((r & 3) + 8 * (r >> 2)) * N * 4, a.nt);
    }
    // the input BN's partials of dx, and the weight gradient's operand bn_relu(x)
    const bool full = t * TR + TR <= a.M;  // a whole tile (uniform): no row masks
    float yb[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int dm = (r & 3) + 8 * (r >> 2);
      const bool out = !full && mb + dm >= a.M;
      const float x = ex[r];
      if constexpr (BNIN) {
        const float xh = (x - pm) * pis;
        const float v = __builtin_fmaf(pga, xh, pbe);  // bn_out
        const bool dead = !(v > 0.f) & irelu;
        const float gv = (dead | out) ? 0.f : acc[r];
        ps += (double)gv;
        pq += (double)gv * (double)xh;
        yb[r] = (dead | out) ? 0.f : v;
      } else {
        yb[r] = out ? 0.f : x;
      }
    }
    // dW^T[col][k] += bn_relu(x)^T . dy over the tile's 32 pixels (rows past M are zero in yb)
    {
      const float* bp = tile + (4 * h) * SK + 4 * l32;
      f32x4 bv[NU], nb[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) bv[u] = ld4(bp + 128 * u);
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        if (s + 1 < 16) {
          const int pn = ((s + 1) & 3) + 8 * ((s + 1) >> 2);
#pragma unroll
          for (int u = 0; u < NU; ++u) nb[u] = ld4(bp + pn * SK + 128 * u);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < NU; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) dw[4 * u + e] = __builtin_amdgcn_mfma_f32_32x32x2f32(yb[s], bv[u][e], dw[4 * u + e], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < NU; ++u) bv[u] = nb[u];
      }
    }
    }  // wact
    stage(&As[buf ^ 1][0], ng, nx);
    __syncthreads();
    buf ^= 1;
  }
  // the weight-gradient partial row: per k-tile, the 4 waves' 32 x 32 blocks through an LDS tile
  // [32 k][NB + 4] into coalesced row stores (k-tile kt holds channels 4 i + (kt & 3) + 128 (kt >> 2))
  {
    constexpr int ST = NB + 4;
    float* T = &As[0][0];
    float* wp = a.wpart + (size_t)blockIdx.x * KR * N + n0;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 16; ++r) T[l32 * ST + 32 * wave + 4 * h + (r & 3) + 8 * (r >> 2)] = dw[kt][r];
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 32 * NB / 4 / NT; ++j) {
        const int idx = tid + NT * j, i = idx / (NB / 4), c4 = idx % (NB / 4);
        const int k = 4 * i + (kt & 3) + 128 * (kt >> 2);
        if (n0 + 4 * c4 < N) st4(wp + (size_t)k * N + 4 * c4, ld4(T + i * ST + 4 * c4));
      }
    }
  }
  if constexpr (BNIN) partial_row(ps, pq, a.part, N, n0, a.ft, &As[0][0]);
}

// ---------------------------------------------------------------------------------------
// The fused backward on v_mfma_f32_16x16x4_f32 (round 6): bwd_kernel's dgrad + weight gradient with
// dgrad16_kernel's layout -- 8 waves of 16 columns, 16-pixel tiles, the k-permuted LDS dy tile -- so
// that at K = 256 a wave holds 64 VGPRs of B fragments and 64 of weight-gradient accumulators and two
// waves share each SIMD (bwd_kernel<256>: one).  Per tile a wave
//   1. runs the dgrad MFMAs of its 16 columns (dx bit-identical to dgrad16_kernel / dgrad_kernel);
//   2. stores dx and reduces the input BN's partials from its C-layout x loads;
//   3. forms bn_relu(x) for its four C-layout pixels 4 kg + r -- exactly the A operand of
//      v_mfma_f32_16x16x4_f32 with rows = its 16 columns and the 4-deep reduction = pixels
//      (4 kg' + r for k-group kg') -- and accumulates dW^T[col][k] over the tile with B = dy read from
//      the LDS tile (lane (c16, kg) reads dy[pixel 4 kg + r][k = 16 kt + c16], one ds_read_b32 per
//      MFMA, conflict-free: the 16 k of a chunk fall on 16 distinct banks of the permuted row).
// Lane (c16, kg) ends with dW[16 kt + c16][col0 + 4 kg + 0..3] (col0 = the wave's first column), written
// as one 16-byte store per chunk into the partial row wpart[blockIdx.x][KR][N] (bwd_kernel's layout:
// the same fixed-order reduce follows).
// ---------------------------------------------------------------------------------------
template <int KR, bool RES, bool BNIN>
__global__ __launch_bounds__(NT16, 2) void bwd16_kernel(BwdArgs a) {
  using L = K16<KR>;
  constexpr int SK = L::SK, RS = L::RS, KV = L::KV, LV = L::LV, NQ = L::NQ, NKT = KR / 16;
  static_assert(KR % 256 == 0 && (SK / 4) % 2 == 1 && NT16 % KV == 0 && LV >= 1, "pwd::bwd16_kernel shape");
  __shared__ __attribute__((aligned(16))) float As[2][TR16 * SK];
  __shared__ __attribute__((aligned(16))) f32x4 bnt[7][KV];
  static_assert(sizeof(double) * 2 * NT16 <= sizeof(float) * 2 * TR16 * SK, "fold scratch fits in the tiles");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, kg = lane >> 4;
  const int n0 = blockIdx.y * NB, N = a.N;
  const int col = n0 + 16 * wave + c16;
  // staging lanes: lanes 0-31 of a wave take the even float4s of its 64-float4 stretch of a pixel row,
  // lanes 32-63 the odd ones, so the 16 lanes of one LDS store all write one k-group region's 32
  // contiguous floats (in stretch order, even and odd neighbours hit the regions 4 banks apart: 3.6
  // conflict cycles per LDS instruction, profiles/r06g_sq_ratios_c3.md); the wave's global loads still
  // cover the stretch's 1 KB
  const int kvl = tid % KV, r0 = tid / KV;
  const int kv = (kvl & ~63) | ((kvl & 31) << 1) | ((kvl >> 5) & 1);
  if (tid < KV) {
    const f32x4 ga = ld4(a.og + 4 * tid), is = ld4(a.ois + 4 * tid);
    bnt[0][tid] = ld4(a.om + 4 * tid);
    bnt[1][tid] = is;
    bnt[2][tid] = ga;
    bnt[3][tid] = ld4(a.ob + 4 * tid);
    bnt[4][tid] = ld4(a.k12 + 4 * tid);
    bnt[5][tid] = ld4(a.k12 + KR + 4 * tid);
    f32x4 f;
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = ga[e] * is[e];
    bnt[6][tid] = f;
  }
  const float pm = BNIN ? a.im[col] : 0.f, pis = BNIN ? a.iis[col] : 0.f, pga = BNIN ? a.ig[col] : 0.f,
              pbe = BNIN ? a.ib[col] : 0.f;
  const bool orelu = a.orelu != 0, irelu = a.irelu != 0;
  const int ntiles = (a.M + TR16 - 1) / TR16, G = gridDim.x;
  uint32_t lofs[LV];
#pragma unroll
  for (int j = 0; j < LV; ++j) lofs[j] = off4(r0 + j * (NT16 / KV), KR, 4 * kv);
  const uint32_t cbase = off4(4 * kg, N, col);
  const int sreg = (kv & 1) * RS + (kv & ~1);
  // the weight gradient's B operand: k = 16 kt + c16 sits in region ((r8 & 1) << 1) | ((r8 >> 2) & 1) at
  // position 4 kt + 2 (c16 >> 3) + ((r8 >> 1) & 1) of a pixel row (r8 = c16 & 7)
  const int r8 = c16 & 7;
  const int doff = ((((r8 & 1) << 1) | ((r8 >> 2) & 1)) * RS) + 2 * (c16 >> 3) + ((r8 >> 1) & 1);

  auto tile_rsrc16 = [&](const float* p, int ld, int tile, int nrows) {
    const int rows = nrows - tile * TR16;
    return make_rsrc_v(p + (size_t)tile * TR16 * ld, rows > 0 ? (uint32_t)rows * ld * 4u : 0u);
  };
  auto load_tile = [&](int tile, f32x4* sg, f32x4* sx) {
    const __amdgpu_buffer_rsrc_t rg = tile_rsrc16(a.g, KR, tile, a.M), rx = tile_rsrc16(a.xo, KR, tile, a.M);
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      sg[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)lofs[j], 0, 0));
      sx[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)lofs[j], 0, 0));
    }
  };
  auto stage = [&](float* dst, const f32x4* sg, const f32x4* sx) {
    const f32x4 mu = bnt[0][kv], is = bnt[1][kv], ga = bnt[2][kv], be = bnt[3][kv], k1 = bnt[4][kv], k2 = bnt[5][kv],
                f = bnt[6][kv];
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      const int r = r0 + j * (NT16 / KV);
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xe = sx[j][e];
        float ge = sg[j][e];
        const bool kill = (!(bn_out(xe, mu[e], is[e], ga[e], be[e]) > 0.f)) & orelu;
        ge = kill ? 0.f : ge;
        v[e] = bn_bwd_elem(xe, ge, mu[e], is[e], f[e], k1[e], k2[e]);
      }
      float* d = dst + r * SK + sreg;
      *reinterpret_cast<f32x2*>(d) = f32x2{v[0], v[2]};
      *reinterpret_cast<f32x2*>(d + 2 * RS) = f32x2{v[1], v[3]};
    }
  };

  __syncthreads();  // the BN table
  int t = first_tile(ntiles);
  f32x4 bw[NQ];
  {
    f32x4 sg[LV], sx[LV];
    load_tile(t, sg, sx);
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = 4 * q + u;
        const int k = 8 * (i >> 1) + 2 * (i & 1) + (kg >> 1) + 4 * (kg & 1);
        bw[q][u] = a.w[(size_t)k * N + col];
      }
    stage(&As[0][0], sg, sx);
  }
  __syncthreads();
  f32x4 dw[NKT];
#pragma unroll
  for (int i = 0; i < NKT; ++i) dw[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  double ps = 0.0, pq = 0.0;
  int buf = 0;
  for (; t < ntiles; t += G) {
    f32x4 ng[LV], nx[LV];
    load_tile(t + G, ng, nx);
    const int mb = t * TR16 + 4 * kg;
    const __amdgpu_buffer_rsrc_t rxi = tile_rsrc16(a.xi, N, t, a.M);
    const __amdgpu_buffer_rsrc_t rr = tile_rsrc16(RES ? a.res : a.xi, N, t, RES ? a.M : 0);
    const __amdgpu_buffer_rsrc_t rdx = tile_rsrc16(a.dx, N, t, a.M);
    float ex[4], ers[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ex[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rxi, (int)cbase, r * N * 4, 0));
      if constexpr (RES)
        ers[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, (int)cbase, r * N * 4, 0));
    }
    const float* tile = &As[buf][0];
    f32x4 acc;
    mfma16_tile<NQ>(tile + c16 * SK + kg * RS, bw, acc);
    if constexpr (RES) {
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] += ers[r];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = acc[r];
      bstore_nt(__builtin_bit_cast(uint32_t, v), rdx, (int)cbase, r * N * 4, a.nt);
    }
    // the input BN's partials of dx, and the weight gradient's operand bn_relu(x)
    const bool full = t * TR16 + TR16 <= a.M;  // a whole tile (uniform): no row masks
    float yb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool out = !full && mb + r >= a.M;
      const float x = ex[r];
      if constexpr (BNIN) {
        const float xh = (x - pm) * pis;
        const float v = __builtin_fmaf(pga, xh, pbe);  // bn_out
        const bool dead = !(v > 0.f) & irelu;
        const float gv = (dead | out) ? 0.f : acc[r];
        ps += (double)gv;
        pq += (double)gv * (double)xh;
        yb[r] = (dead | out) ? 0.f : v;
      } else {
        yb[r] = out ? 0.f : x;
      }
    }
    // dW^T[col][k] += bn_relu(x)^T . dy over the tile's 16 pixels (rows past M are zero in yb)
    {
      const float* bp = tile + (4 * kg) * SK + doff;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float bv[NKT];
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) bv[kt] = bp[r * SK + 4 * kt];
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) dw[kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(yb[r], bv[kt], dw[kt], 0, 0, 0);
      }
    }
    stage(&As[buf ^ 1][0], ng, nx);
    __syncthreads();
    buf ^= 1;
  }
  // the weight-gradient partial row: lane (c16, kg) holds dW[16 kt + c16][col0 + 4 kg + 0..3]
  {
    float* wp = a.wpart + (size_t)blockIdx.x * KR * N + n0 + 16 * wave + 4 * kg;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) st4(wp + (size_t)(16 * kt + c16) * N, dw[kt]);
  }
  if constexpr (BNIN) {
    double(*const red)[NB] = reinterpret_cast<double(*)[NB]>(&As[0][0]);  // [2][NB]
    ps += __shfl_xor(ps, 16, 64);
    pq += __shfl_xor(pq, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    pq += __shfl_xor(pq, 32, 64);
    __syncthreads();  // the pixel tiles become scratch
    if (kg == 0) {
      red[0][16 * wave + c16] = ps;
      red[1][16 * wave + c16] = pq;
    }
    __syncthreads();
    for (int i = tid; i < 2 * NB; i += NT16) {
      const int which = i / NB, c = i - which * NB;
      pub_store(a.part + ((size_t)blockIdx.x * 2 + which) * N + n0 + c, red[which][c]);
    }
    if (a.ft.part) {
      __syncthreads();
      fold_tail<NT16>(a.ft, blockIdx.x, n0, NB, blockIdx.y, reinterpret_cast<double2*>(&As[0][0]));
    }
  }
}

// ---------------------------------------------------------------------------------------
// Host side: the instantiated reductions and the grid.
// ---------------------------------------------------------------------------------------
#define DK_PWD_KR(X) X(64) X(128) X(256) X(512)
#define DK_PWD_KR_DGRAD(X) X(64) X(128) X(256)  // (K = 512: dgrad16_kernel)

static int occupancy(const void* fn, int nt = NT) {
  int v = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, fn, nt, 0) != hipSuccess || v < 1) v = 1;
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

template <int KR>
static int dgrad16_occ() {
  static const int occ = [] {
    const void* fs[] = {reinterpret_cast<const void*>(&dgrad16_kernel<KR, true, true>),
                        reinterpret_cast<const void*>(&dgrad16_kernel<KR, true, false>),
                        reinterpret_cast<const void*>(&dgrad16_kernel<KR, false, true>),
                        reinterpret_cast<const void*>(&dgrad16_kernel<KR, false, false>)};
    int o = 1 << 20;
    for (const void* f : fs) o = std::min(o, occupancy(f, NT16));
    return o;
  }();
  return occ;
}

template <int KR>
static int bwd16_occ() {
  static const int occ = [] {
    const void* fs[] = {reinterpret_cast<const void*>(&bwd16_kernel<KR, true, true>),
                        reinterpret_cast<const void*>(&bwd16_kernel<KR, true, false>),
                        reinterpret_cast<const void*>(&bwd16_kernel<KR, false, true>),
                        reinterpret_cast<const void*>(&bwd16_kernel<KR, false, false>)};
    int o = 1 << 20;
    for (const void* f : fs) o = std::min(o, occupancy(f, NT16));
    return o;
  }();
  return occ;
}

template <int KR>
static int bwd_occ() {
  static const int occ = [] {
    const void* fs[] = {reinterpret_cast<const void*>(&bwd_kernel<KR, true, true>),
                        reinterpret_cast<const void*>(&bwd_kernel<KR, true, false>),
                        reinterpret_cast<const void*>(&bwd_kernel<KR, false, true>),
                        reinterpret_cast<const void*>(&bwd_kernel<KR, false, false>)};
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
static int grid_x(int M, int N, int occ, int tr = TR) {
  const int ntiles = (M + tr - 1) / tr;
  const int groups = N < NB ? 1 : N / NB;  // (N < NB: the C = 64 fused backward, one column group)
  int slots = occ * 256 / groups;
  if (slots < 1) slots = 1;
  int gx = std::min(ntiles, slots);
  const int g8 = gx / 8 * 8;
  if (g8 >= 8 && (ntiles + g8 - 1) / g8 == (ntiles + gx - 1) / gx) gx = g8;
  return gx;
}

}  // namespace pwd

// Knob 11 = 0 (or the streaming knob 3 = 0) keeps the earlier paths.
static bool pwd_enabled() { return knob(kKnobPwDeep) == 1 && pw_stream_enabled(); }

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
// K = 512 runs the two-waves-per-SIMD 16 x 16 kernel (dgrad16_kernel), 16-pixel tiles.
static bool pwd_dgrad16(int K) { return K == 512; }

int pw_deep_dgrad_rows(int M, int K, int C) {
  if (pwd_dgrad16(K)) return pwd::grid_x(M, C, pwd::dgrad16_occ<512>(), pwd::TR16);
#define DK_ROWS(kr) \
  if (K == kr) return pwd::grid_x(M, C, pwd::dgrad_occ<kr>());
  DK_PWD_KR_DGRAD(DK_ROWS)
#undef DK_ROWS
  return 0;
}
int pw_deep_dgrad_slices(int M, int K, int C) { return C / pwd::NB; }

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
  if (pwd_dgrad16(K)) {
#define DK_L16(R_, P_) hipLaunchKernelGGL((pwd::dgrad16_kernel<512, R_, P_>), grid, dim3(pwd::NT16), 0, st, a)
    if (res && x)
      DK_L16(true, true);
    else if (res)
      DK_L16(true, false);
    else if (x)
      DK_L16(false, true);
    else
      DK_L16(false, false);
#undef DK_L16
    return launch_status();
  }
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
  DK_PWD_KR_DGRAD(DK_DG)
#undef DK_DG
#undef DK_L
  return DK_ERR_ARGS;
}

// The plain deep dgrad (PLAIN: dy given, no BatchNorm around it): dx[M][C] = dy . W, bit-identical to the
// tiled engine's (same MFMA k order).  The downsampling blocks' skip projections at stride 1 into the
// compact lattice.
int pw_deep_dgrad_plain(const float* dy, int M, int K, int C, const float* w, float* dx, hipStream_t st) {
  pwd::DgradArgs a{dy, nullptr, nullptr, w, dx, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                   nullptr, nullptr, nullptr, nullptr, 0, nullptr, M, C};
  a.nt = nt_stores(kNtPwd);
  const dim3 grid(pw_deep_dgrad_rows(M, K, C), C / pwd::NB);
  if (grid.x == 0) return DK_ERR_ARGS;
  if (pwd_dgrad16(K)) {
    hipLaunchKernelGGL((pwd::dgrad16_kernel<512, false, false, true>), grid, dim3(pwd::NT16), 0, st, a);
    return launch_status();
  }
#define DK_DG(kr)                                                                                           \
  if (K == kr) {                                                                                            \
    hipLaunchKernelGGL((pwd::dgrad_kernel<kr, false, false, true>), grid, dim3(pwd::NT), 0, st, a);         \
    return launch_status();                                                                                 \
  }
  DK_PWD_KR_DGRAD(DK_DG)
#undef DK_DG
  return DK_ERR_ARGS;
}

// Fused deep backward (bwd_kernel): reduction K in {128, 256}, C a multiple of the block's 128 columns,
// or K = 128 with C = 64 (one column group, half its waves staging only: the downsampling blocks' first
// pointwise layer at 28 x 28, whose unfused pair stored dy and re-read it on the side stream).
// Default on; knob 14 = 0 keeps the dgrad + side-stream weight gradient pair.
static bool pwd_bwd_enabled() { return knob(kKnobPwDeepBwd) == 1 && pwd_enabled(); }
bool pw_deep_bwd_ok(int K, int C, int M) {
  if (!pwd_bwd_enabled() || M <= 0 || (K != 128 && K != 256) || (C % pwd::NB && !(K == 128 && C == 64)))
    return false;
  return (size_t)M * (K > C ? K : C) * 4 < ((size_t)1 << 31);
}
// K = 256 runs the two-waves-per-SIMD 16 x 16 kernel (bwd16_kernel), 16-pixel tiles.  At K = 128 the
// 16 x 16 layout (four waves per SIMD) measured slower than bwd_kernel<128> (173.6 vs 163.0 us at
// 28 x 28 x 128, profiles/r06f_pwd16_bwd_ab.txt), so bwd16_kernel is instantiated at K = 256 only.
static bool pwd_bwd16(int K) { return K == 256; }

int pw_deep_bwd_rows(int M, int K, int C) {
  if (pwd_bwd16(K)) return pwd::grid_x(M, C, pwd::bwd16_occ<256>(), pwd::TR16);
  if (K == 128) return pwd::grid_x(M, C, pwd::bwd_occ<128>());
  return 0;
}
int pw_deep_bwd_slices(int M, int K, int C) { return C < pwd::NB ? 1 : C / pwd::NB; }

int pw_deep_bwd_bnbwd(const float* g, const float* bn_x, int M, int K, int C, const float* om, const float* ois,
                      const float* og, const float* ob, int orelu, const float* k12, const float* w, float* dx,
                      const float* res, const float* x, const float* im, const float* iis, const float* ig,
                      const float* ib, int irelu, double* part, float* wpart, hipStream_t st, const FoldTail* ft) {
  if ((im != nullptr) != (part != nullptr)) return DK_ERR_ARGS;
  pwd::BwdArgs a{g, bn_x, w, dx, res, x, om, ois, og, ob, k12, orelu, im, iis, ig, ib, irelu, part, wpart, M, C};
  if (ft && part) a.ft = *ft;
  a.nt = nt_stores(kNtPwd);
  const dim3 grid(pw_deep_bwd_rows(M, K, C), pw_deep_bwd_slices(M, K, C));
  if (grid.x == 0) return DK_ERR_ARGS;
  if (pwd_bwd16(K)) {
#define DK_L16(kr, R_, B_) hipLaunchKernelGGL((pwd::bwd16_kernel<kr, R_, B_>), grid, dim3(pwd::NT16), 0, st, a)
#define DK_B16(kr)             \
  if (K == kr) {               \
    if (res && im)             \
      DK_L16(kr, true, true);  \
    else if (res)              \
      DK_L16(kr, true, false); \
    else if (im)               \
      DK_L16(kr, false, true); \
    else                       \
      DK_L16(kr, false, false); \
    return launch_status();    \
  }
    DK_B16(256)
#undef DK_B16
#undef DK_L16
  }
#define DK_L(kr, R_, B_) hipLaunchKernelGGL((pwd::bwd_kernel<kr, R_, B_>), grid, dim3(pwd::NT), 0, st, a)
#define DK_BW(kr)             \
  if (K == kr) {              \
    if (res && im)            \
      DK_L(kr, true, true);   \
    else if (res)             \
      DK_L(kr, true, false);  \
    else if (im)              \
      DK_L(kr, false, true);  \
    else                      \
      DK_L(kr, false, false); \
    return launch_status();   \
  }
  DK_BW(128)
#undef DK_BW
#undef DK_L
  return DK_ERR_ARGS;
}


}  // namespace dk
