// bf16-storage twins of pw_deep.hip for BASELINE config 5's deep pointwise layers (the 28 x 28 /
// 14 x 14 / 7 x 7 units with 128 / 256 / 512 channels, batch 512; layers/pointwise_convolution.py
// :46-75), on v_mfma_f32_32x32x16_bf16.
//
// The round-3 column-sliced kernels they replaced (since deleted) gave every wave its own pixel tile: each wave forms the BatchNorm transform of its tile for every
// 128-column slice, reads the per-channel BN terms from an LDS table per 4 elements and the weight
// fragments from LDS per MFMA -- 20+ VALU and 4-5 LDS reads per bf16 MFMA (r03z_sq_ratios_config5:
// MFMA busy 0.05-0.06, VALU / MFMA 30-35), 0.16-0.26 of HBM.  Here, as in pw_deep.hip:
//   * weight-stationary waves: a wave owns 32 output columns with their B fragments -- the whole
//     reduction, bf16x8 per k-step of 16, KR / 4 VGPRs -- in registers (RNE from the fp32 weights);
//   * a block (4 waves, 128 columns) stages each 32-pixel tile once: 16-byte row loads, the
//     transform in fp32 with the lane's 8 channels' BN terms read from an LDS table once per tile
//     (kept in registers they held the forward at KR = 512 and the dgrad at 256 to one wave per
//     SIMD), RNE to bf16, into an LDS tile (row stride KR + 8 bf16: an odd number of 16-byte units,
//     conflict-free ds_read_b128);
//   * per MFMA a wave reads one ds_read_b128 of A; one barrier per tile; the next tile's loads are
//     in flight during the MFMAs; the epilogue works in the MFMA C layout.
// Bit-identical to the kernels above and to the tiled engine's bf16 mode: the same operand
// rounding (fp32 transform, RNE), k-steps of 16 ascending with k = 16s + 8h + j on both operands,
// the same fp32 epilogue and RNE stores, statistics over the stored values (grouped per block).
#include <stdlib.h>

#include <algorithm>

#include "dk_common.h"
#include "fold_tail.h"

namespace dk {
namespace pwd16 {

constexpr int TR = 32, NW = 4, NB = 32 * NW, NT = 64 * NW;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void unpack8(u32x4 u, f32x4& lo, f32x4& hi) {
  lo = bf16x4_to_f32(uint2{u[0], u[1]});
  hi = bf16x4_to_f32(uint2{u[2], u[3]});
}
__device__ __forceinline__ u32x4 pack8(f32x4 lo, f32x4 hi) {
  const uint2 a = f32_to_bf16x4(lo), b = f32_to_bf16x4(hi);
  return u32x4{a.x, a.y, b.x, b.y};
}
__device__ __forceinline__ uint16_t bf16_bits(float v) { return __builtin_bit_cast(uint16_t, (__bf16)v); }
__device__ __forceinline__ float bf16_val(uint32_t bits) { return __builtin_bit_cast(float, bits << 16); }

template <int KR>
constexpr int fwd_wps() {
  return 2;
}
template <int KR>
constexpr int dgrad_wps() {
  return KR <= 256 ? 2 : 1;
}

// A buffer resource over rows [tile * TR, nrows) of a [nrows][ld] bf16 tensor (see pw_deep.hip).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const bf16_t* p, int ld, int tile, int nrows) {
  const int rows = nrows - tile * TR;
  return make_rsrc_v(p + (size_t)tile * TR * ld, rows > 0 ? (uint32_t)rows * ld * 2u : 0u);
}

// acc = the 32 x 32 product of the LDS pixel tile (lane row l32, k = 16s + 8h + j at ap + 16s) and the
// lane's B fragments, k-steps in ascending order, each A read kAD steps ahead of its MFMA.
constexpr int kAD = 4;
template <int KS>
__device__ __forceinline__ void mfma_tile(const bf16_t* ap, const bf16x8* bw, f32x16& acc) {
  constexpr int D = KS < kAD ? KS : kAD;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  bf16x8 ab[D];
#pragma unroll
  for (int i = 0; i < D; ++i) ab[i] = *reinterpret_cast<const bf16x8*>(ap + 16 * i);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const bf16x8 av = ab[s % D];
    if (s + D < KS) ab[s % D] = *reinterpret_cast<const bf16x8*>(ap + 16 * (s + D));
    __builtin_amdgcn_sched_barrier(0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bw[s], acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// The first row tile of walker blockIdx.x in column group blockIdx.y (pw_deep.hip: the walkers that
// take an extra tile rotated by a multiple of 8 per group).
__device__ __forceinline__ int first_tile(int ntiles) {
  const int G = gridDim.x, r = ntiles % G, s = (r + 7) & ~7;
  return (int)((blockIdx.x + (unsigned)blockIdx.y * (unsigned)s) % (unsigned)G);
}

// The block's partial row (sum, second sum) per column from the lanes' fp64 accumulators, then the
// in-launch fold when armed.
__device__ __forceinline__ void partial_row(double ps, double pq, double* part, int N, int n0, const FoldTail& ft,
                                            void* scratch) {
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
    __syncthreads();
    fold_tail<NT>(ft, blockIdx.x, n0, nc, blockIdx.y, reinterpret_cast<double2*>(scratch));
  }
}

struct FwdArgs {
  const bf16_t* x;    // [M][KR] (the input BN's raw input when BN)
  const float* w;     // [N][KR]
  const float* bias;  // [N] nullable
  bf16_t* y;          // [M][N]
  const float *im, *iis, *ig, *ib;
  int irelu;
  double* part;       // [gridDim.x][2][N]
  int M, N;
  FoldTail ft;
  int nt;             // nontemporal output stores (nt_stores(kNtPwd16))
};

template <int KR, bool BN, bool STATS, bool HB>
__global__ __launch_bounds__(NT, fwd_wps<KR>()) void fwd_kernel(FwdArgs a) {
  constexpr int SK = KR + 8, KV = KR / 8, LV = TR * KV / NT, KS = KR / 16;
  static_assert(KR % 64 == 0 && NT % KV == 0 && LV >= 1, "pwd16::fwd_kernel shape");
  __shared__ __attribute__((aligned(16))) bf16_t As[2][TR * SK];
  // the input BN's terms [4][KR], read by each thread for its 8 channels once per tile (held in
  // registers for the whole launch they cost 32 VGPRs: one wave per SIMD at KR = 512 instead of two)
  __shared__ __attribute__((aligned(16))) float tab[BN ? 4 * KR : 4];
  static_assert(sizeof(double) * 2 * NT <= sizeof(bf16_t) * 2 * TR * SK, "fold scratch fits in the tiles");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * NB, N = a.N, col = n0 + 32 * wave + l32;
  const float bias = HB ? a.bias[col] : 0.f;
  const bool irelu = a.irelu != 0;
  // staging: lane loads 8 channels kv of rows tid / KV + j * (NT / KV)
  const int kv = tid % KV, r0 = tid / KV;
  if constexpr (BN) {
    for (int c = tid; c < KR; c += NT) {
      tab[c] = a.im[c];
      tab[KR + c] = a.iis[c];
      tab[2 * KR + c] = a.ig[c];
      tab[3 * KR + c] = a.ib[c];
    }
    __syncthreads();
  }
  const int ntiles = (a.M + TR - 1) / TR, G = gridDim.x;
  // lane offsets within a tile (bytes), rebuilt per use from one base (an array of them was 24 VGPRs)
  const uint32_t lofs0 = ((uint32_t)r0 * KR + 8 * kv) * 2u, eofs0 = ((uint32_t)(4 * h) * N + col) * 2u;
  constexpr uint32_t kLStep = (uint32_t)(NT / KV) * KR * 2u;

  auto load_tile = [&](int tile, u32x4* st) {
    const __amdgpu_buffer_rsrc_t rt = tile_rsrc(a.x, KR, tile, a.M);
#pragma unroll
    for (int j = 0; j < LV; ++j)
      st[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rt, (int)(lofs0 + j * kLStep), 0, 0));
  };
  // the BatchNorm (+ReLU) on load in fp32, RNE to bf16 (the reference's (r > 0) ? r : 0)
  auto stage = [&](bf16_t* dst, const u32x4* st) {
    f32x4 mu[2], is[2], ga[2], be[2];
    if constexpr (BN) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        mu[p] = *reinterpret_cast<const f32x4*>(tab + 8 * kv + 4 * p);
        is[p] = *reinterpret_cast<const f32x4*>(tab + KR + 8 * kv + 4 * p);
        ga[p] = *reinterpret_cast<const f32x4*>(tab + 2 * KR + 8 * kv + 4 * p);
        be[p] = *reinterpret_cast<const f32x4*>(tab + 3 * KR + 8 * kv + 4 * p);
      }
    }
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      u32x4 q = st[j];
      if constexpr (BN) {
        f32x4 v[2];
        unpack8(q, v[0], v[1]);
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float r = bn_out(v[p][e], mu[p][e], is[p][e], ga[p][e], be[p][e]);
            v[p][e] = (irelu & !(r > 0.f)) ? 0.f : r;
          }
        q = pack8(v[0], v[1]);
      }
      *reinterpret_cast<u32x4*>(dst + (r0 + j * (NT / KV)) * SK + 8 * kv) = q;
    }
  };

  int t = first_tile(ntiles);
  bf16x8 bw[KS];
  {
    u32x4 st[LV];
    load_tile(t, st);
    // this lane's B fragments, W[col][16s + 8h + j] RNE to bf16 (after the first tile's loads, so the
    // first tile's MFMAs wait for each in turn)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float* wp = a.w + (size_t)col * KR + 16 * s + 8 * h;
      bw[s] = __builtin_bit_cast(bf16x8, pack8(ld4(wp), ld4(wp + 4)));
    }
    stage(&As[0][0], st);
  }
  __syncthreads();
  double ps = 0.0, pq = 0.0;
  int buf = 0;
  for (; t < ntiles; t += G) {
    u32x4 nst[LV];
    load_tile(t + G, nst);
    f32x16 acc;
    mfma_tile<KS>(&As[buf][0] + l32 * SK + 8 * h, bw, acc);
    const int mb = t * TR + 4 * h;
    const __amdgpu_buffer_rsrc_t ry = make_rsrc_v(a.y + (size_t)t * TR * N, a.M - t * TR > 0 ? (uint32_t)(a.M - t * TR) * N * 2u : 0u);
    const bool full = t * TR + TR <= a.M;  // (uniform)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float v = acc[r];
      if constexpr (HB) v += bias;
      const uint16_t bits = bf16_bits(v);
      bstore_nt(bits, ry, (int)(eofs0 + (uint32_t)(((r & 3) + 8 * (r >> 2)) * N) * 2u), 0, a.nt);
      if constexpr (STATS) {
        const int dm = (r & 3) + 8 * (r >> 2);
        const double d = (full || mb + dm < a.M) ? (double)bf16_val(bits) : 0.0;
        ps += d;
        pq += d * d;
      }
    }
    stage(&As[buf ^ 1][0], nst);
    __syncthreads();
    buf ^= 1;
  }
  if constexpr (STATS) partial_row(ps, pq, a.part, N, n0, a.ft, &As[0][0]);
}

// BN-backward-on-load dgrad: dy = the following BN's backward of (g, xo) in fp32, RNE to bf16 (the
// MFMA operand, and written through by column group 0 for the weight gradient); dx = dy . W
// (+ residual) stored bf16; the input BN's backward partials over the stored dx.
struct DgradArgs {
  const bf16_t* g;    // [M][KR]
  const bf16_t* xo;   // [M][KR]
  bf16_t* dy_out;     // [M][KR] nullable
  const float* w;     // [KR][N]
  bf16_t* dx;         // [M][N]
  const bf16_t* res;  // [M][N] nullable
  const bf16_t* xi;   // [M][N] nullable (partials)
  const float *om, *ois, *og, *ob, *k12;
  int orelu;
  const float *im, *iis, *ig, *ib;
  int irelu;
  double* part;
  int M, N;
  FoldTail ft;
  int nt;             // nontemporal output stores (nt_stores(kNtPwd16))
};

template <int KR, bool RES, bool PART>
__global__ __launch_bounds__(NT, dgrad_wps<KR>()) void dgrad_kernel(DgradArgs a) {
  constexpr int SK = KR + 8, KV = KR / 8, LV = TR * KV / NT, KS = KR / 16;
  static_assert(KR % 64 == 0 && NT % KV == 0 && LV >= 1, "pwd16::dgrad_kernel shape");
  __shared__ __attribute__((aligned(16))) bf16_t As[2][TR * SK];
  static_assert(sizeof(double) * 2 * NT <= sizeof(bf16_t) * 2 * TR * SK, "fold scratch fits in the tiles");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * NB, N = a.N, col = n0 + 32 * wave + l32;
  const int kv = tid % KV, r0 = tid / KV;
  // the following BN's terms [7][KR] (mean, invstd, gamma, beta, k1, k2, gamma * invstd), read by
  // each thread for its 8 channels once per tile
  __shared__ __attribute__((aligned(16))) float tab[7 * KR];
  for (int c = tid; c < KR; c += NT) {
    const float is = a.ois[c], ga = a.og[c];
    tab[c] = a.om[c];
    tab[KR + c] = is;
    tab[2 * KR + c] = ga;
    tab[3 * KR + c] = a.ob[c];
    tab[4 * KR + c] = a.k12[c];
    tab[5 * KR + c] = a.k12[KR + c];
    tab[6 * KR + c] = ga * is;
  }
  __syncthreads();
  const float pm = PART ? a.im[col] : 0.f, pis = PART ? a.iis[col] : 0.f, pga = PART ? a.ig[col] : 0.f,
              pbe = PART ? a.ib[col] : 0.f;
  const bool orelu = a.orelu != 0, irelu = a.irelu != 0;
  const bool writer = a.dy_out != nullptr && blockIdx.y == 0;
  const int ntiles = (a.M + TR - 1) / TR, G = gridDim.x;
  const uint32_t lofs0 = ((uint32_t)r0 * KR + 8 * kv) * 2u, eofs0 = ((uint32_t)(4 * h) * N + col) * 2u;
  constexpr uint32_t kLStep = (uint32_t)(NT / KV) * KR * 2u;
  auto eofs = [&](int r) { return (int)(eofs0 + (uint32_t)(((r & 3) + 8 * (r >> 2)) * N) * 2u); };

  auto load_tile = [&](int tile, u32x4* sg, u32x4* sx) {
    const __amdgpu_buffer_rsrc_t rg = tile_rsrc(a.g, KR, tile, a.M), rx = tile_rsrc(a.xo, KR, tile, a.M);
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      sg[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)(lofs0 + j * kLStep), 0, 0));
      sx[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(lofs0 + j * kLStep), 0, 0));
    }
  };
  auto stage = [&](int tile, bf16_t* dst, const u32x4* sg, const u32x4* sx) {
    const __amdgpu_buffer_rsrc_t rdy = tile_rsrc(writer ? a.dy_out : a.g, KR, tile, writer ? a.M : 0);
    f32x4 mu[2], is[2], ga[2], be[2], k1[2], k2[2], f[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const float* tp = tab + 8 * kv + 4 * p;
      mu[p] = *reinterpret_cast<const f32x4*>(tp);
      is[p] = *reinterpret_cast<const f32x4*>(tp + KR);
      ga[p] = *reinterpret_cast<const f32x4*>(tp + 2 * KR);
      be[p] = *reinterpret_cast<const f32x4*>(tp + 3 * KR);
      k1[p] = *reinterpret_cast<const f32x4*>(tp + 4 * KR);
      k2[p] = *reinterpret_cast<const f32x4*>(tp + 5 * KR);
      f[p] = *reinterpret_cast<const f32x4*>(tp + 6 * KR);
    }
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      f32x4 gv[2], xv[2];
      unpack8(sg[j], gv[0], gv[1]);
      unpack8(sx[j], xv[0], xv[1]);
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xe = xv[p][e];
          float ge = gv[p][e];
          const bool kill = (!(bn_out(xe, mu[p][e], is[p][e], ga[p][e], be[p][e]) > 0.f)) & orelu;
          ge = kill ? 0.f : ge;
          gv[p][e] = bn_bwd_elem(xe, ge, mu[p][e], is[p][e], f[p][e], k1[p][e], k2[p][e]);
        }
      const u32x4 q = pack8(gv[0], gv[1]);
      *reinterpret_cast<u32x4*>(dst + (r0 + j * (NT / KV)) * SK + 8 * kv) = q;
      bstore_nt(q, rdy, (int)(lofs0 + j * kLStep), 0, a.nt);
    }
  };

  int t = first_tile(ntiles);
  bf16x8 bw[KS];
  {
    u32x4 sg[LV], sx[LV];
    load_tile(t, sg, sx);
    // B fragments W[16s + 8h + j][col] RNE to bf16
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      f32x4 lo, hi;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        lo[e] = a.w[(size_t)(16 * s + 8 * h + e) * N + col];
        hi[e] = a.w[(size_t)(16 * s + 8 * h + 4 + e) * N + col];
      }
      bw[s] = __builtin_bit_cast(bf16x8, pack8(lo, hi));
    }
    stage(t, &As[0][0], sg, sx);
  }
  __syncthreads();
  double ps = 0.0, pq = 0.0;
  int buf = 0;
  for (; t < ntiles; t += G) {
    u32x4 ng[LV], nx[LV];
    load_tile(t + G, ng, nx);
    const int mb = t * TR + 4 * h;
    const int rows = a.M - t * TR;
    const uint32_t nb = rows > 0 ? (uint32_t)rows * N * 2u : 0u;
    const __amdgpu_buffer_rsrc_t rxi = make_rsrc_v(PART ? a.xi + (size_t)t * TR * N : a.g, PART ? nb : 0u);
    const __amdgpu_buffer_rsrc_t rr = make_rsrc_v(RES ? a.res + (size_t)t * TR * N : a.g, RES ? nb : 0u);
    const __amdgpu_buffer_rsrc_t rdx = make_rsrc_v(a.dx + (size_t)t * TR * N, nb);
    uint32_t exi[16], ers[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if constexpr (PART) exi[r] = __builtin_amdgcn_raw_buffer_load_b16(rxi, eofs(r), 0, 0);
      if constexpr (RES) ers[r] = __builtin_amdgcn_raw_buffer_load_b16(rr, eofs(r), 0, 0);
    }
    f32x16 acc;
    mfma_tile<KS>(&As[buf][0] + l32 * SK + 8 * h, bw, acc);
    const bool full = t * TR + TR <= a.M;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float v = acc[r];
      if constexpr (RES) v += bf16_val(ers[r]);
      const uint16_t bits = bf16_bits(v);
      bstore_nt(bits, rdx, eofs(r), 0, a.nt);
      if constexpr (PART) {
        const int dm = (r & 3) + 8 * (r >> 2);
        const float gs = bf16_val(bits), x = bf16_val(exi[r]);
        const float xh = (x - pm) * pis;
        const bool kill = ((!(bn_out(x, pm, pis, pga, pbe) > 0.f)) & irelu) | (!full && mb + dm >= a.M);
        const float g2 = kill ? 0.f : gs;
        ps += (double)g2;
        pq += (double)g2 * (double)xh;
      }
    }
    stage(t + G, &As[buf ^ 1][0], ng, nx);
    __syncthreads();
    buf ^= 1;
  }
  if constexpr (PART) partial_row(ps, pq, a.part, N, n0, a.ft, &As[0][0]);
}


// ---------------------------------------------------------------------------------------
// Fused backward (bf16 storage, K in {128, 256}): the dgrad above plus the weight gradient
//   dW[k][c] = sum_m dy[m][k] * bn_relu(x)[m][c]   (layers/pointwise_convolution.py:61-64)
// in the same pass, dy never stored (pw_deep.hip's bwd_kernel on v_mfma_f32_32x32x16_bf16).  Per
// 32-pixel tile a wave, after its dgrad MFMAs and dx stores:
//   * forms the B operand bn_relu(x) of its 32 columns from the epilogue's C-layout x loads
//     (registers 8s .. 8s + 7 of lane half h = pixels 16s + 8(j >> 2) + 4h + (j & 3)), rounded to
//     bf16 as the tiled engine's BN-on-load loader does, zero past M;
//   * reads the A operand dy^T (rows = channels, k-step = those 16 pixels) from the block's LDS dy
//     tile with ds_read_b64_tr_b16 and accumulates its [KR][32] block of dW in registers.
// dx and the input BN's partials are bit-identical to dgrad_kernel's; dW regroups the sum over
// pixels.  Each wave stores its dW block into the partial row wpart[blockIdx.x][KR][N] at the end.
// ---------------------------------------------------------------------------------------
template <int KR>
constexpr int bwd_wps() {
  return KR <= 128 ? 2 : 1;
}

template <int KR, bool RES, bool BNIN>
__global__ __launch_bounds__(NT, bwd_wps<KR>()) void bwd_kernel(DgradArgs a, float* wpart) {
  constexpr int SK = KR + 8, KV = KR / 8, LV = TR * KV / NT, KS = KR / 16, KT = KR / 32;
  static_assert(KR % 64 == 0 && NT % KV == 0 && LV >= 1, "pwd16::bwd_kernel shape");
  __shared__ __attribute__((aligned(16))) bf16_t As[2][TR * SK];
  static_assert(sizeof(double) * 2 * NT <= sizeof(bf16_t) * 2 * TR * SK, "fold scratch fits in the tiles");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * NB, N = a.N, col = n0 + 32 * wave + l32;
  // C = 64: one column group of 64, waves 2 and 3 only stage the dy tiles (wave-uniform)
  const bool wact = n0 + 32 * wave < N;
  const int kv = tid % KV, r0 = tid / KV;
  __shared__ __attribute__((aligned(16))) float tab[7 * KR];
  for (int c = tid; c < KR; c += NT) {
    const float is = a.ois[c], ga = a.og[c];
    tab[c] = a.om[c];
    tab[KR + c] = is;
    tab[2 * KR + c] = ga;
    tab[3 * KR + c] = a.ob[c];
    tab[4 * KR + c] = a.k12[c];
    tab[5 * KR + c] = a.k12[KR + c];
    tab[6 * KR + c] = ga * is;
  }
  __syncthreads();
  const float pm = BNIN && wact ? a.im[col] : 0.f, pis = BNIN && wact ? a.iis[col] : 0.f,
              pga = BNIN && wact ? a.ig[col] : 0.f, pbe = BNIN && wact ? a.ib[col] : 0.f;
  const bool orelu = a.orelu != 0, irelu = a.irelu != 0;
  const int ntiles = (a.M + TR - 1) / TR, G = gridDim.x;
  const uint32_t lofs0 = ((uint32_t)r0 * KR + 8 * kv) * 2u, eofs0 = ((uint32_t)(4 * h) * N + col) * 2u;
  constexpr uint32_t kLStep = (uint32_t)(NT / KV) * KR * 2u;
  auto eofs = [&](int r) { return (int)(eofs0 + (uint32_t)(((r & 3) + 8 * (r >> 2)) * N) * 2u); };

  auto load_tile = [&](int tile, u32x4* sg, u32x4* sx) {
    const __amdgpu_buffer_rsrc_t rg = tile_rsrc(a.g, KR, tile, a.M), rx = tile_rsrc(a.xo, KR, tile, a.M);
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      sg[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)(lofs0 + j * kLStep), 0, 0));
      sx[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(lofs0 + j * kLStep), 0, 0));
    }
  };
  auto stage = [&](bf16_t* dst, const u32x4* sg, const u32x4* sx) {
    f32x4 mu[2], is[2], ga[2], be[2], k1[2], k2[2], f[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const float* tp = tab + 8 * kv + 4 * p;
      mu[p] = *reinterpret_cast<const f32x4*>(tp);
      is[p] = *reinterpret_cast<const f32x4*>(tp + KR);
      ga[p] = *reinterpret_cast<const f32x4*>(tp + 2 * KR);
      be[p] = *reinterpret_cast<const f32x4*>(tp + 3 * KR);
      k1[p] = *reinterpret_cast<const f32x4*>(tp + 4 * KR);
      k2[p] = *reinterpret_cast<const f32x4*>(tp + 5 * KR);
      f[p] = *reinterpret_cast<const f32x4*>(tp + 6 * KR);
    }
#pragma unroll
    for (int j = 0; j < LV; ++j) {
      f32x4 gv[2], xv[2];
      unpack8(sg[j], gv[0], gv[1]);
      unpack8(sx[j], xv[0], xv[1]);
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xe = xv[p][e];
          float ge = gv[p][e];
          const bool kill = (!(bn_out(xe, mu[p][e], is[p][e], ga[p][e], be[p][e]) > 0.f)) & orelu;
          ge = kill ? 0.f : ge;
          gv[p][e] = bn_bwd_elem(xe, ge, mu[p][e], is[p][e], f[p][e], k1[p][e], k2[p][e]);
        }
      *reinterpret_cast<u32x4*>(dst + (r0 + j * (NT / KV)) * SK + 8 * kv) = pack8(gv[0], gv[1]);
    }
  };

  int t = first_tile(ntiles);
  bf16x8 bw[KS];
  {
    u32x4 sg[LV], sx[LV];
    load_tile(t, sg, sx);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      f32x4 lo, hi;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        lo[e] = wact ? a.w[(size_t)(16 * s + 8 * h + e) * N + col] : 0.f;
        hi[e] = wact ? a.w[(size_t)(16 * s + 8 * h + 4 + e) * N + col] : 0.f;
      }
      bw[s] = __builtin_bit_cast(bf16x8, pack8(lo, hi));
    }
    stage(&As[0][0], sg, sx);
  }
  __syncthreads();
  f32x16 dwa[KT];
#pragma unroll
  for (int i = 0; i < KT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) dwa[i][r] = 0.f;
  double ps = 0.0, pq = 0.0;
  int buf = 0;
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  for (; t < ntiles; t += G) {
    u32x4 ng[LV], nx[LV];
    load_tile(t + G, ng, nx);
    if (wact) {
    const int mb = t * TR + 4 * h;
    const int rows = a.M - t * TR;
    const uint32_t nb = rows > 0 ? (uint32_t)rows * N * 2u : 0u;
    const __amdgpu_buffer_rsrc_t rxi = make_rsrc_v(a.xi + (size_t)t * TR * N, nb);
    const __amdgpu_buffer_rsrc_t rr = make_rsrc_v(RES ? a.res + (size_t)t * TR * N : a.g, RES ? nb : 0u);
    const __amdgpu_buffer_rsrc_t rdx = make_rsrc_v(a.dx + (size_t)t * TR * N, nb);
    uint32_t exi[16], ers[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      exi[r] = __builtin_amdgcn_raw_buffer_load_b16(rxi, eofs(r), 0, 0);
      if constexpr (RES) ers[r] = __builtin_amdgcn_raw_buffer_load_b16(rr, eofs(r), 0, 0);
    }
    const bf16_t* tile = &As[buf][0];
    f32x16 acc;
    mfma_tile<KS>(tile + l32 * SK + 8 * h, bw, acc);
    const bool full = t * TR + TR <= a.M;
    float xb[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int dm = (r & 3) + 8 * (r >> 2);
      float v = acc[r];
      if constexpr (RES) v += bf16_val(ers[r]);
      const uint16_t bits = bf16_bits(v);
      bstore_nt(bits, rdx, eofs(r), 0, a.nt);
      const bool out = !full && mb + dm >= a.M;
      const float x = bf16_val(exi[r]);
      if constexpr (BNIN) {
        const float xh = (x - pm) * pis;
        const float bo = bn_out(x, pm, pis, pga, pbe);
        const bool dead = (!(bo > 0.f)) & irelu;
        const float g2 = (dead | out) ? 0.f : bf16_val(bits);
        ps += (double)g2;
        pq += (double)g2 * (double)xh;
        xb[r] = (dead | out) ? 0.f : bo;
      } else {
        xb[r] = out ? 0.f : x;
      }
    }
    // dW[k][col] += dy^T . bf16(bn_relu(x)) over the tile's 32 pixels, two k-steps of 16
    {
      const int i = lane & 15, g = (lane >> 4) & 1;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 bx = __builtin_bit_cast(
            bf16x8, pack8(f32x4{xb[8 * s2], xb[8 * s2 + 1], xb[8 * s2 + 2], xb[8 * s2 + 3]},
                          f32x4{xb[8 * s2 + 4], xb[8 * s2 + 5], xb[8 * s2 + 6], xb[8 * s2 + 7]}));
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
          const bf16_t* p = tile + (16 * s2 + 4 * h + (i >> 2)) * SK + 32 * kt + 16 * g + 4 * (i & 3);
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 8 * SK));
          const bf16x8 dyt = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          dwa[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dyt, bx, dwa[kt], 0, 0, 0);
        }
      }
    }
    }  // wact
    stage(&As[buf ^ 1][0], ng, nx);
    __syncthreads();
    buf ^= 1;
  }
  // this wave's dW block: element (kt, r) = dW[32 kt + (r & 3) + 8 (r >> 2) + 4h][col]
  if (wact) {
    float* wp = wpart + (size_t)blockIdx.x * KR * N + col;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) wp[(size_t)(32 * kt + (r & 3) + 8 * (r >> 2) + 4 * h) * N] = dwa[kt][r];
  }
  if constexpr (BNIN) partial_row(ps, pq, a.part, N, n0, a.ft, &As[0][0]);
}

// ---------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------
#define DK_PWD16_KR(X) X(128) X(256) X(512)

static int occupancy(const void* fn) {
  int v = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, fn, NT, 0) != hipSuccess || v < 1) v = 1;
  return v;
}
template <int KR>
static int fwd_occ() {
  static const int occ = [] {
#define DK_F(B_, S_) reinterpret_cast<const void*>(&fwd_kernel<KR, B_, S_, false>), \
                     reinterpret_cast<const void*>(&fwd_kernel<KR, B_, S_, true>)
    const void* fs[] = {DK_F(true, true), DK_F(true, false), DK_F(false, true), DK_F(false, false)};
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
// Row-tile walkers per column group (pw_deep.hip's grid_x): every resident slot once, at most one
// per tile, a multiple of 8 when that costs no extra tile per walker.
static int grid_x(int M, int N, int occ) {
  const int ntiles = (M + TR - 1) / TR;
  int slots = occ * 256 / (N < NB ? 1 : N / NB);  // (N < NB: the C = 64 fused backward, one column group)
  if (slots < 1) slots = 1;
  int gx = std::min(ntiles, slots);
  const int g8 = gx / 8 * 8;
  if (g8 >= 8 && (ntiles + g8 - 1) / g8 == (ntiles + gx - 1) / gx) gx = g8;
  return gx;
}

}  // namespace pwd16

// Knob 13 = 0 keeps the tiled engine's bf16 mode for the deep shapes.
static bool pwd16_enabled() { return knob(kKnobPwDeep16) == 1; }
static bool pwd16_kr(int KR) { return KR == 128 || KR == 256 || KR == 512; }

// The deep shapes: reduction 128 / 256 / 512, outputs a multiple of 128 columns, 256+ channels on
// one side when the reduction is 128.
bool pw_deep16_fwd_ok(int K, int C, int M) {
  if (!pwd16_enabled() || M <= 0 || !pwd16_kr(C) || K % pwd16::NB || K > 4096 || (C < 256 && K < 256)) return false;
  return (size_t)M * (K > C ? K : C) * 2 < ((size_t)1 << 31);
}
bool pw_deep16_dgrad_ok(int K, int C, int M) {
  if (!pwd16_enabled() || M <= 0 || !pwd16_kr(K) || C % pwd16::NB || C > 4096 || (K < 256 && C < 256)) return false;
  return (size_t)M * (K > C ? K : C) * 2 < ((size_t)1 << 31);
}
int pw_deep16_fwd_rows(int M, int K, int C) {
#define DK_ROWS(kr) \
  if (C == kr) return pwd16::grid_x(M, K, pwd16::fwd_occ<kr>());
  DK_PWD16_KR(DK_ROWS)
#undef DK_ROWS
  return 0;
}
int pw_deep16_dgrad_rows(int M, int K, int C) {
#define DK_ROWS(kr) \
  if (K == kr) return pwd16::grid_x(M, C, pwd16::dgrad_occ<kr>());
  DK_PWD16_KR(DK_ROWS)
#undef DK_ROWS
  return 0;
}

int pw_deep16_fwd(const bf16_t* x, int M, const float* w, int K, int C, const float* bias, bf16_t* y, const float* im,
                  const float* iis, const float* ig, const float* ib, int irelu, double* part, hipStream_t st,
                  const FoldTail* ft) {
  pwd16::FwdArgs a{x, w, bias, y, im, iis, ig, ib, irelu, part, M, K};
  if (ft && part) a.ft = *ft;
  a.nt = nt_stores(kNtPwd16);
  const dim3 grid(pw_deep16_fwd_rows(M, K, C), K / pwd16::NB);
  if (grid.x == 0) return DK_ERR_ARGS;
#define DK_L(kr, B_, S_)                                                                          \
  do {                                                                                            \
    if (bias)                                                                                     \
      hipLaunchKernelGGL((pwd16::fwd_kernel<kr, B_, S_, true>), grid, dim3(pwd16::NT), 0, st, a);  \
    else                                                                                          \
      hipLaunchKernelGGL((pwd16::fwd_kernel<kr, B_, S_, false>), grid, dim3(pwd16::NT), 0, st, a); \
  } while (0)
#define DK_FWD(kr)               \
  if (C == kr) {                 \
    if (im && part)              \
      DK_L(kr, true, true);      \
    else if (im)                 \
      DK_L(kr, true, false);     \
    else if (part)               \
      DK_L(kr, false, true);     \
    else                         \
      DK_L(kr, false, false);    \
    return launch_status();      \
  }
  DK_PWD16_KR(DK_FWD)
#undef DK_FWD
#undef DK_L
  return DK_ERR_ARGS;
}

int pw_deep16_dgrad_bnbwd(const bf16_t* g, const bf16_t* bn_x, int M, int K, int C, const float* om, const float* ois,
                          const float* og, const float* ob, int orelu, const float* k12, bf16_t* dy_out, const float* w,
                          bf16_t* dx, const bf16_t* res, const bf16_t* x, const float* im, const float* iis,
                          const float* ig, const float* ib, int irelu, double* part, hipStream_t st,
                          const FoldTail* ft) {
  pwd16::DgradArgs a{g, bn_x, dy_out, w, dx, res, x, om, ois, og, ob, k12, orelu, im, iis, ig, ib, irelu, part, M, C};
  if (ft && part) a.ft = *ft;
  a.nt = nt_stores(kNtPwd16);
  const dim3 grid(pw_deep16_dgrad_rows(M, K, C), C / pwd16::NB);
  if (grid.x == 0) return DK_ERR_ARGS;
#define DK_L(kr, R_, P_) hipLaunchKernelGGL((pwd16::dgrad_kernel<kr, R_, P_>), grid, dim3(pwd16::NT), 0, st, a)
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
  DK_PWD16_KR(DK_DG)
#undef DK_DG
#undef DK_L
  return DK_ERR_ARGS;
}

template <int KR>
static int bwd_occ16() {
  static const int occ = [] {
    const void* fs[] = {reinterpret_cast<const void*>(&pwd16::bwd_kernel<KR, true, true>),
                        reinterpret_cast<const void*>(&pwd16::bwd_kernel<KR, true, false>),
                        reinterpret_cast<const void*>(&pwd16::bwd_kernel<KR, false, true>),
                        reinterpret_cast<const void*>(&pwd16::bwd_kernel<KR, false, false>)};
    int o = 1 << 20;
    for (const void* f : fs) o = std::min(o, pwd16::occupancy(f));
    return o;
  }();
  return occ;
}
// The fused bf16 backward: K in {128, 256}, C a multiple of the block's 128 columns, or K = 128 with
// C = 64 (one column group, half the block's waves staging only: config 5's 64 -> 128 unit, whose
// unfused pair stored dy for a side-stream weight GEMM).
bool pw_deep16_bwd_ok(int K, int C, int M) {
  if (!pwd16_enabled() || M <= 0 || (K != 128 && K != 256) || (C % pwd16::NB && !(K == 128 && C == 64)) ||
      C > 4096)
    return false;
  return (size_t)M * (K > C ? K : C) * 2 < ((size_t)1 << 31);
}
int pw_deep16_bwd_rows(int M, int K, int C) {
  if (K == 128) return pwd16::grid_x(M, C, bwd_occ16<128>());
  if (K == 256) return pwd16::grid_x(M, C, bwd_occ16<256>());
  return 0;
}
int pw_deep16_bwd_slices(int M, int K, int C) { return C < pwd16::NB ? 1 : C / pwd16::NB; }
int pw_deep16_bwd_fused(const bf16_t* g, const bf16_t* bn_x, int M, int K, int C, const float* om, const float* ois,
                        const float* og, const float* ob, int orelu, const float* k12, const float* w, bf16_t* dx,
                        const bf16_t* res, const bf16_t* x, const float* im, const float* iis, const float* ig,
                        const float* ib, int irelu, double* part, float* wpart, hipStream_t st, const FoldTail* ft) {
  if (!x || (im != nullptr) != (part != nullptr)) return DK_ERR_ARGS;
  pwd16::DgradArgs a{g, bn_x, nullptr, w, dx, res, x, om, ois, og, ob, k12, orelu, im, iis, ig, ib, irelu, part, M, C};
  if (ft && part) a.ft = *ft;
  a.nt = nt_stores(kNtPwd16);
  const dim3 grid(pw_deep16_bwd_rows(M, K, C), pw_deep16_bwd_slices(M, K, C));
  if (grid.x == 0) return DK_ERR_ARGS;
#define DK_L(kr, R_, B_) hipLaunchKernelGGL((pwd16::bwd_kernel<kr, R_, B_>), grid, dim3(pwd16::NT), 0, st, a, wpart)
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
  DK_BW(256)
#undef DK_BW
#undef DK_L
  return DK_ERR_ARGS;
}

}  // namespace dk
