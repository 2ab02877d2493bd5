// Streaming pointwise kernels for BASELINE config 5's bf16 storage (the MobileNet-style stack at
// batch 512): the forward and the BN-backward-on-load dgrad of the memory-bound 1x1 shapes with
// K, C in {64, 128} (the 56 x 56 and 28 x 28 units: 1.6 M and 0.4 M pixels), on
// v_mfma_f32_32x32x16_bf16.  The same structure as pw_stream.hip's fp32 kernels:
//
//   * persistent waves stream 32-pixel row tiles (tile t, t + W, ... with W = all waves);
//   * the pixel operand goes global -> registers directly: lane (l32, h) loads row l32's 8
//     channels 16s + 8h .. +7 -- one 16-byte load, exactly its bf16x8 MFMA fragment of k-step s;
//   * the weights are staged once per block into LDS as bf16 ([n][k], row stride K + 8 elements:
//     an odd multiple of 16 bytes, conflict-free ds_read_b128);
//   * the next tile's operand loads are in flight while the current tile's MFMAs run;
//   * the epilogue works in the MFMA C layout (lane = output column), so the BatchNorm partial
//     sums stay in registers across the wave's tiles: one partial row per block.
//
// Bit-identical to the tiled engine's bf16 mode (gemm_engine.h, kMfBf16): the same operand
// rounding (fp32 BN transform, then RNE to bf16), the same MFMA sequence over k (k-steps of 16
// in ascending order, k = 16s + 8h + j on both operands), the same fp32 epilogue, RNE stores, and
// statistics over the stored (rounded) values.  Only the grouping of the fp64 partial sums
// differs (one row per block instead of one per 64-pixel tile).
#include "dk_common.h"
#include "fold_tail.h"

namespace dk {
namespace pwsh {

constexpr int WAVES = 4;  // waves per block
constexpr int TR = 32;    // pixels per wave tile
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void drain_vmem_loads() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// 8 bf16 (a 16-byte load) <-> 8 floats (exact widening; RNE narrowing, v_cvt_pk_bf16_f32)
__device__ __forceinline__ void unpack8(u32x4 u, f32x4& lo, f32x4& hi) {
  lo = bf16x4_to_f32(uint2{u[0], u[1]});
  hi = bf16x4_to_f32(uint2{u[2], u[3]});
}
__device__ __forceinline__ u32x4 pack8(f32x4 lo, f32x4 hi) {
  const uint2 a = f32_to_bf16x4(lo), b = f32_to_bf16x4(hi);
  return u32x4{a.x, a.y, b.x, b.y};
}
__device__ __forceinline__ bf16x8 frag(u32x4 u) { return __builtin_bit_cast(bf16x8, u); }
__device__ __forceinline__ uint16_t bf16_bits(float v) { return __builtin_bit_cast(uint16_t, (__bf16)v); }

// Resident blocks per CU of a family of instantiations (the smallest).
static int min_occupancy(const void* const* fs, int n, int threads = 256) {
  int o = 1 << 20;
  for (int i = 0; i < n; ++i) {
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, fs[i], threads, 0) != hipSuccess || v < 1) v = 1;
    o = v < o ? v : o;
  }
  return o;
}
// A persistent grid: every resident slot once, at most one block per 4 tiles; a function of M and
// the (fixed) occupancy only, so callers allocate exactly the partial rows the launch writes.
static int grid_blocks(int M, int occ) {
  const int ntiles = (M + TR - 1) / TR;
  const int want = (ntiles + WAVES - 1) / WAVES;
  const int slots = occ * 256;
  return want < slots ? (want > 0 ? want : 1) : slots;
}

// ---------------------------------------------------------------------------------------
// Forward (layers/pointwise_convolution.py:46-55): y = bn(x) . W^T with the preceding BatchNorm
// (+ReLU) applied on load and the following BatchNorm's statistics of the stored y.
// ---------------------------------------------------------------------------------------
struct FwdArgs {
  const bf16_t* x;    // [M][KR]
  const float* w;     // [NO][KR] (W[k][c]: k = output channel)
  const float* bias;  // [NO] nullable
  bf16_t* y;          // [M][NO]
  const float* im;    // input BN (im == nullptr: none)
  const float* iis;
  const float* ig;
  const float* ib;
  int irelu;
  double* part;       // [gridDim.x][2][NO] nullable
  int M;
  FoldTail ft;
};

template <int KR, int NO, bool BN, bool STATS>
__global__ __launch_bounds__(256, 2) void fwd_kernel(FwdArgs a) {
  constexpr int SKB = KR + 8, KS = KR / 16, NU = NO / 32;
  __shared__ __attribute__((aligned(16))) bf16_t Bs[NO * SKB];
  __shared__ __attribute__((aligned(16))) float tab[4][KR];
  __shared__ double red[WAVES][2][NO];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  for (int i = tid; i < KR * NO / 4; i += 256) {  // 4 k at a time
    const int n = i / (KR / 4), k = 4 * (i - n * (KR / 4));
    *reinterpret_cast<uint2*>(Bs + n * SKB + k) = f32_to_bf16x4(ld4(a.w + (size_t)n * KR + k));
  }
  if constexpr (BN) {
    for (int c = tid; c < KR; c += 256) {
      tab[0][c] = a.im[c];
      tab[1][c] = a.iis[c];
      tab[2][c] = a.ig[c];
      tab[3][c] = a.ib[c];
    }
  }
  float bias[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) bias[u] = a.bias ? a.bias[32 * u + l32] : 0.f;
  const bool irelu = a.irelu != 0;
  __syncthreads();

  const __amdgpu_buffer_rsrc_t rx = make_rsrc_v(a.x, (uint32_t)a.M * KR * 2u);
  const __amdgpu_buffer_rsrc_t ry = make_rsrc_v(a.y, (uint32_t)a.M * NO * 2u);
  const int ntiles = (a.M + TR - 1) / TR;
  const int W = gridDim.x * WAVES;
  int t = blockIdx.x * WAVES + wave;
  double ps[NU], pq[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) ps[u] = pq[u] = 0.0;

  // rows past M (the ragged last tile, the prefetch past the end) read zeros
  auto load_x = [&](int tile, u32x4* lx) {
    const uint32_t base = ((uint32_t)(tile * TR + l32) * KR + 8 * h) * 2u;
#pragma unroll
    for (int s = 0; s < KS; ++s)
      lx[s] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(base + 32u * s), 0, 0));
  };
  u32x4 cx[KS];
  load_x(t, cx);
  drain_vmem_loads();
  for (; t < ntiles; t += W) {
    const int m0 = t * TR;
    int z = 0;
    asm volatile("" : "+s"(z));  // keeps the LDS table / weight reads in the loop (see pw_stream.hip)
    const float* tb = &tab[0][0] + z;
    const bf16_t* bs = Bs + z;
    u32x4 nx[KS];
    load_x(t + W, nx);
    __builtin_amdgcn_sched_barrier(0);

    bf16x8 af[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if constexpr (BN) {
        f32x4 v[2];
        unpack8(cx[s], v[0], v[1]);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int c0 = 16 * s + 8 * h + 4 * p;
          const f32x4 mu = ld4(tb + 0 * KR + c0), is = ld4(tb + 1 * KR + c0), ga = ld4(tb + 2 * KR + c0),
                      be = ld4(tb + 3 * KR + c0);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float r = bn_out(v[p][e], mu[e], is[e], ga[e], be[e]);
            v[p][e] = (irelu & !(r > 0.f)) ? 0.f : r;
          }
        }
        af[s] = frag(pack8(v[0], v[1]));
      } else {
        af[s] = frag(cx[s]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);

    f32x16 acc[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const bf16x8 bf = *reinterpret_cast<const bf16x8*>(bs + (32 * u + l32) * SKB + 16 * s + 8 * h);
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bf, acc[u], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);

    // C layout: lane (l32, h) holds column 32u + l32 of rows (r & 3) + 8 (r >> 2) + 4h
    const int mb = m0 + 4 * h;
    const uint32_t eb = ((uint32_t)mb * NO + l32) * 2u;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dm = (r & 3) + 8 * (r >> 2);
        float v = acc[u][r];
        if (a.bias) v += bias[u];
        const uint16_t bits = bf16_bits(v);
        __builtin_amdgcn_raw_buffer_store_b16(bits, ry, (int)(eb + (uint32_t)(dm * NO + 32 * u) * 2u), 0, 0);
        if constexpr (STATS) {
          const double d = (mb + dm < a.M) ? (double)__builtin_bit_cast(float, (uint32_t)bits << 16) : 0.0;
          ps[u] += d;
          pq[u] += d * d;
        }
      }
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) cx[s] = nx[s];
  }
  if constexpr (!STATS) return;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    ps[u] += __shfl_xor(ps[u], 32, 64);
    pq[u] += __shfl_xor(pq[u], 32, 64);
    if (h == 0) {
      red[wave][0][32 * u + l32] = ps[u];
      red[wave][1][32 * u + l32] = pq[u];
    }
  }
  __syncthreads();
  for (int i = tid; i < 2 * NO; i += 256) {
    const int which = i / NO, c = i - which * NO;
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) s += red[w][which][c];
    pub_store(a.part + ((size_t)blockIdx.x * 2 + which) * NO + c, s);
  }
  if (a.ft.part) fold_tail<256>(a.ft, blockIdx.x, 0, NO, 0);
}

// ---------------------------------------------------------------------------------------
// BN-backward-on-load dgrad (layers/pointwise_convolution.py:57-75 + batch_norm.py:125-174):
// dy = the following BatchNorm's backward of (g, x_out) formed on load in fp32 (bn_bwd_elem),
// rounded to bf16 as the MFMA operand and as written through for the weight gradient;
// dx = dy . W (+ residual) stored bf16, and the input BatchNorm's backward partial sums of the
// stored dx.  KR = the layer's output channels K (the reduction), NO = its input channels C.
// ---------------------------------------------------------------------------------------
struct DgradArgs {
  const bf16_t* g;    // [M][KR]
  const bf16_t* xo;   // [M][KR] the following BN's raw input
  bf16_t* dy_out;     // [M][KR] nullable
  const float* w;     // [KR][NO]
  bf16_t* dx;         // [M][NO]
  const bf16_t* res;  // [M][NO] nullable
  const bf16_t* xi;   // [M][NO] the input BN's raw input (nullable: no partials)
  const float *om, *ois, *og, *ob, *k12;
  int orelu;
  const float *im, *iis, *ig, *ib;
  int irelu;
  double* part;       // [gridDim.x][2][NO]
  int M;
  FoldTail ft;
};

template <int KR, int NO, bool RES, bool PART>
__global__ __launch_bounds__(256, 2) void dgrad_bnbwd_kernel(DgradArgs a) {
  constexpr int SKB = KR + 8, KS = KR / 16, NU = NO / 32;
  __shared__ __attribute__((aligned(16))) bf16_t Bs[NO * SKB];  // Bs[c][k] = W[k][c]
  __shared__ __attribute__((aligned(16))) float tab[7][KR];
  __shared__ double red[WAVES][2][NO];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  for (int i = tid; i < KR * NO / 16; i += 256) {  // 4 k x 4 c blocks, transposed
    const int kq = i / (NO / 4), c = 4 * (i - kq * (NO / 4)), k = 4 * kq;
    f32x4 r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = ld4(a.w + (size_t)(k + j) * NO + c);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      *reinterpret_cast<uint2*>(Bs + (c + e) * SKB + k) = f32_to_bf16x4(f32x4{r[0][e], r[1][e], r[2][e], r[3][e]});
  }
  for (int k = tid; k < KR; k += 256) {
    const float is = a.ois[k], ga = a.og[k];
    tab[0][k] = a.om[k];
    tab[1][k] = is;
    tab[2][k] = ga;
    tab[3][k] = a.ob[k];
    tab[4][k] = a.k12[k];
    tab[5][k] = a.k12[KR + k];
    tab[6][k] = ga * is;
  }
  float pm[NU], pis[NU], pga[NU], pbe[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int c = 32 * u + l32;
    pm[u] = PART ? a.im[c] : 0.f;
    pis[u] = PART ? a.iis[c] : 0.f;
    pga[u] = PART ? a.ig[c] : 0.f;
    pbe[u] = PART ? a.ib[c] : 0.f;
  }
  const bool orelu = a.orelu != 0, irelu = a.irelu != 0;
  __syncthreads();

  const uint32_t kbytes = (uint32_t)a.M * KR * 2u, nbytes = (uint32_t)a.M * NO * 2u;
  const __amdgpu_buffer_rsrc_t rg = make_rsrc_v(a.g, kbytes), rx = make_rsrc_v(a.xo, kbytes);
  const __amdgpu_buffer_rsrc_t rxi = make_rsrc_v(PART ? a.xi : a.g, PART ? nbytes : 0u);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc_v(RES ? a.res : a.g, RES ? nbytes : 0u);
  const __amdgpu_buffer_rsrc_t rdx = make_rsrc_v(a.dx, nbytes);
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc_v(a.dy_out ? a.dy_out : a.dx, a.dy_out ? kbytes : 0u);
  const int ntiles = (a.M + TR - 1) / TR;
  const int W = gridDim.x * WAVES;
  int t = blockIdx.x * WAVES + wave;
  double ps[NU], pq[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) ps[u] = pq[u] = 0.0;

  auto load_a = [&](int tile, u32x4* lg, u32x4* lx) {
    const uint32_t base = ((uint32_t)(tile * TR + l32) * KR + 8 * h) * 2u;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      lg[s] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)(base + 32u * s), 0, 0));
      lx[s] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(base + 32u * s), 0, 0));
    }
  };
  u32x4 cg[KS], cx[KS];
  load_a(t, cg, cx);
  drain_vmem_loads();
  for (; t < ntiles; t += W) {
    const int m0 = t * TR;
    int z = 0;
    asm volatile("" : "+s"(z));
    const float* tb = &tab[0][0] + z;
    const bf16_t* bs = Bs + z;

    // this tile's epilogue operands (C layout) and the next tile's A operands, in flight under the
    // transform and the MFMAs
    const int mb = m0 + 4 * h;
    const uint32_t eb = ((uint32_t)mb * NO + l32) * 2u;
    uint32_t exi[NU][16], ers[NU][16];
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dm = (r & 3) + 8 * (r >> 2);
        const int off = (int)(eb + (uint32_t)(dm * NO + 32 * u) * 2u);
        if constexpr (PART) exi[u][r] = __builtin_amdgcn_raw_buffer_load_b16(rxi, off, 0, 0);
        if constexpr (RES) ers[u][r] = __builtin_amdgcn_raw_buffer_load_b16(rr, off, 0, 0);
      }
    u32x4 ng[KS], nx[KS];
    load_a(t + W, ng, nx);
    __builtin_amdgcn_sched_barrier(0);

    bf16x8 af[KS];
    const uint32_t dbase = ((uint32_t)(m0 + l32) * KR + 8 * h) * 2u;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      f32x4 gv[2], xv[2];
      unpack8(cg[s], gv[0], gv[1]);
      unpack8(cx[s], xv[0], xv[1]);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int k0 = 16 * s + 8 * h + 4 * p;
        const f32x4 mu = ld4(tb + 0 * KR + k0), is = ld4(tb + 1 * KR + k0), ga = ld4(tb + 2 * KR + k0),
                    be = ld4(tb + 3 * KR + k0);
        const f32x4 k1 = ld4(tb + 4 * KR + k0), k2 = ld4(tb + 5 * KR + k0), f = ld4(tb + 6 * KR + k0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xe = xv[p][e];
          float ge = gv[p][e];
          const bool kill = (!(bn_out(xe, mu[e], is[e], ga[e], be[e]) > 0.f)) & orelu;
          ge = kill ? 0.f : ge;
          gv[p][e] = bn_bwd_elem(xe, ge, mu[e], is[e], f[e], k1[e], k2[e]);
        }
      }
      const u32x4 dyq = pack8(gv[0], gv[1]);
      af[s] = frag(dyq);
      __builtin_amdgcn_raw_buffer_store_b128(dyq, rdy, (int)(dbase + 32u * s), 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);

    f32x16 acc[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const bf16x8 bf = *reinterpret_cast<const bf16x8*>(bs + (32 * u + l32) * SKB + 16 * s + 8 * h);
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bf, acc[u], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);

#pragma unroll
    for (int u = 0; u < NU; ++u) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dm = (r & 3) + 8 * (r >> 2);
        float v = acc[u][r];
        if constexpr (RES) v += __builtin_bit_cast(float, ers[u][r] << 16);
        const uint16_t bits = bf16_bits(v);
        __builtin_amdgcn_raw_buffer_store_b16(bits, rdx, (int)(eb + (uint32_t)(dm * NO + 32 * u) * 2u), 0, 0);
        if constexpr (PART) {
          const float gs = __builtin_bit_cast(float, (uint32_t)bits << 16);  // dx as stored
          const float x = __builtin_bit_cast(float, exi[u][r] << 16);
          const float xh = (x - pm[u]) * pis[u];
          const bool kill = ((!(bn_out(x, pm[u], pis[u], pga[u], pbe[u]) > 0.f)) & irelu) | (mb + dm >= a.M);
          const float g2 = kill ? 0.f : gs;
          ps[u] += (double)g2;
          pq[u] += (double)g2 * (double)xh;
        }
      }
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      cg[s] = ng[s];
      cx[s] = nx[s];
    }
  }
  if constexpr (!PART) return;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    ps[u] += __shfl_xor(ps[u], 32, 64);
    pq[u] += __shfl_xor(pq[u], 32, 64);
    if (h == 0) {
      red[wave][0][32 * u + l32] = ps[u];
      red[wave][1][32 * u + l32] = pq[u];
    }
  }
  __syncthreads();
  for (int i = tid; i < 2 * NO; i += 256) {
    const int which = i / NO, c = i - which * NO;
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) s += red[w][which][c];
    pub_store(a.part + ((size_t)blockIdx.x * 2 + which) * NO + c, s);
  }
  if (a.ft.part) fold_tail<256>(a.ft, blockIdx.x, 0, NO, 0);
}


// ---------------------------------------------------------------------------------------
// Fused backward for K = C = 64 (the 56 x 56 units): the dgrad above and the weight gradient
//   dW[k][c] = sum_m dy[m][k] * bn_relu(x)[m][c]   (layers/pointwise_convolution.py:61-64)
// in one pass, so dy is never stored and the layer input is read once (the epilogue's C-layout
// x loads).  Per 32-pixel wave tile, after the dgrad:
//   * the wave writes its bf16 dy fragments (A layout: pixel = row l32) to its own LDS image
//     [32 pixels][SDY] and reads them back transposed with ds_read_b64_tr_b16 -- the A operand of
//     v_mfma_f32_32x32x16_bf16 with rows = channels k and the k-step = 16 pixels;
//   * the B operand is bn_relu(x) from the epilogue's C-layout registers: registers 8s .. 8s + 7
//     of lane half h are pixels 16s + 8(j >> 2) + 4h + (j & 3) (j = 0..7), and the transposed
//     dy reads take those same pixels (rows 16s + 4h + q and 16s + 8 + 4h + q);
//   * dW accumulates in registers across the wave's tiles (2 x 2 tiles of 32 x 32).
// The operands are the ones the unfused path rounds: dy as stored (bf16), bn_relu(x) rounded to
// bf16 as the tiled engine's BN-on-load loader does.  dx and the input BN's partials are
// bit-identical to dgrad_bnbwd_kernel<64, 64>; dW regroups the sum over pixels.  At the end the
// block's 4 waves add their dW in LDS (fixed order) into one partial row wpart[block][64][64].
// ---------------------------------------------------------------------------------------
struct BwdArgs {
  DgradArgs d;   // (d.dy_out unused; d.xi = the layer input, required)
  float* wpart;  // [gridDim.x][64][64]
};

constexpr int kBwdSDY = 96;  // dy image row stride (bf16 elements): an odd multiple of 64 bytes

template <bool RES, bool PART>
__global__ __launch_bounds__(256, 2) void bwd_fused_kernel(BwdArgs ba) {
  constexpr int KR = 64, NO = 64, SKB = KR + 8, KS = KR / 16, NU = NO / 32, KT = KR / 32, SDY = kBwdSDY;
  const DgradArgs& a = ba.d;
  __shared__ __attribute__((aligned(16))) bf16_t Bs[NO * SKB];  // Bs[c][k] = W[k][c]
  __shared__ __attribute__((aligned(16))) float tab[7][KR];
  __shared__ double red[WAVES][2][NO];
  __shared__ __attribute__((aligned(16))) bf16_t dyl[WAVES][TR * SDY];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  for (int i = tid; i < KR * NO / 16; i += 256) {  // 4 k x 4 c blocks, transposed
    const int kq = i / (NO / 4), c = 4 * (i - kq * (NO / 4)), k = 4 * kq;
    f32x4 r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = ld4(a.w + (size_t)(k + j) * NO + c);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      *reinterpret_cast<uint2*>(Bs + (c + e) * SKB + k) = f32_to_bf16x4(f32x4{r[0][e], r[1][e], r[2][e], r[3][e]});
  }
  for (int k = tid; k < KR; k += 256) {
    const float is = a.ois[k], ga = a.og[k];
    tab[0][k] = a.om[k];
    tab[1][k] = is;
    tab[2][k] = ga;
    tab[3][k] = a.ob[k];
    tab[4][k] = a.k12[k];
    tab[5][k] = a.k12[KR + k];
    tab[6][k] = ga * is;
  }
  // the input BatchNorm of this lane's columns (the partials and the weight gradient's operand)
  float pm[NU], pis[NU], pga[NU], pbe[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int c = 32 * u + l32;
    pm[u] = a.im ? a.im[c] : 0.f;
    pis[u] = a.im ? a.iis[c] : 0.f;
    pga[u] = a.im ? a.ig[c] : 0.f;
    pbe[u] = a.im ? a.ib[c] : 0.f;
  }
  const bool bnin = a.im != nullptr;
  const bool orelu = a.orelu != 0, irelu = a.irelu != 0;
  __syncthreads();

  const uint32_t kbytes = (uint32_t)a.M * KR * 2u, nbytes = (uint32_t)a.M * NO * 2u;
  const __amdgpu_buffer_rsrc_t rg = make_rsrc_v(a.g, kbytes), rx = make_rsrc_v(a.xo, kbytes);
  const __amdgpu_buffer_rsrc_t rxi = make_rsrc_v(a.xi, nbytes);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc_v(RES ? a.res : a.g, RES ? nbytes : 0u);
  const __amdgpu_buffer_rsrc_t rdx = make_rsrc_v(a.dx, nbytes);
  const int ntiles = (a.M + TR - 1) / TR;
  const int W = gridDim.x * WAVES;
  int t = blockIdx.x * WAVES + wave;
  double ps[NU], pq[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) ps[u] = pq[u] = 0.0;
  f32x16 dwa[KT][NU];
#pragma unroll
  for (int i = 0; i < KT; ++i)
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) dwa[i][u][r] = 0.f;
  bf16_t* dyw = &dyl[wave][0];

  auto load_a = [&](int tile, u32x4* lg, u32x4* lx) {
    const uint32_t base = ((uint32_t)(tile * TR + l32) * KR + 8 * h) * 2u;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      lg[s] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)(base + 32u * s), 0, 0));
      lx[s] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(base + 32u * s), 0, 0));
    }
  };
  u32x4 cg[KS], cx[KS];
  load_a(t, cg, cx);
  drain_vmem_loads();
  for (; t < ntiles; t += W) {
    const int m0 = t * TR;
    int z = 0;
    asm volatile("" : "+s"(z));
    const float* tb = &tab[0][0] + z;
    const bf16_t* bs = Bs + z;

    const int mb = m0 + 4 * h;
    const uint32_t eb = ((uint32_t)mb * NO + l32) * 2u;
    uint32_t exi[NU][16], ers[NU][16];
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dm = (r & 3) + 8 * (r >> 2);
        const int off = (int)(eb + (uint32_t)(dm * NO + 32 * u) * 2u);
        exi[u][r] = __builtin_amdgcn_raw_buffer_load_b16(rxi, off, 0, 0);
        if constexpr (RES) ers[u][r] = __builtin_amdgcn_raw_buffer_load_b16(rr, off, 0, 0);
      }
    u32x4 ng[KS], nx[KS];
    load_a(t + W, ng, nx);
    __builtin_amdgcn_sched_barrier(0);

    bf16x8 af[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      f32x4 gv[2], xv[2];
      unpack8(cg[s], gv[0], gv[1]);
      unpack8(cx[s], xv[0], xv[1]);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int k0 = 16 * s + 8 * h + 4 * p;
        const f32x4 mu = ld4(tb + 0 * KR + k0), is = ld4(tb + 1 * KR + k0), ga = ld4(tb + 2 * KR + k0),
                    be = ld4(tb + 3 * KR + k0);
        const f32x4 k1 = ld4(tb + 4 * KR + k0), k2 = ld4(tb + 5 * KR + k0), f = ld4(tb + 6 * KR + k0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xe = xv[p][e];
          float ge = gv[p][e];
          const bool kill = (!(bn_out(xe, mu[e], is[e], ga[e], be[e]) > 0.f)) & orelu;
          ge = kill ? 0.f : ge;
          gv[p][e] = bn_bwd_elem(xe, ge, mu[e], is[e], f[e], k1[e], k2[e]);
        }
      }
      const u32x4 dyq = pack8(gv[0], gv[1]);
      af[s] = frag(dyq);
      // the dy image for the weight gradient: row = pixel l32, channels 16s + 8h .. +7 (this wave's
      // own image: LDS operations of a wave complete in order, so its transposed reads below see
      // these stores; the asm barriers keep the compiler from moving loads or stores across)
      asm volatile("" ::: "memory");
      *reinterpret_cast<u32x4*>(dyw + l32 * SDY + 16 * s + 8 * h) = dyq;
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    f32x16 acc[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const bf16x8 bf = *reinterpret_cast<const bf16x8*>(bs + (32 * u + l32) * SKB + 16 * s + 8 * h);
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bf, acc[u], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);

    // epilogue: dx (+ residual) stored bf16, the input BN's partials, and the weight gradient's B
    // operand bn_relu(x) rounded to bf16 (zero for pixels past M)
    const bool full = m0 + TR <= a.M;
    bf16x8 bx[NU][2];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      float xb[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dm = (r & 3) + 8 * (r >> 2);
        float v = acc[u][r];
        if constexpr (RES) v += __builtin_bit_cast(float, ers[u][r] << 16);
        const uint16_t bits = bf16_bits(v);
        __builtin_amdgcn_raw_buffer_store_b16(bits, rdx, (int)(eb + (uint32_t)(dm * NO + 32 * u) * 2u), 0, 0);
        const float x = __builtin_bit_cast(float, exi[u][r] << 16);
        const bool out = !full && mb + dm >= a.M;
        float xo = x;
        if (bnin) {
          const float xh = (x - pm[u]) * pis[u];
          const float bo = bn_out(x, pm[u], pis[u], pga[u], pbe[u]);
          const bool dead = (!(bo > 0.f)) & irelu;
          if constexpr (PART) {
            const float gs = __builtin_bit_cast(float, (uint32_t)bits << 16);  // dx as stored
            const float g2 = (dead | out) ? 0.f : gs;
            ps[u] += (double)g2;
            pq[u] += (double)g2 * (double)xh;
          }
          xo = dead ? 0.f : bo;
        }
        xb[r] = out ? 0.f : xo;
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        bx[u][s2] = frag(pack8(f32x4{xb[8 * s2], xb[8 * s2 + 1], xb[8 * s2 + 2], xb[8 * s2 + 3]},
                               f32x4{xb[8 * s2 + 4], xb[8 * s2 + 5], xb[8 * s2 + 6], xb[8 * s2 + 7]}));
    }
    // dW^T... : dwa[kt][u][k-row, c-col] += dy^T (rows = channels kt*32.., k = pixels) . bx
    {
      const int i = lane & 15, g = (lane >> 4) & 1;
      typedef short s16x4 __attribute__((ext_vector_type(4)));
      typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
          const bf16_t* p = dyw + (16 * s2 + 4 * h + (i >> 2)) * SDY + 32 * kt + 16 * g + 4 * (i & 3);
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 8 * SDY));
          const bf16x8 dyt = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
          for (int u = 0; u < NU; ++u)
            dwa[kt][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dyt, bx[u][s2], dwa[kt][u], 0, 0, 0);
        }
      }
      asm volatile("" ::: "memory");  // the next tile's image stores stay after these reads
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      cg[s] = ng[s];
      cx[s] = nx[s];
    }
  }
  // the block's partial row of dW: the waves' blocks added in LDS in a fixed order,
  // (w0 + w1) + (w2 + w3), through one [64][64] fp32 buffer over the (now idle) dy images;
  // element (kt, u, r) of a lane is dW[32 kt + (r & 3) + 8 (r >> 2) + 4h][32 u + l32]
  static_assert(sizeof(float) * KR * NO <= sizeof(bf16_t) * WAVES * TR * SDY, "dW buffer fits the dy images");
  float* wsum = reinterpret_cast<float*>(&dyl[0][0]);
  auto tile_io = [&](bool add, bool store) __attribute__((always_inline)) {
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float* q = wsum + (32 * kt + (r & 3) + 8 * (r >> 2) + 4 * h) * NO + 32 * u + l32;
          if (add) dwa[kt][u][r] += *q;
          if (store) *q = dwa[kt][u][r];
        }
  };
  __syncthreads();
  if (wave == 1) tile_io(false, true);
  __syncthreads();
  if (wave == 0) tile_io(true, false);
  __syncthreads();
  if (wave == 3) tile_io(false, true);
  __syncthreads();
  if (wave == 2) tile_io(true, true);
  __syncthreads();
  if (wave == 0) tile_io(true, true);
  __syncthreads();
  {
    float* wp = ba.wpart + (size_t)blockIdx.x * KR * NO;
    for (int i = tid; i < KR * NO / 4; i += 256) st4(wp + 4 * i, ld4(wsum + 4 * i));
  }
  if constexpr (!PART) return;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    ps[u] += __shfl_xor(ps[u], 32, 64);
    pq[u] += __shfl_xor(pq[u], 32, 64);
    if (h == 0) {
      red[wave][0][32 * u + l32] = ps[u];
      red[wave][1][32 * u + l32] = pq[u];
    }
  }
  __syncthreads();
  for (int i = tid; i < 2 * NO; i += 256) {
    const int which = i / NO, c = i - which * NO;
    double sm = 0.0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) sm += red[w][which][c];
    pub_store(a.part + ((size_t)blockIdx.x * 2 + which) * NO + c, sm);
  }
  if (a.ft.part) fold_tail<256>(a.ft, blockIdx.x, 0, NO, 0);
}

template <int KR, int NO>
static int fwd_occ() {
  // thread-safe one-time query (a function-local static initialised once)
  static const int occ = [] {
    const void* fs[] = {reinterpret_cast<const void*>(&fwd_kernel<KR, NO, true, true>),
                        reinterpret_cast<const void*>(&fwd_kernel<KR, NO, true, false>),
                        reinterpret_cast<const void*>(&fwd_kernel<KR, NO, false, true>),
                        reinterpret_cast<const void*>(&fwd_kernel<KR, NO, false, false>)};
    return min_occupancy(fs, 4);
  }();
  return occ;
}
template <int KR, int NO>
static int dgrad_occ() {
  // thread-safe one-time query (a function-local static initialised once)
  static const int occ = [] {
    const void* fs[] = {reinterpret_cast<const void*>(&dgrad_bnbwd_kernel<KR, NO, true, true>),
                        reinterpret_cast<const void*>(&dgrad_bnbwd_kernel<KR, NO, true, false>),
                        reinterpret_cast<const void*>(&dgrad_bnbwd_kernel<KR, NO, false, true>),
                        reinterpret_cast<const void*>(&dgrad_bnbwd_kernel<KR, NO, false, false>)};
    return min_occupancy(fs, 4);
  }();
  return occ;
}


// The (reduction, output) channel pairs instantiated.
#define DK_PWSH_SHAPES(X) X(64, 64) X(64, 128) X(128, 64) X(128, 128)

}  // namespace pwsh

// Knob 9 = 0 (or the fp32 streaming knob 3 = 0) keeps the tiled engine.
// (knob kKnobPwsh, kind 9)
static bool pwsh_enabled() { return knob(kKnobPwsh) == 1 && pw_stream_enabled(); }

static bool pwsh_shape(int KR, int NO) { return (KR == 64 || KR == 128) && (NO == 64 || NO == 128); }
constexpr int kDeepCols = 128;  // output columns per block of the deep kernels (pw_deep_bf16.hip)
// The deep shapes (reduction or outputs of 256+) go to the weight-stationary kernels of
// pw_deep_bf16.hip (knob 13); with those off they stay on the tiled engine.
bool pw_stream_bf16_fwd_ok(int K, int C, int M) {
  return pwsh_enabled() && (pwsh_shape(C, K) || pw_deep16_fwd_ok(K, C, M)) && M > 0 &&
         (size_t)M * (K > C ? K : C) * 2 < ((size_t)1 << 31);
}
int pw_stream_bf16_fwd_rows(int M, int K, int C) {
  if (!pwsh_shape(C, K) && pw_deep16_fwd_ok(K, C, M)) return pw_deep16_fwd_rows(M, K, C);
#define DK_ROWS(kr, no) \
  if (C == kr && K == no) return pwsh::grid_blocks(M, pwsh::fwd_occ<kr, no>());
  DK_PWSH_SHAPES(DK_ROWS)
#undef DK_ROWS
  return 0;
}
int pw_stream_bf16_fwd_slices(int K, int C) { return pwsh_shape(C, K) ? 1 : K / kDeepCols; }
bool pw_stream_bf16_dgrad_ok(int K, int C, int M) {
  return pwsh_enabled() && (pwsh_shape(K, C) || pw_deep16_dgrad_ok(K, C, M)) && M > 0 &&
         (size_t)M * (K > C ? K : C) * 2 < ((size_t)1 << 31);
}
int pw_stream_bf16_dgrad_rows(int M, int K, int C) {
  if (!pwsh_shape(K, C) && pw_deep16_dgrad_ok(K, C, M)) return pw_deep16_dgrad_rows(M, K, C);
#define DK_ROWS(kr, no) \
  if (K == kr && C == no) return pwsh::grid_blocks(M, pwsh::dgrad_occ<kr, no>());
  DK_PWSH_SHAPES(DK_ROWS)
#undef DK_ROWS
  return 0;
}
int pw_stream_bf16_dgrad_slices(int K, int C) { return pwsh_shape(K, C) ? 1 : C / kDeepCols; }

int pw_stream_bf16_fwd(const bf16_t* x, int M, const float* w, int K, int C, const float* bias, bf16_t* y,
                       const float* im, const float* iis, const float* ig, const float* ib, int irelu, double* part,
                       hipStream_t st, const FoldTail* ft) {
  if (!pwsh_shape(C, K) && pw_deep16_fwd_ok(K, C, M))  // the weight-stationary kernels (pw_deep_bf16.hip)
    return pw_deep16_fwd(x, M, w, K, C, bias, y, im, iis, ig, ib, irelu, part, st, ft);
  if (!pwsh_shape(C, K)) return DK_ERR_ARGS;
  pwsh::FwdArgs a{x, w, bias, y, im, iis, ig, ib, irelu, part, M};
  if (ft && part) a.ft = *ft;
  const dim3 grid(pw_stream_bf16_fwd_rows(M, K, C));
  if (grid.x == 0) return DK_ERR_ARGS;
#define DK_FWD(kr, no)                                                                                   \
  if (C == kr && K == no) {                                                                              \
    if (im && part)                                                                                      \
      hipLaunchKernelGGL((pwsh::fwd_kernel<kr, no, true, true>), grid, dim3(256), 0, st, a);             \
    else if (im)                                                                                         \
      hipLaunchKernelGGL((pwsh::fwd_kernel<kr, no, true, false>), grid, dim3(256), 0, st, a);            \
    else if (part)                                                                                       \
      hipLaunchKernelGGL((pwsh::fwd_kernel<kr, no, false, true>), grid, dim3(256), 0, st, a);            \
    else                                                                                                 \
      hipLaunchKernelGGL((pwsh::fwd_kernel<kr, no, false, false>), grid, dim3(256), 0, st, a);           \
    return launch_status();                                                                              \
  }
  DK_PWSH_SHAPES(DK_FWD)
#undef DK_FWD
  return DK_ERR_ARGS;
}

int pw_stream_bf16_dgrad_bnbwd(const bf16_t* g, const bf16_t* bn_x, int M, int K, int C, const float* om,
                               const float* ois, const float* og, const float* ob, int orelu, const float* k12,
                               bf16_t* dy_out, const float* w, bf16_t* dx, const bf16_t* res, const bf16_t* x,
                               const float* im, const float* iis, const float* ig, const float* ib, int irelu,
                               double* part, hipStream_t st, const FoldTail* ft) {
  if (!pwsh_shape(K, C) && pw_deep16_dgrad_ok(K, C, M))
    return pw_deep16_dgrad_bnbwd(g, bn_x, M, K, C, om, ois, og, ob, orelu, k12, dy_out, w, dx, res, x, im, iis, ig, ib,
                                 irelu, part, st, ft);
  if (!pwsh_shape(K, C)) return DK_ERR_ARGS;
  pwsh::DgradArgs a{g, bn_x, dy_out, w, dx, res, x, om, ois, og, ob, k12, orelu, im, iis, ig, ib, irelu, part, M};
  if (ft && part) a.ft = *ft;
  const dim3 grid(pw_stream_bf16_dgrad_rows(M, K, C));
  if (grid.x == 0) return DK_ERR_ARGS;
#define DK_DG(kr, no)                                                                                    \
  if (K == kr && C == no) {                                                                              \
    if (res && x)                                                                                        \
      hipLaunchKernelGGL((pwsh::dgrad_bnbwd_kernel<kr, no, true, true>), grid, dim3(256), 0, st, a);     \
    else if (res)                                                                                        \
      hipLaunchKernelGGL((pwsh::dgrad_bnbwd_kernel<kr, no, true, false>), grid, dim3(256), 0, st, a);    \
    else if (x)                                                                                          \
      hipLaunchKernelGGL((pwsh::dgrad_bnbwd_kernel<kr, no, false, true>), grid, dim3(256), 0, st, a);    \
    else                                                                                                 \
      hipLaunchKernelGGL((pwsh::dgrad_bnbwd_kernel<kr, no, false, false>), grid, dim3(256), 0, st, a);   \
    return launch_status();                                                                              \
  }
  DK_PWSH_SHAPES(DK_DG)
#undef DK_DG
  return DK_ERR_ARGS;
}

// ---- the fused K = C = 64 backward (bwd_fused_kernel) ----
static int pwsh_bwd_occ() {
  static const int occ = [] {
    const void* fs[] = {reinterpret_cast<const void*>(&pwsh::bwd_fused_kernel<true, true>),
                        reinterpret_cast<const void*>(&pwsh::bwd_fused_kernel<true, false>),
                        reinterpret_cast<const void*>(&pwsh::bwd_fused_kernel<false, true>),
                        reinterpret_cast<const void*>(&pwsh::bwd_fused_kernel<false, false>)};
    return pwsh::min_occupancy(fs, 4);
  }();
  return occ;
}
bool pw_stream_bf16_bwd_ok(int K, int C, int M) {
  return pwsh_enabled() && K == 64 && C == 64 && M > 0 &&
         (size_t)M * 64 * 2 < ((size_t)1 << 31);
}
int pw_stream_bf16_bwd_rows(int M) { return pwsh::grid_blocks(M, pwsh_bwd_occ()); }

int pw_stream_bf16_bwd_fused(const bf16_t* g, const bf16_t* bn_x, int M, const float* om, const float* ois,
                             const float* og, const float* ob, int orelu, const float* k12, const float* w, bf16_t* dx,
                             const bf16_t* res, const bf16_t* x, const float* im, const float* iis, const float* ig,
                             const float* ib, int irelu, double* part, float* wpart, hipStream_t st,
                             const FoldTail* ft) {
  if (!x || (part && !im)) return DK_ERR_ARGS;
  pwsh::BwdArgs a{pwsh::DgradArgs{g, bn_x, nullptr, w, dx, res, x, om, ois, og, ob, k12, orelu, im, iis, ig, ib, irelu,
                                  part, M},
                  wpart};
  if (ft && part) a.d.ft = *ft;
  const dim3 grid(pw_stream_bf16_bwd_rows(M));
  if (res && part)
    hipLaunchKernelGGL((pwsh::bwd_fused_kernel<true, true>), grid, dim3(256), 0, st, a);
  else if (res)
    hipLaunchKernelGGL((pwsh::bwd_fused_kernel<true, false>), grid, dim3(256), 0, st, a);
  else if (part)
    hipLaunchKernelGGL((pwsh::bwd_fused_kernel<false, true>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((pwsh::bwd_fused_kernel<false, false>), grid, dim3(256), 0, st, a);
  return launch_status();
}

}  // namespace dk
