// Streaming pointwise kernels for the memory-bound 1x1 shapes (K = C = 64: res1/res2 of
// ResNet-18-depsep, P = N*H*W = 802,816 pixels at batch 256).
//
// The general implicit-GEMM engine (gemm_f32.hip) stages every operand tile through LDS and
// runs one block per 64-row tile: at K = 64 that is two K-tiles, a prologue and an epilogue
// per 16 KB of input, and the block's dependent global round trips (operand loads, BN-table
// fill, epilogue operand loads, stores) are exposed at 3-4 resident blocks per CU.  Here:
//
//   * persistent waves: a grid of (resident blocks x CUs) blocks of 4 waves; wave w streams
//     row tiles w, w + W, w + 2W, ... (W = all waves) of 32 pixels each;
//   * the MFMA A operand goes global -> registers directly (no LDS): lane (l32, h) loads the
//     float4s k = 8q + 4h .. +3 of row l32 -- exactly its v_mfma_f32_32x32x2_f32 fragments, in
//     the k order of gemm_f32.hip's engine (k = 8q + 4h + e), so results are bit-identical to
//     it; the B operand (the weights, 16 KB) is loaded into LDS once per block;
//   * software pipeline per wave: tile t+W's operand loads and tile t's epilogue operand loads
//     are in flight while tile t's MFMAs run;
//   * the epilogue works in the MFMA's C layout: each lane owns two output columns for the
//     whole kernel, so the BatchNorm partial sums accumulate in registers across all of a
//     wave's tiles and the kernel writes ONE partial row per block (gridDim.x rows instead of
//     one per 64-pixel tile: the following fold reads 1/25th of the bytes).
//
// dk_pwconv_dgrad_bnbwd_f32 (the step's dominant entry point, layers/pointwise_convolution.py
// :57-75 + layers/batch_norm.py:125-174): dx = dy . W (+ residual) with
// dy = the following BatchNorm's backward applied to its gradient g on load (bn_bwd_elem,
// bit-identical to dk_bn_bwd_apply_f32), dy written through for the weight gradient, and the
// input BatchNorm's backward partial sums (sum g', sum g' x_hat) of dx.
#include <stdlib.h>

#include <type_traits>

#include "dk_common.h"
#include "fold_tail.h"

namespace dk {
namespace pws {

constexpr int KR = 64;          // reduction length (the pointwise layer's output channels K)
constexpr int NO = 64;          // output columns (its input channels C)
constexpr int WAVES = 4;        // waves per block
constexpr int TR = 32;          // rows (pixels) per wave tile
constexpr int SKB = KR + 4;     // LDS row stride of the B image Bs[n][k]: (KR+4)/4 odd -> conflict-free b128
constexpr int KQ = KR / 8;      // float4 groups per lane per operand row
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// vmcnt(0) (expcnt, lgkmcnt left alone; gfx9 encoding).  Issued once after the loop's first
// operand loads: the waitcnt pass then sees no VMEM result pending on the preheader path and
// does not put a wait at the loop head -- which, merged with the back edge, waited for the
// previous tile's output stores before every tile's first MFMA.
__device__ __forceinline__ void drain_vmem_loads() { __builtin_amdgcn_s_waitcnt(0x0F70); }

struct DgradArgs {
  const float* g;     // [M][KR] gradient w.r.t. the following BN's (+ReLU) output
  const float* xo;    // [M][KR] that BN's raw input (= this layer's output)
  float* dy_out;      // [M][KR] dy write-through (nullable)
  const float* w;     // [KR][NO] pointwise weights W[k][c]
  float* dx;          // [M][NO]
  const float* res;   // [M][NO] residual addend (nullable)
  const float* xi;    // [M][NO] the input BN's raw input (nullable: no partials)
  const float* om;    // following BN: mean, invstd, gamma, beta, k12 = [k1[KR], k2[KR]]
  const float* ois;
  const float* og;
  const float* ob;
  const float* k12;
  int orelu;
  const float* im;    // input BN (partials): mean, invstd, gamma, beta
  const float* iis;
  const float* ig;
  const float* ib;
  int irelu;
  double* part;       // [gridDim.x][2][NO]
  int M;
  FoldTail ft;        // ft.part != nullptr: fold the partial rows in this launch (fold_tail.h)
  int nt;             // nontemporal dx stores (tuning knob, nt_stores())
};

__device__ __forceinline__ uint32_t row_off_bytes(int m, int ld, int c) { return ((uint32_t)m * ld + c) * 4u; }
// Every global access of the streaming kernels is a buffer access whose resource covers exactly
// the tensor's M rows: rows >= M (the ragged last tile, the prefetch past the last tile) fall
// outside it in hardware -- loads return 0, stores are dropped -- so the loop needs no
// per-row conditions (which the compiler turns into control flow and conservative vmcnt(0)
// waits) and each access is a base register plus an immediate offset.

template <bool RES, bool PART>
__global__ __launch_bounds__(256, 2) void dgrad_bnbwd_kernel(DgradArgs a) {
  // B image: Bs[c][k] = W[k][c]; the following BN's per-channel table as 7 SoA rows
  __shared__ float Bs[NO * SKB];
  __shared__ float tab[7][KR];
  __shared__ double red[WAVES][2][NO];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  for (int i = tid; i < KR * NO; i += 256) {
    const int k = i / NO, c = i - k * NO;
    Bs[c * SKB + k] = a.w[i];
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
  // this lane's two output columns: the input BN's parameters for the partials
  constexpr bool parts = PART;
  const bool orelu = a.orelu != 0, irelu = a.irelu != 0;
  float pm[2], pis[2], pga[2], pbe[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = 32 * u + l32;
    pm[u] = parts ? a.im[c] : 0.f;
    pis[u] = parts ? a.iis[c] : 0.f;
    pga[u] = parts ? a.ig[c] : 0.f;
    pbe[u] = parts ? a.ib[c] : 0.f;
  }
  __syncthreads();

  const uint32_t kbytes = (uint32_t)a.M * KR * 4u, nbytes = (uint32_t)a.M * NO * 4u;
  const __amdgpu_buffer_rsrc_t rg = make_rsrc_v(a.g, kbytes), rx = make_rsrc_v(a.xo, kbytes);
  const __amdgpu_buffer_rsrc_t rxi = make_rsrc_v(PART ? a.xi : a.g, PART ? nbytes : 0u);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc_v(RES ? a.res : a.g, RES ? nbytes : 0u);
  const __amdgpu_buffer_rsrc_t rdx = make_rsrc_v(a.dx, nbytes);
  // no dy_out: a zero-size resource, every store dropped
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc_v(a.dy_out ? a.dy_out : a.dx, a.dy_out ? kbytes : 0u);
  const int ntiles = (a.M + TR - 1) / TR;
  const int W = gridDim.x * WAVES;
  int t = blockIdx.x * WAVES + wave;

  double ps[2] = {0.0, 0.0}, pq[2] = {0.0, 0.0};
  // A operands (raw g, x of the following BN) of a tile: lane (l32, h) reads row l32's float4s
  // k = 8q + 4h .. +3; rows >= M (incl. tiles past the end) read zeros
  auto load_a = [&](int tile, f32x4* lg, f32x4* lx) {
    const int m = tile * TR + l32;
    const uint32_t base = row_off_bytes(m, KR, 4 * h);
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      lg[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)(base + 32u * q), 0, 0));
      lx[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(base + 32u * q), 0, 0));
    }
  };
  f32x4 cg[KQ], cx[KQ];  // this tile's raw A operands (loaded one iteration ahead)
  load_a(t, cg, cx);
  drain_vmem_loads();
  for (; t < ntiles; t += W) {
    const int m0 = t * TR;
    // an opaque zero: keeps the (loop-invariant) LDS table and weight reads inside the loop,
    // where they cost a few LDS cycles, instead of hoisted into ~290 long-lived registers
    int z = 0;
    asm volatile("" : "+s"(z));
    const float* tb = &tab[0][0] + z;
    const float* bs = Bs + z;

    // (1) issue: tile t's epilogue operands (C layout: column 32u + l32, rows (r&3) + 8(r>>2) + 4h),
    //     then tile t+W's A operands -- in flight during this tile's transform and MFMAs
    float exi[2][16], ers[2][16];
    const int mb = m0 + 4 * h;
    // rows (r&3) + 8(r>>2) of the lane half: two base registers (r < 8, r >= 8), the rest in
    // the 12-bit immediate offset
    const uint32_t eb0 = row_off_bytes(mb, NO, l32), eb1 = eb0 + 16u * NO * 4u;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t imm = (uint32_t)(((r & 3) + 8 * ((r >> 2) & 1)) * NO + 32 * u) * 4u;
        const uint32_t eb = r < 8 ? eb0 : eb1;
        if constexpr (PART)
          exi[u][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rxi, (int)(eb + imm), 0, 0));
        if constexpr (RES)
          ers[u][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, (int)(eb + imm), 0, 0));
      }
    f32x4 ng[KQ], nx[KQ];
    load_a(t + W, ng, nx);
    __builtin_amdgcn_sched_barrier(0);

    // (2) dy = the following BN's backward applied to g (bit-identical to dk_bn_bwd_apply_f32),
    //     written through for the weight gradient
    f32x4 af[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const int k0 = 8 * q + 4 * h;
      const f32x4 mu = ld4(tb + 0 * KR + k0), is = ld4(tb + 1 * KR + k0), ga = ld4(tb + 2 * KR + k0),
                  be = ld4(tb + 3 * KR + k0);
      const f32x4 k1 = ld4(tb + 4 * KR + k0), k2 = ld4(tb + 5 * KR + k0), f = ld4(tb + 6 * KR + k0);
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xe = cx[q][e];
        float ge = cg[q][e];
        // branch-free ReLU mask (a branch on the uniform flag would split the loop into blocks
        // with conservative vmcnt(0) waits)
        const bool kill = (!(bn_out(xe, mu[e], is[e], ga[e], be[e]) > 0.f)) & orelu;
        ge = kill ? 0.f : ge;
        o[e] = bn_bwd_elem(xe, ge, mu[e], is[e], f[e], k1[e], k2[e]);
      }
      af[q] = o;
    }
    {
      const int mrow = m0 + l32;
      const uint32_t dbase = row_off_bytes(mrow, KR, 4 * h);
#pragma unroll
      for (int q = 0; q < KQ; ++q)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, af[q]), rdy, (int)(dbase + 32u * q), 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);

    // (3) dx tile = dy . W : 32 rows x 64 columns, k order 8q + 4h + e as gemm_f32.hip
    f32x16 acc[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      f32x4 bf[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) bf[u] = ld4(bs + (32 * u + l32) * SKB + 8 * q + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q][e], bf[u][e], acc[u], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);

    // (4) epilogue: dx (+ residual), and the input BN's partial sums of what is stored
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dm = (r & 3) + 8 * (r >> 2);
        const uint32_t imm = (uint32_t)(((r & 3) + 8 * ((r >> 2) & 1)) * NO + 32 * u) * 4u;
        float v = acc[u][r];
        if constexpr (RES) v += ers[u][r];
        if (a.nt)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rdx, (int)((r < 8 ? eb0 : eb1) + imm),
                                                0, 2);
        else
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rdx, (int)((r < 8 ? eb0 : eb1) + imm),
                                                0, 0);
        if constexpr (PART) {
          const float x = exi[u][r];
          const float xh = (x - pm[u]) * pis[u];
          float gv = v;
          const bool kill = ((!(bn_out(x, pm[u], pis[u], pga[u], pbe[u]) > 0.f)) & irelu) | (mb + dm >= a.M);
          gv = kill ? 0.f : gv;  // rows past M contribute nothing
          ps[u] += (double)gv;
          pq[u] += (double)gv * (double)xh;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      cg[q] = ng[q];
      cx[q] = nx[q];
    }
  }
  if constexpr (!PART) return;
  // the block's partial row: lane halves, then the 4 waves in order
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    ps[u] += __shfl_xor(ps[u], 32, 64);
    pq[u] += __shfl_xor(pq[u], 32, 64);
    if (h == 0) {
      red[wave][0][32 * u + l32] = ps[u];
      red[wave][1][32 * u + l32] = pq[u];
    }
  }
  __syncthreads();
  if (tid < 2 * NO) {
    const int which = tid / NO, c = tid - which * NO;
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) s += red[w][which][c];
    pub_store(a.part + ((size_t)blockIdx.x * 2 + which) * NO + c, s);
  }
  if (a.ft.part) fold_tail<256>(a.ft, blockIdx.x, 0, NO, 0);
}


// ---------------------------------------------------------------------------------------
// dk_pwconv_fwd_ex_f32 (layers/pointwise_convolution.py:46-55 with the preceding BatchNorm(+ReLU)
// applied on load and the following BatchNorm's statistics emitted): y = bn(x) . W^T (+ bias),
// sa = 2: the reference's X[:, :, ::2, ::2] subsampling as a strided row map.  A operand lane
// (l32, h): bn_relu_out of x[row l32][c = 8q + 4h .. +3] (bit-identical to the tiled engine's
// LdImgKC with its LDS parameter table); B image Bs[k][c] = W[k][c] as stored.
// ---------------------------------------------------------------------------------------
struct FwdArgs {
  const float* x;     // [N*H*W][KR] raw input (the preceding BN's input when bn)
  const float* w;     // [NO][KR]
  const float* bias;  // [NO] nullable
  float* y;           // [M][NO], M = N*OH*OW
  const float* im;    // input BN: mean, invstd, gamma, beta (im == nullptr: no transform)
  const float* iis;
  const float* ig;
  const float* ib;
  int irelu;
  double* part;       // [gridDim.x][2][NO] (sum y, sum y^2) nullable
  int M, H, W, OH, OW, sa;
  uint32_t xbytes;
  FoldTail ft;        // ft.part != nullptr: fold the statistics rows in this launch
  int nt;             // nontemporal y stores (tuning knob, nt_stores())
};

template <int KR_, int NO_, bool BN, bool STATS, bool STRIDED>
__global__ __launch_bounds__(256, KR_ == 64 ? 3 : 2) void fwd_kernel(FwdArgs a) {
  // K = C = 64 (res1/res2) or 128 (res3/res4): the reduction KR, the output columns NO, NU MFMA
  // column blocks of 32; at 128 the transformed A operand overwrites its registers in place
  constexpr int KR = KR_, NO = NO_, SKB = KR + 4, KQ = KR / 8, NU = NO / 32;
  static_assert(KR % 32 == 0 && NO % 32 == 0 && (SKB / 4) % 2 == 1, "pws::fwd_kernel shape");
  __shared__ __attribute__((aligned(16))) float Bs[NO * SKB];
  __shared__ float tab[4][KR];
  // the statistics' block reduction reuses the B image once every wave has left the loop (at
  // K = C = 128 a separate buffer would push the block past 80 KB: one block per CU)
  double(*const red)[2][NO] = reinterpret_cast<double(*)[2][NO]>(Bs);
  static_assert(sizeof(double) * WAVES * 2 * NO <= sizeof(float) * NO * SKB, "red fits in Bs");
  // CO (K = 64, stride 1): the A rows arrive as whole 1 KB wave loads (lane (pr, cq) = (lane / 16,
  // lane % 16) holds pixel pr + 4q, channels 4cq ..) instead of 32-byte pieces of 32 rows, and the
  // transformed tile goes through a per-wave LDS image into the MFMA operand layout (as the fused
  // backward's dy image); 52 KB per block, still 3 blocks per CU
  constexpr bool CO = KR == 64 && !STRIDED;
  constexpr int SKA = KR + 4;
  __shared__ __attribute__((aligned(16))) float Ta[CO ? WAVES * TR * SKA : 4];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  for (int i = tid; i < KR * NO; i += 256) {
    const int n = i / KR, k = i - n * KR;
    Bs[n * SKB + k] = a.w[i];
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

  const uint32_t nbytes = (uint32_t)a.M * NO * 4u;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc_v(a.x, a.xbytes), ry = make_rsrc_v(a.y, nbytes);
  const int ntiles = (a.M + TR - 1) / TR;
  const int W = gridDim.x * WAVES;
  int t = blockIdx.x * WAVES + wave;
  double ps[NU], pq[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) ps[u] = pq[u] = 0.0;

  const int pr = lane >> 4, cq = lane & 15;
  float* const ta = Ta + (CO ? wave * TR * SKA : 0);
  auto load_a = [&](int tile, f32x4* lx) {
    if constexpr (CO) {
      const uint32_t base = row_off_bytes(tile * TR, KR, 0) + 16u * lane;
#pragma unroll
      for (int q = 0; q < KQ; ++q)
        lx[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(base + 1024u * q), 0, 0));
      return;
    }
    const int m = tile * TR + l32;
    int row = m;
    if constexpr (STRIDED) {
      // output pixel (n, oh, ow) reads input pixel (n, sa*oh, sa*ow); rows past M read past the
      // buffer (zeros): n >= N maps beyond N*H*W
      const int ow = m % a.OW, q = m / a.OW, oh = q % a.OH, n = q / a.OH;
      row = (n * a.H + oh * a.sa) * a.W + ow * a.sa;
    }
    const uint32_t base = row_off_bytes(row, KR, 4 * h);
#pragma unroll
    for (int q = 0; q < KQ; ++q)
      lx[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(base + 32u * q), 0, 0));
  };
  // the tile loop is unrolled by two so that the current and the prefetched tile's registers swap
  // roles by name: copying the prefetched registers at the loop latch waited for their loads
  f32x4 xa[KQ], xb[KQ];
  load_a(t, xa);
  drain_vmem_loads();
  auto tile = [&](f32x4 (&cx)[KQ], f32x4 (&nx)[KQ]) __attribute__((always_inline)) {
    const int m0 = t * TR;
    int z = 0;
    asm volatile("" : "+s"(z));
    const float* tb = &tab[0][0] + z;
    const float* bs = Bs + z;

    load_a(t + W, nx);
    __builtin_amdgcn_sched_barrier(0);

    f32x4 afs[KR == 64 ? KQ : 1];
    f32x4* const af = KR == 64 ? afs : cx;  // (in place at 128: cx is dead after the transform)
    if constexpr (CO) {
      f32x4 mu, is, ga, be;
      if constexpr (BN) {
        mu = ld4(tb + 0 * KR + 4 * cq);
        is = ld4(tb + 1 * KR + 4 * cq);
        ga = ld4(tb + 2 * KR + 4 * cq);
        be = ld4(tb + 3 * KR + 4 * cq);
      }
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        f32x4 v = cx[q];
        if constexpr (BN) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float r = bn_out(v[e], mu[e], is[e], ga[e], be[e]);
            v[e] = (irelu & !(r > 0.f)) ? 0.f : r;
          }
        }
        st4(ta + (pr + 4 * q) * SKA + 4 * cq, v);
      }
#pragma unroll
      for (int q = 0; q < KQ; ++q) af[q] = ld4(ta + l32 * SKA + 8 * q + 4 * h);
    }
#pragma unroll
    for (int q = 0; q < (CO ? 0 : KQ); ++q) {
      f32x4 v = cx[q];
      if constexpr (BN) {
        const int k0 = 8 * q + 4 * h;
        const f32x4 mu = ld4(tb + 0 * KR + k0), is = ld4(tb + 1 * KR + k0), ga = ld4(tb + 2 * KR + k0),
                    be = ld4(tb + 3 * KR + k0);
        // rows past M hold zeros, transformed like any other: their outputs are never stored
        // and are masked out of the statistics
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float r = bn_out(v[e], mu[e], is[e], ga[e], be[e]);
          v[e] = (irelu & !(r > 0.f)) ? 0.f : r;
        }
      }
      af[q] = v;
    }
    __builtin_amdgcn_sched_barrier(0);

    f32x16 acc[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      f32x4 bf[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) bf[u] = ld4(bs + (32 * u + l32) * SKB + 8 * q + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int u = 0; u < NU; ++u) acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q][e], bf[u][e], acc[u], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);

    const int mb = m0 + 4 * h;
    const uint32_t eb0 = row_off_bytes(mb, NO, l32), eb1 = eb0 + 16u * NO * 4u;
    if (a.bias) {
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[u][r] += bias[u];
    }
    // one branch around all the stores (the cache policy is an immediate): chosen per store, the
    // branches hid the number of stores in flight from the wait-count pass, and the next tile waited
    // for all of them (vmcnt(0)) before its loads were used
    auto store_tile = [&](auto pol) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t imm = (uint32_t)(((r & 3) + 8 * ((r >> 2) & 1)) * NO + 32 * u) * 4u;
          const float v = acc[u][r];  // (not bit_cast(acc[u][r]): hipcc 7.2 stores element 0 for every r)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), ry, (int)((r < 8 ? eb0 : eb1) + imm),
                                                0, decltype(pol)::value);
        }
    };
    if (a.nt)
      store_tile(std::integral_constant<int, 2>{});
    else
      store_tile(std::integral_constant<int, 0>{});
    if constexpr (STATS) {
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int dm = (r & 3) + 8 * (r >> 2);
          // (the past-M select in fp32, kept ahead of the widening: sunk past it, it became two
          // selects on the fp64 halves)
          float v = (mb + dm < a.M) ? acc[u][r] : 0.f;
          asm volatile("" : "+v"(v));
          const double d = (double)v;
          ps[u] += d;
          pq[u] += d * d;
        }
    }
  };
  while (t < ntiles) {
    tile(xa, xb);
    t += W;
    if (t >= ntiles) break;
    tile(xb, xa);
    t += W;
  }
  if constexpr (!STATS) return;
  __syncthreads();  // Bs becomes red
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
  if (tid < 2 * NO) {
    const int which = tid / NO, c = tid - which * NO;
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) s += red[w][which][c];
    pub_store(a.part + ((size_t)blockIdx.x * 2 + which) * NO + c, s);
  }
  if (a.ft.part) {
    if constexpr (CO)
      fold_tail<256>(a.ft, blockIdx.x, 0, NO, 0, reinterpret_cast<double2*>(Ta));  // (the image is free)
    else
      fold_tail<256>(a.ft, blockIdx.x, 0, NO, 0);
  }
}

// Resident blocks per CU of a family of instantiations (the smallest; queried once per family).
static int min_occupancy(const void* const* fs, int n) {
  int o = 1 << 20;
  for (int i = 0; i < n; ++i) {
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, fs[i], 256, 0) != hipSuccess || v < 1) v = 1;
    o = v < o ? v : o;
  }
  return o;
}

// Blocks of a persistent grid: every resident slot once, at most one block per 4 tiles.  The
// count depends only on M and the (fixed) occupancy, so the partial-row count a caller
// allocates for is the count the launch uses, and the summation order is reproducible.
static int grid_blocks(int M, int occ) {
  const int ntiles = (M + TR - 1) / TR;
  const int want = (ntiles + WAVES - 1) / WAVES;
  const int slots = occ * 256;
  return want < slots ? (want > 0 ? want : 1) : slots;
}

int dgrad_blocks(int M) {
  // thread-safe one-time query (a function-local static initialised once)
  static const int occ = [] {
    const void* fs[] = {reinterpret_cast<const void*>(&dgrad_bnbwd_kernel<false, false>),
                        reinterpret_cast<const void*>(&dgrad_bnbwd_kernel<false, true>),
                        reinterpret_cast<const void*>(&dgrad_bnbwd_kernel<true, false>),
                        reinterpret_cast<const void*>(&dgrad_bnbwd_kernel<true, true>)};
    return min_occupancy(fs, 4);
  }();
  return grid_blocks(M, occ);
}

template <int KR_>
static int fwd_occ() {
  // thread-safe one-time query (a function-local static initialised once)
  static const int occ = [] {
    const void* fs[] = {reinterpret_cast<const void*>(&fwd_kernel<KR_, KR_, true, true, true>),
                        reinterpret_cast<const void*>(&fwd_kernel<KR_, KR_, true, true, false>),
                        reinterpret_cast<const void*>(&fwd_kernel<KR_, KR_, true, false, true>),
                        reinterpret_cast<const void*>(&fwd_kernel<KR_, KR_, true, false, false>),
                        reinterpret_cast<const void*>(&fwd_kernel<KR_, KR_, false, true, true>),
                        reinterpret_cast<const void*>(&fwd_kernel<KR_, KR_, false, true, false>),
                        reinterpret_cast<const void*>(&fwd_kernel<KR_, KR_, false, false, true>),
                        reinterpret_cast<const void*>(&fwd_kernel<KR_, KR_, false, false, false>)};
    return min_occupancy(fs, 8);
  }();
  return occ;
}

int fwd_blocks(int M, int KC) { return grid_blocks(M, KC == 128 ? fwd_occ<128>() : fwd_occ<64>()); }

// ---------------------------------------------------------------------------------------
// dk_pwconv_bwd_bnbwd_f32 at K = C = 64: the whole backward of a stride-1 pointwise layer whose
// output fed a BatchNorm (+ReLU) in one pass (layers/pointwise_convolution.py:57-75 +
// layers/batch_norm.py:125-174): dy = that BN's backward applied to g on load (never stored),
// dx = dy . W (+ residual) with the input BN's backward partials, and the weight gradient
// dW = dy^T . bn(x) accumulated in registers over every tile of the wave.
//   * dgrad as dgrad_bnbwd_kernel (bit-identical dx);
//   * wgrad on v_mfma_f32_32x32x2_f32 with the pixel (reduction) index in MFMA k: for MFMA r the
//     lane half h supplies pixel (r&3) + 8(r>>2) + 4h -- exactly the rows of the C layout, so the
//     input x values the dx epilogue loads for the partials (column 32u + l32 on the lane) ARE
//     the wgrad's B operand; the A operand dy[pixel][32t + l32] is read back from the wave's LDS
//     image of the dy tile (written once per tile, 16-byte stores);
//   * one wave per SIMD (acc dgrad 32 + acc wgrad 64 registers), a tile of operands in flight;
//   * each block leaves one 64 x 64 partial weight gradient (its waves summed in a fixed order)
//     in ws; splitk_reduce folds them in a fixed order and adds l2 * W.
// Bytes per pixel: g, x_out, x_in read, dx written (+ residual read): the unfused pair also
// writes dy and reads dy and x_in again.
// ---------------------------------------------------------------------------------------
struct BwdArgs {
  DgradArgs d;       // g, xo, (dy_out unused), w, dx, res, xi (required), BN params, part, M
  const float* bm;   // the input BN applied to x for the weight gradient (nullable: raw x)
  const float* bis;
  const float* bg;
  const float* bb;
  int brelu;
  float* wpart;      // [gridDim.x][KR][NO]
  // lattice (ls > 1): a stride-ls pointwise layer whose input gradient stays the compact lattice
  // (pointwise_convolution.py:68-72 without the zeros): pixel m of g / dx is output pixel (n, oh, ow)
  // of an lOH x lOW grid, and x (the layer input, lH x lW) is read at (n, ls oh, ls ow)
  int ls, lH, lW, lOH, lOW;
};

constexpr int SKD = KR + 4;  // row stride of the wave's dy image

// PF: prefetch the next tile's A operands (g, x of the following BN) into registers during this
// tile (one wave per SIMD: 256 VGPRs + 88 AGPRs); !PF: load them at the top of each tile and let a
// second wave on the SIMD cover the latency (2 waves per SIMD).
template <bool RES, bool PART, bool BNIN, bool PF = true, bool LAT = false>
__global__ __launch_bounds__(256, PF ? 1 : 2) void bwd_fused_kernel(BwdArgs ba) {
  static_assert(!LAT || (!RES && BNIN), "the lattice form: no residual, the input BN on load");
  const DgradArgs& a = ba.d;
  __shared__ float Bs[NO * SKB];
  __shared__ float tab[7][KR];
  __shared__ double red[WAVES][2][NO];
  __shared__ float Td[WAVES][TR * SKD];  // per-wave dy tile image (also the dW combine buffer)
  __shared__ uint32_t rowoff[WAVES][TR];  // lattice: byte offset of each tile pixel's input row in x

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  for (int i = tid; i < KR * NO; i += 256) {
    const int k = i / NO, c = i - k * NO;
    Bs[c * SKB + k] = a.w[i];
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
  const bool orelu = a.orelu != 0, irelu = a.irelu != 0, brelu = ba.brelu != 0;
  // this lane's two columns 32u + l32: the input BN (partials) and the wgrad operand's BN
  float pm[2], pis[2], pga[2], pbe[2], qm[2], qis[2], qga[2], qbe[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = 32 * u + l32;
    pm[u] = PART ? a.im[c] : 0.f;
    pis[u] = PART ? a.iis[c] : 0.f;
    pga[u] = PART ? a.ig[c] : 0.f;
    pbe[u] = PART ? a.ib[c] : 0.f;
    qm[u] = BNIN ? ba.bm[c] : 0.f;
    qis[u] = BNIN ? ba.bis[c] : 0.f;
    qga[u] = BNIN ? ba.bg[c] : 0.f;
    qbe[u] = BNIN ? ba.bb[c] : 0.f;
  }
  const f32x2 qm2 = {qm[0], qm[1]}, qis2 = {qis[0], qis[1]}, qga2 = {qga[0], qga[1]}, qbe2 = {qbe[0], qbe[1]};
  __syncthreads();

  const uint32_t kbytes = (uint32_t)a.M * KR * 4u, nbytes = (uint32_t)a.M * NO * 4u;
  const __amdgpu_buffer_rsrc_t rg = make_rsrc_v(a.g, kbytes), rx = make_rsrc_v(a.xo, kbytes);
  constexpr bool lat = LAT;
  const uint32_t xibytes = lat ? (uint32_t)(a.M / (ba.lOH * ba.lOW)) * ba.lH * ba.lW * NO * 4u : nbytes;
  const __amdgpu_buffer_rsrc_t rxi = make_rsrc_v(a.xi, xibytes);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc_v(RES ? a.res : a.g, RES ? nbytes : 0u);
  const __amdgpu_buffer_rsrc_t rdx = make_rsrc_v(a.dx, nbytes);
  const int ntiles = (a.M + TR - 1) / TR;
  const int W = gridDim.x * WAVES;
  int t = blockIdx.x * WAVES + wave;
  float* const td = &Td[wave][0];

  double ps[2] = {0.0, 0.0}, pq[2] = {0.0, 0.0};
  f32x16 aw[2][2];  // weight gradient: rows k = 32t + (C-layout row), columns c = 32u + l32
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) aw[i][u][r] = 0.f;

  // the tile's g and x rows as whole 1 KB wave loads: load q gives lane (pr, cq) = (lane / 16, lane % 16)
  // pixel pr + 4q, channels 4cq .. 4cq + 3 (the MFMA operand layout comes back from the LDS dy image)
  const int pr = lane >> 4, cq = lane & 15;
  auto load_a = [&](int tile, f32x4* lg, f32x4* lx) {
    const uint32_t base = row_off_bytes(tile * TR, KR, 0) + 16u * lane;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      lg[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)(base + 1024u * q), 0, 0));
      lx[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(base + 1024u * q), 0, 0));
    }
  };
  // PF: the tile loop is unrolled by two and the current / prefetched registers swap roles by name
  // (copied at the loop latch, the copy waited for the prefetch's loads)
  f32x4 ga_[KQ], xa_[KQ], gb_[KQ], xb_[KQ];
  if constexpr (PF) {
    load_a(t, ga_, xa_);
    drain_vmem_loads();
  }
  auto tile = [&](f32x4 (&cg)[KQ], f32x4 (&cx)[KQ], f32x4 (&ng)[KQ], f32x4 (&nx)[KQ]) __attribute__((always_inline)) {
    const int m0 = t * TR;
    int z = 0;
    asm volatile("" : "+s"(z));
    const float* tb = &tab[0][0] + z;
    const float* bs = Bs + z;
    if constexpr (!PF) load_a(t, cg, cx);

    // (1) tile t's x (and residual) in the C layout, tile t+W's A operands
    float exi[2][16], ers[2][16];
    const int mb = m0 + 4 * h;
    const uint32_t eb0 = row_off_bytes(mb, NO, l32), eb1 = eb0 + 16u * NO * 4u;
    if constexpr (lat) {  // this tile's input rows, one per lane of the low half; LDS is in order per wave
      if (h == 0) {
        const int m = m0 + l32;
        uint32_t off = kOOBBytes;
        if (m < a.M) {
          const int ow = m % ba.lOW, q = m / ba.lOW, oh = q % ba.lOH, n = q / ba.lOH;
          off = (uint32_t)((n * ba.lH + ba.ls * oh) * ba.lW + ba.ls * ow) * (uint32_t)(NO * 4);
        }
        rowoff[wave][l32] = off;
      }
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t imm = (uint32_t)(((r & 3) + 8 * ((r >> 2) & 1)) * NO + 32 * u) * 4u;
        const uint32_t eb = r < 8 ? eb0 : eb1;
        const uint32_t xoff =
            lat ? rowoff[wave][4 * h + (r & 3) + 8 * (r >> 2)] + (uint32_t)(32 * u + l32) * 4u : eb + imm;
        exi[u][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rxi, (int)xoff, 0, 0));
        if constexpr (RES)
          ers[u][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, (int)(eb + imm), 0, 0));
      }
    if constexpr (PF) load_a(t + W, ng, nx);
    __builtin_amdgcn_sched_barrier(0);

    // (2) dy (bit-identical to dk_bn_bwd_apply_f32) into the wave's LDS image, whose rows give back
    //     the MFMA operand layout (lane (l32, h): pixel l32, channels 8q + 4h ..)
    {
      const int k0 = 4 * cq;  // this lane's channels, the same for every q
      const f32x4 mu = ld4(tb + 0 * KR + k0), is = ld4(tb + 1 * KR + k0), ga = ld4(tb + 2 * KR + k0),
                  be = ld4(tb + 3 * KR + k0);
      const f32x4 k1 = ld4(tb + 4 * KR + k0), k2 = ld4(tb + 5 * KR + k0), f = ld4(tb + 6 * KR + k0);
      // in packed fp32 (v_pk_*: per element the IEEE operations of bn_out / bn_bwd_elem, bit-identical):
      // this transform is a third of the kernel's VALU work, and f32 VALU does not overlap the MFMAs
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        const f32x4 xv = cx[q];
        f32x4 gv = cg[q];
        const f32x2 xh0 = (lo2(xv) - lo2(mu)) * lo2(is), xh1 = (hi2(xv) - hi2(mu)) * hi2(is);
        if (orelu) {
          const f32x2 b0 = __builtin_elementwise_fma(lo2(ga), xh0, lo2(be)),
                      b1 = __builtin_elementwise_fma(hi2(ga), xh1, hi2(be));
          gv[0] = b0[0] > 0.f ? gv[0] : 0.f;
          gv[1] = b0[1] > 0.f ? gv[1] : 0.f;
          gv[2] = b1[0] > 0.f ? gv[2] : 0.f;
          gv[3] = b1[1] > 0.f ? gv[3] : 0.f;
        }
        const f32x2 o0 = lo2(f) * __builtin_elementwise_fma(-xh0, lo2(k2), lo2(gv) - lo2(k1));
        const f32x2 o1 = hi2(f) * __builtin_elementwise_fma(-xh1, hi2(k2), hi2(gv) - hi2(k1));
        st4(td + (pr + 4 * q) * SKD + k0, f32x4{o0[0], o0[1], o1[0], o1[1]});
      }
    }
    f32x4 af[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) af[q] = ld4(td + l32 * SKD + 8 * q + 4 * h);

    // (3) dgrad: dx tile = dy . W (no scheduling barrier around (2)-(4): the transform of
    //     q + 1, the wgrad operand work and the epilogue VALU fill the MFMA issue gaps of the
    //     wave, the only one on its SIMD)
    f32x16 acc[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      f32x4 bf[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) bf[u] = ld4(bs + (32 * u + l32) * SKB + 8 * q + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q][e], bf[u][e], acc[u], 0, 0, 0);
    }

    // (4) per pixel pair r: wgrad aw[t][u] += dy[pixels]^T . bn(x)[pixels] (pixels past M contribute
    //     nothing), then (5) the dx epilogue rows of register r (+ residual) and the input BN's
    //     partials.  PF: one branch on the stores' cache policy around all of it (chosen per store,
    //     the branches hid the stores in flight from the wait-count pass: the next tile's loads
    //     waited for every store of this one)
    auto epi = [&](auto pol) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int dm = (r & 3) + 8 * (r >> 2);
      const bool in = mb + dm < a.M;
      // the input BN's x_hat and output of the pixel, computed once: the weight gradient's operand uses
      // them and so do the partials (PART implies BNIN, and the entry points pass the one BatchNorm for
      // both -- pw_stream_bwd_fused checks), in bn_out's exact form (bit-identical), the two columns
      // in packed fp32
      float bx[2], bxh[2], bo[2];
      f32x2 bxh2 = {0.f, 0.f}, bo2 = {0.f, 0.f};
      if constexpr (BNIN) {
        bxh2 = (f32x2{exi[0][r], exi[1][r]} - qm2) * qis2;
        bo2 = __builtin_elementwise_fma(qga2, bxh2, qbe2);  // = bn_out(v, qm, qis, qga, qbe)
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float v = exi[u][r];
        bxh[u] = bxh2[u];
        bo[u] = bo2[u];
        if constexpr (BNIN) v = (brelu & !(bo[u] > 0.f)) ? 0.f : bo[u];
        bx[u] = in ? v : 0.f;
      }
      const float a0 = td[(dm + 4 * h) * SKD + l32], a1 = td[(dm + 4 * h) * SKD + 32 + l32];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        aw[0][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bx[u], aw[0][u], 0, 0, 0);
        aw[1][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bx[u], aw[1][u], 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint32_t imm = (uint32_t)(((r & 3) + 8 * ((r >> 2) & 1)) * NO + 32 * u) * 4u;
        float v = acc[u][r];
        if constexpr (RES) v += ers[u][r];
        if constexpr (decltype(pol)::value >= 0)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rdx, (int)((r < 8 ? eb0 : eb1) + imm),
                                                0, decltype(pol)::value);
        else if (a.nt)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rdx, (int)((r < 8 ? eb0 : eb1) + imm),
                                                0, 2);
        else
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rdx, (int)((r < 8 ? eb0 : eb1) + imm),
                                                0, 0);
        if constexpr (PART) {
          const float xh = bxh[u];
          // the ReLU / past-M kill as fp32 selects, kept ahead of the widening (the compiler sank the
          // select past it: a 0/1 mask built in VGPRs, then two selects on the fp64 halves)
          float gv = (irelu && !(bo[u] > 0.f)) ? 0.f : v;
          gv = in ? gv : 0.f;
          asm volatile("" : "+v"(gv));
          ps[u] += (double)gv;
          pq[u] += (double)gv * (double)xh;
        }
      }
    }
    };
    if constexpr (!PF)
      // nontemporal dx stores always (the default, kNtPwsBwd): a run-time choice per store put a branch
      // around each of the tile's 32 stores, and hoisted around the epilogue it cost this variant 512
      // bytes of spills
      epi(std::integral_constant<int, 2>{});
    else if (a.nt)
      epi(std::integral_constant<int, 2>{});
    else
      epi(std::integral_constant<int, 0>{});
  };
  if constexpr (PF) {
    while (t < ntiles) {
      tile(ga_, xa_, gb_, xb_);
      t += W;
      if (t >= ntiles) break;
      tile(gb_, xb_, ga_, xa_);
      t += W;
    }
  } else {
    for (; t < ntiles; t += W) tile(ga_, xa_, gb_, xb_);
  }

  // the block's weight-gradient partial: the 4 waves summed in order through LDS
  __syncthreads();
  float* const wb = &Td[0][0];  // [KR][NO + 1]
#pragma unroll 1
  for (int w = 0; w < WAVES; ++w) {
    if (wave == w) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float* p = wb + (32 * i + (r & 3) + 8 * (r >> 2) + 4 * h) * (NO + 1) + 32 * u + l32;
            *p = (w == 0) ? aw[i][u][r] : *p + aw[i][u][r];
          }
    }
    __syncthreads();
  }
  for (int i = tid; i < KR * NO; i += 256) {
    const int k = i / NO, c = i - k * NO;
    ba.wpart[(size_t)blockIdx.x * KR * NO + i] = wb[k * (NO + 1) + c];
  }
  if constexpr (PART) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      ps[u] += __shfl_xor(ps[u], 32, 64);
      pq[u] += __shfl_xor(pq[u], 32, 64);
      if (h == 0) {
        red[wave][0][32 * u + l32] = ps[u];
        red[wave][1][32 * u + l32] = pq[u];
      }
    }
    __syncthreads();
    if (tid < 2 * NO) {
      const int which = tid / NO, c = tid - which * NO;
      double s2 = 0.0;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) s2 += red[w][which][c];
      pub_store(a.part + ((size_t)blockIdx.x * 2 + which) * NO + c, s2);
    }
    if (a.ft.part) fold_tail<256>(a.ft, blockIdx.x, 0, NO, 0);
  }
}

// The backward's A-operand prefetch: off (2 waves per SIMD; whole step 9.12 -> 9.02 ms,
// scripts/ab_step.py, r03) except in the residual and lattice variants, which spill without it.
static int bwd_fused_occ() {
  // thread-safe one-time query (a function-local static initialised once)
  static const int occ = [] {
    const void* fs[] = {reinterpret_cast<const void*>(&bwd_fused_kernel<false, true, true, false>),
                        reinterpret_cast<const void*>(&bwd_fused_kernel<false, false, true, false>),
                        reinterpret_cast<const void*>(&bwd_fused_kernel<false, false, false, false>)};
    return min_occupancy(fs, 3);
  }();
  return occ;
}

int bwd_fused_blocks(int M) { return grid_blocks(M, bwd_fused_occ()); }
// (the grid of a residual variant, which always prefetches, follows the same count: a block count
// above its occupancy only adds a second partial round of blocks, never changes the results' order)
}  // namespace pws

// knob kKnobPwStream (default on; kind 3)
bool pw_stream_enabled() { return knob(kKnobPwStream) == 1; }

// Shapes the streaming dgrad takes (the rest go to the tiled engine).
bool pw_stream_dgrad_ok(int K, int C, int M) {
  if (!pw_stream_enabled()) return false;
  return K == pws::KR && C == pws::NO && M > 0 && (size_t)M * 64 * 4 < ((size_t)1 << 31);
}

int pw_stream_dgrad_rows(int M) { return pws::dgrad_blocks(M); }

bool pw_stream_fwd_ok(int K, int C, int M, size_t xbytes) {
  if (!pw_stream_enabled()) return false;
  const bool shape = (K == 64 && C == 64) || (K == 128 && C == 128);
  return shape && M > 0 && xbytes < ((size_t)1 << 31) && (size_t)M * K * 4 < ((size_t)1 << 31);
}
int pw_stream_fwd_rows(int M, int K) { return pws::fwd_blocks(M, K); }

bool pw_stream_bwd_ok(int K, int C, int M) { return pw_stream_dgrad_ok(K, C, M); }
int pw_stream_bwd_rows(int M) { return pws::bwd_fused_blocks(M); }

int pw_stream_bwd_fused(const float* g, const float* bn_x, int M, const float* om, const float* ois,
                        const float* og, const float* ob, int orelu, const float* k12, const float* w, float* dx,
                        const float* res, const float* x, const float* im, const float* iis, const float* ig,
                        const float* ib, int irelu, double* part, const float* bm, const float* bis,
                        const float* bgm, const float* bbt, int brelu, float* wpart, hipStream_t st,
                        const FoldTail* ft, const int* lattice) {
  pws::BwdArgs a{{g, bn_x, nullptr, w, dx, res, x, om, ois, og, ob, k12, orelu, im, iis, ig, ib, irelu, part, M},
                 bm, bis, bgm, bbt, brelu, wpart, 0, 0, 0, 0, 0};
  if (lattice) {  // {stride, H, W, OH, OW}
    if (res || !bm || lattice[0] < 2) return DK_ERR_ARGS;
    a.ls = lattice[0];
    a.lH = lattice[1];
    a.lW = lattice[2];
    a.lOH = lattice[3];
    a.lOW = lattice[4];
  }
  if (ft && part) a.d.ft = *ft;
  a.d.nt = nt_stores(kNtPwsBwd);
  const dim3 grid(pws::bwd_fused_blocks(M));
  const bool r = res != nullptr, pt = part != nullptr, bn = bm != nullptr;
  if (pt && !bn) return DK_ERR_ARGS;
  // the partials' BatchNorm is the weight-gradient operand's (the kernel computes its terms once)
  if (pt && (im != bm || iis != bis || ig != bgm || ib != bbt || (irelu != 0) != (brelu != 0))) return DK_ERR_ARGS;
  if (lattice) {  // (the lattice form keeps the prefetch: without it it spills at 2 waves per SIMD)
    if (pt)
      hipLaunchKernelGGL((pws::bwd_fused_kernel<false, true, true, true, true>), grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((pws::bwd_fused_kernel<false, false, true, true, true>), grid, dim3(256), 0, st, a);
    return launch_status();
  }
  // (the residual variants keep the prefetch: without it they spill at 2 waves per SIMD)
#define DK_BWD(R_, P_, B_) hipLaunchKernelGGL((pws::bwd_fused_kernel<R_, P_, B_, R_>), grid, dim3(256), 0, st, a)
  if (pt) {
    if (r) {
      DK_BWD(true, true, true);
    } else {
      DK_BWD(false, true, true);
    }
  } else if (bn) {
    if (r) {
      DK_BWD(true, false, true);
    } else {
      DK_BWD(false, false, true);
    }
  } else {
    if (r) {
      DK_BWD(true, false, false);
    } else {
      DK_BWD(false, false, false);
    }
  }
#undef DK_BWD
  return launch_status();
}

int pw_stream_fwd(const float* x, int N, int H, int W, int stride, int OH, int OW, const float* w, int KC,
                  const float* bias, float* y, const float* im, const float* iis, const float* ig,
                  const float* ib, int irelu, double* part, hipStream_t st, const FoldTail* ft) {
  if (KC != 64 && KC != 128) return DK_ERR_ARGS;
  const int M = N * OH * OW;
  pws::FwdArgs a{x, w, bias, y, im, iis, ig, ib, irelu, part, M, H, W, OH, OW, stride,
                 (uint32_t)((size_t)N * H * W * KC * 4)};
  if (ft && part) a.ft = *ft;
  a.nt = nt_stores(kNtPwsFwd);
  const dim3 grid(pws::fwd_blocks(M, KC));
  const bool strided = stride != 1;
#define DK_FWD(BN_, ST_)                                                                                \
  if (KC == 128) {                                                                                      \
    if (strided)                                                                                        \
      hipLaunchKernelGGL((pws::fwd_kernel<128, 128, BN_, ST_, true>), grid, dim3(256), 0, st, a);       \
    else                                                                                                \
      hipLaunchKernelGGL((pws::fwd_kernel<128, 128, BN_, ST_, false>), grid, dim3(256), 0, st, a);      \
  } else if (strided)                                                                                   \
    hipLaunchKernelGGL((pws::fwd_kernel<64, 64, BN_, ST_, true>), grid, dim3(256), 0, st, a);           \
  else                                                                                                  \
    hipLaunchKernelGGL((pws::fwd_kernel<64, 64, BN_, ST_, false>), grid, dim3(256), 0, st, a);
  if (im && part) {
    DK_FWD(true, true)
  } else if (im) {
    DK_FWD(true, false)
  } else if (part) {
    DK_FWD(false, true)
  } else {
    DK_FWD(false, false)
  }
#undef DK_FWD
  return launch_status();
}

int pw_stream_dgrad_bnbwd(const float* g, const float* bn_x, int M, const float* om, const float* ois,
                          const float* og, const float* ob, int orelu, const float* k12, float* dy_out,
                          const float* w, float* dx, const float* res, const float* x, const float* im,
                          const float* iis, const float* ig, const float* ib, int irelu, double* part,
                          hipStream_t st, const FoldTail* ft) {
  pws::DgradArgs a{g, bn_x, dy_out, w, dx, res, x, om, ois, og, ob, k12, orelu, im, iis, ig, ib, irelu, part, M};
  if (ft && part) a.ft = *ft;
  a.nt = nt_stores(kNtPwsDgrad);
  const dim3 grid(pws::dgrad_blocks(M));
  if (res && x)
    hipLaunchKernelGGL((pws::dgrad_bnbwd_kernel<true, true>), grid, dim3(256), 0, st, a);
  else if (res)
    hipLaunchKernelGGL((pws::dgrad_bnbwd_kernel<true, false>), grid, dim3(256), 0, st, a);
  else if (x)
    hipLaunchKernelGGL((pws::dgrad_bnbwd_kernel<false, true>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((pws::dgrad_bnbwd_kernel<false, false>), grid, dim3(256), 0, st, a);
  return launch_status();
}

}  // namespace dk
