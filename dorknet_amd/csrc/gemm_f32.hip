// Implicit-GEMM engine on fp32 MFMA (v_mfma_f32_32x32x2_f32) for gfx950.
//
// Every dense contraction on the hot path is one instance of
//     C[m][n] (+)= sum_k  A(m, k) * B(n, k)
// where A and B are *views* of NHWC activations / weights, never materialised:
//   * conv forward  (replaces im2col + cp.dot, layers/convolution.py:58-87, :187-203)
//       m = output pixel (n,oh,ow), n = output channel, k = (r,s,c) with c innermost
//   * conv dgrad    (replaces cp.dot + row2im, convolution.py:101-117, :205-222)
//       stride 1: m = input pixel, k = (r,s,k_out), A gathers dy at (h+p-r, w+p-s)
//       stride >1: dx_cols = dy_rows . W_flat (a plain GEMM) + a deterministic col2im gather
//   * conv wgrad    (replaces cp.dot(upstream.T, patches), convolution.py:93-100)
//       m = output channel, n = (r,s,c), k = output pixel; split-K over pixels with a
//       fixed-order second stage (no atomics, deterministic)
//   * pointwise fwd/dgrad/wgrad (layers/pointwise_convolution.py:46-75) as the
//       R=S=1 case; stride-2 subsampling is a strided gather, the backward "widen"
//       is fused into the epilogue
//   * dense fwd/dgrad/wgrad (layers/dense_layer.py:46-67)
//
// Tiles are staged global -> registers -> LDS with one tile of register prefetch
// and two LDS buffers (one barrier per K-tile).  In LDS every operand tile is
// stored k-major ([BK][rows], rows contiguous), so an MFMA operand fetch is one
// conflict-free ds_read_b32 per lane: lanes 0-31 read k, lanes 32-63 read k+1.
#include "dk_common.h"

namespace dk {

// ----------------------------------------------------------------------------
// Operand descriptors
// ----------------------------------------------------------------------------

// Implicit-im2col view of an NHWC tensor x[n][ih][iw][c] (C % 4 == 0).
// Row/pixel index m -> (n, oh, ow) over an OH x OW grid; tap (r,s) reads
// (ih, iw) = (oh*sa + dr*r + off, ow*sa + dr*s + off), zero outside [0,H)x[0,W).
struct ImgDesc {
  const float* x;
  int H, W, C;
  int OH, OW;
  int R, S;
  int sa, dr, off;
  int M;  // N * OH * OW
};

// Row-major matrix p[row][ld]; `ext` bounds the non-reduction index.
struct MatDesc {
  const float* p;
  int ld;
  int ext;
  int vec;  // 1 when float4 loads are legal (ld, ext/Ktot and base 16B aligned)
};

// ----------------------------------------------------------------------------
// Loaders: each fills an LDS tile T[BK][S] (S >= ROWS, row = k).
// ----------------------------------------------------------------------------

// Source is k-contiguous (rows = i): im2col rows of an NHWC image.
template <int ROWS, int BK, int NT>
struct LdImgKC {
  static constexpr int KQ = BK / 4;
  static constexpr int RSTEP = NT / KQ;
  static constexpr int NR = ROWS >= RSTEP ? ROWS / RSTEP : 1;
  static constexpr int S = ROWS + 2;  // S % 32 == 2: conflict-free transposing writes
  int kq, rb;
  bool active;
  int base[NR], ih0[NR], iw0[NR];
  f32x4 v[NR];

  __device__ __forceinline__ void init(const ImgDesc& d, int row0, int tid) {
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
        iw0[j] = ow * d.sa + d.off;
        base[j] = (n * d.H + ih0[j]) * d.W + iw0[j];
      } else {
        ih0[j] = -(1 << 28);
        iw0[j] = -(1 << 28);
        base[j] = 0;
      }
    }
  }

  __device__ __forceinline__ void load(const ImgDesc& d, int k0, int Ktot) {
    const int k = k0 + 4 * kq;
    const bool kv = k < Ktot;
    const int tap = k / d.C;
    const int c = k - tap * d.C;
    const int r = tap / d.S;
    const int s = tap - r * d.S;
    const int dri = d.dr * r, dsi = d.dr * s;
    const int doff = dri * d.W + dsi;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int ih = ih0[j] + dri, iw = iw0[j] + dsi;
      const bool ok = kv && (unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W;
      v[j] = ok ? ld4(d.x + (size_t)(base[j] + doff) * d.C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }

  __device__ __forceinline__ void store(float* t) const {
    if (!active) return;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int row = rb + j * RSTEP;
#pragma unroll
      for (int e = 0; e < 4; ++e) t[(4 * kq + e) * S + row] = v[j][e];
    }
  }
};

// Source is k-contiguous row-major matrix p[i][ld] (k along the row).
template <int ROWS, int BK, int NT>
struct LdMatKC {
  static constexpr int KQ = BK / 4;
  static constexpr int RSTEP = NT / KQ;
  static constexpr int NR = ROWS >= RSTEP ? ROWS / RSTEP : 1;
  static constexpr int S = ROWS + 2;
  int kq, rb, row0;
  bool active;
  f32x4 v[NR];

  __device__ __forceinline__ void init(const MatDesc& d, int row0_, int tid) {
    kq = tid % KQ;
    rb = tid / KQ;
    row0 = row0_;
    active = rb < ROWS;
  }

  __device__ __forceinline__ void load(const MatDesc& d, int k0, int Ktot) {
    const int k = k0 + 4 * kq;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int i = row0 + rb + j * RSTEP;
      const bool iv = active && i < d.ext;
      if (d.vec) {
        v[j] = (iv && k < Ktot) ? ld4(d.p + (size_t)i * d.ld + k) : f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][e] = (iv && k + e < Ktot) ? d.p[(size_t)i * d.ld + k + e] : 0.f;
      }
    }
  }

  __device__ __forceinline__ void store(float* t) const {
    if (!active) return;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int row = rb + j * RSTEP;
#pragma unroll
      for (int e = 0; e < 4; ++e) t[(4 * kq + e) * S + row] = v[j][e];
    }
  }
};

// Source is i-contiguous row-major matrix p[k][ld] (i along the row).
template <int ROWS, int BK, int NT>
struct LdMatIC {
  static constexpr int IQ = ROWS / 4;
  static constexpr int KSTEP = NT / IQ;
  static constexpr int NK = BK >= KSTEP ? BK / KSTEP : 1;
  static constexpr int S = ROWS;
  int iq, kb, i0;
  bool active;
  f32x4 v[NK];

  __device__ __forceinline__ void init(const MatDesc& d, int row0, int tid) {
    iq = tid % IQ;
    kb = tid / IQ;
    i0 = row0 + 4 * iq;
    active = kb < BK;
  }

  __device__ __forceinline__ void load(const MatDesc& d, int k0, int Ktot) {
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int k = k0 + kb + j * KSTEP;
      const bool kv = active && k < Ktot;
      if (d.vec) {
        v[j] = (kv && i0 < d.ext) ? ld4(d.p + (size_t)k * d.ld + i0) : f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[j][e] = (kv && i0 + e < d.ext) ? d.p[(size_t)k * d.ld + i0 + e] : 0.f;
      }
    }
  }

  __device__ __forceinline__ void store(float* t) const {
    if (!active) return;
#pragma unroll
    for (int j = 0; j < NK; ++j) st4(t + (kb + j * KSTEP) * S + 4 * iq, v[j]);
  }
};

// Source is an implicit-im2col image, i = (r,s,c) (c innermost), k = pixel.
// Used by wgrad: B(i=(r,s,c), k=m) = x[pixel(m) shifted by tap (r,s)][c].
template <int ROWS, int BK, int NT>
struct LdImgIC {
  static constexpr int IQ = ROWS / 4;
  static constexpr int KSTEP = NT / IQ;
  static constexpr int NK = BK >= KSTEP ? BK / KSTEP : 1;
  static constexpr int S = ROWS;
  int iq, kb;
  bool active, colv;
  int c, dri, dsi;
  f32x4 v[NK];

  __device__ __forceinline__ void init(const ImgDesc& d, int row0, int tid) {
    iq = tid % IQ;
    kb = tid / IQ;
    active = kb < BK;
    const int j = row0 + 4 * iq;
    colv = j < d.R * d.S * d.C;
    const int tap = j / d.C;
    c = j - tap * d.C;
    const int r = tap / d.S;
    const int s = tap - r * d.S;
    dri = d.dr * r;
    dsi = d.dr * s;
  }

  __device__ __forceinline__ void load(const ImgDesc& d, int k0, int Ktot) {
#pragma unroll
    for (int jj = 0; jj < NK; ++jj) {
      const int m = k0 + kb + jj * KSTEP;
      bool ok = active && colv && m < d.M;
      int ih = 0, iw = 0, n = 0;
      if (ok) {
        const int ow = m % d.OW;
        const int t = m / d.OW;
        const int oh = t % d.OH;
        n = t / d.OH;
        ih = oh * d.sa + dri + d.off;
        iw = ow * d.sa + dsi + d.off;
        ok = (unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W;
      }
      v[jj] = ok ? ld4(d.x + ((size_t)(n * d.H + ih) * d.W + iw) * d.C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }

  __device__ __forceinline__ void store(float* t) const {
    if (!active) return;
#pragma unroll
    for (int j = 0; j < NK; ++j) st4(t + (kb + j * KSTEP) * S + 4 * iq, v[j]);
  }
};

// ----------------------------------------------------------------------------
// Epilogues
// ----------------------------------------------------------------------------

// out[row(m)][n] = acc (+ bias[n]).  With st > 1 the GEMM row m = (b, oh, ow) of
// an OH x OW grid lands at (b, oh*st, ow*st) of an (OH*st) x (OW*st) grid and
// the other st*st-1 positions of that cell are written as zeros: this is the
// pointwise stride-s backward "widen" (pointwise_convolution.py:68-72) fused.
struct EpStore {
  float* out;
  int ldo;
  const float* bias;
  int OH, OW, st;
  __device__ __forceinline__ void put(int m, int n, float v, int) const {
    if (bias) v += bias[n];
    if (st == 1) {
      out[(size_t)m * ldo + n] = v;
    } else {
      const int ow = m % OW;
      const int t = m / OW;
      const int oh = t % OH;
      const int b = t / OH;
      const int OW2 = OW * st, OH2 = OH * st;
      const size_t cell = (size_t)(b * OH2 + oh * st) * OW2 + (size_t)ow * st;
      for (int dy = 0; dy < st; ++dy)
        for (int dx = 0; dx < st; ++dx)
          out[(cell + (size_t)dy * OW2 + dx) * ldo + n] = (dy | dx) ? 0.f : v;
    }
  }
};

// Split-K partial tile: ws[split][M][N].
struct EpPartial {
  float* ws;
  int M, N;
  __device__ __forceinline__ void put(int m, int n, float v, int split) const {
    ws[((size_t)split * M + m) * N + n] = v;
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
  static_assert(BK % 4 == 0, "BK");
  constexpr int SA = LA::S, SB = LB::S;
  constexpr int ABUF = BK * SA, BBUF = BK * SB;
  __shared__ float smem[2 * (ABUF + BBUF)];
  float* const As = smem;
  float* const Bs = smem + 2 * ABUF;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int l32 = lane & 31, h = lane >> 5;

  const int tiles_n = (N + BN - 1) / BN;
  const int m0 = (blockIdx.x / tiles_n) * BM;
  const int n0 = (blockIdx.x % tiles_n) * BN;
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
    la.load(da, kt0 * BK, Ktot);
    lb.load(db, kt0 * BK, Ktot);
    la.store(As);
    lb.store(Bs);
    __syncthreads();
    int cur = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) {
        la.load(da, (kt + 1) * BK, Ktot);
        lb.load(db, (kt + 1) * BK, Ktot);
      }
      const float* a_t = As + cur * ABUF + h * SA + wm * 32 * TM + l32;
      const float* b_t = Bs + cur * BBUF + h * SB + wn * 32 * TN + l32;
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        float a[TM], b[TN];
#pragma unroll
        for (int t = 0; t < TM; ++t) a[t] = a_t[2 * kk * SA + 32 * t];
#pragma unroll
        for (int u = 0; u < TN; ++u) b[u] = b_t[2 * kk * SB + 32 * u];
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int u = 0; u < TN; ++u)
            acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b[u], acc[t][u], 0, 0, 0);
      }
      if (more) {
        la.store(As + (cur ^ 1) * ABUF);
        lb.store(Bs + (cur ^ 1) * BBUF);
      }
      __syncthreads();
      cur ^= 1;
    }
  }

#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      const int col = n0 + wn * 32 * TN + u * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 32 * TM + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < M && col < N) ep.put(row, col, acc[t][u][r], blockIdx.y);
      }
    }
}

// ----------------------------------------------------------------------------
// Host-side launch helpers and tile selection
// ----------------------------------------------------------------------------

constexpr int kBK = 16;

template <int BM, int BN, int WM, int WN, template <int, int, int> class LA, class DA,
          template <int, int, int> class LB, class DB, class EP>
static int launch_igemm(const DA& da, const DB& db, const EP& ep, int M, int N, int Ktot, int splits,
                        hipStream_t st) {
  constexpr int NT = 64 * WM * WN;
  using A = LA<BM, kBK, NT>;
  using B = LB<BN, kBK, NT>;
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  const int KT = cdiv(Ktot, kBK);
  if (splits < 1) splits = 1;
  if (splits > KT) splits = KT > 0 ? KT : 1;
  const int kps = KT > 0 ? cdiv(KT, splits) : 1;
  splits = KT > 0 ? cdiv(KT, kps) : 1;
  hipLaunchKernelGGL((igemm_f32<BM, BN, kBK, WM, WN, A, DA, B, DB, EP>), dim3(tiles, splits), dim3(NT), 0, st,
                     da, db, ep, M, N, Ktot, kps);
  return launch_status();
}

// Output-stationary problems (fwd / dgrad): tile by the N extent.
template <template <int, int, int> class LA, class DA, template <int, int, int> class LB, class DB, class EP>
static int igemm_rows(const DA& da, const DB& db, const EP& ep, int M, int N, int Ktot, hipStream_t st) {
  if (N <= 32) return launch_igemm<128, 32, 4, 1, LA, DA, LB, DB, EP>(da, db, ep, M, N, Ktot, 1, st);
  if (N <= 64) return launch_igemm<256, 64, 4, 1, LA, DA, LB, DB, EP>(da, db, ep, M, N, Ktot, 1, st);
  if (M <= 4096) return launch_igemm<64, 64, 2, 2, LA, DA, LB, DB, EP>(da, db, ep, M, N, Ktot, 1, st);
  return launch_igemm<128, 128, 2, 2, LA, DA, LB, DB, EP>(da, db, ep, M, N, Ktot, 1, st);
}

// Reduction-heavy problems (wgrad): split K over enough blocks to fill the chip.
static int wgrad_splits(int M, int N, int Kred, int BM, int BN) {
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  const int KT = cdiv(Kred, kBK);
  int splits = cdiv(1024, tiles);
  if (splits > KT) splits = KT;
  if (splits < 1) splits = 1;
  const int kps = cdiv(KT, splits);
  return cdiv(KT, kps);
}

static void wgrad_tile(int M, int N, int* BM, int* BN) {
  if (M >= 128 && N >= 128) {
    *BM = 128;
    *BN = 128;
  } else {
    *BM = 64;
    *BN = 64;
  }
}

template <template <int, int, int> class LA, class DA, template <int, int, int> class LB, class DB>
static int igemm_splitk(const DA& da, const DB& db, float* ws, int M, int N, int Kred, hipStream_t st,
                        int* splits_out) {
  int BM, BN;
  wgrad_tile(M, N, &BM, &BN);
  const int splits = wgrad_splits(M, N, Kred, BM, BN);
  *splits_out = splits;
  EpPartial ep{ws, M, N};
  if (BM == 128) return launch_igemm<128, 128, 2, 2, LA, DA, LB, DB, EpPartial>(da, db, ep, M, N, Kred, splits, st);
  return launch_igemm<64, 64, 2, 2, LA, DA, LB, DB, EpPartial>(da, db, ep, M, N, Kred, splits, st);
}

static size_t splitk_ws_bytes(int M, int N, int Kred) {
  int BM, BN;
  wgrad_tile(M, N, &BM, &BN);
  return (size_t)wgrad_splits(M, N, Kred, BM, BN) * (size_t)M * (size_t)N * sizeof(float);
}

// Second stage of split-K (reduce.hip): fixed-order sum over the partial slabs,
// + l2 * W (regularisers/l2.py:16-17 folded in, as convolution.py:99-100 does), and a
// scatter into the caller's weight layout (mode 0: out[m][n]; mode 1: KCRS from (r,s,c)).

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

// dx[n,h,w,c] = sum over taps (r,s) with h + pad - r = oh*stride (and w likewise) of
// cols[(n,oh,ow)][(c,r,s)] -- the deterministic gather form of row2im
// (convolution.py:205-222, which scatters with atomicAdd).
__global__ void col2im_kernel(const float* __restrict__ cols, int N, int C, int H, int W, int OH, int OW, int R,
                              int S, int stride, int pad, float* __restrict__ dx) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)N * H * W * C;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  long long t = idx / C;
  const int w = (int)(t % W);
  t /= W;
  const int h = (int)(t % H);
  const int n = (int)(t / H);
  const int CRS = C * R * S;
  float acc = 0.f;
  for (int r = 0; r < R; ++r) {
    const int hh = h + pad - r;
    if (hh < 0 || hh % stride) continue;
    const int oh = hh / stride;
    if (oh >= OH) continue;
    for (int s = 0; s < S; ++s) {
      const int ww = w + pad - s;
      if (ww < 0 || ww % stride) continue;
      const int ow = ww / stride;
      if (ow >= OW) continue;
      acc += cols[((size_t)(n * OH + oh) * OW + ow) * CRS + (c * R + r) * S + s];
    }
  }
  dx[idx] = acc;
}

static inline int aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

static inline MatDesc mat(const float* p, int ld, int ext, int kext) {
  MatDesc d{p, ld, ext, 0};
  d.vec = (ld % 4 == 0) && (ext % 4 == 0) && (kext % 4 == 0) && aligned16(p);
  return d;
}

}  // namespace dk

using namespace dk;

// ============================================================================
// C ABI
// ============================================================================

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
DK_API int dk_conv2d_fwd_f32(const float* x, int N, int H, int W, int C, const float* w_krsc, int K, int R, int S,
                             int stride, int pad, const float* bias, float* y, int OH, int OW, void* stream) {
  if (C % 4 || !aligned16(x)) return DK_ERR_ARGS;
  ImgDesc a{x, H, W, C, OH, OW, R, S, stride, 1, -pad, N * OH * OW};
  const int Ktot = R * S * C;
  MatDesc b = mat(w_krsc, Ktot, K, Ktot);
  EpStore ep{y, K, bias, OH, OW, 1};
  return igemm_rows<LdImgKC, ImgDesc, LdMatKC, MatDesc, EpStore>(a, b, ep, N * OH * OW, K, Ktot, as_stream(stream));
}

// Stride-1 dgrad as an implicit GEMM: dx[n,h,w,c] = sum_{r,s,k} dy[n, h+pad-r, w+pad-s, k] * w[k][c][r][s]
DK_API int dk_conv2d_dgrad_f32(const float* dy, int N, int OH, int OW, int K, const float* w_crsk, int C, int R,
                               int S, int pad, float* dx, int H, int W, void* stream) {
  if (K % 4 || !aligned16(dy)) return DK_ERR_ARGS;
  ImgDesc a{dy, OH, OW, K, H, W, R, S, 1, -1, pad, N * H * W};
  const int Ktot = R * S * K;
  MatDesc b = mat(w_crsk, Ktot, C, Ktot);
  EpStore ep{dx, C, nullptr, H, W, 1};
  return igemm_rows<LdImgKC, ImgDesc, LdMatKC, MatDesc, EpStore>(a, b, ep, N * H * W, C, Ktot, as_stream(stream));
}

DK_API size_t dk_conv2d_dgrad_cols_workspace_bytes(int N, int OH, int OW, int C, int R, int S) {
  return (size_t)N * OH * OW * C * R * S * sizeof(float);
}

// Any-stride dgrad: cols = dy_rows . W_flat (GEMM, convolution.py:101-104) then a gather col2im.
DK_API int dk_conv2d_dgrad_strided_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kcrs, int C,
                                       int R, int S, int stride, int pad, float* dx, int H, int W, void* ws,
                                       size_t ws_bytes, void* stream) {
  const int M = N * OH * OW;
  const int CRS = C * R * S;
  if (ws_bytes < dk_conv2d_dgrad_cols_workspace_bytes(N, OH, OW, C, R, S)) return DK_ERR_WORKSPACE;
  float* cols = static_cast<float*>(ws);
  MatDesc a = mat(dy, K, M, K);
  MatDesc b = mat(w_kcrs, CRS, CRS, K);
  EpStore ep{cols, CRS, nullptr, OH, OW, 1};
  int rc = igemm_rows<LdMatKC, MatDesc, LdMatIC, MatDesc, EpStore>(a, b, ep, M, CRS, K, as_stream(stream));
  if (rc) return rc;
  const long long total = (long long)N * H * W * C;
  hipLaunchKernelGGL(col2im_kernel, dim3((unsigned)cdivll(total, 256)), dim3(256), 0, as_stream(stream), cols, N, C,
                     H, W, OH, OW, R, S, stride, pad, dx);
  return launch_status();
}

DK_API size_t dk_conv2d_wgrad_workspace_bytes(int N, int OH, int OW, int K, int Cp, int R, int S) {
  return splitk_ws_bytes(K, R * S * Cp, N * OH * OW);
}

// dw[k][c][r][s] = sum_{n,oh,ow} dy[n,oh,ow,k] * x[n, oh*stride + r - pad, ow*stride + s - pad, c]  (+ l2 * w)
DK_API int dk_conv2d_wgrad_f32(const float* dy, const float* x, int N, int H, int W, int Cp, int C, int K, int R,
                               int S, int stride, int pad, int OH, int OW, const float* w_kcrs, float l2,
                               float* dw_kcrs, void* ws, size_t ws_bytes, void* stream) {
  if (Cp % 4 || !aligned16(x)) return DK_ERR_ARGS;
  const int M = K, Ncol = R * S * Cp, Kred = N * OH * OW;
  if (ws_bytes < splitk_ws_bytes(M, Ncol, Kred)) return DK_ERR_WORKSPACE;
  MatDesc a = mat(dy, K, K, Kred);
  ImgDesc b{x, H, W, Cp, OH, OW, R, S, stride, 1, -pad, Kred};
  int splits = 1;
  int rc = igemm_splitk<LdMatIC, MatDesc, LdImgIC, ImgDesc>(a, b, static_cast<float*>(ws), M, Ncol, Kred,
                                                              as_stream(stream), &splits);
  if (rc) return rc;
  return splitk_reduce(static_cast<float*>(ws), splits, M, Ncol, dw_kcrs, w_kcrs, l2, 1, C, Cp, R, S,
                       as_stream(stream));
}

// Pointwise (1x1) forward with optional stride-s subsampling (pointwise_convolution.py:46-55):
// y[n,oh,ow,k] = sum_c x[n, oh*s, ow*s, c] * w[k][c] (+ bias)
DK_API int dk_pwconv_fwd_f32(const float* x, int N, int H, int W, int C, const float* w_kc, int K, int stride,
                             const float* bias, float* y, int OH, int OW, void* stream) {
  if (C % 4 || !aligned16(x)) return DK_ERR_ARGS;
  ImgDesc a{x, H, W, C, OH, OW, 1, 1, stride, 1, 0, N * OH * OW};
  MatDesc b = mat(w_kc, C, K, C);
  EpStore ep{y, K, bias, OH, OW, 1};
  return igemm_rows<LdImgKC, ImgDesc, LdMatKC, MatDesc, EpStore>(a, b, ep, N * OH * OW, K, C, as_stream(stream));
}

// Pointwise dgrad (pointwise_convolution.py:65-72): dx_rows = dy_rows . W; for stride > 1 the
// result is widened to (OH*s, OW*s) with zeros off the sampling lattice.
DK_API int dk_pwconv_dgrad_f32(const float* dy, int N, int OH, int OW, int K, const float* w_kc, int C, int stride,
                               float* dx, void* stream) {
  if (K % 4 || !aligned16(dy)) return DK_ERR_ARGS;
  ImgDesc a{dy, OH, OW, K, OH, OW, 1, 1, 1, 1, 0, N * OH * OW};
  MatDesc b = mat(w_kc, C, C, K);
  EpStore ep{dx, C, nullptr, OH, OW, stride};
  return igemm_rows<LdImgKC, ImgDesc, LdMatIC, MatDesc, EpStore>(a, b, ep, N * OH * OW, C, K, as_stream(stream));
}

DK_API size_t dk_pwconv_wgrad_workspace_bytes(int N, int OH, int OW, int K, int C) {
  return splitk_ws_bytes(K, C, N * OH * OW);
}

// dw[k][c] = sum_{n,oh,ow} dy[n,oh,ow,k] * x[n, oh*s, ow*s, c]  (+ l2 * w)   (pointwise_convolution.py:61-64)
DK_API int dk_pwconv_wgrad_f32(const float* dy, const float* x, int N, int H, int W, int C, int K, int stride,
                               int OH, int OW, const float* w_kc, float l2, float* dw_kc, void* ws, size_t ws_bytes,
                               void* stream) {
  if (C % 4 || !aligned16(x)) return DK_ERR_ARGS;
  const int Kred = N * OH * OW;
  if (ws_bytes < splitk_ws_bytes(K, C, Kred)) return DK_ERR_WORKSPACE;
  MatDesc a = mat(dy, K, K, Kred);
  ImgDesc b{x, H, W, C, OH, OW, 1, 1, stride, 1, 0, Kred};
  int splits = 1;
  int rc = igemm_splitk<LdMatIC, MatDesc, LdImgIC, ImgDesc>(a, b, static_cast<float*>(ws), K, C, Kred,
                                                              as_stream(stream), &splits);
  if (rc) return rc;
  return splitk_reduce(static_cast<float*>(ws), splits, K, C, dw_kc, w_kc, l2, 0, C, C, 1, 1, as_stream(stream));
}

// Dense (dense_layer.py:46-55): y[b][o] = sum_i x[b][i] * w[i][o] (+ bias[o]);  w stored (in, out).
DK_API int dk_dense_fwd_f32(const float* x, int B, int IN, const float* w_io, int OUT, const float* bias, float* y,
                            void* stream) {
  MatDesc a = mat(x, IN, B, IN);
  MatDesc b = mat(w_io, OUT, OUT, IN);
  EpStore ep{y, OUT, bias, 1, 1, 1};
  return igemm_rows<LdMatKC, MatDesc, LdMatIC, MatDesc, EpStore>(a, b, ep, B, OUT, IN, as_stream(stream));
}

// dx[b][i] = sum_o dy[b][o] * w[i][o]   (dense_layer.py:67)
DK_API int dk_dense_dgrad_f32(const float* dy, int B, int OUT, const float* w_io, int IN, float* dx, void* stream) {
  MatDesc a = mat(dy, OUT, B, OUT);
  MatDesc b = mat(w_io, OUT, IN, OUT);
  EpStore ep{dx, IN, nullptr, 1, 1, 1};
  return igemm_rows<LdMatKC, MatDesc, LdMatKC, MatDesc, EpStore>(a, b, ep, B, IN, OUT, as_stream(stream));
}

DK_API size_t dk_dense_wgrad_workspace_bytes(int B, int IN, int OUT) { return splitk_ws_bytes(IN, OUT, B); }

// dw[i][o] = sum_b x[b][i] * dy[b][o] (+ l2 * w)   (dense_layer.py:61-66)
DK_API int dk_dense_wgrad_f32(const float* x, const float* dy, int B, int IN, int OUT, const float* w_io, float l2,
                              float* dw_io, void* ws, size_t ws_bytes, void* stream) {
  if (ws_bytes < splitk_ws_bytes(IN, OUT, B)) return DK_ERR_WORKSPACE;
  MatDesc a = mat(x, IN, IN, B);
  MatDesc b = mat(dy, OUT, OUT, B);
  int splits = 1;
  int rc = igemm_splitk<LdMatIC, MatDesc, LdMatIC, MatDesc>(a, b, static_cast<float*>(ws), IN, OUT, B,
                                                              as_stream(stream), &splits);
  if (rc) return rc;
  return splitk_reduce(static_cast<float*>(ws), splits, IN, OUT, dw_io, w_io, l2, 0, OUT, OUT, 1, 1,
                       as_stream(stream));
}
