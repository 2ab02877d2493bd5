// Shared helpers for the dorknet_amd HIP library (gfx950 / CDNA4 only).
//
// Conventions of every extern "C" entry point (see include/dorknet_hip.h):
//   * all tensor pointers are device pointers owned by the caller;
//   * activations are NHWC (channels innermost), fp32;
//   * kernels never allocate: scratch comes from a caller-provided workspace
//     whose size is reported by a matching *_workspace_bytes() query;
//   * work is stream-ordered on the caller's stream (a hipStream_t passed as void*);
//   * the return value is a hipError_t cast to int (0 == success).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/dorknet_hip.h"

#define DK_API extern "C" __attribute__((visibility("default")))

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace dk {

// halves of a float4 for packed fp32 (v_pk_mul / v_pk_fma / v_pk_add: two lanes of the same IEEE
// operations per instruction, bit-identical to the scalar form)
__device__ __forceinline__ f32x2 lo2(f32x4 v) { return f32x2{v[0], v[1]}; }
__device__ __forceinline__ f32x2 hi2(f32x4 v) { return f32x2{v[2], v[3]}; }

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline int launch_status() { return static_cast<int>(hipGetLastError()); }

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
static inline long long cdivll(long long a, long long b) { return (a + b - 1) / b; }

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// bf16 storage (BASELINE config 5): activations held as bf16 bits, every kernel computes
// in fp32 -- loads widen (exact), stores round to nearest even (v_cvt_pk_bf16_f32).
typedef uint16_t bf16_t;
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));  // a v_mfma_f32_*_bf16 operand fragment
__device__ __forceinline__ f32x4 bf16x4_to_f32(uint2 u) {
  return __builtin_convertvector(__builtin_bit_cast(bf16x4, u), f32x4);
}
__device__ __forceinline__ uint2 f32_to_bf16x4(f32x4 v) {
  return __builtin_bit_cast(uint2, __builtin_convertvector(v, bf16x4));
}
__device__ __forceinline__ f32x4 ld4(const bf16_t* p) { return bf16x4_to_f32(*reinterpret_cast<const uint2*>(p)); }
__device__ __forceinline__ void st4(bf16_t* p, f32x4 v) { *reinterpret_cast<uint2*>(p) = f32_to_bf16x4(v); }
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const bf16_t* p) {
  return __builtin_bit_cast(float, (uint32_t)*p << 16);
}
// Nontemporal 16-byte / 8-byte stores (global_store ... nt): streamed past the caches.
__device__ __forceinline__ void st4nt(float* p, f32x4 v) { __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p)); }
__device__ __forceinline__ void st4nt(bf16_t* p, f32x4 v) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store(__builtin_bit_cast(u32x2, f32_to_bf16x4(v)), reinterpret_cast<u32x2*>(p));
}
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }
__device__ __forceinline__ void st1(bf16_t* p, float v) { *p = __builtin_bit_cast(bf16_t, (__bf16)v); }
// The value a store of v to T-typed storage keeps (what a consumer reads back).
template <class T>
__device__ __forceinline__ f32x4 rnd4(f32x4 v) {
  if constexpr (sizeof(T) == 2)
    return bf16x4_to_f32(f32_to_bf16x4(v));
  else
    return v;
}
// Store v (optionally nontemporal) and return what the store kept: one conversion for bf16
// (rnd4 followed by st4 converted twice).
__device__ __forceinline__ f32x4 st4_kept(float* p, f32x4 v, int nt) {
  if (nt)
    st4nt(p, v);
  else
    st4(p, v);
  return v;
}
__device__ __forceinline__ f32x4 st4_kept(bf16_t* p, f32x4 v, int nt) {
  uint2 u = f32_to_bf16x4(v);
  // opaque to the optimiser: it otherwise re-derives each kept value with its own conversion
  // (v_cvt_pk_bf16_f32 v, 0 + shift) instead of widening the two packed words
  asm volatile("" : "+v"(u.x), "+v"(u.y));
  typedef uint32_t u32x2_ __attribute__((ext_vector_type(2)));
  if (nt)
    __builtin_nontemporal_store(__builtin_bit_cast(u32x2_, u), reinterpret_cast<u32x2_*>(p));
  else
    *reinterpret_cast<uint2*>(p) = u;
  return bf16x4_to_f32(u);
}
template <class T>
__device__ __forceinline__ float rnd1(float v) {
  if constexpr (sizeof(T) == 2)
    return (float)(__bf16)v;
  else
    return v;
}

// Buffer loads (out-of-range byte offsets return 0 in hardware: padding needs no branch).
constexpr uint32_t kOOBBytes = 0x80000000u;  // past any buffer we build (tensors < 2 GiB)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_v(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// 4 consecutive elements at element index e (ok == false: zeros)
template <class T>
__device__ __forceinline__ f32x4 bload4e(__amdgpu_buffer_rsrc_t r, bool ok, uint32_t e) {
  if constexpr (sizeof(T) == 2) {
    const uint32_t off = ok ? e * 2u : kOOBBytes;
    return bf16x4_to_f32(__builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0)));
  } else {
    const uint32_t off = ok ? e * 4u : kOOBBytes;
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
  }
}

// 4 consecutive elements stored at element index e (ok == false: dropped), RNE for bf16
template <class T>
__device__ __forceinline__ void bstore4e(__amdgpu_buffer_rsrc_t r, bool ok, uint32_t e, f32x4 v) {
  if constexpr (sizeof(T) == 2) {
    const uint32_t off = ok ? e * 2u : kOOBBytes;
    typedef uint32_t u32x2_ __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_, f32_to_bf16x4(v)), r, (int)off, 0, 0);
  } else {
    typedef uint32_t u32x4_ __attribute__((ext_vector_type(4)));
    const uint32_t off = ok ? e * 4u : kOOBBytes;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_, v), r, (int)off, 0, 0);
  }
}

// Buffer stores with the nontemporal bit (cache policy 2: streamed past the caches) chosen at run
// time; the policy operand must be an immediate.
template <class V>
__device__ __forceinline__ void bstore_nt(V v, __amdgpu_buffer_rsrc_t r, int off, int soff, int nt) {
  if constexpr (sizeof(V) == 2) {
    if (nt) __builtin_amdgcn_raw_buffer_store_b16(v, r, off, soff, 2);
    else __builtin_amdgcn_raw_buffer_store_b16(v, r, off, soff, 0);
  } else if constexpr (sizeof(V) == 4) {
    if (nt) __builtin_amdgcn_raw_buffer_store_b32(v, r, off, soff, 2);
    else __builtin_amdgcn_raw_buffer_store_b32(v, r, off, soff, 0);
  } else {
    if (nt) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, soff, 2);
    else __builtin_amdgcn_raw_buffer_store_b128(v, r, off, soff, 0);
  }
}

// bstore4e with the nontemporal bit chosen at run time
template <class T>
__device__ __forceinline__ void bstore4e_nt(__amdgpu_buffer_rsrc_t r, bool ok, uint32_t e, f32x4 v, int nt) {
  if constexpr (sizeof(T) == 2) {
    const uint32_t off = ok ? e * 2u : kOOBBytes;
    typedef uint32_t u32x2_ __attribute__((ext_vector_type(2)));
    const u32x2_ u = __builtin_bit_cast(u32x2_, f32_to_bf16x4(v));
    if (nt) __builtin_amdgcn_raw_buffer_store_b64(u, r, (int)off, 0, 2);
    else __builtin_amdgcn_raw_buffer_store_b64(u, r, (int)off, 0, 0);
  } else {
    typedef uint32_t u32x4_ __attribute__((ext_vector_type(4)));
    const uint32_t off = ok ? e * 4u : kOOBBytes;
    bstore_nt(__builtin_bit_cast(u32x4_, v), r, (int)off, 0, nt);
  }
}

// Wave-level (64 lanes) sum.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// The BN output for one element (layers/batch_norm.py:91-96).  The standalone apply, the
// backward ReLU-mask recompute and every consumer that applies a BN on load call this
// same function, so all of them see bit-identical values.
__device__ __forceinline__ float bn_out(float x, float mean, float invstd, float gamma, float beta) {
  const float xh = (x - mean) * invstd;
  return gamma * xh + beta;
}
__device__ __forceinline__ float bn_relu_out(float x, float mean, float invstd, float gamma, float beta, int relu) {
  const float r = bn_out(x, mean, invstd, gamma, beta);
  return (relu && !(r > 0.f)) ? 0.f : r;
}

// The BN input gradient for one element, given the folded coefficients (stage 3 of
// layers/batch_norm.py:125-174): dx = gamma*invstd * (g - k1 - x_hat*k2), g already masked
// by a fused ReLU.  Written with an explicit fma so that dk_bn_bwd_apply_* and the dgrad
// loaders that form it on load (*_dgrad_bnbwd_f32) round identically.
__device__ __forceinline__ float bn_bwd_elem(float x, float g, float mean, float invstd, float f, float k1,
                                             float k2) {
  const float xh = (x - mean) * invstd;
  return f * __builtin_fmaf(-xh, k2, g - k1);
}

// A BatchNorm (+ ReLU) applied to an operand as it is loaded: the producer's raw output x
// plus per-channel statistics and affine parameters.  mean == nullptr: no transform.
struct BnIn {
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  int relu;
};

__device__ __forceinline__ f32x4 bn_in4(f32x4 v, f32x4 m, f32x4 is, f32x4 g, f32x4 b, int relu) {
  f32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = bn_relu_out(v[e], m[e], is[e], g[e], b[e], relu);
  return o;
}

// XCD-aware block order.  Consecutive hardware block ids are dealt round-robin over the 8
// XCDs, each with its own L2; this bijective remap gives every XCD a contiguous range of
// logical blocks, so neighbouring tiles that share input rows (convolution halos) share an L2.
__device__ __forceinline__ int xcd_block(int b, int n) {
  const int q = n >> 3, r = n & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// Sub-pixel decomposition of a stride-ST correlation's input gradient (conv_subpixel.hip,
// depthwise.hip): with h = ST*i + a, tap r reaches dx row h iff a == phase(r), and then
// reads dy row i + nb(r).  dmin/dmax bound the dy neighbourhood of one ST x ST "quad".
template <int R, int ST, int PAD>
struct SubPix {
  static constexpr int phase(int r) { return ((r - PAD) % ST + ST) % ST; }
  static constexpr int nb(int r) { return (phase(r) + PAD - r) / ST; }
  static constexpr int dmin() {
    int m = 1 << 20;
    for (int r = 0; r < R; ++r) m = nb(r) < m ? nb(r) : m;
    return m;
  }
  static constexpr int dmax() {
    int m = -(1 << 20);
    for (int r = 0; r < R; ++r) m = nb(r) > m ? nb(r) : m;
    return m;
  }
};

// Error codes returned for argument errors detected on the host side.  They
// live above the hipError_t range used by the runtime so callers can tell
// "bad call" from "device fault".
enum : int { DK_ERR_ARGS = 10001, DK_ERR_WORKSPACE = 10002 };
// Success, and the launch also folded the BN partials armed for it (dk_bn_fold_arm_*).
enum : int { DK_FOLDED = 10100 };
// Nontemporal output stores per kernel family (tuning knob dk_debug_set_gemm_config(4, mask)): bit kNt*
// set = that family's main output stores are nontemporal.
enum NtFam : int { kNtDwFwd = 0, kNtDwBwd = 1, kNtBnAdd = 2, kNtPwsBwd = 3, kNtPwsFwd = 4, kNtPwsDgrad = 5, kNtGemm = 6, kNtStem = 7, kNtPwd = 8, kNtPwd16 = 9, kNtDwDgrad = 10, kNtBnBwd = 11, kNtDwDgrad16 = 12 };
constexpr int kNtDefault = 6655;  // families 0-6: config 3 8.868 -> 8.819 ms, config 5 7.596 -> 7.566 (profiles/r03q_ntfam_config*.txt); 7 (the stem's output): config 3 7.861 -> 7.835 ms, 5 of 6 rounds (profiles/r06ay_ab_nt_stem.txt); 8 (fp32 deep pointwise): config 3 8.697 -> 8.650 ms, 3 of 3 (profiles/r04nt_ab.txt); 11 (BN backward apply): config 3 8.719 -> 8.700 ms (profiles/r04nt2_ab.txt); 12 (bf16 strided depthwise dgrad): config 5 5.747 -> 5.718 ms, 4 of 5 rounds (profiles/r06ay_ab_nt_stem.txt); off: 9 (bf16 deep pointwise, neutral), 10 (fp32 strided depthwise dgrad, neutral or slower)
int nt_stores(int fam);

// Path selectors and tuning knobs for tests and A/B runs (knobs.hip): one registry of atomics holding
// the built-in defaults; dk_debug_set_gemm_config(kind = KnobId, v) overrides (-1 = default).  No
// environment variable reaches them.  Numbers of retired knobs stay unused (tests and scripts address
// knobs by number).
enum KnobId : int {
  kKnobRowCfg = 0, kKnobSplitCfg = 1, kKnobFillSplits = 2, kKnobPwStream = 3, kKnobNtStores = 4,
  kKnobDwbBlocks = 7, kKnobDwSeg = 8, kKnobPwsh = 9, kKnobPwDeep = 11, kKnobPwDeep16 = 13, kKnobPwDeepBwd = 14,
  kKnobWgradBlocks = 18, kKnobEwVariant = 19, kKnobDwbCols = 21, kNumKnobs = 23
};
int knob(int id);
void knob_set(int id, int v);

// Split-K second stage (reduce.hip): out = sum_s ws[s][M][N] (+ l2 * w), fixed order.
//   mode 0: out[m][n];  mode 1: columns (r, s, c) with c padded to Cp -> out KCRS.
int splitk_reduce(const float* ws, int splits, int M, int N, float* out, const float* w, float l2, int mode, int C,
                  int Cp, int R, int S, hipStream_t st);
// The weight-gradient reduce (mode 0) at the end of a fused backward entry point: launched on st, or,
// while dk_wgrad_reduce_defer(1) is in effect on this host thread, recorded for dk_wgrad_reduce_flush
// to launch on another stream (the weight-gradient side stream).
int wgrad_reduce(const float* ws, int splits, int M, int N, float* out, const float* w, float l2, hipStream_t st);


// Streaming pointwise kernels (pw_stream.hip) for the K = C = 64 shapes.
bool pw_stream_enabled();  // knob kKnobPwStream (default 1; 0 = the tiled engine everywhere, for A/B runs)
bool pw_stream_dgrad_ok(int K, int C, int M);
int pw_stream_dgrad_rows(int M);
bool pw_stream_bwd_ok(int K, int C, int M);
int pw_stream_bwd_rows(int M);
struct FoldTail;  // fold_tail.h
int pw_stream_bwd_fused(const float* g, const float* bn_x, int M, const float* om, const float* ois,
                        const float* og, const float* ob, int orelu, const float* k12, const float* w, float* dx,
                        const float* res, const float* x, const float* im, const float* iis, const float* ig,
                        const float* ib, int irelu, double* part, const float* bm, const float* bis,
                        const float* bgm, const float* bbt, int brelu, float* wpart, hipStream_t st,
                        const struct FoldTail* ft = nullptr, const int* lattice = nullptr);
bool pw_stream_fwd_ok(int K, int C, int M, size_t xbytes);
int pw_stream_fwd_rows(int M, int K);
int pw_stream_fwd(const float* x, int N, int H, int W, int stride, int OH, int OW, const float* w, int KC,
                  const float* bias, float* y, const float* im, const float* iis, const float* ig,
                  const float* ib, int irelu, double* part, hipStream_t st, const struct FoldTail* ft = nullptr);
int pw_stream_dgrad_bnbwd(const float* g, const float* bn_x, int M, const float* om, const float* ois,
                          const float* og, const float* ob, int orelu, const float* k12, float* dy_out,
                          const float* w, float* dx, const float* res, const float* x, const float* im,
                          const float* iis, const float* ig, const float* ib, int irelu, double* part,
                          hipStream_t st, const struct FoldTail* ft = nullptr);

// fp32 deep streaming pointwise kernels (pw_deep.hip): reduction 64-512 with 128+ channels on a side.
bool pw_deep_fwd_ok(int K, int C, int M, size_t xbytes);
int pw_deep_fwd_rows(int M, int K, int C);
int pw_deep_fwd_slices(int M, int K, int C);
int pw_deep_fwd(const float* x, int N, int H, int W, int stride, int OH, int OW, const float* w, int K, int C,
                const float* bias, float* y, const float* im, const float* iis, const float* ig, const float* ib,
                int irelu, double* part, hipStream_t st, const struct FoldTail* ft = nullptr);
bool pw_deep_dgrad_ok(int K, int C, int M);
int pw_deep_dgrad_rows(int M, int K, int C);
int pw_deep_dgrad_slices(int M, int K, int C);
// The fused deep backward (dgrad + weight gradient in one pass, dy never stored): K in {128, 256}.
bool pw_deep_bwd_ok(int K, int C, int M);
int pw_deep_bwd_rows(int M, int K, int C);
int pw_deep_bwd_slices(int M, int K, int C);
int pw_deep_dgrad_plain(const float* dy, int M, int K, int C, const float* w, float* dx, hipStream_t st);

int pw_deep_bwd_bnbwd(const float* g, const float* bn_x, int M, int K, int C, const float* om, const float* ois,
                      const float* og, const float* ob, int orelu, const float* k12, const float* w, float* dx,
                      const float* res, const float* x, const float* im, const float* iis, const float* ig,
                      const float* ib, int irelu, double* part, float* wpart, hipStream_t st,
                      const struct FoldTail* ft = nullptr);
// bf16 weight-stationary deep pointwise kernels (pw_deep_bf16.hip), used by the pw_stream_bf16 entries.
bool pw_deep16_fwd_ok(int K, int C, int M);
bool pw_deep16_dgrad_ok(int K, int C, int M);
int pw_deep16_fwd_rows(int M, int K, int C);
int pw_deep16_dgrad_rows(int M, int K, int C);
int pw_deep16_fwd(const bf16_t* x, int M, const float* w, int K, int C, const float* bias, bf16_t* y, const float* im,
                  const float* iis, const float* ig, const float* ib, int irelu, double* part, hipStream_t st,
                  const struct FoldTail* ft);
int pw_deep16_dgrad_bnbwd(const bf16_t* g, const bf16_t* bn_x, int M, int K, int C, const float* om, const float* ois,
                          const float* og, const float* ob, int orelu, const float* k12, bf16_t* dy_out, const float* w,
                          bf16_t* dx, const bf16_t* res, const bf16_t* x, const float* im, const float* iis,
                          const float* ig, const float* ib, int irelu, double* part, hipStream_t st,
                          const struct FoldTail* ft);
int pw_deep_dgrad_bnbwd(const float* g, const float* bn_x, int M, int K, int C, const float* om, const float* ois,
                        const float* og, const float* ob, int orelu, const float* k12, float* dy_out, const float* w,
                        float* dx, const float* res, const float* x, const float* im, const float* iis,
                        const float* ig, const float* ib, int irelu, double* part, hipStream_t st,
                        const struct FoldTail* ft = nullptr);

// the fused bf16 deep backward (pw_deep_bf16.hip bwd_kernel): K in {128, 256}
bool pw_deep16_bwd_ok(int K, int C, int M);
int pw_deep16_bwd_rows(int M, int K, int C);
int pw_deep16_bwd_slices(int M, int K, int C);
int pw_deep16_bwd_fused(const bf16_t* g, const bf16_t* bn_x, int M, int K, int C, const float* om, const float* ois,
                        const float* og, const float* ob, int orelu, const float* k12, const float* w, bf16_t* dx,
                        const bf16_t* res, const bf16_t* x, const float* im, const float* iis, const float* ig,
                        const float* ib, int irelu, double* part, float* wpart, hipStream_t st,
                        const struct FoldTail* ft = nullptr);
// bf16 streaming pointwise kernels (pw_stream_bf16.hip, BASELINE config 5): K, C in {64, 128}.
bool pw_stream_bf16_fwd_ok(int K, int C, int M);
int pw_stream_bf16_fwd_rows(int M, int K, int C);
int pw_stream_bf16_fwd(const bf16_t* x, int M, const float* w, int K, int C, const float* bias, bf16_t* y,
                       const float* im, const float* iis, const float* ig, const float* ib, int irelu, double* part,
                       hipStream_t st, const struct FoldTail* ft = nullptr);
bool pw_stream_bf16_dgrad_ok(int K, int C, int M);
int pw_stream_bf16_dgrad_rows(int M, int K, int C);
int pw_stream_bf16_dgrad_bnbwd(const bf16_t* g, const bf16_t* bn_x, int M, int K, int C, const float* om,
                               const float* ois, const float* og, const float* ob, int orelu, const float* k12,
                               bf16_t* dy_out, const float* w, bf16_t* dx, const bf16_t* res, const bf16_t* x,
                               const float* im, const float* iis, const float* ig, const float* ib, int irelu,
                               double* part, hipStream_t st, const struct FoldTail* ft = nullptr);
int pw_stream_bf16_fwd_slices(int K, int C);    // channel slices of the partial rows (fold_take)
// the fused bf16 backward (dgrad + weight gradient, dy never stored) for K = C = 64
bool pw_stream_bf16_bwd_ok(int K, int C, int M);
int pw_stream_bf16_bwd_rows(int M);
int pw_stream_bf16_bwd_fused(const bf16_t* g, const bf16_t* bn_x, int M, const float* om, const float* ois,
                             const float* og, const float* ob, int orelu, const float* k12, const float* w, bf16_t* dx,
                             const bf16_t* res, const bf16_t* x, const float* im, const float* iis, const float* ig,
                             const float* ib, int irelu, double* part, float* wpart, hipStream_t st,
                             const struct FoldTail* ft = nullptr);
int pw_stream_bf16_dgrad_slices(int K, int C);

}  // namespace dk
