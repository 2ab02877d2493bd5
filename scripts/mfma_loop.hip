// Micro-benchmark of the deep pointwise kernels' inner loop (dorknet_amd/csrc/pw_deep.hip): per tile a
// wave runs KR/2 v_mfma_f32_32x32x2_f32 with B fragments in registers and A read from an LDS tile
// (one ds_read_b128 per 4 MFMAs, D reads ahead), then (optionally) a block barrier.  Variants:
//   ACC: 1 = one accumulator chain (the kernels), 2 = two chains (even / odd q)
//   BAR: 1 = __syncthreads() after every tile
//   LDS: 0 = A from registers (no LDS reads)
// Reports TF/s of the MFMA work (fraction of 157.3) for 1..3 blocks of 4 waves per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/bin/mfma_loop scripts/mfma_loop.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int KR = 256, KQ = KR / 8, SK = KR + 4, TR = 32;

template <int ACC, bool BAR, bool LDS, int D>
__global__ __launch_bounds__(256, 2) void kern(float* out, const float* w, int tiles) {
  __shared__ __attribute__((aligned(16))) float As[TR * SK];
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
  for (int i = tid; i < TR * SK; i += 256) As[i] = 0.001f * (i % 97);
  f32x4 bw[KQ];
#pragma unroll
  for (int q = 0; q < KQ; ++q) bw[q] = *reinterpret_cast<const f32x4*>(w + (size_t)(tid % 128) * KR + 8 * q + 4 * h);
  __syncthreads();
  const float* ap = As + l32 * SK + 4 * h;
  f32x16 sink;
#pragma unroll
  for (int r = 0; r < 16; ++r) sink[r] = 0.f;
  for (int t = 0; t < tiles; ++t) {
    f32x16 acc[ACC];
#pragma unroll
    for (int c = 0; c < ACC; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
    if constexpr (LDS) {
      f32x4 ab[D];
#pragma unroll
      for (int i = 0; i < D; ++i) ab[i] = *reinterpret_cast<const f32x4*>(ap + 8 * i);
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        const f32x4 av = ab[q % D];
        if (q + D < KQ) ab[q % D] = *reinterpret_cast<const f32x4*>(ap + 8 * (q + D));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[q % ACC] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], bw[q][e], acc[q % ACC], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < KQ; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[q % ACC] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[(q + 1) % KQ][e], bw[q][e], acc[q % ACC], 0, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < ACC; ++c) sink += acc[c];
    if constexpr (BAR) __syncthreads();
  }
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) r += sink[i];
  out[blockIdx.x * 256 + tid] = r;
}

template <int ACC, bool BAR, bool LDS, int D>
static void run(const char* name, float* out, const float* w) {
  for (int bpc = 1; bpc <= 2; ++bpc) {
    const int blocks = 256 * bpc, tiles = 400;
    hipLaunchKernelGGL((kern<ACC, BAR, LDS, D>), dim3(blocks), dim3(256), 0, 0, out, w, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((kern<ACC, BAR, LDS, D>), dim3(blocks), dim3(256), 0, 0, out, w, tiles);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 32 * 32 * 2 * (KR / 2) * (double)tiles * blocks * 4;
    const double tf = flops / (ms * 1e-3) / 1e12;
    printf("%-28s blocks/CU=%d: %6.1f TF/s (%.2f of 157.3)\n", name, bpc, tf, tf / 157.3);
  }
}


// The loop above plus the kernels' per-tile memory work: STAGE = the next tile's 32 x KR pixel rows
// loaded from HBM (LV 16-byte loads per lane, issued before the MFMAs) and written to the other LDS
// buffer after them; STORE = 16 four-byte C-layout stores per lane of the 32 x 32 output.
template <bool STAGE, bool STORE, int BPC>
__global__ __launch_bounds__(256, BPC) void kern2(float* out, const float* w, const float* x, float* y, int tiles, int M) {
  constexpr int KV = KR / 4, LV = TR * KV / 256;
  __shared__ __attribute__((aligned(16))) float As[2][TR * SK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  for (int i = tid; i < 2 * TR * SK; i += 256) As[0][i] = 0.001f * (i % 97);
  f32x4 bw[KQ];
#pragma unroll
  for (int q = 0; q < KQ; ++q) bw[q] = *reinterpret_cast<const f32x4*>(w + (size_t)(tid % 128) * KR + 8 * q + 4 * h);
  const int kv = tid % KV, r0 = tid / KV;
  const int col = 32 * wave + l32;
  __syncthreads();
  f32x16 sink;
#pragma unroll
  for (int r = 0; r < 16; ++r) sink[r] = 0.f;
  const int ntiles = M / TR;
  int buf = 0;
  for (int t = blockIdx.x; t < blockIdx.x + tiles * gridDim.x; t += gridDim.x) {
    const int tt = t % ntiles;
    f32x4 st[LV];
    if constexpr (STAGE) {
#pragma unroll
      for (int j = 0; j < LV; ++j)
        st[j] = *reinterpret_cast<const f32x4*>(x + ((size_t)tt * TR + r0 + j * (256 / KV)) * KR + 4 * kv);
    }
    const float* ap = &As[buf][0] + l32 * SK + 4 * h;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    f32x4 ab[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ab[i] = *reinterpret_cast<const f32x4*>(ap + 8 * i);
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const f32x4 av = ab[q % 4];
      if (q + 4 < KQ) ab[q % 4] = *reinterpret_cast<const f32x4*>(ap + 8 * (q + 4));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], bw[q][e], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (STORE) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = acc[r];
        y[((size_t)tt * TR + 4 * h + (r & 3) + 8 * (r >> 2)) * 128 + col] = v;
      }
    } else {
      sink += acc;
    }
    if constexpr (STAGE) {
#pragma unroll
      for (int j = 0; j < LV; ++j)
        *reinterpret_cast<f32x4*>(&As[buf ^ 1][0] + (r0 + j * (256 / KV)) * SK + 4 * kv) = st[j];
    }
    __syncthreads();
    buf ^= 1;
  }
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) r += sink[i];
  out[blockIdx.x * 256 + tid] = r;
}

template <bool STAGE, bool STORE, int BPC>
static void run2(const char* name, float* out, const float* w, const float* x, float* y, int M) {
  const int blocks = 256 * BPC, tiles = 100;
  hipLaunchKernelGGL((kern2<STAGE, STORE, BPC>), dim3(blocks), dim3(256), 0, 0, out, w, x, y, 2, M);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((kern2<STAGE, STORE, BPC>), dim3(blocks), dim3(256), 0, 0, out, w, x, y, tiles, M);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 32 * 32 * 2 * (KR / 2) * (double)tiles * blocks * 4;
  const double tf = flops / (ms * 1e-3) / 1e12;
  printf("%-28s blocks/CU=%d: %6.1f TF/s (%.2f of 157.3)\n", name, BPC, tf, tf / 157.3);
}

int main() {
  float *out, *w;
  hipMalloc(&out, 1024 * 256 * 4);
  hipMalloc(&w, 128 * KR * 4);
  static float hw[128 * KR];
  unsigned seed = 12345;
  for (int i = 0; i < 128 * KR; ++i) {
    seed = seed * 1664525u + 1013904223u;
    hw[i] = ((seed >> 8) & 0xffff) / 65536.0f - 0.5f;
  }
  hipMemcpy(w, hw, sizeof(hw), hipMemcpyHostToDevice);
  run<1, false, false, 4>("regs, 1 chain", out, w);
  run<2, false, false, 4>("regs, 2 chains", out, w);
  run<1, false, true, 4>("LDS D4, 1 chain", out, w);
  run<2, false, true, 4>("LDS D4, 2 chains", out, w);
  run<1, true, true, 4>("LDS D4, 1 chain, barrier", out, w);
  run<2, true, true, 4>("LDS D4, 2 chains, barrier", out, w);
  run<1, false, true, 2>("LDS D2, 1 chain", out, w);
  run<1, false, true, 8>("LDS D8, 1 chain", out, w);
  const int M = 50176;  // 14 x 14 x 256 pixels
  float *x, *y;
  hipMalloc(&x, (size_t)M * KR * 4);
  hipMalloc(&y, (size_t)M * 128 * 4);
  hipMemset(x, 0, (size_t)M * KR * 4);
  run2<false, false, 2>("tile loop, barrier", out, w, x, y, M);
  run2<false, true, 2>("+ stores", out, w, x, y, M);
  run2<true, false, 2>("+ staging", out, w, x, y, M);
  run2<true, true, 2>("+ staging + stores", out, w, x, y, M);
  run2<true, true, 1>("+ staging + stores", out, w, x, y, M);
  return 0;
}
