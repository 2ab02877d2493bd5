// Micro-benchmark: does f32 VALU work overlap v_mfma_f32_32x32x2_f32 on one SIMD?
// Each wave runs ITERS iterations of: 4 MFMAs on 4 independent accumulators + NV independent
// v_fma_f32 (+ ND v_fma_f64) + NL ds_read_b128, the MFMA operands fixed registers.  The kernel
// reports cycles per iteration per SIMD (s_memtime around the loop, wave 0 of each block) for
// 1..4 waves per SIMD (blocks of 4 waves, one block per CU per wave-per-SIMD level).
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/bin/mfma_valu scripts/mfma_valu.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NV, int ND, int NL>
__global__ __launch_bounds__(256) void kern(float* out, long long* cyc, int iters, float s) {
  __shared__ f32x4 lds[256 * 4];
  const int tid = threadIdx.x;
  for (int i = tid; i < 256 * 4; i += 256) lds[i] = f32x4{s, s, s, s};
  __syncthreads();
  f32x16 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
  float a = s * tid, b = s + tid;
  float v[NV > 0 ? NV : 1];
#pragma unroll
  for (int j = 0; j < (NV > 0 ? NV : 1); ++j) v[j] = s * j + tid;
  double d[ND > 0 ? ND : 1];
#pragma unroll
  for (int j = 0; j < (ND > 0 ? ND : 1); ++j) d[j] = (double)s * j + tid;
  f32x4 l = {0, 0, 0, 0};
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[u], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = __builtin_fmaf(v[j], s, 1.0f);
#pragma unroll
    for (int j = 0; j < ND; ++j) d[j] = __builtin_fma(d[j], (double)s, 1.0);
#pragma unroll
    for (int j = 0; j < NL; ++j) l += lds[(tid + 64 * j + it) & 1023];
  }
  const long long t1 = __builtin_readcyclecounter();
  float r = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int q = 0; q < 16; ++q) r += acc[u][q];
#pragma unroll
  for (int j = 0; j < NV; ++j) r += v[j];
#pragma unroll
  for (int j = 0; j < ND; ++j) r += (float)d[j];
  r += l[0] + l[1] + l[2] + l[3];
  out[blockIdx.x * 256 + tid] = r;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NV, int ND, int NL>
static void run(int wps) {
  const int blocks = 256 * wps, iters = 4096;
  float* out;
  long long* cyc;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&cyc, blocks * 8);
  hipLaunchKernelGGL((kern<NV, ND, NL>), dim3(blocks), dim3(256), 0, 0, out, cyc, 16, 1.0001f);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((kern<NV, ND, NL>), dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 1.0001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  long long* h = (long long*)malloc(blocks * 8);
  hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
  long long mx = 0, sum = 0;
  for (int i = 0; i < blocks; ++i) {
    mx = h[i] > mx ? h[i] : mx;
    sum += h[i];
  }
  // per SIMD per iteration: wps waves each doing 4 MFMAs (256 pipe cycles if serial)
  const double cyc_it = (double)sum / blocks / iters;
  const double tf = 2.0 * 32 * 32 * 2 * 4 * (double)iters * blocks * 4 / (ms * 1e-3) / 1e12;
  printf("NV=%2d ND=%2d NL=%2d waves/SIMD=%d: %7.1f cyc/iter/wave (MFMA-only floor %4d), %6.1f TF/s (%.2f of 157.3), %.3f ms\n",
         NV, ND, NL, wps, cyc_it, 256 * wps, tf, tf / 157.3, ms);
  free(h);
  hipFree(out);
  hipFree(cyc);
}

template <int NV, int ND, int NL>
static void sweep() {
  for (int w = 1; w <= 3; ++w) run<NV, ND, NL>(w);
}

int main() {
  sweep<0, 0, 0>();
  sweep<4, 0, 0>();
  sweep<8, 0, 0>();
  sweep<16, 0, 0>();
  sweep<32, 0, 0>();
  sweep<0, 4, 0>();
  sweep<0, 8, 0>();
  sweep<0, 0, 2>();
  sweep<0, 0, 4>();
  sweep<8, 0, 2>();
  return 0;
}
