// MFMA peak probe ("confirm the 2.5 PF peak with a measured MFMA
// microbenchmark and record the clock").  Every wave of every CU issues
// v_mfma_f32_32x32x16_bf16 back to back on 8 independent accumulators (no
// memory traffic in the loop); wave 0 of each workgroup stamps s_memtime (shader
// clock) and s_memrealtime (100 MHz constant clock) around the loop, so
// clock = d(memtime) / d(realtime) * 100 MHz (MI355X_MICROARCH.md, DVFS item 6).
// The operands come from a caller buffer: random bf16 (the clock the chip holds
// on real data) or zeros (the undervolted upper bound).
#include "common.h"

namespace {

constexpr int kChains = 8;

__global__ __launch_bounds__(256) void mfma_probe_kernel(unsigned long long* __restrict__ stamps,
                                                         float* __restrict__ sink,
                                                         const bf16_t* __restrict__ operands, int iters) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const bf16_t* src = operands + ((size_t)blockIdx.x * 256 + threadIdx.x) * 16;
  const bf16x8 a = *(const bf16x8*)src;
  const bf16x8 b = *(const bf16x8*)(src + 8);
  f32x16 acc[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) acc[c] = (f32x16){};
  __syncthreads();
  unsigned long long t0 = 0, r0 = 0;
  if (wave == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s += acc[c][lane & 15];
  if (wave == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {  // divergent: vector stores
      stamps[blockIdx.x * 4 + 0] = t0;
      stamps[blockIdx.x * 4 + 1] = t1;
      stamps[blockIdx.x * 4 + 2] = r0;
      stamps[blockIdx.x * 4 + 3] = r1;
    }
  }
  if (s == 1234.5f) sink[blockIdx.x * 256 + threadIdx.x] = s;  // keeps the chains live
}

}  // namespace

extern "C" int vggt_mfma_probe(unsigned long long* stamps, float* sink, const void* operands, int nwg, int iters,
                               void* stream) {
  if (!stamps || !sink || !operands || nwg <= 0 || iters <= 0) return VGGT_ERR_SHAPE;
  hipLaunchKernelGGL(mfma_probe_kernel, dim3(nwg), dim3(256), 0, (hipStream_t)stream, stamps, sink,
                     (const bf16_t*)operands, iters);
  return hipGetLastError() == hipSuccess ? VGGT_OK : VGGT_ERR_HIP;
}
