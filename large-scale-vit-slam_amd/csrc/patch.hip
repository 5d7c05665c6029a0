// Patch-embed input, token assembly and small copy kernels for the aggregator
// (include/vggt_mi355x.h: vggt_patch_im2col, vggt_dino_assemble,
// vggt_special_tokens, vggt_copy_rows_f32).  All HBM-bound elementwise work.
#include "common.h"

namespace {

// A[f*hw + py*w + px][k], k = c*p*p + ky*p + kx (Conv2d weight flattening),
// value = bf16((img - mean[c]) / std[c]); k in [3p^2, Kp) zero-filled.
// One thread per (patch row, 8 consecutive k) -> 16-B stores.
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ img, int F, int H, int W, int p,
                                                     float m0, float m1, float m2, float sd0, float sd1, float sd2,
                                                     bf16_t* __restrict__ A, int Kp) {
  const int h = H / p, w = W / p;
  const int kc = Kp / 8;
  const int64_t total = (int64_t)F * h * w * kc;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / kc;
    const int k0 = (int)(i % kc) * 8;
    const int f = (int)(r / (h * w));
    const int pi = (int)(r % (h * w));
    const int py = pi / w, px = pi % w;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + j;
      float x = 0.f;
      if (k < 3 * p * p) {
        const int c = k / (p * p);
        const int rem = k % (p * p);
        const int ky = rem / p, kx = rem % p;
        const float raw = img[(((int64_t)f * 3 + c) * H + py * p + ky) * W + px * p + kx];
        const float mean = c == 0 ? m0 : (c == 1 ? m1 : m2);
        const float sd = c == 0 ? sd0 : (c == 1 ? sd1 : sd2);
        x = (raw - mean) / sd;
      }
      v[j] = x;
    }
    uint4 u;
    u.x = pack_bf2(v[0], v[1]);
    u.y = pack_bf2(v[2], v[3]);
    u.z = pack_bf2(v[4], v[5]);
    u.w = pack_bf2(v[6], v[7]);
    *(uint4*)(A + r * Kp + k0) = u;
  }
}

// x[f, t, :] for P = 1 + nreg + hw tokens per frame (4 floats per thread).
__global__ __launch_bounds__(256) void dino_assemble_kernel(const bf16_t* __restrict__ patch,
                                                            const float* __restrict__ cls,
                                                            const float* __restrict__ reg,
                                                            const float* __restrict__ pos, int F, int hw, int nreg,
                                                            int C, float* __restrict__ x) {
  const int P = 1 + nreg + hw;
  const int c4 = C / 4;
  const int64_t total = (int64_t)F * P * c4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % c4) * 4;
    const int64_t r = i / c4;
    const int t = (int)(r % P);
    const int f = (int)(r / P);
    f32x4 o;
    if (t == 0) {
      const f32x4 a = *(const f32x4*)(cls + c), b = *(const f32x4*)(pos + c);
      o = a + b;
    } else if (t <= nreg) {
      o = *(const f32x4*)(reg + (int64_t)(t - 1) * C + c);
    } else {
      const int pi = t - 1 - nreg;
      const uint2 u = *(const uint2*)(patch + ((int64_t)f * hw + pi) * C + c);
      const f32x4 b = *(const f32x4*)(pos + (int64_t)(pi + 1) * C + c);
      o = f32x4{bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16)} + b;
    }
    *(f32x4*)(x + r * C + c) = o;
  }
}

__global__ __launch_bounds__(256) void special_tokens_kernel(float* __restrict__ x, int64_t ldx, int F, int S, int P,
                                                             int n, int C, const float* __restrict__ tok) {
  const int c4 = C / 4;
  const int64_t total = (int64_t)F * n * c4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % c4) * 4;
    const int64_t r = i / c4;
    const int t = (int)(r % n);
    const int f = (int)(r / n);
    const int sel = (f % S) == 0 ? 0 : 1;
    *(f32x4*)(x + ((int64_t)f * P + t) * ldx + c) = *(const f32x4*)(tok + ((int64_t)sel * n + t) * C + c);
  }
}

__global__ __launch_bounds__(256) void copy_rows_kernel(const float* __restrict__ src, int64_t lds,
                                                        float* __restrict__ dst, int64_t ldd, int rows, int cols) {
  const int c4 = cols / 4;
  const int64_t total = (int64_t)rows * c4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % c4) * 4;
    const int64_t r = i / c4;
    *(f32x4*)(dst + r * ldd + c) = *(const f32x4*)(src + r * lds + c);
  }
}

inline int grid_for(int64_t total) {
  int64_t g = (total + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" int vggt_patch_im2col(const float* images, int F, int H, int W, int patch, const float* mean,
                                 const float* std_, void* A, int Kp, void* stream) {
  if (F <= 0 || patch <= 0 || H % patch || W % patch || Kp % 8 || Kp < 3 * patch * patch) return VGGT_ERR_SHAPE;
  if ((uintptr_t)A % 16) return VGGT_ERR_ALIGN;
  const int64_t total = (int64_t)F * (H / patch) * (W / patch) * (Kp / 8);
  im2col_kernel<<<grid_for(total), 256, 0, (hipStream_t)stream>>>(images, F, H, W, patch, mean[0], mean[1], mean[2],
                                                                   std_[0], std_[1], std_[2],
                                                                   (bf16_t*)A, Kp);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_dino_assemble(const void* patch, const float* cls, const float* reg, const float* pos, int F,
                                  int hw, int nreg, int C, float* x, void* stream) {
  if (F <= 0 || hw <= 0 || nreg < 0 || C % 4) return VGGT_ERR_SHAPE;
  if (((uintptr_t)patch | (uintptr_t)cls | (uintptr_t)reg | (uintptr_t)pos | (uintptr_t)x) % 16) return VGGT_ERR_ALIGN;
  const int64_t total = (int64_t)F * (1 + nreg + hw) * (C / 4);
  dino_assemble_kernel<<<grid_for(total), 256, 0, (hipStream_t)stream>>>((const bf16_t*)patch, cls, reg, pos, F, hw,
                                                                          nreg, C, x);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_special_tokens(float* x, int64_t ldx, int F, int S, int P, int n, int C, const float* tok,
                                   void* stream) {
  if (F <= 0 || S <= 0 || n <= 0 || n > P || C % 4 || ldx % 4) return VGGT_ERR_SHAPE;
  if (((uintptr_t)x | (uintptr_t)tok) % 16) return VGGT_ERR_ALIGN;
  const int64_t total = (int64_t)F * n * (C / 4);
  special_tokens_kernel<<<grid_for(total), 256, 0, (hipStream_t)stream>>>(x, ldx, F, S, P, n, C, tok);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_copy_rows_f32(const float* src, int64_t lds, float* dst, int64_t ldd, int rows, int cols,
                                  void* stream) {
  if (rows < 0 || cols % 4 || lds % 4 || ldd % 4) return VGGT_ERR_SHAPE;
  if (((uintptr_t)src | (uintptr_t)dst) % 16) return VGGT_ERR_ALIGN;
  if (rows == 0 || cols == 0) return VGGT_OK;
  copy_rows_kernel<<<grid_for((int64_t)rows * cols / 4), 256, 0, (hipStream_t)stream>>>(src, lds, dst, ldd, rows, cols);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}
