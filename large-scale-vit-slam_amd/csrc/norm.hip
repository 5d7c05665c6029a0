// Row LayerNorm and per-head QK-norm + RoPE (include/vggt_mi355x.h:
// vggt_layernorm, vggt_headnorm_rope).  HBM-bound: one wave per row, 16-B
// vectorised loads/stores, fp32 two-pass statistics in registers.
#include "common.h"

namespace {

// ---------------------------------------------------------------- LayerNorm
// NV = C / 256 float4 per lane (C = 256 * NV).
// Row r of the logical [M, C] input maps to group g = r / G, i = r % G:
//   x row = g*xgs + xoff + i,  y row = g*ygs + yoff + i   (identity: G = M).
struct RowMap {
  int G, xgs, xoff, ygs, yoff;
};

template <int NV, bool IN_BF16, bool OUT_BF16>
__global__ __launch_bounds__(256) void layernorm_kernel(const void* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        float eps, int M, void* __restrict__ y, int64_t ldy,
                                                        RowMap rm) {
  constexpr int C = NV * 256;
  const int lane = threadIdx.x & 63;
  const int lrow = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (lrow >= M) return;
  const int gi = lrow / rm.G, ii = lrow % rm.G;
  const int64_t row = (int64_t)gi * rm.xgs + rm.xoff + ii;
  const int64_t orow = (int64_t)gi * rm.ygs + rm.yoff + ii;
  float v[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = i * 256 + lane * 4;
    if constexpr (IN_BF16) {
      const uint2 u = *(const uint2*)((const bf16_t*)x + row * ldx + c);
      v[i][0] = bf2f(u.x & 0xffff);
      v[i][1] = bf2f(u.x >> 16);
      v[i][2] = bf2f(u.y & 0xffff);
      v[i][3] = bf2f(u.y >> 16);
    } else {
      const f32x4 u = *(const f32x4*)((const float*)x + row * ldx + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[i][j] = u[j];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += v[i][j];
  const float mean = wave_sum(s) * (1.f / C);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d = v[i][j] - mean;
      q += d * d;
    }
  const float rstd = rsqrtf(wave_sum(q) * (1.f / C) + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = i * 256 + lane * 4;
    float o[4];
    if (w) {
      const f32x4 wv = *(const f32x4*)(w + c);
      const f32x4 bv = b ? *(const f32x4*)(b + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd * wv[j] + bv[j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd;
    }
    if constexpr (OUT_BF16) {
      uint2 u;
      u.x = pack_bf2(o[0], o[1]);
      u.y = pack_bf2(o[2], o[3]);
      *(uint2*)((bf16_t*)y + orow * ldy + c) = u;
    } else {
      *(f32x4*)((float*)y + orow * ldy + c) = f32x4{o[0], o[1], o[2], o[3]};
    }
  }
}

template <int NV>
int launch_ln(const void* x, int in_bf, int64_t ldx, const float* w, const float* b, float eps, int M, void* y,
              int out_bf, int64_t ldy, RowMap rm, hipStream_t s) {
  const int grid = (M + 3) / 4;
  if (in_bf && out_bf) layernorm_kernel<NV, true, true><<<grid, 256, 0, s>>>(x, ldx, w, b, eps, M, y, ldy, rm);
  else if (in_bf) layernorm_kernel<NV, true, false><<<grid, 256, 0, s>>>(x, ldx, w, b, eps, M, y, ldy, rm);
  else if (out_bf) layernorm_kernel<NV, false, true><<<grid, 256, 0, s>>>(x, ldx, w, b, eps, M, y, ldy, rm);
  else layernorm_kernel<NV, false, false><<<grid, 256, 0, s>>>(x, ldx, w, b, eps, M, y, ldy, rm);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

// ------------------------------------ LayerScale residual add + LayerNorm
// x[m] += gamma * y[m] (fp32 residual, bf16 branch output -- the arithmetic
// of the GEMM's EPI_RESID_F32 epilogue), optionally mirrored into out2, then
// (LN) xn[m] = LayerNorm(x[m]) in bf16, affine when w is given.  One wave per
// row, NV float4 per lane, like layernorm_kernel.
template <int NV, bool LN>
__global__ __launch_bounds__(256) void resid_add_ln_kernel(float* __restrict__ x, int64_t ldx,
                                                           const bf16_t* __restrict__ y, int64_t ldy,
                                                           const float* __restrict__ gamma, float* __restrict__ out2,
                                                           int64_t ldo2, const float* __restrict__ w,
                                                           const float* __restrict__ b, float eps, int M,
                                                           bf16_t* __restrict__ xn, int64_t ldn) {
  constexpr int C = NV * 256;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[NV][4];
  uint2 yu[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) yu[i] = *(const uint2*)(y + (int64_t)row * ldy + i * 256 + lane * 4);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = i * 256 + lane * 4;
    const f32x4 u = *(const f32x4*)(x + (int64_t)row * ldx + c);
    const f32x4 g = *(const f32x4*)(gamma + c);
    const float yv[4] = {bf2f(yu[i].x & 0xffff), bf2f(yu[i].x >> 16), bf2f(yu[i].y & 0xffff), bf2f(yu[i].y >> 16)};
#pragma unroll
    for (int j = 0; j < 4; ++j) v[i][j] = u[j] + g[j] * yv[j];
    *(f32x4*)(x + (int64_t)row * ldx + c) = f32x4{v[i][0], v[i][1], v[i][2], v[i][3]};
    if (out2) *(f32x4*)(out2 + (int64_t)row * ldo2 + c) = f32x4{v[i][0], v[i][1], v[i][2], v[i][3]};
  }
  if constexpr (LN) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) s += v[i][j];
    const float mean = wave_sum(s) * (1.f / C);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
    const float rstd = rsqrtf(wave_sum(q) * (1.f / C) + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = i * 256 + lane * 4;
      float o[4];
      if (w) {
        const f32x4 wv = *(const f32x4*)(w + c);
        const f32x4 bv = b ? *(const f32x4*)(b + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd * wv[j] + bv[j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd;
      }
      uint2 u;
      u.x = pack_bf2(o[0], o[1]);
      u.y = pack_bf2(o[2], o[3]);
      *(uint2*)(xn + (int64_t)row * ldn + c) = u;
    }
  }
}

template <int NV>
void launch_raln(float* x, int64_t ldx, const bf16_t* y, int64_t ldy, const float* gamma, float* out2, int64_t ldo2,
                 const float* w, const float* b, float eps, int M, bf16_t* xn, int64_t ldn, hipStream_t s) {
  const int grid = (M + 3) / 4;
  if (xn)
    resid_add_ln_kernel<NV, true><<<grid, 256, 0, s>>>(x, ldx, y, ldy, gamma, out2, ldo2, w, b, eps, M, xn, ldn);
  else
    resid_add_ln_kernel<NV, false><<<grid, 256, 0, s>>>(x, ldx, y, ldy, gamma, out2, ldo2, w, b, eps, M, xn, ldn);
}

// ------------------------------------------------- per-head norm + RoPE
// One wave per row; each lane owns 8 consecutive values (one 16-B chunk) of
// a head; LPH = D/8 lanes per head, heads processed 64/LPH at a time.
// Heads [0, hsplit) use (w, b), heads [hsplit, H) use (w2, b2): one launch
// normalises q and k of a fused qkv row (different q_norm / k_norm weights).
// Rows are read from src (row stride lds; == buf for the in-place form) and
// written to buf, at the same column offset.
template <int D, int MODE>
__global__ __launch_bounds__(256) void headnorm_rope_kernel(const bf16_t* src, int64_t lds, bf16_t* buf, int64_t ld,
                                                            int col_off, int M,
                                                            int H, const float* __restrict__ w,
                                                            const float* __restrict__ b, float eps,
                                                            const int32_t* __restrict__ pos, int period,
                                                            const float* __restrict__ cs, const float* __restrict__ sn,
                                                            int tab_len, int hsplit, const float* __restrict__ w2,
                                                            const float* __restrict__ b2) {
  constexpr int LPH = D / 8;
  constexpr int HPP = 64 / LPH;  // heads per pass
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int sub = lane % LPH;  // chunk index within the head
  const int e0 = sub * 8;      // first element within the head
  int p0 = 0, p1 = 0;
  if constexpr (MODE == VGGT_ROPE_2D) {
    const int pr = row % period;
    p0 = min(max(pos[2 * pr], 0), tab_len - 1);
    p1 = min(max(pos[2 * pr + 1], 0), tab_len - 1);
  } else if constexpr (MODE == VGGT_ROPE_1D) {
    p0 = min(max(pos[row % period], 0), tab_len - 1);
  }
  // both weight sets preloaded (heads < hsplit use w/b, the rest w2/b2)
  float wa[8], ba[8], wb[8], bb2[8];
  if (w) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      wa[j] = w[e0 + j];
      ba[j] = b ? b[e0 + j] : 0.f;
      wb[j] = w2[e0 + j];
      bb2[j] = b2 ? b2[e0 + j] : 0.f;
    }
  }
  for (int h0 = 0; h0 < H; h0 += HPP) {
    const int h = h0 + lane / LPH;
    const bool act = h < H;
    const bool first_set = h < hsplit;
    float wv[8], bv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      wv[j] = first_set ? wa[j] : wb[j];
      bv[j] = first_set ? ba[j] : bb2[j];
    }
    bf16_t* p = buf + (int64_t)row * ld + col_off + (act ? h : 0) * D + e0;
    float x[8];
    {
      const uint4 u = *(const uint4*)(src + (int64_t)row * lds + col_off + (act ? h : 0) * D + e0);
      const uint32_t uu[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[2 * j] = bf2f(uu[j] & 0xffff);
        x[2 * j + 1] = bf2f(uu[j] >> 16);
      }
    }
    if (w) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) s += x[j];
#pragma unroll
      for (int o = 1; o < LPH; o <<= 1) s += __shfl_xor(s, o, 64);
      const float mean = s * (1.f / D);
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = x[j] - mean;
        q += d * d;
      }
#pragma unroll
      for (int o = 1; o < LPH; o <<= 1) q += __shfl_xor(q, o, 64);
      const float rstd = rsqrtf(q * (1.f / D) + eps);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (x[j] - mean) * rstd * wv[j] + bv[j];
    }
    if constexpr (MODE != VGGT_ROPE_NONE) {
      // rotate_half partner lives RD/2 elements away = (RD/16) lanes away
      constexpr int RD = (MODE == VGGT_ROPE_2D) ? D / 2 : D;
      constexpr int PL = RD / 16;  // partner lane distance
      const int er = e0 % RD;      // element index inside the rotated block
      const int pp = (MODE == VGGT_ROPE_2D && e0 >= D / 2) ? p1 : p0;
      const bool first = er < RD / 2;
      // 8 consecutive table entries from a 32-B aligned offset: two 16-B loads each
      const float4* cp = (const float4*)(cs + pp * RD + er);
      const float4* sp = (const float4*)(sn + pp * RD + er);
      const float4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
      const float cv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      float y[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float partner = __shfl_xor(x[j], PL, 64);
        const float rot = first ? -partner : partner;
        y[j] = x[j] * cv[j] + rot * sv[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = y[j];
    }
    if (act) {
      uint4 u;
      u.x = pack_bf2(x[0], x[1]);
      u.y = pack_bf2(x[2], x[3]);
      u.z = pack_bf2(x[4], x[5]);
      u.w = pack_bf2(x[6], x[7]);
      *(uint4*)p = u;
    }
  }
}

template <int D>
int launch_hnr(const bf16_t* src, int64_t lds, bf16_t* buf, int64_t ld, int col_off, int M, int H, const float* w, const float* b, float eps, int mode,
               const int32_t* pos, int period, const float* cs, const float* sn, int tab_len, hipStream_t s,
               int hsplit, const float* w2, const float* b2) {
  const int grid = (M + 3) / 4;
  switch (mode) {
    case VGGT_ROPE_NONE:
      headnorm_rope_kernel<D, VGGT_ROPE_NONE><<<grid, 256, 0, s>>>(src, lds, buf, ld, col_off, M, H, w, b, eps, pos, period, cs,
                                                                  sn, tab_len, hsplit, w2, b2);
      break;
    case VGGT_ROPE_2D:
      headnorm_rope_kernel<D, VGGT_ROPE_2D><<<grid, 256, 0, s>>>(src, lds, buf, ld, col_off, M, H, w, b, eps, pos, period, cs, sn,
                                                                tab_len, hsplit, w2, b2);
      break;
    case VGGT_ROPE_1D:
      headnorm_rope_kernel<D, VGGT_ROPE_1D><<<grid, 256, 0, s>>>(src, lds, buf, ld, col_off, M, H, w, b, eps, pos, period, cs, sn,
                                                                tab_len, hsplit, w2, b2);
      break;
    default: return VGGT_ERR_UNSUPPORTED;
  }
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

}  // namespace

extern "C" int vggt_layernorm_grouped(const void* x, int in_dtype, int64_t ldx, const float* w, const float* b,
                                      float eps, int M, int C, void* y, int out_dtype, int64_t ldy, int group,
                                      int x_group_stride, int x_row_offset, int y_group_stride, int y_row_offset,
                                      void* stream) {
  if (M <= 0) return M == 0 ? VGGT_OK : VGGT_ERR_SHAPE;
  if (group <= 0) return VGGT_ERR_SHAPE;
  RowMap rm{group, x_group_stride, x_row_offset, y_group_stride, y_row_offset};
  if (C % 256 || C > 4096 || C <= 0) return VGGT_ERR_SHAPE;
  if ((in_dtype != VGGT_DTYPE_F32 && in_dtype != VGGT_DTYPE_BF16) ||
      (out_dtype != VGGT_DTYPE_F32 && out_dtype != VGGT_DTYPE_BF16))
    return VGGT_ERR_UNSUPPORTED;
  if ((ldx % 4) || (ldy % 4) || ((uintptr_t)x % 8) || ((uintptr_t)y % 8)) return VGGT_ERR_ALIGN;
  if (!in_dtype && ((uintptr_t)x % 16)) return VGGT_ERR_ALIGN;
  if (!out_dtype && ((uintptr_t)y % 16)) return VGGT_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const int ib = in_dtype == VGGT_DTYPE_BF16, ob = out_dtype == VGGT_DTYPE_BF16;
  switch (C / 256) {
    case 1: return launch_ln<1>(x, ib, ldx, w, b, eps, M, y, ob, ldy, rm, s);
    case 2: return launch_ln<2>(x, ib, ldx, w, b, eps, M, y, ob, ldy, rm, s);
    case 3: return launch_ln<3>(x, ib, ldx, w, b, eps, M, y, ob, ldy, rm, s);
    case 4: return launch_ln<4>(x, ib, ldx, w, b, eps, M, y, ob, ldy, rm, s);
    case 8: return launch_ln<8>(x, ib, ldx, w, b, eps, M, y, ob, ldy, rm, s);
    case 16: return launch_ln<16>(x, ib, ldx, w, b, eps, M, y, ob, ldy, rm, s);
    default: return VGGT_ERR_SHAPE;
  }
}

extern "C" int vggt_layernorm(const void* x, int in_dtype, int64_t ldx, const float* w, const float* b, float eps,
                              int M, int C, void* y, int out_dtype, int64_t ldy, void* stream) {
  return vggt_layernorm_grouped(x, in_dtype, ldx, w, b, eps, M, C, y, out_dtype, ldy, M > 0 ? M : 1, 0, 0, 0, 0,
                                stream);
}

extern "C" int vggt_resid_add_layernorm(float* x, int64_t ldx, const void* y, int64_t ldy, const float* gamma,
                                        float* out2, int64_t ldo2, const float* w, const float* b, float eps, int M,
                                        int C, void* xn, int64_t ldn, void* stream) {
  if (M <= 0) return M == 0 ? VGGT_OK : VGGT_ERR_SHAPE;
  if (C % 256 || C > 4096 || C <= 0 || !x || !y || !gamma) return VGGT_ERR_SHAPE;
  if ((ldx % 4) || (ldy % 4) || (out2 && (ldo2 % 4)) || (xn && (ldn % 4))) return VGGT_ERR_ALIGN;
  if (((uintptr_t)x | (uintptr_t)gamma | (uintptr_t)out2) % 16 || ((uintptr_t)y | (uintptr_t)xn) % 8)
    return VGGT_ERR_ALIGN;
  if ((w && ((uintptr_t)w % 16)) || (b && ((uintptr_t)b % 16))) return VGGT_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const bf16_t* yb = (const bf16_t*)y;
  bf16_t* nb = (bf16_t*)xn;
  switch (C / 256) {
    case 1: launch_raln<1>(x, ldx, yb, ldy, gamma, out2, ldo2, w, b, eps, M, nb, ldn, s); break;
    case 2: launch_raln<2>(x, ldx, yb, ldy, gamma, out2, ldo2, w, b, eps, M, nb, ldn, s); break;
    case 4: launch_raln<4>(x, ldx, yb, ldy, gamma, out2, ldo2, w, b, eps, M, nb, ldn, s); break;
    case 8: launch_raln<8>(x, ldx, yb, ldy, gamma, out2, ldo2, w, b, eps, M, nb, ldn, s); break;
    default: return VGGT_ERR_SHAPE;
  }
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_headnorm_rope(void* buf, int64_t ld, int col_off, int M, int H, int D, const float* w,
                                  const float* b, float eps, int rope_mode, const int32_t* pos, int period,
                                  const float* cos_tab, const float* sin_tab, int tab_len, void* stream) {
  if (M <= 0) return M == 0 ? VGGT_OK : VGGT_ERR_SHAPE;
  if (H <= 0 || (D != 64 && D != 128)) return VGGT_ERR_SHAPE;
  if ((ld % 8) || (col_off % 8) || ((uintptr_t)buf % 16)) return VGGT_ERR_ALIGN;
  if (rope_mode != VGGT_ROPE_NONE && (!pos || !cos_tab || !sin_tab || period <= 0 || tab_len <= 0))
    return VGGT_ERR_SHAPE;
  if (((uintptr_t)cos_tab | (uintptr_t)sin_tab) % 16) return VGGT_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  if (D == 64) return launch_hnr<64>((const bf16_t*)buf, ld, (bf16_t*)buf, ld, col_off, M, H, w, b, eps, rope_mode, pos, period, cos_tab, sin_tab,
                                     tab_len, s, H, w, b);
  return launch_hnr<128>((const bf16_t*)buf, ld, (bf16_t*)buf, ld, col_off, M, H, w, b, eps, rope_mode, pos, period, cos_tab, sin_tab, tab_len, s,
                         H, w, b);
}

extern "C" int vggt_qknorm_rope(void* qkv, int64_t ld, int M, int H, int D, const float* qw, const float* qb,
                                const float* kw, const float* kb, float eps, int rope_mode, const int32_t* pos,
                                int period, const float* cos_tab, const float* sin_tab, int tab_len, void* stream) {
  if (M <= 0) return M == 0 ? VGGT_OK : VGGT_ERR_SHAPE;
  if (H <= 0 || (D != 64 && D != 128)) return VGGT_ERR_SHAPE;
  if ((ld % 8) || ((uintptr_t)qkv % 16)) return VGGT_ERR_ALIGN;
  if ((qw == nullptr) != (kw == nullptr)) return VGGT_ERR_SHAPE;
  if (rope_mode != VGGT_ROPE_NONE && (!pos || !cos_tab || !sin_tab || period <= 0 || tab_len <= 0))
    return VGGT_ERR_SHAPE;
  if (((uintptr_t)cos_tab | (uintptr_t)sin_tab) % 16) return VGGT_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  if (D == 64) return launch_hnr<64>((const bf16_t*)qkv, ld, (bf16_t*)qkv, ld, 0, M, 2 * H, qw, qb, eps, rope_mode, pos, period, cos_tab,
                                     sin_tab, tab_len, s, H, kw, kb);
  return launch_hnr<128>((const bf16_t*)qkv, ld, (bf16_t*)qkv, ld, 0, M, 2 * H, qw, qb, eps, rope_mode, pos, period, cos_tab, sin_tab, tab_len,
                         s, H, kw, kb);
}

// Out-of-place form of vggt_qknorm_rope: the q|k columns [0, 2*H*D) of src
// (row stride lds) are normalised + rotated into dst (row stride ldd); src is
// left untouched (the training recompute keeps the pre-norm values for the
// backward, and the v columns are read from src directly).
extern "C" int vggt_qknorm_rope_out(const void* src, int64_t lds, void* dst, int64_t ldd, int M, int H, int D,
                                    const float* qw, const float* qb, const float* kw, const float* kb, float eps,
                                    int rope_mode, const int32_t* pos, int period, const float* cos_tab,
                                    const float* sin_tab, int tab_len, void* stream) {
  if (M <= 0) return M == 0 ? VGGT_OK : VGGT_ERR_SHAPE;
  if (H <= 0 || (D != 64 && D != 128)) return VGGT_ERR_SHAPE;
  if ((lds % 8) || (ldd % 8) || ((uintptr_t)src % 16) || ((uintptr_t)dst % 16)) return VGGT_ERR_ALIGN;
  if ((qw == nullptr) != (kw == nullptr)) return VGGT_ERR_SHAPE;
  if (rope_mode != VGGT_ROPE_NONE && (!pos || !cos_tab || !sin_tab || period <= 0 || tab_len <= 0))
    return VGGT_ERR_SHAPE;
  if (((uintptr_t)cos_tab | (uintptr_t)sin_tab) % 16) return VGGT_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  if (D == 64) return launch_hnr<64>((const bf16_t*)src, lds, (bf16_t*)dst, ldd, 0, M, 2 * H, qw, qb, eps, rope_mode,
                                     pos, period, cos_tab, sin_tab, tab_len, s, H, kw, kb);
  return launch_hnr<128>((const bf16_t*)src, lds, (bf16_t*)dst, ldd, 0, M, 2 * H, qw, qb, eps, rope_mode, pos, period,
                         cos_tab, sin_tab, tab_len, s, H, kw, kb);
}

// Out-of-place form of vggt_headnorm_rope: H heads of D columns starting at
// column 0 of src (row stride lds) normalised + rotated into dst (row stride ldd).
extern "C" int vggt_headnorm_rope_out(const void* src, int64_t lds, void* dst, int64_t ldd, int M, int H, int D,
                                      const float* w, const float* b, float eps, int rope_mode, const int32_t* pos,
                                      int period, const float* cos_tab, const float* sin_tab, int tab_len,
                                      void* stream) {
  if (M <= 0) return M == 0 ? VGGT_OK : VGGT_ERR_SHAPE;
  if (H <= 0 || (D != 64 && D != 128)) return VGGT_ERR_SHAPE;
  if ((lds % 8) || (ldd % 8) || ((uintptr_t)src % 16) || ((uintptr_t)dst % 16)) return VGGT_ERR_ALIGN;
  if (rope_mode != VGGT_ROPE_NONE && (!pos || !cos_tab || !sin_tab || period <= 0 || tab_len <= 0))
    return VGGT_ERR_SHAPE;
  if (((uintptr_t)cos_tab | (uintptr_t)sin_tab) % 16) return VGGT_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  if (D == 64) return launch_hnr<64>((const bf16_t*)src, lds, (bf16_t*)dst, ldd, 0, M, H, w, b, eps, rope_mode, pos,
                                     period, cos_tab, sin_tab, tab_len, s, H, w, b);
  return launch_hnr<128>((const bf16_t*)src, lds, (bf16_t*)dst, ldd, 0, M, H, w, b, eps, rope_mode, pos, period,
                         cos_tab, sin_tab, tab_len, s, H, w, b);
}
