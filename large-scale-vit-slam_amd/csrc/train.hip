// Backward-pass kernels for training the alignment head (SURVEY.md §8f row 4;
// aligned_vggt/heads/alignment_head.py, cross_attention.py, gated_update.py
// under the reference's bf16-mixed autocast, run_model.py:472 + the
// train_featureAlignedVGGT_vkitti.yaml freeze list).  Contracts in
// include/vggt_mi355x.h ("Training (backward) entry points").
//
// All of these are HBM-bound row / column sweeps: one wave per row for the
// row-statistics kernels (LayerNorm, per-head norm + RoPE), 4-column vectors
// per thread for the column reductions.  Every parameter-gradient reduction
// is deterministic: fixed row chunks write partial sums to a caller-provided
// workspace, and a finalize pass adds the chunks in index order.
#include <math.h>

#include <stdlib.h>

#include "common.h"
#include "mfma_frag.h"

namespace {

typedef __attribute__((ext_vector_type(4))) float f4;

__device__ __forceinline__ void load4(const void* p, int dtype, int64_t off, float v[4]) {
  if (dtype == VGGT_DTYPE_BF16) {
    const uint2 u = *(const uint2*)((const bf16_t*)p + off);
    v[0] = bf2f(u.x & 0xffff);
    v[1] = bf2f(u.x >> 16);
    v[2] = bf2f(u.y & 0xffff);
    v[3] = bf2f(u.y >> 16);
  } else {
    const f4 u = *(const f4*)((const float*)p + off);
    v[0] = u[0];
    v[1] = u[1];
    v[2] = u[2];
    v[3] = u[3];
  }
}
__device__ __forceinline__ void store4(void* p, int dtype, int64_t off, const float v[4]) {
  if (dtype == VGGT_DTYPE_BF16) {
    uint2 u;
    u.x = pack_bf2(v[0], v[1]);
    u.y = pack_bf2(v[2], v[3]);
    *(uint2*)((bf16_t*)p + off) = u;
  } else {
    *(f4*)((float*)p + off) = f4{v[0], v[1], v[2], v[3]};
  }
}

// exact-erf GELU and its derivative (nn.GELU(approximate='none'))
__device__ __forceinline__ float gelu_d(float x) {
  const float phi_cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
  const float pdf = 0.39894228040143267794f * __expf(-0.5f * x * x);
  return phi_cdf + x * pdf;
}

// ------------------------------------------------------------ finalize
// out[i] (+)= sum_{c < nchunk} part[c * stride + i]   (fixed order)
// Block = 16 columns x 16 chunk slices: slice s sums chunks s, s+16, ...
// (independent loads in flight), then the 16 slice sums are added in slice
// order through LDS -- the same order on every run.
__global__ __launch_bounds__(256) void finalize_kernel(const float* __restrict__ part, int nchunk, int n, int stride,
                                                       float* __restrict__ out, int accumulate) {
  __shared__ float red[16][17];
  const int col = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int i = blockIdx.x * 16 + col;
  float s = 0.f;
  if (i < n) {
#pragma unroll 4
    for (int c = sl; c < nchunk; c += 16) s += part[(int64_t)c * stride + i];
  }
  red[sl][col] = s;
  __syncthreads();
  if (sl == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][col];
    out[i] = accumulate ? out[i] + t : t;
  }
}

// Up to four finalizes of one reduction (same chunk count and length, e.g.
// a LayerNorm's weight and bias sums) in one launch: blockIdx.y = vector.
struct FinJobs {
  const float* part[4];
  int stride[4];
  float* out[4];
};

__global__ __launch_bounds__(256) void finalize_multi_kernel(FinJobs jobs, int nchunk, int n, int accumulate) {
  const int j = blockIdx.y;
  __shared__ float red[16][17];
  const float* __restrict__ part = jobs.part[j];
  const int stride = jobs.stride[j];
  const int col = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int i = blockIdx.x * 16 + col;
  float s = 0.f;
  if (i < n) {
#pragma unroll 4
    for (int c = sl; c < nchunk; c += 16) s += part[(int64_t)c * stride + i];
  }
  red[sl][col] = s;
  __syncthreads();
  if (sl == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][col];
    float* out = jobs.out[j];
    out[i] = accumulate ? out[i] + t : t;
  }
}

// queue the non-null (part, stride, out) triples as one finalize_multi launch
static void finalize_many(hipStream_t s, int nchunk, int n, int accumulate, int count, const float* const* parts,
                          const int* strides, float* const* outs) {
  FinJobs jobs{};
  int k = 0;
  for (int a = 0; a < count; ++a)
    if (outs[a]) {
      jobs.part[k] = parts[a];
      jobs.stride[k] = strides[a];
      jobs.out[k] = outs[a];
      ++k;
    }
  if (k) finalize_multi_kernel<<<dim3((n + 15) / 16, k), 256, 0, s>>>(jobs, nchunk, n, accumulate);
}

// ------------------------------------------------------------ column sums
// Block (x, y): columns [x*1024, x*1024+1024) in 4-column vectors, rows of
// chunk y.  MODE 0: part0 = sum a                       (bias gradients)
//           MODE 1: dbr = bf16(gamma * a); part0 = sum a*b; part1 = sum dbr
//                   (LayerScale + residual backward: a = d(out) f32,
//                    b = branch bf16, gamma = LayerScale)
//           MODE 2: dpre = bf16(a * gelu'(b)); part0 = sum dpre
//                   (GELU backward: a = d(hidden) bf16, b = pre-activation)
template <int MODE>
__global__ __launch_bounds__(256) void colred_kernel(const void* __restrict__ a, int adt, int64_t lda,
                                                     const void* __restrict__ b, int bdt, int64_t ldb,
                                                     const float* __restrict__ gamma, void* __restrict__ out, int odt,
                                                     int64_t ldo, int M, int N, int rpc, float* __restrict__ part) {
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (c0 >= N) return;
  const int r0 = blockIdx.y * rpc;
  const int r1 = min(M, r0 + rpc);
  float s0[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f};
  float g[4] = {1.f, 1.f, 1.f, 1.f};
  if (MODE == 1) {
    const f4 gv = *(const f4*)(gamma + c0);
    g[0] = gv[0];
    g[1] = gv[1];
    g[2] = gv[2];
    g[3] = gv[3];
  }
#pragma unroll 4
  for (int r = r0; r < r1; ++r) {
    float av[4];
    load4(a, adt, (int64_t)r * lda + c0, av);
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) s0[j] += av[j];
    } else if (MODE == 1) {
      float bv[4], o[4];
      load4(b, bdt, (int64_t)r * ldb + c0, bv);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s0[j] += av[j] * bv[j];
        o[j] = g[j] * av[j];
      }
      store4(out, odt, (int64_t)r * ldo + c0, o);
      if (odt == VGGT_DTYPE_BF16) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = round_bf(o[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) s1[j] += o[j];
    } else {
      float bv[4], o[4];
      load4(b, bdt, (int64_t)r * ldb + c0, bv);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = av[j] * gelu_d(bv[j]);
      store4(out, odt, (int64_t)r * ldo + c0, o);
      if (odt == VGGT_DTYPE_BF16) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = round_bf(o[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) s0[j] += o[j];
    }
  }
  float* p0 = part + (int64_t)blockIdx.y * N + c0;
  *(f4*)p0 = f4{s0[0], s0[1], s0[2], s0[3]};
  if (MODE == 1) {
    float* p1 = part + ((int64_t)gridDim.y + blockIdx.y) * N + c0;
    *(f4*)p1 = f4{s1[0], s1[1], s1[2], s1[3]};
  }
}

// ------------------------------------------------------------ elementwise
// MODE 0: y = bf16/f32(GELU(x))           (unfused fc1 activation, training recompute)
// MODE 1: x_f32 = src_f32 + gamma * y     (LayerScale residual add with a saved branch; src == x in place)
template <int MODE>
__global__ __launch_bounds__(256) void ew_kernel(const void* x, int xdt, int64_t ldx, void* __restrict__ y,
                                                 int ydt, int64_t ldy, const float* __restrict__ gamma, int M, int N,
                                                 const float* src = nullptr, int64_t lds = 0) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t nvec = (int64_t)M * N;
  if (i >= nvec) return;
  const int r = (int)(i / N), c = (int)(i % N);
  if (MODE == 0) {
    float v[4], o[4];
    load4(x, xdt, (int64_t)r * ldx + c, v);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = gelu_erf(v[j]);
    store4(y, ydt, (int64_t)r * ldy + c, o);
  } else {
    float br[4], acc[4];
    load4(y, ydt, (int64_t)r * ldy + c, br);
    float* xp = (float*)x + (int64_t)r * ldx + c;
    const f4 xv = *(const f4*)(src + (int64_t)r * lds + c);
    const f4 gv = *(const f4*)(gamma + c);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = xv[j] + gv[j] * br[j];
    *(f4*)xp = f4{acc[0], acc[1], acc[2], acc[3]};
  }
}

// ------------------------------------------------------------ transpose
// dst[c][r] = src[r][c] (r < rows), 0 for rows <= r < rows_pad; 64x64 tiles
// through LDS (+1 column of padding), 2-byte elements.
__global__ __launch_bounds__(256) void transpose_b16_kernel(const uint16_t* __restrict__ src, int64_t lds_,
                                                            int rows, int cols, uint16_t* __restrict__ dst,
                                                            int64_t ldd, int rows_pad) {
  __shared__ uint16_t t[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    t[i][tx] = (r < rows && c < cols) ? src[(int64_t)r * lds_ + c] : (uint16_t)0;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows_pad) dst[(int64_t)c * ldd + r] = t[tx][i];
  }
}

// ------------------------------------------------------------ LayerNorm backward
// One wave per row (C = 256*NV), 4 waves per block; block y covers rows
// [blk*rpb, blk*rpb + rpb).  Row mapping as the forward's RowMap: logical
// row r -> group g = r / G, i = r % G;  x / dx row = g*xgs + xoff + i,
// dy row = g*ygs + yoff + i.
//   xhat = (x - mean) * rstd;  gdy = dy * w
//   dx  (+)= rstd * (gdy - mean(gdy) - xhat * mean(gdy * xhat))
//   dw  += dy * xhat;   db += dy      (partials per block, finalize later)
struct RowMap2 {
  int G, xgs, xoff, ygs, yoff;
};

template <int NV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const void* __restrict__ x, int xdt, int64_t ldx,
                                                     const float* __restrict__ w, float eps,
                                                     const void* __restrict__ dy, int ydt, int64_t ldy,
                                                     void* __restrict__ dx, int dxdt, int64_t lddx, int accumulate,
                                                     int M, RowMap2 rm, int rpb, float* __restrict__ part) {
  constexpr int C = NV * 256;
  __shared__ float red[2][4][C];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float aw[NV][4], ab[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) aw[i][j] = ab[i][j] = 0.f;
  float wv[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = i * 256 + lane * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) wv[i][j] = w ? w[c + j] : 1.f;
  }
  const int rbeg = blockIdx.x * rpb, rend = min(M, rbeg + rpb);
  for (int r = rbeg + wave; r < rend; r += 4) {
    const int gi = r / rm.G, ii = r % rm.G;
    const int64_t xr = (int64_t)gi * rm.xgs + rm.xoff + ii;
    const int64_t yr = (int64_t)gi * rm.ygs + rm.yoff + ii;
    float v[NV][4], g[NV][4], prev[NV][4];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = i * 256 + lane * 4;
      load4(x, xdt, xr * ldx + c, v[i]);
      load4(dy, ydt, yr * ldy + c, g[i]);
      if (accumulate) load4(dx, dxdt, xr * lddx + c, prev[i]);  // issued with the operands, used at the end
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
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float xh = (v[i][j] - mean) * rstd;
        v[i][j] = xh;
        aw[i][j] += g[i][j] * xh;
        ab[i][j] += g[i][j];
        const float gd = g[i][j] * wv[i][j];
        g[i][j] = gd;
        s1 += gd;
        s2 += gd * xh;
      }
    const float m1 = wave_sum(s1) * (1.f / C), m2 = wave_sum(s2) * (1.f / C);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = i * 256 + lane * 4;
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = rstd * (g[i][j] - m1 - v[i][j] * m2);
      if (accumulate) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] += prev[i][j];
      }
      store4(dx, dxdt, xr * lddx + c, o);
    }
  }
  if (!part) return;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[0][wave][i * 256 + lane * 4 + j] = aw[i][j];
      red[1][wave][i * 256 + lane * 4 + j] = ab[i][j];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    part[(int64_t)blockIdx.x * C + c] = (red[0][0][c] + red[0][1][c]) + (red[0][2][c] + red[0][3][c]);
    part[((int64_t)gridDim.x + blockIdx.x) * C + c] = (red[1][0][c] + red[1][1][c]) + (red[1][2][c] + red[1][3][c]);
  }
}

template <int NV>
void launch_ln_bwd(const void* x, int xdt, int64_t ldx, const float* w, float eps, const void* dy, int ydt,
                   int64_t ldy, void* dx, int dxdt, int64_t lddx, int acc, int M, RowMap2 rm, int nblk, int rpb,
                   float* part, hipStream_t s) {
  ln_bwd_kernel<NV><<<nblk, 256, 0, s>>>(x, xdt, ldx, w, eps, dy, ydt, ldy, dx, dxdt, lddx, acc, M, rm, rpb, part);
}

// ------------------------------------------------------------ per-head norm + RoPE backward
// Forward (norm.hip headnorm_rope_kernel / small.hip f32 variant): for head h
// of row m, u = pre-norm values, xhat = LN(u), y = xhat*w + b, z = rope(y).
// Backward: dy[e] = dz[e]*cos[e] + (first half ? dz[e+R/2] : -dz[e-R/2]) * sin[e]
// (sin/cos tables are cat(angles, angles)), then the LayerNorm backward over
// the head's D values.  du overwrites dz in place.  Heads [0, hsplit) belong
// to weight set 0 (q_norm), the rest to set 1 (k_norm); parameter partials
// part[blk][set][w|b][D].
template <int D, int MODE, int DT>
__global__ __launch_bounds__(256) void headnorm_rope_bwd_kernel(const void* __restrict__ pre, int64_t ldp,
                                                                void* __restrict__ grad, int64_t ldg, int M, int H,
                                                                int hsplit, const float* __restrict__ w0,
                                                                const float* __restrict__ w1, float eps,
                                                                const int32_t* __restrict__ pos, int period,
                                                                const float* __restrict__ cs,
                                                                const float* __restrict__ sn, int tab_len, int rpb,
                                                                float* __restrict__ part) {
  constexpr int LPH = D / 8;
  constexpr int HPP = 64 / LPH;
  __shared__ float red[256][33];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane % LPH;
  const int e0 = sub * 8;
  float acc[4][8];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[a][j] = 0.f;
  float wa[8], wb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    wa[j] = w0 ? w0[e0 + j] : 1.f;
    wb[j] = w1 ? w1[e0 + j] : 1.f;
  }
  const int rbeg = blockIdx.x * rpb, rend = min(M, rbeg + rpb);
  for (int row = rbeg + wave; row < rend; row += 4) {
    int p0 = 0, p1 = 0;
    if constexpr (MODE == VGGT_ROPE_2D) {
      const int pr = row % period;
      p0 = min(max(pos[2 * pr], 0), tab_len - 1);
      p1 = min(max(pos[2 * pr + 1], 0), tab_len - 1);
    } else if constexpr (MODE == VGGT_ROPE_1D) {
      p0 = min(max(pos[row % period], 0), tab_len - 1);
    }
    for (int h0 = 0; h0 < H; h0 += HPP) {
      const int h = h0 + lane / LPH;
      const bool act = h < H;
      const int hh = act ? h : 0;
      const bool set0 = hh < hsplit;
      float u[8], dz[8];
      {
        const int64_t po = (int64_t)row * ldp + hh * D + e0, go = (int64_t)row * ldg + hh * D + e0;
        load4(pre, DT, po, u);
        load4(pre, DT, po + 4, u + 4);
        load4(grad, DT, go, dz);
        load4(grad, DT, go + 4, dz + 4);
      }
      float dy[8];
      if constexpr (MODE != VGGT_ROPE_NONE) {
        constexpr int RD = (MODE == VGGT_ROPE_2D) ? D / 2 : D;
        constexpr int PL = RD / 16;
        const int er = e0 % RD;
        const int pp = (MODE == VGGT_ROPE_2D && e0 >= D / 2) ? p1 : p0;
        const bool first = er < RD / 2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float partner = __shfl_xor(dz[j], PL, 64);
          dy[j] = dz[j] * cs[pp * RD + er + j] + (first ? partner : -partner) * sn[pp * RD + er + j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) dy[j] = dz[j];
      }
      const bool norm = set0 ? (w0 != nullptr) : (w1 != nullptr);
      float du[8];
      if (norm) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += u[j];
#pragma unroll
        for (int o = 1; o < LPH; o <<= 1) s += __shfl_xor(s, o, 64);
        const float mean = s * (1.f / D);
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = u[j] - mean;
          q += d * d;
        }
#pragma unroll
        for (int o = 1; o < LPH; o <<= 1) q += __shfl_xor(q, o, 64);
        const float rstd = rsqrtf(q * (1.f / D) + eps);
        float s1 = 0.f, s2 = 0.f, xh[8], gd[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[j] = (u[j] - mean) * rstd;
          gd[j] = dy[j] * (set0 ? wa[j] : wb[j]);
          s1 += gd[j];
          s2 += gd[j] * xh[j];
        }
#pragma unroll
        for (int o = 1; o < LPH; o <<= 1) {
          s1 += __shfl_xor(s1, o, 64);
          s2 += __shfl_xor(s2, o, 64);
        }
        const float m1 = s1 * (1.f / D), m2 = s2 * (1.f / D);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          du[j] = rstd * (gd[j] - m1 - xh[j] * m2);
          if (act) {
            acc[set0 ? 0 : 2][j] += dy[j] * xh[j];
            acc[set0 ? 1 : 3][j] += dy[j];
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) du[j] = dy[j];
      }
      if (act) {
        const int64_t go = (int64_t)row * ldg + hh * D + e0;
        store4(grad, DT, go, du);
        store4(grad, DT, go + 4, du + 4);
      }
    }
  }
  if (!part) return;
  // block reduction: lanes with the same `sub` own the same 8 elements
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x][a * 8 + j] = acc[a][j];
  __syncthreads();
  for (int o = threadIdx.x; o < 4 * D; o += 256) {
    const int a = o / D, e = o % D;
    const int sb = e / 8, j = e % 8;
    float s = 0.f;
    for (int t = sb; t < 256; t += LPH) s += red[t][a * 8 + j];  // t % LPH == sb (LPH | 64)
    part[(int64_t)blockIdx.x * 4 * D + o] = s;
  }
}

// ------------------------------------------------------------ small attention backward
// One 256-thread workgroup per (batch, head); everything in LDS as fp32:
// recompute S = q k^T * scale, P = softmax(S); dP = dO v^T;
// dS = P * (dP - rowsum(P * dP)); dq = scale dS k; dk = scale dS^T q; dv = P^T dO.
// (rowsum(P * dP) = rowsum(dO * O): the same delta without reading O.)
// Operand rows are padded to D+1 floats so the score loops (a thread per
// (query, key), key rows at stride D+1) are bank-conflict free; operands are
// read 16 B per lane when rows are 16-B aligned (vec), and each thread of the
// output loops produces two adjacent columns (one 4-B bf16x2 / 8-B f32x2 store).
__global__ __launch_bounds__(256) void attn_small_bwd_kernel(
    const void* __restrict__ q, int64_t ldq, int64_t qbs, const void* __restrict__ k, int64_t ldk, int64_t kbs,
    const void* __restrict__ v, int64_t ldv, int64_t vbs, const void* __restrict__ dout, int64_t ldo, int64_t obs,
    void* __restrict__ dq, int64_t ldgq, int64_t gqbs, void* __restrict__ dk, void* __restrict__ dv, int64_t ldgk,
    int64_t gkbs, int dtype, int heads, int nq, int nk, int D, float scale, int vec) {
  extern __shared__ float sm[];
  const int DP = D + 1;
  float* sq = sm;                 // [nq][DP]
  float* sdo = sq + nq * DP;      // [nq][DP]
  float* sk = sdo + nq * DP;      // [nk][DP]
  float* sv = sk + nk * DP;       // [nk][DP]
  float* sp = sv + nk * DP;       // [nq][nk]  P, then dS
  float* sdp = sp + nq * nk;      // [nq][nk]  dP, then P
  const int tid = threadIdx.x;
  const int b = blockIdx.x / heads, h = blockIdx.x % heads;
  const bool bf = dtype == VGGT_DTYPE_BF16;
  auto stage = [&](float* dst, const void* base, int64_t bs, int64_t ld, int rows) {
    if (vec) {
      const int cpr = D / 8;
      for (int i = tid; i < rows * cpr; i += 256) {
        const int r = i / cpr, ch = i % cpr;
        const int64_t off = ((int64_t)b * bs + r) * ld + h * D + ch * 8;
        float f[8];
        if (bf) {
          const uint4 u = *(const uint4*)((const bf16_t*)base + off);
          const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            f[2 * t] = bf2f((bf16_t)(w4[t] & 0xffff));
            f[2 * t + 1] = bf2f((bf16_t)(w4[t] >> 16));
          }
        } else {
          const f4 a0 = *(const f4*)((const float*)base + off), a1 = *(const f4*)((const float*)base + off + 4);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            f[t] = a0[t];
            f[4 + t] = a1[t];
          }
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) dst[r * DP + ch * 8 + t] = f[t];
      }
    } else {
      for (int i = tid; i < rows * D; i += 256) {
        const int r = i / D, c = i % D;
        const int64_t off = ((int64_t)b * bs + r) * ld + h * D + c;
        dst[r * DP + c] = bf ? bf2f(((const bf16_t*)base)[off]) : ((const float*)base)[off];
      }
    }
  };
  stage(sq, q, qbs, ldq, nq);
  stage(sdo, dout, obs, ldo, nq);
  stage(sk, k, kbs, ldk, nk);
  stage(sv, v, vbs, ldv, nk);
  __syncthreads();
  for (int i = tid; i < nq * nk; i += 256) {
    const int r = i / nk, c = i % nk;
    const float* qr = sq + r * DP;
    const float* gr = sdo + r * DP;
    const float* kr = sk + c * DP;
    const float* vr = sv + c * DP;
    float s0 = 0.f, s1 = 0.f, t0 = 0.f, t1 = 0.f;
    for (int d = 0; d < D; d += 2) {
      s0 += qr[d] * kr[d];
      s1 += qr[d + 1] * kr[d + 1];
      t0 += gr[d] * vr[d];
      t1 += gr[d + 1] * vr[d + 1];
    }
    sp[i] = (s0 + s1) * scale;
    sdp[i] = t0 + t1;
  }
  __syncthreads();
  for (int r = tid; r < nq; r += 256) {
    float m = -INFINITY;
    for (int c = 0; c < nk; ++c) m = fmaxf(m, sp[r * nk + c]);
    float l = 0.f;
    for (int c = 0; c < nk; ++c) {
      const float e = __expf(sp[r * nk + c] - m);
      sp[r * nk + c] = e;
      l += e;
    }
    const float inv = 1.f / l;
    float delta = 0.f;
    for (int c = 0; c < nk; ++c) {
      sp[r * nk + c] *= inv;
      delta += sp[r * nk + c] * sdp[r * nk + c];
    }
    // keep P in sdp's slot for dv, dS in sp's
    for (int c = 0; c < nk; ++c) {
      const float p = sp[r * nk + c];
      const float ds = p * (sdp[r * nk + c] - delta);
      sdp[r * nk + c] = p;
      sp[r * nk + c] = ds;
    }
  }
  __syncthreads();
  auto st2 = [&](void* base, int64_t off, float a0, float a1) {
    if (bf) {
      *(uint32_t*)((bf16_t*)base + off) = pack_bf2(a0, a1);
    } else {
      ((float*)base)[off] = a0;
      ((float*)base)[off + 1] = a1;
    }
  };
  const int D2 = D / 2;
  for (int i = tid; i < nq * D2; i += 256) {
    const int r = i / D2, c = 2 * (i % D2);
    float s0 = 0.f, s1 = 0.f;
    for (int j = 0; j < nk; ++j) {
      const float ds = sp[r * nk + j];
      s0 += ds * sk[j * DP + c];
      s1 += ds * sk[j * DP + c + 1];
    }
    st2(dq, ((int64_t)b * gqbs + r) * ldgq + h * D + c, s0 * scale, s1 * scale);
  }
  for (int i = tid; i < nk * D2; i += 256) {
    const int r = i / D2, c = 2 * (i % D2);
    float s0 = 0.f, s1 = 0.f, t0 = 0.f, t1 = 0.f;
    for (int j = 0; j < nq; ++j) {
      const float ds = sp[j * nk + r], p = sdp[j * nk + r];
      s0 += ds * sq[j * DP + c];
      s1 += ds * sq[j * DP + c + 1];
      t0 += p * sdo[j * DP + c];
      t1 += p * sdo[j * DP + c + 1];
    }
    st2(dk, ((int64_t)b * gkbs + r) * ldgk + h * D + c, s0 * scale, s1 * scale);
    st2(dv, ((int64_t)b * gkbs + r) * ldgk + h * D + c, t0, t1);
  }
}

// ------------------------------------------------------------ fp32 weight gradient
// dW[n][k] (+)= sum_m dY[m][n] * X[m][k]  (skinny M: the fp32 decoder /
// gated-update linears, M = batch * frames <= a few hundred).  Thread per
// output, 64 consecutive k per wave (coalesced X reads), dY[m][n] broadcast.
// db != NULL: column k == K is the bias (an all-ones X column), db[n] = sum_m dY[m, n]
__global__ __launch_bounds__(256) void wgrad_f32_kernel(const float* __restrict__ dy, int64_t ldy,
                                                        const float* __restrict__ x, int64_t ldx, int M, int N, int K,
                                                        float* __restrict__ dw, int64_t ldw, int accumulate,
                                                        float* __restrict__ db) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  const int n = blockIdx.y;
  if (k > K || (k == K && !db)) return;
  float s = 0.f;
  if (k < K) {
    for (int m = 0; m < M; ++m) s += dy[(int64_t)m * ldy + n] * x[(int64_t)m * ldx + k];
  } else {
    for (int m = 0; m < M; ++m) s += dy[(int64_t)m * ldy + n];
  }
  float* o = k < K ? dw + (int64_t)n * ldw + k : db + n;
  *o = accumulate ? *o + s : s;
}

// out partials: part[chunk][b] = sum over the chunk's elements of a * c
__global__ __launch_bounds__(256) void batch_dot_kernel(const float* __restrict__ a, const float* __restrict__ c,
                                                        int64_t bs, int B, int64_t n, int64_t per_chunk,
                                                        float* __restrict__ part) {
  __shared__ float red[4];
  const int b = blockIdx.y;
  const int64_t i0 = (int64_t)blockIdx.x * per_chunk, i1 = min(n, i0 + per_chunk);
  float s = 0.f;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) s += a[(int64_t)b * bs + i] * c[(int64_t)b * bs + i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[(int64_t)blockIdx.x * B + b] = (red[0] + red[1]) + (red[2] + red[3]);
}


// ------------------------------------------------------------ bf16 weight gradient (split-K over tokens)
// part[z][n][k] = sum_{m in split z} dY[m][n] X[m][k]: both operands read
// row-major from HBM (no transposes); the token dimension m is the MFMA
// reduction, so both fragments come from ds_read_b64_tr_b16 transposed reads
// of the padded [32 m][128] LDS tiles (vggt_frag::trfrag, the same k
// permutation on A and B).  128x128 output tile per workgroup, 4 waves x
// (64 x 64), double-buffered LDS, register-staged loads of tile t+1 in
// flight during tile t's MFMAs.
__global__ __launch_bounds__(256) void wgrad_bf16_kernel(const bf16_t* __restrict__ dy, int64_t ldy,
                                                         const bf16_t* __restrict__ x, int64_t ldx, int M, int N,
                                                         int K, int mchunk, float* __restrict__ part) {
  using namespace vggt_frag;
  constexpr int ROWP = Geo<128>::ROWP;
  constexpr int TB = 32 * ROWP;
  __shared__ __attribute__((aligned(16))) char smem[2][2 * TB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ntn = N / 128;
  const int n0 = (blockIdx.x % ntn) * 128, k0 = (blockIdx.x / ntn) * 128;
  const int mb = blockIdx.y * mchunk, me = min(M, mb + mchunk);
  const int wn = (wave >> 1) * 64, wk = (wave & 1) * 64;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  // staging: 512 16-B chunks per operand tile; thread t moves chunks t and t+256
  uint4 ry[2], rx[2];
  auto load = [&](int m0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = threadIdx.x + 256 * i, row = c >> 4, ch = c & 15;
      const int m = m0 + row;
      ry[i] = m < me ? *(const uint4*)(dy + (int64_t)m * ldy + n0 + ch * 8) : uint4{0u, 0u, 0u, 0u};
      rx[i] = m < me ? *(const uint4*)(x + (int64_t)m * ldx + k0 + ch * 8) : uint4{0u, 0u, 0u, 0u};
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = threadIdx.x + 256 * i, row = c >> 4, ch = c & 15;
      *(uint4*)(&smem[buf][row * ROWP + ch * 16]) = ry[i];
      *(uint4*)(&smem[buf][TB + row * ROWP + ch * 16]) = rx[i];
    }
  };
  const int nt = (me - mb + 31) / 32;  // >= 1: the host never launches an empty split
  load(mb);
  store(0);
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) load(mb + (t + 1) * 32);
    const char* ty = smem[cur];
    const char* tx = smem[cur] + TB;
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = trfrag<128>(ty, (wn >> 5) + i, 0, ss, lane);
        bfr[i] = trfrag<128>(tx, (wk >> 5) + i, 0, ss, lane);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < nt) store(cur ^ 1);
    __syncthreads();
  }
  const int hl = lane >> 5;
  float* pz = part + (int64_t)blockIdx.y * N * K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const int k = k0 + wk + 32 * j + (lane & 31);
        pz[(int64_t)n * K + k] = acc[i][j][r];
      }
}

// The same product with the token tiles staged by LDS-DMA (buffer_load ... lds)
// into a 3-slot ring, two tiles ahead, counted waits: no register round trip,
// so the L2 latency of tile t+2 hides behind tiles t and t+1 (the register-
// staged form waits vmcnt(0) once per 8 MFMAs).  The padded [32][128 + 8] row
// image is reproduced by the per-lane source offsets: LDS unit u (16 B) of a
// tile is row u / 17, 16-B chunk u % 17 (chunk 16 = the pad: loads a duplicate
// of chunk 15); 10 pieces of 64 units per operand tile (640 >= 544 units, the
// surplus lands in the tile's padding).  Rows past the split read zeros through
// the per-tile descriptor's range check (see stage()).
typedef int wg_i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void wg_dma16(wg_i32x4 rsrc, uint32_t voff, uint32_t soff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
               : "memory");
}
__device__ __forceinline__ wg_i32x4 wg_rsrc(const void* base, uint32_t nbytes) {
  const uint64_t b = (uint64_t)base;
  wg_i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((uint32_t)b);
  r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) & 0xffff;
  r[2] = __builtin_amdgcn_readfirstlane(nbytes);
  r[3] = 0x00020000;
  return r;
}

constexpr int WG_TILE = 10 * 1024;       // LDS bytes per operand tile (10 DMA pieces)
constexpr int WG_SLOT = 2 * WG_TILE;     // dY tile + X tile
constexpr int WG_NSLOT = 3;

__global__ __launch_bounds__(256) void wgrad_dma_kernel(const bf16_t* __restrict__ dy, int64_t ldy,
                                                        const bf16_t* __restrict__ x, int64_t ldx, int M, int N,
                                                        int K, int mchunk, float* __restrict__ part) {
  using namespace vggt_frag;
  static_assert(32 * Geo<128>::ROWP <= WG_TILE, "tile image fits its slot");
  extern __shared__ __attribute__((aligned(16))) char wsm[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ntn = N / 128;
  const int n0 = (blockIdx.x % ntn) * 128, k0 = (blockIdx.x / ntn) * 128;
  const int mb = blockIdx.y * mchunk, me = min(M, mb + mchunk);
  const int wn = (wave >> 1) * 64, wk = (wave & 1) * 64;
  // waves 0-1 stage the dY tile, waves 2-3 the X tile, 5 pieces each:
  // piece p = 5 (wave & 1) + i of operand wave >> 1
  const bool xo = wave >= 2;
  const int64_t ld = xo ? ldx : ldy;
  const bf16_t* src0 = xo ? x + (int64_t)mb * ldx : dy + (int64_t)mb * ldy;
  const int rows = me - mb;
  uint32_t voff[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int u = (5 * (wave & 1) + i) * 64 + lane;
    const int r = min(u / 17, 31), c = min(u % 17, 15);
    voff[i] = (uint32_t)(r * ld + (xo ? k0 : n0) + c * 8) * 2u;
  }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(wsm)) + (xo ? WG_TILE : 0) +
                        5 * (wave & 1) * 1024;
  // The buffer range check sees voffset (+ inst offset) only, never soffset, so
  // the descriptor is re-based per tile: base = row 32 t of the split, range =
  // the split's remaining rows.  Rows past the split (the ragged last tile, and
  // the surplus tiles t >= nt staged by the two-ahead prefetch) read zeros and
  // touch no memory; every tile still issues its 5 pieces, so the counted waits
  // below stay exact.
  auto stage = [&](int slot, int t) {
    const uint32_t b = lds0 + slot * WG_SLOT;
    const int rem = max(0, rows - 32 * t);
    const wg_i32x4 rs = wg_rsrc(src0 + (int64_t)32 * t * ld, (uint32_t)((int64_t)rem * ld * 2));
#pragma unroll
    for (int i = 0; i < 5; ++i) wg_dma16(rs, voff[i], 0u, b + i * 1024);
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  const int nt = (me - mb + 31) / 32;  // >= 1: the host never launches an empty split
  stage(0, 0);
  stage(1, 1);
  asm volatile("s_waitcnt vmcnt(5)\n\ts_barrier" ::: "memory");  // tile 0 landed everywhere
  int slot = 0;
  for (int t = 0; t < nt; ++t) {
    // tile t+2 into the slot tile t-1 used (every wave passed the barrier after it);
    // past the split: zero reads into a slot nobody reads again
    const int s2 = slot == 0 ? 2 : slot - 1;
    stage(s2, t + 2);
    const char* ty = wsm + slot * WG_SLOT;
    const char* tx = ty + WG_TILE;
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = trfrag<128>(ty, (wn >> 5) + i, 0, ss, lane);
        bfr[i] = trfrag<128>(tx, (wk >> 5) + i, 0, ss, lane);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    // tile t+1 landed (its 5 pieces are older than tile t+2's 5), reads of slot done
    asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    slot = slot == 2 ? 0 : slot + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the surplus DMA before the workgroup ends
  const int hl = lane >> 5;
  float* pz = part + (int64_t)blockIdx.y * N * K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const int k = k0 + wk + 32 * j + (lane & 31);
        pz[(int64_t)n * K + k] = acc[i][j][r];
      }
}

// out[n][k] (+)= round_bf16(sum_z part[z][n][k])  (fixed split order)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int nz, int64_t nk,
                                                           float* __restrict__ out, int64_t ldo, int K,
                                                           int accumulate, int round) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nk) return;
  float s = 0.f;
  for (int z = 0; z < nz; ++z) s += part[(int64_t)z * nk + i];
  if (round) s = round_bf(s);
  float* o = out + (i / K) * ldo + (i % K);
  *o = accumulate ? *o + s : s;
}

int nchunks_for(int M, int maxc, int rows = 64) {
  int c = (M + rows - 1) / rows;
  return c < 1 ? 1 : (c > maxc ? maxc : c);
}
// Row chunking of the column reductions / row-wise backward kernels: enough
// workgroups (up to ~4 per CU) that the serial per-row loads of each wave
// overlap across waves; more chunks only add fp32 partials (<= 8 MB).
constexpr int COLRED_MAXC = 1024, COLRED_ROWS = 16;
constexpr int ROWBWD_MAXC = 2048, ROWBWD_ROWS = 16;

}  // namespace

// ============================================================ C ABI
extern "C" size_t vggt_colred_workspace_bytes(int M, int N) {
  return (size_t)2 * nchunks_for(M, COLRED_MAXC, COLRED_ROWS) * (size_t)N * sizeof(float);
}

extern "C" int vggt_colsum(const void* x, int dtype, int64_t ldx, int M, int N, float* out, int accumulate, void* ws,
                           size_t ws_bytes, void* stream) {
  if (M <= 0 || N <= 0 || N % 4) return VGGT_ERR_SHAPE;
  if (dtype != VGGT_DTYPE_F32 && dtype != VGGT_DTYPE_BF16) return VGGT_ERR_UNSUPPORTED;
  if (ldx % 4 || (uintptr_t)x % 8) return VGGT_ERR_ALIGN;
  const int nc = nchunks_for(M, COLRED_MAXC, COLRED_ROWS);
  if (!ws || ws_bytes < (size_t)nc * N * sizeof(float)) return VGGT_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  const int rpc = (M + nc - 1) / nc;
  dim3 grid((N / 4 + 255) / 256, nc);
  colred_kernel<0><<<grid, 256, 0, s>>>(x, dtype, ldx, nullptr, 0, 0, nullptr, nullptr, 0, 0, M, N, rpc, (float*)ws);
  finalize_kernel<<<(N + 15) / 16, 256, 0, s>>>((const float*)ws, nc, N, N, out, accumulate);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_layerscale_bwd(const float* dout, int64_t ldd, const void* branch, int bdtype, int64_t ldb,
                                   const float* gamma, void* dbranch, int odtype, int64_t ldo, int M, int N,
                                   float* dgamma, float* dbias, void* ws, size_t ws_bytes, void* stream) {
  if (M <= 0 || N <= 0 || N % 4) return VGGT_ERR_SHAPE;
  if ((ldd | ldb | ldo) % 4 || ((uintptr_t)dout | (uintptr_t)gamma) % 16 || ((uintptr_t)branch | (uintptr_t)dbranch) % 8)
    return VGGT_ERR_ALIGN;
  const int nc = nchunks_for(M, COLRED_MAXC, COLRED_ROWS);
  if (!ws || ws_bytes < (size_t)2 * nc * N * sizeof(float)) return VGGT_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  const int rpc = (M + nc - 1) / nc;
  dim3 grid((N / 4 + 255) / 256, nc);
  colred_kernel<1><<<grid, 256, 0, s>>>(dout, VGGT_DTYPE_F32, ldd, branch, bdtype, ldb, gamma, dbranch, odtype, ldo,
                                        M, N, rpc, (float*)ws);
  const float* parts[2] = {(const float*)ws, (const float*)ws + (size_t)nc * N};
  const int strides[2] = {N, N};
  float* outs[2] = {dgamma, dbias};
  finalize_many(s, nc, N, 1, 2, parts, strides, outs);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_gelu_fwd(const void* x, int xdtype, int64_t ldx, void* y, int ydtype, int64_t ldy, int M, int N,
                             void* stream) {
  if (M <= 0 || N <= 0 || N % 4) return M == 0 ? VGGT_OK : VGGT_ERR_SHAPE;
  if ((ldx | ldy) % 4 || ((uintptr_t)x | (uintptr_t)y) % 8) return VGGT_ERR_ALIGN;
  const int64_t nv = (int64_t)M * N / 4;
  ew_kernel<0><<<(unsigned)((nv + 255) / 256), 256, 0, (hipStream_t)stream>>>(x, xdtype, ldx, y, ydtype, ldy, nullptr,
                                                                               M, N);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_gelu_bwd(const void* dh, int dhdtype, int64_t lddh, const void* pre, int predtype, int64_t ldp,
                             void* dpre, int odtype, int64_t ldo, int M, int N, float* dbias, void* ws,
                             size_t ws_bytes, void* stream) {
  if (M <= 0 || N <= 0 || N % 4) return VGGT_ERR_SHAPE;
  if ((lddh | ldp | ldo) % 4 || ((uintptr_t)dh | (uintptr_t)pre | (uintptr_t)dpre) % 8) return VGGT_ERR_ALIGN;
  const int nc = nchunks_for(M, COLRED_MAXC, COLRED_ROWS);
  if (!ws || ws_bytes < (size_t)nc * N * sizeof(float)) return VGGT_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  const int rpc = (M + nc - 1) / nc;
  dim3 grid((N / 4 + 255) / 256, nc);
  colred_kernel<2><<<grid, 256, 0, s>>>(dh, dhdtype, lddh, pre, predtype, ldp, nullptr, dpre, odtype, ldo, M, N, rpc,
                                        (float*)ws);
  if (dbias) finalize_kernel<<<(N + 15) / 16, 256, 0, s>>>((const float*)ws, nc, N, N, dbias, 1);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_resid_scale_add_from(float* out, int64_t ldo, const float* x, int64_t ldx, const void* branch,
                                         int bdtype, int64_t ldb, const float* gamma, int M, int N, void* stream) {
  if (M <= 0 || N <= 0 || N % 4) return M == 0 ? VGGT_OK : VGGT_ERR_SHAPE;
  if ((ldo | ldx | ldb) % 4 || (uintptr_t)out % 16 || (uintptr_t)x % 16 || (uintptr_t)gamma % 16 ||
      (uintptr_t)branch % 8)
    return VGGT_ERR_ALIGN;
  const int64_t nv = (int64_t)M * N / 4;
  ew_kernel<1><<<(unsigned)((nv + 255) / 256), 256, 0, (hipStream_t)stream>>>(out, VGGT_DTYPE_F32, ldo, (void*)branch,
                                                                               bdtype, ldb, gamma, M, N, x, ldx);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_resid_scale_add(float* x, int64_t ldx, const void* branch, int bdtype, int64_t ldb,
                                    const float* gamma, int M, int N, void* stream) {
  return vggt_resid_scale_add_from(x, ldx, x, ldx, branch, bdtype, ldb, gamma, M, N, stream);
}

extern "C" int vggt_transpose_b16(const void* src, int64_t lds, int rows, int cols, void* dst, int64_t ldd,
                                  int rows_pad, void* stream) {
  if (rows < 0 || cols <= 0 || rows_pad < rows) return VGGT_ERR_SHAPE;
  if (rows_pad == 0) return VGGT_OK;
  dim3 grid((cols + 63) / 64, (rows_pad + 63) / 64);
  transpose_b16_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((const uint16_t*)src, lds, rows, cols, (uint16_t*)dst,
                                                              ldd, rows_pad);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" size_t vggt_layernorm_bwd_workspace_bytes(int M, int C) {
  return (size_t)2 * nchunks_for(M, ROWBWD_MAXC, ROWBWD_ROWS) * (size_t)C * sizeof(float);
}

extern "C" int vggt_layernorm_bwd(const void* x, int xdtype, int64_t ldx, const float* w, float eps, const void* dy,
                                  int dydtype, int64_t ldy, void* dx, int dxdtype, int64_t lddx, int accumulate, int M,
                                  int C, int group, int x_group_stride, int x_row_offset, int y_group_stride,
                                  int y_row_offset, float* dw, float* db, void* ws, size_t ws_bytes, void* stream) {
  if (M <= 0) return M == 0 ? VGGT_OK : VGGT_ERR_SHAPE;
  if (C % 256 || C > 1024 || group <= 0) return VGGT_ERR_SHAPE;
  if (accumulate & ~(VGGT_LN_BWD_DX_ACCUMULATE | VGGT_LN_BWD_PARAMS_WRITE)) return VGGT_ERR_UNSUPPORTED;
  const int param_acc = (accumulate & VGGT_LN_BWD_PARAMS_WRITE) ? 0 : 1;
  accumulate &= VGGT_LN_BWD_DX_ACCUMULATE;
  if (accumulate && dxdtype != VGGT_DTYPE_F32) return VGGT_ERR_UNSUPPORTED;
  if ((ldx | ldy | lddx) % 4 || ((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx) % 8) return VGGT_ERR_ALIGN;
  const int nblk = nchunks_for(M, ROWBWD_MAXC, ROWBWD_ROWS);
  const bool want = dw || db;
  if (want && (!ws || ws_bytes < (size_t)2 * nblk * C * sizeof(float))) return VGGT_ERR_SHAPE;
  const int rpb = (M + nblk - 1) / nblk;
  RowMap2 rm{group, x_group_stride, x_row_offset, y_group_stride, y_row_offset};
  hipStream_t s = (hipStream_t)stream;
  float* part = want ? (float*)ws : nullptr;
  switch (C / 256) {
    case 1: launch_ln_bwd<1>(x, xdtype, ldx, w, eps, dy, dydtype, ldy, dx, dxdtype, lddx, accumulate, M, rm, nblk, rpb, part, s); break;
    case 2: launch_ln_bwd<2>(x, xdtype, ldx, w, eps, dy, dydtype, ldy, dx, dxdtype, lddx, accumulate, M, rm, nblk, rpb, part, s); break;
    case 4: launch_ln_bwd<4>(x, xdtype, ldx, w, eps, dy, dydtype, ldy, dx, dxdtype, lddx, accumulate, M, rm, nblk, rpb, part, s); break;
    default: return VGGT_ERR_SHAPE;
  }
  if (want) {
    const float* parts[2] = {part, part + (size_t)nblk * C};
    const int strides[2] = {C, C};
    float* outs[2] = {dw, db};
    finalize_many(s, nblk, C, param_acc, 2, parts, strides, outs);
  }
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" size_t vggt_headnorm_rope_bwd_workspace_bytes(int M, int D) {
  return (size_t)4 * nchunks_for(M, ROWBWD_MAXC, ROWBWD_ROWS) * (size_t)D * sizeof(float);
}

extern "C" int vggt_headnorm_rope_bwd(const void* pre, int64_t ldp, void* grad, int64_t ldg, int dtype, int M, int H,
                                      int hsplit, int D, const float* w0, const float* w1, float eps, int rope_mode,
                                      const int32_t* pos, int period, const float* cos_tab, const float* sin_tab,
                                      int tab_len, float* dw0, float* db0, float* dw1, float* db1, void* ws,
                                      size_t ws_bytes, void* stream) {
  if (M <= 0) return M == 0 ? VGGT_OK : VGGT_ERR_SHAPE;
  if (H <= 0 || (D != 64 && D != 128) || hsplit < 0 || hsplit > H) return VGGT_ERR_SHAPE;
  if (dtype != VGGT_DTYPE_F32 && dtype != VGGT_DTYPE_BF16) return VGGT_ERR_UNSUPPORTED;
  if ((ldp | ldg) % 8 || ((uintptr_t)pre | (uintptr_t)grad) % 16) return VGGT_ERR_ALIGN;
  if (rope_mode != VGGT_ROPE_NONE && (!pos || !cos_tab || !sin_tab || period <= 0 || tab_len <= 0))
    return VGGT_ERR_SHAPE;
  const int nblk = nchunks_for(M, ROWBWD_MAXC, ROWBWD_ROWS);
  const bool want = (w0 || w1) && (dw0 || db0 || dw1 || db1);
  if (want && (!ws || ws_bytes < (size_t)4 * nblk * D * sizeof(float))) return VGGT_ERR_SHAPE;
  const int rpb = (M + nblk - 1) / nblk;
  float* part = want ? (float*)ws : nullptr;
  hipStream_t s = (hipStream_t)stream;
#define VGGT_HNRB(DD, MM, DT)                                                                                       \
  headnorm_rope_bwd_kernel<DD, MM, DT><<<nblk, 256, 0, s>>>(pre, ldp, grad, ldg, M, H, hsplit, w0, w1, eps, pos,   \
                                                            period, cos_tab, sin_tab, tab_len, rpb, part)
#define VGGT_HNRB_M(DD, DT)                                                     \
  switch (rope_mode) {                                                          \
    case VGGT_ROPE_NONE: VGGT_HNRB(DD, VGGT_ROPE_NONE, DT); break;              \
    case VGGT_ROPE_2D: VGGT_HNRB(DD, VGGT_ROPE_2D, DT); break;                  \
    case VGGT_ROPE_1D: VGGT_HNRB(DD, VGGT_ROPE_1D, DT); break;                  \
    default: return VGGT_ERR_UNSUPPORTED;                                       \
  }
  if (D == 64) {
    if (dtype == VGGT_DTYPE_BF16) { VGGT_HNRB_M(64, VGGT_DTYPE_BF16) } else { VGGT_HNRB_M(64, VGGT_DTYPE_F32) }
  } else {
    if (dtype == VGGT_DTYPE_BF16) { VGGT_HNRB_M(128, VGGT_DTYPE_BF16) } else { VGGT_HNRB_M(128, VGGT_DTYPE_F32) }
  }
#undef VGGT_HNRB_M
#undef VGGT_HNRB
  if (part) {
    float* outs[4] = {dw0, db0, dw1, db1};
    // part layout [blk][a][D] -> finalize each (a) slice with stride 4*D per block
    const float* parts[4] = {part, part + D, part + 2 * D, part + 3 * D};
    const int strides[4] = {4 * D, 4 * D, 4 * D, 4 * D};
    finalize_many(s, nblk, D, 1, 4, parts, strides, outs);
  }
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_attention_small_bwd(const void* q, int64_t ldq, int64_t q_bstride, const void* k, int64_t ldk,
                                        int64_t k_bstride, const void* v, int64_t ldv, const void* dout, int64_t ldo,
                                        int64_t o_bstride, void* dq, int64_t lddq, int64_t dq_bstride, void* dk,
                                        void* dv, int64_t lddkv, int64_t dkv_bstride, int dtype, int batch, int heads,
                                        int nq, int nk, int D, float scale, void* stream) {
  if (batch <= 0 || heads <= 0 || nq <= 0 || nk <= 0 || D <= 0) return VGGT_ERR_SHAPE;
  if (dtype != VGGT_DTYPE_F32 && dtype != VGGT_DTYPE_BF16) return VGGT_ERR_UNSUPPORTED;
  if (D % 2) return VGGT_ERR_SHAPE;
  const int esz = dtype == VGGT_DTYPE_BF16 ? 2 : 4;
  // two adjacent output columns per store: 4-B (bf16x2) / 4-B-aligned f32 pairs
  if ((lddq | lddkv) % 2 || ((uintptr_t)dq | (uintptr_t)dk | (uintptr_t)dv) % (2 * esz > 4 ? 4 : 2 * esz))
    return VGGT_ERR_ALIGN;
  const size_t lds = ((size_t)2 * nq * (D + 1) + (size_t)2 * nk * (D + 1) + (size_t)2 * nq * nk) * sizeof(float);
  if (lds > 64 * 1024) return VGGT_ERR_SHAPE;
  // 16-B operand reads when every row start of every operand is 16-B aligned
  const int64_t al = 16 / esz;
  const int vec = D % 8 == 0 && (ldq | ldk | ldv | ldo) % al == 0 &&
                  ((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)dout) % 16 == 0;
  attn_small_bwd_kernel<<<batch * heads, 256, lds, (hipStream_t)stream>>>(
      q, ldq, q_bstride, k, ldk, k_bstride, v, ldv, k_bstride, dout, ldo, o_bstride, dq, lddq, dq_bstride, dk, dv,
      lddkv, dkv_bstride, dtype, heads, nq, nk, D, scale, vec);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_wgrad_f32(const float* dy, int64_t ldy, const float* x, int64_t ldx, int M, int N, int K, float* dw,
                              int64_t ldw, int accumulate, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return VGGT_ERR_SHAPE;
  if (N > 65535) return VGGT_ERR_SHAPE;
  dim3 grid((K + 255) / 256, N);
  wgrad_f32_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(dy, ldy, x, ldx, M, N, K, dw, ldw, accumulate, nullptr);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_wgrad_bias_f32(const float* dy, int64_t ldy, const float* x, int64_t ldx, int M, int N, int K,
                                   float* dw, int64_t ldw, float* db, int accumulate, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || !db) return VGGT_ERR_SHAPE;
  if (N > 65535) return VGGT_ERR_SHAPE;
  dim3 grid((K + 1 + 255) / 256, N);
  wgrad_f32_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(dy, ldy, x, ldx, M, N, K, dw, ldw, accumulate, db);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" size_t vggt_batch_dot_workspace_bytes(int B, int64_t n) { return (size_t)256 * (B > 0 ? B : 1) * sizeof(float); }

extern "C" int vggt_batch_dot_f32(const float* a, const float* c, int64_t bs, int B, int64_t n, float* out, void* ws,
                                  size_t ws_bytes, void* stream) {
  if (B <= 0 || n <= 0) return VGGT_ERR_SHAPE;
  if (!ws || ws_bytes < vggt_batch_dot_workspace_bytes(B, n)) return VGGT_ERR_SHAPE;
  int64_t nc = (n + 65535) / 65536;
  if (nc > 256) nc = 256;
  const int64_t per = (n + nc - 1) / nc;
  hipStream_t s = (hipStream_t)stream;
  batch_dot_kernel<<<dim3((unsigned)nc, B), 256, 0, s>>>(a, c, bs, B, n, per, (float*)ws);
  finalize_kernel<<<(B + 15) / 16, 256, 0, s>>>((const float*)ws, (int)nc, B, B, out, 0);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" size_t vggt_wgrad_bf16_workspace_bytes(int M, int N, int K) {
  const int tiles = (N / 128) * (K / 128);
  int splits = tiles >= 1024 ? 1 : (1024 + tiles - 1) / (tiles > 0 ? tiles : 1);
  const int maxs = (M + 255) / 256;
  if (splits > maxs) splits = maxs;
  if (splits > 16) splits = 16;
  if (splits < 1) splits = 1;
  return (size_t)splits * N * K * sizeof(float);
}

extern "C" int vggt_wgrad_bf16(const void* dy, int64_t ldy, const void* x, int64_t ldx, int M, int N, int K, float* dw,
                               int64_t ldw, int accumulate, void* ws, size_t ws_bytes, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || N % 128 || K % 128) return VGGT_ERR_SHAPE;
  if ((ldy | ldx) % 8 || ((uintptr_t)dy | (uintptr_t)x) % 16) return VGGT_ERR_ALIGN;
  const size_t need = vggt_wgrad_bf16_workspace_bytes(M, N, K);
  if (!ws || ws_bytes < need) return VGGT_ERR_SHAPE;
  const int splits = (int)(need / ((size_t)N * K * sizeof(float)));
  int mchunk = (M + splits - 1) / splits;
  mchunk = (mchunk + 31) / 32 * 32;
  const int nz = (M + mchunk - 1) / mchunk;
  hipStream_t s = (hipStream_t)stream;
  // VGGT_WGRAD_DMA=0: the register-staged form (A/B)
  static const bool use_dma = [] {
    const char* e = getenv("VGGT_WGRAD_DMA");
    return !(e && atoi(e) == 0);
  }();
  // LDS-DMA form: 32-bit descriptor ranges over one split
  if (use_dma && (int64_t)mchunk * (ldy > ldx ? ldy : ldx) * 2 < (1ll << 31)) {
    static bool attr = [] {
      (void)hipFuncSetAttribute((const void*)wgrad_dma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                WG_NSLOT * WG_SLOT);
      return true;
    }();
    (void)attr;
    wgrad_dma_kernel<<<dim3((N / 128) * (K / 128), nz), 256, WG_NSLOT * WG_SLOT, s>>>(
        (const bf16_t*)dy, ldy, (const bf16_t*)x, ldx, M, N, K, mchunk, (float*)ws);
  } else {
    wgrad_bf16_kernel<<<dim3((N / 128) * (K / 128), nz), 256, 0, s>>>((const bf16_t*)dy, ldy, (const bf16_t*)x, ldx,
                                                                      M, N, K, mchunk, (float*)ws);
  }
  const int64_t nk = (int64_t)N * K;
  wgrad_reduce_kernel<<<(unsigned)((nk + 255) / 256), 256, 0, s>>>((const float*)ws, nz, nk, dw, ldw, K, accumulate, 1);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}
