// Latency-bound pieces of the per-chunk path: skinny fp32 linear layers
// (camera head trunk, alignment decoder, gated memory update), small-window
// attention (temporal cross attention with S queries x T keys, decoder and
// camera-head attention over <= 128 tokens), fp32 QK-norm + RoPE, casts and
// row-remapped LayerNorm.  See include/vggt_mi355x.h for the contracts.
#include <math.h>
#include <stdlib.h>

#include "common.h"
#include "tune.h"

namespace {

// ------------------------------------------------------------------------
// Skinny fp32 GEMM: out[M,N] = epi(act(A)[M,K] . W[N,K]^T + bias); each
// block owns a 64-row slab (blockIdx.y) and 64 columns (blockIdx.x).
// 4 waves per block, each wave owns 16 output columns; K is consumed 16 at a
// time: every lane loads one float4 of W (row n, k-quad) and of A, and the
// four v_mfma_f32_16x16x4_f32 of the chunk each take one component (the k
// order inside a chunk is permuted identically on both operands).
// Exact f32 products/accumulation (the reference heads run with autocast
// disabled: featureAligned_vggt.py:104, alignment_head.py:340).
typedef __attribute__((ext_vector_type(4))) float f4;

// One wave's share of the skinny fp32 GEMM: acc[mt] (rows 16mt + 4q + i, column
// n0 + (lane & 15)) += act(A)[rows, kbeg:kend) . W[col, kbeg:kend)^T.  A rows past M
// read row M-1 (never stored); columns past N read column N-1 (never stored).
template <int ACT_IN, int MT = 4>
__device__ __forceinline__ void wave_linear_f32(const float* __restrict__ A, int64_t lda,
                                                const float* __restrict__ W, int64_t ldw, int M, int N, int K,
                                                int n0, int kbeg, int kend, int lane, f32x4 (&acc)[MT]) {
  const int r = lane & 15, q = lane >> 4;
  const int nrow = min(n0 + r, N - 1);
  const int mt_n = min(MT, (M + 15) / 16);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0, 0, 0, 0};
  const bool vec = ((K & 3) == 0) && ((lda & 3) == 0) && ((ldw & 3) == 0);
  int k0 = kbeg;
  if (vec) {
    // Steady state, 64 k per iteration with no per-element guards: all of an
    // iteration's W and A float4 loads are issued before its MFMAs (4 + 4 x mt_n
    // loads in flight per lane instead of one round trip per 16 k -- the loop is
    // latency-bound at skinny M).  A rows past M read row M-1: their products
    // only reach output rows that are never stored.  The MFMA order per
    // accumulator is the 16-k loop's, so the sums are bitwise those of the tail
    // form below.
    const int kv_end = kbeg + ((kend - kbeg) / 64) * 64;
    const float* wp = W + (int64_t)nrow * ldw + 4 * q;
    const float* ap[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) ap[mt] = A + (int64_t)min(mt * 16 + r, M - 1) * lda + 4 * q;
    for (; k0 < kv_end; k0 += 64) {
      f4 wv[4], av[MT][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) wv[u] = *(const f4*)(wp + k0 + 16 * u);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if (mt < mt_n) {
#pragma unroll
          for (int u = 0; u < 4; ++u) av[mt][u] = *(const f4*)(ap[mt] + k0 + 16 * u);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          if (mt >= mt_n) break;
          f4 a4 = av[mt][u];
          if constexpr (ACT_IN == 1) {
#pragma unroll
            for (int j = 0; j < 4; ++j) a4[j] = a4[j] / (1.f + expf(-a4[j]));
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[j], wv[u][j], acc[mt], 0, 0, 0);
        }
    }
  }
  for (; k0 < kend; k0 += 16) {
    const int kk = k0 + 4 * q;
    f4 wv;
    if (vec && kk + 3 < kend) {
      wv = *(const f4*)(W + (int64_t)nrow * ldw + kk);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) wv[j] = (kk + j < kend) ? W[(int64_t)nrow * ldw + kk + j] : 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      if (mt >= mt_n) break;
      const int m = mt * 16 + r;
      f4 av = f4{0, 0, 0, 0};
      if (m < M) {
        if (vec && kk + 3 < kend) {
          av = *(const f4*)(A + (int64_t)m * lda + kk);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) av[j] = (kk + j < kend) ? A[(int64_t)m * lda + kk + j] : 0.f;
        }
        if constexpr (ACT_IN == 1) {  // SiLU on the input (poseLN_modulation = Sequential(SiLU, Linear))
#pragma unroll
          for (int j = 0; j < 4; ++j) av[j] = av[j] / (1.f + expf(-av[j]));
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], wv[j], acc[mt], 0, 0, 0);
    }
  }
}

template <int ACT_IN, int EPI>
__global__ __launch_bounds__(256) void linear_f32_kernel(const float* __restrict__ A, int64_t lda,
                                                         const float* __restrict__ W, int64_t ldw,
                                                         const float* __restrict__ bias, int M, int N, int K,
                                                         float* out, int64_t ldo, const float* __restrict__ gamma,
                                                         int kchunk, float* __restrict__ part, unsigned* cnt) {
  // split-K (part != NULL): block z covers K range [z*kchunk, (z+1)*kchunk) and
  // stores its raw partial sums to part[z][M][N].  With `cnt` (one zeroed word
  // per 64 x 64 output tile) the LAST of the tile's split blocks to finish sums
  // the partials in split order, applies bias and the epilogue and re-zeroes the
  // word -- one launch, the same bits as linear_f32_reduce (the two-launch form
  // used without `cnt`).
  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * 4 + wave) * 16;
  // a wave past N computes clamped garbage it never stores (no early exit: with
  // `cnt` every wave takes part in the tile's last-block protocol)
  const bool active = n0 < N;
  if (!active && !cnt) return;
  const int Mfull = M;
  const int mbase = blockIdx.y * 64;
  A += (int64_t)mbase * lda;
  out += (int64_t)mbase * ldo;
  M = min(M - mbase, 64);
  const int r = lane & 15, q = lane >> 4;
  const int mt_n = (M + 15) / 16;
  f32x4 acc[4];
  wave_linear_f32<ACT_IN>(A, lda, W, ldw, M, N, K, n0, kbeg, kend, lane, acc);
  // C[m = 16mt + 4q + i][n = n0 + r]
  const int n = n0 + r;
  if (part) {
    if (active && n < N) {
      float* pp = part + ((int64_t)blockIdx.z * gridDim.y * 64 + mbase) * N + n;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        if (mt >= mt_n) break;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = mt * 16 + 4 * q + i;
          if (m < M) pp[(int64_t)m * N] = acc[mt][i];
        }
      }
    }
    if (!cnt) return;
    // this block's partials visible device-wide (every XCD's L2) before its ticket
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    __shared__ unsigned last;
    unsigned* word = cnt + blockIdx.y * gridDim.x + blockIdx.x;
    if (threadIdx.x == 0)
      last = __hip_atomic_fetch_add(word, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.z - 1;
    __syncthreads();
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int64_t mstride = (int64_t)gridDim.y * 64 * N;
    const int c0 = blockIdx.x * 64;
    for (int e = threadIdx.x; e < 64 * 64; e += 256) {
      const int m = e >> 6, nn = c0 + (e & 63);
      if (m >= M || nn >= N) continue;
      const int64_t off = (int64_t)(mbase + m) * N + nn;
      float v = 0.f;
      for (int z = 0; z < (int)gridDim.z; ++z) v += part[z * mstride + off];
      v += bias ? bias[nn] : 0.f;
      float* op = out + (int64_t)m * ldo + nn;
      if constexpr (EPI == VGGT_EPI_GELU_BF16) v = gelu_erf(v);
      if constexpr (EPI == VGGT_EPI_RESID_F32) v = *op + gamma[nn] * v;
      *op = v;
    }
    if (threadIdx.x == 0) __hip_atomic_store(word, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    (void)Mfull;
    return;
  }
  if (n >= N) return;
  const float bv = bias ? bias[n] : 0.f;
  const float g = (EPI == VGGT_EPI_RESID_F32) ? gamma[n] : 0.f;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    if (mt >= mt_n) break;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mt * 16 + 4 * q + i;
      if (m >= M) continue;
      float v = acc[mt][i] + bv;
      float* op = out + (int64_t)m * ldo + n;
      if constexpr (EPI == VGGT_EPI_GELU_BF16) v = gelu_erf(v);  // GELU, f32 out
      if constexpr (EPI == VGGT_EPI_RESID_F32) v = *op + g * v;
      *op = v;
    }
  }
}

// Skinny fp32 GEMM (M <= 256), split along K INSIDE the workgroup: KW waves
// own the same 16 output columns (blockIdx.x) of a 64-row slab (blockIdx.y) and consecutive k ranges of
// kchunk (a multiple of 64); their accumulators are summed through LDS in wave
// order by wave 0, which applies bias and the epilogue.  No partial slabs, no
// device-scope fences or counters (vggt_linear_f32_ws picks it for the
// decoder / camera-trunk shapes; fixed summation order: bitwise run to run).
template <int KW, int MT, int ACT_IN, int EPI>
__global__ __launch_bounds__(64 * KW) void linear_f32_wk_kernel(const float* __restrict__ A, int64_t lda,
                                                                const float* __restrict__ W, int64_t ldw,
                                                                const float* __restrict__ bias, int M, int N, int K,
                                                                float* out, int64_t ldo,
                                                                const float* __restrict__ gamma, int kchunk,
                                                                int64_t a_gs, int64_t w_gs, int64_t b_gs,
                                                                int64_t o_gs) {
  __shared__ f32x4 red[KW - 1][MT][64];
  // blockIdx.z: a group of independent linears with the same shape (grouped form)
  A += (int64_t)blockIdx.z * a_gs + (int64_t)blockIdx.y * 64 * lda;
  W += (int64_t)blockIdx.z * w_gs;
  if (bias) bias += (int64_t)blockIdx.z * b_gs;
  out += (int64_t)blockIdx.z * o_gs + (int64_t)blockIdx.y * 64 * ldo;
  M = min(M - (int)blockIdx.y * 64, 64);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16;
  const int kbeg = min(K, wave * kchunk);
  const int kend = min(K, kbeg + kchunk);
  const int mt_n = (M + 15) / 16;
  f32x4 acc[MT];
  wave_linear_f32<ACT_IN, MT>(A, lda, W, ldw, M, N, K, n0, kbeg, kend, lane, acc);
  if (wave > 0) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      if (mt < mt_n) red[wave - 1][mt][lane] = acc[mt];
  }
  __syncthreads();
  if (wave > 0) return;
#pragma unroll
  for (int w = 0; w < KW - 1; ++w)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      if (mt < mt_n) acc[mt] += red[w][mt][lane];
  const int r = lane & 15, q = lane >> 4;
  const int n = n0 + r;
  if (n >= N) return;
  const float bv = bias ? bias[n] : 0.f;
  const float g = (EPI == VGGT_EPI_RESID_F32) ? gamma[n] : 0.f;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    if (mt >= mt_n) break;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mt * 16 + 4 * q + i;
      if (m >= M) continue;
      float v = acc[mt][i] + bv;
      float* op = out + (int64_t)m * ldo + n;
      if constexpr (EPI == VGGT_EPI_GELU_BF16) v = gelu_erf(v);
      if constexpr (EPI == VGGT_EPI_RESID_F32) v = *op + g * v;
      *op = v;
    }
  }
}

template <int KW, int MT, int ACT_IN>
void launch_linear_wk(const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias, int M, int N, int K,
                      int epi, float* out, int64_t ldo, const float* gamma, hipStream_t s, int groups = 1,
                      int64_t a_gs = 0, int64_t w_gs = 0, int64_t b_gs = 0, int64_t o_gs = 0) {
  // k ranges of whole 64-k steps (the vector loop), the last wave takes the rest
  const int kchunk = ((K + KW - 1) / KW + 63) / 64 * 64;
  const dim3 grid((N + 15) / 16, (M + 63) / 64, groups);
  if (epi == VGGT_EPI_F32)
    linear_f32_wk_kernel<KW, MT, ACT_IN, VGGT_EPI_F32><<<grid, 64 * KW, 0, s>>>(A, lda, W, ldw, bias, M, N, K, out, ldo, gamma, kchunk, a_gs, w_gs, b_gs, o_gs);
  else if (epi == VGGT_EPI_GELU_BF16)
    linear_f32_wk_kernel<KW, MT, ACT_IN, VGGT_EPI_GELU_BF16><<<grid, 64 * KW, 0, s>>>(A, lda, W, ldw, bias, M, N, K, out, ldo, gamma, kchunk, a_gs, w_gs, b_gs, o_gs);
  else
    linear_f32_wk_kernel<KW, MT, ACT_IN, VGGT_EPI_RESID_F32><<<grid, 64 * KW, 0, s>>>(A, lda, W, ldw, bias, M, N, K, out, ldo, gamma, kchunk, a_gs, w_gs, b_gs, o_gs);
}

// The in-workgroup split: each wave keeps ~g_vggt_linear_wk k (2..8 waves).  The
// wave count depends on K only, so a row's result does not depend on M (a
// grouped encode of three chunks gives each chunk's rows the bits of its own
// encode); 64-row slabs along blockIdx.y, groups along blockIdx.z.
void linear_wk_dispatch(const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias, int M, int N,
                        int K, int act_in, int epi, float* out, int64_t ldo, const float* gamma, hipStream_t s,
                        int groups, int64_t a_gs, int64_t w_gs, int64_t b_gs, int64_t o_gs) {
  const int mt = M <= 16 ? 1 : 4;
  const int wk = g_vggt_linear_wk > 0 ? g_vggt_linear_wk : 64;
  int kw = 2;
  while (kw < 8 && K > kw * wk) kw *= 2;
#define WK(KW_, MT_)                                                                                          \
  (act_in ? launch_linear_wk<KW_, MT_, 1>(A, lda, W, ldw, bias, M, N, K, epi, out, ldo, gamma, s, groups, a_gs, \
                                          w_gs, b_gs, o_gs)                                                     \
          : launch_linear_wk<KW_, MT_, 0>(A, lda, W, ldw, bias, M, N, K, epi, out, ldo, gamma, s, groups, a_gs, \
                                          w_gs, b_gs, o_gs))
  if (mt == 1) {
    if (kw == 2) WK(2, 1);
    else if (kw == 4) WK(4, 1);
    else WK(8, 1);
  } else {
    if (kw == 2) WK(2, 4);
    else if (kw == 4) WK(4, 4);
    else WK(8, 4);
  }
#undef WK
}

// ------------------------------------------------------------------------
// GatedUpdate (gated_update.py:43-79) around its grouped linears: one wave per
// (batch, memory token) row, D <= 1024 features, fp32 throughout.
// prep: scale = |update_b|, inp[b, i] = [update_b, scale * memory[b, i], scale * mean_j memory[b, j]]
// and the gate MLP's second input half, scale * memory[b, i], into g_in[:, D:2D].
__global__ __launch_bounds__(256) void gated_update_prep_kernel(const float* __restrict__ memory,
                                                                const float* __restrict__ update, int Nt, int D,
                                                                float* __restrict__ inp, float* __restrict__ g_in) {
  __shared__ float part[4];
  const int row = blockIdx.x, b = row / Nt, tid = threadIdx.x;
  const float* u = update + (int64_t)b * D;
  const float* mb = memory + (int64_t)b * Nt * D;
  const float* mi = memory + (int64_t)row * D;
  float ss = 0.f;
  for (int e = tid; e < D; e += 256) ss += u[e] * u[e];
  ss = wave_sum(ss);
  if ((tid & 63) == 0) part[tid >> 6] = ss;
  __syncthreads();
  const float scale = sqrtf((part[0] + part[1]) + (part[2] + part[3]));
  float* o = inp + (int64_t)row * 3 * D;
  float* g = g_in + (int64_t)row * 2 * D;
  for (int e = tid; e < D; e += 256) {
    float mean = 0.f;
    for (int j = 0; j < Nt; ++j) mean += mb[(int64_t)j * D + e];
    mean = mean / (float)Nt;
    const float ms = mi[e] * scale;
    o[e] = u[e];
    o[D + e] = ms;
    o[2 * D + e] = mean * scale;
    g[D + e] = ms;
  }
}

// gate input first half: diff = deltas - memory into g_in[:, 0:D]
__global__ __launch_bounds__(64) void gated_update_diff_kernel(const float* __restrict__ memory,
                                                               const float* __restrict__ deltas, int D,
                                                               float* __restrict__ g_in) {
  const int row = blockIdx.x, lane = threadIdx.x;
  for (int e = lane; e < D; e += 64)
    g_in[(int64_t)row * 2 * D + e] = deltas[(int64_t)row * D + e] - memory[(int64_t)row * D + e];
}

// out = normalize(memory + sigmoid(logit) * normalize(diff - (diff . memory) memory)),
// F.normalize's max(|x|, 1e-12)
__global__ __launch_bounds__(64) void gated_update_tail_kernel(const float* __restrict__ memory,
                                                               const float* __restrict__ deltas,
                                                               const float* __restrict__ logit, int D,
                                                               float* __restrict__ out) {
  const int row = blockIdx.x, lane = threadIdx.x;
  const float* m = memory + (int64_t)row * D;
  const float* dl = deltas + (int64_t)row * D;
  float dot = 0.f;
  for (int e = lane; e < D; e += 64) dot += (dl[e] - m[e]) * m[e];
  dot = wave_sum(dot);
  float nn = 0.f;
  for (int e = lane; e < D; e += 64) {
    const float o = (dl[e] - m[e]) - dot * m[e];
    nn += o * o;
  }
  const float inv1 = 1.f / fmaxf(sqrtf(wave_sum(nn)), 1e-12f);
  const float g = 1.f / (1.f + expf(-logit[row]));
  float n2 = 0.f;
  for (int e = lane; e < D; e += 64) {
    const float v = m[e] + g * (((dl[e] - m[e]) - dot * m[e]) * inv1);
    n2 += v * v;
  }
  const float inv2 = 1.f / fmaxf(sqrtf(wave_sum(n2)), 1e-12f);
  for (int e = lane; e < D; e += 64) {
    const float v = m[e] + g * (((dl[e] - m[e]) - dot * m[e]) * inv1);
    out[(int64_t)row * D + e] = v * inv2;
  }
}

// split-K combine: out = epi(sum_z part[z] + bias), fixed summation order
template <int EPI>
__global__ __launch_bounds__(256) void linear_f32_reduce(const float* __restrict__ part, int splits, int64_t mstride,
                                                         int M, int N, const float* __restrict__ bias, float* out,
                                                         int64_t ldo, const float* __restrict__ gamma) {
  const int64_t total = (int64_t)M * N;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(e / N), n = (int)(e % N);
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += part[z * mstride + e];
    v += bias ? bias[n] : 0.f;
    float* op = out + (int64_t)m * ldo + n;
    if constexpr (EPI == VGGT_EPI_GELU_BF16) v = gelu_erf(v);
    if constexpr (EPI == VGGT_EPI_RESID_F32) v = *op + gamma[n] * v;
    *op = v;
  }
}

// ------------------------------------------------------------------------
// Small-window attention: one wave per (group, head); K/V of the group in
// LDS as f32; keys spread over lanes (<= 2 per lane, nk <= 128), each query
// row's scores reduced with wave shuffles; output d spread over lanes.
template <typename T>
__device__ __forceinline__ float ld1(const T* p) {
  if constexpr (sizeof(T) == 2) return bf2f(*(const bf16_t*)p);
  else return *(const float*)p;
}
template <typename T>
__device__ __forceinline__ void st1(T* p, float v) {
  if constexpr (sizeof(T) == 2) *(bf16_t*)p = f2bf(v);
  else *(float*)p = v;
}

template <typename T>
__global__ __launch_bounds__(64) void attn_small_kernel(const T* __restrict__ q, int64_t ldq, int64_t qbs,
                                                        const T* __restrict__ k, int64_t ldk, int64_t kbs,
                                                        const T* __restrict__ v, int64_t ldv, T* __restrict__ o,
                                                        int64_t ldo, int64_t obs, int heads, int nq, int nk, int D,
                                                        float scale) {
  extern __shared__ float sm[];  // Ks[nk][D+1], Vs[nk][D+1], Qr[D]
  const int lane = threadIdx.x;
  const int g = blockIdx.x / heads, h = blockIdx.x % heads;
  const int DP = D + 1;
  float* Ks = sm;
  float* Vs = Ks + nk * DP;
  float* Qr = Vs + nk * DP;
  const T* kp = k + (int64_t)g * kbs * ldk + h * D;
  const T* vp = v + (int64_t)g * kbs * ldv + h * D;
  for (int i = lane; i < nk * D; i += 64) {
    const int j = i / D, d = i % D;
    Ks[j * DP + d] = ld1(kp + (int64_t)j * ldk + d);
    Vs[j * DP + d] = ld1(vp + (int64_t)j * ldv + d);
  }
  __syncthreads();
  for (int qi = 0; qi < nq; ++qi) {
    const T* qp = q + ((int64_t)g * qbs + qi) * ldq + h * D;
    for (int d = lane; d < D; d += 64) Qr[d] = ld1(qp + d);
    __syncthreads();
    float s0 = -INFINITY, s1 = -INFINITY;
    if (lane < nk) {
      float a = 0.f;
      for (int d = 0; d < D; ++d) a = fmaf(Qr[d], Ks[lane * DP + d], a);
      s0 = a * scale;
    }
    if (lane + 64 < nk) {
      float a = 0.f;
      for (int d = 0; d < D; ++d) a = fmaf(Qr[d], Ks[(lane + 64) * DP + d], a);
      s1 = a * scale;
    }
    const float m = wave_max(fmaxf(s0, s1));
    const float p0 = lane < nk ? expf(s0 - m) : 0.f;
    const float p1 = lane + 64 < nk ? expf(s1 - m) : 0.f;
    const float inv = 1.f / wave_sum(p0 + p1);
    T* op = o + ((int64_t)g * obs + qi) * ldo + h * D;
    for (int d0 = 0; d0 < D; d0 += 64) {
      const int d = d0 + lane;
      float acc = 0.f;
      for (int j = 0; j < nk; ++j) {
        const float pj = __shfl(j < 64 ? p0 : p1, j & 63, 64);
        if (d < D) acc = fmaf(pj, Vs[j * DP + d], acc);
      }
      if (d < D) st1(op + d, acc * inv);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------
// Small-window attention, workgroup form: one 256-thread workgroup per
// (group, head) with Q, K, V of the group staged once in LDS (fp32); the
// nq x nk scores, the row softmaxes and the nq x D outputs are spread over
// all 256 threads (a thread per score, per row, per output element), so no
// query waits for another.  Same fp32 arithmetic and summation order as the
// one-wave form above (serial over d for a score, over keys for an output).
// Used when the group fits 64 KiB of LDS (temporal attention: 16 x <= 16
// keys x 128; decoder / camera-head blocks).
template <typename T>
__global__ __launch_bounds__(256) void attn_small_wg_kernel(const T* __restrict__ q, int64_t ldq, int64_t qbs,
                                                            const T* __restrict__ k, int64_t ldk, int64_t kbs,
                                                            const T* __restrict__ v, int64_t ldv, T* __restrict__ o,
                                                            int64_t ldo, int64_t obs, int heads, int nq, int nk, int D,
                                                            float scale) {
  extern __shared__ float sm[];
  const int DP = D + 1;
  float* Qs = sm;              // [nq][D+1]
  float* Ks = Qs + nq * DP;    // [nk][D+1]
  float* Vs = Ks + nk * DP;    // [nk][D]
  float* Ps = Vs + nk * D;     // [nq][nk]
  const int tid = threadIdx.x;
  const int g = blockIdx.x / heads, h = blockIdx.x % heads;
  const T* qp = q + (int64_t)g * qbs * ldq + h * D;
  const T* kp = k + (int64_t)g * kbs * ldk + h * D;
  const T* vp = v + (int64_t)g * kbs * ldv + h * D;
  for (int i = tid; i < nq * D; i += 256) {
    const int r = i / D, d = i % D;
    Qs[r * DP + d] = ld1(qp + (int64_t)r * ldq + d);
  }
  for (int i = tid; i < nk * D; i += 256) {
    const int r = i / D, d = i % D;
    Ks[r * DP + d] = ld1(kp + (int64_t)r * ldk + d);
    Vs[r * D + d] = ld1(vp + (int64_t)r * ldv + d);
  }
  __syncthreads();
  for (int p = tid; p < nq * nk; p += 256) {
    const int i = p / nk, j = p % nk;
    const float* qr = Qs + i * DP;
    const float* kr = Ks + j * DP;
    float a = 0.f;
    for (int d = 0; d < D; ++d) a = fmaf(qr[d], kr[d], a);
    Ps[p] = a * scale;
  }
  __syncthreads();
  for (int i = tid; i < nq; i += 256) {
    float* pr = Ps + i * nk;
    float m = -INFINITY;
    for (int j = 0; j < nk; ++j) m = fmaxf(m, pr[j]);
    float l = 0.f;
    for (int j = 0; j < nk; ++j) {
      const float e = expf(pr[j] - m);
      pr[j] = e;
      l += e;
    }
    const float inv = 1.f / l;
    for (int j = 0; j < nk; ++j) pr[j] *= inv;
  }
  __syncthreads();
  T* op = o + (int64_t)g * obs * ldo + h * D;
  for (int p = tid; p < nq * D; p += 256) {
    const int i = p / D, d = p % D;
    const float* pr = Ps + i * nk;
    float acc = 0.f;
    for (int j = 0; j < nk; ++j) acc = fmaf(pr[j], Vs[j * D + d], acc);
    st1(op + (int64_t)i * ldo + d, acc);
  }
}

// ------------------------------------------------------------------------
// Small-window bf16 attention on the matrix cores (nq <= 16 queries, nk <= 16
// keys, D % 16 == 0: the alignment head's temporal cross attention, 16 frames
// against the 5 overlap frames, per patch token and head).  One wave per
// (group, head), four per workgroup.  S^T = K Q^T with
// v_mfma_f32_16x16x16_bf16 (lane l: keys 4(l>>4)..+3 of query l&15 in its
// accumulator), the softmax over keys across the 4 lane groups (two xor
// shuffles), then O^T = V^T P^T: the lane's own P values (rounded to bf16, as
// the reference's bf16 SDPA does) are already the B operand, and its
// accumulator holds 4 consecutive features of its query -- one 8-byte store per
// 16 features.
typedef __attribute__((ext_vector_type(4))) short s16x4;
// DT: D as a compile-time constant (64 / 128: every load of the wave issued before
// its first MFMA), 0: runtime D
template <int DT>
__global__ __launch_bounds__(256) void attn_small_mfma_kernel(const bf16_t* __restrict__ q, int64_t ldq, int64_t qbs,
                                                              const bf16_t* __restrict__ k, int64_t ldk, int64_t kbs,
                                                              const bf16_t* __restrict__ v, int64_t ldv,
                                                              bf16_t* __restrict__ o, int64_t ldo, int64_t obs,
                                                              int pairs, int heads, int nq, int nk, int D_, float scale) {
  const int D = DT ? DT : D_;
  const int lane = threadIdx.x & 63;
  const int pair = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pair >= pairs) return;
  const int g = pair / heads, h = pair % heads;
  const int r = lane & 15, grp = lane >> 4;
  const bf16_t* qp = q + (int64_t)g * qbs * ldq + h * D;
  const bf16_t* kp = k + (int64_t)g * kbs * ldk + h * D;
  const bf16_t* vp = v + (int64_t)g * kbs * ldv + h * D;
  // S^T[key][query]: A = K rows (key r), B = Q^T (query r); k-slice 4 grp .. +3 of each 16
  f32x4 st = f32x4{0, 0, 0, 0};
  const bool krow = r < nk, qrow = r < nq;
  if constexpr (DT > 0) {
    s16x4 ka[DT / 16], qb[DT / 16];
#pragma unroll
    for (int t = 0; t < DT / 16; ++t) {
      ka[t] = krow ? *(const s16x4*)(kp + (int64_t)r * ldk + 16 * t + 4 * grp) : s16x4{0, 0, 0, 0};
      qb[t] = qrow ? *(const s16x4*)(qp + (int64_t)r * ldq + 16 * t + 4 * grp) : s16x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int t = 0; t < DT / 16; ++t) st = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ka[t], qb[t], st, 0, 0, 0);
  } else {
    for (int d0 = 0; d0 < D; d0 += 16) {
      s16x4 ka = s16x4{0, 0, 0, 0}, qb = s16x4{0, 0, 0, 0};
      if (krow) ka = *(const s16x4*)(kp + (int64_t)r * ldk + d0 + 4 * grp);
      if (qrow) qb = *(const s16x4*)(qp + (int64_t)r * ldq + d0 + 4 * grp);
      st = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ka, qb, st, 0, 0, 0);
    }
  }
  // softmax over the keys 4 grp + i of query r (keys >= nk masked)
  float p[4];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    p[i] = (4 * grp + i < nk) ? st[i] * scale : -INFINITY;
    m = fmaxf(m, p[i]);
  }
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float l = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    p[i] = (4 * grp + i < nk) ? expf(p[i] - m) : 0.f;
    l += p[i];
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float inv = 1.f / l;
  s16x4 pb;
#pragma unroll
  for (int i = 0; i < 4; ++i) pb[i] = (short)f2bf(p[i] * inv);
  // V (nk x D, zero rows up to 16) into this wave's LDS slab with 8-byte loads, then
  // O^T[feature][query] = V^T P^T: A = V^T (feature r of the tile, keys 4 grp .. +3)
  extern __shared__ bf16_t vs_all[];
  bf16_t* vs = vs_all + (threadIdx.x >> 6) * 16 * D;
#pragma unroll 8
  for (int c = lane; c < 16 * (D / 4); c += 64) {
    const int key = c / (D / 4), d = (c % (D / 4)) * 4;
    uint2 u = make_uint2(0u, 0u);
    if (key < nk) u = *(const uint2*)(vp + (int64_t)key * ldv + d);
    *(uint2*)(vs + key * D + d) = u;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slab is this wave's only: no barrier
  bf16_t* op = o + (int64_t)g * obs * ldo + h * D;
#pragma unroll 8
  for (int d0 = 0; d0 < D; d0 += 16) {
    s16x4 va;
#pragma unroll
    for (int j = 0; j < 4; ++j) va[j] = (short)vs[(4 * grp + j) * D + d0 + r];
    const f32x4 ot = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(va, pb, f32x4{0, 0, 0, 0}, 0, 0, 0);
    // lane: query r, features d0 + 4 grp .. +3
    if (qrow) {
      uint2 u;
      u.x = pack_bf2(ot[0], ot[1]);
      u.y = pack_bf2(ot[2], ot[3]);
      *(uint2*)(op + (int64_t)r * ldo + d0 + 4 * grp) = u;
    }
  }
}

// ------------------------------------------------------------------------
// fp32 per-head LayerNorm + RoPE (decoder / camera head run in fp32).
template <int MODE>
__global__ __launch_bounds__(64) void headnorm_rope_f32_kernel(float* __restrict__ buf, int64_t ld, int col_off,
                                                               int H, int D, const float* __restrict__ w,
                                                               const float* __restrict__ b, float eps,
                                                               const int32_t* __restrict__ pos, int period,
                                                               const float* __restrict__ cs,
                                                               const float* __restrict__ sn, int tab_len) {
  extern __shared__ float xs[];
  const int row = blockIdx.x / H, h = blockIdx.x % H;
  const int lane = threadIdx.x;
  float* p = buf + (int64_t)row * ld + col_off + h * D;
  float s = 0.f;
  for (int d = lane; d < D; d += 64) {
    xs[d] = p[d];
    s += xs[d];
  }
  __syncthreads();
  if (w) {
    const float mean = wave_sum(s) / D;
    float qv = 0.f;
    for (int d = lane; d < D; d += 64) {
      const float t = xs[d] - mean;
      qv += t * t;
    }
    const float rstd = rsqrtf(wave_sum(qv) / D + eps);
    __syncthreads();
    for (int d = lane; d < D; d += 64) xs[d] = (xs[d] - mean) * rstd * w[d] + (b ? b[d] : 0.f);
    __syncthreads();
  }
  for (int d = lane; d < D; d += 64) {
    float y = xs[d];
    if constexpr (MODE != VGGT_ROPE_NONE) {
      const int pr = row % period;
      int rd, e, pp;
      if constexpr (MODE == VGGT_ROPE_2D) {
        rd = D / 2;
        e = d % rd;
        pp = pos[2 * pr + (d >= rd ? 1 : 0)];
      } else {
        rd = D;
        e = d;
        pp = pos[pr];
      }
      pp = min(max(pp, 0), tab_len - 1);
      const int base = d - e;
      const float partner = e < rd / 2 ? -xs[base + e + rd / 2] : xs[base + e - rd / 2];
      y = xs[d] * cs[pp * rd + e] + partner * sn[pp * rd + e];
    }
    p[d] = y;
  }
}

// ------------------------------------------------------------------------
// fp32 -> bf16 cast of a row-major [rows, cols] view (cols % 4 == 0).
__global__ __launch_bounds__(256) void cast_kernel(const float* __restrict__ x, int64_t ldx, bf16_t* __restrict__ y,
                                                   int64_t ldy, int rows, int cols) {
  const int c4 = cols / 4;
  const int64_t total = (int64_t)rows * c4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / c4;
    const int c = (int)(i % c4) * 4;
    const f32x4 v = *(const f32x4*)(x + r * ldx + c);
    uint2 u;
    u.x = pack_bf2(v[0], v[1]);
    u.y = pack_bf2(v[2], v[3]);
    *(uint2*)(y + r * ldy + c) = u;
  }
}

inline int grid_for(int64_t total) {
  int64_t g = (total + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" int vggt_linear_f32_ws(const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias, int M,
                                  int N, int K, int act_in, int epi, float* out, int64_t ldo, const float* gamma,
                                  void* ws, size_t ws_bytes, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return VGGT_ERR_SHAPE;
  if (epi == VGGT_EPI_RESID_F32 && !gamma) return VGGT_ERR_SHAPE;
  if ((act_in != 0 && act_in != 1) || (epi != VGGT_EPI_F32 && epi != VGGT_EPI_GELU_BF16 && epi != VGGT_EPI_RESID_F32))
    return VGGT_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  if (M <= 256 && g_vggt_linear_wk > 0) {
    linear_wk_dispatch(A, lda, W, ldw, bias, M, N, K, act_in, epi, out, ldo, gamma, s, 1, 0, 0, 0, 0);
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  const int gy = (M + 63) / 64;
  const int blocks = ((N + 63) / 64) * gy;
  // split K until one block per CU is busy or a split would keep fewer than
  // g_vggt_linear_split_k k (skinny M: camera head, decoder)
  int splits = 1;
  while (splits < VGGT_LINEAR_F32_MAX_SPLITS && blocks * splits * 2 <= 512 && K / (splits * 2) >= g_vggt_linear_split_k)
    splits *= 2;
  const int64_t mstride = (int64_t)gy * 64 * N;
  // ws = [VGGT_LINEAR_F32_WS_COUNTERS zeroed tile words][partials]
  const size_t cbytes = VGGT_LINEAR_F32_WS_COUNTERS * sizeof(unsigned);
  while (splits > 1 && (!ws || ws_bytes < cbytes + (size_t)splits * mstride * sizeof(float))) splits /= 2;
  const int kchunk = splits > 1 ? ((K + splits - 1) / splits + 15) / 16 * 16 : K;
  float* part = splits > 1 ? (float*)((char*)ws + cbytes) : nullptr;
  // one launch (last block per tile combines) while the tile words fit
  unsigned* cnt =
      (splits > 1 && blocks <= VGGT_LINEAR_F32_WS_COUNTERS && g_vggt_linear_one_launch) ? (unsigned*)ws : nullptr;
  const dim3 grid((N + 63) / 64, gy, splits);
#define LAUNCH(AI, E) \
  linear_f32_kernel<AI, E><<<grid, 256, 0, s>>>(A, lda, W, ldw, bias, M, N, K, out, ldo, gamma, kchunk, part, cnt)
  if (act_in == 0) {
    if (epi == VGGT_EPI_F32) LAUNCH(0, VGGT_EPI_F32);
    else if (epi == VGGT_EPI_GELU_BF16) LAUNCH(0, VGGT_EPI_GELU_BF16);
    else LAUNCH(0, VGGT_EPI_RESID_F32);
  } else {
    if (epi == VGGT_EPI_F32) LAUNCH(1, VGGT_EPI_F32);
    else if (epi == VGGT_EPI_GELU_BF16) LAUNCH(1, VGGT_EPI_GELU_BF16);
    else LAUNCH(1, VGGT_EPI_RESID_F32);
  }
#undef LAUNCH
  if (part && !cnt) {
    const int64_t total = (int64_t)M * N;
    const int rg = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    if (epi == VGGT_EPI_F32) linear_f32_reduce<VGGT_EPI_F32><<<rg, 256, 0, s>>>(part, splits, mstride, M, N, bias, out, ldo, gamma);
    else if (epi == VGGT_EPI_GELU_BF16) linear_f32_reduce<VGGT_EPI_GELU_BF16><<<rg, 256, 0, s>>>(part, splits, mstride, M, N, bias, out, ldo, gamma);
    else linear_f32_reduce<VGGT_EPI_RESID_F32><<<rg, 256, 0, s>>>(part, splits, mstride, M, N, bias, out, ldo, gamma);
  }
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_linear_f32_grouped(const float* A, int64_t lda, int64_t a_gstride, const float* W, int64_t ldw,
                                       int64_t w_gstride, const float* bias, int64_t b_gstride, int M, int N, int K,
                                       int groups, int act_in, int epi, float* out, int64_t ldo, int64_t o_gstride,
                                       void* stream) {
  if (M <= 0 || M > 256 || N <= 0 || K <= 0 || groups <= 0 || groups > 65535) return VGGT_ERR_SHAPE;
  if ((act_in != 0 && act_in != 1) || (epi != VGGT_EPI_F32 && epi != VGGT_EPI_GELU_BF16)) return VGGT_ERR_UNSUPPORTED;
  linear_wk_dispatch(A, lda, W, ldw, bias, M, N, K, act_in, epi, out, ldo, nullptr, (hipStream_t)stream, groups,
                     a_gstride, w_gstride, b_gstride, o_gstride);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_gated_update_prep(const float* memory, const float* update, int B, int Nt, int D, float* inp,
                                      float* g_in, void* stream) {
  if (B <= 0 || Nt <= 0 || D <= 0) return VGGT_ERR_SHAPE;
  gated_update_prep_kernel<<<B * Nt, 256, 0, (hipStream_t)stream>>>(memory, update, Nt, D, inp, g_in);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_gated_update_diff(const float* memory, const float* deltas, int rows, int D, float* g_in,
                                      void* stream) {
  if (rows <= 0 || D <= 0) return VGGT_ERR_SHAPE;
  gated_update_diff_kernel<<<rows, 64, 0, (hipStream_t)stream>>>(memory, deltas, D, g_in);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_gated_update_tail(const float* memory, const float* deltas, const float* logit, int rows, int D,
                                      float* out, void* stream) {
  if (rows <= 0 || D <= 0) return VGGT_ERR_SHAPE;
  gated_update_tail_kernel<<<rows, 64, 0, (hipStream_t)stream>>>(memory, deltas, logit, D, out);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_linear_f32(const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias, int M,
                               int N, int K, int act_in, int epi, float* out, int64_t ldo, const float* gamma,
                               void* stream) {
  return vggt_linear_f32_ws(A, lda, W, ldw, bias, M, N, K, act_in, epi, out, ldo, gamma, nullptr, 0, stream);
}

extern "C" int vggt_attention_small(const void* q, int64_t ldq, int64_t q_bstride, const void* k, int64_t ldk,
                                    int64_t k_bstride, const void* v, int64_t ldv, void* o, int64_t ldo,
                                    int64_t o_bstride, int dtype, int batch, int heads, int nq, int nk, int D,
                                    float scale, void* stream) {
  if (batch <= 0 || heads <= 0 || nq <= 0 || nk <= 0 || nk > 128 || D <= 0 || D > 256) return VGGT_ERR_SHAPE;
  const size_t lds = (size_t)(2 * nk * (D + 1) + D) * sizeof(float);
  if (lds > 160 * 1024) return VGGT_ERR_SHAPE;
  static bool attr_set = false;  // allow > 64 KiB dynamic LDS (gfx950: 160 KiB per workgroup)
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)attn_small_kernel<float>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)attn_small_kernel<bf16_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    attr_set = true;
  }
  hipStream_t s = (hipStream_t)stream;
  // the matrix-core form for bf16 windows of <= 16 x 16 (VGGT_ATTN_SMALL_MFMA=0: the fp32 LDS form)
  static const int use_mfma = getenv("VGGT_ATTN_SMALL_MFMA") ? atoi(getenv("VGGT_ATTN_SMALL_MFMA")) : 1;
  const bool exact = (dtype & VGGT_ATTN_SMALL_EXACT) != 0;
  dtype &= ~VGGT_ATTN_SMALL_EXACT;
  if (use_mfma && !exact && dtype == VGGT_DTYPE_BF16 && nq <= 16 && nk <= 16 && D % 16 == 0 && D <= 256 &&
      (ldq | ldk | ldv | ldo) % 4 == 0 && (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) & 7) == 0) {
    const int pairs = batch * heads;
    const int nwg = (pairs + 3) / 4;
    const size_t lds_v = 4 * 16 * D * 2;
#define VGGT_SMALL_MFMA(DT_)                                                                                       \
  attn_small_mfma_kernel<DT_><<<nwg, 256, lds_v, s>>>((const bf16_t*)q, ldq, q_bstride, (const bf16_t*)k, ldk,       \
                                                      k_bstride, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, o_bstride, \
                                                      pairs, heads, nq, nk, D, scale)
    if (D == 128) VGGT_SMALL_MFMA(128);
    else if (D == 64) VGGT_SMALL_MFMA(64);
    else VGGT_SMALL_MFMA(0);
#undef VGGT_SMALL_MFMA
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  const int grid = batch * heads;
  const size_t lds_wg = ((size_t)(nq + nk) * (D + 1) + (size_t)nk * D + (size_t)nq * nk) * sizeof(float);
  static const int use_wg = getenv("VGGT_ATTN_SMALL_WG") ? atoi(getenv("VGGT_ATTN_SMALL_WG")) : 1;
  if (use_wg && lds_wg <= 64 * 1024) {
    if (dtype == VGGT_DTYPE_BF16)
      attn_small_wg_kernel<bf16_t><<<grid, 256, lds_wg, s>>>((const bf16_t*)q, ldq, q_bstride, (const bf16_t*)k, ldk,
                                                             k_bstride, (const bf16_t*)v, ldv, (bf16_t*)o, ldo,
                                                             o_bstride, heads, nq, nk, D, scale);
    else if (dtype == VGGT_DTYPE_F32)
      attn_small_wg_kernel<float><<<grid, 256, lds_wg, s>>>((const float*)q, ldq, q_bstride, (const float*)k, ldk,
                                                            k_bstride, (const float*)v, ldv, (float*)o, ldo, o_bstride,
                                                            heads, nq, nk, D, scale);
    else
      return VGGT_ERR_UNSUPPORTED;
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if (dtype == VGGT_DTYPE_BF16)
    attn_small_kernel<bf16_t><<<grid, 64, lds, s>>>((const bf16_t*)q, ldq, q_bstride, (const bf16_t*)k, ldk, k_bstride,
                                                    (const bf16_t*)v, ldv, (bf16_t*)o, ldo, o_bstride, heads, nq, nk,
                                                    D, scale);
  else if (dtype == VGGT_DTYPE_F32)
    attn_small_kernel<float><<<grid, 64, lds, s>>>((const float*)q, ldq, q_bstride, (const float*)k, ldk, k_bstride,
                                                   (const float*)v, ldv, (float*)o, ldo, o_bstride, heads, nq, nk, D,
                                                   scale);
  else
    return VGGT_ERR_UNSUPPORTED;
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_headnorm_rope_f32(float* buf, int64_t ld, int col_off, int M, int H, int D, const float* w,
                                      const float* b, float eps, int rope_mode, const int32_t* pos, int period,
                                      const float* cos_tab, const float* sin_tab, int tab_len, void* stream) {
  if (M <= 0) return M == 0 ? VGGT_OK : VGGT_ERR_SHAPE;
  if (H <= 0 || D <= 0 || D > 1024 || (D % 4)) return VGGT_ERR_SHAPE;
  if (rope_mode != VGGT_ROPE_NONE && (!pos || !cos_tab || !sin_tab || period <= 0 || tab_len <= 0))
    return VGGT_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  const size_t lds = D * sizeof(float);
  const int grid = M * H;
  switch (rope_mode) {
    case VGGT_ROPE_NONE:
      headnorm_rope_f32_kernel<VGGT_ROPE_NONE><<<grid, 64, lds, s>>>(buf, ld, col_off, H, D, w, b, eps, pos, period,
                                                                    cos_tab, sin_tab, tab_len);
      break;
    case VGGT_ROPE_2D:
      headnorm_rope_f32_kernel<VGGT_ROPE_2D><<<grid, 64, lds, s>>>(buf, ld, col_off, H, D, w, b, eps, pos, period,
                                                                  cos_tab, sin_tab, tab_len);
      break;
    case VGGT_ROPE_1D:
      headnorm_rope_f32_kernel<VGGT_ROPE_1D><<<grid, 64, lds, s>>>(buf, ld, col_off, H, D, w, b, eps, pos, period,
                                                                  cos_tab, sin_tab, tab_len);
      break;
    default: return VGGT_ERR_UNSUPPORTED;
  }
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_cast_f32_bf16(const float* x, int64_t ldx, void* y, int64_t ldy, int rows, int cols,
                                  void* stream) {
  if (rows < 0 || cols % 4 || ldx % 4 || ldy % 4) return VGGT_ERR_SHAPE;
  if (((uintptr_t)x % 16) || ((uintptr_t)y % 8)) return VGGT_ERR_ALIGN;
  if (rows == 0) return VGGT_OK;
  cast_kernel<<<grid_for((int64_t)rows * cols / 4), 256, 0, (hipStream_t)stream>>>(x, ldx, (bf16_t*)y, ldy, rows, cols);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}
