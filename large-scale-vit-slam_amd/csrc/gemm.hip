// bf16 MFMA GEMM with fused epilogues for every autocast nn.Linear on the
// VGGT hot path (see include/vggt_mi355x.h: vggt_gemm_bf16).
//
//   out[M,N] = epi( A[M,K] . W[N,K]^T + bias )      A, W: bf16, K-contiguous
//
// Design (gfx950):
//  * 128x128x64 block tile, 4 waves (2x2), each wave a 64x64 sub-tile of
//    4x4 v_mfma_f32_16x16x32_bf16 accumulators (64 acc VGPRs).
//  * Operands staged global->LDS with global_load_lds_dwordx4 (LDS-DMA, no
//    VGPR round trip), double-buffered; the XOR swizzle chunk^(row&7) that
//    makes the ds_read_b128 fragment reads conflict-free is applied on the
//    per-lane SOURCE address (the LDS image of an LDS-DMA is lane-linear).
//  * The MFMA computes C^T (W as the A-operand) so each lane ends with 4
//    consecutive output features of one token: the epilogue packs them into
//    one ds_write_b64, then the tile is re-read from LDS as whole 256-B rows
//    and written with 16-B coalesced stores (fp32 residual read-modify-write
//    likewise), applying bias / GELU / LayerScale+residual there.
//  * XCD-aware bijective block remap so the N-tiles of one M-panel share an L2.
#include <stdlib.h>

#include "common.h"
#include "tune.h"
#include "gelu_lut.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE = BM * BK * 2;        // 16 KiB per operand tile
constexpr int STAGE_BYTES = 2 * TILE;    // A + W
constexpr int CROW = BN * 2 + 16;        // epilogue C-tile row stride (bytes), 16-B aligned

struct Epi {
  const float* bias;
  void* out;
  int64_t ldo;
  const float* gamma;
  float* out2;
  int64_t ldo2;
  // EPI_QKNORM (vggt_gemm_qkv): per-head LayerNorm of the q / k column blocks
  // + RoPE, v block stored as is
  const float *qw, *qb, *kw, *kb;
  float eps;
  int hd;  // H * D: width of each of the q / k / v column blocks
  int rope_mode, period, tab_len;
  const int32_t* pos;
  const float *cs, *sn;
  // leading column blocks that are normalised (+ RoPE): 2 = q and k of a fused
  // qkv row; 1 = the first block only (vggt_gemm_headnorm: a q, or the k of a kv)
  int nreg = 2;
};

constexpr int EPI_QKNORM_D64 = 16, EPI_QKNORM_D128 = 17;  // internal epilogue ids
// GELU that also stores the pre-activation (bf16 Linear output) into out2 for
// the GELU backward (vggt_gemm_bf16_gelu_pre): the persistent form's id
constexpr int EPI_GELU_PRE = 18;

// bf16 GELU of the two bf16 values packed in d, from gelu_lut (global memory)
// or its LDS copy (|x| in [2^-16, 2^6): positive half, then negative half).  Outside
// the table (rare: a wave-uniform branch) the limits of torch's float32
// formula: bf16(0.5 x) below it, x or -0.0 above it (scripts/gen_gelu_lut.py
// checks both rules against torch for every bf16 value).
template <typename TP>
__device__ __forceinline__ uint32_t gelu1_lut(uint32_t b, TP lut) {
  const uint32_t u = b & 0x7fff;
  const uint32_t t = u - (GELU_LUT_E0 << 7);
  if (t < (uint32_t)GELU_LUT_N) return lut[t + ((b >> 15) & 1) * GELU_LUT_N];
  if (u < (GELU_LUT_E0 << 7)) return f2bf(0.5f * bf2f((bf16_t)b));
  return (b & 0x8000) ? 0x8000u : b;
}
template <typename TP>
__device__ __forceinline__ uint32_t gelu2_lut(uint32_t d, TP lut) {
  const uint32_t tlo = (d & 0x7fff) - (GELU_LUT_E0 << 7);
  const uint32_t thi = ((d >> 16) & 0x7fff) - (GELU_LUT_E0 << 7);
  if (__builtin_amdgcn_ballot_w64(max(tlo, thi) >= (uint32_t)GELU_LUT_N) == 0) {
    const uint32_t lo = lut[tlo + ((d >> 15) & 1) * GELU_LUT_N];
    const uint32_t hi = lut[thi + (d >> 31) * GELU_LUT_N];
    return lo | (hi << 16);
  }
  return gelu1_lut(d & 0xffff, lut) | (gelu1_lut(d >> 16, lut) << 16);
}
// Branch-free form for a group of packed pairs: both halves' indices clamped into the
// table (packed u16 ops), so every lookup is issued with no control flow in between;
// `oor` collects whether any half was clamped, and the caller re-does the group with
// gelu2_lut (a wave-uniform branch per group, rare) when a lane saw one.
__device__ __forceinline__ uint32_t gelu2_clamped(uint32_t d, const uint16_t* lut, uint32_t& oor) {
  typedef unsigned short us2 __attribute__((ext_vector_type(2)));
  const us2 m = __builtin_bit_cast(us2, d & 0x7fff7fffu);
  const us2 t = m - (us2)(unsigned short)(GELU_LUT_E0 << 7);                // wraps below the table
  const us2 tc = __builtin_elementwise_min(t, (us2)(unsigned short)(GELU_LUT_N - 1));
  oor |= __builtin_bit_cast(uint32_t, t) ^ __builtin_bit_cast(uint32_t, tc);
  const us2 sg = __builtin_bit_cast(us2, (d >> 15) & 0x00010001u);
  const uint32_t ix = __builtin_bit_cast(uint32_t, (us2)(tc + sg * (us2)(unsigned short)GELU_LUT_N));
  return (uint32_t)lut[ix & 0xffff] | ((uint32_t)lut[ix >> 16] << 16);
}
// the global-memory table (the LDS-staged epilogues of the one-shot forms)
__device__ __forceinline__ uint32_t gelu2_tab(uint32_t d, const uint16_t* lut) { return gelu2_lut(d, lut); }

// ---- epilogue 2 (shared): the bf16 C tile staged in LDS (row stride CROW
// bytes) re-read as whole rows, 16 B (8 features) per thread, and written with
// coalesced stores, applying GELU / LayerScale + fp32 residual there.
template <int EPI, int BM, int BN, int NT, int CROW>
__device__ __forceinline__ void write_tile(const char* Cs, int m0, int n0, int M, const Epi& ep,
                                           const float* tcs = nullptr, const float* tsn = nullptr) {
  constexpr int CPR = BN / 8;        // 16-B chunks per row
  constexpr int RPP = NT / CPR;      // rows per pass (NT % CPR threads idle when BN = 192)
  const int ch = threadIdx.x % CPR;
  const int n = n0 + ch * 8;
  if (threadIdx.x >= RPP * CPR) return;
  float g[8];
  // EPI_QKNORM: this thread's 8 norm weights / biases (fixed column), RoPE
  // tables from LDS when the caller staged them there.  The q / k / v region
  // is per thread: a 192-wide tile can straddle a region boundary (heads and
  // regions are multiples of 64 columns, so a head never does).
  float nwv[8], nbv[8];
  if constexpr (EPI == EPI_QKNORM_D64 || EPI == EPI_QKNORM_D128) {
    constexpr int D = EPI == EPI_QKNORM_D64 ? 64 : 128;
    const int region = n / ep.hd;
    const int e0 = (n % ep.hd) % D;
    const float* nw = region ? ep.kw : ep.qw;
    const float* nb = region ? ep.kb : ep.qb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      nwv[j] = (region < ep.nreg && nw) ? nw[e0 + j] : 1.f;
      nbv[j] = (region < ep.nreg && nb) ? nb[e0 + j] : 0.f;
    }
    if (!tcs) {
      tcs = ep.cs;
      tsn = ep.sn;
    }
  }
  if constexpr (EPI == VGGT_EPI_RESID_F32) {
    const f32x4 g0 = *(const f32x4*)(ep.gamma + n);
    const f32x4 g1 = *(const f32x4*)(ep.gamma + n + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      g[j] = g0[j];
      g[4 + j] = g1[j];
    }
  }
#pragma unroll 2
  for (int ml = threadIdx.x / CPR; ml < BM; ml += RPP) {
    const int m = m0 + ml;
    if (m >= M) continue;
    const uint4 cv = *(const uint4*)(Cs + ml * CROW + ch * 16);
    if constexpr (EPI == VGGT_EPI_BF16) {
      *(uint4*)((bf16_t*)ep.out + (int64_t)m * ep.ldo + n) = cv;
    } else if constexpr (EPI == EPI_QKNORM_D64 || EPI == EPI_QKNORM_D128) {
      // q / k blocks: q_norm / k_norm (fp32 LayerNorm over the head's D bf16
      // linear outputs) then RoPE on the fp32 result, one bf16 rounding at the
      // end -- the arithmetic of headnorm_rope_kernel (norm.hip), in registers.
      constexpr int D = EPI == EPI_QKNORM_D64 ? 64 : 128;
      constexpr int LPH = D / 8;  // lanes per head (consecutive: ch is the low index)
      const int region = n / ep.hd;  // 0 q, 1 k, 2 v
      if (region >= ep.nreg) {
        *(uint4*)((bf16_t*)ep.out + (int64_t)m * ep.ldo + n) = cv;
        continue;
      }
      const uint32_t w4[4] = {cv.x, cv.y, cv.z, cv.w};
      float x[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[2 * j] = bf2f((bf16_t)(w4[j] & 0xffff));
        x[2 * j + 1] = bf2f((bf16_t)(w4[j] >> 16));
      }
      const int e0 = (n % ep.hd) % D;
      if (ep.qw) {
        float sm = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) sm += x[j];
#pragma unroll
        for (int o = 1; o < LPH; o <<= 1) sm += __shfl_xor(sm, o, 64);
        const float mean = sm * (1.f / D);
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = x[j] - mean;
          q += d * d;
        }
#pragma unroll
        for (int o = 1; o < LPH; o <<= 1) q += __shfl_xor(q, o, 64);
        const float rstd = rsqrtf(q * (1.f / D) + ep.eps);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = (x[j] - mean) * rstd * nwv[j] + nbv[j];
      }
      if (ep.rope_mode != VGGT_ROPE_NONE) {
        const bool two_d = ep.rope_mode == VGGT_ROPE_2D;
        const int RD = two_d ? D / 2 : D;  // rotated block
        const int PL = RD / 16;            // partner lane distance (rotate_half: RD/2 elements)
        const int er = e0 % RD;
        const int pr = m % ep.period;
        int pp = two_d ? ep.pos[2 * pr + (e0 >= D / 2 ? 1 : 0)] : ep.pos[pr];
        pp = min(max(pp, 0), ep.tab_len - 1);
        const bool first = er < RD / 2;
        const f32x4* cp = (const f32x4*)(tcs + pp * RD + er);  // 32-B aligned: two 16-B reads each
        const f32x4* sp = (const f32x4*)(tsn + pp * RD + er);
        const f32x4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
        const float cv[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
        const float sv[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
        float y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float partner = __shfl_xor(x[j], PL, 64);
          y[j] = x[j] * cv[j] + (first ? -partner : partner) * sv[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = y[j];
      }
      uint4 o;
      o.x = pack_bf2(x[0], x[1]);
      o.y = pack_bf2(x[2], x[3]);
      o.z = pack_bf2(x[4], x[5]);
      o.w = pack_bf2(x[6], x[7]);
      *(uint4*)((bf16_t*)ep.out + (int64_t)m * ep.ldo + n) = o;
    } else {
      const uint32_t w4[4] = {cv.x, cv.y, cv.z, cv.w};
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[2 * j] = bf2f((bf16_t)(w4[j] & 0xffff));
        v[2 * j + 1] = bf2f((bf16_t)(w4[j] >> 16));
      }
      if constexpr (EPI == VGGT_EPI_GELU_BF16) {
        // the pre-activation (bf16 Linear output) for the GELU backward
        if (ep.out2) *(uint4*)((bf16_t*)(void*)ep.out2 + (int64_t)m * ep.ldo2 + n) = cv;
        // GELU of the bf16 Linear output from the table of torch's float32
        // GELU (the persistent form reads the same table from LDS): every
        // GEMM form gives bit-identical activations
        uint4 o;
        o.x = gelu2_tab(cv.x, gelu_lut);
        o.y = gelu2_tab(cv.y, gelu_lut);
        o.z = gelu2_tab(cv.z, gelu_lut);
        o.w = gelu2_tab(cv.w, gelu_lut);
        *(uint4*)((bf16_t*)ep.out + (int64_t)m * ep.ldo + n) = o;
      } else if constexpr (EPI == VGGT_EPI_RESID_F32) {
        float* xp = (float*)ep.out + (int64_t)m * ep.ldo + n;
        f32x4 x0 = *(f32x4*)xp, x1 = *(f32x4*)(xp + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x0[j] += g[j] * v[j];
          x1[j] += g[4 + j] * v[4 + j];
        }
        *(f32x4*)xp = x0;
        *(f32x4*)(xp + 4) = x1;
        if (ep.out2) {
          float* yp = ep.out2 + (int64_t)m * ep.ldo2 + n;
          *(f32x4*)yp = x0;
          *(f32x4*)(yp + 4) = x1;
        }
      } else {  // VGGT_EPI_F32
        float* yp = (float*)ep.out + (int64_t)m * ep.ldo + n;
        *(f32x4*)yp = f32x4{v[0], v[1], v[2], v[3]};
        *(f32x4*)(yp + 4) = f32x4{v[4], v[5], v[6], v[7]};
      }
    }
  }
}

template <int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                          const bf16_t* __restrict__ W, int64_t ldw, int M, int N,
                                                          int K, Epi ep) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tiles_n = N / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * BM;
  const int n0 = (t % tiles_n) * BN;
  const int nk = K / BK;

  // ---- LDS-DMA staging of one (A, W) K-slice into buffer `buf` ----
  auto stage = [&](int buf, int k0) {
    char* As = smem + buf * STAGE_BYTES;
    char* Ws = As + TILE;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int inst = wave * 4 + j;  // 16 x 1 KiB per tile, 4 per wave
      const int row = inst * 8 + (lane >> 3);
      const int chunk = (lane & 7) ^ (row & 7);
      const int am = min(m0 + row, M - 1);
      __builtin_amdgcn_global_load_lds((const void*)(A + (int64_t)am * lda + k0 + chunk * 8), LDS_PTR(As + inst * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(W + (int64_t)(n0 + row) * ldw + k0 + chunk * 8),
                                       LDS_PTR(Ws + inst * 1024), 16, 0, 0);
    }
  };

  const int wm = wave >> 1, wn = wave & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  auto compute = [&](int cur) {
    const char* As = smem + cur * STAGE_BYTES;
    const char* Ws = As + TILE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 wf[4], af[4];
      const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rw = wn * 64 + i * 16 + (lane & 15);
        wf[i] = *(const bf16x8*)(Ws + rw * 128 + ((chunk ^ (rw & 7)) << 4));
        const int ra = wm * 64 + i * 16 + (lane & 15);
        af[i] = *(const bf16x8*)(As + ra * 128 + ((chunk ^ (ra & 7)) << 4));
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni], af[mi], acc[ni][mi], 0, 0, 0);
    }
  };
  for (int kt = 0; kt < nk - 1; ++kt) {
    stage((kt & 1) ^ 1, (kt + 1) * BK);
    compute(kt & 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // LayerScale + residual epilogue: this thread's fp32 residual rows (the
  // write_tile mapping) are loaded now, all at once, so their HBM latency hides
  // behind the last K-step and the C-tile staging instead of serialising the
  // read-modify-write passes at the end
  constexpr int RCPR = BN / 8, RRPP = NT / RCPR, RNP = BM / RRPP;
  f32x4 rx[RNP][2];
  if constexpr (EPI == VGGT_EPI_RESID_F32) {
    const int n = n0 + (threadIdx.x % RCPR) * 8;
#pragma unroll
    for (int i = 0; i < RNP; ++i) {
      const int m = min(m0 + (int)threadIdx.x / RCPR + RRPP * i, M - 1);
      const float* xp = (const float*)ep.out + (int64_t)m * ep.ldo + n;
      rx[i][0] = __builtin_nontemporal_load((const f32x4*)xp);
      rx[i][1] = __builtin_nontemporal_load((const f32x4*)(xp + 4));
    }
  }
  compute((nk - 1) & 1);
  __syncthreads();

  // ---- epilogue 1: acc (C^T fragments) + bias -> bf16 C tile in LDS ----
  char* Cs = smem;
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int nl = wn * 64 + ni * 16 + 4 * (lane >> 4);
    const f32x4 bv = *(const f32x4*)(ep.bias + n0 + nl);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int ml = wm * 64 + mi * 16 + (lane & 15);
      uint2 pk;
      pk.x = pack_bf2(acc[ni][mi][0] + bv[0], acc[ni][mi][1] + bv[1]);
      pk.y = pack_bf2(acc[ni][mi][2] + bv[2], acc[ni][mi][3] + bv[3]);
      *(uint2*)(Cs + ml * CROW + nl * 2) = pk;
    }
  }
  __syncthreads();

  if constexpr (EPI == EPI_QKNORM_D64 || EPI == EPI_QKNORM_D128) {
    // RoPE cos/sin tables (a few KiB) into the LDS left over by the C tile
    constexpr int D = EPI == EPI_QKNORM_D64 ? 64 : 128;
    const int rd = ep.rope_mode == VGGT_ROPE_2D ? D / 2 : D;
    const int tab = ep.rope_mode != VGGT_ROPE_NONE ? ep.tab_len * rd : 0;
    float* ts = (float*)(smem + BM * CROW);
    if (tab > 0 && n0 < 2 * ep.hd && 2 * tab * 4 <= (int)sizeof(smem) - BM * CROW) {
      for (int i = threadIdx.x; i < tab; i += NT) {
        ts[i] = ep.cs[i];
        ts[tab + i] = ep.sn[i];
      }
      __syncthreads();
      write_tile<EPI, BM, BN, NT, CROW>(Cs, m0, n0, M, ep, ts, ts + tab);
      return;
    }
  }
  if constexpr (EPI == VGGT_EPI_RESID_F32) {
    const int ch = threadIdx.x % RCPR;
    const int n = n0 + ch * 8;
    const f32x4 g0 = *(const f32x4*)(ep.gamma + n);
    const f32x4 g1 = *(const f32x4*)(ep.gamma + n + 4);
#pragma unroll
    for (int i = 0; i < RNP; ++i) {
      const int ml = threadIdx.x / RCPR + RRPP * i;
      const int m = m0 + ml;
      if (m >= M) continue;
      const uint4 cv = *(const uint4*)(Cs + ml * CROW + ch * 16);
      const uint32_t w4[4] = {cv.x, cv.y, cv.z, cv.w};
      f32x4 x0 = rx[i][0], x1 = rx[i][1];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        x0[2 * j] += g0[2 * j] * bf2f((bf16_t)(w4[j] & 0xffff));
        x0[2 * j + 1] += g0[2 * j + 1] * bf2f((bf16_t)(w4[j] >> 16));
        x1[2 * j] += g1[2 * j] * bf2f((bf16_t)(w4[2 + j] & 0xffff));
        x1[2 * j + 1] += g1[2 * j + 1] * bf2f((bf16_t)(w4[2 + j] >> 16));
      }
      float* xp = (float*)ep.out + (int64_t)m * ep.ldo + n;
      *(f32x4*)xp = x0;
      *(f32x4*)(xp + 4) = x1;
      if (ep.out2) {
        float* yp = ep.out2 + (int64_t)m * ep.ldo2 + n;
        *(f32x4*)yp = x0;
        *(f32x4*)(yp + 4) = x1;
      }
    }
    return;
  }
  write_tile<EPI, BM, BN, NT, CROW>(Cs, m0, n0, M, ep);
}


// ===========================================================================
// Large-tile form: 256 x BN (BN = 256 or 128) block tile, 8 waves, BK = 32,
// a 4-slot LDS ring filled by buffer_load ... lds (LDS-DMA) three K-steps
// ahead, ONE barrier per K-step behind a COUNTED vmcnt, so the prefetch stays
// in flight across barriers (cdna_hip_programming.md §5 "what does break the
// ~900 TF ceiling").  64-B LDS rows; the swizzle chunk ^ h((row >> 2) & 3),
// h = {0,3,2,1}, makes every ds_read_b128 fragment read conflict-free over the
// four 16-lane groups; it is applied on the DMA source offset (the DMA image
// is lane-linear) and on the read.
// ===========================================================================
typedef int int32x4 __attribute__((ext_vector_type(4)));

constexpr int RBM = 256, RBK = 32, RNT = 512, RSLOTS = 4;

__device__ __forceinline__ int32x4 make_rsrc_u(const void* base) {
  const uint64_t b = (uint64_t)base;
  int32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((uint32_t)b);
  r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) & 0xffff;
  r[2] = -1;  // num_records: whole 4 GiB window (offsets are bounded by the caller)
  r[3] = 0x00020000;
  return r;
}

// 16 B per lane from (rsrc, voff + soff) into LDS at the wave-uniform address
// `lds` (+ lane * 16).  Kept in asm so hipcc's alias analysis does not drain
// vmcnt before the ring's ds_reads; completion is tracked by the counted
// vmcnt + barrier in the K-loop.
__device__ __forceinline__ void dma16s(int32x4 rsrc, uint32_t voff, uint32_t soff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
               : "memory");
}

__device__ __forceinline__ int ring_swz(int row, int chunk) { return chunk ^ ((4 - ((row >> 2) & 3)) & 3); }

template <int BN>
struct RingCfg {
  static constexpr int WM = BN == 256 ? 2 : 4;     // waves along M
  static constexpr int WN = 8 / WM;                // waves along N
  static constexpr int TM = RBM / WM;              // wave tile rows (M)
  static constexpr int TN = BN / WN;               // wave tile cols (N)
  static constexpr int MI = TM / 16, NI = TN / 16; // 16x16 fragments
  static constexpr int ABYTES = RBM * RBK * 2;     // 16 KiB
  static constexpr int WBYTES = BN * RBK * 2;
  static constexpr int SLOT = ABYTES + WBYTES;
  static constexpr int AL = ABYTES / 1024 / 8;     // DMA instructions per wave per stage (A)
  static constexpr int WL = WBYTES / 1024 / 8;     // (W)
  static constexpr int LPS = AL + WL;              // vmcnt units per stage
  static constexpr int CROW = BN * 2 + 16;
  static constexpr int LDS = (RSLOTS * SLOT > RBM * CROW) ? RSLOTS * SLOT : RBM * CROW;
};

template <int EPI, int BN>
__global__ __launch_bounds__(RNT, 1) void gemm_ring_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                           const bf16_t* __restrict__ W, int64_t ldw, int M, int N,
                                                           int K, Epi ep) {
  using C = RingCfg<BN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tiles_n = N / BN;
  const int tiles_m = (M + RBM - 1) / RBM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * RBM;
  const int n0 = (t % tiles_n) * BN;
  const int nk = K / RBK;

  // ---- loop-invariant DMA offsets: instruction i of this wave covers rows
  // (wave*L + i)*16 + lane/4, source chunk swizzled; rows past M clamp to M-1.
  const int32x4 ra = make_rsrc_u(A + (int64_t)m0 * lda);
  const int32x4 rw = make_rsrc_u(W + (int64_t)n0 * ldw);
  uint32_t aoff[C::AL], woff[C::WL];
#pragma unroll
  for (int i = 0; i < C::AL; ++i) {
    const int row = (wave * C::AL + i) * 16 + (lane >> 2);
    const int rr = min(m0 + row, M - 1) - m0;
    aoff[i] = (uint32_t)(rr * lda + ring_swz(row, lane & 3) * 8) * 2u;
  }
#pragma unroll
  for (int i = 0; i < C::WL; ++i) {
    const int row = (wave * C::WL + i) * 16 + (lane >> 2);
    woff[i] = (uint32_t)(row * ldw + ring_swz(row, lane & 3) * 8) * 2u;
  }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));
  auto stage = [&](int kt) {
    const uint32_t slot = lds0 + (kt & (RSLOTS - 1)) * C::SLOT;
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(kt * RBK * 2));
#pragma unroll
    for (int i = 0; i < C::AL; ++i) dma16s(ra, aoff[i], soff, slot + (wave * C::AL + i) * 1024);
#pragma unroll
    for (int i = 0; i < C::WL; ++i) dma16s(rw, woff[i], soff, slot + C::ABYTES + (wave * C::WL + i) * 1024);
  };

  // ---- loop-invariant fragment read offsets (row & 15 == lane & 15)
  const int wm = wave / C::WN, wn = wave % C::WN;
  const int fr = lane & 15, fc = lane >> 4;
  const uint32_t lane_off = fr * 64 + (ring_swz(fr, fc) << 4);
  const uint32_t a_off = (wm * C::TM) * 64 + lane_off;
  const uint32_t w_off = C::ABYTES + (wn * C::TN) * 64 + lane_off;

  f32x4 acc[C::NI][C::MI];
#pragma unroll
  for (int i = 0; i < C::NI; ++i)
#pragma unroll
    for (int j = 0; j < C::MI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- K-loop.  Step j's fragments are read into registers during step
  // j-1's MFMAs (register double buffer F0/F1), so a slot is free for
  // restaging as soon as its reads retired: the DMA runs four steps ahead.
  auto wait_landed = [&](int newer) {  // own DMA with `newer` later stages still in flight, then everyone's
    if constexpr (C::LPS == 4) {
      if (newer >= 3) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
      else if (newer == 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
      else if (newer == 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      if (newer >= 3) asm volatile("s_waitcnt vmcnt(9)\n\ts_barrier" ::: "memory");
      else if (newer == 2) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
      else if (newer == 1) asm volatile("s_waitcnt vmcnt(3)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
  };
  auto read_frags = [&](int kt, bf16x8(&wf)[C::NI], bf16x8(&af)[C::MI]) {
    const char* base = smem + (kt & (RSLOTS - 1)) * C::SLOT;
#pragma unroll
    for (int i = 0; i < C::NI; ++i) wf[i] = *(const bf16x8*)(base + w_off + i * 16 * 64);
#pragma unroll
    for (int i = 0; i < C::MI; ++i) af[i] = *(const bf16x8*)(base + a_off + i * 16 * 64);
  };
  // one K-step: MFMAs on (cw, ca) with the next step's reads into (nw, na)
  // issued after the first MI of them (sched_group_barrier pins the order)
  auto step = [&](int kt, bf16x8(&cw)[C::NI], bf16x8(&ca)[C::MI], bf16x8(&nw)[C::NI], bf16x8(&na)[C::MI]) {
    // this step's fragments retired (and with them every read of slot kt, which
    // is restaged below); step kt+1 landed for every wave
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (kt + 1 < nk) wait_landed(min(nk - 2 - kt, 2));
    else asm volatile("s_barrier" ::: "memory");
    if (kt + 4 < nk) stage(kt + 4);
    read_frags(kt + 1, nw, na);  // unconditional (a stale slot on the last step, unused): keeps one basic block
#pragma unroll
    for (int mi = 0; mi < C::MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < C::NI; ++ni)
        acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[ni], ca[mi], acc[ni][mi], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, C::NI, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, C::NI + C::MI, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, C::NI * (C::MI - 1), 0);
  };

  stage(0);
  if (nk > 1) stage(1);
  if (nk > 2) stage(2);
  if (nk > 3) stage(3);
  wait_landed(min(nk - 1, 3));
  bf16x8 w0[C::NI], a0[C::MI], w1[C::NI], a1[C::MI];
  read_frags(0, w0, a0);
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, w0, a0, w1, a1);
    if (kt + 1 < nk) step(kt + 1, w1, a1, w0, a0);
  }
  // all waves done with the ring (no DMA or read pending): reuse it as the C tile
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // ---- epilogue 1: acc (C^T fragments) + bias -> bf16 C tile in LDS ----
  char* Cs = smem;
#pragma unroll
  for (int ni = 0; ni < C::NI; ++ni) {
    const int nl = wn * C::TN + ni * 16 + 4 * (lane >> 4);
    const f32x4 bv = *(const f32x4*)(ep.bias + n0 + nl);
#pragma unroll
    for (int mi = 0; mi < C::MI; ++mi) {
      const int ml = wm * C::TM + mi * 16 + (lane & 15);
      uint2 pk;
      pk.x = pack_bf2(acc[ni][mi][0] + bv[0], acc[ni][mi][1] + bv[1]);
      pk.y = pack_bf2(acc[ni][mi][2] + bv[2], acc[ni][mi][3] + bv[3]);
      *(uint2*)(Cs + ml * C::CROW + nl * 2) = pk;
    }
  }
  __syncthreads();
  write_tile<EPI, RBM, BN, RNT, C::CROW>(Cs, m0, n0, M, ep);
}

template <int EPI, int BN>
int launch_ring(const bf16_t* a, int64_t lda, const bf16_t* w, int64_t ldw, int M, int N, int K, const Epi& ep,
                hipStream_t s) {
  using C = RingCfg<BN>;
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)gemm_ring_kernel<EPI, BN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              C::LDS);
    return true;
  }();
  (void)attr;
  const int nwg = ((M + RBM - 1) / RBM) * (N / BN);
  gemm_ring_kernel<EPI, BN><<<nwg, RNT, C::LDS, s>>>(a, lda, w, ldw, M, N, K, ep);
  return VGGT_OK;
}

// ===========================================================================
// Two-per-CU form: 256 x 128 block tile, 4 waves (2 M x 2 N; wave tile
// 128 x 64 = 8 x 4 fragments of v_mfma_f32_16x16x32_bf16), BK = 32, a 3-slot
// LDS ring filled by LDS-DMA two K-steps ahead behind a counted vmcnt and a
// raw barrier (one per K-step), fragments double-buffered in registers.
// __launch_bounds__(256, 2) and 72 KiB of LDS: TWO workgroups per CU, meant
// to run one workgroup's epilogue beside the other's MFMA main loop.
// Measured and not used by default (scripts/gemmbench.py, r3c-r3f): the
// 64-B-row K-steps make its main loop slower than the 256x256 ping-pong
// form (fc1 plain 193-197 vs 173-179 us), and the epilogue still does not
// overlap (GELU +37-44 us in both forms), with or without a half-tile start
// stagger of the second workgroup slot or s_setprio around the MFMAs.
// ===========================================================================
constexpr int TBM = 256, TBN = 128, TBK = 32, TNT = 256, TSLOTS = 3;

struct TwoCfg {
  static constexpr int WN = 2;                    // waves along N
  static constexpr int TM = 128, TN = 64;         // wave tile
  static constexpr int MI = TM / 32, NI = TN / 32;  // 32x32 fragments
  static constexpr int ABYTES = TBM * TBK * 2;    // 16 KiB
  static constexpr int WBYTES = TBN * TBK * 2;    // 8 KiB
  static constexpr int SLOT = ABYTES + WBYTES;    // 24 KiB
  static constexpr int AL = ABYTES / 1024 / 4;    // LDS-DMA instructions per wave per stage (A)
  static constexpr int WL = WBYTES / 1024 / 4;    // (W)
  static constexpr int LPS = AL + WL;             // vmcnt units per stage
  static constexpr int CROW = TBN * 2 + 16;
  static constexpr int LDS = TSLOTS * SLOT;
};
static_assert(TwoCfg::LDS >= TBM * TwoCfg::CROW, "the bf16 C tile reuses the ring");
static_assert(TwoCfg::LPS == 6, "wait counts below assume 6 DMA instructions per stage");

// The main loop runs on v_mfma_f32_32x32x16_bf16, which holds the SIMD's
// vector issue for 8 of its 32 cycles (the 16x16x32 form: 8 of 16), so the
// other workgroup's epilogue VALU finds issue slots beside it.
template <int EPI>
__global__ __launch_bounds__(TNT, 2) void gemm_two_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                          const bf16_t* __restrict__ W, int64_t ldw, int M, int N,
                                                          int K, Epi ep) {
  using C = TwoCfg;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tiles_n = N / TBN;
  const int tiles_m = (M + TBM - 1) / TBM;
  const int ntiles = tiles_m * tiles_n;
  const int nk = K / TBK;
  // Persistent: workgroup b runs tiles b, b + grid, ... (all on b's XCD; the
  // remap keeps each XCD's tiles contiguous in M-panel order).
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));
  auto slot_of = [](int kt) -> uint32_t { return (uint32_t)(kt % TSLOTS) * C::SLOT; };
  // ---- loop-invariant fragment read offsets: fragment row & 31 == lane & 31,
  // k chunk 2*ks + (lane >> 5) of the 64-B row, swizzled
  const int wm = wave / C::WN, wn = wave % C::WN;
  const int fr = lane & 31, hl = lane >> 5;
  uint32_t a_off[2], w_off[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const uint32_t lo = fr * 64 + (ring_swz(fr, 2 * ks + hl) << 4);
    a_off[ks] = (wm * C::TM) * 64 + lo;
    w_off[ks] = C::ABYTES + (wn * C::TN) * 64 + lo;
  }

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int t = xcd_remap(tile, ntiles);
    const int m0 = (t / tiles_n) * TBM;
    const int n0 = (t % tiles_n) * TBN;

    // ---- DMA offsets: instruction i of this wave covers rows
    // (wave*L + i)*16 + lane/4 (64-B rows), source chunk swizzled; rows past M
    // clamp to M-1.
    const int32x4 ra = make_rsrc_u(A + (int64_t)m0 * lda);
    const int32x4 rw = make_rsrc_u(W + (int64_t)n0 * ldw);
    uint32_t aoff[C::AL], woff[C::WL];
#pragma unroll
    for (int i = 0; i < C::AL; ++i) {
      const int row = (wave * C::AL + i) * 16 + (lane >> 2);
      const int rr = min(m0 + row, M - 1) - m0;
      aoff[i] = (uint32_t)(rr * lda + ring_swz(row, lane & 3) * 8) * 2u;
    }
#pragma unroll
    for (int i = 0; i < C::WL; ++i) {
      const int row = (wave * C::WL + i) * 16 + (lane >> 2);
      woff[i] = (uint32_t)(row * ldw + ring_swz(row, lane & 3) * 8) * 2u;
    }
    auto stage = [&](int kt) {
      const uint32_t slot = lds0 + slot_of(kt);
      const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(kt * TBK * 2));
#pragma unroll
      for (int i = 0; i < C::AL; ++i) dma16s(ra, aoff[i], soff, slot + (wave * C::AL + i) * 1024);
#pragma unroll
      for (int i = 0; i < C::WL; ++i) dma16s(rw, woff[i], soff, slot + C::ABYTES + (wave * C::WL + i) * 1024);
    };

    f32x16 acc[C::NI][C::MI];
#pragma unroll
    for (int i = 0; i < C::NI; ++i)
#pragma unroll
      for (int j = 0; j < C::MI; ++j) acc[i][j] = f32x16{};

    // fragments of one 16-deep half K-step, double-buffered per half: the
    // MFMAs of half h run beside the reads of half h+1
    struct Frag {
      bf16x8 w[C::NI], a[C::MI];
    };
    auto read_half = [&](int kt, int ks, Frag& f) {
      const char* base = smem + slot_of(kt);
#pragma unroll
      for (int i = 0; i < C::NI; ++i) f.w[i] = *(const bf16x8*)(base + w_off[ks] + i * 32 * 64);
#pragma unroll
      for (int i = 0; i < C::MI; ++i) f.a[i] = *(const bf16x8*)(base + a_off[ks] + i * 32 * 64);
    };
    auto mfmas = [&](const Frag& f) {
#pragma unroll
      for (int mi = 0; mi < C::MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < C::NI; ++ni)
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.w[ni], f.a[mi], acc[ni][mi], 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, C::NI + C::MI, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, C::NI * C::MI - 1, 0);
    };
    // one K-step on slot kt: half 0 (reads of half 1 beside it), then -- once
    // every read of slot kt retired and slot kt+1 landed for every wave (slot
    // kt+2 stays in flight across the barrier) -- restage slot kt with kt+3
    // and run half 1 beside the reads of the next step's half 0
    Frag f0, f1;
    auto step = [&](int kt) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      read_half(kt, 1, f1);
      mfmas(f0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      if (kt + 3 < nk) stage(kt + 3);  // into slot kt % 3
      read_half(kt + 1, 0, f0);  // unconditional (a stale slot after the last step, unused)
      mfmas(f1);
    };

    stage(0);
    if (nk > 1) stage(1);
    if (nk > 2) stage(2);
    if (nk > 2) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
    else if (nk > 1) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    read_half(0, 0, f0);
    for (int kt = 0; kt < nk; ++kt) step(kt);
    // all waves done with the ring (no DMA or read pending): reuse it as the C tile
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");

    // ---- epilogue 1: acc (C^T fragments: lane = token, rows 8g + 4hl + 0..3 =
    // features) + bias -> bf16 C tile in LDS
    char* Cs = smem;
#pragma unroll
    for (int ni = 0; ni < C::NI; ++ni)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nl = wn * C::TN + ni * 32 + 8 * g + 4 * hl;
        const f32x4 bv = *(const f32x4*)(ep.bias + n0 + nl);
#pragma unroll
        for (int mi = 0; mi < C::MI; ++mi) {
          const int ml = wm * C::TM + mi * 32 + fr;
          uint2 pk;
          pk.x = pack_bf2(acc[ni][mi][4 * g] + bv[0], acc[ni][mi][4 * g + 1] + bv[1]);
          pk.y = pack_bf2(acc[ni][mi][4 * g + 2] + bv[2], acc[ni][mi][4 * g + 3] + bv[3]);
          *(uint2*)(Cs + ml * C::CROW + nl * 2) = pk;
        }
      }
    __syncthreads();
    write_tile<EPI, TBM, TBN, TNT, C::CROW>(Cs, m0, n0, M, ep);
    __syncthreads();  // the C tile (= the ring) is read out before the next tile's DMA
  }
}

template <int EPI>
int launch_two(const bf16_t* a, int64_t lda, const bf16_t* w, int64_t ldw, int M, int N, int K, const Epi& ep,
               hipStream_t s) {
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)gemm_two_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              TwoCfg::LDS);
    return true;
  }();
  (void)attr;
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  const int ntiles = ((M + TBM - 1) / TBM) * (N / TBN);
  const int nwg = ntiles < 2 * cus ? ntiles : 2 * cus;
  gemm_two_kernel<EPI><<<nwg, TNT, TwoCfg::LDS, s>>>(a, lda, w, ldw, M, N, K, ep);
  return VGGT_OK;
}

// ===========================================================================
// Ping-pong form: 256 x BN block tile (BN = 256 / 192 / 128), BK = 64, two
// LDS buffers filled by LDS-DMA, 8 waves as 2 (M) x 4 (N); wave (wm, wn) owns
// rows wm*128.. and columns wn*BN/4.. of the tile.  Each K-tile is two
// k-steps; per k-step a wave runs a READ segment (its fragments for the step
// from LDS -- and, on the first step, the DMA of the next K-tile) and a MATH
// segment (8 x BN/64 MFMAs), separated by workgroup barriers.  The two M
// halves are staggered by one barrier (waves 4-7 start with an extra one),
// and each SIMD holds one wave of each half, so on every SIMD one wave's
// MFMAs run beside the other wave's LDS reads (cdna_hip_programming.md §5,
// "256² 8-phase template"; MI355X_MICROARCH.md "Two waves per SIMD").
//
// LDS hazards (two buffers, K-tile kt in buffer kt & 1):
//  * WAR: the DMA of K-tile kt+1 is issued in READ(kt, 0).  The last reads of
//    its buffer are READ(kt-1, 1) of both halves, each ending with
//    lgkmcnt(0) before its barrier; READ(kt, 0) of a half starts after the
//    barrier that ends the other half's READ(kt-1, 1).
//  * RAW: every wave waits vmcnt(0) for its own DMA at the end of READ(kt, 1)
//    (before that segment's barrier); READ(kt+1, 0) of either half starts at
//    least one barrier later.
// ===========================================================================
constexpr int PBM = 256, PBK = 64, PNT = 512;

template <int BN>
struct PPCfg {
  static constexpr int WN = BN / 4;               // wave tile columns
  static constexpr int NI = WN / 16;              // 16-column fragments per wave
  static constexpr int MI = 8;                    // 16-row fragments per wave (128 rows)
  static constexpr int ABYTES = PBM * PBK * 2;    // 32 KiB
  static constexpr int WBYTES = BN * PBK * 2;
  static constexpr int BUF = ABYTES + WBYTES;
  static constexpr int AL = ABYTES / 1024 / 8;    // LDS-DMA instructions per wave per K-tile (A)
  static constexpr int WL = WBYTES / 1024 / 8;    // (W)
  static constexpr int CROW = BN * 2 + 16;
  static constexpr int LDS = (2 * BUF > PBM * CROW) ? 2 * BUF : PBM * CROW;
};

template <int EPI, int BN>
__global__ __launch_bounds__(PNT, 1) void gemm_pp_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                         const bf16_t* __restrict__ W, int64_t ldw, int M, int N,
                                                         int K, Epi ep) {
  using C = PPCfg<BN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tiles_n = N / BN;
  const int tiles_m = (M + PBM - 1) / PBM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * PBM;
  const int n0 = (t % tiles_n) * BN;
  const int nk = K / PBK;
  const int wm = wave >> 2, wn = wave & 3;

  // ---- LDS-DMA: piece p (1 KiB) of an operand image = rows 8p..8p+7 (128-B
  // rows); lane -> row 8p + lane/8, 16-B chunk lane%8 XOR-swizzled on the
  // source (the DMA image is lane-linear); rows past M clamp to M-1.
  const int32x4 ra = make_rsrc_u(A + (int64_t)m0 * lda);
  const int32x4 rw = make_rsrc_u(W + (int64_t)n0 * ldw);
  uint32_t aoff[C::AL], woff[C::WL];
#pragma unroll
  for (int i = 0; i < C::AL; ++i) {
    const int row = (wave * C::AL + i) * 8 + (lane >> 3);
    const int rr = min(m0 + row, M - 1) - m0;
    aoff[i] = (uint32_t)(rr * lda + ((lane & 7) ^ (row & 7)) * 8) * 2u;
  }
#pragma unroll
  for (int i = 0; i < C::WL; ++i) {
    const int row = (wave * C::WL + i) * 8 + (lane >> 3);
    woff[i] = (uint32_t)(row * ldw + ((lane & 7) ^ (row & 7)) * 8) * 2u;
  }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));
  auto stage = [&](int buf, int kt) {
    const uint32_t b = lds0 + buf * C::BUF;
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(kt * PBK * 2));
#pragma unroll
    for (int i = 0; i < C::AL; ++i) dma16s(ra, aoff[i], soff, b + (wave * C::AL + i) * 1024);
#pragma unroll
    for (int i = 0; i < C::WL; ++i) dma16s(rw, woff[i], soff, b + C::ABYTES + (wave * C::WL + i) * 1024);
  };

  // ---- fragment read offsets: row & 7 == lane & 7, so the swizzled chunk of
  // k-step ks is lane-only; everything else is an immediate
  const int fr = lane & 15, fc = lane >> 4;
  uint32_t a_off[2], w_off[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const uint32_t sw = (uint32_t)(((ks * 4 + fc) ^ (fr & 7)) << 4);
    a_off[ks] = (wm * 128 + fr) * 128 + sw;
    w_off[ks] = C::ABYTES + (wn * C::WN + fr) * 128 + sw;
  }

  f32x4 acc[C::NI][C::MI];
#pragma unroll
  for (int i = 0; i < C::NI; ++i)
#pragma unroll
    for (int j = 0; j < C::MI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[C::MI], wf[C::NI];

  auto read_frags = [&](int buf, int ks) {
    const char* base = smem + buf * C::BUF;
#pragma unroll
    for (int i = 0; i < C::NI; ++i) wf[i] = *(const bf16x8*)(base + w_off[ks] + i * 16 * 128);
#pragma unroll
    for (int i = 0; i < C::MI; ++i) af[i] = *(const bf16x8*)(base + a_off[ks] + i * 16 * 128);
  };
  auto math = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mi = 0; mi < C::MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < C::NI; ++ni)
        acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni], af[mi], acc[ni][mi], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (wm == 1) asm volatile("s_barrier" ::: "memory");  // stagger the second M half by one segment
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    // READ(kt, 0): next K-tile's DMA into the other buffer, this step's fragments
    if (kt + 1 < nk) stage(buf ^ 1, kt + 1);
    read_frags(buf, 0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    math();  // MATH(kt, 0)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    // READ(kt, 1); own DMA of K-tile kt+1 retired before the barrier
    read_frags(buf, 1);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    math();  // MATH(kt, 1)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
  }
  if (wm == 0) asm volatile("s_barrier" ::: "memory");  // balance the stagger
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // ---- epilogue 1: acc (C^T fragments) + bias -> bf16 C tile in LDS ----
  char* Cs = smem;
#pragma unroll
  for (int ni = 0; ni < C::NI; ++ni) {
    const int nl = wn * C::WN + ni * 16 + 4 * (lane >> 4);
    const f32x4 bv = *(const f32x4*)(ep.bias + n0 + nl);
#pragma unroll
    for (int mi = 0; mi < C::MI; ++mi) {
      const int ml = wm * 128 + mi * 16 + (lane & 15);
      uint2 pk;
      pk.x = pack_bf2(acc[ni][mi][0] + bv[0], acc[ni][mi][1] + bv[1]);
      pk.y = pack_bf2(acc[ni][mi][2] + bv[2], acc[ni][mi][3] + bv[3]);
      *(uint2*)(Cs + ml * C::CROW + nl * 2) = pk;
    }
  }
  __syncthreads();
  if constexpr (EPI == EPI_QKNORM_D64 || EPI == EPI_QKNORM_D128) {
    constexpr int D = EPI == EPI_QKNORM_D64 ? 64 : 128;
    const int rd = ep.rope_mode == VGGT_ROPE_2D ? D / 2 : D;
    const int tab = ep.rope_mode != VGGT_ROPE_NONE ? ep.tab_len * rd : 0;
    float* ts = (float*)(smem + PBM * C::CROW);
    if (tab > 0 && n0 < 2 * ep.hd && PBM * C::CROW + 2 * tab * 4 <= C::LDS) {
      for (int i = threadIdx.x; i < tab; i += PNT) {
        ts[i] = ep.cs[i];
        ts[tab + i] = ep.sn[i];
      }
      __syncthreads();
      write_tile<EPI, PBM, BN, PNT, C::CROW>(Cs, m0, n0, M, ep, ts, ts + tab);
      return;
    }
  }
  write_tile<EPI, PBM, BN, PNT, C::CROW>(Cs, m0, n0, M, ep);
}

template <int EPI, int BN>
int launch_pp(const bf16_t* a, int64_t lda, const bf16_t* w, int64_t ldw, int M, int N, int K, const Epi& ep,
              hipStream_t s) {
  using C = PPCfg<BN>;
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)gemm_pp_kernel<EPI, BN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              C::LDS);
    return true;
  }();
  (void)attr;
  const int nwg = ((M + PBM - 1) / PBM) * (N / BN);
  gemm_pp_kernel<EPI, BN><<<nwg, PNT, C::LDS, s>>>(a, lda, w, ldw, M, N, K, ep);
  return VGGT_OK;
}

// ===========================================================================
// Persistent ping-pong form (mode 9): the 256 x 256 ping-pong main loop above,
// one workgroup per CU looping over tiles, with the epilogue written straight
// from the accumulators (bias from an LDS copy, GELU, bf16 pack, buffer
// stores) and the NEXT tile's first two K-tiles issued by LDS-DMA before the
// epilogue: the operand loads land while the epilogue runs, and the stores
// drain during the next tile's first K-tile instead of before the workgroup
// may retire (the one-shot forms pay prologue latency + epilogue + store
// drain per tile: ~9 us of a ~30 us fc1 tile, scripts/gemmbench.py K=64 runs).
//
// vmcnt bookkeeping (gfx9: one in-order counter for loads, stores and
// LDS-DMA, max 63): per wave a K-tile is LPS = AL + WL DMA pieces and the
// epilogue issues exactly NST buffer stores (always issued: rows past M are
// dropped by the descriptor's num_records), so
//   * after the epilogue: vmcnt(LPS + NST) = this wave's K-tile 0 landed;
//   * READ(0, 1) of a tile after the first: vmcnt(NST) = K-tile 1 landed;
//   * every other READ(kt, 1): vmcnt(0) (K-tile kt+1 is the youngest).
// The bias of all N columns is copied to LDS once (N <= 4096), so the
// epilogue issues no compiler-visible global load (whose wait would drain
// the in-flight DMA).
// ===========================================================================
constexpr int PP_MAXN = 4096;
constexpr int PP_LDS_MAX = 160 * 1024;

// VGGT_GEMM_PERSIST (A/B of the auto policy): bit 0 = the persistent form for
// the bf16 / GELU / f32 GEMMs, bit 1 = for the fused qkv GEMM, bit 2 = for the
// LayerScale-residual GEMMs (default all)
inline int persist_policy(hipStream_t s) {
  static int p = [] {
    const char* e = getenv("VGGT_GEMM_PERSIST");
    return e ? atoi(e) : 7;
  }();
  // a stream configured for short workgroups (vggt_set_stream_config) gets none of the persistent forms
  return (vggt_stream_flags(s) & VGGT_STREAM_SHORT_WORKGROUPS) ? 0 : p;
}

// sum over the four 16-lane rows of a wave (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float rows4_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Tile BMT x 256 (BMT = 256, or 192 where 256-row tiles quantise badly: the
// N = 1024 projections, 344 -> 460 tiles on 256 CUs); wave tile (BMT/2) x 64.
template <int BMT>
struct PPXCfg {
  static constexpr int BN = 256, WN = 64, NI = 4, MI = BMT / 32, HM = BMT / 2;
  static constexpr int ABYTES = BMT * PBK * 2;
  static constexpr int WBYTES = BN * PBK * 2;
  static constexpr int BUF = ABYTES + WBYTES;
  static constexpr int AL = ABYTES / 1024 / 8;
  static constexpr int WL = WBYTES / 1024 / 8;
};

// Tile t -> (M-tile, N-tile), grouped by gm M-tiles (gm <= 1: row-major).  An
// XCD's concurrent tiles are consecutive t, so with gm = 4 and 32 CUs per XCD a
// round covers 4 M-panels x 8 N-panels instead of 2 x 16 (fc1): 12 instead of 18
// distinct K-slices per K-step fetched into that XCD's L2.
__device__ __forceinline__ void grouped_tile(int t, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  if (gm <= 1) {
    tm = t / tiles_n;
    tn = t - tm * tiles_n;
    return;
  }
  const int per = gm * tiles_n;
  const int g = t / per, r = t - g * per;
  const int rows = min(gm, tiles_m - g * gm);
  tm = g * gm + r % rows;
  tn = r / rows;
}

template <int EPI, int BMT, bool FK>
__global__ __launch_bounds__(PNT, 1) void gemm_ppp_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                          const bf16_t* __restrict__ W, int64_t ldw, int M, int N,
                                                          int K, Epi ep, int sched) {
  constexpr int BN = 256;
  using C = PPXCfg<BMT>;
  static_assert(C::AL * 1024 * 8 == C::ABYTES, "whole DMA pieces per wave");
  constexpr int LPS = C::AL + C::WL;
  // buffer stores per wave per tile (RESID: the residual and its optional mirror)
  constexpr bool GELU = EPI == VGGT_EPI_GELU_BF16 || EPI == EPI_GELU_PRE;
  constexpr int NST = EPI == VGGT_EPI_F32 || EPI == EPI_GELU_PRE ? C::NI * C::MI
                      : EPI == VGGT_EPI_RESID_F32 ? 2 * C::NI * C::MI : C::NI * C::MI / 2;
  static_assert(LPS + NST <= 63, "vmcnt range");
  static_assert(EPI != VGGT_EPI_RESID_F32 || BMT == 192, "residual tiles are 192 rows (register budget)");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* bias_s = (float*)(smem + 2 * C::BUF);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tiles_n = N / BN;
  const int tiles_m = (M + BMT - 1) / BMT;
  const int ntiles = tiles_m * tiles_n;
  const int nk = K / PBK;
  const int wm = wave >> 2, wn = wave & 3;
  const bool split = (sched >> 8) & 1;
  const int gm = sched & 255;

  for (int i = threadIdx.x; i < N; i += PNT) bias_s[i] = ep.bias[i];
  float* gam_s = bias_s + N;  // RESID: LayerScale gamma
  if constexpr (EPI == VGGT_EPI_RESID_F32)
    for (int i = threadIdx.x; i < N; i += PNT) gam_s[i] = ep.gamma[i];
  uint16_t* lut_s = (uint16_t*)(bias_s + N);  // GELU: the bf16 table
  if constexpr (GELU)
    for (int i = threadIdx.x; i < GELU_LUT_N; i += PNT) ((uint32_t*)lut_s)[i] = ((const uint32_t*)gelu_lut)[i];
  // EPI_QKNORM_D64: q/k norm weights (qw qb kw kb, 64 each), RoPE-2D cos / sin
  // tables [tab_len][32] and the positions (y | x << 8 per position index)
  float* qkn_s = bias_s + N;
  float* cs_s = qkn_s + 256;
  const int tab = (EPI == EPI_QKNORM_D64 && ep.rope_mode == VGGT_ROPE_2D) ? ep.tab_len : 0;
  float* sn_s = cs_s + tab * 32;
  uint16_t* pos_s = (uint16_t*)(sn_s + tab * 32);
  if constexpr (EPI == EPI_QKNORM_D64) {
    for (int i = threadIdx.x; i < 64; i += PNT) {
      qkn_s[i] = ep.qw ? ep.qw[i] : 1.f;
      qkn_s[64 + i] = ep.qb ? ep.qb[i] : 0.f;
      qkn_s[128 + i] = ep.kw ? ep.kw[i] : 1.f;
      qkn_s[192 + i] = ep.kb ? ep.kb[i] : 0.f;
    }
    for (int i = threadIdx.x; i < tab * 32; i += PNT) {
      cs_s[i] = ep.cs[i];
      sn_s[i] = ep.sn[i];
    }
    if (tab)
      for (int i = threadIdx.x; i < ep.period; i += PNT) {
        const int py = min(max(ep.pos[2 * i], 0), tab - 1), px = min(max(ep.pos[2 * i + 1], 0), tab - 1);
        pos_s[i] = (uint16_t)(py | (px << 8));
      }
  }
  __syncthreads();  // no DMA in flight yet: a plain barrier

  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));
  const int fr = lane & 15, fc = lane >> 4;
  uint32_t a_off[2], w_off[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const uint32_t sw = (uint32_t)(((ks * 4 + fc) ^ (fr & 7)) << 4);
    a_off[ks] = (wm * C::HM + fr) * 128 + sw;
    w_off[ks] = C::ABYTES + (wn * C::WN + fr) * 128 + sw;
  }
  // per-tile DMA state
  int32x4 ra, rw;
  uint32_t aoff[C::AL], woff[C::WL];
  auto setup = [&](int tile) {
    int tm, tn;
    grouped_tile(xcd_remap(tile, ntiles), tiles_m, tiles_n, gm, tm, tn);
    const int m0 = tm * BMT, n0 = tn * BN;
    ra = make_rsrc_u(A + (int64_t)m0 * lda);
    rw = make_rsrc_u(W + (int64_t)n0 * ldw);
#pragma unroll
    for (int i = 0; i < C::AL; ++i) {
      const int row = (wave * C::AL + i) * 8 + (lane >> 3);
      const int rr = min(m0 + row, M - 1) - m0;
      aoff[i] = (uint32_t)(rr * lda + ((lane & 7) ^ (row & 7)) * 8) * 2u;
    }
#pragma unroll
    for (int i = 0; i < C::WL; ++i) {
      const int row = (wave * C::WL + i) * 8 + (lane >> 3);
      woff[i] = (uint32_t)(row * ldw + ((lane & 7) ^ (row & 7)) * 8) * 2u;
    }
  };
  auto stage = [&](int buf, int kt) {
    const uint32_t b = lds0 + buf * C::BUF;
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(kt * PBK * 2));
#pragma unroll
    for (int i = 0; i < C::AL; ++i) dma16s(ra, aoff[i], soff, b + (wave * C::AL + i) * 1024);
#pragma unroll
    for (int i = 0; i < C::WL; ++i) dma16s(rw, woff[i], soff, b + C::ABYTES + (wave * C::WL + i) * 1024);
  };
  // split staging (sched bit 8, default; VGGT_GEMM_SPLITDMA=0 turns it off): the W
  // pieces at READ(kt, 0), the A pieces at READ(kt, 1), so both READ segments carry
  // half of the K-tile's DMA instead of one carrying all of it next to its 12
  // ds_reads (gemmbench r3v: fc1 at K = 4096 597.6 -> 569.6 us, plain qkv 146 -> 140 us)
  auto stage_w = [&](int buf, int kt) {
    const uint32_t b = lds0 + buf * C::BUF;
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(kt * PBK * 2));
#pragma unroll
    for (int i = 0; i < C::WL; ++i) dma16s(rw, woff[i], soff, b + C::ABYTES + (wave * C::WL + i) * 1024);
  };
  // the W pieces of the other wave half (rows + 128: the swizzle is row & 7, the same)
  auto stage_w2 = [&](int buf, int kt) {
    const uint32_t b = lds0 + buf * C::BUF;
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(kt * PBK * 2 + 4 * C::WL * 8 * ldw * 2));
#pragma unroll
    for (int i = 0; i < C::WL; ++i) dma16s(rw, woff[i], soff, b + C::ABYTES + ((wave + 4) * C::WL + i) * 1024);
  };
  auto stage_a = [&](int buf, int kt) {
    const uint32_t b = lds0 + buf * C::BUF;
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(kt * PBK * 2));
#pragma unroll
    for (int i = 0; i < C::AL; ++i) dma16s(ra, aoff[i], soff, b + (wave * C::AL + i) * 1024);
  };

  f32x4 acc[C::NI][C::MI];
  bf16x8 af[C::MI], wf[C::NI];
  auto read_frags = [&](int buf, int ks) {
    const char* base = smem + buf * C::BUF;
#pragma unroll
    for (int i = 0; i < C::NI; ++i) wf[i] = *(const bf16x8*)(base + w_off[ks] + i * 16 * 128);
#pragma unroll
    for (int i = 0; i < C::MI; ++i) af[i] = *(const bf16x8*)(base + a_off[ks] + i * 16 * 128);
  };
  auto math = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mi = 0; mi < C::MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < C::NI; ++ni)
        acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni], af[mi], acc[ni][mi], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // FK: one READ / MATH segment per whole K-tile (both K halves' fragments held)
  bf16x8 af2[FK ? C::MI : 1], wf2[FK ? C::NI : 1];
  auto read_frags2 = [&](int buf) {
    const char* base = smem + buf * C::BUF;
#pragma unroll
    for (int i = 0; i < C::NI; ++i) wf2[i] = *(const bf16x8*)(base + w_off[1] + i * 16 * 128);
#pragma unroll
    for (int i = 0; i < C::MI; ++i) af2[i] = *(const bf16x8*)(base + a_off[1] + i * 16 * 128);
  };
  auto math2 = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mi = 0; mi < C::MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < C::NI; ++ni)
        acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni], af[mi], acc[ni][mi], 0, 0, 0);
#pragma unroll
    for (int mi = 0; mi < C::MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < C::NI; ++ni)
        acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf2[ni], af2[mi], acc[ni][mi], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  // prologue: the first tile's K-tiles 0 and 1
  setup(tile);
  int b0 = 0;  // buffer of the current tile's K-tile 0
  stage(0, 0);
  if (nk > 1) {
    stage(1, 1);
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(LPS) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  bool stores_out = false;  // this wave has NST epilogue stores younger than K-tile 1's DMA
  for (;;) {
    int tm, tn;
    grouped_tile(xcd_remap(tile, ntiles), tiles_m, tiles_n, gm, tm, tn);
    const int m0 = tm * BMT, n0 = tn * BN;
#pragma unroll
    for (int i = 0; i < C::NI; ++i)
#pragma unroll
      for (int j = 0; j < C::MI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (wm == 1) asm volatile("s_barrier" ::: "memory");  // stagger the second M half by one segment
    if constexpr (FK) {
      // whole-K-tile loop.  DMA placement: half 0 issues every W piece of K-tile kt+1 (its own
      // rows and, through the scalar offset, half 1's 128 rows on) and half 1 only its A pieces;
      // both wait for them at the end of MATH(kt), so no READ segment waits on DMA
      // (profiles/r7c-r7d: aggregator step 102.4 -> 99.3 ms against waiting at the end of READ;
      // the other placements measured -- half 0 deferring only its own wait, half 1 staging
      // K-tile kt+2 inside MATH, half 1 issuing its W pieces after its MFMAs, fragment reads
      // ahead of the DMA issue -- were slower and are gone)
      for (int kt = 0; kt < nk; ++kt) {
        const int buf = (b0 + kt) & 1;
        const bool pf = kt >= 1 && kt + 1 < nk;
        // READ(kt): K-tile kt+1's DMA pieces, then both K halves' fragments
        if (pf) {
          if (wm == 0) {
            stage_w(buf ^ 1, kt + 1);
            stage_w2(buf ^ 1, kt + 1);
          }
          stage_a(buf ^ 1, kt + 1);
        }
        read_frags(buf, 0);
        read_frags2(buf);
        // half 1's K-tile 0 was staged before the loop: it waits for it here
        const bool lead = !(wm == 1 && kt == 0);
        if (lead) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else if (stores_out) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(NST) : "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        math2();
        __builtin_amdgcn_sched_barrier(0);
        if (lead) {
          if (kt == 0 && stores_out) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(NST) : "memory");
          else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        } else {
          asm volatile("s_barrier" ::: "memory");
        }
      }
    } else {
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = (b0 + kt) & 1;
      const bool pf = kt >= 1 && kt + 1 < nk;  // this step issues K-tile kt+1 (K-tile 1 was issued ahead)
      // READ(kt, 0): K-tile kt+1's DMA (split: its W half), this step's fragments
      if (pf) {
        if (split) stage_w(buf ^ 1, kt + 1);
        else stage(buf ^ 1, kt + 1);
      }
      read_frags(buf, 0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      math();
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_barrier" ::: "memory");
      // READ(kt, 1); own DMA of K-tile kt+1 retired before the barrier (split: the W
      // half here, the A half -- read first by this wave half, one segment later --
      // at the end of MATH(kt, 1))
      if (pf && split) {
        stage_a(buf ^ 1, kt + 1);
        read_frags(buf, 1);
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(C::AL) : "memory");
      } else {
        read_frags(buf, 1);
        if (kt == 0 && stores_out) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(NST) : "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      math();
      __builtin_amdgcn_sched_barrier(0);
      if (pf && split) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_barrier" ::: "memory");
    }
    }
    if (wm == 0) asm volatile("s_barrier" ::: "memory");  // balance the stagger
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every read of both buffers retired

    // RESID: this tile's fp32 residual rows, loaded BEFORE the next tile's DMA
    // (the compiler's waits for them then never cover the younger DMA)
    f32x4 rx[C::NI][EPI == VGGT_EPI_RESID_F32 ? C::MI : 1];
    if constexpr (EPI == VGGT_EPI_RESID_F32) {
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((float*)ep.out + (int64_t)m0 * ep.ldo), 0, (int)(min(M - m0, BMT) * ep.ldo * 4), 0x00020000);
#pragma unroll
      for (int ni = 0; ni < C::NI; ++ni)
#pragma unroll
        for (int mi = 0; mi < C::MI; ++mi) {
          const int ml = wm * C::HM + mi * 16 + (lane & 15);
          const int nl = n0 + wn * C::WN + ni * 16 + 4 * (lane >> 4);
          rx[ni][mi] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, (ml * (int)ep.ldo + nl) * 4, 0, 0));
        }
    }
    // the next tile's K-tiles 0 and 1, in flight during this epilogue
    const int next = tile + gridDim.x;
    const bool more = next < ntiles;
    const int nb0 = (b0 + nk) & 1;
    if (more) {
      setup(next);
      stage(nb0, 0);
      if (nk > 1) stage(nb0 ^ 1, 1);
    }

    // ---- epilogue straight from the accumulators: lane holds features
    // n..n+3 of token m (C^T fragments).  bf16: fragments ni, ni+1 packed to
    // 2 dwords each, then one v_permlane16_swap per dword pairs the 16-lane
    // rows so every lane holds 8 consecutive features (cdna_hip_programming.md
    // T21, the 16x16 form): one 16-B buffer store per fragment pair.  f32: one
    // 16-B store per fragment.
    constexpr int OB = (EPI == VGGT_EPI_F32 || EPI == VGGT_EPI_RESID_F32) ? 4 : 2;  // output element bytes
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((char*)ep.out + (int64_t)m0 * ep.ldo * OB), 0, (int)(min(M - m0, BMT) * ep.ldo * OB), 0x00020000);
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
    const int rg = lane >> 4;
    if constexpr (EPI == VGGT_EPI_RESID_F32) {
      // x += gamma * bf16(acc + bias) (LayerScale on the bf16 Linear output,
      // fp32 residual), mirrored into out2 (the kept-layer concat) -- with no
      // out2 the mirror stores go to an empty descriptor and are dropped, so
      // the store count stays NST
      const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(
          ep.out2 ? (void*)(ep.out2 + (int64_t)m0 * ep.ldo2) : ep.out, 0,
          ep.out2 ? (int)(min(M - m0, BMT) * ep.ldo2 * 4) : 0, 0x00020000);
#pragma unroll
      for (int ni = 0; ni < C::NI; ++ni) {
        const int nl = n0 + wn * C::WN + ni * 16 + 4 * rg;
        const f32x4 bv = *(const f32x4*)(bias_s + nl);
        const f32x4 gv = *(const f32x4*)(gam_s + nl);
#pragma unroll
        for (int mi = 0; mi < C::MI; ++mi) {
          const int ml = wm * C::HM + mi * 16 + (lane & 15);
          const f32x4 v = acc[ni][mi] + bv;
          f32x4 x = rx[ni][mi];
#pragma unroll
          for (int j = 0; j < 4; ++j) x[j] += gv[j] * round_bf(v[j]);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), ro, (ml * (int)ep.ldo + nl) * 4, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), r2, (ml * (int)ep.ldo2 + nl) * 4, 0, 0);
        }
      }
    } else if constexpr (EPI == VGGT_EPI_F32) {
#pragma unroll
      for (int ni = 0; ni < C::NI; ++ni) {
        const int nl = n0 + wn * C::WN + ni * 16 + 4 * rg;
        const f32x4 bv = *(const f32x4*)(bias_s + nl);
#pragma unroll
        for (int mi = 0; mi < C::MI; ++mi) {
          const int ml = wm * C::HM + mi * 16 + (lane & 15);
          f32x4 v = acc[ni][mi] + bv;
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = round_bf(v[j]);  // the reference's bf16 Linear output, widened
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ro, (ml * (int)ep.ldo + nl) * 4, 0, 0);
        }
      }
    } else if (EPI == EPI_QKNORM_D64 && (n0 + wn * C::WN) / ep.hd < 2) {
      // q or k head (this wave's 64 columns = one head): fp32 LayerNorm over the
      // head's 64 bf16 Linear outputs (lane: 16 of them, the rest in lanes
      // +-16 / +-32 of the same token) then RoPE-2D (y rotates features 0-31,
      // x 32-63; rotate_half partners e, e+16 are fragments ni, ni+1 of the
      // same lane), one bf16 rounding -- the arithmetic of headnorm_rope_kernel
      const int hb = n0 + wn * C::WN;
      const int region = hb / ep.hd;
      const bool norm = region ? ep.kw != nullptr : ep.qw != nullptr;
      f32x4 lw[C::NI], lb[C::NI], bv[C::NI];
#pragma unroll
      for (int ni = 0; ni < C::NI; ++ni) {
        const int e = ni * 16 + 4 * rg;
        lw[ni] = *(const f32x4*)(qkn_s + region * 128 + e);
        lb[ni] = *(const f32x4*)(qkn_s + region * 128 + 64 + e);
        bv[ni] = *(const f32x4*)(bias_s + hb + e);
      }
      const int ncol = (rg & 1) * 16 + (rg >> 1) * 8;
#pragma unroll
      for (int mi = 0; mi < C::MI; ++mi) {
        const int ml = wm * C::HM + mi * 16 + (lane & 15);
        f32x4 x[C::NI];
#pragma unroll
        for (int ni = 0; ni < C::NI; ++ni) {
          x[ni] = acc[ni][mi] + bv[ni];
#pragma unroll
          for (int j = 0; j < 4; ++j) x[ni][j] = round_bf(x[ni][j]);
        }
        if (norm) {
          float sm = 0.f;
#pragma unroll
          for (int ni = 0; ni < C::NI; ++ni) sm += (x[ni][0] + x[ni][1]) + (x[ni][2] + x[ni][3]);
          const float mean = rows4_sum(sm) * (1.f / 64);
          float q = 0.f;
#pragma unroll
          for (int ni = 0; ni < C::NI; ++ni)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float d = x[ni][j] - mean;
              q += d * d;
            }
          const float rstd = rsqrtf(rows4_sum(q) * (1.f / 64) + ep.eps);
#pragma unroll
          for (int ni = 0; ni < C::NI; ++ni)
#pragma unroll
            for (int j = 0; j < 4; ++j) x[ni][j] = (x[ni][j] - mean) * rstd * lw[ni][j] + lb[ni][j];
        }
        if (tab) {
          const int pr = (m0 + ml) % ep.period;
          const uint32_t pc = pos_s[pr];
#pragma unroll
          for (int h = 0; h < 2; ++h) {  // h 0: y rotates ni 0/1, h 1: x rotates ni 2/3
            const int pp = h ? (int)(pc >> 8) : (int)(pc & 255);
            const float* cp = cs_s + pp * 32 + 4 * rg;
            const float* sp = sn_s + pp * 32 + 4 * rg;
            const f32x4 c0 = *(const f32x4*)cp, c1 = *(const f32x4*)(cp + 16);
            const f32x4 s0 = *(const f32x4*)sp, s1 = *(const f32x4*)(sp + 16);
            const f32x4 a = x[2 * h], b = x[2 * h + 1];
            x[2 * h] = a * c0 - b * s0;
            x[2 * h + 1] = b * c1 + a * s1;
          }
        }
#pragma unroll
        for (int np = 0; np < C::NI; np += 2) {
          const uint32_t a0 = pack_bf2(x[np][0], x[np][1]), a1 = pack_bf2(x[np][2], x[np][3]);
          const uint32_t b0 = pack_bf2(x[np + 1][0], x[np + 1][1]), b1 = pack_bf2(x[np + 1][2], x[np + 1][3]);
          const auto s0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
          const u32x4 pk = {s0[0], s1[0], s0[1], s1[1]};
          __builtin_amdgcn_raw_buffer_store_b128(pk, ro, (ml * (int)ep.ldo + hb + np * 16 + ncol) * 2, 0, 0);
        }
      }
    } else {
      // after the swap, row group rg holds fragment ni + (rg & 1), features 8 * (rg >> 1) ..
      const int ncol = (rg & 1) * 16 + (rg >> 1) * 8;
      const __amdgpu_buffer_rsrc_t rpre = __builtin_amdgcn_make_buffer_rsrc(
          EPI == EPI_GELU_PRE ? (void*)((bf16_t*)(void*)ep.out2 + (int64_t)m0 * ep.ldo2) : ep.out, 0,
          EPI == EPI_GELU_PRE ? (int)(min(M - m0, BMT) * ep.ldo2 * 2) : 0, 0x00020000);
      (void)rpre;
#pragma unroll
      for (int np = 0; np < C::NI; np += 2) {
        const f32x4 bv0 = *(const f32x4*)(bias_s + n0 + wn * C::WN + np * 16 + 4 * rg);
        const f32x4 bv1 = *(const f32x4*)(bias_s + n0 + wn * C::WN + (np + 1) * 16 + 4 * rg);
        const int nl = n0 + wn * C::WN + np * 16 + ncol;
#pragma unroll
        for (int mi = 0; mi < C::MI; ++mi) {
          const int ml = wm * C::HM + mi * 16 + (lane & 15);
          const f32x4 v0 = acc[np][mi] + bv0, v1 = acc[np + 1][mi] + bv1;
          uint32_t a0 = pack_bf2(v0[0], v0[1]), a1 = pack_bf2(v0[2], v0[3]);
          uint32_t b0 = pack_bf2(v1[0], v1[1]), b1 = pack_bf2(v1[2], v1[3]);
          if constexpr (EPI == EPI_GELU_PRE) {
            // the pre-activation, same pairing and row as the activation store
            const auto p0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
            const auto p1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
            const u32x4 pp = {p0[0], p1[0], p0[1], p1[1]};
            __builtin_amdgcn_raw_buffer_store_b128(pp, rpre, (ml * (int)ep.ldo2 + nl) * 2, 0, 0);
          }
          if constexpr (GELU) {
            // GELU of the bf16 Linear output (autocast), from the LDS table of
            // torch's float32 GELU rounded to bf16 (gelu_lut.h): the four words'
            // eight lookups back to back, the out-of-table values (|x| < 2^-16 or
            // >= 64) re-done on a wave-uniform rare path
            uint32_t oor = 0;
            const uint32_t ra0 = a0, ra1 = a1, rb0 = b0, rb1 = b1;
            a0 = gelu2_clamped(ra0, lut_s, oor);
            a1 = gelu2_clamped(ra1, lut_s, oor);
            b0 = gelu2_clamped(rb0, lut_s, oor);
            b1 = gelu2_clamped(rb1, lut_s, oor);
            if (__builtin_amdgcn_ballot_w64(oor != 0) != 0) {
              a0 = gelu2_lut(ra0, lut_s);
              a1 = gelu2_lut(ra1, lut_s);
              b0 = gelu2_lut(rb0, lut_s);
              b1 = gelu2_lut(rb1, lut_s);
            }
          }
          // rows 1 <-> 0 and 3 <-> 2 of (a = fragment np, b = fragment np+1)
          const auto s0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
          const u32x4 pk = {s0[0], s1[0], s0[1], s1[1]};
          __builtin_amdgcn_raw_buffer_store_b128(pk, ro, (ml * (int)ep.ldo + nl) * 2, 0, 0);
        }
      }
    }
    if (!more) break;
    // own K-tile 0 of the next tile landed (K-tile 1 and the stores may still
    // be in flight), then everyone's
    if (nk > 1) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(LPS + NST) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(NST) : "memory");
    stores_out = true;
    tile = next;
    b0 = nb0;
  }
}

// LDS bytes of the persistent form: two K-tile buffers, the bias (and the
// LayerScale gamma), and for the fused q/k norm + RoPE epilogue its parameters
// and tables; 0 = does not fit
inline int ppp_lds_bytes(int epi, int bmt, int N, const Epi& ep) {
  int64_t b = 2 * ((int64_t)bmt * PBK * 2 + 256 * PBK * 2) + (int64_t)N * 4;
  if (epi == VGGT_EPI_RESID_F32) b += (int64_t)N * 4;
  if (epi == VGGT_EPI_GELU_BF16 || epi == EPI_GELU_PRE) b += (int64_t)GELU_LUT_N * 2 * 2;
  if (epi == EPI_QKNORM_D64) {
    b += 256 * 4;
    if (ep.rope_mode == VGGT_ROPE_2D) b += 2 * (int64_t)ep.tab_len * 32 * 4 + (((int64_t)ep.period * 2 + 15) & ~15);
  }
  return b <= PP_LDS_MAX ? (int)b : 0;
}

inline int cu_count() {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  return cus;
}
// CUs a launch on stream s can occupy: fewer than the device's for a stream
// created with a CU mask (vggt_set_stream_config) -- a persistent grid of
// one workgroup per CU would otherwise leave the masked-off CUs' share for a
// second, almost empty round
inline int cu_count(hipStream_t s) {
  const int n = vggt_stream_cu_count(s);
  return n > 0 ? n : cu_count();
}

// Row tile of the persistent form: 256, or 192 when whole rounds of 192-row
// tiles over the CUs cost at least 10% less (the N = 1024 projections at
// M = 21,984: 344 tiles = 1.34 rounds at 256 rows, 460 = 1.80 at 192); the
// residual epilogue always uses 192 rows (register budget: rx + acc)
inline int ppp_pick_bm(int epi, int M, int N, hipStream_t s) {
  if (epi == VGGT_EPI_RESID_F32) return 192;
  static int force = [] {  // VGGT_GEMM_BM=192/256: A/B override
    const char* e = getenv("VGGT_GEMM_BM");
    return e ? atoi(e) : 0;
  }();
  if (force == 192 || force == 256) return force;
  const int cus = cu_count(s);
  const long r256 = ((long)((M + 255) / 256) * (N / 256) + cus - 1) / cus;
  const long r192 = ((long)((M + 191) / 192) * (N / 256) + cus - 1) / cus;
  return r192 * 192 * 10 < r256 * 256 * 9 ? 192 : 256;
}

template <int EPI, int BMT, bool FK>
int launch_ppp_fk(const bf16_t* a, int64_t lda, const bf16_t* w, int64_t ldw, int M, int N, int K, const Epi& ep,
                  hipStream_t s) {
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)gemm_ppp_kernel<EPI, BMT, FK>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              PP_LDS_MAX);
    return true;
  }();
  (void)attr;
  const int lds = ppp_lds_bytes(EPI, BMT, N, ep);
  if (!lds) return VGGT_ERR_SHAPE;
  const int ntiles = ((M + BMT - 1) / BMT) * (N / 256);
  const int cus = cu_count(s);
  const int nwg = ntiles < cus ? ntiles : cus;
  // M-tiles per tile group (VGGT_GEMM_GM overrides; 0 = row-major).  Aggregator
  // step 98.45 -> 97.3-97.6 ms at 4 (8: 97.55, 16: 98.5); fc1 at K = 4096 625 ->
  // 591 us (r3y, r3z)
  static int sched = [] {
    const char* e = getenv("VGGT_GEMM_GM");
    const char* d = getenv("VGGT_GEMM_SPLITDMA");
    return (e ? atoi(e) & 255 : 4) | (d && !atoi(d) ? 0 : 256);
  }();
  gemm_ppp_kernel<EPI, BMT, FK><<<nwg, PNT, lds, s>>>(a, lda, w, ldw, M, N, K, ep, sched);
  return VGGT_OK;
}

template <int EPI, int BMT>
int launch_ppp_bm(const bf16_t* a, int64_t lda, const bf16_t* w, int64_t ldw, int M, int N, int K, const Epi& ep,
                  hipStream_t s) {
  // Whole-K-tile READ / MATH segments (VGGT_GEMM_FULLK bits: 1 bf16 / GELU / f32,
  // 2 qkv, 4 residual; default 5).  In the model (same box, r3x kernel traces):
  // fc2 + residual 206.6 -> 199.9 us, fc1 + GELU 196.3 -> 193.5 us.  The fused qkv
  // form keeps the half-K segments: with both halves' fragments live its q/k-norm +
  // RoPE epilogue spills (256 VGPRs + scratch), +2 ms per step.
  static int fk = [] {
    const char* e = getenv("VGGT_GEMM_FULLK");
    return e ? atoi(e) : 5;
  }();
  // (GELU + pre-activation keeps half-K segments: whole-K ones spill at 256 rows)
  const int bit = EPI == EPI_QKNORM_D64 ? 2 : EPI == VGGT_EPI_RESID_F32 ? 4 : EPI == EPI_GELU_PRE ? 8 : 1;
  if (fk & bit) return launch_ppp_fk<EPI, BMT, true>(a, lda, w, ldw, M, N, K, ep, s);
  return launch_ppp_fk<EPI, BMT, false>(a, lda, w, ldw, M, N, K, ep, s);
}

template <int EPI>
int launch_ppp(const bf16_t* a, int64_t lda, const bf16_t* w, int64_t ldw, int M, int N, int K, const Epi& ep,
               hipStream_t s) {
  if constexpr (EPI == VGGT_EPI_RESID_F32) {
    // (128-row residual tiles measured slower: proj 81.7 vs 67.4 us on the
    // 128x128 form, aggregator step 104.9 vs 101.3 ms, r3r)
    return launch_ppp_bm<EPI, 192>(a, lda, w, ldw, M, N, K, ep, s);
  } else {
    if (ppp_pick_bm(EPI, M, N, s) == 192) return launch_ppp_bm<EPI, 192>(a, lda, w, ldw, M, N, K, ep, s);
    return launch_ppp_bm<EPI, 256>(a, lda, w, ldw, M, N, K, ep, s);
  }
}

// Ping-pong tile width for an N-wide output: the BN whose whole rounds of
// 256-row tiles over the CUs cost least (per-tile time ~ BN), larger BN on a
// tie; 192 only where the epilogue allows it.
inline int pp_pick_bn(int M, int N, bool allow192) {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  const int tm = (M + PBM - 1) / PBM;
  int best = 0;
  long best_cost = 0;
  for (int bn : {256, 192, 128}) {
    if (N % bn || (bn == 192 && !allow192)) continue;
    const long rounds = ((long)tm * (N / bn) + cus - 1) / cus;
    const long cost = rounds * bn;
    if (best == 0 || cost < best_cost) {
      best = bn;
      best_cost = cost;
    }
  }
  return best;
}

// Auto width for the ping-pong form: 256-wide tiles where they fill at least
// two rounds of CUs (measured best on the 21,984-row chunk shapes), else the
// quantisation-aware pick.  Short M (the 154x518 sequence chunks, 6,592 rows)
// would leave a partial last round almost empty: qkv N = 3072 at 256 wide is
// 312 tiles = 1.22 rounds, at 192 wide 416 tiles = 1.63.
inline int pp_auto_bn(int M, int N, bool allow192) {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  const long tiles256 = (long)((M + PBM - 1) / PBM) * (N / 256);
  if (N % 256 == 0 && tiles256 >= 2l * cus) return 256;
  return pp_pick_bn(M, N, allow192);
}

}  // namespace

namespace {
int gemm_impl(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int M, int N, int K, int epi,
              void* out, int64_t ldo, const float* gamma, float* out2, int64_t ldo2, void* stream, int force = -1) {
  if (M <= 0 || N <= 0 || K <= 0 || N % 128 || K % 32) return VGGT_ERR_SHAPE;
  if ((lda % 8) || (ldw % 8) || ((uintptr_t)A & 15) || ((uintptr_t)W & 15) || ((uintptr_t)bias & 15))
    return VGGT_ERR_ALIGN;
  if (epi == VGGT_EPI_RESID_F32 && (!gamma || ((uintptr_t)gamma & 15) || (out2 && (ldo2 % 4))))
    return VGGT_ERR_ALIGN;
  if (epi == VGGT_EPI_GELU_BF16 && out2 && ((ldo2 % 8) || ((uintptr_t)out2 & 15))) return VGGT_ERR_ALIGN;
  if (epi != VGGT_EPI_RESID_F32 && epi != VGGT_EPI_GELU_BF16) out2 = nullptr;
  if ((epi == VGGT_EPI_BF16 || epi == VGGT_EPI_GELU_BF16) ? (ldo % 8) : (ldo % 4)) return VGGT_ERR_ALIGN;
  Epi ep{bias, out, ldo, gamma, out2, ldo2};
  hipStream_t s = (hipStream_t)stream;
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* w = (const bf16_t*)W;
  // Tile choice (vggt_tune VGGT_TUNE_GEMM_TILE): 0 the 128x128 form, 1 the
  // 256x256 ring, 2 the 256x128 ring.  Auto (-1): the 256x256 ring for the MLP
  // up-projection (N >= 4096: fc1, 256 vs 278 us in the aggregator run r1i), the
  // 128x128 form elsewhere (qkv N = 3072: 154 vs 165 us; N = 1024 proj / fc2,
  // where 256x256 tiles leave the last of only ~1.3 rounds of workgroups idle).
  // Auto (-1), from the in-model kernel tables (profiles/r1s_*): the ping-pong
  // form with 256-wide tiles for the wide bf16-output projections (fc1 with
  // GELU 234 vs 240 us ring, plain qkv 146 vs 191 us); the 128x128 form (two
  // workgroups per CU, so one's fp32 residual read-modify-write overlaps the
  // other's MFMAs) for the LayerScale+residual projections (proj 83 vs 90 us,
  // fc2 225 vs 234 us) and for small M.
  int mode = force >= 0 ? force : g_vggt_gemm_tile;
  if (mode < 0)
    mode = (M >= 4096 && K % PBK == 0 && N % 256 == 0 && N >= 2048 && epi != VGGT_EPI_RESID_F32) ? 7 : 0;
  // VGGT_GEMM_MID=1 (A/B): the 128-wide ping-pong form for the narrow (N <= 1024)
  // LayerScale-residual / plain projections between 4,096 and 16,383 rows (the
  // alignment head's 6,608-row proj / fc2: fc2 68.9 -> 64.0 us, gemmbench r10e)
  static const int mid = getenv("VGGT_GEMM_MID") ? atoi(getenv("VGGT_GEMM_MID")) : 0;
  if (g_vggt_gemm_tile < 0 && mid && mode == 0 && M >= 4096 && M < 16384 && N <= 1024 && N % 128 == 0 &&
      K % PBK == 0 && (epi == VGGT_EPI_RESID_F32 || (mid & 2)))
    mode = 6;
  // auto: the persistent ping-pong form where 256x256 tiles fill several
  // rounds of CUs (the 16x518^2 chunk: fc1 + GELU 217 -> 204 us, plain qkv
  // shape 159 -> 139 us, scripts/gemmbench.py r3i); it falls back to mode 7
  // for the epilogues it does not cover
  // (GELU from M = 4,096: the 154x518 sequence chunk's fc1, 6,592 rows: 72.9 -> 64.8 us, r3w; plain bf16 stays on
  // the one-shot forms below 16,384 rows: qkv shape 49-55 vs 55 us)
  if (g_vggt_gemm_tile < 0 && mode == 7 && (M >= 16384 || epi == VGGT_EPI_GELU_BF16) && N <= PP_MAXN &&
      (persist_policy(s) & 1))
    mode = 9;
  // ... and the narrow (N = 1024) bf16 / f32-output GEMMs of the training
  // recompute and backward (dX = dY W): 192-row persistent tiles instead of
  // 128x128 at 22,000 rows: K = 4096 177 -> 144 us, K = 3072 132 -> 112 us,
  // K = 1024 51.5 -> 45.4 us (gemmbench r3tr)
  if (g_vggt_gemm_tile < 0 && mode == 0 && epi != VGGT_EPI_RESID_F32 && M >= 16384 && N % 256 == 0 &&
      N <= PP_MAXN && K % PBK == 0 && (persist_policy(s) & 1))
    mode = 9;
  // the LayerScale-residual fc2 (N = 1024, K = 4096) on 192-row persistent tiles:
  // 216 -> 201 us, aggregator step 104.0 -> 102.3 ms (same box, r3o); the
  // K = 1024 proj stays on the 128x128 form (76 vs 80 us)
  if (g_vggt_gemm_tile < 0 && epi == VGGT_EPI_RESID_F32 && M >= 16384 && N % 256 == 0 && N <= PP_MAXN &&
      K % PBK == 0 && K >= 2048 && (persist_policy(s) & 4))
    mode = 9;
  if (mode >= 3 && mode <= 7 && K % PBK) mode = 2;    // the ping-pong form steps K by 64
  if (mode == 0 && K % BK) mode = 2;     // the 128x128 form steps K by 64
  if (mode == 1 && N % 256) mode = 2;
  // per-lane 32-bit DMA offsets span one 256-row panel
  if (mode != 0 && (int64_t)RBM * (lda > ldw ? lda : ldw) * 2 >= (1ll << 31)) return VGGT_ERR_SHAPE;
  if (mode == 9 && (N % 256 || N > PP_MAXN || K % PBK ||
                    (int64_t)PBM * (ldo > ldo2 ? ldo : ldo2) * 4 >= (1ll << 31)))
    mode = K % PBK ? 2 : epi == VGGT_EPI_RESID_F32 ? 0 : 7;  // the persistent form: N % 256 == 0, N <= 4096
  // Round balance (knob 10): the persistent form hands tile t to workgroup t mod CUs, so
  // 1,376 fc1 tiles (86 x 16, M = 21,984) take 6 tile-times on 256 CUs for 5.375 tiles
  // of work.  With VGGT_GEMM_BALANCE=1 the whole rounds of row panels run persistent and
  // the remaining rows on the 128x128 form (finer tiles, two per CU); rows are
  // independent and both forms accumulate K in the same order: bitwise equal.
  if (mode == 9 && force < 0 && g_vggt_gemm_balance) {
    const int bm = epi == VGGT_EPI_RESID_F32 ? 192 : ppp_pick_bm(epi == VGGT_EPI_GELU_BF16 && out2 ? EPI_GELU_PRE : epi, M, N, s);
    const int tpr = N / 256, cus = cu_count(s);
    const int64_t ntiles = (int64_t)((M + bm - 1) / bm) * tpr;
    const int64_t full = ntiles / cus, rem = ntiles % cus;
    const int m1 = (int)((full * cus / tpr) * bm);
    if (full >= 1 && rem > 0 && rem * 10 <= (int64_t)cus * 6 && m1 > 0 && m1 < M && K % BK == 0) {
      int rc = gemm_impl(A, lda, W, ldw, bias, m1, N, K, epi, out, ldo, gamma, out2, ldo2, stream, 9);
      if (rc != VGGT_OK) return rc;
      const size_t osz = (epi == VGGT_EPI_BF16 || epi == VGGT_EPI_GELU_BF16) ? 2 : 4;
      const size_t o2sz = epi == VGGT_EPI_GELU_BF16 ? 2 : 4;
      return gemm_impl((const bf16_t*)A + (int64_t)m1 * lda, lda, W, ldw, bias, M - m1, N, K, epi,
                       (char*)out + (size_t)m1 * ldo * osz, ldo, gamma,
                       out2 ? (float*)((char*)out2 + (size_t)m1 * ldo2 * o2sz) : nullptr, ldo2, stream, 0);
    }
  }
  if (mode == 9) {
    int rc;
    switch (epi) {
      case VGGT_EPI_BF16: rc = launch_ppp<VGGT_EPI_BF16>(a, lda, w, ldw, M, N, K, ep, s); break;
      case VGGT_EPI_GELU_BF16:
        rc = out2 ? launch_ppp<EPI_GELU_PRE>(a, lda, w, ldw, M, N, K, ep, s)
                  : launch_ppp<VGGT_EPI_GELU_BF16>(a, lda, w, ldw, M, N, K, ep, s);
        break;
      case VGGT_EPI_RESID_F32: rc = launch_ppp<VGGT_EPI_RESID_F32>(a, lda, w, ldw, M, N, K, ep, s); break;
      case VGGT_EPI_F32: rc = launch_ppp<VGGT_EPI_F32>(a, lda, w, ldw, M, N, K, ep, s); break;
      default: return VGGT_ERR_UNSUPPORTED;
    }
    if (rc != VGGT_OK) return rc;
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if (mode == 8) {
    switch (epi) {
      case VGGT_EPI_BF16: launch_two<VGGT_EPI_BF16>(a, lda, w, ldw, M, N, K, ep, s); break;
      case VGGT_EPI_GELU_BF16: launch_two<VGGT_EPI_GELU_BF16>(a, lda, w, ldw, M, N, K, ep, s); break;
      case VGGT_EPI_RESID_F32: launch_two<VGGT_EPI_RESID_F32>(a, lda, w, ldw, M, N, K, ep, s); break;
      case VGGT_EPI_F32: launch_two<VGGT_EPI_F32>(a, lda, w, ldw, M, N, K, ep, s); break;
      default: return VGGT_ERR_UNSUPPORTED;
    }
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if (mode >= 3) {
    int bn = mode == 4 ? 256 : mode == 5 ? 192 : mode == 6 ? 128 : mode == 7 ? pp_auto_bn(M, N, true) : pp_pick_bn(M, N, true);
    if (bn == 0 || N % bn) bn = pp_pick_bn(M, N, true);
    if (bn == 0) return VGGT_ERR_SHAPE;
#define VGGT_PP(E)                                                    \
  (bn == 256   ? launch_pp<E, 256>(a, lda, w, ldw, M, N, K, ep, s)   \
   : bn == 192 ? launch_pp<E, 192>(a, lda, w, ldw, M, N, K, ep, s)   \
               : launch_pp<E, 128>(a, lda, w, ldw, M, N, K, ep, s))
    switch (epi) {
      case VGGT_EPI_BF16: VGGT_PP(VGGT_EPI_BF16); break;
      case VGGT_EPI_GELU_BF16: VGGT_PP(VGGT_EPI_GELU_BF16); break;
      case VGGT_EPI_RESID_F32: VGGT_PP(VGGT_EPI_RESID_F32); break;
      case VGGT_EPI_F32: VGGT_PP(VGGT_EPI_F32); break;
      default: return VGGT_ERR_UNSUPPORTED;
    }
#undef VGGT_PP
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if (mode == 1) {
    switch (epi) {
      case VGGT_EPI_BF16: launch_ring<VGGT_EPI_BF16, 256>(a, lda, w, ldw, M, N, K, ep, s); break;
      case VGGT_EPI_GELU_BF16: launch_ring<VGGT_EPI_GELU_BF16, 256>(a, lda, w, ldw, M, N, K, ep, s); break;
      case VGGT_EPI_RESID_F32: launch_ring<VGGT_EPI_RESID_F32, 256>(a, lda, w, ldw, M, N, K, ep, s); break;
      case VGGT_EPI_F32: launch_ring<VGGT_EPI_F32, 256>(a, lda, w, ldw, M, N, K, ep, s); break;
      default: return VGGT_ERR_UNSUPPORTED;
    }
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if (mode == 2) {
    switch (epi) {
      case VGGT_EPI_BF16: launch_ring<VGGT_EPI_BF16, 128>(a, lda, w, ldw, M, N, K, ep, s); break;
      case VGGT_EPI_GELU_BF16: launch_ring<VGGT_EPI_GELU_BF16, 128>(a, lda, w, ldw, M, N, K, ep, s); break;
      case VGGT_EPI_RESID_F32: launch_ring<VGGT_EPI_RESID_F32, 128>(a, lda, w, ldw, M, N, K, ep, s); break;
      case VGGT_EPI_F32: launch_ring<VGGT_EPI_F32, 128>(a, lda, w, ldw, M, N, K, ep, s); break;
      default: return VGGT_ERR_UNSUPPORTED;
    }
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  const int nwg = ((M + BM - 1) / BM) * (N / BN);
  switch (epi) {
    case VGGT_EPI_BF16: gemm_bf16_kernel<VGGT_EPI_BF16><<<nwg, NT, 0, s>>>(a, lda, w, ldw, M, N, K, ep); break;
    case VGGT_EPI_GELU_BF16: gemm_bf16_kernel<VGGT_EPI_GELU_BF16><<<nwg, NT, 0, s>>>(a, lda, w, ldw, M, N, K, ep); break;
    case VGGT_EPI_RESID_F32: gemm_bf16_kernel<VGGT_EPI_RESID_F32><<<nwg, NT, 0, s>>>(a, lda, w, ldw, M, N, K, ep); break;
    case VGGT_EPI_F32: gemm_bf16_kernel<VGGT_EPI_F32><<<nwg, NT, 0, s>>>(a, lda, w, ldw, M, N, K, ep); break;
    default: return VGGT_ERR_UNSUPPORTED;
  }
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}
}  // namespace

extern "C" int vggt_gemm_bf16(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int M, int N,
                              int K, int epi, void* out, int64_t ldo, const float* gamma, float* out2, int64_t ldo2,
                              void* stream) {
  return gemm_impl(A, lda, W, ldw, bias, M, N, K, epi, out, ldo, gamma, epi == VGGT_EPI_RESID_F32 ? out2 : nullptr,
                   ldo2, stream);
}

extern "C" int vggt_gemm_bf16_gelu_pre(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int M,
                                       int N, int K, void* out, int64_t ldo, void* pre, int64_t ldp, void* stream) {
  return gemm_impl(A, lda, W, ldw, bias, M, N, K, VGGT_EPI_GELU_BF16, out, ldo, nullptr, (float*)pre, ldp, stream);
}

namespace {
// the fused-epilogue GEMM of vggt_gemm_qkv (N = 3 hd, nreg = 2) and vggt_gemm_headnorm
// (N = hd or 2 hd, nreg = 1)
int qkv_impl(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int M, int H, int D, int K,
             void* out, int64_t ldo, const float* qw, const float* qb, const float* kw, const float* kb, float eps,
             int rope_mode, const int32_t* pos, int period, const float* cos_tab, const float* sin_tab, int tab_len,
             void* stream, int N, int nreg) {
  const int hd = H * D;
  if (M <= 0 || H <= 0 || K <= 0 || K % 32 || (D != 64 && D != 128) || hd % 128) return VGGT_ERR_SHAPE;
  if (nreg == 2 && (qw == nullptr) != (kw == nullptr)) return VGGT_ERR_UNSUPPORTED;
  if (rope_mode != VGGT_ROPE_NONE && rope_mode != VGGT_ROPE_2D && rope_mode != VGGT_ROPE_1D) return VGGT_ERR_UNSUPPORTED;
  if (rope_mode != VGGT_ROPE_NONE && (!pos || !cos_tab || !sin_tab || period <= 0 || tab_len <= 0))
    return VGGT_ERR_SHAPE;
  if ((lda % 8) || (ldw % 8) || (ldo % 8) || ((uintptr_t)A & 15) || ((uintptr_t)W & 15) || ((uintptr_t)bias & 15) ||
      ((uintptr_t)out & 15) || (rope_mode != VGGT_ROPE_NONE && (((uintptr_t)cos_tab | (uintptr_t)sin_tab) & 15)))
    return VGGT_ERR_ALIGN;
  Epi ep{bias, out, ldo, nullptr, nullptr, 0, qw, qb, kw, kb, eps, hd, rope_mode, period, tab_len, pos, cos_tab,
         sin_tab, nreg};
  hipStream_t s = (hipStream_t)stream;
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* w = (const bf16_t*)W;
  // auto: the 256-wide ping-pong form on long M (fused qkv 179 vs 239 us for the
  // 128x128 form, r1s), the 128x128 form otherwise
  int mode = g_vggt_gemm_tile;
  // vggt_gemm_headnorm only: VGGT_HEADNORM_TILE picks its form (A/B)
  static const int hn_tile = getenv("VGGT_HEADNORM_TILE") ? atoi(getenv("VGGT_HEADNORM_TILE")) : -1;
  if (nreg == 1 && mode < 0) mode = hn_tile;
  if (mode < 0) mode = (M >= 4096 && K % PBK == 0) ? (N % 256 == 0 ? 7 : 6) : 0;
  if (mode >= 3 && mode <= 7 && K % PBK) mode = 2;
  if (mode == 0 && K % BK) mode = 2;
  if (mode == 1 && hd % 256) mode = 2;
  if (mode != 0 && (int64_t)RBM * (lda > ldw ? lda : ldw) * 2 >= (1ll << 31)) return VGGT_ERR_SHAPE;
  // auto: the persistent form on the chunk shapes (D = 64 heads, RoPE-2D or none)
  // (fused qkv of the 154x518 sequence chunk, 6,592 rows: 68.9 -> 53.6 us, r3w)
  if (g_vggt_gemm_tile < 0 && mode == 7 && M >= 4096 && (persist_policy(s) & 2)) mode = 9;
  if (mode == 9) {
    bool ok = D == 64 && nreg == 2 && N % 256 == 0 && N <= PP_MAXN && K % PBK == 0 && rope_mode != VGGT_ROPE_1D &&
              (int64_t)PBM * ldo * 2 < (1ll << 31) && ppp_lds_bytes(EPI_QKNORM_D64, ppp_pick_bm(EPI_QKNORM_D64, M, N, s), N, ep) > 0;
    if (ok && rope_mode == VGGT_ROPE_2D) {
      // positions are staged as bytes; tables of at most 256 positions
      ok = tab_len <= 256;
    }
    if (ok) {
      launch_ppp<EPI_QKNORM_D64>(a, lda, w, ldw, M, N, K, ep, s);
      HIP_LAUNCH_CHECK();
      return VGGT_OK;
    }
    mode = K % PBK ? 2 : 7;
  }
  if (mode == 8) {
    if (D == 64) launch_two<EPI_QKNORM_D64>(a, lda, w, ldw, M, N, K, ep, s);
    else launch_two<EPI_QKNORM_D128>(a, lda, w, ldw, M, N, K, ep, s);
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if (mode >= 3) {
    // 192-wide tiles only with 64-wide heads (the norm's lane groups stay aligned)
    int bn = mode == 4 ? 256 : mode == 5 ? 192 : mode == 6 ? 128 : mode == 7 ? pp_auto_bn(M, N, D == 64) : pp_pick_bn(M, N, D == 64);
    if (bn == 0 || N % bn || (bn == 192 && D != 64)) bn = pp_pick_bn(M, N, D == 64);
    if (bn == 0) return VGGT_ERR_SHAPE;
    if (D == 64) {
      if (bn == 256) launch_pp<EPI_QKNORM_D64, 256>(a, lda, w, ldw, M, N, K, ep, s);
      else if (bn == 192) launch_pp<EPI_QKNORM_D64, 192>(a, lda, w, ldw, M, N, K, ep, s);
      else launch_pp<EPI_QKNORM_D64, 128>(a, lda, w, ldw, M, N, K, ep, s);
    } else {
      if (bn == 256) launch_pp<EPI_QKNORM_D128, 256>(a, lda, w, ldw, M, N, K, ep, s);
      else launch_pp<EPI_QKNORM_D128, 128>(a, lda, w, ldw, M, N, K, ep, s);
    }
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if (mode == 0) {
    const int nwg = ((M + BM - 1) / BM) * (N / BN);
    if (D == 64) gemm_bf16_kernel<EPI_QKNORM_D64><<<nwg, NT, 0, s>>>(a, lda, w, ldw, M, N, K, ep);
    else gemm_bf16_kernel<EPI_QKNORM_D128><<<nwg, NT, 0, s>>>(a, lda, w, ldw, M, N, K, ep);
  } else if (mode == 1) {
    if (D == 64) launch_ring<EPI_QKNORM_D64, 256>(a, lda, w, ldw, M, N, K, ep, s);
    else launch_ring<EPI_QKNORM_D128, 256>(a, lda, w, ldw, M, N, K, ep, s);
  } else {
    if (D == 64) launch_ring<EPI_QKNORM_D64, 128>(a, lda, w, ldw, M, N, K, ep, s);
    else launch_ring<EPI_QKNORM_D128, 128>(a, lda, w, ldw, M, N, K, ep, s);
  }
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}
}  // namespace

extern "C" int vggt_gemm_qkv(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int M, int H,
                             int D, int K, void* out, int64_t ldo, const float* qw, const float* qb, const float* kw,
                             const float* kb, float eps, int rope_mode, const int32_t* pos, int period,
                             const float* cos_tab, const float* sin_tab, int tab_len, void* stream) {
  return qkv_impl(A, lda, W, ldw, bias, M, H, D, K, out, ldo, qw, qb, kw, kb, eps, rope_mode, pos, period, cos_tab,
                  sin_tab, tab_len, stream, 3 * H * D, 2);
}

extern "C" int vggt_gemm_headnorm(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int M,
                                  int N, int H, int D, int K, void* out, int64_t ldo, const float* nw, const float* nb,
                                  float eps, int rope_mode, const int32_t* pos, int period, const float* cos_tab,
                                  const float* sin_tab, int tab_len, void* stream) {
  if (N != H * D && N != 2 * H * D) return VGGT_ERR_SHAPE;
  return qkv_impl(A, lda, W, ldw, bias, M, H, D, K, out, ldo, nw, nb, nullptr, nullptr, eps, rope_mode, pos, period,
                  cos_tab, sin_tab, tab_len, stream, N, 1);
}
