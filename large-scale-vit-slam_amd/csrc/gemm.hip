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
#include "common.h"

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
};

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

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * BK);
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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

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

  // ---- epilogue 2: coalesced row write-out ----
  const int ch = threadIdx.x & 15;  // 16-B chunk (8 features) within the 128-wide row
  const int n = n0 + ch * 8;
  float g[8];
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
  for (int it = 0; it < BM / 16; ++it) {
    const int ml = it * 16 + (threadIdx.x >> 4);
    const int m = m0 + ml;
    if (m >= M) continue;
    const uint4 cv = *(const uint4*)(Cs + ml * CROW + ch * 16);
    if constexpr (EPI == VGGT_EPI_BF16) {
      *(uint4*)((bf16_t*)ep.out + (int64_t)m * ep.ldo + n) = cv;
    } else {
      const uint32_t w4[4] = {cv.x, cv.y, cv.z, cv.w};
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[2 * j] = bf2f((bf16_t)(w4[j] & 0xffff));
        v[2 * j + 1] = bf2f((bf16_t)(w4[j] >> 16));
      }
      if constexpr (EPI == VGGT_EPI_GELU_BF16) {
        uint4 o;
        o.x = pack_bf2(gelu_erf(v[0]), gelu_erf(v[1]));
        o.y = pack_bf2(gelu_erf(v[2]), gelu_erf(v[3]));
        o.z = pack_bf2(gelu_erf(v[4]), gelu_erf(v[5]));
        o.w = pack_bf2(gelu_erf(v[6]), gelu_erf(v[7]));
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

}  // namespace

extern "C" int vggt_gemm_bf16(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int M, int N,
                              int K, int epi, void* out, int64_t ldo, const float* gamma, float* out2, int64_t ldo2,
                              void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || N % BN || K % BK) return VGGT_ERR_SHAPE;
  if ((lda % 8) || (ldw % 8) || ((uintptr_t)A & 15) || ((uintptr_t)W & 15) || ((uintptr_t)bias & 15))
    return VGGT_ERR_ALIGN;
  if (epi == VGGT_EPI_RESID_F32 && (!gamma || ((uintptr_t)gamma & 15) || (out2 && (ldo2 % 4))))
    return VGGT_ERR_ALIGN;
  if ((epi == VGGT_EPI_BF16 || epi == VGGT_EPI_GELU_BF16) ? (ldo % 8) : (ldo % 4)) return VGGT_ERR_ALIGN;
  Epi ep{bias, out, ldo, gamma, out2, ldo2};
  const int nwg = ((M + BM - 1) / BM) * (N / BN);
  hipStream_t s = (hipStream_t)stream;
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* w = (const bf16_t*)W;
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
