// Flash-attention forward for the VGGT hot path (include/vggt_mi355x.h:
// vggt_attention_fwd): softmax(Q K^T * scale) V, bf16 in/out, fp32 online
// softmax, head_dim D in {64, 128}, non-causal, ragged nk (masked last tile).
//
// gfx950 design:
//  * Workgroup = 4 waves = 128 query rows (32 per wave); KV tiles of 64 keys
//    staged global->LDS by LDS-DMA (global_load_lds_dwordx4), double-buffered.
//  * "Swapped" QK^T: each wave computes S^T = K . Q^T with
//    v_mfma_f32_32x32x16_bf16, so a lane owns one query row (lane & 31) and
//    the two lanes l, l+32 hold all 64 keys of the tile -> the row max needs a
//    single v_permlane32_swap, the row sum stays lane-partial until the end.
//  * The S^T accumulator, rounded to bf16, is directly the B operand of
//    O^T = V^T . P^T (no LDS round trip for P); the V^T A-operand comes from
//    ds_read_b64_tr_b16 transposed reads of the row-major V tile.
//  * LDS images are XOR-swizzled on the DMA source address so that the K
//    ds_read_b128 fragment reads and the V transposed reads are bank-conflict
//    free (chunk ^ ((key>>1)&7) / chunk ^ (((key>>1)&1)<<2) at D=64,
//    chunk ^ (key&15) / chunk ^ ((key&3)<<2) at D=128).
//  * XCD-aware block order: consecutive query blocks of one (batch, head)
//    share an XCD so its K/V stream is served from one L2.
#include <math.h>

#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

// LDS-DMA of 16 B per lane into the wave-uniform LDS address `lds` (+lane*16).
// Issued as inline asm so hipcc does not treat the pending LDS write as
// aliasing the other buffer's reads (it otherwise drains vmcnt(0) before the
// first transposed read of every tile); completion is waited for by the
// explicit vmcnt(0) + barrier at the end of each tile.
__device__ __forceinline__ void glds16(const void* g, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds)
               : "memory");
}

constexpr int BQ = 128, BKV = 64, NT = 256;

struct AttnArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* o;
  int64_t ldq, ldk, ldv, ldo;
  int64_t qbs, kbs, vbs, obs;
  int batch, heads, nq, nk;
  float c;  // scale * log2(e)
};

template <int D>
__device__ __forceinline__ int k_swz(int row, int chunk) {
  if constexpr (D == 64) return chunk ^ ((row >> 1) & 7);
  else return chunk ^ (row & 15);
}
template <int D>
__device__ __forceinline__ int v_swz(int row, int chunk) {
  if constexpr (D == 64) return chunk ^ (((row >> 1) & 1) << 2);
  else return chunk ^ ((row & 3) << 2);
}

template <int D>
__global__ __launch_bounds__(NT, 2) void attn_fwd_kernel(AttnArgs a) {
  constexpr int ROWB = D * 2;              // bytes per K/V row in LDS
  constexpr int TILEB = BKV * ROWB;        // bytes per K (or V) tile
  constexpr int RPI = 1024 / ROWB;         // rows per 1-KiB DMA instruction
  constexpr int CPR = ROWB / 16;           // 16-B chunks per row
  constexpr int IPW = TILEB / 1024 / 4;    // DMA instructions per wave per operand
  constexpr int NKS = D / 16;              // k-steps of the QK^T MFMA
  constexpr int NDB = D / 32;              // 32-row output blocks of O^T
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILEB];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hl = lane >> 5;  // lane half
  const int nqb = (a.nq + BQ - 1) / BQ;
  const int bid = xcd_remap(blockIdx.x, nqb * a.heads * a.batch);
  const int qb = bid % nqb;
  const int bh = bid / nqb;
  const int h = bh % a.heads;
  const int b = bh / a.heads;

  const bf16_t* qp = a.q + (int64_t)b * a.qbs * a.ldq + h * D;
  const bf16_t* kp = a.k + (int64_t)b * a.kbs * a.ldk + h * D;
  const bf16_t* vp = a.v + (int64_t)b * a.vbs * a.ldv + h * D;

  // Q fragments = B operand of S^T = K Q^T: Q[q][16ks + 8*hl + j]
  const int qrow = qb * BQ + wave * 32 + (lane & 31);
  const int qr = min(qrow, a.nq - 1);
  bf16x8 qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) qf[ks] = *(const bf16x8*)(qp + (int64_t)qr * a.ldq + ks * 16 + 8 * hl);
  // Retire the Q loads here: hipcc would otherwise place their vmcnt wait at
  // the first use inside the tile loop, where it also drains the (uncounted)
  // LDS-DMA prefetch of the next tile.
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) asm volatile("" : "+v"(qf[ks]));

  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));
  auto stage = [&](int buf, int kv0) {
    char* Ks = smem + buf * 2 * TILEB;
    char* Vs = Ks + TILEB;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int inst = wave * IPW + i;
      const int row = inst * RPI + lane / CPR;
      const int cp = lane % CPR;
      const int src = min(kv0 + row, a.nk - 1);
      glds16(kp + (int64_t)src * a.ldk + k_swz<D>(row, cp) * 8, lds_base + (uint32_t)(Ks - smem) + inst * 1024);
      glds16(vp + (int64_t)src * a.ldv + v_swz<D>(row, cp) * 8, lds_base + (uint32_t)(Vs - smem) + inst * 1024);
    }
  };

  f32x16 o[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) o[i] = f32x16{};
  float m_run = -INFINITY, l_run = 0.f;

  const int nt = (a.nk + BKV - 1) / BKV;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) stage(cur ^ 1, (t + 1) * BKV);
    const char* Ks = smem + cur * 2 * TILEB;
    const char* Vs = Ks + TILEB;

    // ---- S^T = K . Q^T for two 32-key blocks ----
    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      s[kb] = f32x16{};
      const int key = kb * 32 + (lane & 31);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 kf = *(const bf16x8*)(Ks + key * ROWB + (k_swz<D>(key, 2 * ks + hl) << 4));
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[kb], 0, 0, 0);
      }
    }
    const int kv0 = t * BKV;
    if (kv0 + BKV > a.nk) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kv0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (key >= a.nk) s[kb][r] = -INFINITY;
        }
    }
    // ---- online softmax (log2 domain) ----
    float mx = s[0][0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s[0][r]);
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[1][r]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    const float m_new = fmaxf(m_run, mx * a.c);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    m_run = m_new;
    float rs = 0.f;
    bf16x8 pf[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[kb][8 * ss + j], a.c, -m_new));
          rs += p;
          pf[kb][ss][j] = (__bf16)p;
        }
      }
    l_run = l_run * alpha + rs;
#pragma unroll
    for (int db = 0; db < NDB; ++db) o[db] *= alpha;

    // ---- O^T += V^T . P^T ----
    const int g = (lane >> 4) & 1;
    const int qq = (lane >> 2) & 3;
    const int pp = lane & 3;
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      const int col = db * 32 + 16 * g + 4 * pp;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const int r0 = kb * 32 + 16 * ss + 4 * hl + qq;
          const int r1 = r0 + 8;
          const char* a0 = Vs + r0 * ROWB + (v_swz<D>(r0, col >> 3) << 4) + (col & 7) * 2;
          const char* a1 = Vs + r1 * ROWB + (v_swz<D>(r1, col >> 3) << 4) + (col & 7) * 2;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a1);
          const bf16x8 vf = __builtin_bit_cast(bf16x8, (s16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kb][ss], o[db], 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: normalise, O[q][d] bf16 ----
  {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_run), __float_as_uint(l_run), false, false);
    l_run = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  const float inv = 1.f / l_run;
  if (qrow < a.nq) {
    bf16_t* op = a.o + ((int64_t)b * a.obs + qrow) * a.ldo + h * D;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        uint2 pk;
        pk.x = pack_bf2(o[db][4 * gq] * inv, o[db][4 * gq + 1] * inv);
        pk.y = pack_bf2(o[db][4 * gq + 2] * inv, o[db][4 * gq + 3] * inv);
        *(uint2*)(op + db * 32 + 8 * gq + 4 * hl) = pk;
      }
  }
}

}  // namespace

extern "C" int vggt_attention_fwd(const void* q, int64_t ldq, int64_t q_bstride, const void* k, int64_t ldk,
                                  int64_t k_bstride, const void* v, int64_t ldv, int64_t v_bstride, void* o,
                                  int64_t ldo, int64_t o_bstride, int batch, int heads, int nq, int nk, int D,
                                  float scale, void* stream) {
  if (batch <= 0 || heads <= 0 || nq <= 0 || nk <= 0) return VGGT_ERR_SHAPE;
  if (D != 64 && D != 128) return VGGT_ERR_UNSUPPORTED;
  if ((ldq | ldk | ldv | ldo) % 8 || ((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) % 16)
    return VGGT_ERR_ALIGN;
  AttnArgs a{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, ldq, ldk, ldv, ldo,
             q_bstride, k_bstride, v_bstride, o_bstride, batch, heads, nq, nk,
             scale * 1.4426950408889634f};
  const int nwg = ((nq + BQ - 1) / BQ) * heads * batch;
  hipStream_t s = (hipStream_t)stream;
  if (D == 64) attn_fwd_kernel<64><<<nwg, NT, 0, s>>>(a);
  else attn_fwd_kernel<128><<<nwg, NT, 0, s>>>(a);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}
