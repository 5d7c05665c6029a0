// Flash-attention backward for training the alignment head's frame blocks
// (8 heads x 128 over the P+1 tokens of each frame; alignment_head.py:347-366
// via checkpoint(frame_blocks[i]) in training mode) -- include/vggt_mi355x.h
// vggt_attention_bwd.  bf16 q/k/v/o/dO, fp32 accumulation, bf16 dq/dk/dv
// (the gradients autocast produces for bf16 SDPA inputs).
//
// Recomputes P from the forward's per-row log2-sum-exp (vggt_attention_fwd_lse):
//   p = exp2(s * c - lse2),  c = scale * log2(e)
//   dP = dO V^T,  delta = rowsum(dO * O),  dS = P * (dP - delta)
//   dQ = scale dS K,  dK = scale dS^T Q,  dV = P^T dO
// Two launches, no atomics, deterministic:
//  * dq kernel: a wave owns 32 query rows (swapped products as in the
//    forward: S^T = K Q^T and dP^T = V dO^T with v_mfma_f32_32x32x16_bf16, so
//    the lane owns one query and its lse / delta are lane scalars); the dS^T
//    accumulator rounded to bf16 is directly the B operand of
//    dQ^T = K^T dS^T, whose K^T A operand comes from ds_read_b64_tr_b16
//    transposed reads of the row-major K tile.  It also writes delta.
//  * dkdv kernel: a wave owns 32 keys; per 32-query tile S = Q K^T and
//    dP = dO V^T (key on the lane), then dV^T += dO^T P and dK^T += Q^T dS
//    with transposed reads of the Q / dO tiles.
// LDS rows are padded by 16 B (no swizzle: every tile is read both by rows
// and transposed); tiles are staged global -> VGPR -> LDS, double-buffered.
#include <math.h>

#include "common.h"
#include "mfma_frag.h"

namespace {

using namespace vggt_frag;

struct BwdArgs {
  const bf16_t *q, *k, *v, *o, *dout;
  bf16_t *dq, *dk, *dv;
  const float* lse;  // [batch*heads*nq] log2 units
  float* delta;      // [batch*heads*nq]
  int64_t ldq, ldk, ldv, ldo, lddq, lddkv;
  int64_t qbs, kbs, obs;  // batch strides in rows (q & dq share qbs, k/v & dk/dv share kbs, o & dO share obs)
  int batch, heads, nq, nk;
  float scale, c;
};

// Register-prefetched staging: tile t+1 is loaded into VGPRs before tile t's
// MFMAs and written to the other LDS buffer after them.
template <int D, int NR>
struct TilePrefetch {  // NR rows x D of a bf16 operand, spread over 256 threads
  static constexpr int CPR = D / 8, PER = NR * CPR / 256;
  uint4 v[PER];
  __device__ __forceinline__ void load(const bf16_t* src, int64_t ld, int r0, int valid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = threadIdx.x + 256 * i, row = idx / CPR, ch = idx % CPR;
      const int r = r0 + row;
      v[i] = r < valid ? *(const uint4*)(src + (int64_t)r * ld + ch * 8) : uint4{0u, 0u, 0u, 0u};
    }
  }
  __device__ __forceinline__ void store(char* tile) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = threadIdx.x + 256 * i, row = idx / CPR, ch = idx % CPR;
      *(uint4*)(tile + row * Geo<D>::ROWP + ch * 16) = v[i];
    }
  }
};

// ------------------------------------------------------------------ dQ
template <int D>
constexpr size_t dq_lds_bytes() {
  return (size_t)2 * 2 * 64 * Geo<D>::ROWP;
}

template <int D>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(BwdArgs a) {
  using G = Geo<D>;
  constexpr int BK = 64;
  constexpr int TILEB = BK * G::ROWP;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [buf][K | V][64][ROWP]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hl = lane >> 5;
  const int nqb = (a.nq + 127) / 128;
  const int bid = xcd_remap(blockIdx.x, nqb * a.heads * a.batch);
  const int qb = bid % nqb, bh = bid / nqb;
  const int h = bh % a.heads, b = bh / a.heads;
  const bf16_t* qp = a.q + (int64_t)b * a.qbs * a.ldq + h * D;
  const bf16_t* kp = a.k + (int64_t)b * a.kbs * a.ldk + h * D;
  const bf16_t* vp = a.v + (int64_t)b * a.kbs * a.ldv + h * D;
  const bf16_t* op = a.o + (int64_t)b * a.obs * a.ldo + h * D;
  const bf16_t* gp = a.dout + (int64_t)b * a.obs * a.ldo + h * D;

  const int qrow = qb * 128 + wave * 32 + (lane & 31);
  const int qr = min(qrow, a.nq - 1);
  bf16x8 qf[G::NKS], gf[G::NKS];
  float dpart = 0.f;
#pragma unroll
  for (int ks = 0; ks < G::NKS; ++ks) {
    qf[ks] = *(const bf16x8*)(qp + (int64_t)qr * a.ldq + ks * 16 + 8 * hl);
    gf[ks] = *(const bf16x8*)(gp + (int64_t)qr * a.ldo + ks * 16 + 8 * hl);
    const bf16x8 of = *(const bf16x8*)(op + (int64_t)qr * a.ldo + ks * 16 + 8 * hl);
#pragma unroll
    for (int j = 0; j < 8; ++j) dpart += (float)gf[ks][j] * (float)of[j];
  }
  const float delta = dpart + __shfl_xor(dpart, 32, 64);
  const int64_t rix = ((int64_t)b * a.heads + h) * a.nq + qr;
  const float lse = a.lse[rix];
  if (hl == 0 && qrow < a.nq) a.delta[rix] = delta;

  f32x16 dq[G::NDB];
#pragma unroll
  for (int i = 0; i < G::NDB; ++i) dq[i] = f32x16{};
  const int nt = (a.nk + BK - 1) / BK;
  TilePrefetch<D, BK> pk, pv;
  pk.load(kp, a.ldk, 0, a.nk);
  pv.load(vp, a.ldv, 0, a.nk);
  pk.store(smem);
  pv.store(smem + TILEB);
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const char* sk = smem + (t & 1) * 2 * TILEB;
    const char* sv = sk + TILEB;
    if (t + 1 < nt) {
      pk.load(kp, a.ldk, (t + 1) * BK, a.nk);
      pv.load(vp, a.ldv, (t + 1) * BK, a.nk);
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      f32x16 st = f32x16{}, dpt = f32x16{};
#pragma unroll
      for (int ks = 0; ks < G::NKS; ++ks) {
        st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<D>(sk, kb * 32, ks, lane), qf[ks], st, 0, 0, 0);
        dpt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<D>(sv, kb * 32, ks, lane), gf[ks], dpt, 0, 0, 0);
      }
      f32x16 ds;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = t * BK + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const float p = key < a.nk ? __builtin_amdgcn_exp2f(st[r] * a.c - lse) : 0.f;
        ds[r] = p * (dpt[r] - delta);
      }
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const bf16x8 dsf = pack8(ds, ss);
#pragma unroll
        for (int db = 0; db < G::NDB; ++db)
          dq[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag<D>(sk, db, kb, ss, lane), dsf, dq[db], 0, 0, 0);
      }
    }
    if (t + 1 < nt) {
      char* nb = smem + ((t + 1) & 1) * 2 * TILEB;
      pk.store(nb);
      pv.store(nb + TILEB);
    }
    __syncthreads();
  }
  if (qrow < a.nq) {
    bf16_t* dp = a.dq + ((int64_t)b * a.qbs + qrow) * a.lddq + h * D;
#pragma unroll
    for (int db = 0; db < G::NDB; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        uint2 pk;
        pk.x = pack_bf2(dq[db][4 * gq] * a.scale, dq[db][4 * gq + 1] * a.scale);
        pk.y = pack_bf2(dq[db][4 * gq + 2] * a.scale, dq[db][4 * gq + 3] * a.scale);
        *(uint2*)(dp + db * 32 + 8 * gq + 4 * hl) = pk;
      }
  }
}

// ------------------------------------------------------------------ dK, dV
// A wave owns 32 keys: its K rows live in registers as the B operand of
// S = Q K^T (loaded once), the workgroup's 128 V rows in LDS (B operand of
// dP = dO V^T).  The 32-query Q / dO tiles and their lse / delta are
// double-buffered: tile t+1 is loaded into registers before tile t's MFMAs
// and written to the other LDS buffer after them, one barrier per tile.
// 70 KB of LDS -> two workgroups per CU.
template <int D>
constexpr size_t dkdv_lds_bytes() {
  return (size_t)128 * Geo<D>::ROWP + (size_t)2 * 2 * 32 * Geo<D>::ROWP + 2 * 2 * 32 * 4;
}

template <int D>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_kernel(BwdArgs a) {
  using G = Geo<D>;
  constexpr int BKEY = 128, BQT = 32;
  constexpr int QTB = BQT * G::ROWP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sv = smem;                                  // V rows of the block [128][ROWP]
  char* sqg = smem + BKEY * G::ROWP;                // [buf][Q | dO][32][ROWP]
  float* sld = (float*)(sqg + 4 * QTB);             // [buf][lse | delta][32]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hl = lane >> 5;
  const int nkb = (a.nk + BKEY - 1) / BKEY;
  const int bid = xcd_remap(blockIdx.x, nkb * a.heads * a.batch);
  const int kb0 = bid % nkb, bh = bid / nkb;
  const int h = bh % a.heads, b = bh / a.heads;
  const bf16_t* qp = a.q + (int64_t)b * a.qbs * a.ldq + h * D;
  const bf16_t* kp = a.k + (int64_t)b * a.kbs * a.ldk + h * D;
  const bf16_t* vp = a.v + (int64_t)b * a.kbs * a.ldv + h * D;
  const bf16_t* gp = a.dout + (int64_t)b * a.obs * a.ldo + h * D;
  const int64_t rbase = ((int64_t)b * a.heads + h) * a.nq;

  // this wave's K rows (B operand of S = Q K^T: column = key)
  const int krow = kb0 * BKEY + wave * 32 + (lane & 31);
  const int kr = min(krow, a.nk - 1);
  bf16x8 kf[G::NKS];
#pragma unroll
  for (int ks = 0; ks < G::NKS; ++ks) kf[ks] = *(const bf16x8*)(kp + (int64_t)kr * a.ldk + ks * 16 + 8 * hl);
  stage_rows<D>(sv, vp, a.ldv, kb0 * BKEY, BKEY, a.nk);

  TilePrefetch<D, 32> pq, pg;
  float pls = 0.f;
  auto load_tile = [&](int t) {
    pq.load(qp, a.ldq, t * BQT, a.nq);
    pg.load(gp, a.ldo, t * BQT, a.nq);
    if (threadIdx.x < 2 * BQT) {
      const int qq = t * BQT + (threadIdx.x & (BQT - 1));
      pls = threadIdx.x < BQT ? (qq < a.nq ? a.lse[rbase + qq] : INFINITY) : (qq < a.nq ? a.delta[rbase + qq] : 0.f);
    }
  };
  auto store_tile = [&](int buf) {
    pq.store(sqg + (2 * buf) * QTB);
    pg.store(sqg + (2 * buf + 1) * QTB);
    if (threadIdx.x < 2 * BQT) sld[buf * 2 * BQT + threadIdx.x] = pls;
  };

  f32x16 dk[G::NDB], dv[G::NDB];
#pragma unroll
  for (int i = 0; i < G::NDB; ++i) dk[i] = dv[i] = f32x16{};
  const int nt = (a.nq + BQT - 1) / BQT;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1;
    if (t + 1 < nt) load_tile(t + 1);
    const char* sq = sqg + (2 * buf) * QTB;
    const char* sg = sqg + (2 * buf + 1) * QTB;
    const float* slse = sld + buf * 2 * BQT;
    const float* sdel = slse + BQT;
    f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
    for (int ks = 0; ks < G::NKS; ++ks) {
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<D>(sq, 0, ks, lane), kf[ks], s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<D>(sg, 0, ks, lane), rowfrag<D>(sv, wave * 32, ks, lane),
                                                   dp, 0, 0, 0);
    }
    f32x16 p, ds;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qi = (r & 3) + 8 * (r >> 2) + 4 * hl;
      const float pv = __builtin_amdgcn_exp2f(s[r] * a.c - slse[qi]);
      p[r] = pv;
      ds[r] = pv * (dp[r] - sdel[qi]);
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const bf16x8 pf = pack8(p, ss), dsf = pack8(ds, ss);
#pragma unroll
      for (int db = 0; db < G::NDB; ++db) {
        dv[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag<D>(sg, db, 0, ss, lane), pf, dv[db], 0, 0, 0);
        dk[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag<D>(sq, db, 0, ss, lane), dsf, dk[db], 0, 0, 0);
      }
    }
    if (t + 1 < nt) store_tile(buf ^ 1);
    __syncthreads();
  }
  if (krow < a.nk) {
    bf16_t* kq = a.dk + ((int64_t)b * a.kbs + krow) * a.lddkv + h * D;
    bf16_t* vq = a.dv + ((int64_t)b * a.kbs + krow) * a.lddkv + h * D;
#pragma unroll
    for (int db = 0; db < G::NDB; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        uint2 pk;
        pk.x = pack_bf2(dk[db][4 * gq] * a.scale, dk[db][4 * gq + 1] * a.scale);
        pk.y = pack_bf2(dk[db][4 * gq + 2] * a.scale, dk[db][4 * gq + 3] * a.scale);
        *(uint2*)(kq + db * 32 + 8 * gq + 4 * hl) = pk;
        pk.x = pack_bf2(dv[db][4 * gq], dv[db][4 * gq + 1]);
        pk.y = pack_bf2(dv[db][4 * gq + 2], dv[db][4 * gq + 3]);
        *(uint2*)(vq + db * 32 + 8 * gq + 4 * hl) = pk;
      }
  }
}

}  // namespace

extern "C" int vggt_attention_bwd(const void* q, int64_t ldq, int64_t q_bstride, const void* k, int64_t ldk,
                                  int64_t k_bstride, const void* v, int64_t ldv, const void* o, const void* dout,
                                  int64_t ldo, int64_t o_bstride, const float* lse, float* delta, void* dq,
                                  int64_t lddq, void* dk, void* dv, int64_t lddkv, int batch, int heads, int nq,
                                  int nk, int D, float scale, void* stream) {
  if (batch <= 0 || heads <= 0 || nq <= 0 || nk <= 0) return VGGT_ERR_SHAPE;
  if (D != 64 && D != 128) return VGGT_ERR_UNSUPPORTED;
  if ((ldq | ldk | ldv | ldo | lddq | lddkv) % 8) return VGGT_ERR_ALIGN;
  if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o | (uintptr_t)dout | (uintptr_t)dq | (uintptr_t)dk |
       (uintptr_t)dv) % 16)
    return VGGT_ERR_ALIGN;
  if (!lse || !delta) return VGGT_ERR_SHAPE;
  BwdArgs a{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)o, (const bf16_t*)dout,
            (bf16_t*)dq, (bf16_t*)dk, (bf16_t*)dv, lse, delta, ldq, ldk, ldv, ldo, lddq, lddkv,
            q_bstride, k_bstride, o_bstride, batch, heads, nq, nk, scale, scale * 1.4426950408889634f};
  hipStream_t s = (hipStream_t)stream;
  const int g1 = ((nq + 127) / 128) * heads * batch;
  const int g2 = ((nk + 127) / 128) * heads * batch;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_dkdv_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)dkdv_lds_bytes<64>());
    (void)hipFuncSetAttribute((const void*)attn_bwd_dkdv_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)dkdv_lds_bytes<128>());
    (void)hipFuncSetAttribute((const void*)attn_bwd_dq_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)dq_lds_bytes<64>());
    (void)hipFuncSetAttribute((const void*)attn_bwd_dq_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)dq_lds_bytes<128>());
    attr_set = true;
  }
  if (D == 64) {
    attn_bwd_dq_kernel<64><<<g1, 256, dq_lds_bytes<64>(), s>>>(a);
    attn_bwd_dkdv_kernel<64><<<g2, 256, dkdv_lds_bytes<64>(), s>>>(a);
  } else {
    attn_bwd_dq_kernel<128><<<g1, 256, dq_lds_bytes<128>(), s>>>(a);
    attn_bwd_dkdv_kernel<128><<<g2, 256, dkdv_lds_bytes<128>(), s>>>(a);
  }
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}
