// Flash-attention forward for the VGGT hot path (include/vggt_mi355x.h:
// vggt_attention_fwd): softmax(Q K^T * scale) V, bf16 in/out, fp32 online
// softmax, head_dim D in {64, 128}, non-causal, ragged nk (masked last tile).
//
// gfx950 design:
//  * Workgroup = 4 waves = 128 query rows (32 per wave); KV tiles of 64 keys
//    staged global->LDS by LDS-DMA (buffer_load_dwordx4 ... lds),
//    double-buffered.  The buffer descriptor is re-based per tile by SALU
//    (base += 64 rows, num_records = remaining rows), so the per-lane offsets
//    are loop-invariant (no VALU address math in the loop) and rows past nk
//    read as zeros by the hardware range check.
//  * "Swapped" QK^T: each wave computes S^T = K . Q^T with
//    v_mfma_f32_32x32x16_bf16, so a lane owns one query row (lane & 31) and
//    the two lanes l, l+32 hold all 64 keys of the tile -> the row max needs a
//    single v_permlane32_swap, the row sum stays lane-partial until the end.
//  * The S^T accumulator, rounded to bf16, is directly the B operand of
//    O^T = V^T . P^T (no LDS round trip for P); the V^T A-operand comes from
//    ds_read_b64_tr_b16 transposed reads of the row-major V tile.
//  * LDS images are XOR-swizzled on the DMA source offset so that the K
//    ds_read_b128 fragment reads and the V transposed reads are bank-conflict
//    free; the swizzles touch only row bits that are lane-constant, so every
//    LDS read is a loop-invariant base register + immediate offset (the tile
//    loop is unrolled x2 so the double-buffer index is compile-time).
//  * Online softmax in the log2 domain with a deferred rescale (T13): O and l
//    are rescaled only when some row's max grows by more than THR=8 (P <= 2^8).
//  * XCD-aware block order: consecutive query blocks of one (batch, head)
//    share an XCD so its K/V stream is served from one L2.
#include <math.h>
#include <stdlib.h>

#include <type_traits>

#include "common.h"
#include "tune.h"

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef int int32x4 __attribute__((ext_vector_type(4)));

constexpr int BKV = 64;
constexpr float THR = 8.0f;

struct AttnArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* o;
  int64_t ldq, ldk, ldv, ldo;
  int64_t qbs, kbs, vbs, obs;
  int batch, heads, nq, nk;
  float c;     // scale * log2(e)
  float* lse;  // optional [batch*heads*nq]: log2 sum exp2(scores * c) per row (training recompute)
};

// LDS-DMA: 16 B per lane from buffer `rsrc` at per-lane byte offset `voff`
// into the wave-uniform LDS address `lds` (+lane*16).  Inline asm keeps the
// pending LDS write invisible to hipcc's alias analysis (it would otherwise
// drain vmcnt(0) before reads of the other buffer); completion is waited for
// by the explicit vmcnt(0) + barrier at the end of every tile.
__device__ __forceinline__ void dma16(int32x4 rsrc, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(lds)
               : "memory");
}

__device__ __forceinline__ int32x4 make_rsrc(const void* base, uint32_t nbytes) {
  const uint64_t b = (uint64_t)base;
  int32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((uint32_t)b);
  r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) & 0xffff;
  r[2] = __builtin_amdgcn_readfirstlane(nbytes);
  r[3] = 0x00020000;
  return r;
}

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

// VAR (schedule variants, A/B-tested through vggt_tune): bit 0 = all K
// fragment reads before the QK^T MFMAs, bit 1 = four-chain row max, bit 2 =
// four partial row sums, bit 3 = row sums on the matrix core (an all-ones
// V^T block times P^T: 4 extra MFMAs per tile replace 32 VALU adds per lane;
// the sum is then over the bf16-rounded P that also feeds P.V).  Bit 10
// (1024, diagnostic, on top of 33): s_memtime stamps per tile segment, summed
// per wave into a.lse reinterpreted as unsigned long long[nwg][NW][STAMP_N]
// (vggt_attention_stamps; the kernel writes no lse then).
constexpr int STAMP_N = 8;
template <int D, int NW, int VAR>
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_fwd_kernel(AttnArgs a) {
  constexpr int BQ = NW * 32;            // query rows per workgroup (32 per wave)
  constexpr int ROWB = D * 2;            // bytes per K/V row in LDS
  constexpr int TILEB = BKV * ROWB;      // bytes per K (or V) tile
  constexpr int NKS = D / 16;            // k-steps of the QK^T MFMA
  constexpr int NDB = D / 32;            // 32-row output blocks of O^T
  constexpr int RPI = 1024 / ROWB;       // rows per 1-KiB DMA instruction
  constexpr int CPR = ROWB / 16;         // 16-B chunks per row
  constexpr int IPW = TILEB / 1024 / NW;  // DMA instructions per wave per operand
  constexpr int NSLOT = (VAR & (16 | 512)) ? 3 : 2;  // K|V tile slots (3: pipelined QK^T / DMA two ahead)
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * 2 * TILEB];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hl = lane >> 5;
  // 8-wave form: the second-dispatched half (waves 4-7) shares each SIMD with
  // an older wave and loses VALU arbitration on every segment; one static
  // priority raise for it (cdna_hip_programming.md T5, static form).
  // (VAR & 4096: no priority raise -- re-measured with the segment stamps, r11)
  if constexpr (NW == 8 && !(VAR & 4096)) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  }
  const int nqb = (a.nq + BQ - 1) / BQ;
  const int bid = xcd_remap(blockIdx.x, nqb * a.heads * a.batch);
  const int qb = bid % nqb;
  const int bh = bid / nqb;
  const int h = bh % a.heads;
  const int b = bh / a.heads;

  const bf16_t* qp = a.q + (int64_t)b * a.qbs * a.ldq + h * D;
  const bf16_t* kp = a.k + (int64_t)b * a.kbs * a.ldk + h * D;
  const bf16_t* vp = a.v + (int64_t)b * a.vbs * a.ldv + h * D;

  // ---- Q fragments = B operand of S^T = K Q^T: Q[q][16ks + 8*hl + j]
  const int qrow = qb * BQ + wave * 32 + (lane & 31);
  const int qr = min(qrow, a.nq - 1);
  bf16x8 qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) qf[ks] = *(const bf16x8*)(qp + (int64_t)qr * a.ldq + ks * 16 + 8 * hl);
  if constexpr ((VAR & 32) && !(VAR & 64)) {
    // scores come out of the MFMA already in log2 units: Q * (scale log2 e),
    // re-rounded to bf16 (one extra rounding of Q, ~2^-9 relative)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = (__bf16)((float)qf[ks][j] * a.c);
  }
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) asm volatile("" : "+v"(qf[ks]));  // retire the Q loads before the loop

  // ---- loop-invariant DMA offsets and LDS destinations
  // VAR & 2048 (8-wave form): only the priority-1 half (waves 4-7) issues the
  // tile's LDS-DMA, two pieces per operand each.  Segment stamps (VAR & 1024,
  // profiles/r11) showed those waves finish each tile ~870 cycles before their
  // SIMD partners and wait at the barrier, while the partners' tile work is the
  // tile's critical path: the DMA issue moves off it.
  constexpr bool DMAH = (VAR & 2048) && NW == 8;
  constexpr int IPWX = DMAH ? 2 * IPW : IPW;  // pieces per issuing wave per operand
  const int pbase = DMAH ? (wave >= 4 ? wave - 4 : 0) * IPWX : wave * IPW;
  uint32_t koff[IPWX], voff[IPWX];
#pragma unroll
  for (int i = 0; i < IPWX; ++i) {
    const int row = (pbase + i) * RPI + lane / CPR;
    const int cp = lane % CPR;
    koff[i] = (uint32_t)(row * a.ldk + k_swz<D>(row, cp) * 8) * 2u;
    voff[i] = (uint32_t)(row * a.ldv + v_swz<D>(row, cp) * 8) * 2u;
  }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem)) + pbase * 1024;
  // 32-bit scalar descriptor arithmetic (host: nk * ld * 2 < 2^31): a 64-bit
  // "remaining bytes" compare has no SALU form and would run on the VALU
  const int kstep = BKV * (int)a.ldk * 2, vstep = BKV * (int)a.ldv * 2;
  const int kbytes = a.nk * (int)a.ldk * 2, vbytes = a.nk * (int)a.ldv * 2;

  auto stage = [&](int buf, int t) {
    const int ko = kstep * t, vo = vstep * t;
    const int32x4 kr = make_rsrc((const char*)kp + ko, (uint32_t)max(kbytes - ko, 0));
    const int32x4 vr = make_rsrc((const char*)vp + vo, (uint32_t)max(vbytes - vo, 0));
    const uint32_t d = lds0 + buf * 2 * TILEB;
    if (!DMAH || wave >= 4) {
#pragma unroll
      for (int i = 0; i < IPWX; ++i) {
        dma16(kr, koff[i], d + i * 1024);
        dma16(vr, voff[i], d + TILEB + i * 1024);
      }
    }
  };

  // ---- loop-invariant LDS read addresses (bytes within one K|V buffer pair)
  uint32_t ka[NKS];
  {
    const int key = lane & 31;  // + kb*32: swizzle-invariant
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) ka[ks] = key * ROWB + (k_swz<D>(key, 2 * ks + hl) << 4);
  }
  uint32_t va[NDB];
  {
    const int g = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
    const int r0 = 4 * hl + qq;  // + kb*32 + 16*ss + 8*half: swizzle-invariant
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      const int col = db * 32 + 16 * g + 4 * pp;
      va[db] = TILEB + r0 * ROWB + (v_swz<D>(r0, col >> 3) << 4) + (col & 7) * 2;
    }
  }

  f32x16 o[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) o[i] = f32x16{};
  // VAR & 32 starts from a finite "unset" offset: masked scores (-inf) minus
  // it stay -inf (-inf - -inf would be a NaN, and the kernel is built with
  // -fno-honor-nans, so a NaN could slip past the range guard)
  constexpr float M_UNSET = -1e30f;
  float m_run = (VAR & 32) ? M_UNSET : -INFINITY, l_run = 0.f;
  f32x16 lsum = f32x16{};  // VAR & 8: every row of the ones-block product holds l[q]
  // VAR & 32: per-row bound exponent of the offset mode (60 at offset 0, THR
  // once the row carries a max offset) and whether every row of the wave sits
  // at offset 0 (then p = exp2(s) with no subtraction at all)
  float lim = THR, limv = 256.0f;
  bool zero_off = false;
  const float c = a.c;
  const int nt = (a.nk + BKV - 1) / BKV;
  // VAR & 1024: per-wave cycle sums of the tile segments (s_memtime, one scalar
  // statement with its lgkmcnt(0)); 32-bit sums, no tile counter (the host
  // knows the tile count): so instrumented, the kernel keeps the default's 113
  // VGPRs and occupancy (a per-tile counter, VGPR-pinned sums or scheduling
  // barriers around the stamps each pushed it to 119-153)
  uint32_t st_acc[STAMP_N] = {}, st_prev = 0;
#define VGGT_SEG(i)                                                                                  \
  do {                                                                                               \
    if constexpr (VAR & 1024) {                                                                      \
      /* no sched_barrier: it pushed the kernel to 150 VGPRs */                                     \
      unsigned long long now_;                                                                       \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(now_)::"memory");                     \
      if ((i) >= 0) st_acc[(i) >= 0 ? (i) : 0] += (uint32_t)now_ - st_prev;                          \
      st_prev = (uint32_t)now_;                                                                      \
      /* no sched_barrier: it pushed the kernel to 150 VGPRs */                                     \
    }                                                                                                \
  } while (0)

  struct S2 {
    f32x16 v[2];
  };
  // ---- S^T = K . Q^T for the two 32-key blocks of the tile in slot BUF
  auto qk = [&](auto bufc) -> S2 {
    constexpr int BUF = decltype(bufc)::value;
    const char* base = smem + BUF * 2 * TILEB;
    f32x16 s[2];
    if constexpr (VAR & 1) {
      // all K fragment reads first, then the two 32-key accumulator chains
      // interleaved (no MFMA waits on a just-issued LDS read)
      bf16x8 kf[2][NKS];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) kf[kb][ks] = *(const bf16x8*)(base + ka[ks] + kb * 32 * ROWB);
      s[0] = f32x16{};
      s[1] = f32x16{};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
          s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kb][ks], qf[ks], s[kb], 0, 0, 0);
    } else {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        s[kb] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const bf16x8 kf = *(const bf16x8*)(base + ka[ks] + kb * 32 * ROWB);
          s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[kb], 0, 0, 0);
        }
      }
    }
    return S2{{s[0], s[1]}};
  };
  // ---- the same scores recomputed on a rare path (VAR & 32): the LDS offset
  // goes through an empty asm so the reads are not CSE'd with the common
  // path's (which would keep 32 K-fragment registers live across the tile)
  // and the MFMAs cannot be speculated out of the branch
  auto qk_again = [&](auto bufc) -> S2 {
    constexpr int BUF = decltype(bufc)::value;
    uint32_t opq = BUF * 2 * TILEB;
    asm volatile("" : "+v"(opq));
    const char* base = smem + opq;
    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      s[kb] = f32x16{};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 kf = *(const bf16x8*)(base + ka[ks] + kb * 32 * ROWB);
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[kb], 0, 0, 0);
      }
    }
    return S2{{s[0], s[1]}};
  };
  // ---- mask, online softmax and O^T += V^T . P^T for the tile in slot BUF
  auto soft_pv = [&](auto bufc, int t, S2 sc, auto zc) {
    constexpr int BUF = decltype(bufc)::value;
    const char* base = smem + BUF * 2 * TILEB;
    f32x16 s[2] = {sc.v[0], sc.v[1]};
    const int kv0 = t * BKV;
    auto mask = [&]() {
      if (kv0 + BKV > a.nk) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kv0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
            if (key >= a.nk) s[kb][r] = -INFINITY;
          }
      }
    };
    mask();
    bf16x8 pf[2][2];
    if constexpr (VAR & 32) {
      // Offset-free online softmax.  softmax is shift-invariant, and bf16 / fp32
      // keep their relative precision at any exponent, so the max subtraction
      // only guards the exponent range.  Each row carries an offset m_run
      // (log2 units), fixed at its first tile: 0 when that tile's max lies in
      // [-60, 60] (then p = exp2(s) -- no max, no subtraction; the first
      // tile's max term keeps l >= 2^-60), else the max itself.  A lane's
      // partial sum over its 32 keys <= 2^lim bounds every p of it by 2^lim
      // (lim = 60 at offset 0, THR otherwise -- the T13 bound), so no row max
      // is computed on the common path.  Only when some lane's sum exceeds its
      // bound (first tile: m_run = -inf -> p = inf) does the wave recompute the
      // raw scores from LDS, take the true row max and move the offset of the
      // rows that need it -- before this tile's P.V (the textbook order).
      // VAR & 64: exact scores (s * c per element, no Q prescale).
      float rs[4];
      auto exps = [&](auto shc) {
        constexpr bool shifted = decltype(shc)::value;
#pragma unroll
        for (int i = 1; i < 4; ++i) rs[i] = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) {
            bf16x8 t;  // whole-vector write: the previous pf is dead here, not an insert operand
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              float x = s[kb][8 * ss + j];
              if constexpr (VAR & 64) x = shifted ? fmaf(x, c, -m_run) : x * c;
              else if constexpr (shifted) x -= m_run;
              const float p = __builtin_amdgcn_exp2f(x);
              // one chain: split sums get SLP-packed into v_pk_add_f32; started from the
              // first p (p >= +0, so 0 + p == p bitwise: one v_add fewer per tile)
              if (kb == 0 && ss == 0 && j == 0) rs[0] = p;
              else rs[0] += p;
              t[j] = (__bf16)p;
            }
            pf[kb][ss] = t;
          }
      };
      // zero-offset loop (zc true): p = exp2(s); a wave that has left offset 0
      // (zero_off false: also before its first tile) takes the rare path
      constexpr bool ZL = decltype(zc)::value;
      exps(std::integral_constant<bool, !ZL>{});
      float rsum = (rs[0] + rs[1]) + (rs[2] + rs[3]);
      // the ballot of the compare alone (a v_cmp straight into an SGPR mask), OR'd with the
      // wave-uniform mode flag on the scalar side (one ballot over both materialised the
      // mask into a VGPR and compared it again: two VALU per tile)
      if ((__builtin_amdgcn_ballot_w64(!(rsum <= limv)) != 0) || (ZL && !zero_off)) {
        const S2 raw = qk_again(bufc);
        s[0] = raw.v[0];
        s[1] = raw.v[1];
        mask();
        float mx = fmaxf(s[0][0], s[0][1]);
#pragma unroll
        for (int r = 2; r < 16; r += 2) mx = fmaxf(fmaxf(mx, s[0][r]), s[0][r + 1]);
#pragma unroll
        for (int r = 0; r < 16; r += 2) mx = fmaxf(fmaxf(mx, s[1][r]), s[1][r + 1]);
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
        if constexpr (VAR & 64) mx *= c;
        // a lane sum > 2^lim implies a p > 2^(lim-5): move the offset exactly
        // for those rows (mx > m_run + lim - 5), so afterwards p <= 1 there and
        // every other row still has p <= 2^(lim-5), sum <= 2^lim
        float m_new = m_run;
        if (m_run == M_UNSET) m_new = fabsf(mx) <= 60.f ? 0.f : mx;
        else if (mx > m_run + (lim - 5.f)) m_new = mx;
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        lim = m_run == 0.f ? 60.f : THR;
        limv = m_run == 0.f ? 0x1p60f : 256.0f;  // 2^lim
        zero_off = __builtin_amdgcn_ballot_w64(m_run != 0.f) == 0;
        l_run *= alpha;
#pragma unroll
        for (int db = 0; db < NDB; ++db) o[db] *= alpha;
        exps(std::true_type{});
        rsum = (rs[0] + rs[1]) + (rs[2] + rs[3]);
      }
      l_run += rsum;
    } else {
    // ---- row max (lane-partial over 32 keys, then the partner half)
    float mx;
    if constexpr (VAR & 2) {
      // four independent v_max3 chains (built with -fno-honor-nans), merged:
      // dependency depth 5 instead of 16
      float mc[4];
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        const f32x16& sv = s[cc >> 1];
        const int r0 = (cc & 1) * 8;
        float m = fmaxf(sv[r0], sv[r0 + 1]);
#pragma unroll
        for (int r = r0 + 2; r < r0 + 8; r += 2) m = fmaxf(fmaxf(m, sv[r]), sv[r + 1]);
        mc[cc] = m;
      }
      mx = fmaxf(fmaxf(mc[0], mc[1]), fmaxf(mc[2], mc[3]));
    } else {
      mx = fmaxf(s[0][0], s[0][1]);  // one v_max3 chain
#pragma unroll
      for (int r = 2; r < 16; r += 2) mx = fmaxf(fmaxf(mx, s[0][r]), s[0][r + 1]);
#pragma unroll
      for (int r = 0; r < 16; r += 2) mx = fmaxf(fmaxf(mx, s[1][r]), s[1][r + 1]);
    }
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1])) * c;
    }
    // ---- deferred rescale: only when some row's max grew by > THR
    if (__builtin_amdgcn_ballot_w64(mx > m_run + THR) != 0) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      m_run = m_new;
      if constexpr (VAR & 8) lsum *= alpha;
      else l_run *= alpha;
#pragma unroll
      for (int db = 0; db < NDB; ++db) o[db] *= alpha;
    }
    float rs[4] = {0.f, 0.f, 0.f, 0.f};  // four partial row sums (short add chains)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[kb][8 * ss + j], c, -m_run));
          if constexpr (!(VAR & 8)) rs[(VAR & 4) ? 2 * kb + ss : 0] += p;
          pf[kb][ss][j] = (__bf16)p;
        }
    if constexpr (!(VAR & 8)) l_run += (rs[0] + rs[1]) + (rs[2] + rs[3]);
    }
    // ---- O^T += V^T . P^T
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const char* p0 = base + va[db] + (kb * 32 + 16 * ss) * ROWB;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)LDS_PTR(p0));
          const s16x4 hi =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)LDS_PTR(p0 + 8 * ROWB));
          const bf16x8 vf = __builtin_bit_cast(bf16x8, (s16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kb][ss], o[db], 0, 0, 0);
        }
    if constexpr (VAR & 8) {
      bf16x8 ones;
#pragma unroll
      for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) lsum = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[kb][ss], lsum, 0, 0, 0);
    }
  };

  // ---- VAR & 256 (offset-free only; full tiles): the tile as two 32-key
  // halves, software-pipelined inside the wave -- the QK^T MFMAs of half 1
  // are issued between the exps of half 0, and the P.V MFMAs of half 0
  // between the exps of half 1, so a wave keeps its own matrix pipe busy
  // while its VALU works (the default form runs QK^T, softmax and P.V of a
  // tile as three phases and relies on the other waves of the SIMD for
  // overlap).  The range guard runs per half: a half whose lane sum (16
  // keys) exceeds 2^lim moves the offsets of its rows exactly as the whole-
  // tile guard does (a 16-key sum > 2^lim implies a p > 2^(lim-4)), and a
  // P.V already accumulated for half 0 is rescaled with O and l (its p were
  // finite).  Same products in the same order per row: results equal the
  // default form's up to the order of the fp32 row-sum adds.
  auto tile_split = [&](auto bufc, auto zc) {
    constexpr int BUF = decltype(bufc)::value;
    constexpr bool ZL = decltype(zc)::value;
    const char* base = smem + BUF * 2 * TILEB;
    f32x16 s0 = f32x16{}, s1 = f32x16{};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const bf16x8 kf = *(const bf16x8*)(base + ka[ks]);
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s0, 0, 0, 0);
    }
    bf16x8 k1[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) k1[ks] = *(const bf16x8*)(base + ka[ks] + 32 * ROWB);
    bf16x8 p0[2], p1[2];
    auto exph = [&](const f32x16& sv, bf16x8 (&pf)[2], auto shc) -> float {
      constexpr bool shifted = decltype(shc)::value;
      float r = 0.f;
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        bf16x8 tv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float x = sv[8 * ss + j];
          if constexpr (shifted) x -= m_run;
          const float pv = __builtin_amdgcn_exp2f(x);
          if (ss == 0 && j == 0) r = pv;
          else r += pv;
          tv[j] = (__bf16)pv;
        }
        pf[ss] = tv;
      }
      return r;
    };
    auto pv_half = [&](int kb, const bf16x8 (&pf)[2]) {
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const char* p0_ = base + va[db] + (kb * 32 + 16 * ss) * ROWB;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)LDS_PTR(p0_));
          const s16x4 hi =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)LDS_PTR(p0_ + 8 * ROWB));
          const bf16x8 vf = __builtin_bit_cast(bf16x8, (s16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[ss], o[db], 0, 0, 0);
        }
    };
    auto rowmax = [&](const f32x16& a0, const f32x16* a1) {
      float mx = fmaxf(a0[0], a0[1]);
#pragma unroll
      for (int r = 2; r < 16; r += 2) mx = fmaxf(fmaxf(mx, a0[r]), a0[r + 1]);
      if (a1) {
#pragma unroll
        for (int r = 0; r < 16; r += 2) mx = fmaxf(fmaxf(mx, (*a1)[r]), (*a1)[r + 1]);
      }
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      return fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    };
    auto move_offset = [&](float mx) {
      float m_new = m_run;
      if (m_run == M_UNSET) m_new = fabsf(mx) <= 60.f ? 0.f : mx;
      else if (mx > m_run + (lim - 5.f)) m_new = mx;
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      m_run = m_new;
      lim = m_run == 0.f ? 60.f : THR;
      limv = m_run == 0.f ? 0x1p60f : 256.0f;
      zero_off = __builtin_amdgcn_ballot_w64(m_run != 0.f) == 0;
      l_run *= alpha;
#pragma unroll
      for (int db = 0; db < NDB; ++db) o[db] *= alpha;
    };
    // QK^T of half 1 beside the exps of half 0
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k1[ks], qf[ks], s1, 0, 0, 0);
    float r0 = exph(s0, p0, std::integral_constant<bool, !ZL>{});
    if ((__builtin_amdgcn_ballot_w64(!(r0 <= limv)) != 0) || (ZL && !zero_off)) {
      // rare: the whole tile from raw scores (first tile, or an offset move in half 0)
      const S2 raw = qk_again(bufc);
      move_offset(rowmax(raw.v[0], &raw.v[1]));
      l_run += exph(raw.v[0], p0, std::true_type{});
      l_run += exph(raw.v[1], p1, std::true_type{});
      pv_half(0, p0);
      pv_half(1, p1);
      return;
    }
    l_run += r0;
    // P.V of half 0 beside the exps of half 1
    pv_half(0, p0);
    float r1 = exph(s1, p1, std::integral_constant<bool, !ZL>{});
    if (__builtin_amdgcn_ballot_w64(!(r1 <= limv)) != 0) {
      const S2 raw = qk_again(bufc);
      move_offset(rowmax(raw.v[1], nullptr));
      r1 = exph(raw.v[1], p1, std::true_type{});
    }
    l_run += r1;
    pv_half(1, p1);
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;

  if constexpr (VAR & 16) {
    // Pipelined: the QK^T MFMAs of tile t+1 are issued before tile t's softmax
    // (T15), so the matrix pipe works while the VALU does exp / max / cvt.
    // 3 slots: t (V read by P.V), t+1 (K read by QK^T), t+2 (DMA in flight,
    // issued after the barrier that retires slot t-1).
    stage(0, 0);
    if (nt > 1) stage(1, 1);
    if (nt > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * IPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    S2 cur = qk(I0{});
    auto step = [&](auto sc, auto sn, auto sf, int t) {
      // tile t+1 landed everywhere; every wave done with slot (t-1)%3 = (t+2)%3
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t + 2 < nt) stage(decltype(sf)::value, t + 2);
      S2 nxt = cur;
      if (t + 1 < nt) nxt = qk(sn);
      soft_pv(sc, t, cur, std::false_type{});
      cur = nxt;
    };
    for (int t = 0; t < nt; t += 3) {
      step(I0{}, I1{}, I2{}, t);
      if (t + 1 >= nt) break;
      step(I1{}, I2{}, I0{}, t + 1);
      if (t + 2 >= nt) break;
      step(I2{}, I0{}, I1{}, t + 2);
    }
  } else if constexpr (VAR & 512) {
    // Three K|V slots, the DMA two tiles ahead: tile t+2 is staged at the start
    // of tile t (into the slot tile t-1 used, retired by the barrier that ended
    // tile t-1), and the end of tile t waits only for tile t+1's pieces
    // (vmcnt counts in order: the 2*IPW pieces of t+2 may stay in flight), so
    // each tile's loads have two tiles' compute to land instead of one.
    stage(0, 0);
    if (nt > 1) stage(1, 1);
    if (nt > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * IPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    auto step = [&](auto sc, auto sf, auto zc, int t) {
      if (t + 2 < nt) stage(decltype(sf)::value, t + 2);
      soft_pv(sc, t, qk(sc), zc);
      if (t + 2 < nt) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * IPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    };
    // the offset mode may change only at a multiple of 3 tiles (slot = t % 3)
    auto run = [&](auto zc, int t0) -> int {
      for (int t = t0; t < nt; t += 3) {
        step(I0{}, I2{}, zc, t);
        if (t + 1 >= nt) break;
        step(I1{}, I0{}, zc, t + 1);
        if (t + 2 >= nt) break;
        step(I2{}, I1{}, zc, t + 2);
        if constexpr (decltype(zc)::value) {
          if (!zero_off) return t + 3;
        }
      }
      return nt;
    };
    const int t1 = run(std::true_type{}, 0);
    if (t1 < nt) run(std::false_type{}, t1);
  } else {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // VAR & 32: two copies of the tile loop, one per offset mode (one loop with
    // a per-tile choice between the two exp forms costs ~25 VGPRs at the merge:
    // occupancy 4 -> 3).  Every wave starts in the zero-offset loop and leaves
    // it for good, at a tile pair boundary, once one of its rows took an offset.
    // VAR & 1024 segments of one tile: [2] the tile's work (DMA issue, QK^T, softmax,
    // P.V issue, up to its last LDS read), [3] end-of-tile vmcnt(0) wait for the next
    // tile's DMA, [4] barrier.  (Stamps inside the tile body, between the
    // DMA issue and QK^T or between the softmax and P.V, serialise what the compiler
    // overlaps there and pushed the kernel from 113 to 152 VGPRs: not kept.)
    auto run = [&](auto zc, int t0) -> int {
      for (int t = t0; t < nt; t += 2) {
        VGGT_SEG(-1);
        if (t + 1 < nt) stage(1, t + 1);
        if ((VAR & 256) && (t + 1) * BKV <= a.nk) tile_split(I0{}, zc);
        else soft_pv(I0{}, t, qk(I0{}), zc);
        VGGT_SEG(2);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        VGGT_SEG(3);
        __syncthreads();
        VGGT_SEG(4);
        if (t + 1 >= nt) break;
        if (t + 2 < nt) stage(0, t + 2);
        if ((VAR & 256) && (t + 2) * BKV <= a.nk) tile_split(I1{}, zc);
        else soft_pv(I1{}, t + 1, qk(I1{}), zc);
        VGGT_SEG(2);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        VGGT_SEG(3);
        __syncthreads();
        VGGT_SEG(4);
        if constexpr (decltype(zc)::value) {
          if (!zero_off) return t + 2;
        }
      }
      return nt;
    };
    if constexpr (VAR & 32) {
      const int t1 = run(std::true_type{}, 0);
      if (t1 < nt) run(std::false_type{}, t1);
    } else {
      run(std::false_type{}, 0);
    }
  }

  // ---- epilogue: normalise, O[q][d] bf16
  if constexpr (VAR & 8) {
    l_run = lsum[0];
  } else {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_run), __float_as_uint(l_run), false, false);
    l_run = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  const float inv = 1.f / l_run;
  if constexpr (VAR & 1024) {
    VGGT_SEG(-1);
    st_acc[6] = st_prev;  // the wave's end (low 32 bits), to place it against the others of its workgroup
    if (lane == 0) {
      unsigned long long* out = (unsigned long long*)(void*)a.lse + ((int64_t)blockIdx.x * NW + wave) * STAMP_N;
#pragma unroll
      for (int i = 0; i < STAMP_N; ++i) out[i] = st_acc[i];
    }
  } else {
    if (a.lse && hl == 0 && qrow < a.nq) a.lse[((int64_t)b * a.heads + h) * a.nq + qrow] = m_run + __log2f(l_run);
  }
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

// ---------------------------------------------------------------------------
// D = 64 forward on v_mfma_f32_16x16x32_bf16 (variant 161 = 33 | 128).
//  * Matrix-core shape: per wave 32 query rows = two 16-query blocks qb, per
//    64-key tile four 16-key blocks kb; S^T[kb][qb] = K_kb . Q_qb^T leaves
//    lane l with keys kb*16 + 4*(l/16) + i (i < 4) of query qb*16 + (l & 15).
//    Under sustained load the chip holds a higher clock on 16x16x32 than on
//    32x32x16 for the same work (MI355X_MICROARCH.md 'DVFS give-back' item 7).
//  * P^T is the B operand of O^T += V^T . P^T straight from the accumulators:
//    register j of lane group g in P.V k-step kk is the key
//    32*kk + 16*(j/4) + 4*g + (j&3) -- a permutation of the tile's keys, which
//    the sum over keys does not see; the V^T A operand reads exactly those
//    keys with two ds_read_b64_tr_b16 (rows 32kk + 4g + 0..3 and +16).
//  * Softmax without any per-tile max or branch: softmax is shift-invariant
//    and fp32 / bf16 keep their relative precision at any exponent, so every
//    row uses offset 0 (p = exp2(s), s already in log2 units through the Q
//    prescale).  That is exact as long as the row's p stay inside the fp32
//    range with room to spare; the sum says so at the end: 2^-60 <= l <= 2^100
//    (a row max below -60 or a p overflow to inf fails it).  If any row of the
//    workgroup fails, the workgroup recomputes its rows in two exact passes
//    (row max over all keys, then exp2(s - max) and P.V) -- a path only
//    extreme scores take (tests/test_gpu_kernels.py offset-free extremes).
//  * K swizzle as attn_fwd_kernel<64> (conflict-free for this read pattern
//    too); V swizzle chunk ^ (((row >> 1) & 3) << 1): conflict-free for the
//    8 rows x 32 B each half-wave of the transposed reads covers.
__device__ __forceinline__ int k16_swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
__device__ __forceinline__ int v16_swz(int row, int chunk) { return chunk ^ (((row >> 1) & 3) << 1); }

template <int NW>
__global__ __launch_bounds__(NW * 64, 16 / NW) void attn16_fwd_kernel(AttnArgs a) {
  constexpr int D = 64;
  constexpr int BQ = NW * 32;
  constexpr int ROWB = D * 2;
  constexpr int TILEB = BKV * ROWB;
  constexpr int RPI = 1024 / ROWB;
  constexpr int CPR = ROWB / 16;
  constexpr int IPW = TILEB / 1024 / NW;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILEB];
  __shared__ int redo;  // workgroup vote: some row needs the exact two-pass path

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  if constexpr (NW == 8) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  }
  const int nqb = (a.nq + BQ - 1) / BQ;
  const int bid = xcd_remap(blockIdx.x, nqb * a.heads * a.batch);
  const int qblk = bid % nqb;
  const int bh = bid / nqb;
  const int h = bh % a.heads;
  const int b = bh / a.heads;

  const bf16_t* qp = a.q + (int64_t)b * a.qbs * a.ldq + h * D;
  const bf16_t* kp = a.k + (int64_t)b * a.kbs * a.ldk + h * D;
  const bf16_t* vp = a.v + (int64_t)b * a.vbs * a.ldv + h * D;
  const int q0 = qblk * BQ + wave * 32 + c16;  // query of block qb: q0 + 16 qb

  // ---- Q fragments (B operand of S^T = K Q^T), prescaled into log2 units
  bf16x8 qf[2][2];  // [qb][ks]: Q[query][32 ks + 8 g + j] * scale * log2(e)
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int qr = min(q0 + 16 * qb, a.nq - 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[qb][ks] = *(const bf16x8*)(qp + (int64_t)qr * a.ldq + ks * 32 + 8 * g);
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[qb][ks][j] = (__bf16)((float)qf[qb][ks][j] * a.c);
    }
  }
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) asm volatile("" : "+v"(qf[qb][ks]));

  // ---- loop-invariant DMA offsets
  uint32_t koff[IPW], voff[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int row = (wave * IPW + i) * RPI + lane / CPR;
    const int cp = lane % CPR;
    koff[i] = (uint32_t)(row * a.ldk + k16_swz(row, cp) * 8) * 2u;
    voff[i] = (uint32_t)(row * a.ldv + v16_swz(row, cp) * 8) * 2u;
  }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem)) + wave * IPW * 1024;
  const int kstep = BKV * (int)a.ldk * 2, vstep = BKV * (int)a.ldv * 2;
  const int kbytes = a.nk * (int)a.ldk * 2, vbytes = a.nk * (int)a.ldv * 2;
  auto stage = [&](int buf, int t) {
    const int ko = kstep * t, vo = vstep * t;
    const int32x4 kr = make_rsrc((const char*)kp + ko, (uint32_t)max(kbytes - ko, 0));
    const int32x4 vr = make_rsrc((const char*)vp + vo, (uint32_t)max(vbytes - vo, 0));
    const uint32_t d = lds0 + buf * 2 * TILEB;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      dma16(kr, koff[i], d + i * 1024);
      dma16(vr, voff[i], d + TILEB + i * 1024);
    }
  };

  // ---- loop-invariant LDS read addresses (the kb / kk / half row steps keep the swizzles)
  uint32_t ka[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) ka[ks] = c16 * ROWB + (k16_swz(c16, 4 * ks + g) << 4);
  uint32_t va[4];
  {
    const int qq = (lane >> 2) & 3, pp = lane & 3;
    const int r0 = 4 * g + qq;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const int col = db * 16 + 4 * pp;
      va[db] = TILEB + r0 * ROWB + (v16_swz(r0, col >> 3) << 4) + (col & 7) * 2;
    }
  }
  const int nt = (a.nk + BKV - 1) / BKV;

  struct S8 {
    f32x4 v[4][2];
  };
  // S^T of the tile in slot BUF, keys past nk at -inf
  auto scores = [&](auto bufc, int t) -> S8 {
    constexpr int BUF = decltype(bufc)::value;
    const char* base = smem + BUF * 2 * TILEB;
    S8 s;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const bf16x8 k0 = *(const bf16x8*)(base + ka[0] + kb * 16 * ROWB);
      const bf16x8 k1 = *(const bf16x8*)(base + ka[1] + kb * 16 * ROWB);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        s.v[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf[qb][0], f32x4{}, 0, 0, 0);
        s.v[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf[qb][1], s.v[kb][qb], 0, 0, 0);
      }
    }
    const int kv0 = t * BKV;
    if (kv0 + BKV > a.nk) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (kv0 + kb * 16 + 4 * g + i >= a.nk) {
            s.v[kb][0][i] = -INFINITY;
            s.v[kb][1][i] = -INFINITY;
          }
    }
    return s;
  };

  f32x4 o[4][2];  // [db][qb]: O^T[db*16 + 4g + i][query q0 + 16 qb]
  float l[2];     // lane-partial row sums
  float m[2] = {0.f, 0.f};  // row offsets (0 on the fast path)

  // p = exp2(s - m) rounded to bf16, row sums, O^T += V^T . P^T
  auto soft_pv = [&](auto bufc, int t, auto shc) {
    constexpr int BUF = decltype(bufc)::value;
    constexpr bool SHIFT = decltype(shc)::value;
    const char* base = smem + BUF * 2 * TILEB;
    const S8 s = scores(bufc, t);
    bf16x8 pf[2][2];  // [qb][kk]
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float rs = 0.f;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 tv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float x = s.v[2 * kk + (j >> 2)][qb][j & 3];
          if constexpr (SHIFT) x -= m[qb];
          const float p = __builtin_amdgcn_exp2f(x);
          rs += p;
          tv[j] = (__bf16)p;
        }
        pf[qb][kk] = tv;
      }
      l[qb] += rs;
    }
    const char* vb = base;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const char* p0 = vb + va[db] + kk * 32 * ROWB;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)LDS_PTR(p0));
        const s16x4 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)LDS_PTR(p0 + 16 * ROWB));
        const bf16x8 vf = __builtin_bit_cast(bf16x8, (s16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
          o[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qb][kk], o[db][qb], 0, 0, 0);
      }
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // one sweep over the key tiles, double-buffered: body(slot, t)
  auto sweep = [&](auto body) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nt; t += 2) {
      if (t + 1 < nt) stage(1, t + 1);
      body(I0{}, t);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t + 1 >= nt) break;
      if (t + 2 < nt) stage(0, t + 2);
      body(I1{}, t + 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  };
  auto reset = [&]() {
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) o[db][qb] = f32x4{};
    l[0] = l[1] = 0.f;
  };
  // sum (or max) over the four 16-lane groups holding one query's keys
  auto allsum = [](float x) {
    const auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(s16[0]) + __uint_as_float(s16[1]);
    const auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(s32[0]) + __uint_as_float(s32[1]);
  };
  auto allmax = [](float x) {
    const auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = fmaxf(__uint_as_float(s16[0]), __uint_as_float(s16[1]));
    const auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(s32[0]), __uint_as_float(s32[1]));
  };

  // ---- fast path: offset 0 everywhere
  if (threadIdx.x == 0) redo = 0;  // ordered before the reads by the sweep's barriers
  reset();
  sweep([&](auto bufc, int t) { soft_pv(bufc, t, std::false_type{}); });
  l[0] = allsum(l[0]);
  l[1] = allsum(l[1]);
  const bool bad = !(l[0] >= 0x1p-60f && l[0] <= 0x1p100f) || !(l[1] >= 0x1p-60f && l[1] <= 0x1p100f);
  if (__builtin_amdgcn_ballot_w64(bad) != 0 && lane == 0) redo = 1;
  __syncthreads();
  if (redo) {
    // ---- exact two-pass path: row max over all keys, then exp2(s - max)
    float mx[2] = {-INFINITY, -INFINITY};
    sweep([&](auto bufc, int t) {
      const S8 s = scores(bufc, t);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
          mx[qb] = fmaxf(fmaxf(mx[qb], fmaxf(s.v[kb][qb][0], s.v[kb][qb][1])), fmaxf(s.v[kb][qb][2], s.v[kb][qb][3]));
    });
    m[0] = allmax(mx[0]);
    m[1] = allmax(mx[1]);
    reset();
    sweep([&](auto bufc, int t) { soft_pv(bufc, t, std::true_type{}); });
    l[0] = allsum(l[0]);
    l[1] = allsum(l[1]);
  }

  // ---- epilogue: normalise, O[q][d] bf16
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int qrow = q0 + 16 * qb;
    const float inv = 1.f / l[qb];
    if (a.lse && g == 0 && qrow < a.nq) a.lse[((int64_t)b * a.heads + h) * a.nq + qrow] = m[qb] + __log2f(l[qb]);
    if (qrow < a.nq) {
      bf16_t* op = a.o + ((int64_t)b * a.obs + qrow) * a.ldo + h * D;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        uint2 pk;
        pk.x = pack_bf2(o[db][qb][0] * inv, o[db][qb][1] * inv);
        pk.y = pack_bf2(o[db][qb][2] * inv, o[db][qb][3] * inv);
        *(uint2*)(op + db * 16 + 4 * g) = pk;
      }
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
  // 32-bit DMA offsets and descriptor arithmetic: K / V of one (batch, head) must span < 2 GiB
  if ((uint64_t)nk * (uint64_t)(ldk > ldv ? ldk : ldv) * 2 >= (1ull << 31)) return VGGT_ERR_SHAPE;
  AttnArgs a{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, ldq, ldk, ldv, ldo,
             q_bstride, k_bstride, v_bstride, o_bstride, batch, heads, nq, nk,
             scale * 1.4426950408889634f, nullptr};
  // 8-wave workgroups (256 query rows) for long sequences; 4-wave ones
  // (128 rows) when the query count is short enough that the padding of a
  // 256-row block would cost more than the pairing gains.
  // 2-wave workgroups (64 query rows; only the default offset-free variant 33
  // is instantiated) for grids that fill a fraction of one round of slots.
  const bool two_ok = (g_vggt_attn_variant & 32) && (g_vggt_attn_variant & 65) == 1;
  const int nw = (g_vggt_attn_waves == 8 && nq >= 4096) ? 8 : (g_vggt_attn_waves == 2 && two_ok) ? 2 : 4;
  const int nwg = ((nq + nw * 32 - 1) / (nw * 32)) * heads * batch;
  hipStream_t s = (hipStream_t)stream;
  // 16x16x32 matrix-core form: variant 161 forces it; variant 33 takes it for
  // D = 64 when VGGT_ATTN16=1.  Off by default: faster back to back in kbench
  // (profiles/r6c: global 1.80 vs 1.83 ms, frame 128-134 vs 135-137 us) but not
  // in the model (r6d: global 1.87 vs 1.84 ms per launch, step 100.8 vs 100.5
  // ms, configs[3] 1329 vs 1299 ms)
  // VGGT_ATTN16=2: the 16x16 form only for the 4-wave (nq < 4096: frame / DINOv2) launches
  // (never with an lse: the training recompute, vggt_attention_fwd_lse, always
  // takes the exact-score 32x32 form whose lse the backward recomputes bit for bit)
  const bool use16 = a.lse == nullptr && D == 64 && nw != 2 &&
                     (g_vggt_attn_variant == 161 ||
                      (g_vggt_attn_variant == 33 && (g_vggt_attn16 == 1 || (g_vggt_attn16 == 2 && nw == 4))));
  if (use16) {
    if (nw == 8) attn16_fwd_kernel<8><<<nwg, 512, 0, s>>>(a);
    else attn16_fwd_kernel<4><<<nwg, 256, 0, s>>>(a);
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if ((g_vggt_attn_variant == 19 || g_vggt_attn_variant == 23) && D == 64 && nw != 2) {  // pipelined QK^T (3 LDS slots)
    if (nw == 8 && g_vggt_attn_variant == 23) attn_fwd_kernel<64, 8, 23><<<nwg, 512, 0, s>>>(a);
    else if (nw == 8) attn_fwd_kernel<64, 8, 19><<<nwg, 512, 0, s>>>(a);
    else if (g_vggt_attn_variant == 23) attn_fwd_kernel<64, 4, 23><<<nwg, 256, 0, s>>>(a);
    else attn_fwd_kernel<64, 4, 19><<<nwg, 256, 0, s>>>(a);
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  // Default (round 6): the 8-wave D = 64 form of variant 33 issues its LDS-DMA from the
  // priority half only (variant 2081): global attention 1,858-1,860 -> 1,814-1,819 us,
  // aggregator step 97.66-97.75 -> 96.56-97.21 ms, interleaved on one box
  // (profiles/r11/ab_attn_dma_half.md).  VGGT_ATTN_DMA_HALF=0: every wave issues its piece.
  static const bool dma_half = getenv("VGGT_ATTN_DMA_HALF") ? atoi(getenv("VGGT_ATTN_DMA_HALF")) != 0 : true;
  if (dma_half && g_vggt_attn_variant == 33 && D == 64 && nw == 8 && !a.lse) {
    attn_fwd_kernel<64, 8, 2081><<<nwg, 512, 0, s>>>(a);
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if (g_vggt_attn_variant == 4129 && D == 64 && nw != 2 && !a.lse) {  // 33 without the priority raise (8-wave form)
    if (nw == 8) attn_fwd_kernel<64, 8, 4129><<<nwg, 512, 0, s>>>(a);
    else attn_fwd_kernel<64, 4, 33><<<nwg, 256, 0, s>>>(a);
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if (g_vggt_attn_variant == 2081 && D == 64 && nw != 2 && !a.lse) {  // 33, DMA by the priority half (8-wave form)
    if (nw == 8) attn_fwd_kernel<64, 8, 2081><<<nwg, 512, 0, s>>>(a);
    else attn_fwd_kernel<64, 4, 33><<<nwg, 256, 0, s>>>(a);
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if (g_vggt_attn_variant == 545 && D == 64 && nw != 2 && !a.lse) {  // offset-free, 3 slots, DMA two tiles ahead
    if (nw == 8) attn_fwd_kernel<64, 8, 545><<<nwg, 512, 0, s>>>(a);
    else attn_fwd_kernel<64, 4, 545><<<nwg, 256, 0, s>>>(a);
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if (g_vggt_attn_variant == 289 && D == 64 && nw != 2 && !a.lse) {  // offset-free, split-tile pipelined
    if (nw == 8) attn_fwd_kernel<64, 8, 289><<<nwg, 512, 0, s>>>(a);
    else attn_fwd_kernel<64, 4, 289><<<nwg, 256, 0, s>>>(a);
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  if (g_vggt_attn_variant & 32) {  // offset-free softmax (bit 0 and the exact-score bit 64 combine)
    const int v = (g_vggt_attn_variant & 1) + ((g_vggt_attn_variant & 64) ? 2 : 0);
    switch ((D == 64 ? 0 : 16) + (nw == 8 ? 4 : nw == 2 ? 8 : 0) + v) {
#define VGGT_ATTN_SCASE(DD, NWW, V)                                                               \
  case (DD == 64 ? 0 : 16) + (NWW == 8 ? 4 : NWW == 2 ? 8 : 0) + V:                                \
    attn_fwd_kernel<DD, NWW, 32 + (V & 1) + ((V & 2) ? 64 : 0)><<<nwg, NWW * 64, 0, s>>>(a); \
    break;
      VGGT_ATTN_SCASE(64, 4, 0) VGGT_ATTN_SCASE(64, 4, 1) VGGT_ATTN_SCASE(64, 4, 2) VGGT_ATTN_SCASE(64, 4, 3)
      VGGT_ATTN_SCASE(64, 8, 0) VGGT_ATTN_SCASE(64, 8, 1) VGGT_ATTN_SCASE(64, 8, 2) VGGT_ATTN_SCASE(64, 8, 3)
      VGGT_ATTN_SCASE(128, 4, 0) VGGT_ATTN_SCASE(128, 4, 1) VGGT_ATTN_SCASE(128, 4, 2) VGGT_ATTN_SCASE(128, 4, 3)
      VGGT_ATTN_SCASE(128, 8, 0) VGGT_ATTN_SCASE(128, 8, 1) VGGT_ATTN_SCASE(128, 8, 2) VGGT_ATTN_SCASE(128, 8, 3)
      VGGT_ATTN_SCASE(64, 2, 1) VGGT_ATTN_SCASE(128, 2, 1)
#undef VGGT_ATTN_SCASE
      default: return VGGT_ERR_UNSUPPORTED;
    }
    HIP_LAUNCH_CHECK();
    return VGGT_OK;
  }
  switch ((D == 64 ? 0 : 32) + (nw == 8 ? 16 : 0) + (g_vggt_attn_variant & 15)) {
#define VGGT_ATTN_CASE(DD, NWW, V) \
  case (DD == 64 ? 0 : 32) + (NWW == 8 ? 16 : 0) + V: attn_fwd_kernel<DD, NWW, V><<<nwg, NWW * 64, 0, s>>>(a); break;
#define VGGT_ATTN_CASES(DD, NWW)                                                                            \
  VGGT_ATTN_CASE(DD, NWW, 0) VGGT_ATTN_CASE(DD, NWW, 1) VGGT_ATTN_CASE(DD, NWW, 2) VGGT_ATTN_CASE(DD, NWW, 3)  \
  VGGT_ATTN_CASE(DD, NWW, 4) VGGT_ATTN_CASE(DD, NWW, 5) VGGT_ATTN_CASE(DD, NWW, 6) VGGT_ATTN_CASE(DD, NWW, 7)  \
  VGGT_ATTN_CASE(DD, NWW, 8) VGGT_ATTN_CASE(DD, NWW, 9) VGGT_ATTN_CASE(DD, NWW, 10) VGGT_ATTN_CASE(DD, NWW, 11) \
  VGGT_ATTN_CASE(DD, NWW, 12) VGGT_ATTN_CASE(DD, NWW, 13) VGGT_ATTN_CASE(DD, NWW, 14) VGGT_ATTN_CASE(DD, NWW, 15)
    VGGT_ATTN_CASES(64, 4)
    VGGT_ATTN_CASES(64, 8)
    VGGT_ATTN_CASES(128, 4)
    VGGT_ATTN_CASES(128, 8)
#undef VGGT_ATTN_CASES
#undef VGGT_ATTN_CASE
    default: return VGGT_ERR_UNSUPPORTED;
  }
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

// Training recompute (alignment-head frame blocks under checkpoint, SURVEY §8f
// row 4): the exact-score offset-free form (variant 96: no Q prescale, so the
// backward's recomputed scores match bit for bit) that also stores the per-row
// log2-sum-exp consumed by vggt_attention_bwd.
// Diagnostic: the default forward (variant 33 -- 2081 in the 8-wave form unless
// VGGT_ATTN_DMA_HALF=0 --, 32x32x16 form, the same 8- / 4-wave choice as
// vggt_attention_fwd) with s_memtime segment stamps (VAR bit 1024).
extern "C" int vggt_attention_stamps(const void* q, int64_t ldq, int64_t q_bstride, const void* k, int64_t ldk,
                                     int64_t k_bstride, const void* v, int64_t ldv, int64_t v_bstride, void* o,
                                     int64_t ldo, int64_t o_bstride, unsigned long long* stamps, int batch, int heads,
                                     int nq, int nk, float scale, void* stream) {
  if (batch <= 0 || heads <= 0 || nq <= 0 || nk <= 0 || !stamps) return VGGT_ERR_SHAPE;
  if ((ldq | ldk | ldv | ldo) % 8 || ((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) % 16)
    return VGGT_ERR_ALIGN;
  if ((uint64_t)nk * (uint64_t)(ldk > ldv ? ldk : ldv) * 2 >= (1ull << 31)) return VGGT_ERR_SHAPE;
  AttnArgs a{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, ldq, ldk, ldv, ldo,
             q_bstride, k_bstride, v_bstride, o_bstride, batch, heads, nq, nk,
             scale * 1.4426950408889634f, (float*)(void*)stamps};
  const int nw = (g_vggt_attn_waves == 8 && nq >= 4096) ? 8 : 4;
  const int nwg = ((nq + nw * 32 - 1) / (nw * 32)) * heads * batch;
  hipStream_t s = (hipStream_t)stream;
  static const bool dma_half = getenv("VGGT_ATTN_DMA_HALF") ? atoi(getenv("VGGT_ATTN_DMA_HALF")) != 0 : true;
  if (nw == 8 && (g_vggt_attn_variant == 2081 || (g_vggt_attn_variant == 33 && dma_half)))
    attn_fwd_kernel<64, 8, 2081 | 1024><<<nwg, 512, 0, s>>>(a);
  else if (nw == 8 && g_vggt_attn_variant == 4129) attn_fwd_kernel<64, 8, 4129 | 1024><<<nwg, 512, 0, s>>>(a);
  else if (nw == 8) attn_fwd_kernel<64, 8, 33 | 1024><<<nwg, 512, 0, s>>>(a);
  else attn_fwd_kernel<64, 4, 33 | 1024><<<nwg, 256, 0, s>>>(a);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_attention_fwd_lse(const void* q, int64_t ldq, int64_t q_bstride, const void* k, int64_t ldk,
                                      int64_t k_bstride, const void* v, int64_t ldv, int64_t v_bstride, void* o,
                                      int64_t ldo, int64_t o_bstride, float* lse, int batch, int heads, int nq, int nk,
                                      int D, float scale, void* stream) {
  if (batch <= 0 || heads <= 0 || nq <= 0 || nk <= 0 || !lse) return VGGT_ERR_SHAPE;
  if (D != 64 && D != 128) return VGGT_ERR_UNSUPPORTED;
  if ((ldq | ldk | ldv | ldo) % 8 || ((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) % 16)
    return VGGT_ERR_ALIGN;
  if ((uint64_t)nk * (uint64_t)(ldk > ldv ? ldk : ldv) * 2 >= (1ull << 31)) return VGGT_ERR_SHAPE;
  AttnArgs a{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, ldq, ldk, ldv, ldo,
             q_bstride, k_bstride, v_bstride, o_bstride, batch, heads, nq, nk,
             scale * 1.4426950408889634f, lse};
  const int nwg = ((nq + 127) / 128) * heads * batch;
  hipStream_t s = (hipStream_t)stream;
  if (D == 64) attn_fwd_kernel<64, 4, 96><<<nwg, 256, 0, s>>>(a);
  else attn_fwd_kernel<128, 4, 96><<<nwg, 256, 0, s>>>(a);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}
