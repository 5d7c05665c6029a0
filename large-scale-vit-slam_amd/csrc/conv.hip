// DPT head convolutions (include/vggt_mi355x.h: vggt_conv2d_f32,
// vggt_upsample_bilinear_f32, vggt_dpt_activate).
//
// The reference runs the DPT heads with autocast disabled
// (featureAligned_vggt.py:104), i.e. in fp32.  Two forms of one implicit GEMM
// over NHWC activations: exact-f32 MFMA (v_mfma_f32_16x16x4_f32,
// conv_f32_kernel) and split-bf16 (conv_bf16x3_kernel, below: fp32 operands
// as bf16 hi + lo pairs on the bf16 matrix path, ~2^-16 per product).
//   out[pixel, co] = sum_{ky,kx,ci} act(x[pixel@(ky,kx), ci]) * W[co, ky, kx, ci]
// K is ordered (ky, kx, ci) with Ci % 32 == 0, so every 32-wide K slice is one
// tap and a contiguous channel run (16-B loads, zero for padding taps).
// Block tile 128 pixels x 64 channels x 32 K, 4 waves (2x2), register-staged
// double buffer through XOR-swizzled LDS.  Fused epilogue: bias, ReLU,
// up to two residual adds (one optionally ReLU'd: the in-place-ReLU skip of
// DPT's ResidualConvUnit), a per-pixel positional table, and the
// pixel-shuffle store of a stride == kernel ConvTranspose2d.
#include <math.h>

#include "common.h"
#include "tune.h"

namespace {

constexpr int BM = 128, BN = 64, BK = 32, NT = 256;

struct ConvArgs {
  const float* x;
  const float* w;
  const float* bias;
  float* y;
  const float* res1;
  const float* res2;
  const float* pos;
  int64_t ldx, ldy, ldr1, ldr2;
  int nimg, hi, wi, ci, ho, wo, co, kh, kw, stride, pad;
  int relu_in, relu_out, res1_relu;
  int shuffle;  // >0: ConvT pixel shuffle factor s; co is then the per-tap output channels
  int ncols;    // GEMM N (= co, or s*s*co for the shuffle)
  // optional split output (the next conv's pre-split input): yh / yl = split(relu?(y))
  bf16_t* yh;
  bf16_t* yl;
  int64_t ldys;
  int split_relu;
};

// ---- shared epilogue: lane holds C[m = 4q + i][n = r16] of each 16x16 tile;
// bias, ReLU, positional table, residual adds, pixel-shuffle store
template <int NTN>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, const f32x4 (&acc)[4][NTN], int M, int m0, int n0,
                                              int wm, int wn, int r16, int q) {
#pragma unroll
  for (int nt = 0; nt < NTN; ++nt) {
    const int n = n0 + wn * NTN * 16 + nt * 16 + r16;
    if (n >= a.ncols) continue;
    int co = n, dy = 0, dx = 0;
    if (a.shuffle) {
      const int tap = n / a.co;
      co = n % a.co;
      dy = tap / a.shuffle;
      dx = tap % a.shuffle;
    }
    const float bv = a.bias ? a.bias[co] : 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 64 + mt * 16 + 4 * q + i;
        if (m >= M) continue;
        float v = acc[mt][nt][i] + bv;
        if (a.relu_out) v = fmaxf(v, 0.f);
        int64_t opix;
        if (a.shuffle) {
          const int img = m / (a.ho * a.wo), rem = m % (a.ho * a.wo);
          const int oy = (rem / a.wo) * a.shuffle + dy, ox = (rem % a.wo) * a.shuffle + dx;
          opix = ((int64_t)img * a.ho * a.shuffle + oy) * (a.wo * a.shuffle) + ox;
        } else {
          opix = m;
          if (a.pos) v += a.pos[(int64_t)(m % (a.ho * a.wo)) * a.co + co];
          if (a.res1) {
            const float r = a.res1[(int64_t)m * a.ldr1 + co];
            v += a.res1_relu ? fmaxf(r, 0.f) : r;
          }
          if (a.res2) v += a.res2[(int64_t)m * a.ldr2 + co];
        }
        if (a.y) a.y[opix * a.ldy + co] = v;
        if (a.yh) {
          const float sv = a.split_relu ? fmaxf(v, 0.f) : v;
          const float hv = round_bf(sv);
          a.yh[opix * a.ldys + co] = f2bf(hv);
          a.yl[opix * a.ldys + co] = f2bf(sv - hv);
        }
      }
  }
}

__global__ __launch_bounds__(NT, 2) void conv_f32_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) float As[2][BM * BK];
  __shared__ __attribute__((aligned(16))) float Ws[2][BN * BK];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int M = a.nimg * a.ho * a.wo;
  const int tiles_n = (a.ncols + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * BM;
  const int n0 = (t % tiles_n) * BN;
  const int K = a.kh * a.kw * a.ci;
  const int nk = K / BK;

  // per-thread A rows: r = tid/8 + 32*i, channel quad c4 = tid%8
  const int c4 = tid & 7;
  int pn[4], py[4], px[4];
  bool pv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    pv[i] = m < M;
    const int mm = pv[i] ? m : 0;
    pn[i] = mm / (a.ho * a.wo);
    const int rem = mm % (a.ho * a.wo);
    py[i] = (rem / a.wo) * a.stride - a.pad;
    px[i] = (rem % a.wo) * a.stride - a.pad;
  }
  // per-thread W rows: r = tid/8 + 32*i (i < 2)
  f32x4 ra[4], rw[2];

  auto load = [&](int kt) {
    const int k0 = kt * BK;
    const int tap = k0 / a.ci;
    const int ci0 = k0 % a.ci + c4 * 4;
    const int ky = tap / a.kw, kx = tap % a.kw;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int iy = py[i] + ky, ix = px[i] + kx;
      if (pv[i] && iy >= 0 && iy < a.hi && ix >= 0 && ix < a.wi) {
        f32x4 v = *(const f32x4*)(a.x + (((int64_t)pn[i] * a.hi + iy) * a.wi + ix) * a.ldx + ci0);
        if (a.relu_in) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
        }
        ra[i] = v;
      } else {
        ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = n0 + (tid >> 3) + 32 * i;  // weights are padded to a multiple of BN rows
      rw[i] = *(const f32x4*)(a.w + (int64_t)n * K + k0 + c4 * 4);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (tid >> 3) + 32 * i;
      *(f32x4*)(&As[buf][r * BK + ((c4 ^ (r & 7)) << 2)]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (tid >> 3) + 32 * i;
      *(f32x4*)(&Ws[buf][r * BK + ((c4 ^ (r & 7)) << 2)]) = rw[i];
    }
  };

  const int wm = wave >> 1, wn = wave & 1;
  const int r16 = lane & 15, q = lane >> 4;
  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load(kt + 1);
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      const int ch = kc * 4 + q;
      f32x4 af[4], wf[2];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int r = wm * 64 + mt * 16 + r16;
        af[mt] = *(const f32x4*)(&As[cur][r * BK + ((ch ^ (r & 7)) << 2)]);
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int r = wn * 32 + nt * 16 + r16;
        wf[nt] = *(const f32x4*)(&Ws[cur][r * BK + ((ch ^ (r & 7)) << 2)]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mt][j], wf[nt][j], acc[mt][nt], 0, 0, 0);
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

  conv_epilogue(a, acc, M, m0, n0, wm, wn, r16, q);
}


// ===========================================================================
// Split-bf16 ("bf16x3") form of the same implicit GEMM: every fp32 operand is
// split as x = hi + lo with hi = bf16(x), lo = bf16(x - hi) (16 significant
// bits), and the product is accumulated in fp32 as hi.hi + hi.lo + lo.hi on
// v_mfma_f32_16x16x32_bf16 (the dropped lo.lo term and the split residue are
// ~2^-16 relative).  Three bf16 MFMAs replace eight f32 ones per 32-deep K
// slice, so the conv runs on the 2.5 PF bf16 matrix path instead of the
// 157 TF f32 one.  Weights come pre-split (vggt_split_bf16x2); activations
// are split on the fly after the (optional) input ReLU.
// LDS: 64-B rows (32 bf16), swizzle chunk ^ h((row>>2)&3), h = {0,3,2,1}:
// conflict-free ds_read_b128 fragment reads (as the GEMM ring).
// ===========================================================================
__device__ __forceinline__ int swz64(int row, int chunk) { return chunk ^ ((4 - ((row >> 2) & 3)) & 3); }

typedef int int32x4c __attribute__((ext_vector_type(4)));

// 16 B per lane from (rsrc, voff + soff) into LDS at the wave-uniform address
// `lds` (+ lane * 16): buffer_load ... lds (LDS-DMA).  In asm so the
// compiler does not drain vmcnt around it; completion is waited for
// explicitly before the barrier that publishes the stage.
__device__ __forceinline__ void cdma16(int32x4c rsrc, uint32_t voff, uint32_t soff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
               : "memory");
}

template <int BNX, bool PF2>
__global__ __launch_bounds__(NT, 2) void conv_bf16x3_kernel(ConvArgs a, const bf16_t* __restrict__ whi,
                                                            const bf16_t* __restrict__ wlo, uint32_t xbytes) {
  constexpr int NTN = BNX / 32;                       // 16-col fragments per wave (2 waves along N)
  constexpr int AT = BM * BK * 2, WT = BNX * BK * 2;  // bytes of one bf16 A / W tile
  constexpr int STG = 2 * AT + 2 * WT;               // Ahi, Alo, Whi, Wlo
  constexpr int WPW = WT / 1024 / 4 > 0 ? WT / 1024 / 4 : 1;  // W DMA pieces per wave per half (BNX 32: waves 0-1)
  __shared__ __attribute__((aligned(16))) char smem[2 * STG];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = a.nimg * a.ho * a.wo;
  const int tiles_n = (a.ncols + BNX - 1) / BNX;
  const int tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * BM;
  const int n0 = (t % tiles_n) * BNX;
  const int K = a.kh * a.kw * a.ci;
  const int nk = K / BK;
  // K-step order: channel slice outer, tap inner.  Step s covers tap s % ntap
  // and channels (s / ntap)*32 .. +32, i.e. weight columns tap*ci + slice*32
  // (the (ky, kx, ci) weight layout is unchanged).  The ntap consecutive steps
  // of one slice gather overlapping input windows (3x3 shifts of the same
  // pixels and channels), so the gather hits L2 instead of re-streaming the
  // activation from HBM once per tap.
  const int ntap = a.kh * a.kw;
  auto kcol = [&](int s) { return (s % ntap) * a.ci + (s / ntap) * BK; };

  // A: rows r = tid/8 + 32*i, fp32 channel quad c4 = tid%8 (4 K values)
  const int c4 = tid & 7;
  int pn[4], py[4], px[4];
  bool pv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    pv[i] = m < M;
    const int mm = pv[i] ? m : 0;
    pn[i] = mm / (a.ho * a.wo);
    const int rem = mm % (a.ho * a.wo);
    py[i] = (rem / a.wo) * a.stride - a.pad;
    px[i] = (rem % a.wo) * a.stride - a.pad;
  }
  // W (pre-split bf16, rows padded to a multiple of 128) by LDS-DMA: piece p
  // (1 KiB) of a half = rows 16p..16p+15 (64-B rows); lane -> row 16p + lane/4,
  // LDS chunk lane%4, which must hold global chunk (lane%4) ^ h(row) -- the
  // swz64 swizzle applied on the source address (the DMA image is lane-linear).
  const bool wdma = wave * WPW * 1024 < WT;
  uint32_t woff[WPW];
#pragma unroll
  for (int i = 0; i < WPW; ++i) {
    const int row = (wave * WPW + i) * 16 + (lane >> 2);
    const int g = swz64(row, lane & 3);
    woff[i] = (uint32_t)(row * K + g * 8) * 2u;
  }
  int32x4c rwh, rwl;
  {
    const uint64_t bh = (uint64_t)(whi + (int64_t)n0 * K), bl = (uint64_t)(wlo + (int64_t)n0 * K);
    rwh[0] = __builtin_amdgcn_readfirstlane((uint32_t)bh);
    rwh[1] = __builtin_amdgcn_readfirstlane((uint32_t)(bh >> 32)) & 0xffff;
    rwl[0] = __builtin_amdgcn_readfirstlane((uint32_t)bl);
    rwl[1] = __builtin_amdgcn_readfirstlane((uint32_t)(bl >> 32)) & 0xffff;
    rwh[2] = rwl[2] = -1;
    rwh[3] = rwl[3] = 0x00020000;
  }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));
  auto wstage = [&](int buf, int kt) {
    if (!wdma) return;
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(kcol(kt) * 2));
    const uint32_t b = lds0 + buf * STG + 2 * AT + wave * WPW * 1024;
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      cdma16(rwh, woff[i], soff, b + i * 1024);
      cdma16(rwl, woff[i], soff, b + WT + i * 1024);
    }
  };
  // A gather staged through registers, one K-step ahead: issued at the start
  // of step kt, split and stored at its end (no use of the loaded values in
  // between -- the input ReLU is applied at the store -- so the loads stay in
  // flight during the MFMAs)
  struct Stage {
    f32x4 ra[4];
  };
  Stage s0;

  auto load = [&](Stage& st, int kt) {
    f32x4 (&ra)[4] = st.ra;
    const int tap = kt % ntap;
    const int ci0 = (kt / ntap) * BK + c4 * 4;
    const int ky = tap / a.kw, kx = tap % a.kw;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int iy = py[i] + ky, ix = px[i] + kx;
      // no use of the loaded value here (the input ReLU is applied at the
      // store): the gather stays in flight for two MFMA steps
      ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (pv[i] && iy >= 0 && iy < a.hi && ix >= 0 && ix < a.wi)
        ra[i] = *(const f32x4*)(a.x + (((int64_t)pn[i] * a.hi + iy) * a.wi + ix) * a.ldx + ci0);
    }
  };
  // PF2: the gather as raw buffer loads -- every lane issues exactly its 4
  // loads (taps outside the image get an offset past num_records and read
  // zeros), so the K-loop can wait with a COUNTED vmcnt and keep the next
  // step's gather in flight across a barrier (two register stages)
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)xbytes, 0x00020000);
  auto load2 = [&](Stage& st, int kt) {
    const int tap = kt % ntap;
    const int ci0 = (kt / ntap) * BK + c4 * 4;
    const int ky = tap / a.kw, kx = tap % a.kw;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int iy = py[i] + ky, ix = px[i] + kx;
      const bool ok = pv[i] && iy >= 0 && iy < a.hi && ix >= 0 && ix < a.wi;
      const uint32_t off = ok ? (uint32_t)((((pn[i] * a.hi + iy) * a.wi + ix) * (uint32_t)a.ldx + ci0) * 4u)
                              : 0xfffffff0u;
      st.ra[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)off, 0, 0));
    }
  };
  auto store = [&](const Stage& st, int buf) {
    char* base = smem + buf * STG;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (tid >> 3) + 32 * i;
      uint2 h, l;
      float xv[4], hv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xv[j] = a.relu_in ? fmaxf(st.ra[i][j], 0.f) : st.ra[i][j];
        hv[j] = round_bf(xv[j]);
      }
      h.x = pack_bf2(hv[0], hv[1]);
      h.y = pack_bf2(hv[2], hv[3]);
      l.x = pack_bf2(xv[0] - hv[0], xv[1] - hv[1]);
      l.y = pack_bf2(xv[2] - hv[2], xv[3] - hv[3]);
      const int off = r * 64 + (swz64(r, c4 >> 1) << 4) + (c4 & 1) * 8;
      *(uint2*)(base + off) = h;
      *(uint2*)(base + AT + off) = l;
    }
  };

  const int wm = wave >> 1, wn = wave & 1;
  const int r16 = lane & 15, q = lane >> 4;
  const int roff = r16 * 64 + (swz64(r16, q) << 4);  // fragment read offset (row & 15 == r16)
  f32x4 acc[4][NTN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NTN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int cur) {
    const char* base = smem + cur * STG;
    bf16x8 ah[4], al[4], bh[NTN], bl[NTN];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int o = (wm * 64 + mt * 16) * 64 + roff;
      ah[mt] = *(const bf16x8*)(base + o);
      al[mt] = *(const bf16x8*)(base + AT + o);
    }
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) {
      const int o = (wn * NTN * 16 + nt * 16) * 64 + roff;
      bh[nt] = *(const bf16x8*)(base + 2 * AT + o);
      bl[nt] = *(const bf16x8*)(base + 2 * AT + WT + o);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NTN; ++nt) {
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[mt], bh[nt], acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bl[nt], acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bh[nt], acc[mt][nt], 0, 0, 0);
      }
  };

  // Per step kt (LDS buffer kt & 1): W DMA of tile kt+1 into the other
  // buffer, the A gather of tile kt+1 into registers, the MFMAs of tile kt,
  // the split + store of A tile kt+1, then every wave's DMA retired
  // (vmcnt(0)) before the barrier that publishes the next buffer.
  if constexpr (PF2) {
    // Two register stages, loop unrolled by two (s0 <-> buffer 0, s1 <->
    // buffer 1, no loop-carried copies): in step kt the gather of tile kt+2
    // is issued before the MFMAs of tile kt and stays in flight across the
    // step's barrier (vmcnt(4) = only this step's 4 gather loads may remain;
    // the W DMA and the previous gather are older).
    Stage s1;
    wstage(0, 0);
    load2(s0, 0);
    store(s0, 0);
    if (nk > 1) {
      load2(s1, 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // steady state: every operation unconditional, so the compiler's own
    // waitcnt tracking sees the same pending loads on both loop entries
    int kt = 0;
    for (; kt + 3 < nk; kt += 2) {
      wstage(1, kt + 1);
      load2(s0, kt + 2);
      compute(0);
      store(s1, 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      __syncthreads();
      wstage(0, kt + 2);
      load2(s1, kt + 3);
      compute(1);
      store(s0, 0);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      __syncthreads();
    }
    // the last 1-3 steps (no gather beyond tile kt+2)
    const bool h1 = kt + 1 < nk, h2 = kt + 2 < nk;
    if (h1) wstage(1, kt + 1);
    if (h2) load2(s0, kt + 2);
    compute(0);
    if (h1) {
      store(s1, 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (h2) wstage(0, kt + 2);
      compute(1);
      if (h2) {
        store(s0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        compute(0);
      }
    }
  } else {
  wstage(0, 0);
  load(s0, 0);
  store(s0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      wstage(cur ^ 1, kt + 1);
      load(s0, kt + 1);
    }
    compute(cur);
    if (kt + 1 < nk) store(s0, cur ^ 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  }

  conv_epilogue<NTN>(a, acc, M, m0, n0, wm, wn, r16, q);
}

// ===========================================================================
// Pre-split form (vggt_conv2d_bf16x3_pre): the activation arrives already
// split into bf16 hi / lo maps (vggt_split_act_bf16x2, input ReLU applied
// there), so the im2col gather is LDS-DMA like the weights -- per lane one
// 16-B piece of a 64-B (32-channel) pixel row, out-of-image taps get an offset
// past num_records and land as zeros.  The register-staged form above spends
// ~230 VALU instructions per wave per K-step on the gather addressing, the
// split and the LDS stores (4.75 per MFMA, VALU-issue-bound at 34% MFMA busy,
// 148^2 x 256 -> 256: profiles r3c); here the K-step is 8 DMA pieces and two
// address selects per wave.  Same K order, same MFMA sequence: bitwise equal
// to conv_bf16x3_kernel.
// ===========================================================================
template <int BNX>
__global__ __launch_bounds__(NT, 2) void conv_pre_kernel(ConvArgs a, const bf16_t* __restrict__ xhi,
                                                         const bf16_t* __restrict__ xlo, uint32_t xbytes,
                                                         const bf16_t* __restrict__ whi, const bf16_t* __restrict__ wlo) {
  constexpr int NTN = BNX / 32;
  constexpr int AT = BM * BK * 2, WT = BNX * BK * 2;
  constexpr int STG = 2 * AT + 2 * WT;  // Ahi, Alo, Whi, Wlo
  constexpr int WPW = WT / 1024 / 4 > 0 ? WT / 1024 / 4 : 1;
  constexpr int APW = AT / 1024 / 4;  // A pieces per wave per half (2)
  __shared__ __attribute__((aligned(16))) char smem[2 * STG];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = a.nimg * a.ho * a.wo;
  const int tiles_n = (a.ncols + BNX - 1) / BNX;
  const int tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * BM;
  const int n0 = (t % tiles_n) * BNX;
  const int K = a.kh * a.kw * a.ci;
  const int nk = K / BK;
  const int ntap = a.kh * a.kw;
  auto kcol = [&](int s) { return (s % ntap) * a.ci + (s / ntap) * BK; };

  // A pieces: rows (wave*APW + j)*16 + lane/4, LDS chunk lane%4 <- global chunk swz64(row, lane%4)
  int pb[APW], py[APW], px[APW];
#pragma unroll
  for (int j = 0; j < APW; ++j) {
    const int row = (wave * APW + j) * 16 + (lane >> 2);
    const int m = m0 + row;
    const int mm = m < M ? m : 0;
    const int img = mm / (a.ho * a.wo), rem = mm % (a.ho * a.wo);
    py[j] = (rem / a.wo) * a.stride - a.pad;
    px[j] = (rem % a.wo) * a.stride - a.pad;
    pb[j] = ((img * a.hi + py[j]) * a.wi + px[j]) * (int)a.ldx + swz64(row, lane & 3) * 8;
    if (m >= M) py[j] = -(1 << 20);  // rows past M: never inside the image (read as zeros)
  }
  uint32_t woff[WPW];
#pragma unroll
  for (int i = 0; i < WPW; ++i) {
    const int row = (wave * WPW + i) * 16 + (lane >> 2);
    woff[i] = (uint32_t)(row * K + swz64(row, lane & 3) * 8) * 2u;
  }
  const bool wdma = wave * WPW * 1024 < WT;
  auto rsrc = [](const void* p, uint32_t bytes) {
    int32x4c r;
    const uint64_t b = (uint64_t)p;
    r[0] = __builtin_amdgcn_readfirstlane((uint32_t)b);
    r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) & 0xffff;
    r[2] = (int)bytes;
    r[3] = 0x00020000;
    return r;
  };
  const int32x4c rwh = rsrc(whi + (int64_t)n0 * K, 0xffffffffu), rwl = rsrc(wlo + (int64_t)n0 * K, 0xffffffffu);
  const int32x4c rxh = rsrc(xhi, xbytes), rxl = rsrc(xlo, xbytes);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));
  auto stage = [&](int buf, int kt) {
    const uint32_t b = lds0 + buf * STG;
    const int tap = kt % ntap, ky = tap / a.kw, kx = tap % a.kw;
    const int sh = (ky * a.wi + kx) * (int)a.ldx + (kt / ntap) * BK;  // wave-uniform element shift
#pragma unroll
    for (int j = 0; j < APW; ++j) {
      const int iy = py[j] + ky, ix = px[j] + kx;
      const bool ok = (unsigned)iy < (unsigned)a.hi && (unsigned)ix < (unsigned)a.wi;
      const uint32_t off = ok ? (uint32_t)(pb[j] + sh) * 2u : 0xfffffff0u;
      cdma16(rxh, off, 0, b + (wave * APW + j) * 1024);
      cdma16(rxl, off, 0, b + AT + (wave * APW + j) * 1024);
    }
    if (wdma) {
      const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(kcol(kt) * 2));
#pragma unroll
      for (int i = 0; i < WPW; ++i) {
        cdma16(rwh, woff[i], soff, b + 2 * AT + (wave * WPW + i) * 1024);
        cdma16(rwl, woff[i], soff, b + 2 * AT + WT + (wave * WPW + i) * 1024);
      }
    }
  };

  const int wm = wave >> 1, wn = wave & 1;
  const int r16 = lane & 15, q = lane >> 4;
  const int roff = r16 * 64 + (swz64(r16, q) << 4);
  f32x4 acc[4][NTN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NTN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ah[4], al[4], bh[NTN], bl[NTN];
  auto reads = [&](int cur) {
    const char* base = smem + cur * STG;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int o = (wm * 64 + mt * 16) * 64 + roff;
      ah[mt] = *(const bf16x8*)(base + o);
      al[mt] = *(const bf16x8*)(base + AT + o);
    }
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) {
      const int o = (wn * NTN * 16 + nt * 16) * 64 + roff;
      bh[nt] = *(const bf16x8*)(base + 2 * AT + o);
      bl[nt] = *(const bf16x8*)(base + 2 * AT + WT + o);
    }
  };
  auto mfmas = [&]() {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NTN; ++nt) {
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[mt], bh[nt], acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bl[nt], acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bh[nt], acc[mt][nt], 0, 0, 0);
      }
  };

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
    reads(cur);
    mfmas();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  conv_epilogue<NTN>(a, acc, M, m0, n0, wm, wn, r16, q);
}

// hi / lo = split(relu?(x)) of a [rows, cols] f32 map with row stride ldx
// (cols % 4 == 0) into contiguous [rows, cols] bf16 maps
__global__ __launch_bounds__(256) void split_act_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows, int cols,
                                                        int relu, bf16_t* __restrict__ hi, bf16_t* __restrict__ lo) {
  const int c4n = cols / 4;
  const int64_t total = rows * c4n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / c4n;
    const int c = (int)(i - r * c4n) * 4;
    f32x4 v = *(const f32x4*)(x + r * ldx + c);
    float h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (relu) v[j] = fmaxf(v[j], 0.f);
      h[j] = round_bf(v[j]);
    }
    uint2 ph, pl;
    ph.x = pack_bf2(h[0], h[1]);
    ph.y = pack_bf2(h[2], h[3]);
    pl.x = pack_bf2(v[0] - h[0], v[1] - h[1]);
    pl.y = pack_bf2(v[2] - h[2], v[3] - h[3]);
    *(uint2*)(hi + r * cols + c) = ph;
    *(uint2*)(lo + r * cols + c) = pl;
  }
}

__global__ __launch_bounds__(256) void split_bf16x2_kernel(const float* __restrict__ x, int64_t n, bf16_t* __restrict__ hi,
                                                           bf16_t* __restrict__ lo) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    const float h = round_bf(v);
    hi[i] = f2bf(h);
    lo[i] = f2bf(v - h);
  }
}

// Bilinear resize, align_corners=True, NHWC f32 (F.interpolate semantics),
// optional positional table added to the result: [ho*wo, C] (pos_sep 0), or
// separable (pos_sep 1: DPT's UV sin/cos embedding, whose first C/2 channels
// depend on x only and the last C/2 on y only) as [wo + ho, C/2] = U rows
// then V rows -- 1/ho of the full table's bytes, which the full form re-reads
// for every frame (16 x 137 MB per 16-frame 518^2 chunk, profiles/r5c).
__global__ __launch_bounds__(256) void upsample_kernel(const float* __restrict__ x, int nimg, int hi, int wi, int C,
                                                       float* __restrict__ y, int ho, int wo,
                                                       const float* __restrict__ pos, bf16_t* __restrict__ yh,
                                                       bf16_t* __restrict__ yl, int split_relu, int pos_sep = 0) {
  const int c4n = C / 4;
  const int64_t total = (int64_t)nimg * ho * wo * c4n;
  const float sh = ho > 1 ? (float)(hi - 1) / (float)(ho - 1) : 0.f;
  const float sw = wo > 1 ? (float)(wi - 1) / (float)(wo - 1) : 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % c4n) * 4;
    const int64_t p = i / c4n;
    const int img = (int)(p / ((int64_t)ho * wo));
    const int rem = (int)(p % ((int64_t)ho * wo));
    const int oy = rem / wo, ox = rem % wo;
    const float fy = sh * oy, fx = sw * ox;
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = min(y0 + 1, hi - 1), x1 = min(x0 + 1, wi - 1);
    const float ly = fy - y0, lx = fx - x0;
    const float hy = 1.f - ly, hx = 1.f - lx;
    const float* b = x + (int64_t)img * hi * wi * C;
    const f32x4 v00 = *(const f32x4*)(b + ((int64_t)y0 * wi + x0) * C + c);
    const f32x4 v01 = *(const f32x4*)(b + ((int64_t)y0 * wi + x1) * C + c);
    const f32x4 v10 = *(const f32x4*)(b + ((int64_t)y1 * wi + x0) * C + c);
    const f32x4 v11 = *(const f32x4*)(b + ((int64_t)y1 * wi + x1) * C + c);
    f32x4 o = hy * (hx * v00 + lx * v01) + ly * (hx * v10 + lx * v11);
    if (pos) {
      if (pos_sep) {
        const int hc = C / 2;
        o += c < hc ? *(const f32x4*)(pos + (int64_t)ox * hc + c) : *(const f32x4*)(pos + (int64_t)(wo + oy) * hc + c - hc);
      } else {
        o += *(const f32x4*)(pos + (int64_t)rem * C + c);
      }
    }
    if (y) *(f32x4*)(y + p * C + c) = o;
    if (yh) {
      float h[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (split_relu) o[j] = fmaxf(o[j], 0.f);
        h[j] = round_bf(o[j]);
      }
      uint2 ph, pl;
      ph.x = pack_bf2(h[0], h[1]);
      ph.y = pack_bf2(h[2], h[3]);
      pl.x = pack_bf2(o[0] - h[0], o[1] - h[1]);
      pl.y = pack_bf2(o[2] - h[2], o[3] - h[3]);
      *(uint2*)(yh + p * C + c) = ph;
      *(uint2*)(yl + p * C + c) = pl;
    }
  }
}

// DPT activate_head: x [P, ncl] NHWC (last channel = confidence).
//   act 0: exp, 1: inv_log (sign(x)*expm1(|x|)); conf: 1 + exp(c) (expp1).
//   pts[p, j] = act(x[p, j]) * scale[img]   (j < ncl-1),  conf[p] = 1 + exp(x[p, ncl-1])
__global__ __launch_bounds__(256) void dpt_act_kernel(const float* __restrict__ x, int64_t ldx, int64_t npix,
                                                      int ppi, int ncl, int act, const float* __restrict__ scale,
                                                      float* __restrict__ pts, float* __restrict__ conf) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x) {
    const float s = scale ? scale[p / ppi] : 1.f;
    for (int j = 0; j < ncl - 1; ++j) {
      const float v = x[p * ldx + j];
      const float a = act == 0 ? expf(v) : copysignf(expm1f(fabsf(v)), v) * (v == 0.f ? 0.f : 1.f);
      pts[p * (ncl - 1) + j] = a * s;
    }
    conf[p] = 1.f + expf(x[p * ldx + ncl - 1]);
  }
}

inline int grid_for(int64_t total) {
  int64_t g = (total + 255) / 256;
  return (int)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" int vggt_conv2d_f32(const float* x, int64_t ldx, int nimg, int hi, int wi, int ci, const float* w,
                               const float* bias, int co, int kh, int kw, int stride, int pad, float* y, int64_t ldy,
                               int relu_in, int relu_out, const float* res1, int64_t ldr1, int res1_relu,
                               const float* res2, int64_t ldr2, const float* pos, int shuffle, void* stream) {
  if (nimg <= 0 || hi <= 0 || wi <= 0 || ci <= 0 || co <= 0 || kh <= 0 || kw <= 0 || stride <= 0 || pad < 0)
    return VGGT_ERR_SHAPE;
  if (ci % BK) return VGGT_ERR_SHAPE;
  if (shuffle && (kh != 1 || kw != 1 || stride != 1 || pad != 0 || res1 || res2 || pos)) return VGGT_ERR_UNSUPPORTED;
  if ((ldx % 4) || ((uintptr_t)x % 16) || ((uintptr_t)w % 16)) return VGGT_ERR_ALIGN;
  ConvArgs a;
  a.x = x; a.w = w; a.bias = bias; a.y = y; a.res1 = res1; a.res2 = res2; a.pos = pos;
  a.ldx = ldx; a.ldy = ldy; a.ldr1 = ldr1; a.ldr2 = ldr2;
  a.nimg = nimg; a.hi = hi; a.wi = wi; a.ci = ci;
  a.ho = (hi + 2 * pad - kh) / stride + 1;
  a.wo = (wi + 2 * pad - kw) / stride + 1;
  a.co = co; a.kh = kh; a.kw = kw; a.stride = stride; a.pad = pad;
  a.relu_in = relu_in; a.relu_out = relu_out; a.res1_relu = res1_relu;
  a.shuffle = shuffle;
  a.ncols = shuffle ? shuffle * shuffle * co : co;
  a.yh = a.yl = nullptr;
  a.ldys = 0;
  a.split_relu = 0;
  const int64_t M = (int64_t)nimg * a.ho * a.wo;
  const int64_t nwg = ((M + BM - 1) / BM) * ((a.ncols + BN - 1) / BN);
  if (nwg > 0x7fffffff) return VGGT_ERR_SHAPE;
  conv_f32_kernel<<<(int)nwg, NT, 0, (hipStream_t)stream>>>(a);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

static int conv_args(ConvArgs& a, const float* x, int64_t ldx, int nimg, int hi, int wi, int ci, const float* w,
                     const float* bias, int co, int kh, int kw, int stride, int pad, float* y, int64_t ldy, int relu_in,
                     int relu_out, const float* res1, int64_t ldr1, int res1_relu, const float* res2, int64_t ldr2,
                     const float* pos, int shuffle, int64_t* nwg) {
  if (nimg <= 0 || hi <= 0 || wi <= 0 || ci <= 0 || co <= 0 || kh <= 0 || kw <= 0 || stride <= 0 || pad < 0)
    return VGGT_ERR_SHAPE;
  if (ci % BK) return VGGT_ERR_SHAPE;
  if (shuffle && (kh != 1 || kw != 1 || stride != 1 || pad != 0 || res1 || res2 || pos)) return VGGT_ERR_UNSUPPORTED;
  if ((ldx % 4) || ((uintptr_t)x % 16)) return VGGT_ERR_ALIGN;
  a.x = x; a.w = w; a.bias = bias; a.y = y; a.res1 = res1; a.res2 = res2; a.pos = pos;
  a.ldx = ldx; a.ldy = ldy; a.ldr1 = ldr1; a.ldr2 = ldr2;
  a.nimg = nimg; a.hi = hi; a.wi = wi; a.ci = ci;
  a.ho = (hi + 2 * pad - kh) / stride + 1;
  a.wo = (wi + 2 * pad - kw) / stride + 1;
  a.co = co; a.kh = kh; a.kw = kw; a.stride = stride; a.pad = pad;
  a.relu_in = relu_in; a.relu_out = relu_out; a.res1_relu = res1_relu;
  a.shuffle = shuffle;
  a.ncols = shuffle ? shuffle * shuffle * co : co;
  a.yh = a.yl = nullptr;
  a.ldys = 0;
  a.split_relu = 0;
  const int64_t M = (int64_t)nimg * a.ho * a.wo;
  *nwg = ((M + BM - 1) / BM) * ((a.ncols + BN - 1) / BN);
  if (*nwg > 0x7fffffff) return VGGT_ERR_SHAPE;
  return VGGT_OK;
}

extern "C" int vggt_conv2d_bf16x3(const float* x, int64_t ldx, int nimg, int hi, int wi, int ci, const void* w_hi,
                                  const void* w_lo, const float* bias, int co, int kh, int kw, int stride, int pad,
                                  float* y, int64_t ldy, int relu_in, int relu_out, const float* res1, int64_t ldr1,
                                  int res1_relu, const float* res2, int64_t ldr2, const float* pos, int shuffle,
                                  void* stream) {
  ConvArgs a;
  int64_t nwg;
  const int rc = conv_args(a, x, ldx, nimg, hi, wi, ci, nullptr, bias, co, kh, kw, stride, pad, y, ldy, relu_in,
                           relu_out, res1, ldr1, res1_relu, res2, ldr2, pos, shuffle, &nwg);
  if (rc) return rc;
  if (((uintptr_t)w_hi % 16) || ((uintptr_t)w_lo % 16)) return VGGT_ERR_ALIGN;
  // 128-wide N tiles when there are at least 128 GEMM columns (more MFMA work
  // per split of the activation tile), else 64
  // two-deep gather (buffer loads with 32-bit byte offsets) when the input spans < 4 GiB
  const int64_t xb = ((int64_t)nimg * hi * wi - 1) * ldx * 4 + (int64_t)ci * 4;
  const bool pf2 = xb < (int64_t)0xffffff00ll && g_vggt_conv_pf2;
  const uint32_t xbytes = pf2 ? (uint32_t)xb : 0u;
  hipStream_t s = (hipStream_t)stream;
  const bf16_t *wh = (const bf16_t*)w_hi, *wl = (const bf16_t*)w_lo;
#define VGGT_CONV(BNX, G)                                                            \
  (pf2 ? conv_bf16x3_kernel<BNX, true><<<(int)(G), NT, 0, s>>>(a, wh, wl, xbytes)   \
       : conv_bf16x3_kernel<BNX, false><<<(int)(G), NT, 0, s>>>(a, wh, wl, xbytes))
  if (a.ncols >= 128) {
    const int64_t nw2 = (nwg / ((a.ncols + BN - 1) / BN)) * ((a.ncols + 127) / 128);
    VGGT_CONV(128, nw2);
  } else if (a.ncols > 32) {
    VGGT_CONV(64, nwg);
  } else {  // output_conv2 (128 -> 32): 32-wide N tiles, no padded MFMA columns
    VGGT_CONV(32, nwg);
  }
#undef VGGT_CONV
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_conv2d_bf16x3_pre(const void* x_hi, const void* x_lo, int64_t ldx, int nimg, int hi, int wi,
                                      int ci, const void* w_hi, const void* w_lo, const float* bias, int co, int kh,
                                      int kw, int stride, int pad, float* y, int64_t ldy, int relu_out,
                                      const float* res1, int64_t ldr1, int res1_relu, const float* res2, int64_t ldr2,
                                      const float* pos, int shuffle, void* y_hi, void* y_lo, int64_t ldys,
                                      int split_relu, void* stream) {
  ConvArgs a;
  int64_t nwg;
  const int rc = conv_args(a, (const float*)x_hi, ldx, nimg, hi, wi, ci, nullptr, bias, co, kh, kw, stride, pad, y, ldy,
                           0, relu_out, res1, ldr1, res1_relu, res2, ldr2, pos, shuffle, &nwg);
  if (rc) return rc;
  if (!y && !y_hi) return VGGT_ERR_SHAPE;
  if (!y_hi != !y_lo || (y_hi && ldys < co)) return VGGT_ERR_SHAPE;
  a.yh = (bf16_t*)y_hi;
  a.yl = (bf16_t*)y_lo;
  a.ldys = ldys;
  a.split_relu = split_relu;
  if (((uintptr_t)x_lo % 16) || ((uintptr_t)w_hi % 16) || ((uintptr_t)w_lo % 16) || (ldx % 8)) return VGGT_ERR_ALIGN;
  // 32-bit byte offsets: the whole map (plus the widest tap shift) below 4 GiB
  const int64_t xb = ((int64_t)nimg * hi * wi - 1) * ldx * 2 + (int64_t)ci * 2;
  if (xb >= (int64_t)0x7fffff00ll) return VGGT_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  const bf16_t *xh = (const bf16_t*)x_hi, *xl = (const bf16_t*)x_lo;
  const bf16_t *wh = (const bf16_t*)w_hi, *wl = (const bf16_t*)w_lo;
  if (a.ncols >= 128) {
    const int64_t nw2 = (nwg / ((a.ncols + BN - 1) / BN)) * ((a.ncols + 127) / 128);
    conv_pre_kernel<128><<<(int)nw2, NT, 0, s>>>(a, xh, xl, (uint32_t)xb, wh, wl);
  } else if (a.ncols > 32) {
    conv_pre_kernel<64><<<(int)nwg, NT, 0, s>>>(a, xh, xl, (uint32_t)xb, wh, wl);
  } else {
    conv_pre_kernel<32><<<(int)nwg, NT, 0, s>>>(a, xh, xl, (uint32_t)xb, wh, wl);
  }
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_split_act_bf16x2(const float* x, int64_t ldx, int64_t rows, int cols, int relu, void* hi, void* lo,
                                     void* stream) {
  if (rows < 0 || cols <= 0 || cols % 4 || ldx < cols) return VGGT_ERR_SHAPE;
  if ((ldx % 4) || ((uintptr_t)x % 16) || ((uintptr_t)hi % 8) || ((uintptr_t)lo % 8)) return VGGT_ERR_ALIGN;
  if (rows == 0) return VGGT_OK;
  split_act_kernel<<<grid_for(rows * (cols / 4)), 256, 0, (hipStream_t)stream>>>(x, ldx, rows, cols, relu,
                                                                              (bf16_t*)hi, (bf16_t*)lo);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_split_bf16x2(const float* x, int64_t n, void* hi, void* lo, void* stream) {
  if (n < 0) return VGGT_ERR_SHAPE;
  if (n == 0) return VGGT_OK;
  split_bf16x2_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(x, n, (bf16_t*)hi, (bf16_t*)lo);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_upsample_bilinear_f32(const float* x, int nimg, int hi, int wi, int C, float* y, int ho, int wo,
                                          const float* pos, void* stream) {
  if (nimg <= 0 || hi <= 0 || wi <= 0 || ho <= 0 || wo <= 0 || C % 4) return VGGT_ERR_SHAPE;
  if (((uintptr_t)x | (uintptr_t)y) % 16) return VGGT_ERR_ALIGN;
  upsample_kernel<<<grid_for((int64_t)nimg * ho * wo * (C / 4)), 256, 0, (hipStream_t)stream>>>(x, nimg, hi, wi, C, y,
                                                                                                 ho, wo, pos, nullptr,
                                                                                                 nullptr, 0);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_upsample_bilinear_split(const float* x, int nimg, int hi, int wi, int C, float* y, int ho, int wo,
                                            const float* pos, void* y_hi, void* y_lo, int split_relu, void* stream) {
  if (nimg <= 0 || hi <= 0 || wi <= 0 || ho <= 0 || wo <= 0 || C % 4 || (!y && !y_hi) || (!y_hi != !y_lo))
    return VGGT_ERR_SHAPE;
  if (((uintptr_t)x | (uintptr_t)y) % 16 || ((uintptr_t)y_hi | (uintptr_t)y_lo) % 8) return VGGT_ERR_ALIGN;
  upsample_kernel<<<grid_for((int64_t)nimg * ho * wo * (C / 4)), 256, 0, (hipStream_t)stream>>>(
      x, nimg, hi, wi, C, y, ho, wo, pos, (bf16_t*)y_hi, (bf16_t*)y_lo, split_relu);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_upsample_bilinear_split_sep(const float* x, int nimg, int hi, int wi, int C, float* y, int ho,
                                                int wo, const float* pos_sep, void* y_hi, void* y_lo, int split_relu,
                                                void* stream) {
  if (nimg <= 0 || hi <= 0 || wi <= 0 || ho <= 0 || wo <= 0 || C % 8 || (!y && !y_hi) || (!y_hi != !y_lo) || !pos_sep)
    return VGGT_ERR_SHAPE;
  if (((uintptr_t)x | (uintptr_t)y | (uintptr_t)pos_sep) % 16 || ((uintptr_t)y_hi | (uintptr_t)y_lo) % 8)
    return VGGT_ERR_ALIGN;
  upsample_kernel<<<grid_for((int64_t)nimg * ho * wo * (C / 4)), 256, 0, (hipStream_t)stream>>>(
      x, nimg, hi, wi, C, y, ho, wo, pos_sep, (bf16_t*)y_hi, (bf16_t*)y_lo, split_relu, 1);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}

extern "C" int vggt_dpt_activate(const float* x, int64_t ldx, int64_t npix, int pix_per_img, int ncl, int act,
                                 const float* scale, float* pts, float* conf, void* stream) {
  if (npix <= 0 || ncl < 2 || pix_per_img <= 0 || (act != 0 && act != 1)) return VGGT_ERR_SHAPE;
  dpt_act_kernel<<<grid_for(npix), 256, 0, (hipStream_t)stream>>>(x, ldx, npix, pix_per_img, ncl, act, scale, pts,
                                                                  conf);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}
