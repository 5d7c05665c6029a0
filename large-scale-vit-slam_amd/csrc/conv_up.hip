// Fused last stage of the DPT head (vggt_conv2d_upsample_bf16x3):
//   y = conv3x3_pad1( split_bf16x2( resize_bilinear_align_corners(x, ho, wo) + pos ) )
// i.e. the output_conv1 -> F.interpolate(size = (H, W)) -> + _apply_pos_embed ->
// output_conv2[0] sequence of DPTHead.forward (dpt_head ext; featureAligned_vggt.py
// :166), without materialising the resized map: at 16 x 518^2 x 128 channels
// its split halves are 2.2 GB written by the upsample and gathered back by the
// convolution (profiles/r5c: upsample 1.1 ms at ~6.4 TB/s + conv 1.7 ms).
//
// Output tile: 4 rows x 32 columns of pixels (128 GEMM rows) x all co (<= 32).
// Per 32-channel slice the workgroup builds the (4+2) x (32+2) input patch of
// the resized map in LDS -- each patch pixel interpolated ONCE from the source
// map (the im2col form would interpolate it for every one of the 9 taps),
// positional table added, split into bf16 hi / lo exactly as the unfused
// upsample kernel does -- while the slice's 9 weight tiles arrive by LDS-DMA;
// then the 9 taps run as MFMAs whose A fragments are read straight out of the
// patch at the tap's (ky, kx) shift.  Products and K order (channel slice
// outer, tap inner) are those of conv_pre_kernel: split-bf16, hi.hi + hi.lo +
// lo.hi accumulated in fp32.
#include "common.h"

namespace {

constexpr int UT_R = 4, UT_C = 32;              // output tile rows x columns (128 pixels)
constexpr int PR = UT_R + 2, PC = UT_C + 2;     // patch 6 x 34
constexpr int PP = PR * PC;                     // 204 patch pixels
constexpr int CS = 32;                          // channels per slice (one 32-deep K step per tap)
constexpr int PATCH = PP * CS * 2;              // bytes of one bf16 patch half
constexpr int UNT = 256;
constexpr int NTAP = 9;

// 64-B rows (32 bf16), swizzle chunk ^ h((row >> 2) & 3): conflict-free
// ds_read_b128 for any 16 consecutive rows (conv.hip swz64)
__device__ __forceinline__ int uswz(int row, int chunk) { return chunk ^ ((4 - ((row >> 2) & 3)) & 3); }

typedef int i32x4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void udma16(i32x4u rsrc, uint32_t voff, uint32_t soff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
               : "memory");
}

struct UpConvArgs {
  const float* x;        // source map [nimg, hi, wi, C] f32 (row stride C)
  const float* pos_sep;  // [wo + ho, C/2] separable positional table, or null
  const float* bias;     // [co] or null
  float* y;              // [nimg*ho*wo, ldy] f32 output, or null
  bf16_t* yh;            // split output halves of relu?(y), or null
  bf16_t* yl;
  int64_t ldy, ldys;
  int nimg, hi, wi, C, ho, wo, co, relu_out, split_relu;
};

template <int BNX>
__global__ __launch_bounds__(UNT, 2) void conv_up_kernel(UpConvArgs a, const bf16_t* __restrict__ whi,
                                                         const bf16_t* __restrict__ wlo) {
  constexpr int NTN = BNX / 32;
  constexpr int WT = BNX * CS * 2;  // one tap's weight tile, one half
  constexpr int WPIECES = 2 * NTAP * WT / 1024;       // 1-KiB DMA pieces per slice (hi + lo)
  constexpr int WPW = WPIECES / 4;                    // per wave
  static_assert(WPW * 4 == WPIECES, "weight pieces split evenly over the 4 waves");
  __shared__ __attribute__((aligned(16))) char smem[2 * PATCH + 2 * NTAP * WT];
  char* const ph = smem;
  char* const pl = smem + PATCH;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int C = a.C, K = NTAP * C;
  const int tiles_x = (a.wo + UT_C - 1) / UT_C, tiles_y = (a.ho + UT_R - 1) / UT_R;
  const int t = xcd_remap(blockIdx.x, a.nimg * tiles_y * tiles_x);
  const int img = t / (tiles_y * tiles_x), rem = t % (tiles_y * tiles_x);
  const int oy0 = (rem / tiles_x) * UT_R, ox0 = (rem % tiles_x) * UT_C;
  const float sh = a.ho > 1 ? (float)(a.hi - 1) / (float)(a.ho - 1) : 0.f;
  const float sw = a.wo > 1 ? (float)(a.wi - 1) / (float)(a.wo - 1) : 0.f;
  const float* xb = a.x + (int64_t)img * a.hi * a.wi * C;
  const int hc = C / 2;

  // weight pieces: piece q (0..WPIECES-1) of a slice = half q / (WPIECES/2),
  // tap (q % (WPIECES/2)) / (WT/1024), rows 16 * ((q % (WPIECES/2)) % (WT/1024)) + lane/4
  // (64-B rows), LDS chunk lane%4 <- global chunk uswz(row, lane%4) (swizzle on the source)
  auto rsrc = [](const void* p) {
    i32x4u r;
    const uint64_t b = (uint64_t)p;
    r[0] = __builtin_amdgcn_readfirstlane((uint32_t)b);
    r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) & 0xffff;
    r[2] = -1;
    r[3] = 0x00020000;
    return r;
  };
  const i32x4u rwh = rsrc(whi), rwl = rsrc(wlo);
  uint32_t woff[WPW];
  bool wlo_piece[WPW];
  uint32_t wdst[WPW];
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(smem));
#pragma unroll
  for (int i = 0; i < WPW; ++i) {
    const int q = wave * WPW + i;
    const int hl = q / (WPIECES / 2), qq = q % (WPIECES / 2);
    const int tap = qq / (WT / 1024), sub = qq % (WT / 1024);
    const int row = sub * 16 + (lane >> 2);
    woff[i] = (uint32_t)(row * K + tap * C + uswz(row, lane & 3) * 8) * 2u;
    wlo_piece[i] = hl != 0;
    wdst[i] = lds0 + 2 * PATCH + (hl * NTAP + tap) * WT + sub * 1024;
  }

  // MFMA fragment geometry (conv_pre_kernel's): waves 2 (M) x 2 (N), lane
  // r16 = row within a 16-row fragment, q = 16-B chunk of the 32 channels
  const int wm = wave >> 1, wn = wave & 1;
  const int r16 = lane & 15, qc = lane >> 4;
  int pbase[4];  // patch pixel of fragment row r16 at tap (0, 0)
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int r = wm * 64 + mt * 16 + r16;
    pbase[mt] = (r >> 5) * PC + (r & 31);
  }
  const int roff_w = r16 * 64 + (uswz(r16, qc) << 4);
  f32x4 acc[4][NTN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NTN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nslice = C / CS;
  for (int s = 0; s < nslice; ++s) {
    // this slice's 9 weight tiles by LDS-DMA (in flight during the patch build)
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(s * CS * 2));
#pragma unroll
    for (int i = 0; i < WPW; ++i) udma16(wlo_piece[i] ? rwl : rwh, woff[i], soff, wdst[i]);
    // the resized + positional + split patch: item = (patch pixel, 8-channel chunk)
    for (int it = tid; it < PP * 4; it += UNT) {
      const int pidx = it >> 2, cc = it & 3;
      const int iy = oy0 - 1 + pidx / PC, ix = ox0 - 1 + pidx % PC;
      uint4 hv = {0u, 0u, 0u, 0u}, lv = {0u, 0u, 0u, 0u};
      if (iy >= 0 && iy < a.ho && ix >= 0 && ix < a.wo) {
        const int c = s * CS + cc * 8;
        const float fy = sh * iy, fx = sw * ix;
        const int y0 = (int)fy, x0 = (int)fx;
        const int y1 = min(y0 + 1, a.hi - 1), x1 = min(x0 + 1, a.wi - 1);
        const float ly = fy - y0, lx = fx - x0;
        const float hy = 1.f - ly, hx = 1.f - lx;
        uint32_t hw[4], lw[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // two 4-channel halves, the upsample kernel's arithmetic
          const int ch = c + 4 * h;
          const f32x4 v00 = *(const f32x4*)(xb + ((int64_t)y0 * a.wi + x0) * C + ch);
          const f32x4 v01 = *(const f32x4*)(xb + ((int64_t)y0 * a.wi + x1) * C + ch);
          const f32x4 v10 = *(const f32x4*)(xb + ((int64_t)y1 * a.wi + x0) * C + ch);
          const f32x4 v11 = *(const f32x4*)(xb + ((int64_t)y1 * a.wi + x1) * C + ch);
          f32x4 o = hy * (hx * v00 + lx * v01) + ly * (hx * v10 + lx * v11);
          if (a.pos_sep)
            o += ch < hc ? *(const f32x4*)(a.pos_sep + (int64_t)ix * hc + ch)
                         : *(const f32x4*)(a.pos_sep + (int64_t)(a.wo + iy) * hc + ch - hc);
          float hf[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) hf[j] = round_bf(o[j]);
          hw[2 * h] = pack_bf2(hf[0], hf[1]);
          hw[2 * h + 1] = pack_bf2(hf[2], hf[3]);
          lw[2 * h] = pack_bf2(o[0] - hf[0], o[1] - hf[1]);
          lw[2 * h + 1] = pack_bf2(o[2] - hf[2], o[3] - hf[3]);
        }
        hv = uint4{hw[0], hw[1], hw[2], hw[3]};
        lv = uint4{lw[0], lw[1], lw[2], lw[3]};
      }
      const int off = pidx * 64 + (uswz(pidx, cc) << 4);
      *(uint4*)(ph + off) = hv;
      *(uint4*)(pl + off) = lv;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll 1
    for (int tap = 0; tap < NTAP; ++tap) {
      const int sh_ = (tap / 3) * PC + (tap % 3);
      const char* wb = smem + 2 * PATCH + tap * WT;
      bf16x8 ah[4], al[4], bh[NTN], bl[NTN];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int pp = pbase[mt] + sh_;
        const int o = pp * 64 + (uswz(pp, qc) << 4);
        ah[mt] = *(const bf16x8*)(ph + o);
        al[mt] = *(const bf16x8*)(pl + o);
      }
#pragma unroll
      for (int nt = 0; nt < NTN; ++nt) {
        const int o = (wn * NTN * 16 + nt * 16) * 64 + roff_w;
        bh[nt] = *(const bf16x8*)(wb + o);
        bl[nt] = *(const bf16x8*)(wb + NTAP * WT + o);
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt) {
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[mt], bh[nt], acc[mt][nt], 0, 0, 0);
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bl[nt], acc[mt][nt], 0, 0, 0);
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bh[nt], acc[mt][nt], 0, 0, 0);
        }
    }
    __syncthreads();  // every fragment read of this slice's patch / weights done
  }

  // epilogue: lane holds C[row 4q + i][col r16] of each 16 x 16 tile; tile row
  // r = pixel (oy0 + r / 32, ox0 + r % 32)
#pragma unroll
  for (int nt = 0; nt < NTN; ++nt) {
    const int n = wn * NTN * 16 + nt * 16 + r16;
    if (n >= a.co) continue;
    const float bv = a.bias ? a.bias[n] : 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + mt * 16 + 4 * qc + i;
        const int oy = oy0 + (r >> 5), ox = ox0 + (r & 31);
        if (oy >= a.ho || ox >= a.wo) continue;
        const int64_t opix = ((int64_t)img * a.ho + oy) * a.wo + ox;
        float v = acc[mt][nt][i] + bv;
        if (a.relu_out) v = fmaxf(v, 0.f);
        if (a.y) a.y[opix * a.ldy + n] = v;
        if (a.yh) {
          const float sv = a.split_relu ? fmaxf(v, 0.f) : v;
          const float hv = round_bf(sv);
          a.yh[opix * a.ldys + n] = f2bf(hv);
          a.yl[opix * a.ldys + n] = f2bf(sv - hv);
        }
      }
  }
}

}  // namespace

extern "C" int vggt_conv2d_upsample_bf16x3(const float* x, int nimg, int hi, int wi, int C, const float* pos_sep,
                                           int ho, int wo, const void* w_hi, const void* w_lo, const float* bias,
                                           int co, int relu_out, float* y, int64_t ldy, void* y_hi, void* y_lo,
                                           int64_t ldys, int split_relu, void* stream) {
  if (nimg <= 0 || hi <= 0 || wi <= 0 || ho <= 0 || wo <= 0 || C <= 0 || C % CS || co <= 0 || co > 32)
    return VGGT_ERR_SHAPE;
  if (!y && !y_hi) return VGGT_ERR_SHAPE;
  if (!y_hi != !y_lo || (y && ldy < co) || (y_hi && ldys < co)) return VGGT_ERR_SHAPE;
  if ((int64_t)31 * 9 * C + 9 * C > 0x3fffffff) return VGGT_ERR_SHAPE;
  if (((uintptr_t)x | (uintptr_t)pos_sep) % 16 || ((uintptr_t)w_hi | (uintptr_t)w_lo) % 16) return VGGT_ERR_ALIGN;
  UpConvArgs a;
  a.x = x;
  a.pos_sep = pos_sep;
  a.bias = bias;
  a.y = y;
  a.yh = (bf16_t*)y_hi;
  a.yl = (bf16_t*)y_lo;
  a.ldy = ldy;
  a.ldys = ldys;
  a.nimg = nimg;
  a.hi = hi;
  a.wi = wi;
  a.C = C;
  a.ho = ho;
  a.wo = wo;
  a.co = co;
  a.relu_out = relu_out;
  a.split_relu = split_relu;
  const int64_t nwg = (int64_t)nimg * ((ho + UT_R - 1) / UT_R) * ((wo + UT_C - 1) / UT_C);
  if (nwg > 0x7fffffff) return VGGT_ERR_SHAPE;
  conv_up_kernel<32><<<(int)nwg, UNT, 0, (hipStream_t)stream>>>(a, (const bf16_t*)w_hi, (const bf16_t*)w_lo);
  HIP_LAUNCH_CHECK();
  return VGGT_OK;
}
