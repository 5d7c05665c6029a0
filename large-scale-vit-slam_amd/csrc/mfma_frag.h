// 32x32x16 bf16 MFMA operand fragments from padded row-major LDS tiles,
// shared by the backward kernels (attention_bwd.hip, train.hip wgrad).
// Conventions (v_mfma_f32_32x32x16_bf16): A fragment lane l = row l&31,
// k = 8(l>>5) + j; B fragment lane l = column l&31, same k; accumulator
// column l&31, row (r&3) + 8(r>>2) + 4(l>>5).
#pragma once
#include "common.h"

namespace vggt_frag {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;


template <int D>
struct Geo {
  static constexpr int ROWP = D * 2 + 16;  // padded LDS row (bytes)
  static constexpr int NKS = D / 16;       // k-steps over the head dim
  static constexpr int NDB = D / 32;       // 32-wide output blocks over the head dim
  static constexpr int CPR = D / 8;        // 16-B chunks per row
};

// A/B fragment of a row-major LDS tile: lane l reads row (row0 + l&31),
// elements 16ks + 8(l>>5) .. +7  (the 32x32x16 operand layout).
template <int D>
__device__ __forceinline__ bf16x8 rowfrag(const char* tile, int row0, int ks, int lane) {
  return *(const bf16x8*)(tile + (row0 + (lane & 31)) * Geo<D>::ROWP + (16 * ks + 8 * (lane >> 5)) * 2);
}

// A fragment of X^T for a row-major LDS tile X[row][d]: rows d in
// [32db, 32db+32), k = tile rows 32kb + 16ss + {4hl + 0..3, 8 + 4hl + 0..3}
// -- the k permutation of a 32x32 accumulator's rows 16ss..16ss+15 packed as
// bf16x8 (attention.hip, O^T = V^T P^T).
template <int D>
__device__ __forceinline__ bf16x8 trfrag(const char* tile, int db, int kb, int ss, int lane) {
  const int hl = lane >> 5, g = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
  const int r0 = 32 * kb + 16 * ss + 4 * hl + qq;
  const int col = db * 32 + 16 * g + 4 * pp;
  const char* p0 = tile + r0 * Geo<D>::ROWP + col * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)LDS_PTR(p0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)LDS_PTR(p0 + 8 * Geo<D>::ROWP));
  return __builtin_bit_cast(bf16x8, (s16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// rows [r0, r0+nrows) of a strided bf16 [rows, D] operand -> padded LDS tile
// (zeros past `valid`)
template <int D>
__device__ __forceinline__ void stage_rows(char* tile, const bf16_t* src, int64_t ld, int r0, int nrows, int valid) {
  constexpr int CPR = Geo<D>::CPR;
  for (int i = threadIdx.x; i < nrows * CPR; i += blockDim.x) {
    const int row = i / CPR, ch = i % CPR;
    const int r = r0 + row;
    uint4 v = {0u, 0u, 0u, 0u};
    if (r < valid) v = *(const uint4*)(src + (int64_t)r * ld + ch * 8);
    *(uint4*)(tile + row * Geo<D>::ROWP + ch * 16) = v;
  }
}


__device__ __forceinline__ bf16x8 pack8(const f32x16& c, int ss) {
  bf16x8 t;
#pragma unroll
  for (int j = 0; j < 8; ++j) t[j] = (__bf16)c[8 * ss + j];
  return t;
}

}  // namespace vggt_frag
