/*
 * vggt_mi355x.h -- C ABI of the MI355X (gfx950) hot path for the per-chunk
 * VGGT forward + feature-alignment head of ruppelb/Large-Scale-ViT-SLAM.
 *
 * The reference has no FFI: every op on its hot path is a stock PyTorch op
 * called from Python.  Each entry point below replaces one
 * such op (or a fused group of them); the reference call site it stands in
 * for is cited per function.  All pointers are DEVICE pointers owned by the
 * caller; nothing here allocates.  `stream` is a hipStream_t passed as void*.
 * Every function returns VGGT_OK (0) or a negative error code and never
 * throws; the Python host layer turns codes into RuntimeError, mirroring the
 * reference's assert/ValueError conventions (alignment_head.py:86,:251;
 * cross_attention.py:30,:50).
 *
 * Data types: "bf16" buffers hold raw bfloat16 bits (uint16); "f32" is IEEE
 * float.  Leading dimensions (ld*) are in ELEMENTS.  Row-major everywhere.
 */
#ifndef VGGT_MI355X_H
#define VGGT_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VGGT_OK 0
#define VGGT_ERR_SHAPE (-1)       /* unsupported / inconsistent shape        */
#define VGGT_ERR_ALIGN (-2)       /* pointer or leading dim misaligned       */
#define VGGT_ERR_HIP (-3)         /* HIP launch / runtime error              */
#define VGGT_ERR_UNSUPPORTED (-4) /* unsupported mode / dtype                */

#define VGGT_DTYPE_F32 0
#define VGGT_DTYPE_BF16 1

/* GEMM epilogues (all round acc+bias to bf16 first, = autocast Linear out) */
#define VGGT_EPI_BF16 0      /* out_bf16 = bf16(acc + bias)                               */
#define VGGT_EPI_GELU_BF16 1 /* out_bf16 = bf16(gelu(bf16(acc + bias)))   (Mlp fc1 + GELU) */
#define VGGT_EPI_RESID_F32 2 /* out_f32 += gamma * bf16(acc + bias) [; out2 = out_f32]      */
#define VGGT_EPI_F32 3       /* out_f32 = bf16(acc + bias) widened to f32                  */

/* RoPE modes of vggt_headnorm_rope */
#define VGGT_ROPE_NONE 0
#define VGGT_ROPE_2D 1 /* VGGT RotaryPositionEmbedding2D: half D by y, half by x      */
#define VGGT_ROPE_1D 2 /* aligned_vggt/layers/rope.py RotaryPositionEmbedding          */

/* Library identification (build string) -- for load checks. */
const char* vggt_version(void);

/*
 * out[M,N] = epi( A[M,K] . W[N,K]^T + bias[N] ), bf16 MFMA (v_mfma_f32_16x16x32_bf16),
 * fp32 accumulation.  Replaces every autocast nn.Linear on the bf16 tier:
 * vggt Attention.qkv/proj, Mlp.fc1/fc2 (aggregator / DINOv2 blocks, via
 * featureAligned_vggt.py:78), CrossAttention.q/k/v/proj (cross_attention.py:37-43,55-57,76),
 * AlignmentHead.project_in (alignment_head.py:242), and the DINOv2 patch-embed
 * conv as an im2col GEMM.  Requires N % 128 == 0, K % 64 == 0, 16-B aligned
 * rows; A must have >= roundup(M,128) readable rows.  `gamma`/`out2`/`ldo2`
 * are used by VGGT_EPI_RESID_F32 only (LayerScale; out2 may be NULL).
 */
int vggt_gemm_bf16(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int M, int N, int K,
                   int epi, void* out, int64_t ldo, const float* gamma, float* out2, int64_t ldo2, void* stream);

/*
 * Row LayerNorm over C (fp32 statistics): y = (x-mean)/sqrt(var+eps)*w + b.
 * w/b may be NULL (elementwise_affine=False).  Replaces nn.LayerNorm
 * (norm1/norm2 of every Block, alignment_head.py:203-206, DPT norm, ...).
 * C must be a multiple of 256 and <= 4096.
 */
int vggt_layernorm(const void* x, int in_dtype, int64_t ldx, const float* w, const float* b, float eps, int M, int C,
                   void* y, int out_dtype, int64_t ldy, void* stream);

/*
 * In-place per-head LayerNorm (QK-norm) + RoPE on a bf16 [M, ld] buffer:
 * for each row m and head h, the D values at columns col_off + h*D are
 * normalised with (w,b,eps) (skipped if w == NULL) and rotated (rope_mode).
 * Positions: pos is int32 [period][2] (2D: y,x) or [period] (1D); row m uses
 * pos[m % period].  cos/sin tables are f32 [tab_len][rd] with rd = D/2 (2D)
 * or D (1D), layout cat(angles, angles) as in rope.py:23-44.
 * Replaces Attention.q_norm/k_norm + rope (vggt attention.py, ext) and
 * CrossAttention q_norm/k_norm + rope1d (cross_attention.py:59-62).
 */
int vggt_headnorm_rope(void* buf, int64_t ld, int col_off, int M, int H, int D, const float* w, const float* b,
                       float eps, int rope_mode, const int32_t* pos, int period, const float* cos_tab,
                       const float* sin_tab, int tab_len, void* stream);

/*
 * Flash attention forward, bf16 in/out, fp32 online softmax, D in {64,128}.
 * For batch b, head h:  O = softmax(Q K^T * scale) V  with
 *   Q row i at q + (b*q_bstride + i)*ldq + h*D   (i < nq), same for K, V (j < nk)
 *   O row i at o + (b*o_bstride + i)*ldo + h*D.
 * Replaces F.scaled_dot_product_attention in vggt Attention (frame / global
 * blocks of the aggregator, DINOv2 blocks, alignment frame blocks).
 */
int vggt_attention_fwd(const void* q, int64_t ldq, int64_t q_bstride, const void* k, int64_t ldk, int64_t k_bstride,
                       const void* v, int64_t ldv, int64_t v_bstride, void* o, int64_t ldo, int64_t o_bstride,
                       int batch, int heads, int nq, int nk, int D, float scale, void* stream);

/*
 * DINOv2 patch-embed input: ResNet-normalise fp32 images (F,3,H,W) and write
 * the bf16 im2col matrix A[F*h*w, Kp] (k = c*p*p + ky*p + kx, zero pad to Kp).
 * (vggt aggregator.py normalisation + DINOv2 PatchEmbed conv, ext.)
 * `mean` / `std_` are HOST pointers to 3 floats each (the ResNet constants).
 */
int vggt_patch_im2col(const float* images, int F, int H, int W, int patch, const float* mean, const float* std_,
                      void* A, int Kp, void* stream);

/*
 * DINOv2 token assembly: x[f, t] (f32, P = 1 + nreg + hw rows per frame):
 *   t = 0: cls + pos[0];  1..nreg: reg[t-1];  t > nreg: patch[f*hw + t-1-nreg] + pos[t-nreg]
 * patch is the bf16 patch-embed GEMM output [F*hw, C]; pos is f32 [1+hw, C].
 */
int vggt_dino_assemble(const void* patch, const float* cls, const float* reg, const float* pos, int F, int hw,
                       int nreg, int C, float* x, void* stream);

/*
 * Write per-frame special tokens into rows [f*P, f*P + n) of x (f32, ld C):
 * frame (f % S) == 0 takes tok[0, :n], other frames tok[1, :n]
 * (slice_expand_and_flatten, alignment_head.py:543-568 / aggregator, ext).
 * tok is f32 [2, n, C].
 */
int vggt_special_tokens(float* x, int64_t ldx, int F, int S, int P, int n, int C, const float* tok, void* stream);

/* Strided 2-D copy of f32 rows: dst[r*ldd + c] = src[r*lds + c], r < rows, c < cols. */
int vggt_copy_rows_f32(const float* src, int64_t lds, float* dst, int64_t ldd, int rows, int cols, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VGGT_MI355X_H */
