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

#include <stddef.h>
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

/* Process-wide kernel-variant knobs (defaults: the VGGT_GEMM / VGGT_ATTN_WAVES
 * environment variables, else the tuned choice).  Returns the previous value,
 * or VGGT_ERR_UNSUPPORTED for an unknown knob / value.  Results do not depend
 * on the variant beyond fp32 summation order inside one MFMA tile. */
#define VGGT_TUNE_GEMM_TILE 1  /* -1 auto, 0: 128x128 tile, 1: 256x256 ring, 2: 256x128 ring, 3: ping-pong (width by
                                  round quantisation), 4/5/6: ping-pong 256/192/128 wide, 7: ping-pong 256 wide when
                                  that fills two rounds of CUs, else as 3, 8: two-per-CU 256x128 (32x32x16 MFMA),
                                  9: persistent 256x256 ping-pong with register epilogue (bf16 / GELU / f32
                                  epilogues, N <= 4096; others as 7) */
#define VGGT_TUNE_ATTN_WAVES 2 /* 2, 4 or 8 waves (64 / 128 / 256 query rows) per attention workgroup */
#define VGGT_TUNE_ATTN_VARIANT 3 /* 0-15: attention instruction-schedule variant bits */
#define VGGT_TUNE_CONV_PF2 4     /* split-bf16 conv gather: 1 two-deep (buffer loads, default), 0 one-deep */
#define VGGT_TUNE_ATTN16 5       /* 1: D = 64 attention on the 16x16x32 matrix-core form, 0: 32x32x16 (default),
                                    2: 16x16x32 for 4-wave (nq < 4096) launches only */
#define VGGT_TUNE_LINEAR_ONE_LAUNCH 6 /* vggt_linear_f32_ws split-K: 1 the last split block of a tile combines the
                                         partials in the same launch (default), 0 a separate reduce launch (same
                                         fixed summation order: bitwise equal; kept for A/B and tests) */
#define VGGT_TUNE_LINEAR_SPLIT_K 7 /* vggt_linear_f32_ws split-K: split while each split keeps at least this many
                                      k (power of two, 16..4096; default 128).  Changes the fp32 summation order */
#define VGGT_TUNE_LINEAR_WK 8 /* vggt_linear_f32_ws with M <= 256: 0 the split-K form above, else the k range
                                 (power of two, 64..4096; default 64) each wave of an in-workgroup split keeps (2..8 waves on
                                 16 columns x 64 rows, partials summed in LDS: no scratch, no counters; the split depends
                                 on K only, so each row's bits do not depend on M) */
/* (knob 9 is unassigned: a round-balance split of the global attention measured no faster) */
#define VGGT_TUNE_GEMM_BALANCE 10 /* vggt_gemm_bf16 on the persistent form: 1 the whole rounds of row panels
                                     persistent and the remaining rows on the 128x128 form when the last round
                                     would be under 60 % full (bitwise equal), 0 one launch */
/* (knob 6, the persistent GEMM's DMA-placement bits, is retired: its measured-best placement is the only
   one compiled; vggt_tune(6, ...) returns VGGT_ERR_UNSUPPORTED) */
int vggt_tune(int knob, int value);

/* Per-stream launch configuration, host-side only (no GPU call); no reference
 * counterpart: the MI355X multi-GPU pipeline's encode stream (aligned_vggt/dist/pipeline.py).
 *   cus    the CUs launches on `stream` may occupy (a stream created with
 *          hipExtStreamCreateWithCUMask; 0 = the device's): the persistent kernels size
 *          their one-workgroup-per-CU grids and tile-rounding heuristics to it;
 *   flags  VGGT_STREAM_SHORT_WORKGROUPS: no persistent GEMM forms on this stream -- every
 *          workgroup runs one output tile, so kernels of a concurrent high-priority stream
 *          (the alignment recurrence) find free CUs within microseconds instead of
 *          waiting for a whole persistent launch.  Results are unchanged up to fp32
 *          summation order inside a tile.
 * cus = flags = 0 forgets the stream.  Returns the previous setting (cus | flags << 16,
 * 0 if none), or VGGT_ERR_* (up to 16 streams). */
#define VGGT_STREAM_SHORT_WORKGROUPS 1
int vggt_set_stream_config(void* stream, int cus, int flags);

/*
 * out[M,N] = epi( A[M,K] . W[N,K]^T + bias[N] ), bf16 MFMA (v_mfma_f32_16x16x32_bf16),
 * fp32 accumulation.  Replaces every autocast nn.Linear on the bf16 tier:
 * vggt Attention.qkv/proj, Mlp.fc1/fc2 (aggregator / DINOv2 blocks, via
 * featureAligned_vggt.py:78), CrossAttention.q/k/v/proj (cross_attention.py:37-43,55-57,76),
 * AlignmentHead.project_in (alignment_head.py:242), and the DINOv2 patch-embed
 * conv as an im2col GEMM.  Requires N % 128 == 0, K % 32 == 0, 16-B aligned
 * rows (rows past M are never read or written).  `gamma`/`out2`/`ldo2`
 * are used by VGGT_EPI_RESID_F32 only (LayerScale; out2 may be NULL).
 */
int vggt_gemm_bf16(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int M, int N, int K,
                   int epi, void* out, int64_t ldo, const float* gamma, float* out2, int64_t ldo2, void* stream);

/*
 * vggt_gemm_bf16 with VGGT_EPI_GELU_BF16 that also stores the bf16 pre-activation A.W^T + bias to `pre`
 * (row stride ldp): the training recompute of Mlp.fc1 -> GELU keeps both for the GELU backward
 * (alignment_head.py:351-393 under checkpoint), in one pass instead of a GEMM + a separate GELU kernel.
 */
int vggt_gemm_bf16_gelu_pre(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int M, int N,
                            int K, void* out, int64_t ldo, void* pre, int64_t ldp, void* stream);

/*
 * Fused attention input projection: qkv[M, 3*H*D] = bf16(A . W^T + bias), then,
 * in the same epilogue, the q and k column blocks get the per-head LayerNorm
 * (q_norm / k_norm: weights [D], eps; NULL weights = no norm) and RoPE
 * (rope_mode/pos/period/cos/sin as vggt_headnorm_rope), computed in fp32 on
 * the bf16 linear outputs and rounded once; the v block is stored as is.
 * Replaces qkv Linear + q_norm/k_norm + rope of VGGT Attention.forward (ext
 * layers/attention.py; aggregator frame/global blocks and the alignment
 * head's frame blocks, alignment_head.py:351-366).  D in {64, 128},
 * (H*D) % 128 == 0, K % 32 == 0.
 */
int vggt_gemm_qkv(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int M, int H, int D, int K,
                  void* out, int64_t ldo, const float* qw, const float* qb, const float* kw, const float* kb, float eps,
                  int rope_mode, const int32_t* pos, int period, const float* cos_tab, const float* sin_tab,
                  int tab_len, void* stream);

/*
 * The same fused epilogue on the separate projections of a cross attention:
 * out[M, N] = bf16(A . W^T + bias) with the FIRST H*D columns normalised
 * (weights nw/nb [D], NULL = no norm) and rotated (rope_mode/pos/period as
 * above; row m takes position pos[m % period]) and, for N = 2*H*D, the
 * second block stored as is.  N = H*D: a q projection (+ q_norm + RoPE);
 * N = 2*H*D: a packed kv projection (+ k_norm + RoPE on k).  Replaces the
 * q / kv Linears + vggt_headnorm_rope pair of the alignment head's temporal
 * blocks (CrossAttention, alignment_head.py:369-380): bitwise the same
 * values, one HBM pass fewer.  Shape rules as vggt_gemm_qkv.
 */
int vggt_gemm_headnorm(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int M, int N, int H,
                       int D, int K, void* out, int64_t ldo, const float* nw, const float* nb, float eps, int rope_mode,
                       const int32_t* pos, int period, const float* cos_tab, const float* sin_tab, int tab_len,
                       void* stream);

/*
 * Row LayerNorm over C (fp32 statistics): y = (x-mean)/sqrt(var+eps)*w + b.
 * w/b may be NULL (elementwise_affine=False).  Replaces nn.LayerNorm
 * (norm1/norm2 of every Block, alignment_head.py:203-206, DPT norm, ...).
 * C must be a multiple of 256 and <= 4096.
 */
int vggt_layernorm(const void* x, int in_dtype, int64_t ldx, const float* w, const float* b, float eps, int M, int C,
                   void* y, int out_dtype, int64_t ldy, void* stream);

/*
 * Residual LayerScale add fused with the NEXT LayerNorm:
 *   x[m] += gamma * y[m]          (x fp32 [M, C] in place, y bf16 [M, C])
 *   out2[m] = x[m]                (if out2 != NULL: the kept-layer concat half)
 *   xn[m] = LayerNorm(x[m]; w, b) (bf16, if xn != NULL; w/b may be NULL)
 * The add is the arithmetic of vggt_gemm_bf16's VGGT_EPI_RESID_F32 epilogue
 * on the bf16-rounded branch output.  Replaces `x = x + ls2(mlp(norm2(x)))`
 * followed by the next block's `norm1(x)` (vggt layers/block.py, ext; the
 * aggregator's frame/global alternation, featureAligned_vggt.py:78-82).
 * C a multiple of 256 in {256, 512, 1024, 2048}.
 */
int vggt_resid_add_layernorm(float* x, int64_t ldx, const void* y, int64_t ldy, const float* gamma, float* out2,
                             int64_t ldo2, const float* w, const float* b, float eps, int M, int C, void* xn,
                             int64_t ldn, void* stream);

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
 * Fused q_norm/k_norm + RoPE on a fused qkv row: q heads at columns [0, H*D)
 * normalised with (qw, qb), k heads at [H*D, 2*H*D) with (kw, kb); one launch
 * (vggt Attention.q_norm/k_norm + rope, ext; featureAligned_vggt.py:78).
 * Same position/table conventions as vggt_headnorm_rope.
 */
int vggt_qknorm_rope(void* qkv, int64_t ld, int M, int H, int D, const float* qw, const float* qb, const float* kw,
                     const float* kb, float eps, int rope_mode, const int32_t* pos, int period, const float* cos_tab,
                     const float* sin_tab, int tab_len, void* stream);

/*
 * Out-of-place forms (training recompute, alignment_head.py:351-393 under checkpoint: the backward needs the
 * pre-norm projections, so they are not overwritten): heads are read from src (row stride lds) and the
 * normalised + rotated values written to dst (row stride ldd).  vggt_qknorm_rope_out covers the q|k columns
 * [0, 2*H*D) of a fused projection, vggt_headnorm_rope_out H heads from column 0.
 */
int vggt_qknorm_rope_out(const void* src, int64_t lds, void* dst, int64_t ldd, int M, int H, int D, const float* qw,
                         const float* qb, const float* kw, const float* kb, float eps, int rope_mode,
                         const int32_t* pos, int period, const float* cos_tab, const float* sin_tab, int tab_len,
                         void* stream);
int vggt_headnorm_rope_out(const void* src, int64_t lds, void* dst, int64_t ldd, int M, int H, int D, const float* w,
                           const float* b, float eps, int rope_mode, const int32_t* pos, int period,
                           const float* cos_tab, const float* sin_tab, int tab_len, void* stream);

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

/*
 * Row-remapped LayerNorm: logical row r (< M) = group g = r / group, i = r % group,
 * reads x row g*x_group_stride + x_row_offset + i and writes y row
 * g*y_group_stride + y_row_offset + i.  Used to skip/insert per-frame special
 * tokens without copies: DPT patch-token norm (dpt_head, ext, via
 * featureAligned_vggt.py:166) and AlignmentHead.token_norm writing after the
 * per-frame alignment token (alignment_head.py:247,269-270).
 */
int vggt_layernorm_grouped(const void* x, int in_dtype, int64_t ldx, const float* w, const float* b, float eps, int M,
                           int C, void* y, int out_dtype, int64_t ldy, int group, int x_group_stride,
                           int x_row_offset, int y_group_stride, int y_row_offset, void* stream);

/*
 * Skinny fp32 linear layer (weight-streaming, small M), exact-f32 MFMA:
 *   out[M,N] = epi( act_in(A)[M,K] . W[N,K]^T + bias )
 * act_in: 0 none, 1 SiLU.  epi: VGGT_EPI_F32 (plain), VGGT_EPI_GELU_BF16 (GELU,
 * f32 out here), VGGT_EPI_RESID_F32 (out += gamma * v; out is the residual).
 * Replaces the fp32 nn.Linear calls of the camera head (camera_head, ext:
 * embed_pose, poseLN_modulation, trunk Blocks, pose_branch), the alignment
 * decoder (alignment_head.py:463,475,534-538, cross blocks, gated_update.py:22-36).
 */
int vggt_linear_f32(const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias, int M, int N, int K,
                    int act_in, int epi, float* out, int64_t ldo, const float* gamma, void* stream);
/* Same with a caller-provided scratch (device, >= VGGT_LINEAR_F32_WS_COUNTERS * 4 +
 * VGGT_LINEAR_F32_MAX_SPLITS * roundup(M,64) * N * 4 bytes to allow the maximum split;
 * a smaller one caps the split): skinny-M calls are
 * split along K into up to VGGT_LINEAR_F32_MAX_SPLITS deterministic partial sums combined in a fixed order
 * (camera head trunk, alignment decoder: M = 16 frames) by the last split block of
 * each output tile, in the same launch.  The scratch's first
 * VGGT_LINEAR_F32_WS_COUNTERS words are per-tile counters: zero-fill them before a
 * scratch's first use; every call leaves them zero.  ws == NULL: no split. */
/* `groups` independent skinny fp32 linears of one shape in one launch (M <= 256):
 * group g reads A + g*a_gstride, W + g*w_gstride, bias + g*b_gstride and writes
 * out + g*o_gstride (element strides); epi VGGT_EPI_F32 or VGGT_EPI_GELU_BF16.
 * Each group's values are bitwise those of its own vggt_linear_f32_ws call
 * (the in-workgroup split form).  Replaces GatedUpdate's per-token delta MLPs
 * (gated_update.py:51-57: one Linear pair per memory token). */
int vggt_linear_f32_grouped(const float* A, int64_t lda, int64_t a_gstride, const float* W, int64_t ldw,
                            int64_t w_gstride, const float* bias, int64_t b_gstride, int M, int N, int K, int groups,
                            int act_in, int epi, float* out, int64_t ldo, int64_t o_gstride, void* stream);
/* GatedUpdate's elementwise stages (gated_update.py:43-79, fp32; rows = B x Nt memory
 * tokens of D features, contiguous):
 *   prep: inp[b, i] = [update_b, |update_b| memory[b, i], |update_b| mean_j memory[b, j]]
 *         ([B*Nt, 3D]) and g_in[:, D:2D] = |update_b| memory[b, i]  ([B*Nt, 2D]);
 *   diff: g_in[:, 0:D] = deltas - memory;
 *   tail: out = normalize(memory + sigmoid(logit) normalize(diff - (diff . memory) memory))
 *         with F.normalize's max(|x|, 1e-12). */
int vggt_gated_update_prep(const float* memory, const float* update, int B, int Nt, int D, float* inp, float* g_in,
                           void* stream);
int vggt_gated_update_diff(const float* memory, const float* deltas, int rows, int D, float* g_in, void* stream);
int vggt_gated_update_tail(const float* memory, const float* deltas, const float* logit, int rows, int D, float* out,
                           void* stream);
#define VGGT_LINEAR_F32_WS_COUNTERS 1024
#define VGGT_LINEAR_F32_MAX_SPLITS 32
int vggt_linear_f32_ws(const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias, int M, int N, int K,
                       int act_in, int epi, float* out, int64_t ldo, const float* gamma, void* ws, size_t ws_bytes,
                       void* stream);

/*
 * Small-window attention (nk <= 128, D <= 256), one wave per (batch, head),
 * f32 softmax; dtype VGGT_DTYPE_BF16 or VGGT_DTYPE_F32 for all of q/k/v/o.
 * Layout as vggt_attention_fwd (v shares k's batch stride).  Replaces the SDPA
 * of CrossAttention (cross_attention.py:64-73) in the temporal blocks (S
 * queries x T keys per spatial token, alignment_head.py:368-390) and the
 * decoder (alignment_head.py:494-530), and the camera-head trunk attention.
 * bf16 windows of <= 16 queries x <= 16 keys (D % 16 == 0) run on the matrix cores
 * (fp32 scores, P rounded to bf16 for P.V, as the reference's bf16 SDPA) unless
 * dtype carries VGGT_ATTN_SMALL_EXACT: the training forward, whose backward
 * (vggt_attention_small_bwd) recomputes P in fp32 from the same formula.
 */
#define VGGT_ATTN_SMALL_EXACT 0x100
int vggt_attention_small(const void* q, int64_t ldq, int64_t q_bstride, const void* k, int64_t ldk, int64_t k_bstride,
                         const void* v, int64_t ldv, void* o, int64_t ldo, int64_t o_bstride, int dtype, int batch,
                         int heads, int nq, int nk, int D, float scale, void* stream);

/* fp32 variant of vggt_headnorm_rope (decoder / camera head run in fp32). */
int vggt_headnorm_rope_f32(float* buf, int64_t ld, int col_off, int M, int H, int D, const float* w, const float* b,
                           float eps, int rope_mode, const int32_t* pos, int period, const float* cos_tab,
                           const float* sin_tab, int tab_len, void* stream);

/* y_bf16[r, c] = bf16(x_f32[r, c])  (autocast input cast of a Linear). */
int vggt_cast_f32_bf16(const float* x, int64_t ldx, void* y, int64_t ldy, int rows, int cols, void* stream);

/*
 * fp32 NHWC implicit-GEMM convolution (exact-f32 MFMA), DPT head
 * (dpt_head, ext; featureAligned_vggt.py:166,183):
 *   y[p, co] = relu_out?( sum act(x) * W + bias ) [+ pos[p % (ho*wo), co]]
 *              [+ (res1_relu ? relu(res1) : res1)[p, co]] [+ res2[p, co]]
 * x: [nimg, hi, wi, ci] with pixel stride ldx; W: [roundup(co',64), kh*kw*ci]
 * (K order ky, kx, ci; rows beyond co' zero-padded); ci % 32 == 0.
 * shuffle = s > 0 turns a 1x1 GEMM with co' = s*s*co columns (column
 * (dy*s+dx)*co + c) into a stride==kernel ConvTranspose2d pixel-shuffle store
 * onto the [nimg, hi*s, wi*s, co] grid.
 */
int vggt_conv2d_f32(const float* x, int64_t ldx, int nimg, int hi, int wi, int ci, const float* w, const float* bias,
                    int co, int kh, int kw, int stride, int pad, float* y, int64_t ldy, int relu_in, int relu_out,
                    const float* res1, int64_t ldr1, int res1_relu, const float* res2, int64_t ldr2, const float* pos,
                    int shuffle, void* stream);

/*
 * Same convolution as vggt_conv2d_f32 on the bf16 matrix path with split
 * operands: x = hi + lo (hi = bf16(x), lo = bf16(x - hi)), accumulating
 * hi.hi + hi.lo + lo.hi in fp32 (~2^-16 relative per product instead of
 * fp32's 2^-24; ~5x faster).  w_hi / w_lo: the vggt_conv2d_f32 weight layout
 * split by vggt_split_bf16x2 (bf16), rows zero-padded to a multiple of 128.
 */
int vggt_conv2d_bf16x3(const float* x, int64_t ldx, int nimg, int hi, int wi, int ci, const void* w_hi,
                       const void* w_lo, const float* bias, int co, int kh, int kw, int stride, int pad, float* y,
                       int64_t ldy, int relu_in, int relu_out, const float* res1, int64_t ldr1, int res1_relu,
                       const float* res2, int64_t ldr2, const float* pos, int shuffle, void* stream);

/*
 * vggt_conv2d_bf16x3 on an activation split beforehand (vggt_split_act_bf16x2,
 * which also applies the input ReLU): x_hi / x_lo bf16 [nimg, hi, wi, ci] with
 * pixel stride ldx (elements, % 8 == 0), whole map < 2 GiB.  The im2col gather
 * is LDS-DMA of the bf16 halves (out-of-image taps read as zeros); results are
 * bitwise equal to vggt_conv2d_bf16x3 with relu_in on the f32 input.  y (f32) and/or
 * y_hi / y_lo (the NEXT conv's pre-split input: split(split_relu ? max(y, 0) : y),
 * bf16 rows of stride ldys) are written; either may be NULL, not both.
 */
int vggt_conv2d_bf16x3_pre(const void* x_hi, const void* x_lo, int64_t ldx, int nimg, int hi, int wi, int ci,
                           const void* w_hi, const void* w_lo, const float* bias, int co, int kh, int kw, int stride,
                           int pad, float* y, int64_t ldy, int relu_out, const float* res1, int64_t ldr1,
                           int res1_relu, const float* res2, int64_t ldr2, const float* pos, int shuffle,
                           void* y_hi, void* y_lo, int64_t ldys, int split_relu, void* stream);

/* hi / lo = split(relu ? max(x, 0) : x) of a [rows, cols] f32 map (row stride ldx, cols % 4 == 0)
 * into contiguous bf16 [rows, cols] maps: hi = bf16(v), lo = bf16(v - hi) (DPT conv inputs). */
int vggt_split_act_bf16x2(const float* x, int64_t ldx, int64_t rows, int cols, int relu, void* hi, void* lo,
                          void* stream);

/* hi[i] = bf16(x[i]), lo[i] = bf16(x[i] - hi[i]) for i < n (weight split for vggt_conv2d_bf16x3). */
int vggt_split_bf16x2(const float* x, int64_t n, void* hi, void* lo, void* stream);

/* NHWC bilinear resize with align_corners=True (custom_interpolate, dpt_head ext), + optional pos table. */
int vggt_upsample_bilinear_f32(const float* x, int nimg, int hi, int wi, int C, float* y, int ho, int wo,
                               const float* pos, void* stream);
/* Same, writing y (f32, may be NULL) and/or the split bf16 halves of relu?(y) (contiguous [.., C]). */
int vggt_upsample_bilinear_split(const float* x, int nimg, int hi, int wi, int C, float* y, int ho, int wo,
                                 const float* pos, void* y_hi, void* y_lo, int split_relu, void* stream);
/* Same as vggt_upsample_bilinear_split with a SEPARABLE positional table (DPT's
 * UV sin/cos embedding, dpt_head ext `_apply_pos_embed`: channels [0, C/2) depend on
 * x only, [C/2, C) on y only): pos_sep = [wo + ho, C/2] fp32, rows 0..wo-1 the x
 * part, rows wo..wo+ho-1 the y part.  C % 8 == 0. */
int vggt_upsample_bilinear_split_sep(const float* x, int nimg, int hi, int wi, int C, float* y, int ho, int wo,
                                     const float* pos_sep, void* y_hi, void* y_lo, int split_relu, void* stream);

/*
 * Fused last stage of the DPT head (output_conv1's output -> F.interpolate(size=(ho, wo),
 * bilinear, align_corners=True) -> + _apply_pos_embed -> output_conv2[0], dpt_head ext,
 * featureAligned_vggt.py:166): y = conv3x3_pad1(split(resize(x) + pos)) without
 * materialising the resized map.  x [nimg, hi, wi, C] f32 NHWC (C % 32 == 0), pos_sep
 * [wo + ho, C/2] (the separable table of vggt_upsample_bilinear_split_sep) or NULL,
 * w_hi / w_lo the split packed weights of vggt_conv2d_bf16x3_pre ([>= 32 rows, 9*C], the
 * (ky, kx, ci) column order), co <= 32.  Outputs as conv2d_bf16x3_pre: y [nimg*ho*wo, ldy]
 * f32 and/or the split halves of relu?(y).  Same products and K order as the unfused
 * upsample + conv2d_bf16x3_pre.
 */
int vggt_conv2d_upsample_bf16x3(const float* x, int nimg, int hi, int wi, int C, const float* pos_sep, int ho,
                                int wo, const void* w_hi, const void* w_lo, const float* bias, int co, int relu_out,
                                float* y, int64_t ldy, void* y_hi, void* y_lo, int64_t ldys, int split_relu,
                                void* stream);

/*
 * DPT activate_head (ext): x [npix, ncl] NHWC with the confidence last;
 * pts[p, j] = act(x[p, j]) * scale[p / pix_per_img]  (act 0 = exp, 1 = inv_log),
 * conf[p] = 1 + exp(x[p, ncl-1]) (expp1).  scale may be NULL (depth *= chunk
 * scale, featureAligned_vggt.py:171).
 */
int vggt_dpt_activate(const float* x, int64_t ldx, int64_t npix, int pix_per_img, int ncl, int act,
                      const float* scale, float* pts, float* conf, void* stream);

/*
 * Robust Sim(3) between two point-map sets, one per batch element:
 * irls_sim3_umeyama + weighted_umeyama_sim3 (aligned_vggt/models/
 * pointAligned_wrapped_vggt.py:159-305; called at :69-100).  src/dst:
 * n points x 3 fp32 per batch element (batch strides in floats), conf_src /
 * conf_dst: n fp32.  Points whose sqrt(conf_src*conf_dst) is below
 * factor * (lower) median get weight 0; Huber IRLS with `delta`, at most
 * max_iters iterations after the initial solve, stop when |dR|_F, |dt|, |ds|
 * all < tol.  Outputs R_out [B,3,3], t_out [B,3], s_out [B] fp32, written on
 * the stream (no host synchronisation); a batch element whose total weight
 * is < 1e-6 (the reference raises ValueError) gets NaN outputs.
 * conf_dst == NULL: conf_src holds the weights themselves; factor <= 0: no
 * confidence threshold; max_iters == 0 with both is weighted_umeyama_sim3
 * (pointAligned_wrapped_vggt.py:159-219).
 * workspace: >= vggt_irls_workspace_bytes(B), 16-B aligned, device memory.
 */
size_t vggt_irls_workspace_bytes(int B);
int vggt_irls_sim3(const float* src, int64_t src_bs, const float* dst, int64_t dst_bs, const float* conf_src,
                   int64_t cs_bs, const float* conf_dst, int64_t cd_bs, int B, int64_t n, float factor, float delta,
                   int max_iters, float tol, float* R_out, float* t_out, float* s_out, void* workspace,
                   size_t ws_bytes, void* stream);

/*
 * out[b, i] = T_b[:3,:3] (scale_b * pts[b, i]) + T_b[:3,3] for n points (x,y,z)
 * per batch element; T: [B,4,4] fp32 device, scale: [B] device or NULL.
 * apply_sim3_alignment_on_point_maps (aligned_vggt/utils/alignment.py:491-526)
 * and the point transform of featureAligned_vggt.py:200-206.  In place allowed.
 */
int vggt_sim3_points(const float* pts, int64_t p_bs, int B, int64_t n, const float* T, const float* scale, float* out,
                     int64_t o_bs, void* stream);

/* x[b, i] *= scale[b] (i < n) in place; scale: [B] device (depth *= chunk scale,
 * featureAligned_vggt.py:171; pointAligned_wrapped_vggt.py:130-132). */
int vggt_scale_f32(float* x, int64_t bs, int B, int64_t n, const float* scale, void* stream);

/*
 * Per-chunk pose / Sim(3) composition of FeatureAlignedVGGT.forward
 * (featureAligned_vggt.py:96-143 and the point transform of :187-196), one
 * launch, no host synchronisation:
 *   chunk_se3 = pose_encoding_to_extri(chunk_sim3[:7]), scale = chunk_sim3[7];
 *   per_frame_se3 = [chunk_se3, pose_encoding_to_extri(frame_se3[f]) @ chunk_se3];
 *   extr = camera extrinsics (pose_encoding_to_extri_intri of cam_pose_enc)
 *          @ inv(extr[0]), translation * scale;
 *   mean = I (no context) | gt_first[b] | Markley mean over the overlap of
 *          inv(extr[k]) @ pose_encoding_to_extri(ctx_pose_enc[S_prev-ov+k])
 *          (averagePoseEncodings, geometry.py:4-37; ov == 1: the one transform);
 *   aligned_pose_enc = extri_intri_to_pose_encoding(extr @ (per_frame_se3 @ mean)).
 * chunk_sim3 [B,8], frame_se3 [B,S-1,7], cam_pose_enc [B,S,9] (T, quat xyzw,
 * FoV h/w), ctx_pose_enc [B,S_prev,9] = context["pose_enc"][-1] or NULL (first
 * chunk), gt_first [B,4,4] = gt_poses[:, 0] or NULL; all fp32 contiguous device.
 * Outputs aligned_pose_enc [B,S,9]; point_transform [B,4,4] (or NULL) =
 * context ? inv(per_frame_se3[:,0]) @ extr_raw[:,0] : extr_raw[:,0].
 * Requires 1 <= overlap <= min(S, S_prev, 64) when the Markley path runs.
 */
int vggt_pose_compose(const float* chunk_sim3, const float* frame_se3, const float* cam_pose_enc,
                      const float* ctx_pose_enc, int S_prev, const float* gt_first, int B, int S, int overlap, int H,
                      int W, float* aligned_pose_enc, float* point_transform, void* stream);

/* ======================================================================
 * Training (backward) entry points -- alignment-head training, SURVEY.md §8f
 * row 4: train_featureAlignedVGGT_vkitti.yaml freezes the aggregator, camera
 * and depth heads (:80-83) and trains AlignmentHead (alignment_head.py) under
 * bf16-mixed autocast (run_model.py:472), with checkpoint()-recomputed blocks
 * (alignment_head.py:351-426).  Gradients of bf16 tensors are bf16 (what
 * autocast produces), parameter gradients fp32.  Column / row reductions
 * into parameter gradients are deterministic: fixed row chunks write partial
 * sums to `ws` (>= the size the matching *_workspace_bytes returns) and a
 * second pass ADDS them, in chunk order, to the fp32 gradient buffer.
 * ====================================================================== */

/* Forward attention as vggt_attention_fwd (exact scores, no Q prescale) that
 * also stores lse[(b*heads + h)*nq + q] = log2 sum_k exp2(q.k * scale * log2 e),
 * consumed by vggt_attention_bwd (recompute of the frame blocks' SDPA). */
int vggt_attention_fwd_lse(const void* q, int64_t ldq, int64_t q_bstride, const void* k, int64_t ldk,
                           int64_t k_bstride, const void* v, int64_t ldv, int64_t v_bstride, void* o, int64_t ldo,
                           int64_t o_bstride, float* lse, int batch, int heads, int nq, int nk, int D, float scale,
                           void* stream);

/*
 * Flash-attention backward (bf16, D in {64,128}; F.scaled_dot_product_attention
 * backward in vggt Attention, ext, called by the alignment head's frame blocks).
 * q/k/v/o/dout strided as vggt_attention_fwd (v shares k's batch stride, dout
 * shares o's layout); lse from vggt_attention_fwd_lse; delta: fp32
 * [batch*heads*nq] scratch (written).  Writes bf16 dq [.., lddq] (q's batch
 * stride) and dk, dv [.., lddkv] (k's batch stride), e.g. straight into the
 * dqkv buffer laid out like qkv.
 */
int vggt_attention_bwd(const void* q, int64_t ldq, int64_t q_bstride, const void* k, int64_t ldk, int64_t k_bstride,
                       const void* v, int64_t ldv, const void* o, const void* dout, int64_t ldo, int64_t o_bstride,
                       const float* lse, float* delta, void* dq, int64_t lddq, void* dk, void* dv, int64_t lddkv,
                       int batch, int heads, int nq, int nk, int D, float scale, void* stream);

/*
 * Small-window attention backward (vggt_attention_small's shapes: temporal
 * cross attention, cross_attention.py:64-75, and the fp32 decoder blocks):
 * one wave per (batch, head), recomputes P; dtype for every operand.
 * dq [.., lddq] batch stride dq_bstride; dk, dv [.., lddkv] batch stride
 * dkv_bstride.  Needs (2*nq*D + 2*nk*D + 2*nq*nk)*4 <= 64 KiB.
 */
int vggt_attention_small_bwd(const void* q, int64_t ldq, int64_t q_bstride, const void* k, int64_t ldk,
                             int64_t k_bstride, const void* v, int64_t ldv, const void* dout, int64_t ldo,
                             int64_t o_bstride, void* dq, int64_t lddq, int64_t dq_bstride, void* dk, void* dv,
                             int64_t lddkv, int64_t dkv_bstride, int dtype, int batch, int heads, int nq, int nk, int D,
                             float scale, void* stream);

/*
 * LayerNorm backward (nn.LayerNorm / F.layer_norm backward; every norm of the
 * alignment head): x = the forward input, dy the output gradient, same row
 * map as vggt_layernorm_grouped (logical row r -> group r/group; x and dx rows
 * g*x_group_stride + x_row_offset + i, dy rows g*y_group_stride +
 * y_row_offset + i).  accumulate: bit VGGT_LN_BWD_DX_ACCUMULATE (1) dx += (f32
 * only, else dx =); dw/db (may be NULL) get the parameter gradients added, or
 * written with bit VGGT_LN_BWD_PARAMS_WRITE (2).  C % 256 == 0, C <= 1024.
 */
#define VGGT_LN_BWD_DX_ACCUMULATE 1
#define VGGT_LN_BWD_PARAMS_WRITE 2
size_t vggt_layernorm_bwd_workspace_bytes(int M, int C);
int vggt_layernorm_bwd(const void* x, int xdtype, int64_t ldx, const float* w, float eps, const void* dy, int dydtype,
                       int64_t ldy, void* dx, int dxdtype, int64_t lddx, int accumulate, int M, int C, int group,
                       int x_group_stride, int x_row_offset, int y_group_stride, int y_row_offset, float* dw,
                       float* db, void* ws, size_t ws_bytes, void* stream);

/*
 * Per-head LayerNorm + RoPE backward (q_norm/k_norm + rope of vggt Attention,
 * ext, and CrossAttention, cross_attention.py:59-62): pre = the bf16/f32
 * values before the norm (the linear's output), grad = d(output) in, d(pre)
 * out, in place.  Heads [0, hsplit) use w0 (gradients into dw0/db0), heads
 * [hsplit, H) use w1 (dw1/db1); NULL w = no norm.  RoPE conventions as
 * vggt_headnorm_rope.
 */
size_t vggt_headnorm_rope_bwd_workspace_bytes(int M, int D);
int vggt_headnorm_rope_bwd(const void* pre, int64_t ldp, void* grad, int64_t ldg, int dtype, int M, int H, int hsplit,
                           int D, const float* w0, const float* w1, float eps, int rope_mode, const int32_t* pos,
                           int period, const float* cos_tab, const float* sin_tab, int tab_len, float* dw0,
                           float* db0, float* dw1, float* db1, void* ws, size_t ws_bytes, void* stream);

/* Column-reduction workspace for vggt_colsum / vggt_layerscale_bwd / vggt_gelu_bwd. */
size_t vggt_colred_workspace_bytes(int M, int N);

/* out[n] (+)= sum_m x[m, n]  (Linear bias gradients).  N % 4 == 0. */
int vggt_colsum(const void* x, int dtype, int64_t ldx, int M, int N, float* out, int accumulate, void* ws,
                size_t ws_bytes, void* stream);

/*
 * LayerScale + residual backward (x + gamma * branch, vggt layers/block.py /
 * cross_attention.py:130-131): dbranch = gamma * dout (rounded to odtype),
 * dgamma += sum_m dout * branch, dbias += sum_m dbranch (the bias gradient of
 * the Linear that produced the branch).  dgamma / dbias may be NULL.
 */
int vggt_layerscale_bwd(const float* dout, int64_t ldd, const void* branch, int bdtype, int64_t ldb,
                        const float* gamma, void* dbranch, int odtype, int64_t ldo, int M, int N, float* dgamma,
                        float* dbias, void* ws, size_t ws_bytes, void* stream);

/* y = GELU(x) (exact erf), any f32/bf16 combination (Mlp.act, unfused training form). */
int vggt_gelu_fwd(const void* x, int xdtype, int64_t ldx, void* y, int ydtype, int64_t ldy, int M, int N,
                  void* stream);

/* dpre = dh * GELU'(pre) (rounded to odtype); dbias += sum_m dpre (fc1 bias gradient; may be NULL). */
int vggt_gelu_bwd(const void* dh, int dhdtype, int64_t lddh, const void* pre, int predtype, int64_t ldp, void* dpre,
                  int odtype, int64_t ldo, int M, int N, float* dbias, void* ws, size_t ws_bytes, void* stream);

/* x_f32[m, n] += gamma[n] * branch[m, n]  (LayerScale residual add with a saved branch). */
int vggt_resid_scale_add(float* x, int64_t ldx, const void* branch, int bdtype, int64_t ldb, const float* gamma, int M,
                         int N, void* stream);

/* out_f32[m, n] = x_f32[m, n] + gamma[n] * branch[m, n]  (out may equal x). */
int vggt_resid_scale_add_from(float* out, int64_t ldo, const float* x, int64_t ldx, const void* branch, int bdtype,
                              int64_t ldb, const float* gamma, int M, int N, void* stream);

/* dst[c, r] = src[r, c] for 2-byte elements; columns r in [rows, rows_pad) of dst are zero
 * (weight-gradient GEMM operands: dW = dY^T X as vggt_gemm_bf16(dY^T, X^T)). */
int vggt_transpose_b16(const void* src, int64_t lds, int rows, int cols, void* dst, int64_t ldd, int rows_pad,
                       void* stream);

/* dW[n, k] (+)= bf16(sum_m dY[m, n] X[m, k]) for bf16 row-major dY [M, N], X [M, K] (the bf16-tier
 * Linear weight gradients, rounded like autocast's bf16 weight gradient): split-K over the token
 * dimension into fp32 partials in ws (>= vggt_wgrad_bf16_workspace_bytes), summed in split order.
 * N % 128 == 0, K % 128 == 0. */
size_t vggt_wgrad_bf16_workspace_bytes(int M, int N, int K);
int vggt_wgrad_bf16(const void* dy, int64_t ldy, const void* x, int64_t ldx, int M, int N, int K, float* dw,
                    int64_t ldw, int accumulate, void* ws, size_t ws_bytes, void* stream);

/* dW[n, k] (+)= sum_m dY[m, n] X[m, k]  fp32 (skinny-M decoder / gated-update Linear weight gradients). */
int vggt_wgrad_f32(const float* dy, int64_t ldy, const float* x, int64_t ldx, int M, int N, int K, float* dw,
                   int64_t ldw, int accumulate, void* stream);
/* The same and db[n] (+)= sum_m dY[m, n] in the one launch (LinearF32Fn backward: weight and bias gradients). */
int vggt_wgrad_bias_f32(const float* dy, int64_t ldy, const float* x, int64_t ldx, int M, int N, int K, float* dw,
                        int64_t ldw, float* db, int accumulate, void* stream);

/* out[b] = sum_{i<n} a[b*bs + i] * c[b*bs + i]  (d chunk_scale of depth *= chunk_scale,
 * featureAligned_vggt.py:171, in training).  ws >= vggt_batch_dot_workspace_bytes(B, n). */
size_t vggt_batch_dot_workspace_bytes(int B, int64_t n);
int vggt_batch_dot_f32(const float* a, const float* c, int64_t bs, int B, int64_t n, float* out, void* ws,
                       size_t ws_bytes, void* stream);

/* MFMA peak probe (diagnostic; BASELINE.md §2 asks for a measured MFMA microbenchmark with its clock):
 * nwg workgroups of 4 waves issue iters x 8 v_mfma_f32_32x32x16_bf16 each on the bf16 operands
 * (nwg * 256 * 16 elements: random or zeros), 32768 FLOP per MFMA; stamps[4 * wg] = s_memtime before /
 * after the loop, s_memrealtime (100 MHz) before / after.  sink: nwg * 256 floats, never read. */
int vggt_mfma_probe(unsigned long long* stamps, float* sink, const void* operands, int nwg, int iters, void* stream);

/* Attention segment stamps (diagnostic; VERDICT r5: where the global attention's waits go).  Runs the
 * default D = 64 forward (variant 33, the 8- / 4-wave choice of vggt_attention_fwd, o written as there) with
 * s_memtime stamps at each tile's boundaries; per wave (index (blockIdx * NW + wave) * 8) the cycle sums
 * [2] the tile's work up to its last LDS read, [3] end-of-tile vmcnt(0), [4] barrier ([0], [1], [5] unused),
 * [6] the wave's final s_memtime (low 32 bits); every wave runs ceil(nk / 64) tiles.  stamps: nwg * NW * 8 entries, NW = 8 for nq >= 4096 else 4. */
int vggt_attention_stamps(const void* q, int64_t ldq, int64_t q_bstride, const void* k, int64_t ldk, int64_t k_bstride,
                          const void* v, int64_t ldv, int64_t v_bstride, void* o, int64_t ldo, int64_t o_bstride,
                          unsigned long long* stamps, int batch, int heads, int nq, int nk, float scale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VGGT_MI355X_H */
