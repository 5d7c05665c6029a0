// Process-wide kernel-variant knobs behind vggt_tune() (capi.cpp).
#pragma once
extern int g_vggt_gemm_tile;   // -1 auto, 0 128x128, 1 256x256 ring, 2 256x128 ring, 3-7 ping-pong, 8 two-per-CU, 9 persistent ping-pong
extern int g_vggt_attn_waves;  // 2, 4 or 8 (8: only for nq >= 4096; 2: offset-free variant 33 only)
extern int g_vggt_attn_variant; // attention schedule variant bits (attention.hip)
extern int g_vggt_attn16;       // 1: variant 33 runs the 16x16x32 form for D = 64 (attn16_fwd_kernel), 2: only for 4-wave launches; default 0
extern int g_vggt_conv_pf2;     // split-bf16 conv: 1 two-deep buffer-load gather, 0 one-deep
extern int g_vggt_linear_split_k;    // split-K vggt_linear_f32_ws: split while each split keeps >= this many k (2 splits' worth)
extern int g_vggt_linear_one_launch; // split-K vggt_linear_f32_ws: 1 combine in the same launch (default), 0 reduce launch
extern int g_vggt_linear_wk;         // vggt_linear_f32_ws, M <= 256: in-workgroup split-K, ~this many k per wave (0: off)
extern int g_vggt_gemm_balance;      // 1: persistent GEMMs with a partial last round split (whole rounds persistent, rest 128x128)
// per-stream launch configuration (vggt_set_stream_config): the CUs a CU-masked
// stream may use (0: the device's) and its VGGT_STREAM_* flags
int vggt_stream_cu_count(void* stream);
int vggt_stream_flags(void* stream);
