// Library identification for the C ABI (include/vggt_mi355x.h).
#include "../../include/vggt_mi355x.h"

extern "C" const char* vggt_version(void) { return "vggt_mi355x 0.1 gfx950"; }

#include <stdlib.h>

#include <atomic>
#include <mutex>

#include "tune.h"

namespace {
int env_or(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
}  // namespace

int g_vggt_gemm_tile = env_or("VGGT_GEMM", -1);
int g_vggt_attn_waves = env_or("VGGT_ATTN_WAVES", 8);  // 8-wave groups for nq >= 4096 (profiles/r2c/ab_attn_w8)
int g_vggt_attn_variant = env_or("VGGT_ATTN_VARIANT", 33);
// 2: the 16x16x32 form for the 4-wave (frame / DINOv2) launches only -- all launches measured slower in the model
// (profiles/r6d), frame-only faster (r7b: step 98.9-99.0 -> 98.3 ms)
int g_vggt_attn16 = env_or("VGGT_ATTN16", 2);
int g_vggt_conv_pf2 = env_or("VGGT_CONV_PF2", 1);
int g_vggt_linear_one_launch = env_or("VGGT_LINEAR_ONE_LAUNCH", 1);
int g_vggt_linear_split_k = env_or("VGGT_LINEAR_SPLIT_K", 128);
int g_vggt_linear_wk = env_or("VGGT_LINEAR_WK", 64);
int g_vggt_gemm_balance = env_or("VGGT_GEMM_BALANCE", 0);  // whole rounds persistent + tail on 128x128: bitwise equal but
// slower in the model (aggregator step 99.4-99.96 vs 98.7-99.0 ms, profiles/r10/ab_r10n_head_*.json), so off

extern "C" int vggt_tune(int knob, int value) {
  int prev;
  switch (knob) {
    case VGGT_TUNE_GEMM_TILE:
      // -1 auto, 0 128x128, 1/2 256-row ring (BN 256/128), 3 ping-pong (BN picked), 4/5/6 ping-pong BN 256/192/128,
      // 7 ping-pong BN 256 when it fills two rounds of CUs, else picked; 8 two-per-CU 256x128;
      // 9 persistent ping-pong 256x256 (bf16 / GELU / f32 epilogues, else as 7)
      if (value < -1 || value > 9) return VGGT_ERR_UNSUPPORTED;
      prev = g_vggt_gemm_tile;
      g_vggt_gemm_tile = value;
      return prev;
    case VGGT_TUNE_ATTN_WAVES:
      if (value != 2 && value != 4 && value != 8) return VGGT_ERR_UNSUPPORTED;
      prev = g_vggt_attn_waves;
      g_vggt_attn_waves = value;
      return prev;
    case VGGT_TUNE_ATTN_VARIANT:
      // 0-15: bit combinations of the max-tracking kernel; 19/23: pipelined QK^T;
      // 32/33 (+64 exact scores): offset-free softmax; 161 = 33 on the 16x16x32 MFMA shape (D = 64)
      // 289 = 33 with the split-tile in-wave pipeline (D = 64); 545 = 33 with 3 K|V slots, DMA two tiles ahead;
      // 2081 = 33 with the LDS-DMA issued by the priority half of the 8-wave form; 4129 = 33 without the priority raise
      // (an asynchronous ring and dynamic priorities were measured and removed: profiles/r11/ab_attn_dma_half.md)
      if (value < 0 || (value > 15 && value != 19 && value != 23 && value != 32 && value != 33 && value != 96 &&
                        value != 97 && value != 161 && value != 289 && value != 545 && value != 2081 && value != 4129))
        return VGGT_ERR_UNSUPPORTED;
      prev = g_vggt_attn_variant;
      g_vggt_attn_variant = value;
      return prev;
    case VGGT_TUNE_ATTN16:
      if (value < 0 || value > 2) return VGGT_ERR_UNSUPPORTED;
      prev = g_vggt_attn16;
      g_vggt_attn16 = value;
      return prev;
    case VGGT_TUNE_LINEAR_ONE_LAUNCH:
      if (value != 0 && value != 1) return VGGT_ERR_UNSUPPORTED;
      prev = g_vggt_linear_one_launch;
      g_vggt_linear_one_launch = value;
      return prev;
    case VGGT_TUNE_LINEAR_SPLIT_K:
      if (value < 16 || value > 4096 || (value & (value - 1))) return VGGT_ERR_UNSUPPORTED;
      prev = g_vggt_linear_split_k;
      g_vggt_linear_split_k = value;
      return prev;
    case VGGT_TUNE_LINEAR_WK:
      if (value != 0 && (value < 64 || value > 4096 || (value & (value - 1)))) return VGGT_ERR_UNSUPPORTED;
      prev = g_vggt_linear_wk;
      g_vggt_linear_wk = value;
      return prev;
    case VGGT_TUNE_GEMM_BALANCE:
      if (value != 0 && value != 1) return VGGT_ERR_UNSUPPORTED;
      prev = g_vggt_gemm_balance;
      g_vggt_gemm_balance = value;
      return prev;
    case VGGT_TUNE_CONV_PF2:
      if (value != 0 && value != 1) return VGGT_ERR_UNSUPPORTED;
      prev = g_vggt_conv_pf2;
      g_vggt_conv_pf2 = value;
      return prev;
    default: return VGGT_ERR_UNSUPPORTED;
  }
}

// Per-stream launch configuration (a handful of streams: the multi-GPU pipeline's
// encode streams): the CUs launches may use (CU-masked streams) and flags.
// Written under a lock, read lock-free.
namespace {
constexpr int kMaxStreams = 16;
std::atomic<void*> g_cfg_stream[kMaxStreams];
std::atomic<int> g_cfg_cus[kMaxStreams];
std::atomic<int> g_cfg_flags[kMaxStreams];
std::mutex g_cfg_mu;
int find_cfg(void* stream) {
  if (!stream) return -1;
  for (int i = 0; i < kMaxStreams; ++i)
    if (g_cfg_stream[i].load(std::memory_order_acquire) == stream) return i;
  return -1;
}
}  // namespace

int vggt_stream_cu_count(void* stream) {
  const int i = find_cfg(stream);
  return i < 0 ? 0 : g_cfg_cus[i].load(std::memory_order_relaxed);
}

int vggt_stream_flags(void* stream) {
  const int i = find_cfg(stream);
  return i < 0 ? 0 : g_cfg_flags[i].load(std::memory_order_relaxed);
}

extern "C" int vggt_set_stream_config(void* stream, int cus, int flags) {
  if (!stream || cus < 0 || (flags & ~VGGT_STREAM_SHORT_WORKGROUPS)) return VGGT_ERR_SHAPE;
  std::lock_guard<std::mutex> lk(g_cfg_mu);
  int slot = find_cfg(stream);
  const int prev = slot < 0 ? 0 : (g_cfg_cus[slot].load(std::memory_order_relaxed) |
                                    g_cfg_flags[slot].load(std::memory_order_relaxed) << 16);
  if (cus == 0 && flags == 0) {
    if (slot >= 0) g_cfg_stream[slot].store(nullptr, std::memory_order_release);
    return prev;
  }
  if (slot < 0) {
    for (int i = 0; i < kMaxStreams && slot < 0; ++i)
      if (!g_cfg_stream[i].load(std::memory_order_relaxed)) slot = i;
    if (slot < 0) return VGGT_ERR_UNSUPPORTED;
    g_cfg_cus[slot].store(cus, std::memory_order_relaxed);
    g_cfg_flags[slot].store(flags, std::memory_order_relaxed);
    g_cfg_stream[slot].store(stream, std::memory_order_release);
  } else {
    g_cfg_cus[slot].store(cus, std::memory_order_relaxed);
    g_cfg_flags[slot].store(flags, std::memory_order_relaxed);
  }
  return prev;
}
