// Process-wide dispatch switches of libmde_hip (internal).
//
// Every runtime switch of the library lives in one table (tuning.hip): each
// entry starts at its default, is overridden ONCE per process from the
// environment variable MDE_<NAME> (the only getenv site of the library), and
// can be changed afterwards through the C ABI (mde_tuning_set / _get,
// include/mde.h) -- the parity tests toggle them that way to compare a path
// against its alternative.  A captured hipGraph keeps the choice it was
// captured with.  Every switch has a GPU test that exercises both settings
// (tests/test_gpu_*.py, named beside each entry below).
#pragma once

namespace mde {

enum Knob : int {
  // E_STORE / E_RESID split-K of small-grid GEMMs and DPT convs (1: on).
  // test_fc2_splitk_matches_unsplit, test_conv3x3_splitk
  KNOB_SPLITK = 0,
  // LayerNorm folded into the consumer GEMMs of f16-residual engines (1: on;
  // read at context creation).  test_lnfold_matches_layernorm
  KNOB_LNFOLD,
  // narrower direct-conv channel tiles on small grids (1: on).
  // test_conv_narrow_tiles_bit_exact
  KNOB_CONV_NARROW,
  // separable upsampling conv for the 32-channel head convs (1: on).
  // test_upconv_matches_conv3
  KNOB_UPCONV,
  // 256^2 phase-pipelined GEMM for large long-K problems (0 never, 1 auto, 2
  // whenever legal).  test_gemm256_modes_match
  KNOB_GEMM256,
  // 4-deep LDS ring for small-grid 64^2 tiles (1: on).
  // test_gemm_small_grid_variants_bit_exact
  KNOB_DEEP64,
  // 8 waves on small-grid 128^2 tiles (1: on).
  // test_gemm_small_grid_variants_bit_exact
  KNOB_W8SMALL,
  // persistent 64 -> 64 channel direct conv with LDS-resident weights (0 off,
  // 1: 16 x 16-pixel tiles on 8 waves, 2: 8 x 16 on 4 waves).
  // test_conv_persist_bit_exact
  KNOB_CONV_PERSIST,
  // A-stationary panel GEMM (gemm_panel.hip) for the K = 384 E_STORE /
  // E_QKV problems at large batch -- the ViT-S fc1 and qkv (1: on; 2: also
  // the f16-residual proj, slower in the engine).  test_panel_gemm_bit_exact
  KNOB_PANEL,
  // the panel GEMM's qkv / fc1 on v_mfma_f32_32x32x16_f16 with the folded
  // LayerNorm's mean term in the accumulator's initial value (panel32_kernel;
  // 1: on; default off: no step gain, gemm_panel.hip).
  // test_panel32_matches_tile_kernel
  KNOB_PANEL32,
  // small-grid residual updates (ViT-S batch 1: fc2 / proj, 1370 x 384) on
  // 32 x 64 tiles with the whole K loop and a 4-deep ring instead of split-K
  // slices + the reduce launch (1: on).  test_narrow_resid_matches_split
  KNOB_NARROW_RESID,
  // the large-grid attention (8 waves, unsplit: B = 48) on
  // v_mfma_f32_16x16x32_f16 (attn16_fwd_kernel; 1: on; 0: the 32x32x16
  // attn_fwd_kernel).  test_attention_16x16_matches
  KNOB_ATTN16,
  // the split-K slices and their reduce as one launch (GemmParams::tile_cnt:
  // the last slice of a tile to arrive adds the slots in slice order and runs
  // the epilogue; 1: on; 0, the default: slices + splitk_resid / splitk_store
  // kernels -- the fused tail's system-scope round trips measured slower,
  // ViT-L B=1 3.17 -> 3.79 ms).  test_splitk_fused_matches_two_kernel
  KNOB_SPLITK_FUSED,
  // attn16's partial last query block of every sequence dispatched after all
  // full blocks (1: work order only, bit-identical; 2, the default: and a
  // partial block of <= 128 queries run as two key groups of 4 query waves;
  // 0: the XCD-remapped (sequence, block) order).
  // test_attention_tail_order_bit_exact
  KNOB_ATTN_TAIL,
  // the DPT fusion blocks' x2 resize read on the fly by the next block's
  // residual conv (GemmParams::res1_up: the direct conv's epilogue blends the
  // four taps) instead of a resize launch (1: on).  Same bits.
  // test_resize_fold_bit_exact
  KNOB_RESIZE_FOLD,
  KNOB_COUNT
};

// current value of a switch (relaxed atomic read; cheap enough per launch)
int knob(Knob k);

}  // namespace mde
