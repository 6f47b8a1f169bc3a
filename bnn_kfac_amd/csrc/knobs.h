// The library's environment knobs: read ONCE, when libkfac_hip.so is loaded (capi.hip),
// never per launch.  Each is documented in INTEGRATION.md; defaults are the measured
// best.  kfac_set_knob / kfac_get_knob (include/kfac_hip.h) change or read the
// per-call ones at run time (tests compare the graph-replayed inversion with the
// per-step launches in one process).
#pragma once

namespace kfac {

struct Knobs {
  // factor-product kernel selection (-1 auto, 0 off, 1 forced): fixed at load, since a
  // pass's accumulator plan and its launches must agree on the kernel
  int syrk3;       // KFAC_SYRK3: kfac_factor_syrk3 for row-major groups (auto: largest n >= 2048)
  int tiles_x3;    // KFAC_TILES_X3: kfac_factor_tiles_x3 (auto: largest n >= 256)
  int conv_small;  // KFAC_CONV_SMALL: channel factors with n <= 8 on kfac_factor_channel_small (1)
  int conv_k;      // KFAC_CONV_K: images per conv task (0: the planner's)
  int conv_x3;     // KFAC_CONV_X3: im2col factors with n > 32 on kfac_factor_conv_x3 (bf16x3) (1)
  // per call (kfac_set_knob may change them between calls)
  int inv_graph;      // KFAC_INV_GRAPH: replay the merged inversion steps from a cached hipGraph (1)
  int inv_lookahead;  // KFAC_INV_LOOKAHEAD: large inversions' bulk update split over a helper stream (1)
  int eig_g;          // KFAC_EIG_G: workgroups of the tridiagonalisation (0: ~n/8)
  int eig_rb;         // KFAC_EIG_RB: rows per batch of the tridiagonalisation (4 or 8)
};

const Knobs& knobs();

}  // namespace kfac
